"""Data layer: directory scan / sort, per-category splits, label encodings, noise, synthetic generator."""
import numpy as np
import pytest
import torch

from mtl_das_pytorch_amd.data import (DataCollector, Dataset_mat_MTL, DeviceDataset, add_gaussian, data_process,
                                      generate, measured_snr, split_category, write_mat_tree)


@pytest.fixture(scope="module")
def tree(tmp_path_factory):
    root = tmp_path_factory.mktemp("das")
    return write_mat_tree(str(root), n_per_class=5, n_test_per_class=2, seed=3)


def test_collector_sorts_categories_numerically(tree):
    c = DataCollector(tree["striking_train"], ["data"])
    cats = c.get_all_categorys()
    assert cats == [f"{i}m" for i in range(16)]
    files = c.get_fileFullnameList_by_category("10m")
    assert files == sorted(files) and len(files) == 5
    m = c.get_mat_by_categoryIndex("3m", 0)
    assert m.shape == (100, 250)


def test_kfold_split_sizes_and_labels(tree):
    ds = Dataset_mat_MTL(tree["striking_train"], tree["excavating_train"], random_state=1, ram=True,
                         fold_index=0, progress=False)
    tr, va = ds.dataset["train"], ds.dataset["val"]
    assert len(tr) == 2 * 16 * 4 and len(va) == 2 * 16 * 1  # 5 files per category -> 4/1
    x, d, e = tr[0]
    assert x.shape == (1, 100, 250) and x.dtype == np.float32
    labels = np.asarray(tr.label_list)
    assert set(labels[:, 0]) == set(range(16)) and set(labels[:, 1]) == {0, 1}
    assert not set(tr.mat_list) & set(va.mat_list)


def test_train_test_split_mode(tree):
    ds = Dataset_mat_MTL(tree["striking_train"], tree["excavating_train"], ram=False, fold_index=None)
    assert len(ds.dataset["train"]) + len(ds.dataset["val"]) == 160
    assert len(ds.dataset["val"]) == 2 * 16 * 1  # ceil(0.17647 * 5) = 1 per category


def test_test_mode_duplicates_all_files(tree):
    ds = Dataset_mat_MTL(tree["striking_test"], tree["excavating_test"], is_test=True, ram=True, progress=False)
    assert ds.dataset["train"].mat_list == ds.dataset["val"].mat_list
    assert len(ds.dataset["val"]) == 64


def test_joint_labels(tree):
    ds = Dataset_mat_MTL(tree["striking_test"], tree["excavating_test"], is_test=True, multi_categories=True)
    for path, lab in zip(ds.dataset["val"].mat_list, ds.dataset["val"].label_list):
        d = int(path.split("/")[-2][:-1])
        e = 1 if "excavating" in path else 0
        assert lab == d + 16 * e
    x, lab = ds.dataset["val"][0]
    assert isinstance(lab, int)


def test_split_category_matches_sklearn_kfold():
    from sklearn.model_selection import KFold
    files = [f"f{i}" for i in range(10)]
    tr, te = split_category(files, False, 2, random_state=1)
    idx = list(KFold(5, shuffle=True, random_state=1).split(files))[2]
    assert tr == [files[i] for i in idx[0]] and te == [files[i] for i in idx[1]]


def test_add_gaussian_hits_target_snr():
    rng = np.random.RandomState(0)
    sig = np.sin(np.linspace(0, 20, 2000)) + 0.1 * rng.randn(2000)
    noisy = add_gaussian(sig, SNR=8)
    assert abs(measured_snr(sig, noisy) - 8) < 0.2
    assert np.array_equal(noisy, add_gaussian(sig, SNR=8))  # fixed seed, like the reference


def test_data_process():
    m = np.zeros((100, 250))
    out = data_process(m)
    assert out.shape == (1, 100, 250) and out.dtype == np.float32


def test_synthetic_deterministic_and_labelled():
    x1, d1, e1 = generate(8, seed=5)
    x2, d2, e2 = generate(8, seed=5)
    assert torch.equal(x1, x2) and torch.equal(d1, d2) and torch.equal(e1, e2)
    assert x1.shape == (8, 1, 100, 250)
    x3, _, _ = generate(4, seed=5, in_channels=2)
    assert x3.shape == (4, 2, 100, 250)
    # class separability sanity: event types have different temporal spectra
    d = torch.full((32,), 3)
    xs, _, _ = generate(32, seed=1, distance=d, event=torch.zeros(32, dtype=torch.long))
    xd, _, _ = generate(32, seed=1, distance=d, event=torch.ones(32, dtype=torch.long))
    hi = lambda x: torch.fft.rfft(x[:, 0], dim=-1).abs()[..., 30:60].mean()  # noqa: E731
    assert hi(xs) > 1.5 * hi(xd)


def test_device_dataset_batches():
    ds = DeviceDataset.synthetic(20, "cpu", seed=1)
    b = ds.batch_indices(8, shuffle=True, generator=torch.Generator().manual_seed(0))
    assert [len(i) for i in b] == [8, 8, 4]
    assert sorted(torch.cat(b).tolist()) == list(range(20))
