"""Disk-streaming input path (--dataset_ram False, reference DatasetDisk) and the native MAT reader."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lib():
    from mtl_das_pytorch_amd.ops.hip import available, lib
    if not available():
        pytest.skip("native extension not built")
    return lib()


@pytest.mark.parametrize("compress", [False, True])
@pytest.mark.parametrize("arr", ["f64", "f32", "i16", "u8", "3d"])
def test_native_mat_reader_matches_scipy(tmp_path, arr, compress):
    import scipy.io as sio
    L = _lib()
    rng = np.random.default_rng(3)
    a = {"f64": rng.standard_normal((100, 250)), "f32": rng.standard_normal((17, 5)).astype(np.float32),
         "i16": (rng.standard_normal((7, 9)) * 300).astype(np.int16),
         "u8": rng.integers(0, 255, (4, 6)).astype(np.uint8), "3d": rng.standard_normal((3, 10, 25))}[arr]
    p = str(tmp_path / "x.mat")
    sio.savemat(p, {"aaa": np.ones(5), "data": a, "zzz": np.zeros((2, 2))}, do_compression=compress)
    rc, shape = L.mat_shape(p, "data")
    assert rc == 0 and tuple(shape) == a.shape
    out = torch.empty(a.size, dtype=torch.float32)
    assert L.mat_read(p, "data", out.data_ptr(), a.size) == 0
    np.testing.assert_array_equal(out.numpy().reshape(a.shape), sio.loadmat(p)["data"].astype(np.float32))
    assert L.mat_read(p, "missing", out.data_ptr(), a.size) != 0
    assert L.mat_read(p, "data", out.data_ptr(), a.size + 1) != 0  # shape mismatch is reported


def test_native_reader_rejects_v4_and_loader_falls_back(tmp_path):
    import scipy.io as sio
    from mtl_das_pytorch_amd.data.mat_dataset import DatasetDisk
    from mtl_das_pytorch_amd.data.stream import DiskBatchStream
    L = _lib()
    rng = np.random.default_rng(4)
    arrs = [rng.standard_normal((100, 250)) for _ in range(5)]
    paths = []
    for i, a in enumerate(arrs):
        p = str(tmp_path / f"{i}.mat")
        sio.savemat(p, {"data": a}, format="4" if i == 2 else "5")
        paths.append(p)
    assert L.mat_shape(paths[2], "data")[0] != 0
    ds = DatasetDisk(paths, [[i, i % 2] for i in range(5)])
    st = DiskBatchStream(ds, batch=2, device="cpu", ring=2)
    got = []
    for rows, n in st.batches([[0, 1], [2, 3], [4]]):
        got.append(st.X[rows].clone())
    st.close()
    x = torch.cat(got)
    np.testing.assert_array_equal(x.numpy()[:, 0], np.stack(arrs).astype(np.float32))
    assert st.fallbacks == 1


@pytest.fixture(scope="module")
def tree(tmp_path_factory):
    from mtl_das_pytorch_amd.data import write_mat_tree
    return write_mat_tree(str(tmp_path_factory.mktemp("das_stream")), n_per_class=5, n_test_per_class=1, seed=5)


def test_stream_ring_recycles_slots_in_order(tree):
    """ring=2 with many batches: every batch read back from the ring equals the resident dataset's rows."""
    from mtl_das_pytorch_amd.data.mat_dataset import Dataset_mat_MTL
    from mtl_das_pytorch_amd.data.stream import DiskBatchStream
    ram = Dataset_mat_MTL(tree["striking_train"], tree["excavating_train"], ram=True, fold_index=0, progress=False)
    disk = Dataset_mat_MTL(tree["striking_train"], tree["excavating_train"], ram=False, fold_index=0)
    xr, yr = ram.dataset["train"].as_arrays()
    st = DiskBatchStream(disk.dataset["train"], batch=5, device="cpu", ring=2, threads=3)
    order = torch.randperm(len(xr), generator=torch.Generator().manual_seed(0))
    chunks = [order[i:i + 5] for i in range(0, len(order), 5)]
    for (rows, n), idx in zip(st.batches(chunks), chunks):
        assert n == len(idx)
        np.testing.assert_array_equal(st.X[rows].numpy(), xr[idx.numpy()])
        np.testing.assert_array_equal(st.labels[rows].numpy(), yr[idx.numpy()])
    st.close()
    assert st.X.shape[0] == 10  # ring * batch rows, whatever the dataset size


def test_trainer_disk_stream_matches_ram(tree, tmp_path):
    """--dataset_ram False trains on exactly the same batches as the RAM path (CPU, torch backend)."""
    from mtl_das_pytorch_amd.engine.trainer import Trainer
    from mtl_das_pytorch_amd.utils.config import TrainConfig
    res = {}
    for ram in (True, False):
        torch.manual_seed(0)
        cfg = TrainConfig(model="MTL", batch_size=8, epoch_num=1, val_every=1, log_every=4,
                          output_savedir=str(tmp_path / str(ram)), GPU_device=False, save_threshold=2.0,
                          dataset_ram=ram, stream_ring=3, trainVal_set_striking=tree["striking_train"],
                          trainVal_set_excavating=tree["excavating_train"])
        tr = Trainer(cfg)
        tr.run()
        res[ram] = (tr.last_val, {k: v.clone() for k, v in tr.model.state_dict().items()})
    assert res[True][0]["acc"] == res[False][0]["acc"]
    assert res[True][0]["loss"] == res[False][0]["loss"]
    for k, v in res[True][1].items():
        assert torch.equal(v, res[False][1][k]), k


_RSS_SCRIPT = r"""
import psutil, sys, threading, time, torch
sys.path.insert(0, {root!r})
from mtl_das_pytorch_amd.engine.trainer import Trainer
from mtl_das_pytorch_amd.utils.config import TrainConfig
torch.set_num_threads(4)
cfg = TrainConfig(model="single_event", batch_size=8, epoch_num=1, val_every=1, log_every=1000,
                  output_savedir={out!r}, GPU_device=False, save_threshold=2.0, dataset_ram={ram},
                  trainVal_set_striking={s!r}, trainVal_set_excavating={e!r})
tr = Trainer(cfg)
# warm-up outside the measured window: CPU autograd / oneDNN workspaces, sklearn + matplotlib imports
import sklearn.model_selection, matplotlib.pyplot
tr.model(torch.randn(8, 1, 100, 250)).sum().backward()
proc = psutil.Process()
base = peak = proc.memory_info().rss
done = threading.Event()
def sample():
    global peak
    while not done.is_set():
        peak = max(peak, proc.memory_info().rss)
        time.sleep(0.002)
th = threading.Thread(target=sample)
th.start()
tr.run()
done.set()
th.join()
print("RSS_B", base, peak)
"""


@pytest.mark.slow
def test_disk_stream_peak_rss_below_dataset_size(tmp_path):
    """End to end on a 3200-file tree (320 MB as float32): the streamed run's peak RSS grows by far less
    than the dataset (ring + optimizer state), the RAM run's by at least the dataset."""
    from mtl_das_pytorch_amd.data import write_mat_tree
    t = write_mat_tree(str(tmp_path / "big"), n_per_class=100, n_test_per_class=0, seed=9, splits=("train",))
    ds_bytes = 3200 * 100 * 250 * 4
    growth = {}
    for ram in (False, True):
        code = _RSS_SCRIPT.format(root=ROOT, out=str(tmp_path / f"o{ram}"), ram=ram, s=t["striking_train"],
                                  e=t["excavating_train"])
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=900,
                           env=dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES=""))
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        line = [l for l in r.stdout.splitlines() if l.startswith("RSS_B")][-1]
        base, peak = (int(v) for v in line.split()[1:])
        growth[ram] = peak - base
    print({k: v / 2 ** 20 for k, v in growth.items()}, "dataset MB", ds_bytes / 2 ** 20)
    assert growth[False] < ds_bytes / 2, growth  # ring + activations only
    assert growth[True] - growth[False] > ds_bytes * 0.8, growth


def test_native_loader_rejects_transposed_and_non_regular_files(tmp_path):
    """A variable with the right numel but other dims (250 x 100 for a 100 x 250 slot) is rejected by the
    native batch loader -- it would land transposed -- and a directory entry returns an error status instead
    of crashing a worker thread; the streaming dataset then raises on the scipy fallback's shape check."""
    import scipy.io as sio
    from mtl_das_pytorch_amd.data.mat_dataset import DatasetDisk
    from mtl_das_pytorch_amd.data.stream import DiskBatchStream
    L = _lib()
    rng = np.random.default_rng(5)
    good, bad = str(tmp_path / "good.mat"), str(tmp_path / "bad.mat")
    sio.savemat(good, {"data": rng.standard_normal((100, 250))})
    sio.savemat(bad, {"data": rng.standard_normal((250, 100))})
    (tmp_path / "adir").mkdir()
    ld = L.MatBatchLoader([good, bad, str(tmp_path / "adir")], "data", [100, 250], 2)
    out = torch.empty(3, 100 * 250)
    st = ld.load([0, 1, 2], out.data_ptr())
    assert st[0] == 0 and st[1] != 0 and st[2] != 0
    assert L.mat_read(str(tmp_path / "adir"), "data", out.data_ptr(), 100 * 250) != 0
    ds = DatasetDisk([good, bad], [[0, 0], [1, 1]])
    s = DiskBatchStream(ds, batch=2, device="cpu", ring=2)
    with pytest.raises(ValueError, match="shape"):
        for _ in s.batches([[0, 1]]):
            pass
    s.close()
