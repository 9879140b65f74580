"""On-disk DAS dataset: directory scan, per-category splits, labels and RAM/disk datasets.

Behavioural parity with reference dataset_preparation.py:
  * ``DataCollector``      -> :17-80   category dirs sorted by their first integer; ``.mat`` key lookup
  * ``add_gaussian``       -> :83-105  white noise at a target SNR (fixed seed 1)
  * ``Dataset_mat_MTL``    -> :108-239 per-category KFold(5, shuffle, random_state) fold ``fold_index``
                                       (or train_test_split(test_size=0.17647)); label = [metres, event];
                                       test mode puts every file in both 'train' and 'val'; optional
                                       joint label ``d + 16 e``
  * ``data_process``       -> :242-249 add the channel axis, cast to float32
  * ``Datasetram/DatasetDisk`` -> :252-344

Documented deviations: file listings are *sorted* (the reference uses raw
``os.listdir`` order, which makes splits filesystem-dependent); everything else is unchanged.
The datasets additionally expose ``as_arrays()`` so the trainer can upload the whole split to HBM
once (288 GB per MI355X) instead of collating per batch on the host.
"""
from __future__ import annotations

import os
import re
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.utils.data

try:  # scipy is the .mat reader (reference uses scipy.io.loadmat too)
    import scipy.io as sio
except Exception:  # pragma: no cover
    sio = None

TEST_RATE = 0.17647  # = 0.15 / 0.85 (70/15/15 protocol), reference dataset_preparation.py:118
N_FOLDS = 5


def _category_index(name: str) -> int:
    found = re.findall(r"\d+", name)
    if not found:
        raise ValueError(f"category directory {name!r} has no integer in its name")
    return int(found[0])


def load_mat(path: str, keys: Sequence[str] = ("data",)) -> np.ndarray:
    if sio is None:
        raise RuntimeError("scipy is required to read .mat files")
    content = sio.loadmat(path)
    if len(keys) == 1:
        return content[keys[0]]
    for k in keys:
        if k in content:
            return content[k]
    raise ValueError(f"none of {keys} found in {path}")


class DataCollector:
    """Index of ``<root>/<N>m/<file>.mat``: category -> sorted list of full file paths."""

    def __init__(self, dirPath: str, keyList: Sequence[str] = ("data",)):
        self.dirPath = dirPath
        self.keyList = list(keyList)
        self.allFileFullNameDict: Dict[str, List[str]] = {
            c: self.get_fileFullnameList_by_category(c) for c in self.get_all_categorys()}

    def get_all_categorys(self) -> List[str]:
        entries = [d for d in os.listdir(self.dirPath) if os.path.isdir(os.path.join(self.dirPath, d))]
        return sorted(entries, key=_category_index)

    def get_fileFullnameList_by_category(self, categoryName: str) -> List[str]:
        base = os.path.join(self.dirPath, categoryName)
        return [base + "/" + n for n in sorted(os.listdir(base))]

    def get_one_mat(self, fileFullName: str) -> np.ndarray:
        return load_mat(fileFullName, self.keyList)

    def get_mat_by_categoryIndex(self, category: str, index: int) -> np.ndarray:
        return self.get_one_mat(self.allFileFullNameDict[category][index])

    def get_mat_name_by_categoryIndex(self, category: str, index: int):
        name = self.allFileFullNameDict[category][index]
        return self.get_one_mat(name), name


def add_gaussian(signal: np.ndarray, SNR: float = 8, seed: Optional[int] = 1) -> np.ndarray:
    """Add zero-mean white Gaussian noise so that the result has the requested SNR (dB).

    Same estimator as the reference: signal power from the mean-removed signal, noise rescaled by its
    own std.  ``seed=1`` reproduces the reference's fixed ``np.random.seed(1)``; pass ``None`` for
    fresh noise.
    """
    signal = np.asarray(signal, dtype=np.float64)
    rng = np.random.RandomState(seed) if seed is not None else np.random
    noise = rng.randn(*signal.shape)
    noise = noise - noise.mean()
    centred = signal - signal.mean()
    signal_power = np.sum(centred ** 2) / signal.size
    noise_var = signal_power / (10.0 ** (SNR / 10.0))
    return signal + (np.sqrt(noise_var) / noise.std()) * noise


def measured_snr(clean: np.ndarray, noisy: np.ndarray) -> float:
    ps = np.sum((clean - clean.mean()) ** 2)
    pn = np.sum((clean - noisy) ** 2)
    return float(10 * np.log10(ps / pn))


def data_process(mat: np.ndarray, snr_db: Optional[float] = None) -> np.ndarray:
    """``[H, W] -> [1, H, W] float32`` (optionally with per-row SNR noise, the reference's disabled hook).
    A ``[C, H, W]`` array (multi-channel synthetic data) is passed through."""
    mat = np.asarray(mat)
    if snr_db is not None:
        mat = np.stack([add_gaussian(row, SNR=snr_db, seed=None) for row in mat.reshape(-1, mat.shape[-1])]
                       ).reshape(mat.shape)
    if mat.ndim == 2:
        mat = mat[np.newaxis, :]
    return mat.astype(np.float32)


def split_category(files: List[str], is_test: bool, fold_index: Optional[int], random_state: int,
                   test_rate: float = TEST_RATE):
    """Per-category split (reference dataset_preparation.py:136-212)."""
    if is_test:
        return list(files), list(files)
    if fold_index is None:
        from sklearn.model_selection import train_test_split
        tr, te = train_test_split(files, test_size=test_rate, random_state=random_state)
        return list(tr), list(te)
    from sklearn.model_selection import KFold
    folds = list(KFold(n_splits=N_FOLDS, shuffle=True, random_state=random_state).split(files))
    tr_idx, te_idx = folds[fold_index]
    return [files[i] for i in tr_idx], [files[i] for i in te_idx]


class _MatDatasetBase(torch.utils.data.Dataset):
    def __init__(self, mat_list, label_list, key="data", paper_single=False, snr_db=None):
        assert len(mat_list) == len(label_list)
        self.mat_list = list(mat_list)
        self.label_list = list(label_list)
        self.key = key
        self.paper_single = paper_single
        self.snr_db = snr_db

    def __len__(self):
        return len(self.mat_list)

    def _load(self, i):
        return data_process(load_mat(self.mat_list[i], (self.key,)), self.snr_db)

    def _item(self, mat, i):
        if self.paper_single:
            return mat, self.label_list[i]
        d, e = self.label_list[i]
        return mat, d, e

    def labels_array(self) -> np.ndarray:
        """``[N]`` joint labels (paper_single) or ``[N, 2]`` (distance, event)."""
        return np.asarray(self.label_list, dtype=np.int64)

    def as_arrays(self):
        x = np.stack([self[i][0] for i in range(len(self))]) if len(self) else np.zeros((0, 1, 100, 250), np.float32)
        return x, self.labels_array()

    def get_name_label_csv(self, savedir="./name_label.csv", paper_single=False):
        import pandas as pd
        if paper_single or self.paper_single:
            table = {"mat name": self.mat_list, "label": self.label_list}
        else:
            table = {"mat name": self.mat_list, "distance label": [l[0] for l in self.label_list],
                     "event label": [l[1] for l in self.label_list]}
        pd.DataFrame(table).to_csv(savedir, encoding="gbk")


class Datasetram(_MatDatasetBase):
    """Loads every file at construction (reference ``Datasetram``)."""

    def __init__(self, mat_list, label_list, key="data", paper_single=False, snr_db=None, progress=True):
        super().__init__(mat_list, label_list, key, paper_single, snr_db)
        self._arr = self._load_native() if snr_db is None else None
        if self._arr is not None:
            self.mat_file_list = list(self._arr)
            return
        it = range(len(self.mat_list))
        if progress:
            try:
                from tqdm import tqdm
                it = tqdm(it)
            except Exception:
                pass
        self.mat_file_list = [self._load(i) for i in it]

    def _load_native(self):
        """All files in one call of the native multi-threaded MAT reader (csrc/matio.cpp) into one
        contiguous float32 array; files it does not parse are read with scipy.  None if unavailable."""
        if not self.mat_list:
            return None
        try:
            from ..ops.hip import available, lib
            if not available():
                return None
            L = lib()
        except Exception:  # pragma: no cover
            return None
        first = self._load(0)
        dims = list(np.shape(load_mat(self.mat_list[0], (self.key,))))  # MATLAB dims every file must have
        if int(np.prod(dims)) != first.size:
            return None
        arr = np.empty((len(self.mat_list),) + first.shape, np.float32)
        st = L.MatBatchLoader(self.mat_list, self.key, dims, min(16, os.cpu_count() or 1)).load(
            list(range(len(self.mat_list))), arr.ctypes.data)
        for j, rc in enumerate(st):
            if rc != 0:
                arr[j] = self._load(j)
        return arr

    def __getitem__(self, item):
        return self._item(self.mat_file_list[item], item)

    def as_arrays(self):
        if not self.mat_file_list:
            return np.zeros((0, 1, 100, 250), np.float32), self.labels_array()
        if self._arr is not None:
            return self._arr, self.labels_array()
        return np.stack(self.mat_file_list), self.labels_array()


class DatasetDisk(_MatDatasetBase):
    """Lazily loads each file in ``__getitem__`` (reference ``DatasetDisk``)."""

    def __getitem__(self, item):
        return self._item(self._load(item), item)


class Dataset_mat_MTL:
    """Builds ``self.dataset = {'train': ..., 'val': ...}`` from the striking and excavating trees."""

    def __init__(self, dataset_dir_striking, dataset_dir_excavating, testRate=TEST_RATE, random_state=1,
                 category_dir_list0324=None, category_dir_listwajue=None, ram=False, multi_categories=False,
                 is_test=False, fold_index=None, snr_db=None, progress=True):
        self.matpathListTrain: List[str] = []
        self.labelListTrain: list = []
        self.matpathListTest: List[str] = []
        self.labelListTest: list = []
        for event, root, cats in ((0, dataset_dir_striking, category_dir_list0324),
                                  (1, dataset_dir_excavating, category_dir_listwajue)):
            collector = DataCollector(root, ["data"])
            for cat in (cats if cats is not None else collector.get_all_categorys()):
                files = collector.get_fileFullnameList_by_category(cat)
                tr, te = split_category(files, is_test, fold_index, random_state, testRate)
                label = [_category_index(cat), event]
                self.matpathListTrain += tr
                self.labelListTrain += [list(label) for _ in tr]
                self.matpathListTest += te
                self.labelListTest += [list(label) for _ in te]
        if multi_categories:
            self.labelListTrain = [d + 16 * e for d, e in self.labelListTrain]
            self.labelListTest = [d + 16 * e for d, e in self.labelListTest]
        cls = Datasetram if ram else DatasetDisk
        kw = dict(paper_single=multi_categories, snr_db=snr_db)
        if ram:
            kw["progress"] = progress
        self.dataset = {"train": cls(self.matpathListTrain, self.labelListTrain, **kw),
                        "val": cls(self.matpathListTest, self.labelListTest, **kw)}
