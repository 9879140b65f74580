"""Disk-streaming input pipeline (``--dataset_ram False``): .mat files -> pinned host ring -> HBM ring.

The reference's ``DatasetDisk`` (dataset_preparation.py:300-344, selected by ``ram=dataset_ram`` in
utils.py:148-150) reads every sample from disk inside the DataLoader on each epoch, so host memory holds
only the batches in flight.  The MI355X version keeps that property and overlaps every stage with the
training step:

  loader thread   native MAT reader (csrc/matio.cpp, a C++ worker pool, GIL released) fills pinned host
                  slot ``k`` with batch ``i`` (float32, row-major, the reference's data_process layout);
  copy stream     async H2D copy of the slot into HBM ring slot ``k`` once the step that last read that
                  slot has finished (event), then records ``ready[k]``;
  compute stream  waits ``ready[k]`` and runs the step, whose gather kernel reads ring rows
                  ``k*B .. k*B+B-1`` -- the same gather + HIP-graph path as the HBM-resident dataset,
                  because the ring is one persistent device tensor.

``ring`` batches are in flight (loading / copying / training); host and device memory is
``ring * batch`` samples whatever the dataset size.  Files the native reader cannot parse (MAT v4,
v7.3/HDF5, non-numeric variables) fall back to ``scipy.io.loadmat`` for that file.
"""
from __future__ import annotations

import concurrent.futures as cf
from typing import Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .mat_dataset import add_gaussian, data_process, load_mat


def _native_loader():
    try:
        from ..ops.hip import available, lib
        if available() and hasattr(lib(), "MatBatchLoader"):
            return lib()
    except Exception:  # pragma: no cover - extension not built: scipy path
        pass
    return None


class DiskBatchStream:
    """Streams batches of a file-backed dataset into a device ring buffer.

    ``ds`` is a ``Datasetram``/``DatasetDisk`` (its ``mat_list`` / ``labels_array()`` are used, never
    its in-memory copy).  ``X`` ``[ring*B, C, H, W]`` float32 and ``labels`` (``[ring*B, 2]`` or
    ``[ring*B]``) are the device tensors a backend reads; :meth:`batches` yields, per batch of dataset
    indices, the ring row indices to train/evaluate on (a device tensor) and the number of valid rows.
    """

    def __init__(self, ds, batch: int, device, ring: int = 4, threads: int = 8, key: str = "data",
                 snr_db: Optional[float] = None):
        if ring < 2:
            raise ValueError("ring must hold at least 2 batches")
        self.paths: List[str] = list(ds.mat_list)
        self.lab_host = torch.as_tensor(ds.labels_array())
        self.B, self.R, self.key = batch, ring, key
        self.snr_db = snr_db if snr_db is not None else getattr(ds, "snr_db", None)
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        first = self._load_scipy(0) if self.paths else np.zeros((1, 100, 250), np.float32)
        self.sample_shape: Tuple[int, ...] = tuple(first.shape)
        self.numel = int(np.prod(self.sample_shape))
        lab_shape = tuple(self.lab_host.shape[1:])
        pin = self.cuda
        self.host = [torch.empty((batch,) + self.sample_shape, dtype=torch.float32, pin_memory=pin)
                     for _ in range(ring)]
        self.host_lab = [torch.empty((batch,) + lab_shape, dtype=torch.int64, pin_memory=pin) for _ in range(ring)]
        self.X = torch.zeros((ring * batch,) + self.sample_shape, dtype=torch.float32, device=self.device)
        self.labels = torch.zeros((ring * batch,) + lab_shape, dtype=torch.int64, device=self.device)
        self._rows = torch.arange(ring * batch, device=self.device).view(ring, batch)
        lib = _native_loader()
        self.native = None
        if lib is not None and self.paths:
            # the raw variable's dims (a same-numel transposed file is then rejected and read by scipy,
            # which raises on the shape like the reference's collate would)
            dims = list(np.shape(load_mat(self.paths[0], (key,))))
            if int(np.prod(dims)) == self.numel:
                self.native = lib.MatBatchLoader(self.paths, key, dims, threads)
        self.fallbacks = 0
        self._pool = cf.ThreadPoolExecutor(max_workers=1, thread_name_prefix="mda-disk")
        if self.cuda:
            self.copy_stream = torch.cuda.Stream(device=self.device)
            self.ready = [torch.cuda.Event() for _ in range(ring)]     # H2D of slot k done (copy stream)
            self.consumed = [None] * ring                              # last step reading slot k (compute)

    def __len__(self):
        return len(self.paths)

    # ------------------------------------------------------------------------------------------------
    def _load_scipy(self, i: int) -> np.ndarray:
        return data_process(load_mat(self.paths[i], (self.key,)))

    def _fill(self, slot: int, idx: np.ndarray):
        """Loader thread: read the files of one batch into host slot ``slot``."""
        if self.cuda:  # the previous H2D copy out of this host slot must have finished
            self.ready[slot].synchronize()
        buf = self.host[slot]
        n = len(idx)
        if self.native is not None:
            st = self.native.load([int(i) for i in idx], buf.data_ptr())
            bad = [j for j, s in enumerate(st) if s != 0]
        else:
            bad = list(range(n))
        for j in bad:  # files the native reader does not handle
            a = self._load_scipy(int(idx[j]))
            if a.shape != self.sample_shape:
                raise ValueError(f"{self.paths[int(idx[j])]}: shape {a.shape} != {self.sample_shape}")
            buf[j].copy_(torch.from_numpy(a))
        self.fallbacks += len(bad) if self.native is not None else 0
        if self.snr_db is not None:  # the reference's (disabled) per-row SNR noise hook
            for j in range(n):
                a = buf[j].numpy()
                rows = a.reshape(-1, a.shape[-1])
                rows[:] = np.stack([add_gaussian(r, SNR=self.snr_db, seed=None) for r in rows]).astype(np.float32)
        self.host_lab[slot][:n].copy_(self.lab_host[torch.as_tensor(idx, dtype=torch.long)])
        return n

    def _upload(self, slot: int, n: int):
        rows = slice(slot * self.B, slot * self.B + n)
        if not self.cuda:
            self.X[rows].copy_(self.host[slot][:n])
            self.labels[rows].copy_(self.host_lab[slot][:n])
            return
        cs, cur = self.copy_stream, torch.cuda.current_stream(self.device)
        with torch.cuda.stream(cs):
            if self.consumed[slot] is not None:  # the step that read this ring slot last must be done
                cs.wait_event(self.consumed[slot])
            self.X[rows].copy_(self.host[slot][:n], non_blocking=True)
            self.labels[rows].copy_(self.host_lab[slot][:n], non_blocking=True)
            self.ready[slot].record(cs)
        cur.wait_event(self.ready[slot])

    # ------------------------------------------------------------------------------------------------
    def batches(self, index_batches: Sequence) -> Iterator[Tuple[torch.Tensor, int]]:
        """Yield ``(ring_rows, nvalid)`` for each batch of dataset indices, loading ``ring - 1`` batches
        ahead.  The caller must enqueue its step on the current stream before asking for the next batch
        (the slot is recycled once that step has run)."""
        idx = [np.asarray(b.cpu() if torch.is_tensor(b) else b, dtype=np.int64).reshape(-1) for b in index_batches]
        for b in idx:
            if len(b) > self.B:
                raise ValueError(f"batch of {len(b)} > ring batch {self.B}")
        futs = {}
        ahead = self.R - 1

        def submit(i):
            futs[i] = self._pool.submit(self._fill, i % self.R, idx[i])

        for i in range(min(ahead, len(idx))):
            submit(i)
        prev_slot = None
        for i in range(len(idx)):
            slot = i % self.R
            if prev_slot is not None and self.cuda:  # the previous step has been enqueued: mark its slot
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.device))
                self.consumed[prev_slot] = ev
            n = futs.pop(i).result()
            self._upload(slot, n)
            if i + ahead < len(idx):
                submit(i + ahead)
            prev_slot = slot
            yield self._rows[slot][:n], n
        if prev_slot is not None and self.cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self.consumed[prev_slot] = ev

    def close(self):
        self._pool.shutdown(wait=True)
