"""Canary guard bands around every device buffer the engine's kernels write (out-of-bounds write detector).

The engine's kernels write through raw pointers into buffers it allocates itself: arena activations and
gradients, BN statistic replicas, weight-gradient split slabs, the LDS conv kernels' split-K workspaces and
arrival tickets, the finalize / Adam targets (the flat parameter, gradient and moment buffers), the bf16
weight images, head metrics.  An out-of-bounds write by one of them lands in a neighbouring allocation --
possibly a tensor of PyTorch itself -- and shows up far away, e.g. as an illegal address inside a later
library call.

With the guard on (``MDA_GUARD=1`` in the environment, or :func:`enable` before the program is built) every
such buffer is allocated inside a larger byte buffer whose head and tail bands (``PAD`` bytes each) hold a
fixed byte pattern; :func:`check` compares every band with the pattern and names the buffers whose bands
changed.  Off (the default) the allocators are plain ``torch.empty`` / ``torch.zeros``.
"""
from __future__ import annotations

import os
from typing import List, Sequence, Tuple

import torch

PAD = 4096          # bytes of each guard band (a multiple of every vector width the kernels use)
PATTERN = 0x5A      # band byte

_enabled = os.environ.get("MDA_GUARD") == "1"
_registry: List[Tuple[str, torch.Tensor, int]] = []  # (label, full uint8 buffer, body bytes)


def enable(on: bool = True):
    global _enabled
    _enabled = on


def enabled() -> bool:
    return _enabled


def reset():
    _registry.clear()


def alloc(shape, dtype=torch.float32, device="cpu", zero: bool = False, label: str = "") -> torch.Tensor:
    """``torch.zeros`` (zero=True) / ``torch.empty`` of ``shape``; guarded when the guard is enabled."""
    if not _enabled or torch.device(device).type != "cuda":
        return torch.zeros(shape, dtype=dtype, device=device) if zero else torch.empty(shape, dtype=dtype, device=device)
    shape = tuple(int(s) for s in (shape if isinstance(shape, (tuple, list, torch.Size)) else (shape,)))
    n = 1
    for s in shape:
        n *= s
    nbytes = n * torch.empty((), dtype=dtype).element_size()
    full = torch.full((PAD + nbytes + PAD,), PATTERN, dtype=torch.uint8, device=device)  # tail band: right after
    t = full[PAD:PAD + nbytes].view(dtype).view(shape)
    if zero:
        t.zero_()
    _registry.append((label or f"{tuple(shape)} {dtype}", full, nbytes))
    return t


def alloc_like(t: torch.Tensor, zero: bool = True, label: str = "") -> torch.Tensor:
    return alloc(tuple(t.shape), t.dtype, t.device, zero, label)


def check() -> List[str]:
    """Labels (with the first corrupted byte offset) of every guarded buffer whose bands changed."""
    bad = []
    for label, full, body in _registry:
        head, tail = full[:PAD], full[PAD + body:]
        for name, band, base in (("head", head, -PAD), ("tail", tail, body)):
            diff = (band != PATTERN).nonzero()
            if diff.numel():
                bad.append(f"{label}: {name} band written at byte {base + int(diff[0])} "
                           f"({int(diff.numel())} bytes changed)")
    return bad


def count() -> int:
    return len(_registry)


def labels() -> Sequence[str]:
    return [r[0] for r in _registry]
