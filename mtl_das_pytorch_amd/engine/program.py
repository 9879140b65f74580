"""A lowered program: an ordered list of prebuilt HIP launches (forward, backward, optimizer).

Launch arguments (device pointers, geometry, descriptor tables) are resolved once at lowering time,
so executing a phase is a tight loop of pybind calls; on the GPU the loop is captured once into a
HIP graph and replayed (engine/step.py)."""
from __future__ import annotations

from typing import Callable, List

from ..ops.hip import lib, stream


class Launch:
    __slots__ = ("name", "fn", "args", "owner")

    def __init__(self, name: str, fn: Callable, *args, owner=None):
        self.name = name
        self.fn = fn
        self.args = args
        self.owner = owner  # the layer object that emitted it (used by the autotuner)

    def __call__(self, st: int):
        self.fn(*self.args, st)


class Phase:
    def __init__(self, name: str):
        self.name = name
        self.launches: List[Launch] = []

    def add(self, name, fn, *args, owner=None):
        self.launches.append(Launch(name, fn, *args, owner=owner))

    def run(self, st=None):
        st = stream() if st is None else st
        for l in self.launches:
            l(st)

    def __len__(self):
        return len(self.launches)


# thin adapters giving every launch the signature fn(*args, stream)
def k_conv(mode, cfg, G, d, st):
    lib().conv(mode, cfg, G, st, d)


def k_wgrad(cfg, G, d, st):
    lib().wgrad(cfg, G, st, d)


def k_tail_fwd(kind, G, blocks, d, st):
    lib().tail_fwd(kind, G, blocks, st, d)


def k_tail_bwd(kind, G, blocks, d, st):
    lib().tail_bwd(kind, G, blocks, st, d)


def k_head(d, st):
    lib().mtl_head(st, d)


def k_cls_head(d, st):
    lib().cls_head(st, d)


def k_pool(is_max, bwd, d, st):
    lib().pool3(is_max, bwd, st, d)


def k_wgfin(table, nd, nblocks, st):
    lib().wgrad_finalize(table.data_ptr(), nd, nblocks, 1.0, st)


def k_adam(d, st):
    lib().adam_pack(st, d)


def k_gather(X, idx, lab, lab_w, out, lab_out, B, Cin, H, W, st):
    lib().gather_batch(X.data_ptr(), idx.data_ptr(), lab.data_ptr(), lab_w, out.data_ptr(), lab_out.data_ptr(),
                       B, Cin, H, W, st)
