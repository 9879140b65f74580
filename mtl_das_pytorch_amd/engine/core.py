"""Engine core: flat parameter state, persistent device arena, and conv / BatchNorm layer handles.

The engine does not use autograd.  A model is *lowered* once (for a fixed per-GPU batch size) into a
static program of HIP kernel launches over preallocated NHWC buffers; forward and backward are both
explicit, gradient buffers are written exactly once, and the whole train step is captured into a HIP
graph (``engine/step.py``).  Parameters stay ordinary ``nn.Parameter`` objects of the reference module
tree (so ``state_dict`` keys and checkpoints are unchanged) but their storage is re-pointed into one
flat fp32 buffer, which is at the same time

  * the DP all-reduce bucket (one RCCL call, ``parallel/``),
  * the fused-Adam operand (one kernel, ``csrc/optim.hip``),
  * grouped so that the per-task copies of a branch layer are adjacent with a constant stride: both task
    branches of Model A run as ONE launch with ``grid.z = task`` (the shared input is read with group
    stride 0).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn

from ..ops.functional import (WGRAD_BIG0, WGRAD_LEAN0, WGRAD_LEAN_N, WGRAD_PATCH, WGRAD_TILES, bnb_plan, patch_plan, patch_valid, wgrad_cfg,
                              wgrad_ktiles)
from ..ops.hip import lib, ptr
from . import guard

NREP = 32  # must match csrc/common.h
# storage type of every activation gradient (data gradients, gradient sources, BN-tail side outputs and dz
# buffers): bf16 as under autocast -- producers accumulate in fp32 and round once at the store, consumers sum
# their sources in fp32 (csrc/common.h); half the bytes of the fp32 gradients every backward kernel moved
GRAD_DT = torch.bfloat16
# forward BN-statistic replicas: about one per this many pixels.  512 vs 256: A +0.3 % (6 of 6 interleaved
# pairs over two calls, round 5), C neutral
BN_PX_PER_REP = 512


def pad_to(x: int, m: int) -> int:
    return (x + m - 1) // m * m


# ------------------------------------------------------------------------------------------------
class FlatState:
    """Flat fp32 parameter / gradient / Adam-moment buffers and flat BN running-stat buffers."""

    def __init__(self, module: nn.Module, device, param_groups: Sequence[Sequence[nn.Parameter]] = (),
                 bn_groups: Sequence[Sequence[nn.BatchNorm2d]] = ()):
        self.module = module
        self.device = torch.device(device)
        order: List[nn.Parameter] = []
        seen = set()
        for grp in param_groups:
            for p in grp:
                if id(p) not in seen:
                    order.append(p)
                    seen.add(id(p))
        for p in module.parameters():
            if id(p) not in seen:
                order.append(p)
                seen.add(id(p))
        self.offsets: Dict[int, int] = {}
        off = 0
        for p in order:
            self.offsets[id(p)] = off
            off += pad_to(p.numel(), 4)  # 16-byte aligned slots
        self.numel = off
        self.params = guard.alloc(off, torch.float32, self.device, zero=True, label="flat params")
        self.grads = guard.alloc(off, torch.float32, self.device, zero=True, label="flat grads")
        self.exp_avg = guard.alloc(off, torch.float32, self.device, zero=True, label="flat exp_avg")
        self.exp_avg_sq = guard.alloc(off, torch.float32, self.device, zero=True, label="flat exp_avg_sq")
        self.order = order
        for p in order:
            o = self.offsets[id(p)]
            view = self.params[o:o + p.numel()].view_as(p)
            view.copy_(p.data.to(self.device))
            p.data = view
        # BN buffers
        bns: List[nn.BatchNorm2d] = []
        seen = set()
        for grp in bn_groups:
            for m in grp:
                if id(m) not in seen:
                    bns.append(m)
                    seen.add(id(m))
        for m in module.modules():
            if isinstance(m, nn.BatchNorm2d) and id(m) not in seen:
                bns.append(m)
                seen.add(id(m))
        self.bn_offsets: Dict[int, int] = {}
        off = 0
        for m in bns:
            self.bn_offsets[id(m)] = off
            off += pad_to(m.num_features, 4)
        self.bn_mean = guard.alloc(off, torch.float32, self.device, zero=True, label="bn running mean")
        self.bn_var = guard.alloc(off, torch.float32, self.device, label="bn running var").fill_(1.0)
        self.bn_nbt = guard.alloc(len(bns), torch.int64, self.device, zero=True, label="bn num_batches_tracked")
        self.bn_index = {id(m): i for i, m in enumerate(bns)}
        self.bns = bns
        for m in bns:
            o, c = self.bn_offsets[id(m)], m.num_features
            rm = self.bn_mean[o:o + c]
            rv = self.bn_var[o:o + c]
            nb = self.bn_nbt[self.bn_index[id(m)]:self.bn_index[id(m)] + 1].view(())
            rm.copy_(m.running_mean.to(self.device))
            rv.copy_(m.running_var.to(self.device))
            nb.copy_(m.num_batches_tracked.to(self.device))
            m.running_mean = rm
            m.running_var = rv
            m.num_batches_tracked = nb
        # SyncBN (engine.lowering enable_sync_bn): BN batch statistics span this many ranks; every BNLayer
        # of the program registers itself here
        self.bn_world = 1
        self.bn_layers: List["BNLayer"] = []
        # Adam device scalars: [lr, step]
        self.lr = guard.alloc(1, torch.float32, self.device, zero=True, label="lr")
        self.step = guard.alloc(1, torch.float32, self.device, zero=True, label="adam step")

    def off(self, p: nn.Parameter) -> int:
        return self.offsets[id(p)]

    def grad_of(self, p: nn.Parameter) -> torch.Tensor:
        o = self.off(p)
        return self.grads[o:o + p.numel()].view_as(p)

    def group_stride(self, ps: Sequence[nn.Parameter]) -> int:
        """Element stride between consecutive members of a layer group (0 for a single member)."""
        if len(ps) == 1:
            return 0
        o = [self.off(p) for p in ps]
        st = o[1] - o[0]
        if any(o[i + 1] - o[i] != st for i in range(len(o) - 1)):
            raise ValueError("parameter group is not evenly strided in the flat buffer")
        return st

    def bn_stride(self, ms: Sequence[nn.BatchNorm2d]) -> int:
        if len(ms) == 1:
            return 0
        o = [self.bn_offsets[id(m)] for m in ms]
        st = o[1] - o[0]
        idx = [self.bn_index[id(m)] for m in ms]
        if any(o[i + 1] - o[i] != st for i in range(len(o) - 1)) or any(idx[i + 1] - idx[i] != 1 for i in range(len(o) - 1)):
            raise ValueError("BN group is not evenly strided")
        # gamma/beta share the stride of the parameters; both must agree
        return st

    def sync_module_grads(self):
        """Expose the flat gradients as ``p.grad`` (views, no copy) -- for inspection/tests."""
        for p in self.order:
            p.grad = self.grad_of(p)


class Arena:
    """Persistent device buffers for one lowered program.  ``zeroed`` buffers live in a single region
    that is cleared with one memset at the start of every step (BN statistic accumulators, backward
    workspaces, metric counters)."""

    def __init__(self, device):
        self.device = torch.device(device)
        self._zero_specs: List[tuple] = []
        self._zero: Dict[torch.dtype, torch.Tensor] = {}
        self.views: List[torch.Tensor] = []

    def empty(self, shape, dtype=torch.bfloat16) -> torch.Tensor:
        return guard.alloc(shape, dtype, self.device, label=f"arena {tuple(shape)} {dtype}")

    def zeros(self, shape, dtype=torch.bfloat16) -> torch.Tensor:
        return guard.alloc(shape, dtype, self.device, zero=True, label=f"arena {tuple(shape)} {dtype}")

    def zeroed(self, shape, dtype=torch.float32) -> "LazyView":
        lv = LazyView(tuple(int(s) for s in shape), dtype)
        self._zero_specs.append(lv)
        return lv

    def finalize(self):
        if guard.enabled():  # every zeroed view in its own guarded buffer (cleared one by one)
            for v in self._zero_specs:
                v.bind(guard.alloc(v.shape, v.dtype, self.device, zero=True, label=f"zeroed {v.shape} {v.dtype}"))
            self._zero = {}
            return
        # one backing buffer per dtype (fp64 BN replica sums, fp32 workspaces, int32 counters)
        for dt in sorted({v.dtype for v in self._zero_specs}, key=str):
            specs = [v for v in self._zero_specs if v.dtype == dt]
            n_tot = sum(pad_to(int(np.prod(v.shape)), 64) for v in specs)
            buf = torch.zeros(max(n_tot, 64), device=self.device, dtype=dt)
            self._zero[dt] = buf
            o = 0
            for v in specs:
                n = int(np.prod(v.shape))
                v.bind(buf[o:o + n].view(v.shape))
                o += pad_to(n, 64)

    def zero_ranges(self):
        """(pointer, bytes) of the zeroed backing buffers, for a kernel that clears them itself (the batch
        gather); None under the guard allocator (banded per-view buffers: use clear())."""
        if guard.enabled() or len(self._zero) > 4:
            return None
        return [(b.data_ptr(), b.numel() * b.element_size()) for b in self._zero.values()]

    def clear(self):
        if guard.enabled():
            for v in self._zero_specs:
                v.t.zero_()
            return
        for buf in self._zero.values():
            buf.zero_()


class LazyView:
    """Placeholder for a slice of the arena's zeroed region (bound by ``Arena.finalize``)."""

    def __init__(self, shape, dtype):
        self.shape = shape
        self.dtype = dtype
        self.t: Optional[torch.Tensor] = None

    def bind(self, t):
        self.t = t

    def __getattr__(self, k):
        if k in ("shape", "dtype", "t", "bind"):
            raise AttributeError(k)
        return getattr(self.t, k)


def P(x, off: int = 0) -> int:
    """Device pointer of a tensor / LazyView (+ element offset)."""
    if x is None:
        return 0
    t = x.t if isinstance(x, LazyView) else x
    return t.data_ptr() + off * t.element_size()


# ------------------------------------------------------------------------------------------------
@dataclass
class Act:
    """A bf16 NHWC activation (possibly a channel slice of a wider buffer, possibly per-group)."""
    t: torch.Tensor          # backing buffer
    off: int                 # element offset of channel 0 of group 0 / pixel 0
    ld: int                  # pixel pitch (elements)
    C: int                   # channels
    gs: int = 0              # element stride between groups (0 = shared by all groups)
    B: int = 0
    H: int = 0
    W: int = 0

    @property
    def p(self) -> int:
        return P(self.t, self.off)

    @property
    def M(self) -> int:
        return self.B * self.H * self.W

    def slice(self, c0: int, C: int) -> "Act":
        return Act(self.t, self.off + c0, self.ld, C, self.gs, self.B, self.H, self.W)


def new_act(arena: Arena, G: int, B: int, H: int, W: int, C: int, dtype=torch.bfloat16, shared=False) -> Act:
    t = arena.empty((G, B * H * W, C), dtype)
    return Act(t, 0, C, C, 0 if (shared or G == 1) else B * H * W * C, B, H, W)


def src_dict(a: Act, b: Optional[Act] = None) -> dict:
    d = {"p0": a.p, "gs0": a.gs, "ld0": a.ld, "C0": a.C, "C1": 0}
    if b is not None:
        d.update({"p1": b.p, "gs1": b.gs, "ld1": b.ld, "C1": b.C})
    return d


def gsrc(x, off: int, gs: int, ld: int) -> tuple:
    return (P(x, off), gs, ld)


def grads_of(acts: Sequence[Act]) -> List[tuple]:
    return [(a.p, a.gs, a.ld) for a in acts]


# ------------------------------------------------------------------------------------------------
class BNLayer:
    """Training-mode BatchNorm state for one BN module or a group of identically shaped per-task BNs."""

    # upper bound of the backward replica count: every backward consumer block (BN-tail apply, fused dgrad
    # prologue) reads pnrep x 3 x C fp64, every producer spreads its atomics over them.  Same box, interleaved
    # (docs/PERF.md round 5): 32 / 16 / 8 -> A 35,403 / 35,556 / 35,483 (4 pairs), C 9,331 / 9,410 / 9,439 (3)
    PNREP_MAX = 16

    def __init__(self, mods: Sequence[nn.BatchNorm2d], flat: FlatState, arena: Arena, count: int,
                 stats_share: Optional[tuple] = None):
        """``stats_share`` = (combined replica buffer [G][NREP][2][W], channel offset, W): the forward sums of this
        BN are produced by a horizontally fused conv (ConvLayer ``concat``) whose output channels feed several
        BNs -- its epilogue writes one combined replica buffer, and this BN reads its W-pitched channel range."""
        self.mods = list(mods)
        self.G = len(mods)
        m0 = mods[0]
        self.C = m0.num_features
        self.eps = float(m0.eps)
        self.momentum = float(m0.momentum if m0.momentum is not None else 0.1)
        self.M = count                      # pixels per channel of this rank's batch
        self.count = count * flat.bn_world  # elements per channel of the (Sync)BN batch statistics
        self.flat = flat
        flat.bn_layers.append(self)
        self.pstride = flat.group_stride([m.weight for m in mods])
        rs = flat.bn_stride(mods)
        if self.G > 1 and rs != self.pstride:
            raise ValueError("BN running-stat stride must equal the affine-parameter stride")
        # fp64 replica sums: summation order no longer perturbs results (csrc/common.h BNArgs::stats)
        if stats_share is None:
            self.stats, self.stats_off, self.sld = arena.zeroed((self.G, NREP, 2, self.C), torch.float64), 0, self.C
        else:
            self.stats, self.stats_off, self.sld = stats_share
        # backward: fp64 replica sums of the 2-D tiled BN backward (csrc/bn.hip bnb_*), zeroed per step
        self.nchunk, self.chunk_px = bnb_plan(count, self.C, self.G)
        self.part = arena.zeroed((self.G, NREP, 3, self.C), torch.float64)
        # batch constants (scale, shift, mean, invstd) published by the forward tail for the backward
        self.consts = arena.empty((self.G, 4, self.C), torch.float32)
        # forward replicas in use: about one per BN_PX_PER_REP pixels (the producing conv then has at most
        # ~16 blocks per replica address), so small maps are not read back as 32 mostly-empty replicas by
        # every consumer block (BN_PX_PER_REP above)
        self.nrep = min(NREP, 1 << max(0, math.ceil(math.log2(max(1, count) / BN_PX_PER_REP))))
        # backward partial sums (bnb reduce chunks, dgrad epilogues): the same count, and every chunk of
        # the reduce pass in a replica of its own when there are few
        self.pnrep = min(self.PNREP_MAX, max(self.nrep, min(NREP, 1 << max(0, math.ceil(math.log2(max(1, self.nchunk)))))))
        self.arena = arena
        self.dzbuf = None
        self.part_off = 0            # element offset of this BN's rows in ``part`` (coalesce_replicas)
        self.coalesced = set()       # {"stats", "part"}: rows live in a buffer shared with sibling BNs

    def used_stats(self):
        """The forward replica rows that hold data (what a SyncBN collective reduces): this BN's region of a
        coalesced buffer, else its first ``nrep`` replicas (all groups for a grouped BN)."""
        t = self.stats.t if hasattr(self.stats, "bind") else self.stats
        if "stats" in self.coalesced:
            return t[self.stats_off:self.stats_off + self.nrep * 2 * self.C]
        return t[0, :self.nrep] if t.shape[0] == 1 else t

    def used_part(self):
        """The backward partial-sum rows that hold data (see used_stats)."""
        t = self.part.t if hasattr(self.part, "bind") else self.part
        if "part" in self.coalesced:
            return t[self.part_off:self.part_off + self.pnrep * 3 * self.C]
        return t[0, :self.pnrep] if t.shape[0] == 1 else t

    def args(self, training: bool) -> dict:
        f = self.flat
        m0 = self.mods[0]
        return {"stats": P(self.stats, self.stats_off), "sld": self.sld,
                "gamma": P(f.params, f.off(m0.weight)), "beta": P(f.params, f.off(m0.bias)),
                "run_mean": P(f.bn_mean, f.bn_offsets[id(m0)]), "run_var": P(f.bn_var, f.bn_offsets[id(m0)]),
                "nbt": P(f.bn_nbt, f.bn_index[id(m0)]), "pstride": self.pstride, "C": self.C, "count": self.count,
                "eps": self.eps, "momentum": self.momentum, "training": 1 if training else 0,
                "consts": P(self.consts), "nrep": self.nrep, "pnrep": self.pnrep}

    def grad_ptrs(self) -> dict:
        f = self.flat
        m0 = self.mods[0]
        return {"dgamma": P(f.grads, f.off(m0.weight)), "dbeta": P(f.grads, f.off(m0.bias)), "pgs": self.pstride}


def coalesce_replicas(bns: Sequence["BNLayer"], which: str, arena: "Arena"):
    """Give the ``which`` ("stats": forward sums, "part": backward partial sums) replica rows of ``bns`` ONE
    contiguous zeroed buffer, each BN's used replicas (nrep / pnrep rows of C) back to back, so that a SyncBN
    step all-reduces them with a single collective (engine/inception.py: the branch-output BNs of an
    Inception block, whose statistics complete together at the block's join).  Kernels index only the used
    replicas of a one-group BN, so the region of each BN is exactly what they touch.  Returns the buffer.
    Must run before the arena is finalized."""
    rows = 2 if which == "stats" else 3
    sizes = []
    for bn in bns:
        if bn.G != 1 or (which == "stats" and bn.sld != bn.C) or which in bn.coalesced:
            raise ValueError("only one-group BNs with their own replica rows can be coalesced")
        sizes.append((bn.nrep if which == "stats" else bn.pnrep) * rows * bn.C)
    buf = arena.zeroed((sum(sizes),), torch.float64)
    off = 0
    for bn, n in zip(bns, sizes):
        if which == "stats":
            bn.stats, bn.stats_off = buf, off
        else:
            bn.part, bn.part_off = buf, off
        bn.coalesced.add(which)
        off += n
    return buf


def stem_pack_geom(m: nn.Conv2d, Hi: int, Wi: int) -> Optional[dict]:
    """Vertical tap packing of a single-channel stem conv (MI355X-specific lowering; csrc/misc.hip gather).

    The engine stores the 1-channel input as 8 bf16 channels so that every conv runs on the 8-channel
    k-groups of the MFMA implicit GEMM; for the stem that makes 7/8 of the reduction dimension zeros
    (Model A: K = 7*7*8 = 392 for 49 real taps).  Instead the gather writes x[h - ph + j][w] into channel j
    (j < KH), and the stem becomes a 1 x KW conv over KH stored channels with vertical padding folded into
    the packing: K = KW * 8 (Model A 416 -> 64 padded, Model C 96 -> 32).  The virtual weight
    [Co][Ci=KH][1][KW] has exactly the memory layout of the real [Co][1][KH][KW], so the packed images,
    the weight-gradient finalize and the checkpoint format are unchanged.  Returns the virtual geometry,
    or None when the conv does not qualify (more than one input channel, KH > 8, groups/dilation)."""
    KH, KW = m.kernel_size
    if m.in_channels != 1 or KH > 8 or m.groups != 1 or m.dilation != (1, 1):
        return None
    sh, sw = m.stride
    ph, pw = m.padding
    Ho = (Hi + 2 * ph - KH) // sh + 1
    Wo = (Wi + 2 * pw - KW) // sw + 1
    if (Ho - 1) * sh >= Hi:  # the packed rows read are h' = oh * sh, all inside the stored image
        return None
    return {"Ci": KH, "KH": 1, "KW": KW, "sh": sh, "sw": sw, "ph": 0, "pw": pw, "Ho": Ho, "Wo": Wo,
            "taps": KH, "off": ph}


class ConvLayer:
    """One convolution (or a group of identically shaped per-task convolutions) lowered to the MFMA
    implicit-GEMM kernels.  Holds the packed bf16 weight images, the wgrad slab and the finalize /
    Adam-pack descriptors.  ``geom`` overrides the module's geometry with a virtual one (stem_pack_geom)."""

    def __init__(self, mods: Sequence[nn.Conv2d], flat: FlatState, arena: Arena, B: int, Hi: int, Wi: int,
                 cin_stored: Optional[int] = None, geom: Optional[dict] = None, concat: bool = False):
        """``concat``: the modules are SIBLING convolutions of one input, lowered as ONE conv whose output
        channels are their concatenation (horizontal fusion: one GEMM with N = sum of Co, one data gradient over
        the concatenated dy, one weight-gradient job) -- Inception's 1x1 branch heads, or Model A's 3x3/s2
        residual conv with its 1x1/s2 projection shortcut.  The first module sets the kernel; every other one
        has the same kernel or is a 1x1 whose window is the kernel's centre tap (same stride, padding reduced
        by the offset: its weights occupy that tap of the packed images, the other taps stay zero).
        ``members`` = [(module, channel offset, tap offset)].  Otherwise the modules are G identically shaped
        per-task copies (grid.z groups)."""
        self.mods = list(mods)
        self.concat = concat
        self.G = 1 if concat else len(mods)
        m = mods[0]
        self.flat = flat
        self.Co, self.Ci = m.out_channels, m.in_channels
        self.members = [(m, 0, 0)]
        if concat:
            self.members, n0 = [], 0
            KH, KW = m.kernel_size
            for x in self.mods:
                dh, dw = (KH - x.kernel_size[0]) // 2, (KW - x.kernel_size[1]) // 2
                centre = x.kernel_size == (1, 1) and KH % 2 == 1 and KW % 2 == 1
                if (x.in_channels != m.in_channels or x.stride != m.stride or x.groups != 1 or x.dilation != (1, 1)
                        or x.bias is not None or x.out_channels % 8 or m.groups != 1
                        or not (x.kernel_size == m.kernel_size or centre)
                        or (x.padding[0] + dh, x.padding[1] + dw) != tuple(m.padding)):
                    raise ValueError("horizontal fusion needs bias-free siblings of one input with Cout % 8 == 0 and "
                                     "the first one's kernel, or 1x1 at its centre tap (same stride, aligned padding)")
                self.members.append((x, n0, dh * KW + dw))
                n0 += x.out_channels
            self.Co = n0
        self.KH, self.KW = m.kernel_size
        self.sh, self.sw = m.stride
        self.ph, self.pw = m.padding
        if m.groups != 1 or m.dilation != (1, 1):
            raise ValueError("grouped / dilated convolutions are not supported")
        self.stem_geom = geom
        self.src_C0, self.src_C1 = None, 0  # input segments, known once the backward is emitted (wgrad_args)
        if geom is not None:
            self.Ci, self.KH, self.KW = geom["Ci"], geom["KH"], geom["KW"]
            self.sh, self.sw, self.ph, self.pw = geom["sh"], geom["sw"], geom["ph"], geom["pw"]
        self.Cs = cin_stored if cin_stored is not None else self.Ci
        if self.Cs % 8 or self.Co % 8:
            raise ValueError(f"channels must be multiples of 8 (Cin stored {self.Cs}, Cout {self.Co})")
        self.B, self.Hi, self.Wi = B, Hi, Wi
        self.Ho = (Hi + 2 * self.ph - self.KH) // self.sh + 1
        self.Wo = (Wi + 2 * self.pw - self.KW) // self.sw + 1
        if geom is not None:
            self.Ho, self.Wo = geom["Ho"], geom["Wo"]
        self.M_out = B * self.Ho * self.Wo
        self.M_in = B * Hi * Wi
        self.has_bias = m.bias is not None
        self.wstride = 0 if concat else flat.group_stride([x.weight for x in mods])
        self.bstride = flat.group_stride([x.bias for x in mods]) if self.has_bias and not concat else 0
        taps = self.KH * self.KW
        self.Npad = pad_to(self.Co, 16)
        self.Kpad = pad_to(taps * self.Cs, 32)
        self.Npad_d = pad_to(self.Cs, 16)
        self.Kpad_d = pad_to(taps * self.Co, 32)
        self.wf = arena.zeros((self.G, self.Npad, self.Kpad))
        self.wd = arena.zeros((self.G, self.Npad_d, self.Kpad_d))
        # weight-gradient decomposition (tile config chosen by the autotuner; the slab is sized for the
        # largest split count any config can ask for)
        self.Kpad_w = pad_to(taps * self.Cs, 64)
        self._wgrad_args = None
        max_splits = max(self.wgrad_plan(c)[0] for c in list(WGRAD_TILES) + list(WGRAD_PATCH) if self.wgrad_valid(c))
        self.slab = arena.empty((self.G, max_splits, self.Npad, self.Kpad_w), torch.float32)
        self.set_wgrad_cfg(wgrad_cfg(self.Co, self.Kpad_w))

    # every split-M block reduces at least this many output pixels: with the weight gradients of all
    # convs batched into one launch (csrc/conv.hip conv_wgrad_batched_kernel) the grid no longer has to
    # be filled by one conv's splits, and each extra split costs a full Npad x Kpad slab read in the
    # finalize (Model C: ~0.9 GB/step of slab traffic with grid-filling splits)
    # (512 / 2048 / 4096 measured within noise on A, C 7.10k at 1024 vs 6.83k at 2048)
    MIN_SPLIT_PX = 1024
    # the large 32x32x16 tiles (configs 32-35) at 256 pixels per split: Model C's batches 624 -> 440 us but
    # the finalize's split slabs 102 -> 197 us; at 1024: 515 us and 103 us (tools/wgrad_assign.py)
    MIN_SPLIT_PX_BIG = 1024
    LEAN_MIN_CHUNKS = 2
    LEAN_BLOCKS = 512
    LEAN_MAX_SPLITS = 64

    def wgrad_valid(self, cfg: int) -> bool:
        """The K tiles of ``cfg`` cover this conv's padded reduction (exactly, except for the large-tile
        configs; patch configs: a 3x3 / s1 / p1 conv whose input channels split into whole CB slices and
        whose rows fit the tile width)."""
        if cfg in WGRAD_PATCH:
            return self.stem_geom is None and patch_valid(cfg, self.Cs, self.KH, self.KW, (self.sh, self.sw),
                                                          (self.ph, self.pw), self.Hi, self.Wi, self.Ho, self.Wo,
                                                          self.src_C0, self.src_C1)
        return wgrad_ktiles(cfg, self.Kpad_w) > 0

    def wgrad_plan(self, cfg: int):
        if cfg in WGRAD_PATCH:
            # splits sized for ~128 blocks per job on Model A's layers (32 / 64 / 256 measured slower there);
            # the wide-row configs (128-pixel rows: Model C's 47x122 / 21x58 stem layers) fill the GPU with
            # ~512 blocks (tools/wgrad_cfg_sweep.py: 47x122 32->64 29 us at 512 blocks vs 53 us at 128)
            wide = WGRAD_PATCH[cfg][2] >= 128
            return patch_plan(cfg, self.B, self.Ho, self.Npad, self.Cs, self.G, 512 if wide else 128)
        TN, TK, MCH = WGRAD_TILES[cfg]
        tiles = math.ceil(self.Npad / TN) * wgrad_ktiles(cfg, self.Kpad_w) * self.G
        if WGRAD_LEAN0 <= cfg < WGRAD_LEAN0 + WGRAD_LEAN_N:
            # lean staging (csrc/wgrad_lean.hip) is bound by the load latency of its serial chunks: ~LEAN_BLOCKS
            # blocks per job, at least LEAN_MIN_CHUNKS chunks each, at most LEAN_MAX_SPLITS split slabs for the
            # finalize to sum (it runs on the step's tail)
            splits = max(1, min(math.ceil(self.M_out / (self.LEAN_MIN_CHUNKS * MCH)), math.ceil(self.LEAN_BLOCKS / tiles),
                                self.LEAN_MAX_SPLITS))
            mps = pad_to(math.ceil(self.M_out / splits), MCH)
            return math.ceil(self.M_out / mps), mps
        # whole-reduction tiles (TK >= 128) have one tile per channel block: shorter per-block pixel
        # ranges keep enough blocks in flight (the finalize sums the extra splits with several lanes)
        if cfg >= WGRAD_BIG0:
            min_px = self.MIN_SPLIT_PX_BIG
        else:
            min_px = self.MIN_SPLIT_PX // 2 if TK >= 128 else self.MIN_SPLIT_PX
        splits = max(1, min(math.ceil(self.M_out / MCH), math.ceil(512 / tiles),
                            math.ceil(self.M_out / min_px)))
        mps = pad_to(math.ceil(self.M_out / splits), MCH)
        return math.ceil(self.M_out / mps), mps

    def set_wgrad_cfg(self, cfg: int):
        self.wcfg = cfg
        self.splits, self.m_per_split = self.wgrad_plan(cfg)
        if self._wgrad_args is not None:
            self._wgrad_args.update(splits=self.splits, m_per_split=self.m_per_split)

    def fwd_cfg(self, N: int, M: int) -> int:
        if N <= 16:
            return 0
        if N <= 32:
            return 1
        if N <= 64:
            return 2 if M >= 64 * 256 else 4
        return 3 if M >= 64 * 128 else 4

    # ---- packed weight images / optimizer descriptors ------------------------------------------
    def opt_segments(self) -> List[dict]:
        """Optimizer jobs (csrc/optim.hip adam_pack_kernel, kind 3): every member weight's Adam update and
        its forward and data-gradient bf16 images, rebuilt from the updated fp32 masters each step."""
        segs = []
        if self.concat:
            # member rows [n0, n0 + Co) of the forward image, its taps at the group's tap offset t0 (a centre-tap
            # 1x1 writes the Cs columns of that tap only); its columns n0.. of each tap of the data-gradient image
            # (tap stride = the group's Co)
            for m, n0, t0 in self.members:
                kh, kw = m.kernel_size
                segs.append({"kind": 3, "off": self.flat.off(m.weight), "n": m.weight.numel(), "Co": m.out_channels,
                             "Ci": self.Ci, "KH": kh, "KW": kw, "Cs": self.Cs, "Kpad_f": self.Kpad,
                             "Kpad_d": self.Kpad_d, "tap_ld": self.Co, "kext_f": kh * kw * self.Cs if t0 else 0,
                             "wf": P(self.wf, n0 * self.Kpad + t0 * self.Cs), "wd": P(self.wd, t0 * self.Co + n0)})
            return segs
        for g, m in enumerate(self.mods):
            segs.append({"kind": 3, "off": self.flat.off(m.weight), "n": m.weight.numel(), "Co": self.Co, "Ci": self.Ci,
                         "KH": self.KH, "KW": self.KW, "Cs": self.Cs, "Kpad_f": self.Kpad, "Kpad_d": self.Kpad_d,
                         "wf": P(self.wf, g * self.Npad * self.Kpad), "wd": P(self.wd, g * self.Npad_d * self.Kpad_d)})
        return segs

    def finalize_descs(self) -> List[dict]:
        """Finalize descriptors: one per member of a horizontally fused conv (its slab rows [n0, n0 + Co) into its
        own weight's gradient), else the conv's one."""
        if not self.concat:
            return [self.finalize_desc()]
        return [{"slab": P(self.slab, n0 * self.Kpad_w + t0 * self.Cs), "grad": P(self.flat.grads, self.flat.off(m.weight)),
                 "ggs": 0, "G": 1, "splits": self.splits, "Npad": self.Npad, "Kpad": self.Kpad_w, "Co": m.out_channels,
                 "Ci": self.Ci, "Cs": self.Cs, "KH": m.kernel_size[0], "KW": m.kernel_size[1],
                 "elems": m.out_channels * self.Ci * m.kernel_size[0] * m.kernel_size[1]}
                for m, n0, t0 in self.members]

    def finalize_desc(self) -> dict:
        m0 = self.mods[0]
        return {"slab": P(self.slab), "grad": P(self.flat.grads, self.flat.off(m0.weight)), "ggs": self.wstride,
                "G": self.G, "splits": self.splits, "Npad": self.Npad, "Kpad": self.Kpad_w, "Co": self.Co,
                "Ci": self.Ci, "Cs": self.Cs, "KH": self.KH, "KW": self.KW,
                "elems": self.G * self.Co * self.KH * self.KW * self.Ci}

    # ---- launches --------------------------------------------------------------------------------
    def fwd_args(self, src: dict, out: Act, bn: Optional[BNLayer], training: bool) -> tuple:
        f = self.flat
        d = {"src": src, "w": P(self.wf), "wgs": self.Npad * self.Kpad if self.G > 1 else 0,
             "bias": P(f.params, f.off(self.mods[0].bias)) if self.has_bias else 0, "bgs": self.bstride,
             "out": out.p, "ogs": out.gs, "ldo": out.ld,
             "stats": P(bn.stats, bn.stats_off) if (bn is not None and training) else 0,
             "stats_nrep": bn.nrep if bn is not None else NREP,
             "B": self.B, "Hs": self.Hi, "Ws": self.Wi, "Ho": self.Ho, "Wo": self.Wo, "N": self.Co, "Npad": self.Npad,
             "Cs": self.Cs, "KH": self.KH, "KW": self.KW, "sh": self.sh, "sw": self.sw, "ph": self.ph, "pw": self.pw,
             "Kpad": self.Kpad}
        return (0, self.fwd_cfg(self.Co, self.M_out), self.G, d)

    def dgrad_args(self, dy: Act, dx_out: Act) -> tuple:
        d = {"src": src_dict(dy), "w": P(self.wd), "wgs": self.Npad_d * self.Kpad_d if self.G > 1 else 0,
             "out": dx_out.p, "ogs": dx_out.gs, "ldo": dx_out.ld,
             "B": self.B, "Hs": self.Ho, "Ws": self.Wo, "Ho": self.Hi, "Wo": self.Wi, "N": self.Cs, "Npad": self.Npad_d,
             "Cs": self.Co, "KH": self.KH, "KW": self.KW, "sh": self.sh, "sw": self.sw, "ph": self.ph, "pw": self.pw,
             "Kpad": self.Kpad_d}
        return (1, self.fwd_cfg(self.Cs, self.M_in), self.G, d)

    def wgrad_args(self, src: dict, dy: Act) -> tuple:
        self.src_C0, self.src_C1 = src.get("C0"), src.get("C1", 0)
        self._wgrad_args = d = {"src": src, "dy": dy.p, "dgs": dy.gs, "ldd": dy.ld, "slab": P(self.slab), "splits": self.splits,
             "m_per_split": self.m_per_split, "B": self.B, "Hi": self.Hi, "Wi": self.Wi, "Ho": self.Ho, "Wo": self.Wo,
             "Co": self.Co, "Npad": self.Npad, "Cs": self.Cs, "KH": self.KH, "KW": self.KW, "sh": self.sh,
             "sw": self.sw, "ph": self.ph, "pw": self.pw, "Kpad": self.Kpad_w}
        return (self.wcfg, self.G, d)


# ------------------------------------------------------------------------------------------------
# descriptor tables (uploaded once; read by wgrad_finalize / adam_pack)
def finalize_lanes(splits: int) -> int:
    """Threads per weight in wgrad_finalize: about 8 splits per thread, a power of two <= 16."""
    lanes = 1
    while lanes < 16 and splits > 8 * lanes:
        lanes *= 2
    return lanes


# convs with at most this many wgrad splits are finalized in output order (contiguous gradient stores);
# more splits: slab order with several lanes per weight (coalesced split reads); 0 / 2 / 8 swept (docs/PERF.md)
FIN_OUT_MAX_SPLITS = 2


def build_wgfin_table(descs: List[dict], device) -> tuple:
    """Pack WgFinDesc structs (layout must match csrc/kernels.h)."""
    dt = np.dtype([("slab", "<u8"), ("grad", "<u8"), ("ggs", "<i8"), ("G", "<i4"), ("splits", "<i4"),
                   ("Npad", "<i4"), ("Kpad", "<i4"), ("Co", "<i4"), ("Ci", "<i4"), ("Cs", "<i4"), ("KH", "<i4"),
                   ("KW", "<i4"), ("lanes", "<i4"), ("order", "<i4"), ("_pad", "<i4"), ("elems", "<i8"),
                   ("block0", "<i8")])
    assert dt.itemsize == lib().SIZEOF_WGFIN, (dt.itemsize, lib().SIZEOF_WGFIN)
    arr = np.zeros(len(descs), dtype=dt)
    b0 = 0
    for i, d in enumerate(descs):
        for k, v in d.items():
            arr[i][k] = v
        lanes = finalize_lanes(d["splits"])
        arr[i]["block0"] = b0
        if d["splits"] <= FIN_OUT_MAX_SPLITS:  # output order, one lane, FIN_EPT weights per thread
            arr[i]["lanes"], arr[i]["order"] = 1, 1
            b0 += math.ceil(d["elems"] / (256 * lib().FIN_EPT))
        else:  # slab-order mapping (csrc/conv.hip wgrad_finalize_kernel): padded channels included
            arr[i]["lanes"] = lanes
            arr[i]["elems"] = d["G"] * d["Co"] * d["KH"] * d["KW"] * d["Cs"]
            b0 += math.ceil(int(arr[i]["elems"]) * lanes / 256)
    t = torch.from_numpy(arr.view(np.uint8).copy()).to(device)
    return t, len(descs), b0


PACK_TCO, PACK_TILE_FLOATS = 8, 512  # csrc/kernels.h


def pack_tile_ci(taps: int) -> int:
    return max(8, (256 // taps) & ~7)


def optimizer_segments(conv_segs: List[dict], numel: int) -> List[dict]:
    """The fused optimizer's segments: the conv weights' tiles (kind 3) plus plain Adam ranges (kind 0)
    covering every other element of the flat buffer, each element exactly once, in flat order."""
    segs, pos = [], 0
    for s in sorted(conv_segs, key=lambda s: s["off"]):
        if s["off"] < pos:
            raise ValueError(f"optimizer segments overlap at flat offset {s['off']}")
        if s["off"] > pos:
            segs.append({"kind": 0, "off": pos, "n": s["off"] - pos})
        segs.append(s)
        pos = s["off"] + s["n"]
    if pos > numel:
        raise ValueError("optimizer segments run past the flat buffer")
    if pos < numel:
        segs.append({"kind": 0, "off": pos, "n": numel - pos})
    return segs


def build_optseg_table(segs: List[dict], device) -> tuple:
    dt = np.dtype([("off", "<i8"), ("n", "<i8"), ("kind", "<i4"), ("_pad0", "<i4"), ("wf", "<u8"), ("wd", "<u8"),
                   ("Co", "<i4"), ("Ci", "<i4"), ("KH", "<i4"), ("KW", "<i4"), ("Cs", "<i4"), ("Kpad_f", "<i4"),
                   ("Kpad_d", "<i4"), ("kext_f", "<i4"), ("tap_ld", "<i4"), ("_pad1", "<i4"), ("block0", "<i8")])
    assert dt.itemsize == lib().SIZEOF_OPTSEG, (dt.itemsize, lib().SIZEOF_OPTSEG)
    arr = np.zeros(len(segs), dtype=dt)
    b0 = 0
    for i, s in enumerate(segs):
        for k, v in s.items():
            arr[i][k] = v
        arr[i]["block0"] = b0
        if s["kind"] == 0:  # plain Adam range, 1024 elements per block
            b0 += math.ceil(s["n"] / 1024)
        else:  # (8 co) x (ci tile) x all taps through LDS (csrc/optim.hip adam_pack_kernel)
            taps = s["KH"] * s["KW"]
            if 8 * taps > PACK_TILE_FLOATS:
                raise ValueError(f"pack: {taps} taps exceed the {PACK_TILE_FLOATS}-float LDS tile")
            if s["n"] != s["Co"] * s["Ci"] * taps:
                raise ValueError("pack: a conv segment must cover its whole weight")
            b0 += math.ceil(s["Co"] / PACK_TCO) * math.ceil(s["Ci"] / pack_tile_ci(taps))
    t = torch.from_numpy(arr.view(np.uint8).copy()).to(device)
    return t, len(segs), b0
