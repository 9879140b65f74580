"""Lowering of the Inception-v3 multi-classifier (reference Model C, modelC_multiClassifier.py:28-172).

The network is lowered as a DAG of *values* (bf16 NHWC activations).  Every ``BasicConv2d`` becomes
one MFMA implicit-GEMM conv (BN sums fused into its epilogue) plus one fused BN+ReLU tail; the Inception
pools are the 3x3 pool kernels.  There is no concatenation: the branches of a block write their
outputs straight into channel slices of the block's output buffer (the tail / pool output pitch is the
concat width), and the next block's convs read that buffer in place.

Backward walks the ops in reverse.  Each consumer of a value writes the gradient w.r.t. its input ONCE
into its own bf16 buffer and registers it as a *gradient source* of the value; the producing kernel
(the BN-tail backward, or the pool backward) sums the sources on load.  A branch output that lives in a
slice of a concat buffer gets the matching channel slices of the concat value's sources, so the
concat backward is free as well.  The classifier (GAP -> Dropout -> Linear -> CE) is the fused
``cls_head`` kernel (csrc/head.hip) which also writes d(fc) into the flat gradient buffer.

Launch counts per training step (B fixed): forward 94 conv + 94 tails + 13 pools + head, backward
94 tail-bwd + 94 wgrad + 93 dgrad + 13 pool-bwd + one finalize, one fused Adam.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import torch

from ..models.multi_classifier import (BasicConv2d, InceptionA, InceptionB, InceptionC, InceptionD, InceptionE,
                                       Multi_Classifier)
from . import guard
from .core import (GRAD_DT, NREP, Act, Arena, BNLayer, ConvLayer, FlatState, P, coalesce_replicas, grads_of, new_act,
                   src_dict, stem_pack_geom)
from .lowering import ACT_RELU, LoweredProgram
from ..ops.hip import lib
from .program import Phase, k_allreduce, k_cls_head, k_pool, k_wgfin


class Val:
    """A bf16 activation of the lowered graph and the bf16 gradient sources its consumers register.
    ``parent``/``coff``: this value is channels [coff, coff+C) of a concat value."""

    def __init__(self, act: Act, parent: "Val" = None, coff: int = 0, needs_grad: bool = True):
        self.act = act
        self.parent = parent
        self.coff = coff
        self.needs_grad = needs_grad
        self.grads: List[Act] = []

    def grad_sources(self) -> List[Act]:
        g = list(self.grads)
        if self.parent is not None:
            g += [a.slice(self.coff, self.act.C) for a in self.parent.grad_sources()]
        if not g or len(g) > 6:
            raise RuntimeError(f"value has {len(g)} gradient sources (1..6 supported)")
        return g


class CBR:
    """conv -> BN -> ReLU (one BasicConv2d).  ``fused`` = (HConv, channel offset): the conv is a member of a
    horizontally fused sibling group -- the HConv op runs it, this op is the member's BN + ReLU only (its y / dy
    are channel slices of the group's buffers, its BN sums a slice of the group's replica rows)."""

    def __init__(self, prog: "InceptionProgram", bc: BasicConv2d, src: Val, out: Val, geom: Optional[dict] = None,
                 fused: Optional[tuple] = None):
        A, B, f = prog.arena, prog.B, prog.flat
        self.src, self.out = src, out
        self.module = bc
        s = src.act
        self.fused = fused
        if fused is not None:
            hc, n0 = fused
            self.conv = None
            Ho, Wo, Co = hc.conv.Ho, hc.conv.Wo, bc.conv.out_channels
            self.bn = BNLayer([bc.bn], f, A, B * Ho * Wo, stats_share=(hc.stats, n0, hc.conv.Co))
            self.y, self.dy, self.dx = hc.y.slice(n0, Co), hc.dy.slice(n0, Co), None
        else:
            self.conv = c = ConvLayer([bc.conv], f, A, B, s.H, s.W, cin_stored=s.C, geom=geom)
            Ho, Wo, Co = c.Ho, c.Wo, c.Co
            self.bn = BNLayer([bc.bn], f, A, B * Ho * Wo)
            self.y = new_act(A, 1, B, Ho, Wo, Co)
            self.dy = new_act(A, 1, B, Ho, Wo, Co)
            self.dx = new_act(A, 1, B, s.H, s.W, s.C, GRAD_DT) if src.needs_grad else None
        if (Ho, Wo, Co) != (out.act.H, out.act.W, out.act.C):
            raise ValueError(f"shape mismatch lowering {bc}: conv gives {(Ho, Wo, Co)}, "
                             f"destination {(out.act.H, out.act.W, out.act.C)}")
        self.nol_from: Optional["CBR"] = None  # producer whose BN+ReLU this conv applies on load
        self.skip_tail = False                 # the (single) consumer normalises self.y on load
        self.defer_tail = False                # the tail joins its block's batched tail launch

    def _src(self):
        if self.nol_from is not None:
            return src_dict(self.nol_from.y), (self.nol_from.bn, ACT_RELU)
        return src_dict(self.src.act), None

    def forward(self, prog, ph: Phase, training: bool):
        if self.conv is not None:
            src, nol = self._src()
            prog._conv_fwd(ph, self.conv, src, self.y, self.bn, training, nol=nol)
        if self.defer_tail:
            prog._pending_tails.append(prog._tail_args(self.y, self.bn, self.out.act, training))
        elif not self.skip_tail:
            prog._tail(ph, ACT_RELU, 1, self.y, self.bn, self.out.act, training)

    def backward(self, prog, ph: Phase):
        prog._tail_bwd(ph, ACT_RELU, 1, self.y, self.bn, grads_of(self.out.grad_sources()), self.dy)
        if self.defer_tail:  # a block-output tail: InceptionProgram.batch_tails may batch its backward too
            ph.launches[-1].owner = self
        if self.conv is None:  # a fused member: its HConv's data / weight gradient run over the group's dy
            return
        src, nol = self._src()
        prog._conv_bwd(ph, self.conv, src, self.dy, self.dx, nol=nol)
        if self.dx is not None:
            self.src.grads.append(self.dx)


class HConv:
    """Horizontal fusion of sibling 1x1 BasicConv2d convs that read the same input (an Inception block's
    branch1x1 / branchNxN_1 heads, reference modelC_multiClassifier.py:70-83 via torchvision InceptionA/C/D/E):
    ONE implicit GEMM with N = sum of the members' Cout writes their pre-BN outputs side by side (each member's
    BN sums land in its slice of one combined replica buffer), and in the backward ONE data gradient over the
    concatenated dy (K = sum of Cout) replaces the members' separate data gradients -- and their separate
    gradient sources of the input -- plus one weight-gradient job for all of them.  The members' BN + ReLU
    tails (and their backward) stay per member, on their branches' streams (``CBR`` with ``fused``)."""

    def __init__(self, prog: "InceptionProgram", bcs: List[BasicConv2d], src: Val):
        A, B, f = prog.arena, prog.B, prog.flat
        self.src = src
        s = src.act
        self.conv = c = ConvLayer([bc.conv for bc in bcs], f, A, B, s.H, s.W, cin_stored=s.C, concat=True)
        self.stats = A.zeroed((1, NREP, 2, c.Co), torch.float64)
        self.y = new_act(A, 1, B, c.Ho, c.Wo, c.Co)
        self.dy = new_act(A, 1, B, c.Ho, c.Wo, c.Co)
        self.dx = new_act(A, 1, B, s.H, s.W, s.C, GRAD_DT) if src.needs_grad else None
        self.members: List[CBR] = []  # filled by InceptionProgram._hconv

    def forward(self, prog, ph: Phase, training: bool):
        # the members' BNs share the combined replica buffer: any member's layer names it (offset 0 = base)
        prog._conv_fwd(ph, self.conv, src_dict(self.src.act), self.y, self.members[0].bn, training)

    def backward(self, prog, ph: Phase):
        prog._conv_bwd(ph, self.conv, src_dict(self.src.act), self.dy, self.dx)
        if self.dx is not None:
            self.src.grads.append(self.dx)


class Pool:
    """maxpool 3x3/s2 (valid) or avgpool 3x3/s1/p1 (count_include_pad)."""

    def __init__(self, prog: "InceptionProgram", is_max: bool, src: Val, out: Val):
        self.is_max, self.src, self.out = int(is_max), src, out
        s = src.act
        Ho, Wo = ((s.H - 3) // 2 + 1, (s.W - 3) // 2 + 1) if is_max else (s.H, s.W)
        if (Ho, Wo, s.C) != (out.act.H, out.act.W, out.act.C):
            raise ValueError("pool output shape mismatch")
        self.dx = new_act(prog.arena, 1, prog.B, s.H, s.W, s.C, GRAD_DT) if src.needs_grad else None
        # max pool: the training forward stores each output's window argmax (1 byte) for the backward
        self.am = None
        if is_max and self.dx is not None:
            self.am = prog.arena.zeros((prog.B * Ho * Wo * s.C,), torch.uint8)

    def _geom(self, B):
        s, o = self.src.act, self.out.act
        return {"x": s.p, "ldx": s.ld, "B": B, "H": s.H, "W": s.W, "C": s.C, "Ho": o.H, "Wo": o.W}

    def forward(self, prog, ph: Phase, training: bool):
        d = dict(self._geom(prog.B), y=self.out.act.p, ldy=self.out.act.ld)
        if training and self.am is not None:
            d["am"] = P(self.am)
        ph.add("pool_fwd", k_pool, self.is_max, 0, d)

    def backward(self, prog, ph: Phase):
        if self.dx is None:
            return
        d = dict(self._geom(prog.B), g=grads_of(self.out.grad_sources()), dx=self.dx.p, lddx=self.dx.ld)
        if self.am is not None:
            d["am"] = P(self.am)
        ph.add("pool_bwd", k_pool, self.is_max, 1, d)
        self.src.grads.append(self.dx)


def _mixed6_hw(in_hw):
    """Spatial size of Mixed_6a..6e's output for an input of ``in_hw`` (valid 3x3/s2 stem conv, two valid
    3x3 convs... as in modelC_multiClassifier.py:63-86)."""
    def s2(x):
        return (x - 3) // 2 + 1
    out = []
    for x in in_hw:
        x = s2(x) - 2       # Conv2d_1a (s2), Conv2d_2a; 2b keeps the size (pad 1)
        x = s2(x) - 2       # maxpool1, Conv2d_3b (1x1), Conv2d_4a
        x = s2(s2(x))       # maxpool2, Mixed_6a (s2)
        out.append(x)
    return tuple(out)


class InceptionProgram(LoweredProgram):
    """Static train/eval programs of a :class:`Multi_Classifier` for a fixed per-GPU batch size."""

    label_width = 1  # joint label (distance + 16 * event)
    # DP: 4 buckets of ~22 MB cut at Inception-block boundaries (fc+Mixed_7c, 7b, 7a-6c, the rest); the
    # first three all-reduces overlap the remaining blocks' backward
    default_buckets = 4
    # the step counter stays after the last Adam launch here: on the forward's first side stream it cost Model C
    # 0.7 % (9,567 / 9,566 vs 9,629 / 9,634 samples/s, interleaved; Model A +0.3 %, docs/PERF.md round 6)
    EARLY_STEP_COUNTER = False
    # module order puts the stem (stream 0) first: build_for_stream_buckets rebuilds with stream_param_order
    REORDER_FOR_STREAM_BUCKETS = True

    def __init__(self, model: Multi_Classifier, batch: int, device, in_hw=(100, 250), p_drop: float = 0.5,
                 sync_world: int = 1, param_order=None):
        """``param_order``: parameters laid out first in the flat buffers, in this order (LoweredProgram.
        stream_param_order); the rest follow in module order."""
        if model.aux_logits:
            h6 = _mixed6_hw(in_hw)
            if min(h6) < 5:
                # InceptionAux opens with avg_pool(5, stride 3) on Mixed_6e's output, 4 x 13 for the DAS input
                # (100 x 250): the reference model (modelC_multiClassifier.py:78-80,134-141) raises in
                # F.avg_pool2d at such a shape, so there is no trainable configuration to lower
                raise ValueError(f"aux_logits=True: InceptionAux needs >= 5 x 5 at Mixed_6e, input {tuple(in_hw)} gives "
                                 f"{h6[0]} x {h6[1]} (the reference raises in avg_pool2d too); use aux_logits=False")
            raise NotImplementedError("aux_logits=True is lowered only by the torch backend (the reference trains "
                                      "without it)")
        if model.transform_input:
            raise NotImplementedError("transform_input is not lowered")
        if model.num_classes > 64:
            raise ValueError("the fused classifier head supports at most 64 classes")
        self.model = model
        self.B = batch
        self.device = torch.device(device)
        self.H0, self.W0 = in_hw
        self.cin = model.Conv2d_1a_3x3.conv.in_channels
        if self.cin > 8:
            raise ValueError("in_channels > 8 not supported by the gather kernel")
        self.p_drop = float(p_drop)
        model.to(self.device)
        self.flat = FlatState(model, self.device, [list(param_order)] if param_order else ())
        self.flat.bn_world = sync_world  # SyncBN: global BN counts (enable_sync_bn adds the collectives)
        self.arena = Arena(self.device)
        self._alloc()
        self.arena.finalize()
        self._emit()

    # -------------------------------------------------------------------------------------------
    def _val(self, H, W, C) -> Val:
        return Val(new_act(self.arena, 1, self.B, H, W, C))

    def _at(self, branch: Optional[int]):
        """Subsequent ops belong to ``branch`` of the current block (None: stem / head, stream 0)."""
        self._cur = None if branch is None else (self._bi, branch)

    def _push(self, op):
        self.ops.append(op)
        self.op_meta.append(self._cur)

    def _cbr(self, bc: BasicConv2d, src: Val, out: Optional[Val] = None, geom: Optional[dict] = None) -> Val:
        if out is None:
            kh, kw = bc.conv.kernel_size
            sh, sw = bc.conv.stride
            ph, pw = bc.conv.padding
            H = (src.act.H + 2 * ph - kh) // sh + 1
            W = (src.act.W + 2 * pw - kw) // sw + 1
            out = self._val(H, W, bc.conv.out_channels)
        self._push(CBR(self, bc, src, out, geom))
        return out

    def _pool(self, is_max: bool, src: Val, out: Optional[Val] = None) -> Val:
        if out is None:
            s = src.act
            H, W = ((s.H - 3) // 2 + 1, (s.W - 3) // 2 + 1) if is_max else (s.H, s.W)
            out = self._val(H, W, s.C)
        self._push(Pool(self, is_max, src, out))
        return out

    def hfuse_enabled(self) -> bool:
        """Horizontal fusion of sibling 1x1 convs (HConv; MDA_HFUSE=0 lowers every BasicConv2d on its own)."""
        return os.environ.get("MDA_HFUSE", "1") == "1"

    def _hconv(self, bcs: List[BasicConv2d], src: Val, outs: List[Optional[Val]], branches: List[int]) -> List[Val]:
        """Sibling 1x1 convs ``bcs`` of ``src`` (member i on branch ``branches[i]``, writing ``outs[i]`` or a new
        value): one fused conv (stream 0, before the block's branches fork; in the backward after they join)
        plus per-member BN + ReLU ops on the branches.  Returns the members' output values."""
        if not self.hfuse_enabled():
            vals = []
            for bc, out, b in zip(bcs, outs, branches):
                self._at(b)
                vals.append(self._cbr(bc, src, out))
            return vals
        blk = self._cur
        self._cur = None
        hc = HConv(self, bcs, src)
        self._push(hc)
        vals = []
        for (bc, out, b), (_, n0, _) in zip(zip(bcs, outs, branches), hc.conv.members):
            if out is None:
                out = self._val(hc.conv.Ho, hc.conv.Wo, bc.conv.out_channels)
            self._at(b)
            m = CBR(self, bc, src, out, fused=(hc, n0))
            hc.members.append(m)
            self._push(m)
            vals.append(out)
        self._cur = blk
        return vals

    def _concat(self, H, W, widths) -> tuple:
        cat = self._val(H, W, sum(widths))
        parts, o = [], 0
        for w in widths:
            parts.append(Val(cat.act.slice(o, w), parent=cat, coff=o))
            o += w
        return cat, parts

    def _block(self, blk, x: Val) -> Val:
        """Lower one Inception block; returns its concat output value."""
        H, W = x.act.H, x.act.W
        if isinstance(blk, InceptionA):
            pf = blk.branch_pool.conv.out_channels
            cat, (o1, o5, o3, op) = self._concat(H, W, [64, 64, 96, pf])
            _, h5, h3 = self._hconv([blk.branch1x1, blk.branch5x5_1, blk.branch3x3dbl_1], x, [o1, None, None], [0, 1, 2])
            self._at(1); self._cbr(blk.branch5x5_2, h5, o5)
            self._at(2); self._cbr(blk.branch3x3dbl_3, self._cbr(blk.branch3x3dbl_2, h3), o3)
            self._at(3); self._cbr(blk.branch_pool, self._pool(False, x), op)
        elif isinstance(blk, InceptionB):
            Ho, Wo = (H - 3) // 2 + 1, (W - 3) // 2 + 1
            cat, (o3, od, om) = self._concat(Ho, Wo, [384, 96, x.act.C])
            self._at(0); self._cbr(blk.branch3x3, x, o3)
            self._at(1); self._cbr(blk.branch3x3dbl_3, self._cbr(blk.branch3x3dbl_2, self._cbr(blk.branch3x3dbl_1, x)), od)
            self._at(2); self._pool(True, x, om)
        elif isinstance(blk, InceptionC):
            cat, (o1, o7, od, op) = self._concat(H, W, [192, 192, 192, 192])
            _, h7, hd = self._hconv([blk.branch1x1, blk.branch7x7_1, blk.branch7x7dbl_1], x, [o1, None, None], [0, 1, 2])
            self._at(1); self._cbr(blk.branch7x7_3, self._cbr(blk.branch7x7_2, h7), o7)
            self._at(2)
            v = hd
            for i in range(2, 5):
                v = self._cbr(getattr(blk, f"branch7x7dbl_{i}"), v)
            self._cbr(blk.branch7x7dbl_5, v, od)
            self._at(3); self._cbr(blk.branch_pool, self._pool(False, x), op)
        elif isinstance(blk, InceptionD):
            Ho, Wo = (H - 3) // 2 + 1, (W - 3) // 2 + 1
            cat, (o3, o7, om) = self._concat(Ho, Wo, [320, 192, x.act.C])
            h3, h7 = self._hconv([blk.branch3x3_1, blk.branch7x7x3_1], x, [None, None], [0, 1])
            self._at(0); self._cbr(blk.branch3x3_2, h3, o3)
            self._at(1)
            v = h7
            for i in range(2, 4):
                v = self._cbr(getattr(blk, f"branch7x7x3_{i}"), v)
            self._cbr(blk.branch7x7x3_4, v, o7)
            self._at(2); self._pool(True, x, om)
        elif isinstance(blk, InceptionE):
            cat, (o1, o3a, o3b, oda, odb, op) = self._concat(H, W, [320, 384, 384, 384, 384, 192])
            _, s, d1 = self._hconv([blk.branch1x1, blk.branch3x3_1, blk.branch3x3dbl_1], x, [o1, None, None], [0, 1, 2])
            self._at(1)
            self._cbr(blk.branch3x3_2a, s, o3a)
            self._cbr(blk.branch3x3_2b, s, o3b)
            self._at(2)
            d = self._cbr(blk.branch3x3dbl_2, d1)
            self._cbr(blk.branch3x3dbl_3a, d, oda)
            self._cbr(blk.branch3x3dbl_3b, d, odb)
            self._at(3); self._cbr(blk.branch_pool, self._pool(False, x), op)
        else:
            raise TypeError(f"cannot lower block {type(blk).__name__}")
        self._at(None)
        self._bi += 1
        return cat

    def _alloc(self):
        m, A, B = self.model, self.arena, self.B
        self.x = A.zeros((B, self.H0, self.W0, 8))
        self.labels = guard.alloc((B,), torch.int64, self.device, zero=True, label="labels")
        self.ops = []
        self.op_meta = []   # per op: None (stem, stream 0) or (block index, branch index)
        self._bi, self._cur = 0, None
        v = Val(Act(self.x, 0, 8, 8, 0, B, self.H0, self.W0), needs_grad=False)
        geom = stem_pack_geom(m.Conv2d_1a_3x3.conv, self.H0, self.W0)  # 1-channel input: taps as channels
        if geom is not None:
            self.stem_pack = (geom["taps"], geom["off"])
        v = self._cbr(m.Conv2d_1a_3x3, v, geom=geom)
        v = self._cbr(m.Conv2d_2a_3x3, v)
        v = self._cbr(m.Conv2d_2b_3x3, v)
        v = self._pool(True, v)
        v = self._cbr(m.Conv2d_3b_1x1, v)
        v = self._cbr(m.Conv2d_4a_3x3, v)
        v = self._pool(True, v)
        for blk in m.mixed:
            v = self._block(blk, v)
        self.feat = v
        a = v.act
        if a.C != m.fc.in_features:
            raise ValueError("feature width does not match fc")
        self.HWf = a.H * a.W
        N = m.num_classes
        self.dfeat = new_act(A, 1, B, a.H, a.W, a.C, GRAD_DT)
        v.grads.append(self.dfeat)
        self.fc_feat = A.empty((B, a.C), torch.float32)
        self.logp = guard.alloc((B, N), torch.float32, self.device, zero=True, label="logits")  # of the last batch
        self.dlogits = A.empty((B, N), torch.float32)
        self.seed = guard.alloc(1, torch.int64, self.device, zero=True, label="dropout counter")
        self.extra_state = [self.seed]
        # metrics [joint, distance, event] x [loss, correct, count, abs_err]; confusion: distance, event
        self.metrics = guard.alloc((3, 4), torch.float32, self.device, zero=True, label="metrics")
        self.confusion = guard.alloc((2, 16, 16), torch.int32, self.device, zero=True, label="confusion")
        self.nvalid = torch.full((1,), B, device=self.device, dtype=torch.int64)
        self.convs: List[ConvLayer] = [op.conv for op in self.ops if getattr(op, "conv", None) is not None]
        self._plan_nol()
        self._plan_tail_batches()

    def set_rng_stream(self, seed: int, rank: int = 0):
        """Select the dropout RNG stream (high word of the device counter; the low word counts training
        steps): masks differ across DP ranks and across --seed values, as torch's per-sample dropout does."""
        stream = (int(seed) * 1000003 + int(rank) * 7919 + 1) & 0x7FFFFFFF
        self.seed.fill_(stream << 32)

    # the stem's 47x122 and 21x58 convs keep their BN+ReLU tails (C at bs 32: 7.55k -> 7.66k samples/s,
    # three runs each of a limit of all / 1e5 / 3e4 output pixels)
    NOL_MAX_PX = 30000

    def tail_batch_enabled(self) -> bool:
        """One batched BN+ReLU tail launch per Inception block (MDA_TAIL_BATCH=0: a tail per branch output)."""
        return os.environ.get("MDA_TAIL_BATCH", "1") == "1"

    def _plan_tail_batches(self):
        """The BN+ReLU tails of an Inception block's branch outputs -- channel slices of the block's concat
        buffer, read only by the next block -- run as ONE launch after the block's branches join
        (_emit_streamed) instead of one per branch at the end of each branch stream."""
        self._pending_tails: List[tuple] = []
        self.n_tail_batched = 0
        if not self.tail_batch_enabled():
            return
        by_block: Dict[int, List[CBR]] = {}
        for i, op in enumerate(self.ops):
            if (isinstance(op, CBR) and not op.skip_tail and op.out.parent is not None
                    and self.op_meta[i] is not None):
                op.defer_tail = True
                self.n_tail_batched += 1
                by_block.setdefault(self.op_meta[i][0], []).append(op)
        # the block's branch-output BNs complete together (forward: at the join, before the batched tail;
        # backward: the batched reduce): their replica rows share one buffer each way, so SyncBN all-reduces
        # them with ONE collective per block and direction (enable_sync_bn, batch_tails).  Members of a
        # horizontally fused conv keep the fused conv's forward rows (reduced when that conv ran).
        self._stat_groups, self._part_groups = [], {}
        for blk, ops in by_block.items():
            own = [op.bn for op in ops if op.fused is None]
            if len(own) >= 2:
                self._stat_groups.append((coalesce_replicas(own, "stats", self.arena), own))
            if len(ops) >= 2:
                bns = [op.bn for op in ops]
                self._part_groups[blk] = (coalesce_replicas(bns, "part", self.arena), bns)

    def batch_tails(self) -> int:
        """The backward of the branch-output BN+ReLU tails of each Inception block as ONE reduce and ONE apply
        launch on stream 0 right after the block's backward fork (their gradient sources -- the next block's
        data gradients -- are complete there), instead of a reduce + apply (or the single-launch kernel) at
        the head of every branch stream (csrc/bn.hip bnb_batched_kernel).  Each branch's first remaining
        launch waits for the batch.  Runs after the autotuner (which picks the per-tail variants the batch
        replaces); not with SyncBN (its collectives sit between the passes).  Returns the tails batched."""
        from .program import Launch, k_tail_bwd_batched
        sync = getattr(self, "sync_bn_world", None) is not None
        if not self.tail_batch_enabled():
            return 0
        ls = self.bwd.launches
        fork_at, groups = self._tail_bwd_groups()
        if sync:  # only the blocks whose collective enable_sync_bn left to this batch (one per block)
            groups = {b: t for b, t in groups.items() if b in self._sync_part_groups}
        n = 0
        removed = set()
        inserts = []
        for blk, tails in groups.items():
            cgb = 8
            while any((t.args[3]["C"] // 8) % cgb for t in tails):
                cgb //= 2
            jobs = [dict(t.args[3], fused=0) for t in tails]
            if sync:  # the apply writes d(gamma), d(beta) / world (enable_sync_bn)
                for j in jobs:
                    j["gscale"] = 1.0 / self.sync_bn_world
            blocks = [t.args[2] * (t.args[3]["C"] // (8 * cgb)) for t in tails]
            raw, nblocks, _ = lib().tail_table(jobs, blocks, True)
            table = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device)
            self._tail_tables = getattr(self, "_tail_tables", [])
            self._tail_tables.append(table)
            tag = f"tailbatch_{blk[len('fork:'):]}"
            red = Launch("tailbatchbwd_reduce", k_tail_bwd_batched, ACT_RELU, cgb, 1, table, len(jobs), nblocks,
                         owner=tails, stream=0)
            app = Launch("tailbatchbwd_apply", k_tail_bwd_batched, ACT_RELU, cgb, 0, table, len(jobs), nblocks,
                         owner=tails, stream=0, record=tag)
            mid = []
            if sync:  # the block's partial sums all-reduced between the passes: one collective
                mid = [Launch("allreduce_bn", k_allreduce, self._sync_allreduce, self._sync_part_groups[blk].t,
                              stream=0)]
                self._sync_bwd_pending.discard(blk)
            inserts.append((fork_at[blk] + 1, [red] + mid + [app]))
            for t in tails:
                if t.record is not None:
                    raise RuntimeError(f"batched tail backward records event {t.record}")
                removed.add(id(t))
                # the branch's next launch inherits the tail's waits, now on the batch
                nxt = next((k for k in ls[ls.index(t) + 1:] if k.stream == t.stream), None)
                if nxt is not None and t.stream != 0:
                    nxt.waits = tuple(w for w in nxt.waits if w not in t.waits) + (tag,)
            n += len(tails)
        out = []
        ins = dict(inserts)
        for i, l in enumerate(ls):
            if id(l) not in removed:
                out.append(l)
            if i + 1 in ins:
                out += ins[i + 1]
        self.bwd.launches = out
        self.n_tail_bwd_batched = n
        return n

    def check_sync_bn(self):
        """enable_sync_bn drops the per-BN backward collective of every coalesced block's branch-output
        BNs and leaves ONE per block to batch_tails (autotune_program with batch_wgrads) -- raise if a step would
        run without it (those BNs would silently train on per-rank statistics).  StepRunner calls this."""
        pending = getattr(self, "_sync_bwd_pending", None)
        if pending:
            raise RuntimeError(f"SyncBN: the coalesced backward collective of {len(pending)} Inception blocks was never "
                               "inserted -- run batch_tails (autotune_program(..., batch_wgrads=True)) before stepping")

    def _tail_bwd_groups(self):
        """The block-output BN-tail backward launches batch_tails batches, per block (keyed by the block's
        backward fork pseudo-launch), and the index of each fork."""
        fork_at, groups, blk = {}, {}, None
        for i, l in enumerate(self.bwd.launches):
            if l.name.startswith("fork:backward_f"):
                blk = l.name
                fork_at[blk] = i
            elif (l.name.startswith("tailbwd") and isinstance(l.owner, CBR) and l.owner.defer_tail and blk is not None
                  and l.args[3].get("fused", 0) in (0, 1) and l.args[0] == ACT_RELU and l.args[1] == 1
                  and not l.args[3].get("side")):
                groups.setdefault(blk, []).append(l)
        return fork_at, groups

    def enable_sync_bn(self, allreduce) -> int:
        """SyncBN (LoweredProgram.enable_sync_bn) with the branch-output BNs of every Inception block coalesced:
        forward, one all-reduce of the block's own replica rows right before its batched BN+ReLU tail (after
        the join, where all of them are complete); backward, one all-reduce of the block's partial sums
        between the batched reduce and apply passes (batch_tails).  Blocks whose tails do not all batch
        (e.g. statistics fused into a data gradient) keep one collective per BN.  Returns the all-reduces per
        training step (Model C: 188 -> 126)."""
        from .program import Launch
        skip_fwd = {P(bn.stats, bn.stats_off) for _, g in self._stat_groups for bn in g}
        _, groups = self._tail_bwd_groups()
        self._sync_part_groups = {}
        by_buf = {id(buf): (buf, bns) for buf, bns in self._part_groups.values()}
        for blk, tails in groups.items():
            bufs = {id(t.owner.bn.part) for t in tails}
            if self.tail_batch_enabled() and len(bufs) == 1 and len(by_buf[next(iter(bufs))][1]) == len(tails):
                self._sync_part_groups[blk] = by_buf[next(iter(bufs))][0]
        # the blocks whose backward collective batch_tails must still insert (check_sync_bn)
        self._sync_bwd_pending = set(self._sync_part_groups)
        skip_bwd = {P(t.owner.bn.part, t.owner.bn.part_off) for blk in self._sync_part_groups for t in groups[blk]}
        n = super().enable_sync_bn(allreduce, skip_fwd=skip_fwd, skip_bwd=skip_bwd)
        self._sync_allreduce = allreduce
        new = []
        for l in self.fwd_train.launches:
            if l.name.startswith("tailbatch") and isinstance(l.owner, list):
                ptrs = {d["bn"]["stats"] for d, _ in l.owner}
                for buf, bns in self._stat_groups:
                    if {P(bn.stats, bn.stats_off) for bn in bns} <= ptrs:
                        # after the join events (the branches' convs), before the tail that normalises
                        new.append(Launch("allreduce_bn", k_allreduce, allreduce, buf.t, stream=0, waits=l.waits))
                        l.waits = ()
                        n += 1
            new.append(l)
        self.fwd_train.launches = new
        return n + len(self._sync_part_groups)

    def _patch_forward(self, conv: ConvLayer) -> bool:
        """The conv's training forward runs a 3x3 patch config in the shipped table: its input strip is staged
        once, so normalise-on-load transforms each element once instead of KH*KW times as the im2col does --
        the reason for NOL_MAX_PX -- and the cap does not apply (the stem's 47x122 / 21x58 consumers)."""
        from ..ops.functional import CONV_PATCH_CFG0, CONV_PATCH_NCFG, CONV_PATCHP_CFG0, CONV_PATCHP_NCFG, CONV_XCD
        from .tune import conv_signature, load_cache
        if not hasattr(self, "_table"):
            self._table = load_cache()
        d = {"B": conv.B, "Hs": conv.Hi, "Ws": conv.Wi, "Ho": conv.Ho, "Wo": conv.Wo, "N": conv.Co, "Cs": conv.Cs,
             "KH": conv.KH, "KW": conv.KW, "sh": conv.sh, "sw": conv.sw, "ph": conv.ph, "pw": conv.pw,
             "src": {"C1": conv.src_C1}, "stats": 1}
        cfg = self._table.get(conv_signature(0, conv.G, d))
        if cfg is None:
            return False
        cfg &= ~CONV_XCD
        return (CONV_PATCH_CFG0 <= cfg < CONV_PATCH_CFG0 + CONV_PATCH_NCFG
                or CONV_PATCHP_CFG0 <= cfg < CONV_PATCHP_CFG0 + CONV_PATCHP_NCFG)

    def _plan_nol(self):
        """Normalise-on-load: a BasicConv2d output consumed by exactly one other BasicConv2d (and not a
        slice of a block's concat buffer) is never materialised -- the consumer reads the producer's
        pre-BN y and applies BN + ReLU to its operand (engine/lowering.py nol_enabled)."""
        self.n_nol = 0
        if not self.nol_enabled():
            return
        max_px = self.NOL_MAX_PX
        consumers = {}
        for op in self.ops:
            if getattr(op, "fused", None) is None:  # fused members read nothing: their HConv reads the input
                consumers[id(op.src)] = consumers.get(id(op.src), 0) + 1
        consumers[id(self.feat)] = consumers.get(id(self.feat), 0) + 1
        producer = {id(op.out): op for op in self.ops if isinstance(op, CBR)}
        for op in self.ops:
            p = producer.get(id(op.src))
            if (isinstance(op, CBR) and op.conv is not None and p is not None and op.src.parent is None
                    and consumers[id(op.src)] == 1 and op.conv.Cs == p.out.act.C
                    and (op.conv.M_out <= max_px or self._patch_forward(op.conv))):
                op.nol_from = p
                p.skip_tail = True
                self.n_nol += 1

    # -------------------------------------------------------------------------------------------
    def _head_args(self, training: bool) -> dict:
        m, f, a = self.model, self.flat, self.feat.act
        d = {"x": a.p, "ldx": a.ld, "W": P(f.params, f.off(m.fc.weight)), "bias": P(f.params, f.off(m.fc.bias)),
             "labels": P(self.labels), "B": self.B, "HW": self.HWf, "C": a.C, "N": m.num_classes,
             "p_drop": self.p_drop if training else 0.0, "seed": P(self.seed), "feat": P(self.fc_feat),
             "logits": P(self.logp), "dlogits": P(self.dlogits), "metrics": P(self.metrics),
             "confusion": P(self.confusion), "nvalid": P(self.nvalid)}
        if training:
            d.update({"dx": self.dfeat.p, "dW": P(f.grads, f.off(m.fc.weight)), "db": P(f.grads, f.off(m.fc.bias))})
        return d

    def _emit(self):
        self.fwd_train = self._emit_forward(True)
        self.fwd_eval = self._emit_forward(False)
        self.bwd = self._emit_backward()
        self.fuse_dgrad_bn_stats()
        self.opt = self._emit_optimizer()

    def _emit_streamed(self, ph: Phase, order, run) -> List[str]:
        """Emit ops in ``order``; the branches of an Inception block run on streams 0..3 (branch b on
        stream b), join-then-fork per block: a kernel-free fork point on stream 0 waits for the previous
        block's side streams and records one event, and every side branch waits only for that event
        (the block input -- in backward the block output's gradient sources -- is then complete).
        Returns the side-stream events the caller's next stream-0 launch must wait for.  With
        MDA_STREAMS=0 the annotations are inert and the ops run in list order."""
        owed0: List[str] = []       # last block's side-stream end events (joined at the next fork)
        self._block_fork = getattr(self, "_block_fork", {})
        cur_block, used = None, set()

        def close_block():
            nonlocal owed0, cur_block, used
            owed0 = []
            for st in sorted(used - {0}):
                ph.cur_stream = st
                tag = f"{ph.name}_e{cur_block}_{st}"
                ph.mark(tag)
                owed0.append(tag)
            if self._pending_tails:  # the block's deferred branch-output tails, after the join, on stream 0
                ph.cur_stream = 0
                ph.pending_waits.extend(owed0)
                owed0 = []
                self._tail_batch(ph, ACT_RELU, self._pending_tails)
                self._pending_tails = []
            cur_block, used = None, set()

        for i in order:
            meta = self.op_meta[i]
            blk = None if meta is None else meta[0]
            if blk != cur_block and cur_block is not None:
                close_block()
            if meta is None:
                ph.cur_stream = 0
                ph.pending_waits.extend(owed0)
                owed0 = []
                run(self.ops[i])
                continue
            if cur_block is None:
                cur_block = blk
                ph.cur_stream = 0
                ph.fork_point(f"{ph.name}_f{blk}", waits=owed0)
                self._block_fork[(ph.name, blk)] = ph.launches[-1]
                owed0 = []
            st = meta[1] % 4
            ph.cur_stream = st
            first = st not in used
            fork = f"{ph.name}_f{blk}"
            if first and st != 0:
                ph.pending_waits.append(fork)
            n_before = len(ph.launches)
            run(self.ops[i])
            if len(ph.launches) > n_before:
                used.add(st)
            elif first and st != 0:  # the op launched nothing (a fused member whose tail its consumer folded):
                ph.pending_waits.remove(fork)  # the stream's first real launch waits for the fork instead
        if cur_block is not None:
            close_block()
        ph.cur_stream = 0
        return owed0

    def _emit_forward(self, training: bool) -> Phase:
        ph = Phase("forward_train" if training else "forward_eval")
        owed = self._emit_streamed(ph, range(len(self.ops)), lambda op: op.forward(self, ph, training))
        ph.add("cls_head", k_cls_head, self._head_args(training), waits=owed)
        return ph

    def bucket_cut_candidates(self) -> List[tuple]:
        """A cut before each Inception block's backward (its fork point, where the later blocks' streams
        have joined): the fc layer and every later block are complete, i.e. the flat range from that
        block's successor's first parameter to the end (module order = flat order = forward order)."""
        f, m = self.flat, self.model
        out = []
        for b in range(len(m.mixed) - 1, 0, -1):
            done = [p for blk in list(m.mixed)[b:] for p in blk.parameters()] + list(m.fc.parameters())
            lo = min(f.off(p) for p in done)
            ids = {id(p) for p in done}
            if any(f.off(p) >= lo for p in m.parameters() if id(p) not in ids):
                raise ValueError("Inception parameters are not in forward order in the flat buffer")
            anchor = self._block_fork.get(("backward", b - 1))
            if anchor is not None:
                out.append((anchor, lo, f.numel))
        return out

    def _emit_backward(self) -> Phase:
        ph = Phase("backward")
        owed = self._emit_streamed(ph, reversed(range(len(self.ops))), lambda op: op.backward(self, ph))
        assert not owed, "the stem's backward must have joined the first block's branches"
        ph.launches[self._last_wgrad].record = "wgrads"
        ph.add("wgrad_finalize", k_wgfin, *self._wgfin_args(), waits=("wgrads",))
        return ph
