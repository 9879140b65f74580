"""Lowering of the MTL network (reference Model A) and its single-task variant (Model B).

Forward (reference modelA_MTL.py:127-174), per step, all on one HIP stream:

    gather          dataset rows -> bf16 NHWC batch (C padded to 8) + labels
    conv1           7x7/s3 MFMA conv (+BN sums)           -> tail BN+ReLU
    resblock i      conv a (+sums) -> tail BN+ReLU -> conv b (+sums) [-> shortcut conv (+sums)]
                    -> tail relu(BN(b) + BN(s) | x)        = F_i
    level l, ALL TASKS IN ONE LAUNCH (grid.z = task; shared inputs read with group stride 0):
                    1x1 conv(+bias) on F_{2l-1} or the two-segment input [F_{2l-1} | B_{l-1,t}]
                    -> tail BN+ReLU -> 3x3 conv(+bias) -> tail sigmoid(BN) * F_{2l}   = A_{l,t}
                    l<4: 3x3 conv -> tail maxpool2x2ceil(relu(BN))                   = B_{l,t}
    head            GAP -> channel-group mean -> log_softmax -> NLL (+metrics, +dL/dA_4)

Backward mirrors it level 4 -> 1 then resblock 8 -> 1 -> conv1; every activation gradient is written
once and multi-consumer gradients (each F_k feeds the next block AND the task branches) are summed by
the consuming kernel from a list of sources.  Weight gradients go to split-M slabs that one launch
reduces into the flat gradient buffer; then one fused Adam launch updates the flat master weights and
re-packs the bf16 MFMA images.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import torch

from ..models.mtl import MTLNet
from ..ops.hip import lib
from . import guard
from .core import GRAD_DT, NREP, Act, Arena, BNLayer, ConvLayer, FlatState, P, new_act, src_dict, stem_pack_geom
from .lowering import ACT_NONE, ACT_RELU, ACT_SIGMOID, ADD_RELU, POOL_RELU, SIGMUL, LoweredProgram
from .program import Phase, k_head, k_wgfin


class MTLProgram(LoweredProgram):
    """Static train/eval programs of an :class:`MTLNet` for a fixed per-GPU batch size."""

    # DP: the task-branch gradients (38% of the 4.5 MB buffer) are all-reduced while RB1, the stem and
    # the backbone's weight gradients still run; the backbone bucket follows (bucket_cut_candidates)
    default_buckets = 2
    # the level branches' weight-gradient batches on a persistent grid of 512 blocks: the backbone's data-
    # gradient chain finds CU slots for its blocks (in-step ramp of a 33x83 dgrad 10-16 us beside an uncapped
    # batch, tools/kernel_phases.py); A 34.71-34.91 k -> 35.08-35.34 k (5 pairs, docs/PERF.md round 5)
    SIDE_WGRAD_GRID = 512
    # stream 0's weight gradients (after its data-gradient chain, the step's serial tail) in 2 batched launches
    # instead of 3: A 35,502 -> 35,700 (4 pairs), B_event 37,784 -> 38,246 (2 pairs); all streams at 2: A
    # 35,676, B 38,112 (docs/PERF.md round 5)
    WGRAD_MAX_BATCHES_S0 = 2
    # normalise-on-load only for consumer convs of at most this many output pixels: the 33x83 convs (87,648
    # px at batch 32) read a materialised BN+ReLU output instead -- the im2col's KH*KW-fold on-load transform
    # costs them more than the tail launch it saves.  Large-tile weight-gradient splits of >= 2048 pixels
    # (fewer split slabs for the finalize).  Together A +0.45 % (3 of 4 interleaved pairs), B_distance +1 %
    # (docs/PERF.md round 5); Model C keeps its own values (its weight gradients lose 0.9 % at 2048)
    NOL_MAX_PX = 60000
    WGRAD_MIN_SPLIT_PX_BIG = 2048

    def __init__(self, model: MTLNet, batch: int, device, in_hw=(100, 250), loss_weights: Optional[Sequence[float]] = None,
                 sync_world: int = 1):
        self.model = model
        self.B = B = batch
        self.T = T = len(model.tasks)
        self.device = torch.device(device)
        self.H0, self.W0 = in_hw
        self.cin = model.in_channels
        if self.cin > 8:
            raise ValueError("in_channels > 8 not supported by the gather kernel")
        self.loss_weights = list(loss_weights) if loss_weights is not None else [1.0] * T
        if len(self.loss_weights) != T:
            raise ValueError("one loss weight per task")
        # label column of each task in the [B, 2] (distance, event) label tensor
        self.lab_off = [0 if t == "distance" else 1 for t in model.tasks]
        if T == 2 and self.lab_off != [0, 1]:
            raise ValueError("two-task model must be (distance, event)")

        gens = model.att_generators
        outs = model.output_layers
        pgroups, bgroups = [], []
        for lvl in range(4):
            g = gens[lvl]
            for idx in (0, 3):
                pgroups += [[g[t][idx].weight for t in range(T)], [g[t][idx].bias for t in range(T)]]
            for idx in (1, 4):
                pgroups += [[g[t][idx].weight for t in range(T)], [g[t][idx].bias for t in range(T)]]
                bgroups.append([g[t][idx] for t in range(T)])
            if lvl < 3:
                o = outs[lvl]
                pgroups += [[o[t][0].weight for t in range(T)], [o[t][1].weight for t in range(T)],
                            [o[t][1].bias for t in range(T)]]
                bgroups.append([o[t][1] for t in range(T)])
        model.to(self.device)
        self.flat = FlatState(model, self.device, pgroups, bgroups)
        self.flat.bn_world = sync_world  # SyncBN: global BN counts (enable_sync_bn adds the collectives)
        self.arena = A = Arena(self.device)
        self._alloc()
        A.finalize()
        self._emit()

    # -------------------------------------------------------------------------------------------
    FOLD_SOURCES = True  # the residual-block tails' sources are summed by the last dgrad (fold_tail_sources)

    def _alloc(self):
        m, A, B, T, f = self.model, self.arena, self.B, self.T, self.flat
        self.x = A.zeros((B, self.H0, self.W0, 8))
        self.labels = guard.alloc((B, 2), torch.int64, self.device, zero=True, label="labels")
        self.xin = Act(self.x, 0, 8, 8, 0, B, self.H0, self.W0)
        # stem
        geom = stem_pack_geom(m.conv1[0], self.H0, self.W0)  # 1-channel input: taps packed as channels
        if geom is not None:
            self.stem_pack = (geom["taps"], geom["off"])
        c1 = ConvLayer([m.conv1[0]], f, A, B, self.H0, self.W0, cin_stored=8, geom=geom)
        self.conv1 = c1
        H, W = c1.Ho, c1.Wo
        self.bn1 = BNLayer([m.conv1[1]], f, A, B * H * W)
        self.y0 = new_act(A, 1, B, H, W, c1.Co)
        self.f0 = new_act(A, 1, B, H, W, c1.Co)
        # residual blocks
        self.rbs = []
        prev = self.f0
        for rb in m.resblocks:
            L = {}
            L["proj"] = rb.has_projection
            L["fused"] = rb.has_projection and self.hfuse_enabled()
            if L["fused"]:
                # horizontal fusion: conv a (3x3/s2) and the projection shortcut (1x1/s2, the centre tap of conv
                # a's window) read the same input -- ONE conv with N = 2C writes [ya | ys], its epilogue the BN sums
                # of both BNs into one combined replica buffer; one data gradient over [dya | dys]
                cas = ConvLayer([rb.left[0], rb.shortcut[0]], f, A, B, prev.H, prev.W, concat=True)
                Ho, Wo, C = cas.Ho, cas.Wo, cas.Co // 2
                st = A.zeroed((1, NREP, 2, 2 * C), torch.float64)
                L["cas"], L["stats"] = cas, st
                L["bna"] = BNLayer([rb.left[1]], f, A, B * Ho * Wo, stats_share=(st, 0, 2 * C))
                L["bns"] = BNLayer([rb.shortcut[1]], f, A, B * Ho * Wo, stats_share=(st, C, 2 * C))
                yas, dyas = new_act(A, 1, B, Ho, Wo, 2 * C), new_act(A, 1, B, Ho, Wo, 2 * C)
                L["yas"], L["dyas"] = yas, dyas
                L["ya"], L["ys"] = yas.slice(0, C), yas.slice(C, C)
                L["dya"], L["dys"] = dyas.slice(0, C), dyas.slice(C, C)
            else:
                ca = ConvLayer([rb.left[0]], f, A, B, prev.H, prev.W)
                Ho, Wo, C = ca.Ho, ca.Wo, ca.Co
                L["ca"], L["bna"] = ca, BNLayer([rb.left[1]], f, A, B * Ho * Wo)
                L["ya"], L["dya"] = new_act(A, 1, B, Ho, Wo, C), new_act(A, 1, B, Ho, Wo, C)
            L["cb"], L["bnb"] = ConvLayer([rb.left[3]], f, A, B, Ho, Wo), BNLayer([rb.left[4]], f, A, B * Ho * Wo)
            if rb.has_projection and not L["fused"]:
                L["cs"] = ConvLayer([rb.shortcut[0]], f, A, B, prev.H, prev.W)
                L["bns"] = BNLayer([rb.shortcut[1]], f, A, B * Ho * Wo)
                L["ys"] = new_act(A, 1, B, Ho, Wo, C)
                L["dys"] = new_act(A, 1, B, Ho, Wo, C)
                L["dxs"] = new_act(A, 1, B, prev.H, prev.W, prev.C, GRAD_DT)
            elif not rb.has_projection:
                L["side"] = new_act(A, 1, B, Ho, Wo, C, GRAD_DT)
            L["in"] = prev
            L["ha"], L["yb"] = (new_act(A, 1, B, Ho, Wo, C) for _ in range(2))
            L["out"] = new_act(A, 1, B, Ho, Wo, C)
            L["dyb"] = new_act(A, 1, B, Ho, Wo, C)
            L["dha"] = new_act(A, 1, B, Ho, Wo, C, GRAD_DT)
            L["dxa"] = new_act(A, 1, B, prev.H, prev.W, prev.C, GRAD_DT)
            self.rbs.append(L)
            prev = L["out"]
        self.F = [L["out"] for L in self.rbs]  # F1..F8 (index 0..7)
        # task levels (grouped over T)
        gens, outs = m.att_generators, m.output_layers
        self.levels = []
        prevB = None
        for lvl in range(4):
            Fa, Fb = self.F[2 * lvl], self.F[2 * lvl + 1]
            H, W, C = Fa.H, Fa.W, Fa.C
            g = gens[lvl]
            L = {"H": H, "W": W, "C": C, "Fa": Fa, "Fb": Fb, "prevB": prevB}
            cin = C + (prevB.C if prevB is not None else 0)
            L["c0"] = ConvLayer([g[t][0] for t in range(T)], f, A, B, H, W)
            assert L["c0"].Ci == cin
            cm = L["c0"].Co
            L["bn0"] = BNLayer([g[t][1] for t in range(T)], f, A, B * H * W)
            L["c3"] = ConvLayer([g[t][3] for t in range(T)], f, A, B, H, W)
            L["bn3"] = BNLayer([g[t][4] for t in range(T)], f, A, B * H * W)
            L["ym1"], L["hm"] = new_act(A, T, B, H, W, cm), new_act(A, T, B, H, W, cm)
            L["ym2"], L["Aout"] = new_act(A, T, B, H, W, C), new_act(A, T, B, H, W, C)
            L["dym2"] = new_act(A, T, B, H, W, C)
            L["dF"] = new_act(A, T, B, H, W, C, GRAD_DT)   # side: gradient of F_{2l} per task
            L["dhm"] = new_act(A, T, B, H, W, cm, GRAD_DT)
            L["dym1"] = new_act(A, T, B, H, W, cm)
            L["dcat"] = new_act(A, T, B, H, W, cin, GRAD_DT)
            if lvl < 3:
                o = outs[lvl]
                L["co"] = ConvLayer([o[t][0] for t in range(T)], f, A, B, H, W)
                L["bno"] = BNLayer([o[t][1] for t in range(T)], f, A, B * H * W)
                Co = L["co"].Co
                L["yo"], L["dyo"] = new_act(A, T, B, H, W, Co), new_act(A, T, B, H, W, Co)
                L["dA"] = new_act(A, T, B, H, W, C, GRAD_DT)
                Hp, Wp = (H + 1) // 2, (W + 1) // 2
                L["Bp"] = new_act(A, T, B, Hp, Wp, Co)
                prevB = L["Bp"]
            self.levels.append(L)
        L4 = self.levels[3]
        self.dA4 = new_act(A, T, B, L4["H"], L4["W"], L4["C"], GRAD_DT)
        self.levels[3]["dA"] = self.dA4
        # head outputs / metrics (NOT in the per-step zeroed region: they accumulate across steps)
        self.logp = guard.alloc((T, B, 16), torch.float32, self.device, zero=True, label="logp")
        self.metrics = guard.alloc((T, 4), torch.float32, self.device, zero=True, label="metrics")
        self.confusion = guard.alloc((T, 16, 16), torch.int32, self.device, zero=True, label="confusion")
        self.nvalid = torch.full((1,), B, device=self.device, dtype=torch.int64)
        self.convs: List[ConvLayer] = self._backbone_convs() + \
                                      [L[k] for L in self.levels for k in ("c0", "c3", "co") if k in L]
        if self.WGRAD_MIN_SPLIT_PX_BIG < ConvLayer.MIN_SPLIT_PX_BIG:  # the slabs are sized for the default
            raise ValueError("WGRAD_MIN_SPLIT_PX_BIG below ConvLayer.MIN_SPLIT_PX_BIG")
        for c in self.convs:
            c.MIN_SPLIT_PX_BIG = self.WGRAD_MIN_SPLIT_PX_BIG
            c.set_wgrad_cfg(c.wcfg)

    @staticmethod
    def hfuse_enabled() -> bool:
        """Horizontal fusion of each projection block's conv a with its shortcut (MDA_HFUSE=0: separate convs)."""
        import os
        return os.environ.get("MDA_HFUSE", "1") == "1"

    def _emit(self):
        self.nol = self.nol_enabled()
        self.fwd_train = self._emit_forward(True)
        self.fwd_eval = self._emit_forward(False)
        self.bwd = self._emit_backward()
        self.fold_tail_sources()
        self.fuse_dgrad_bn_stats()
        self.opt = self._emit_optimizer()

    def _emit_forward(self, training: bool) -> Phase:
        ph = Phase("forward_train" if training else "forward_eval")
        T = self.T
        self._conv_fwd(ph, self.conv1, src_dict(self.xin), self.y0, self.bn1, training)
        self._tail(ph, ACT_RELU, 1, self.y0, self.bn1, self.f0, training)
        ph.cur_stream = 0
        for ri, L in enumerate(self.rbs):
            s = src_dict(L["in"])
            if L["fused"]:  # [ya | ys] and both BNs' sums in one launch (bna names the combined replica rows)
                self._conv_fwd(ph, L["cas"], s, L["yas"], L["bna"], training)
            else:
                self._conv_fwd(ph, L["ca"], s, L["ya"], L["bna"], training)
            if self.nol_for(L["cb"]):  # conv b normalises ya on load: no BN+ReLU tail, ha never materialised
                self._conv_fwd(ph, L["cb"], src_dict(L["ya"]), L["yb"], L["bnb"], training, nol=(L["bna"], ACT_RELU))
            else:
                self._tail(ph, ACT_RELU, 1, L["ya"], L["bna"], L["ha"], training)
                self._conv_fwd(ph, L["cb"], src_dict(L["ha"]), L["yb"], L["bnb"], training)
            if L["proj"] and not L["fused"]:
                self._conv_fwd(ph, L["cs"], s, L["ys"], L["bns"], training)
            if L["proj"]:
                self._tail(ph, ADD_RELU, 1, L["yb"], L["bnb"], L["out"], training, r=L["ys"], bn2=L["bns"])
            else:
                self._tail(ph, ADD_RELU, 1, L["yb"], L["bnb"], L["out"], training, r=L["in"])
            ph.mark(f"F{ri + 1}")
            ph.cur_stream = 0
        # task branches (both tasks per launch) on side stream 1, overlapping the backbone
        ph.cur_stream = 1
        for lvl, L in enumerate(self.levels):
            # the mask generator needs only F_{2l+1} (and the previous level, same stream); F_{2l+2} is
            # waited for right before the mask multiply, so the generator overlaps the next residual block
            ph.pending_waits.append(f"F{2 * lvl + 1}")
            s = src_dict(L["Fa"], L["prevB"]) if L["prevB"] is not None else src_dict(L["Fa"])
            self._conv_fwd(ph, L["c0"], s, L["ym1"], L["bn0"], training)
            if self.nol_for(L["c3"]):
                self._conv_fwd(ph, L["c3"], src_dict(L["ym1"]), L["ym2"], L["bn3"], training, nol=(L["bn0"], ACT_RELU))
            else:
                self._tail(ph, ACT_RELU, T, L["ym1"], L["bn0"], L["hm"], training)
                self._conv_fwd(ph, L["c3"], src_dict(L["hm"]), L["ym2"], L["bn3"], training)
            ph.pending_waits.append(f"F{2 * lvl + 2}")
            self._tail(ph, SIGMUL, T, L["ym2"], L["bn3"], L["Aout"], training, r=L["Fb"])
            if "co" in L:
                self._conv_fwd(ph, L["co"], src_dict(L["Aout"]), L["yo"], L["bno"], training)
                self._tail(ph, POOL_RELU, T, L["yo"], L["bno"], L["Bp"], training)
        ph.mark("levels")
        ph.cur_stream = 0
        ph.pending_waits.append("levels")
        A4 = self.levels[3]["Aout"]
        hd = {"feat": A4.p, "fgs": A4.gs, "ldf": A4.ld, "labels": P(self.labels), "lab_stride": 2,
              "lab_off": self.lab_off[0], "T": T, "B": self.B, "HW": A4.H * A4.W, "C": A4.C,
              "ncls": list(self.model.task_cate_num), "w": [float(w) for w in self.loss_weights],
              "logp": P(self.logp), "dfeat": self.dA4.p if training else 0, "dgs": self.dA4.gs,
              "metrics": P(self.metrics), "confusion": P(self.confusion), "nvalid": P(self.nvalid)}
        if T == 2:
            hd["lab_off"] = 0
        ph.add("mtl_head", k_head, hd)
        return ph

    def bucket_cut_candidates(self) -> List[tuple]:
        """One cut: right before residual block 1's backward, every task-branch (level) gradient is
        complete -- the level parameters lead the flat buffer (FlatState param_groups), so they form the
        first bucket and its all-reduce overlaps RB1, conv1 and the backbone's weight gradients."""
        f = self.flat
        lv = [p for c in self.convs if c not in self._backbone_convs() for m in c.mods for p in m.parameters()]
        lv += [p for L in self.levels for k in ("bn0", "bn3", "bno") if k in L for m in L[k].mods
               for p in m.parameters()]
        hi = max(f.off(p) + p.numel() for p in lv)
        hi = (hi + 3) // 4 * 4
        rest = [p for p in self.model.parameters() if all(p is not q for q in lv)]
        if any(f.off(p) < hi for p in rest) or min(f.off(p) for p in lv) != 0:
            raise ValueError("task-branch parameters do not lead the flat buffer")
        return [(self._rb1_anchor, 0, hi)]

    def _backbone_convs(self) -> list:
        return [self.conv1] + [L[k] for L in self.rbs for k in ("ca", "cas", "cb", "cs") if k in L]

    def _emit_backward(self) -> Phase:
        ph = Phase("backward")
        T, lv = self.T, self.levels
        ph.cur_stream = 1
        for li in range(3, -1, -1):
            L = lv[li]
            if "co" in L:
                nxt = lv[li + 1]
                Cn = nxt["Fa"].C
                dcat = nxt["dcat"]
                g = [(P(dcat.t, Cn), dcat.gs, dcat.ld)]  # B_l part of d cat[F, B_l]
                self._tail_bwd(ph, POOL_RELU, T, L["yo"], L["bno"], g, L["dyo"])
                self._conv_bwd(ph, L["co"], src_dict(L["Aout"]), L["dyo"], L["dA"])
            self._tail_bwd(ph, SIGMUL, T, L["ym2"], L["bn3"], [(L["dA"].p, L["dA"].gs, L["dA"].ld)], L["dym2"],
                           r=L["Fb"], side=L["dF"])
            ph.mark(f"dF{li}")  # F_{2l+2}'s gradient from this level is complete here
            if self.nol_for(L["c3"]):
                self._conv_bwd(ph, L["c3"], src_dict(L["ym1"]), L["dym2"], L["dhm"], nol=(L["bn0"], ACT_RELU))
            else:
                self._conv_bwd(ph, L["c3"], src_dict(L["hm"]), L["dym2"], L["dhm"])
            self._tail_bwd(ph, ACT_RELU, T, L["ym1"], L["bn0"], [(L["dhm"].p, L["dhm"].gs, L["dhm"].ld)], L["dym1"])
            s = src_dict(L["Fa"], L["prevB"]) if L["prevB"] is not None else src_dict(L["Fa"])
            self._conv_bwd(ph, L["c0"], s, L["dym1"], L["dcat"])
            ph.mark(f"lvl{li}")
        ph.cur_stream = 0
        # gradient sources of each shared feature F_k (index k-1), plus f0
        def sources(k: int) -> list:
            src = []
            if k >= 1:
                lvl = (k - 1) // 2
                L = lv[lvl]
                for t in range(T):
                    if k % 2 == 1:  # F_{2l-1}: first channel segment of the level's AMG input
                        src.append((P(L["dcat"].t, t * L["dcat"].gs), 0, L["dcat"].ld))
                    else:           # F_{2l}: attention-mask target
                        src.append((P(L["dF"].t, t * L["dF"].gs), 0, L["dF"].ld))
            if k < 8:
                R = self.rbs[k]  # resblock k+1 consumes F_k (or f0 when k == 0)
                src.append((R["dxa"].p, 0, R["dxa"].ld))
                if R["proj"] and not R["fused"]:  # (fused: the one data gradient covers the shortcut too)
                    src.append((R["dxs"].p, 0, R["dxs"].ld))
                elif not R["proj"]:
                    src.append((R["side"].p, 0, R["side"].ld))
            return src
        for i in range(7, -1, -1):
            R = self.rbs[i]
            g = sources(i + 1)
            if i == 0:  # bucket cut candidate: every task-branch gradient is complete before RB1's backward
                self._rb1_bwd_first = len(ph.launches)
            # F_{i+1}'s task-branch gradients: for F_{2l+2} (i odd) the mask-target gradient dF, ready right
            # after the level's sigmoid-mask backward; for F_{2l+1} the concat gradient of the whole level
            task_tag = f"dF{i // 2}" if i % 2 == 1 else f"lvl{i // 2}"
            ph.pending_waits.append(task_tag)
            if R["proj"]:
                self._tail_bwd(ph, ADD_RELU, 1, R["yb"], R["bnb"], g, R["dyb"], r=R["ys"], bn2=R["bns"], dy2=R["dys"])
            else:
                self._tail_bwd(ph, ADD_RELU, 1, R["yb"], R["bnb"], g, R["dyb"], r=R["in"], side=R["side"])
            if self.nol_for(R["cb"]):
                self._conv_bwd(ph, R["cb"], src_dict(R["ya"]), R["dyb"], R["dha"], nol=(R["bna"], ACT_RELU))
            else:
                self._conv_bwd(ph, R["cb"], src_dict(R["ha"]), R["dyb"], R["dha"])
            self._tail_bwd(ph, ACT_RELU, 1, R["ya"], R["bna"], [(R["dha"].p, 0, R["dha"].ld)], R["dya"])
            if R["fused"]:
                self._conv_bwd(ph, R["cas"], src_dict(R["in"]), R["dyas"], R["dxa"])
            else:
                self._conv_bwd(ph, R["ca"], src_dict(R["in"]), R["dya"], R["dxa"])
            if R["proj"] and not R["fused"]:
                self._conv_bwd(ph, R["cs"], src_dict(R["in"]), R["dys"], R["dxs"])
        self.dy0 = new_act(self.arena, 1, self.B, self.y0.H, self.y0.W, self.y0.C)
        self._tail_bwd(ph, ACT_RELU, 1, self.y0, self.bn1, sources(0), self.dy0)
        self._conv_bwd(ph, self.conv1, src_dict(self.xin), self.dy0, None)
        self._rb1_anchor = ph.launches[self._rb1_bwd_first]
        # weight-gradient slabs -> flat fp32 gradients (one launch for every conv), after all wgrads
        ph.launches[self._last_wgrad].record = "wgrads"
        ph.add("wgrad_finalize", k_wgfin, *self._wgfin_args(), waits=("wgrads",))
        return ph

