"""Shared lowering machinery: the emit helpers every model program uses (conv forward / backward,
fused BN tails and their backward, wgrad finalize, fused Adam + weight packing, batch gather)."""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch

from ..ops.functional import PATCH_R, WGRAD_PATCH, WGRAD_TILES
from ..ops.hip import lib
from .core import Act, BNLayer, ConvLayer, P, build_optseg_table, build_wgfin_table, pad_to, plain_ranges
from .program import (Launch, Phase, k_adam, k_allreduce, k_conv, k_gather, k_tail_bwd, k_tail_fwd, k_wgfin, k_wgrad,
                      k_wgrad_batched)

ACT_NONE, ACT_RELU, ACT_SIGMOID, SIGMUL, ADD_RELU, POOL_RELU = range(6)


WGRAD_AOL_CFG = 100  # batched-wgrad cfg offset of the apply-on-load kernels (csrc/kernels.h)


def _wgrad_cost(cfg: int, G: int, d: dict) -> int:
    """MFMA work (MACs incl. tile padding) of one weight-gradient launch -- used to balance fan-out."""
    if cfg in WGRAD_PATCH:
        TN, CB, _ = WGRAD_PATCH[cfg]
        px = d["splits"] * d["m_per_split"] * PATCH_R * pad_to(d["Wo"], 8)
        return px * G * math.ceil(d["Npad"] / TN) * TN * 9 * d["Cs"]
    TN, TK, MCH = WGRAD_TILES[cfg]
    return d["splits"] * d["m_per_split"] * G * TN * TK * math.ceil(d["Npad"] / TN) * (d["Kpad"] // TK)


def _refers_to(args, ptr: int) -> bool:
    """Whether a launch's argument tree names the device address ``ptr``."""
    if isinstance(args, dict):
        return any(_refers_to(v, ptr) for v in args.values())
    if isinstance(args, (list, tuple)):
        return any(_refers_to(v, ptr) for v in args)
    return isinstance(args, int) and not isinstance(args, bool) and args == ptr


_GRAD_KEYS = ("dgamma", "dbeta", "dgamma2", "dbeta2", "dW", "db")


def _grad_offsets(l, gbase: int, numel: int) -> List[int]:
    """Flat-gradient element offsets a launch writes directly (BN affine parameters of every group, the
    fc layer), found in its argument tree; conv weights are written by the finalize and not listed."""
    G = l.args[1] if l.name.startswith("tailbwd") else (l.args[2] if l.name.startswith("conv_") else 1)
    out = []

    def walk(d):
        if isinstance(d, dict):
            pgs = d.get("pgs", 0)
            for k in _GRAD_KEYS:
                v = d.get(k)
                if isinstance(v, int) and not isinstance(v, bool) and gbase <= v < gbase + 4 * numel:
                    out.extend((v - gbase) // 4 + g * pgs for g in range(G))
            for v in d.values():
                walk(v)
        elif isinstance(d, (list, tuple)):
            for v in d:
                walk(v)

    walk(l.args)
    return out


def _blocks(M: int, C: int, cap: int = 1024, per_thread: int = 4) -> int:
    cg = max(1, C // 8)
    pl = max(1, 256 // cg)
    return int(max(1, min(cap, math.ceil(M / (pl * per_thread)))))


class LoweredProgram:
    """Base class: subclasses allocate buffers / layers, then emit ``fwd_train``, ``fwd_eval``, ``bwd``
    and ``opt`` phases with these helpers.  ``self.convs`` lists every ConvLayer (for the finalize and
    packing descriptor tables) and ``self.label_width`` the columns of the stored label tensor."""

    label_width = 2
    default_buckets = 1  # gradient buckets under data parallelism (segment_backward); MDA_BUCKETS overrides

    def dp_buckets(self, world: int) -> int:
        import os
        return 1 if world <= 1 else int(os.environ.get("MDA_BUCKETS", str(self.default_buckets)))

    # -------------------------------------------------------------------------------------------
    def _tail(self, ph: Phase, kind: int, G: int, y: Act, bn: BNLayer, out: Act, training: bool, r: Act = None,
              bn2: BNLayer = None, H=None, W=None):
        d = {"y": y.p, "ygs": y.gs, "ldy": y.ld, "bn": bn.args(training), "out": out.p, "ogs": out.gs, "ldo": out.ld,
             "B": self.B, "H": y.H if H is None else H, "W": y.W if W is None else W, "C": y.C}
        if r is not None:
            d.update({"r": r.p, "rgs": r.gs, "ldr": r.ld})
        if bn2 is not None:
            d["bn2"] = bn2.args(training)
        M = self.B * d["H"] * d["W"]
        ph.add(f"tail{kind}", k_tail_fwd, kind, G, _blocks(M, y.C, per_thread=2), d)

    def _tail_bwd(self, ph: Phase, kind: int, G: int, y: Act, bn: BNLayer, g: list, dy: Act, r: Act = None,
                  bn2: BNLayer = None, side: Act = None, dy2: Act = None, apply_only: bool = False):
        """BN-tail backward launch.  ``apply_only``: the tail's statistics are accumulated by the producers
        of its gradient sources (and partial reduces, ``_tail_partial``), so only the apply pass runs."""
        d = {"y": y.p, "ygs": y.gs, "ldy": y.ld, "bn": bn.args(True), "B": self.B, "H": y.H, "W": y.W, "C": y.C,
             "g": g, "part": P(bn.part), "chunk_px": bn.chunk_px, "dy": dy.p, "dgs": dy.gs, "ldd": dy.ld}
        if apply_only:
            d["fused"] = 2
        elif kind in (SIGMUL, POOL_RELU) or len(g) > 1:
            # the apply pass reads the stored dz instead of re-reading several gradient sources /
            # re-evaluating the pool window
            if bn.dzbuf is None:
                bn.dzbuf = self.arena.empty((G, y.M, y.C), torch.float32)
            d.update({"dzbuf": P(bn.dzbuf), "dzgs": y.M * y.C if G > 1 else 0, "lddz": y.C})
        d.update(bn.grad_ptrs())
        if r is not None:
            d.update({"r": r.p, "rgs": r.gs, "ldr": r.ld})
        if bn2 is not None:
            d["bn2"] = bn2.args(True)
            gp = bn2.grad_ptrs()
            d.update({"dgamma2": gp["dgamma"], "dbeta2": gp["dbeta"], "dy2": dy2.p, "d2gs": dy2.gs, "ldd2": dy2.ld})
        if side is not None:
            d.update({"side": side.p, "sgs": side.gs, "lds": side.ld})
        if bn.M != y.M:
            raise ValueError("BN backward chunking assumes the BN pixel count equals the tail's pixel count")
        ph.add(f"tailbwd{kind}", k_tail_bwd, kind, G, bn.nchunk, d)

    def _tail_partial(self, ph: Phase, kind: int, y: Act, bn: BNLayer, g: list, r: Act = None, bn2: BNLayer = None,
                      stream: int = 0, waits=(), record=None):
        """Reduce-only launch (csrc/bn.hip fused = 3): the statistics sum(dz), sum(dz xhat) (, sum(dz xhat2))
        of a G = 1 tail over the gradient sources ``g`` only, accumulated into the tail's replica rows; the
        tail's other sources add theirs in their producers' epilogues and the tail runs apply-only."""
        d = {"y": y.p, "ygs": y.gs, "ldy": y.ld, "bn": bn.args(True), "B": self.B, "H": y.H, "W": y.W, "C": y.C,
             "g": g, "part": P(bn.part), "chunk_px": bn.chunk_px, "fused": 3}
        if r is not None:
            d.update({"r": r.p, "rgs": r.gs, "ldr": r.ld})
        if bn2 is not None:
            d["bn2"] = bn2.args(True)
        ph.add(f"tailpart{kind}", k_tail_bwd, kind, 1, bn.nchunk, d, stream=stream, waits=waits, record=record)

    @staticmethod
    def _tail_stats_args(kind: int, y: Act, bn: BNLayer, r: Act = None, bn2: BNLayer = None) -> dict:
        """Producer-side description of a G = 1 BN tail whose statistics a gradient producer accumulates:
        ConvArgs::bnb of a dgrad (csrc/conv.hip) or TailArgs::prev of an apply pass (csrc/bn.hip)."""
        d = {"y": y.p, "ygs": 0, "ldy": y.ld, "bn": bn.args(True), "part": P(bn.part), "kind": kind, "C": y.C}
        if r is not None:
            d.update({"r": r.p, "rgs": 0, "ldr": r.ld})
        if bn2 is not None:
            d["bn2"] = bn2.args(True)
        return d

    def enable_sync_bn(self, allreduce) -> int:
        """SyncBN across data-parallel ranks (``--sync_bn`` with the engine).

        The program must have been lowered with ``flat.bn_world = world`` (BN counts are global).  Then
          * forward: right after the conv epilogue that accumulated a BN's fp64 replica sums (sum y,
            sum y^2), ``allreduce`` sums them over ranks -- every tail / normalise-on-load consumer then
            normalises with the global batch mean and variance and updates the running statistics with
            them (identically on every rank);
          * backward: every BN-tail backward becomes reduce (or the dgrad epilogue's fused statistics) ->
            all-reduce of sum(dz), sum(dz xhat) -> apply, so the input gradient uses the global batch
            sums (torch.nn.SyncBatchNorm); the apply writes d(gamma), d(beta) scaled by 1/world, so after
            the data-parallel gradient average they equal torch's mean of the per-rank local sums.
        Single-launch BN backwards (fused = 1) cannot be split and are replaced by reduce + apply.
        The collectives run between kernels, so the step runs eagerly (no HIP graph).  Returns the number
        of all-reduces inserted per training step."""
        world = self.flat.bn_world
        if world <= 1:
            return 0
        by_stats = {P(bn.stats): bn for bn in self.flat.bn_layers}
        by_part = {P(bn.part): bn for bn in self.flat.bn_layers}
        n = 0
        new = []
        for l in self.fwd_train.launches:
            new.append(l)
            bn = by_stats.get(l.args[3].get("stats") or 0) if l.name == "conv_fwd" else None
            if bn is not None:
                ar = Launch("allreduce_bn", k_allreduce, allreduce, bn.stats, stream=l.stream, record=l.record,
                            bucket=l.bucket)
                l.record = None
                new.append(ar)
                n += 1
        self.fwd_train.launches = new
        new = []
        for l in self.bwd.launches:
            if not l.name.startswith("tailbwd") or l.args[3].get("fused") == 3:
                new.append(l)
                continue
            kind, G, nchunk, d = l.args
            bn = by_part[d["part"]]
            name, record = l.name, l.record
            # the original Launch object becomes the first of the new launches (it keeps its waits and its
            # identity: bucket-cut anchors refer to it), the apply carries its event
            l.record = None
            if d.get("fused", 0) != 2:  # statistics of this tail: a reduce-only pass first
                red = {k: v for k, v in d.items() if k not in ("dzbuf", "dzgs", "lddz", "dy", "dgs", "ldd", "side",
                                                                "sgs", "lds", "dgamma", "dbeta", "dgamma2", "dbeta2",
                                                                "dy2", "d2gs", "ldd2", "pgs")}
                red["fused"] = 3
                l.name, l.args = f"tailpart{kind}", (kind, G, nchunk, red)
                new += [l, Launch("allreduce_bn", k_allreduce, allreduce, bn.part, stream=l.stream, bucket=l.bucket)]
            else:  # statistics from the producing dgrad's epilogue: all-reduce them, then apply
                l.name, l.fn, l.args = "allreduce_bn", k_allreduce, (allreduce, bn.part)
                new.append(l)
            d = {k: v for k, v in d.items() if k not in ("dzbuf", "dzgs", "lddz")}
            d["fused"], d["gscale"] = 2, 1.0 / world
            new.append(Launch(name, k_tail_bwd, kind, G, nchunk, d, owner=l.owner, stream=l.stream, record=record,
                              bucket=l.bucket))
            n += 1
        self.bwd.launches = new
        self.sync_bn_world = world
        return n

    @staticmethod
    def nol_enabled() -> bool:
        """Normalise-on-load (MDA_NOL, default on): a conv whose input is the single-consumer output of a
        BN + ReLU tail reads the pre-BN y and applies the BN affine + ReLU to its im2col operand (and so
        does its weight gradient), so that tail is never launched (csrc/conv.hip MODE_FWD_NOL)."""
        import os
        return os.environ.get("MDA_NOL", "1") == "1"

    NOL_MAX_PX = 1 << 30  # per-model default of MDA_NOL_MAX_PX

    def nol_max_px(self) -> int:
        """Normalise-on-load only for consumer convs with at most this many output pixels (B*Ho*Wo):
        on the large stem maps the on-load transform (repeated KH*KW times per element by the im2col)
        costs more than the BN+ReLU tail it removes (MDA_NOL_MAX_PX overrides the model's default)."""
        import os
        return int(os.environ.get("MDA_NOL_MAX_PX", str(self.NOL_MAX_PX)))

    def nol_for(self, conv: ConvLayer) -> bool:
        return self.nol and conv.M_out <= self.nol_max_px()

    def _conv_fwd(self, ph: Phase, c: ConvLayer, src: dict, out: Act, bn: BNLayer, training: bool, nol=None):
        mode, cfg, G, d = c.fwd_args(src, out, bn, training)
        if nol is not None:  # (BNLayer of the input, activation kind[, residual Act, residual BNLayer or None])
            d["nol"] = {"bn": nol[0].args(training), "kind": nol[1]}
            if len(nol) > 2:  # residual-on-load: relu(BN(y) + r') of a residual block's output
                r = nol[2]
                d["nol"].update(r={"p": r.p, "gs": r.gs, "ld": r.ld},
                                bn2=nol[3].args(training) if nol[3] is not None else None)
        ph.add("conv_fwd", k_conv, mode, cfg, G, d, owner=c)

    def _conv_bwd(self, ph: Phase, c: ConvLayer, src: dict, dy: Act, dx: Optional[Act], nol=None):
        # data gradient first (it is on the critical chain, and under apply-on-load it writes the
        # coefficient table the weight gradient reads), then the per-conv weight gradient on the same
        # stream (production programs replace these by the batched launches at the end of the backward
        # pass: batch_wgrads)
        if dx is not None:
            mode, cfg, G, d = c.dgrad_args(dy, dx)
            ph.add("conv_dgrad", k_conv, mode, cfg, G, d, owner=c)
        cfg, G, d = c.wgrad_args(src, dy)
        if nol is not None:  # the forward normalised its input on load: rebuild the operand the same way
            d["nol"] = {"consts": P(nol[0].consts), "kind": nol[1]}
        ph.add("conv_wgrad", k_wgrad, cfg, G, d, owner=c)
        self._last_wgrad = len(ph.launches) - 1

    def fuse_dgrad_bn_stats(self) -> int:
        """Move the BN-backward reduction of single-source elementwise tails into the producing dgrad.

        A BN tail whose activation is elementwise (none / ReLU / sigmoid) and whose output gradient has
        exactly ONE source -- the data gradient of the next conv, written once as fp32 on the tail's own
        pixel grid -- gets its per-channel sum(dz), sum(dz * xhat) from that dgrad's epilogue
        (csrc/conv.hip, ConvArgs::bpart), and its backward runs the apply pass only (``fused = 2``): one
        launch and one full pass over the gradient less per such layer (Model A: the 8 residual-block
        inner BNs and the 4 attention-generator BNs; Model C: every BasicConv2d feeding exactly one
        other).  MDA_DGRAD_BNSTATS=0 disables it.  Returns the number of fused layers."""
        import os
        self.n_dgrad_bnstats = 0
        if os.environ.get("MDA_DGRAD_BNSTATS", "1") != "1":
            return 0
        producers = {}
        for l in self.bwd.launches:
            if l.name == "conv_dgrad":
                producers[l.args[3]["out"]] = l
            elif l.name.startswith("tailbwd"):
                kind, G, nchunk, d = l.args
                if kind not in (ACT_NONE, ACT_RELU, ACT_SIGMOID) or len(d["g"]) != 1 or d.get("dzbuf"):
                    continue
                gp, ggs, gld = d["g"][0]
                prod = producers.get(gp)
                if prod is None:
                    continue
                mode, cfg, PG, pd = prod.args
                if (PG != G or pd["ogs"] != ggs or pd["ldo"] != gld or pd["N"] != d["C"] or pd["B"] != d["B"]
                        or (pd["Ho"], pd["Wo"]) != (d["H"], d["W"]) or d["bn"]["C"] != d["C"]):
                    continue
                pd["bnb"] = {"y": d["y"], "ygs": d["ygs"], "ldy": d["ldy"], "bn": d["bn"], "part": d["part"],
                             "kind": kind}
                d["fused"] = 2
                self.n_dgrad_bnstats += 1
        return self.n_dgrad_bnstats

    def apply_on_load(self) -> int:
        """Fold apply-only BN tails (``fused = 2``, after fuse_dgrad_bn_stats) into their consumers.

        Such a tail reads the fp32 gradient g and the pre-BN y and writes the bf16 dy of its conv, whose
        only readers are that conv's dgrad and wgrad.  Both now rebuild dy from g and y while loading
        their operand (csrc/conv.hip MODE_DGRAD_AOL, wgrad_block<AOL>): the dgrad derives the per-channel
        coefficients from the fused statistics, writes d(gamma), d(beta) and the coefficient table, and
        the wgrad (after it on the same stream) reads that table.  The tail launch and one bf16 write +
        two reads of dy disappear from the backward chain.  ReLU / identity tails only.

        Opt-in (MDA_AOL=1: every eligible conv, MDA_AOL=pw: 1x1 convs only).  Measured on MI355X it
        loses: an im2col operand is loaded KH*KW times, so a 3x3 dgrad re-reads fp32 g + bf16 y and
        redoes the transform 9x per element, and every dgrad block reduces the NREP statistic replicas
        again (Model A backward 767 -> 900 us, Model C -4.5%; 1x1-only: A -2%, C -2.5%).  Returns the number of folded tails."""
        import os
        self.n_aol = 0
        mode = os.environ.get("MDA_AOL", "0")
        if mode not in ("1", "pw"):
            return 0
        ls = self.bwd.launches
        removed = set()
        for i, l in enumerate(ls):
            if not l.name.startswith("tailbwd"):
                continue
            kind, G, nchunk, d = l.args
            if d.get("fused") != 2 or kind not in (ACT_NONE, ACT_RELU) or d.get("dy2") or len(d["g"]) != 1:
                continue
            if l.record is not None and l.waits:
                continue
            dy = d["dy"]
            users = [(j, k) for j, k in enumerate(ls) if j != i and _refers_to(k.args, dy)]
            dg = [(j, k) for j, k in users if k.name == "conv_dgrad" and k.args[3]["src"]["p0"] == dy]
            wg = [(j, k) for j, k in users if k.name == "conv_wgrad" and k.args[2]["dy"] == dy]
            if len(users) != 2 or len(dg) != 1 or len(wg) != 1:
                continue
            (jd, ld), (jw, lw) = dg[0], wg[0]
            _, cfg, DG, dd = ld.args
            if mode == "pw" and dd["KH"] * dd["KW"] != 1:
                continue
            wcfg, WG, wd = lw.args
            if (not (i < jd < jw) or ld.stream != lw.stream or ld.stream != l.stream or DG != G or WG != G
                    or dd["src"].get("C1", 0) != 0 or dd["src"]["gs0"] != d["dgs"] or dd["src"]["ld0"] != d["ldd"]
                    or wd["dgs"] != d["dgs"] or wd["ldd"] != d["ldd"] or dd["Cs"] != d["C"] or wd["Co"] != d["C"]):
                continue
            gp, ggs, gld = d["g"][0]
            ao = {"g": gp, "ggs": ggs, "ldg": gld, "y": d["y"], "ygs": d["ygs"], "ldy": d["ldy"],
                  "coef": P(self._aol_coef(G, d["C"])), "kind": kind}
            dd["aol"] = dict(ao, bn=d["bn"], part=d["part"], dgamma=d.get("dgamma", 0), dbeta=d.get("dbeta", 0),
                             pgs=d.get("pgs", 0))
            wd["aol"] = ao
            nxt = next((k for k in ls[i + 1:] if k.stream == l.stream), None)
            if l.waits:
                nxt.waits = tuple(nxt.waits) + tuple(l.waits)
            if l.record is not None:
                prev = next((k for k in reversed(ls[:i]) if k.stream == l.stream and id(k) not in removed), None)
                if prev is None:
                    continue
                if prev.record is None:
                    prev.record = l.record
                else:
                    self.bwd.alias[l.record] = prev.record
            removed.add(id(l))
            self.n_aol += 1
        self.bwd.launches = [k for k in ls if id(k) not in removed]
        return self.n_aol

    def _aol_coef(self, G: int, C: int) -> torch.Tensor:
        t = torch.empty(G * 5 * C, dtype=torch.float32, device=self.device)
        self.aol_coefs = getattr(self, "aol_coefs", []) + [t]
        return t

    def set_source(self, X: torch.Tensor, labels: torch.Tensor, idx: torch.Tensor):
        """Bind the dataset tensors the gather launch reads (X [N,C,H,W] fp32, labels [N,2], idx [B])."""
        self.src = (X, labels, idx)

    stem_pack = (0, 0)  # (taps, offset) of the gather's vertical tap packing (core.stem_pack_geom)

    def gather_phase(self, X, labels, idx) -> Phase:
        ph = Phase("gather")
        if self.stem_pack[0] and X.shape[1] != 1:
            raise ValueError("stem tap packing needs a single-channel input")
        ph.add("gather", k_gather, X, idx, labels, self.label_width, self.x, self.labels, self.B, X.shape[1], self.H0,
               self.W0, *self.stem_pack)
        return ph

    def _wgfin_args(self, convs=None):
        t, nd, nblocks = build_wgfin_table([c.finalize_desc() for c in (self.convs if convs is None else convs)],
                                           self.device)
        if convs is None:
            self.wgfin_table = t
        self._fin_tables = getattr(self, "_fin_tables", {})
        self._fin_tables[id(convs)] = t  # keep the device table alive for the captured graphs
        return t, nd, nblocks

    def refresh_wgrad_finalize(self):
        """Rebuild the finalize descriptor table(s) after wgrad configs (split counts) changed.  A finalize
        launch's ``owner`` lists the convs it reduces (a gradient bucket's); None means every conv."""
        for l in self.bwd.launches:
            if l.name == "wgrad_finalize":
                l.args = self._wgfin_args(l.owner)

    # ---- gradient buckets (data parallelism) ---------------------------------------
    def bucket_cut_candidates(self) -> List[tuple]:
        """Points of the backward where a gradient bucket could end: ``(anchor, lo, hi)`` means that
        cutting the backward right before launch ``anchor`` completes the gradients of the flat range
        [lo, hi) (cumulative, in backward order; every later launch writes gradients outside it).
        Subclasses override; the default offers none (one bucket)."""
        return []

    def segment_backward(self, n_buckets: int) -> List[tuple]:
        """Split the flat gradient into up to ``n_buckets`` contiguous buckets that complete one after the
        other during the backward, and cut the backward phase accordingly.

        Bucket k's weight gradients (batched per stream by batch_wgrads) and its finalize run at the end of
        backward piece k; the DP step (engine/step.py) replays piece k, issues bucket k's RCCL all-reduce
        on the communication stream and replays piece k+1 meanwhile, so all but the last bucket's
        all-reduce overlap the rest of the backward.  Cuts are chosen among bucket_cut_candidates so that
        the buckets have about equal size.  Must run before autotune_program (which batches the weight
        gradients).  Returns the buckets [(lo, hi)] in completion order."""
        f = self.flat
        self.buckets = [(0, f.numel)]
        if n_buckets <= 1 or any(l.name == "cut" for l in self.bwd.launches):
            return self.buckets
        ls = self.bwd.launches
        cands = [c for c in self.bucket_cut_candidates() if 0 < c[2] - c[1] < f.numel]
        chosen, start = [], 0
        for k in range(1, n_buckets):
            target = k * f.numel / n_buckets
            best = None
            for j in range(start, len(cands)):
                if best is None or abs((cands[j][2] - cands[j][1]) - target) < abs(
                        (cands[best][2] - cands[best][1]) - target):
                    best = j
            if best is None:
                break
            chosen.append(cands[best])
            start = best + 1
        if not chosen:
            return self.buckets
        buckets, prev = [], None
        for _, lo, hi in chosen + [(None, 0, f.numel)]:
            if prev is None:
                b = (lo, hi)
            elif lo == prev[0] and hi >= prev[1]:
                b = (prev[1], hi)
            elif hi == prev[1] and lo <= prev[0]:
                b = (lo, prev[0])
            else:
                raise ValueError(f"bucket ranges are not nested intervals: {prev} then {(lo, hi)}")
            if b[1] > b[0]:
                buckets.append(b)
            prev = (lo, hi)
        bucket_of = lambda off: next(i for i, (lo, hi) in enumerate(buckets) if lo <= off < hi)  # noqa: E731
        anchors = [next(i for i, l in enumerate(ls) if l is a) for a, _, _ in chosen]
        if anchors != sorted(anchors):
            raise ValueError("bucket cut anchors out of backward order")
        seg_of = lambda i: sum(1 for a in anchors if a <= i)  # noqa: E731
        fin = next(i for i, l in enumerate(ls) if l.name == "wgrad_finalize")
        if fin != len(ls) - 1:
            raise ValueError("the weight-gradient finalize must be the backward's last launch")
        # every gradient writer must run no later than its bucket's piece
        gbase = P(f.grads)
        for i, l in enumerate(ls[:fin]):
            seg = seg_of(i)
            if l.name == "conv_wgrad":
                bs = {bucket_of(f.off(m.weight)) for m in l.owner.mods}
                if len(bs) != 1 or seg > min(bs):
                    raise ValueError(f"weight gradient of a bucket-{bs} conv runs in backward piece {seg}")
                l.bucket = bs.pop()
            for off in _grad_offsets(l, gbase, f.numel):
                if seg > bucket_of(off):
                    raise ValueError(f"{l.name} writes bucket {bucket_of(off)} gradients in piece {seg}")
        # cut markers + one finalize per bucket at the end of its piece (waiting for the piece's streams)
        new, bounds = [], anchors + [fin]
        for k in range(len(buckets)):
            lo_i = 0 if k == 0 else bounds[k - 1]
            piece = ls[lo_i:bounds[k]]
            waits = []
            for st in sorted({l.stream for l in piece} - {0}):
                last = [l for l in piece if l.stream == st][-1]
                if last.record is None:
                    last.record = f"bwd_piece{k}_s{st}"
                waits.append(last.record)
            convs = [c for c in self.convs if bucket_of(f.off(c.mods[0].weight)) == k]
            if not convs:
                raise ValueError(f"gradient bucket {k} holds no conv weights")
            new += piece
            new.append(Launch("wgrad_finalize", k_wgfin, *self._wgfin_args(convs), owner=convs, waits=waits,
                              bucket=k))
            if k < len(buckets) - 1:
                new.append(Launch("cut", None))
        self.bwd.launches = new
        self.buckets = buckets
        return buckets

    # ---- early optimizer (single GPU) -------------------------------------------------------------
    def early_opt_enabled(self) -> bool:
        """Adam + re-pack of the side streams' parameters inside the backward (MDA_EARLY_OPT=1, opt-in).
        Measured on MI355X: Model C's optimizer tail 174 -> 14 us, but the backward 2,634 -> 2,826 us (the
        side-stream updates contend with the main stream's stem backward), full step 4,297 vs 4,279 us;
        Model A 32.7k vs 32.5k.  Only without data parallelism: the gradients must be complete before any update, so a program whose
        optimizer averages over ranks (grad_scale != 1), is cut into gradient buckets or runs SyncBN keeps
        the single optimizer launch after the backward."""
        import os
        return (os.environ.get("MDA_EARLY_OPT", "0") == "1" and self._opt_hparams.get("grad_scale", 1.0) == 1.0
                and self.flat.bn_world == 1 and not any(l.name == "cut" for l in self.bwd.launches))

    def _grad_writer_streams(self, bwd_launches) -> Dict[int, set]:
        """Flat offset of each directly written gradient (BN affine parameters, fc) -> the streams that write
        it (-1: written in the forward phase, e.g. the classifier head's fc gradient)."""
        gbase, n = P(self.flat.grads), self.flat.numel
        out: Dict[int, set] = {}
        for l in bwd_launches:
            if l.fn is not None:
                for off in _grad_offsets(l, gbase, n):
                    out.setdefault(off, set()).add(l.stream)
        for l in self.fwd_train.launches:
            if l.fn is not None:
                for off in _grad_offsets(l, gbase, n):
                    out.setdefault(off, set()).add(-1)
        return out

    def _early_segments(self, st: int, convs, writers) -> tuple:
        """Fused Adam + pack segments of the parameters stream ``st`` alone produces: the weights of the convs
        whose weight gradients it batches (finalized just before on the same stream), and every parameter
        whose gradient only ``st`` writes (the BN layers of those convs).  Conv biases stay late."""
        f = self.flat
        segs = [sg for c in convs for sg in c.fused_segments()]
        ranges = [(sg["off"], sg["n"]) for sg in segs]
        conv_params = {id(m.weight) for c in self.convs for m in c.mods}
        conv_params |= {id(m.bias) for c in self.convs for m in c.mods if m.bias is not None}
        for p in self.model.parameters():
            if id(p) in conv_params:
                continue
            o = f.off(p)
            if writers.get(o) == {st}:
                segs.append({"kind": 0, "off": o, "n": p.numel()})
                ranges.append((o, p.numel()))
        segs.sort(key=lambda sg: sg["off"])
        return segs, ranges

    def _set_late_optimizer(self, early_ranges):
        """The optimizer phase after the backward: fused Adam + pack over every parameter not updated early
        (the main stream's convs, conv biases, the head, BN layers written on the main stream), advancing
        the step counter at its end."""
        f = self.flat
        covered = set(early_ranges)
        late = [sg for c in self.convs for sg in c.fused_segments() if (sg["off"], sg["n"]) not in covered]
        conv_w = [(sg["off"], sg["n"]) for c in self.convs for sg in c.fused_segments()]
        late += plain_ranges(f.numel, conv_w + [r for r in early_ranges if r not in set(conv_w)])
        late.sort(key=lambda sg: sg["off"])
        self.late_segs = late
        self.optseg_late, ns, nb = build_optseg_table(late, self.device)
        self.adam_ticket = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._opt_upd = dict(self._opt_base, segs=P(self.optseg_late), nsegs=ns, nblocks=nb, ticket=P(self.adam_ticket))
        upd = Phase("adam")
        upd.add("adam_pack", k_adam, dict(self._opt_upd, update=1, **self._opt_hparams))
        self.opt["adam"] = upd

    def merge_wgrad_cfgs(self, max_batches: Optional[int] = None) -> int:
        """Cap the number of distinct weight-gradient tile configs per stream (= batched launches, which run
        back to back at the end of the stream's backward): repeatedly move the cheapest config group whose
        convs are all valid under another config of the stream into the most expensive such config.  The
        autotuner picks each conv's config from its isolated time, but a batch that holds one small conv
        still costs a full dependent launch on the step's tail (~20 us each on Model A's main stream).
        MDA_WGRAD_MAXB (default 3) sets the cap.  Returns the number of convs moved."""
        import os
        if max_batches is None:
            max_batches = int(os.environ.get("MDA_WGRAD_MAXB", "3"))
        wg = [l for l in self.bwd.launches if l.name == "conv_wgrad" and l.owner is not None]
        moved = 0
        # one batch set per (gradient bucket, stream): a segmented backward batches each bucket separately
        for bk, st in sorted({(l.bucket, l.stream) for l in wg}):
            mine = [l for l in wg if l.stream == st and l.bucket == bk and not l.args[2].get("aol")]
            while True:
                groups = {}
                for l in mine:
                    groups.setdefault(l.args[0], []).append(l)
                if len(groups) <= max_batches:
                    break
                cost = {c: sum(_wgrad_cost(c, l.args[1], l.args[2]) for l in ls) for c, ls in groups.items()}
                move = None
                for c in sorted(groups, key=lambda c: cost[c]):
                    targets = [t for t in groups if t != c and all(l.owner.wgrad_valid(t) for l in groups[c])]
                    if targets:
                        move = (c, max(targets, key=lambda t: cost[t]))
                        break
                if move is None:
                    break
                for l in groups[move[0]]:
                    l.owner.set_wgrad_cfg(move[1])
                    l.args = (move[1],) + tuple(l.args[1:])
                    moved += 1
        self.n_wgrad_merged = moved
        return moved

    def batch_wgrads(self):
        """Replace the per-conv weight-gradient launches by batched launches, one per (stream, tile
        config) (csrc/conv.hip conv_wgrad_batched_kernel).  Each stream's batch goes after that stream's
        last kernel -- after its join events, so nothing waits for the batch except the finalize, and e.g.
        Model A's level-branch weight gradients overlap the backbone's backward.  Called after the
        autotuner has fixed every conv's wgrad config and split count."""
        ls = self.bwd.launches
        wg = [l for l in ls if l.name == "conv_wgrad"]
        if not wg:
            return
        if any(l.name == "cut" for l in ls):
            return self._batch_wgrads_segmented()
        fin = next(i for i, l in enumerate(ls) if l.name == "wgrad_finalize")
        keep = []
        anchor_of = {}  # stream-0 wgrad -> the last kept stream-0 launch before it (its dy producer)
        for l in ls[:fin]:
            if l.name != "conv_wgrad":
                keep.append(l)
                continue
            if l.stream == 0:
                anchor_of[id(l)] = next((k for k in reversed(keep) if k.stream == 0), None)
            if l.record is not None and l.record != "wgrads":
                # an event recorded on a removed launch now stands for the stream's previous kept launch
                prev = next((k for k in reversed(keep) if k.stream == l.stream), None)
                if prev is None:
                    raise RuntimeError(f"cannot re-anchor event {l.record}")
                if prev.record is None:
                    prev.record = l.record
                else:
                    self.bwd.alias[l.record] = prev.record
        import os
        if os.environ.get("MDA_WGRAD_MAIN", "0") == "1" and len({l.stream for l in wg}) > 1:
            # every weight gradient at the main stream's tail (after its last join, so every dy is ready):
            # the side streams' batches no longer contend with the critical backbone chain, and one
            # merged set of at most MDA_WGRAD_MAXB batches fills the GPU
            for l in wg:
                l.stream = 0
            self.merge_wgrad_cfgs()
            self.refresh_wgrad_finalize()
        staged = self._stage_wgrads(wg, ls, anchor_of)
        # MDA_FIN_SPLIT=1 (opt-in; measured neutral: A 31.53-31.58k vs 31.57-31.62k, C 6.89k vs 6.86k): one
        # finalize per stream, right after that stream's batches
        split_ok = (not staged and not self._fan_out_wgrads() and any(l.stream == 0 for l in wg)
                    and all(l.owner is not None for l in wg))
        # early optimizer: each side stream finalizes its convs and runs Adam + the bf16 re-pack on every
        # parameter only it produces gradients for, overlapping the main stream's remaining backward
        early = split_ok and self.early_opt_enabled() and not any(l.args[2].get("aol") for l in wg)
        split_fin = split_ok and (early or os.environ.get("MDA_FIN_SPLIT", "0") == "1")
        writers = self._grad_writer_streams(ls) if early else None
        self.early_adam = []
        self.early_segs = {}
        early_ranges = []
        self.wgfin_tables = []
        self.wgrad_tables = []
        inserts, tags = [], []
        for st in sorted({l.stream for l in wg}):
            batched, costs = [], []
            # key: tile config, + WGRAD_AOL_CFG for the apply-on-load instantiation
            key_of = lambda l: l.args[0] + (WGRAD_AOL_CFG if l.args[2].get("aol") else 0)  # noqa: E731
            for key in sorted({key_of(l) for l in wg if l.stream == st}):
                group = [l for l in wg if l.stream == st and key_of(l) == key]
                raw, nblocks = lib().wgrad_table(key, [l.args[2] for l in group], [l.args[1] for l in group])
                table = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device)
                self.wgrad_tables.append(table)
                batched.append(Launch("wgrad_batched", k_wgrad_batched, key, table, len(group), nblocks, stream=st))
                costs.append(sum(_wgrad_cost(key % WGRAD_AOL_CFG, l.args[1], l.args[2]) for l in group))
            pos = max((i for i, k in enumerate(keep) if k.stream == st), default=len(keep) - 1) + 1
            if staged and st in staged:
                anchor, tag = staged[st]
                pos = keep.index(anchor) + 1
                batched[0].waits = (tag,)
            if st == 0 and len(batched) > 1 and pos > 0 and self._fan_out_wgrads():
                # the main stream's batches form the step's tail (nothing else is left to overlap them):
                # fan them out over the side streams from one fork point so the tile configs run side by
                # side instead of back to back
                batched = self._fan_out(keep, pos, batched, costs)
                tags += [l.record for l in batched if l.record is not None]
            else:
                if split_fin and st != 0:
                    # this stream's convs are finalized on the stream itself, off the main stream's tail
                    t, nd, nb = build_wgfin_table([l.owner.finalize_desc() for l in wg if l.stream == st], self.device)
                    self.wgfin_tables.append(t)
                    batched.append(Launch("wgrad_finalize", k_wgfin, t, nd, nb, stream=st))
                    if early:
                        segs, ranges = self._early_segments(st, [l.owner for l in wg if l.stream == st], writers)
                        self.early_segs[st] = segs
                        if segs:
                            table, ns, nb = build_optseg_table(segs, self.device)
                            self.wgfin_tables.append(table)
                            d = dict(self._opt_base, segs=P(table), nsegs=ns, nblocks=nb, fused=1, ticket=0,
                                     update=1, **self._opt_hparams)
                            batched.append(Launch("adam_early", k_adam, d, stream=st))
                            self.early_adam.append(batched[-1])
                            early_ranges += ranges
                batched[-1].record = f"wgrads_s{st}"
                tags.append(batched[-1].record)
            inserts.append((pos, batched))
        for pos, batched in sorted(inserts, key=lambda x: -x[0]):
            keep[pos:pos] = batched
        for l in keep:  # the per-conv "wgrads" event is gone
            if l.record == "wgrads":
                l.record = None
        fin_l = ls[fin]
        fin_l.waits = tuple(tags)
        if split_fin:  # the main stream's finalize covers its own convs only; the phase end joins the rest
            t, nd, nb = build_wgfin_table([l.owner.finalize_desc() for l in wg if l.stream == 0], self.device)
            self.wgfin_tables.append(t)
            fin_l.args = (t, nd, nb)
            fin_l.waits = ()
        if self.early_adam:
            self._set_late_optimizer(early_ranges)
        self.bwd.launches = keep + ls[fin:]
        self.wgrads_batched = True

    def _batch_wgrads_segmented(self):
        """batch_wgrads for a backward cut into gradient-bucket pieces (segment_backward): in every piece,
        the weight gradients of that piece's bucket are batched per (stream, tile config) after the
        stream's last launch of the piece (a stream without launches there uses stream 0), and the piece's
        finalize waits for those batches.  Weight gradients of a later bucket whose launches sat in an
        earlier piece move to their bucket's piece (their dy is complete by then)."""
        ls = self.bwd.launches
        pieces, cur = [], []
        for l in ls:
            if l.name == "cut":
                pieces.append(cur)
                cur = []
            else:
                cur.append(l)
        pieces.append(cur)
        by_bucket: Dict[int, List[Launch]] = {}
        kept_pieces = []
        for piece in pieces:
            keep = []
            for l in piece:
                if l.name != "conv_wgrad":
                    keep.append(l)
                    continue
                by_bucket.setdefault(l.bucket, []).append(l)
                if l.record is not None:  # the event now stands for the stream's previous kept launch
                    prev = next((k for k in reversed(keep) if k.stream == l.stream), None)
                    if prev is None:
                        raise RuntimeError(f"cannot re-anchor event {l.record}")
                    if prev.record is None:
                        prev.record = l.record
                    else:
                        self.bwd.alias[l.record] = prev.record
            kept_pieces.append(keep)
        self.wgrad_tables = []
        key_of = lambda l: l.args[0] + (WGRAD_AOL_CFG if l.args[2].get("aol") else 0)  # noqa: E731
        out = []
        for k, keep in enumerate(kept_pieces):
            fin = keep.pop()  # segment_backward put the bucket's finalize last in its piece
            assert fin.name == "wgrad_finalize" and fin.bucket == k, fin.name
            mine = by_bucket.get(k, [])
            streams_here = {l.stream for l in keep}
            for l in mine:
                if l.stream not in streams_here:
                    l.stream = 0
            tags = []
            for st in sorted({l.stream for l in mine}):
                batched = []
                for key in sorted({key_of(l) for l in mine if l.stream == st}):
                    group = [l for l in mine if l.stream == st and key_of(l) == key]
                    raw, nblocks = lib().wgrad_table(key, [l.args[2] for l in group], [l.args[1] for l in group])
                    table = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device)
                    self.wgrad_tables.append(table)
                    batched.append(Launch("wgrad_batched", k_wgrad_batched, key, table, len(group), nblocks,
                                          stream=st, bucket=k))
                batched[-1].record = f"wgrads_b{k}_s{st}"
                tags.append(batched[-1].record)
                pos = max((i for i, l in enumerate(keep) if l.stream == st), default=len(keep) - 1) + 1
                keep[pos:pos] = batched
            fin.waits = tuple(fin.waits) + tuple(tags)
            out += keep + [fin]
            if k < len(kept_pieces) - 1:
                out.append(Launch("cut", None))
        self.bwd.launches = out
        self.wgrads_batched = True

    STAGE_STREAM = 2

    def _stage_wgrads(self, wg: List[Launch], ls: List[Launch], anchor_of: dict):
        """MDA_WGRAD_STAGE=f (0 < f < 1): the first fraction f (program order) of the main stream's weight
        gradients -- the deep layers, whose backward kernels leave most CUs idle -- are batched on side
        stream 2 right after their last dy is produced (one fork event), overlapping the rest of the
        backbone's backward instead of queueing at the step's tail.  Only when stream 2 is otherwise
        unused (Model A/B).  Returns (stream, anchor launch) or None."""
        import os
        mode = os.environ.get("MDA_WGRAD_STAGE", self.default_wgrad_stage)
        if mode in ("join", "join2"):
            return self._stage_wgrads_join(wg, ls, anchor_of if mode == "join2" else None)
        frac = float(mode)
        wg0 = [l for l in wg if l.stream == 0]
        n1 = int(len(wg0) * frac)
        if not 0 < n1 < len(wg0) or any(l.stream == self.STAGE_STREAM for l in ls):
            return None
        anchor = anchor_of[id(wg0[n1 - 1])]
        if anchor is None:
            return None
        if anchor.record is None:
            anchor.record = "wgstage"
        else:
            self.bwd.alias["wgstage"] = anchor.record
        for l in wg0[:n1]:
            l.stream = self.STAGE_STREAM
        return {self.STAGE_STREAM: (anchor, "wgstage")}

    def _mark(self, anchor: Launch, tag: str):
        if anchor.record is None:
            anchor.record = tag
        else:
            self.bwd.alias[tag] = anchor.record

    default_wgrad_stage = "0"  # engine/inception.py: "join"

    def _stage_wgrads_join(self, wg: List[Launch], ls: List[Launch], anchor_of: Optional[dict] = None):
        """MDA_WGRAD_STAGE=join: once side stream 2 has issued its last backward launch (the Inception blocks
        are done and only the single-stream stem is left on the main stream), the main stream's weight
        gradients of every layer before that point are batched on stream 2, waiting on the next main-stream
        launch -- they overlap the stem's backward chain instead of queueing at the step's tail.
        MDA_WGRAD_STAGE=join2 (``anchor_of`` given) also moves the first half (program order: the deepest) of
        the remaining main-stream weight gradients -- the stem's -- to stream 1, right after the last of
        their dy producers.  Returns {stream: (anchor launch, event tag)} or None."""
        S = self.STAGE_STREAM
        fin = next(i for i, l in enumerate(ls) if l.name == "wgrad_finalize")
        last2 = max((i for i in range(fin) if ls[i].stream == S and ls[i].name != "conv_wgrad"), default=None)
        if last2 is None:
            return None
        ai = next((i for i in range(last2 + 1, fin) if ls[i].stream == 0 and ls[i].name != "conv_wgrad"), None)
        if ai is None:
            return None
        staged = [l for l in wg if l.stream == 0 and ls.index(l) < ai]
        if not staged:
            return None
        out = {S: (ls[ai], "wgstage")}
        self._mark(ls[ai], "wgstage")
        for l in staged:
            l.stream = S
        if anchor_of is not None:
            rest = [l for l in wg if l.stream == 0 and ls.index(l) > ai]
            g1 = rest[:len(rest) // 2]
            a1 = anchor_of.get(id(g1[-1])) if g1 else None
            last1 = max((i for i in range(fin) if ls[i].stream == 1 and ls[i].name != "conv_wgrad"), default=-1)
            if a1 is not None and ls.index(a1) > last1:
                out[1] = (a1, "wgstage1")
                self._mark(a1, "wgstage1")
                for l in g1:
                    l.stream = 1
        return out

    @staticmethod
    def _fan_out_wgrads() -> bool:
        # opt-in (MDA_WGRAD_FANOUT=1): measured on MI355X, Model A 25.8k -> 23.3k samples/s with the
        # fan-out, Model C 6.47k -> 6.51k (docs/PERF.md "Rejected")
        import os
        return os.environ.get("MDA_WGRAD_FANOUT", "0") == "1"

    def _fan_out(self, keep: List[Launch], pos: int, batched: List[Launch], costs: List[float]) -> List[Launch]:
        """Spread the main stream's batched weight-gradient launches over streams 0, 2, 3, 1 (largest
        first, then greedily onto the least-loaded stream).  Every side stream waits on one event recorded
        after the main stream's last backward kernel; each stream's last batch records the tag the
        finalize waits on."""
        anchor = keep[pos - 1]
        if anchor.record is None:
            anchor.record = "wgfork"
        else:
            self.bwd.alias["wgfork"] = anchor.record
        order = sorted(range(len(batched)), key=lambda i: -costs[i])
        sids = [0, 2, 3, 1]
        load = {s: 0.0 for s in sids}
        out: Dict[int, List[Launch]] = {s: [] for s in sids}
        for n, i in enumerate(order):
            s = sids[n] if n < len(sids) else min(sids, key=lambda x: load[x])
            l = batched[i]
            l.stream = s
            if s != 0 and not out[s]:
                l.waits = ("wgfork",)
            out[s].append(l)
            load[s] += costs[i]
        res = []
        for s in sids:
            if out[s]:
                out[s][-1].record = f"wgrads_s0_{s}"
                res += out[s]
        return res

    def _emit_optimizer(self, grad_scale: float = 1.0) -> Dict[str, Phase]:
        segs = [s for c in self.convs for s in c.opt_segments()]
        self.optseg_table, ns, nblocks = build_optseg_table(segs, self.device)
        f = self.flat
        base = {"p": P(f.params), "g": P(f.grads), "m": P(f.exp_avg), "v": P(f.exp_avg_sq), "n": f.numel,
                "lr": P(f.lr), "step": P(f.step), "segs": P(self.optseg_table), "nsegs": ns, "nblocks": nblocks}
        self._opt_base = base
        self._opt_upd = base
        import os
        if os.environ.get("MDA_FUSED_ADAM", "0") == "1":
            # one launch: Adam + both weight images per conv tile, plain Adam over the other ranges.
            # Opt-in: measured neutral on Model A (31.55k vs 31.59k) and 5% slower on Model C (the tiles
            # give fewer, longer blocks than the elementwise Adam + pack pair)
            fsegs = [s for c in self.convs for s in c.fused_segments()]
            fsegs += plain_ranges(f.numel, [(s["off"], s["n"]) for s in fsegs])
            fsegs.sort(key=lambda s: s["off"])
            self.optseg_fused, nsf, nbf = build_optseg_table(fsegs, self.device)
            self.adam_ticket = torch.zeros(1, dtype=torch.int32, device=self.device)
            self._opt_upd = dict(base, segs=P(self.optseg_fused), nsegs=nsf, nblocks=nbf, ticket=P(self.adam_ticket))
        self._opt_hparams = dict(b1=0.9, b2=0.999, eps=1e-8, wd=0.0, grad_scale=grad_scale)
        upd = Phase("adam")
        upd.add("adam_pack", k_adam, dict(self._opt_upd, update=1, **self._opt_hparams))
        pack = Phase("pack")
        pack.add("pack", k_adam, dict(base, update=0))
        return {"adam": upd, "pack": pack}

    def set_optimizer(self, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, grad_scale: float = 1.0):
        early = getattr(self, "early_adam", [])
        if early and grad_scale != 1.0:
            raise RuntimeError("the early optimizer (single GPU) is already placed in the backward: set the data-"
                               "parallel grad_scale before autotune_program / batch_wgrads")
        self._opt_hparams = dict(b1=betas[0], b2=betas[1], eps=eps, wd=weight_decay, grad_scale=grad_scale)
        for l in early:
            l.args[0].update(self._opt_hparams)
        upd = Phase("adam")
        upd.add("adam_pack", k_adam, dict(self._opt_upd, update=1, **self._opt_hparams))
        self.opt["adam"] = upd

    # -------------------------------------------------------------------------------------------
    def num_launches(self) -> dict:
        return {"forward_train": len(self.fwd_train), "backward": len(self.bwd), "adam": len(self.opt["adam"]) + 1}
