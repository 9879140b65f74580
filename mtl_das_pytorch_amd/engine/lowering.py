"""Shared lowering machinery: the emit helpers every model program uses (conv forward / backward,
fused BN tails and their backward, wgrad finalize, fused Adam + weight packing, batch gather)."""
from __future__ import annotations

import math
import os
from typing import Callable, Dict, List, Optional

import torch

from ..ops.functional import WGRAD_PATCH, WGRAD_TILES, wgrad_ktiles
from ..ops.hip import lib
from .core import (GRAD_DT, Act, BNLayer, ConvLayer, P, build_optseg_table, build_wgfin_table, optimizer_segments,
                   pad_to)
from .program import (COMM_STREAM, SPILL_STREAM, Launch, Phase, k_adam, k_step_inc, k_allreduce, k_ext_record, k_conv, k_gather, k_tail_bwd, k_tail_fwd,
                      k_tail_fwd_batched, k_wgfin, k_wgrad,
                      k_wgrad_batched)

ACT_NONE, ACT_RELU, ACT_SIGMOID, SIGMUL, ADD_RELU, POOL_RELU = range(6)


def _wgrad_cost(cfg: int, G: int, d: dict) -> int:
    """MFMA work (MACs incl. tile padding) of one weight-gradient launch -- used to balance fan-out."""
    if cfg in WGRAD_PATCH:
        TN, CB, _, R = WGRAD_PATCH[cfg]
        px = d["splits"] * d["m_per_split"] * R * pad_to(d["Wo"], 8)
        return px * G * math.ceil(d["Npad"] / TN) * TN * 9 * d["Cs"]
    TN, TK, MCH = WGRAD_TILES[cfg]
    return d["splits"] * d["m_per_split"] * G * TN * TK * math.ceil(d["Npad"] / TN) * wgrad_ktiles(cfg, d["Kpad"])


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


# pixels per thread of a forward BN-tail launch (its grid size; the kernel handles two per iteration)
TAIL_PX_PER_THREAD = 2


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
    LOCAL_BUCKETS = 1    # the same segmentation of the backward in a single process (no collectives)

    # a measured all-reduce of the whole flat gradient shorter than this stays one bucket: each further bucket
    # adds an eager collective's event / stream hops (~20 us per step, profiles/r6_dp_rehearsal.md) and pays only
    # when the overlapped share of the all-reduce (A: 40 %) exceeds that
    OVERLAP_MIN_MS = 0.05

    def dp_buckets(self, world: int, allreduce_ms: Optional[float] = None) -> int:
        """Gradient buckets of a data-parallel step of ``world`` ranks.  Every form of the step overlaps the
        buckets' all-reduces with the rest of the backward inside ONE step graph: captured collectives on the
        communication stream (backward_with_allreduce) or eager RCCL all-reduces ordered after the graph's
        external bucket events (backward_with_ext_events, the multi-rank default).  ``allreduce_ms``: the
        time of one all-reduce of the whole flat gradient measured on the live group at start-up
        (parallel.dist.calibrate_allreduce); below OVERLAP_MIN_MS one bucket.  Otherwise the model's
        default_buckets (A 2, C 4: SURVEY 5.8 sizes C's 83 MB in 2-4 buckets); MDA_BUCKETS overrides."""
        import os
        if world <= 1:
            return self.LOCAL_BUCKETS
        if "MDA_BUCKETS" in os.environ:
            return int(os.environ["MDA_BUCKETS"])
        if allreduce_ms is not None and allreduce_ms < self.OVERLAP_MIN_MS:
            return 1
        return self.default_buckets

    # -------------------------------------------------------------------------------------------
    def _tail_args(self, y: Act, bn: BNLayer, out: Act, training: bool, H=None, W=None) -> tuple:
        d = {"y": y.p, "ygs": y.gs, "ldy": y.ld, "bn": bn.args(training), "out": out.p, "ogs": out.gs, "ldo": out.ld,
             "B": self.B, "H": y.H if H is None else H, "W": y.W if W is None else W, "C": y.C}
        return d, _blocks(self.B * d["H"] * d["W"], y.C, per_thread=TAIL_PX_PER_THREAD)

    def _tail_batch(self, ph: Phase, kind: int, jobs: List[tuple]):
        """One launch for several single-group forward tails of one kind (``jobs``: (args, blocks) from
        _tail_args; csrc/bn.hip tail_fwd_batched_kernel)."""
        raw, nblocks, max_c = lib().tail_table([d for d, _ in jobs], [b for _, b in jobs])
        table = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device)
        self._tail_tables = getattr(self, "_tail_tables", [])
        self._tail_tables.append(table)  # alive as long as the program (captured graphs point at it)
        ph.add(f"tailbatch{kind}", k_tail_fwd_batched, kind, table, len(jobs), nblocks, max_c, owner=jobs)

    def _tail(self, ph: Phase, kind: int, G: int, y: Act, bn: BNLayer, out: Act, training: bool, r: Act = None,
              bn2: BNLayer = None, H=None, W=None):
        d = {"y": y.p, "ygs": y.gs, "ldy": y.ld, "bn": bn.args(training), "out": out.p, "ogs": out.gs, "ldo": out.ld,
             "B": self.B, "H": y.H if H is None else H, "W": y.W if W is None else W, "C": y.C}
        if r is not None:
            d.update({"r": r.p, "rgs": r.gs, "ldr": r.ld})
        if bn2 is not None:
            d["bn2"] = bn2.args(training)
        M = self.B * d["H"] * d["W"]
        ph.add(f"tail{kind}", k_tail_fwd, kind, G, _blocks(M, y.C, per_thread=TAIL_PX_PER_THREAD), d)

    def _tail_bwd(self, ph: Phase, kind: int, G: int, y: Act, bn: BNLayer, g: list, dy: Act, r: Act = None,
                  bn2: BNLayer = None, side: Act = None, dy2: Act = None):
        """BN-tail backward launch (reduce + apply, or the single-launch kernel; fuse_dgrad_bn_stats may
        later turn it into an apply-only pass)."""
        d = {"y": y.p, "ygs": y.gs, "ldy": y.ld, "bn": bn.args(True), "B": self.B, "H": y.H, "W": y.W, "C": y.C,
             "g": g, "part": P(bn.part, bn.part_off), "chunk_px": bn.chunk_px, "dy": dy.p, "dgs": dy.gs,
             "ldd": dy.ld}
        if kind in (SIGMUL, POOL_RELU) or len(g) > 1:
            # the apply pass reads the stored dz instead of re-reading several gradient sources /
            # re-evaluating the pool window
            if bn.dzbuf is None:
                bn.dzbuf = self.arena.empty((G, y.M, y.C), GRAD_DT)
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

    def enable_sync_bn(self, allreduce, skip_fwd=(), skip_bwd=()) -> int:
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
        ``skip_fwd`` / ``skip_bwd``: replica-row pointers (forward stats / backward part) of BNs whose
        collective a subclass emits itself, coalesced with their siblings' (engine/inception.py).
        Where the process group's collectives are capturable (DistContext.capturable_collectives: a 1-rank
        RCCL group, or several ranks with MDA_CAPTURE_COLLECTIVES=1) they are captured into the step's HIP
        graph (stream-ordered; those of BNs on streams >= COLLECTIVE_STREAMS go through stream 0); otherwise
        -- gloo, and RCCL with several ranks by default -- the step runs eagerly (EngineBackend warns;
        bench.py --dp-shape 8 --sync_bn measures that form on one GPU).  Returns the number of all-reduces
        inserted per training step."""
        world = self.flat.bn_world
        by_stats = {}
        for bn in self.flat.bn_layers:  # a fused conv's members share its rows: the member at offset 0 stands for all
            by_stats.setdefault(P(bn.stats, bn.stats_off if "stats" in bn.coalesced else 0), bn)
        by_part = {P(bn.part, bn.part_off): bn for bn in self.flat.bn_layers}
        skip_fwd, skip_bwd = set(skip_fwd), set(skip_bwd)
        n = 0
        new = []
        for l in self.fwd_train.launches:
            new.append(l)
            st = l.args[3].get("stats") or 0 if l.name == "conv_fwd" else 0
            bn = by_stats.get(st) if st not in skip_fwd else None
            if bn is not None:
                new += self._collective(allreduce, bn.used_stats(), l.stream, l.bucket, l.record)
                l.record = None
                n += 1
        self.fwd_train.launches = new
        new = []
        for l in self.bwd.launches:
            if not l.name.startswith("tailbwd") or l.args[3].get("fused") == 3 or l.args[3]["part"] in skip_bwd:
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
                new += [l] + self._collective(allreduce, bn.used_part(), l.stream, l.bucket)
            elif l.stream < self.COLLECTIVE_STREAMS:  # statistics from the producing dgrad's epilogue
                l.name, l.fn, l.args = "allreduce_bn", k_allreduce, (allreduce, bn.used_part())
                new.append(l)
            else:  # (the launch keeps its waits as a kernel-free fork point in front of the collective)
                l.name, l.fn, l.args = f"fork:{l.name}", None, ()
                new += [l] + self._collective(allreduce, bn.used_part(), l.stream, l.bucket)
            d = {k: v for k, v in d.items() if k not in ("dzbuf", "dzgs", "lddz")}
            d["fused"], d["gscale"] = 2, 1.0 / world
            new.append(Launch(name, k_tail_bwd, kind, G, nchunk, d, owner=l.owner, stream=l.stream, record=record,
                              bucket=l.bucket))
            n += 1
        self.bwd.launches = new
        self.sync_bn_world = world
        return n

    # Collectives captured into the step graph from at most these streams (0 and 1: Model A's backbone and
    # level branches); a collective of a BN on a later stream (Model C's Inception branches) runs on stream 0
    # between a record / wait pair of events -- issued from four capturing streams, RCCL's internal stream
    # invalidated the HIP graph capture (hipErrorStreamCaptureInvalidated at bench.py --sync_bn, Model C)
    COLLECTIVE_STREAMS = 2

    def _collective(self, allreduce, t, stream: int, bucket, record=None) -> List[Launch]:
        """All-reduce launch(es) of ``t`` ordered after ``stream``'s previous launches and before its next ones;
        ``record``: the event the last of them records (the tag the replaced launch carried)."""
        if stream < self.COLLECTIVE_STREAMS:
            return [Launch("allreduce_bn", k_allreduce, allreduce, t, stream=stream, record=record, bucket=bucket)]
        self._n_routed = getattr(self, "_n_routed", 0) + 1
        tp, ta = f"sbn_p{self._n_routed}", f"sbn_a{self._n_routed}"
        return [Launch(f"fork:{tp}", None, stream=stream, record=tp, bucket=bucket),
                Launch("allreduce_bn", k_allreduce, allreduce, t, stream=0, waits=(tp,), record=ta, bucket=bucket),
                Launch(f"fork:{ta}", None, stream=stream, waits=(ta,), record=record, bucket=bucket)]

    @staticmethod
    def nol_enabled() -> bool:
        """Normalise-on-load (MDA_NOL, default on; 0 is a debugging switch): a conv whose input is the
        single-consumer output of a BN + ReLU tail reads the pre-BN y and applies the BN affine + ReLU to its
        im2col operand (and so does its weight gradient), so that tail is never launched (csrc/conv.hip
        MODE_FWD_NOL)."""
        import os
        return os.environ.get("MDA_NOL", "1") == "1"

    # Normalise-on-load only for consumer convs with at most this many output pixels (B*Ho*Wo): on the
    # large stem maps the on-load transform (repeated KH*KW times per element by the im2col) costs more
    # than the BN+ReLU tail it removes (per-model constant; docs/PERF.md has the sweep)
    NOL_MAX_PX = 1 << 30

    def nol_for(self, conv: ConvLayer) -> bool:
        return self.nol and conv.M_out <= self.NOL_MAX_PX

    def _conv_fwd(self, ph: Phase, c: ConvLayer, src: dict, out: Act, bn: BNLayer, training: bool, nol=None):
        mode, cfg, G, d = c.fwd_args(src, out, bn, training)
        if nol is not None:  # (BNLayer of the input, activation kind)
            d["nol"] = {"bn": nol[0].args(training), "kind": nol[1]}
        ph.add("conv_fwd", k_conv, mode, cfg, G, d, owner=c)

    def _conv_bwd(self, ph: Phase, c: ConvLayer, src: dict, dy: Act, dx: Optional[Act], nol=None):
        # data gradient first (it is on the critical chain), then the per-conv weight gradient on the same
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

    # Fold the gradient sources of multi-source BN tails into the last producing dgrad (fold_tail_sources);
    # programs whose tails join streams (Inception's concat consumers) keep it off: the fold moves the
    # tail's cross-stream waits onto that dgrad, which would serialise the branches
    FOLD_SOURCES = False

    def fold_tail_sources(self) -> int:
        """A BN tail backward with 2-4 fp32 gradient sources, the last of them written by a data gradient on
        the tail's own stream: that dgrad's epilogue adds the other sources (csrc ConvArgs::add), its output
        becomes the tail's only source, and the tail's waits (the other sources' events) move onto the dgrad.
        The tail then qualifies for fuse_dgrad_bn_stats -- the statistics come from the dgrad epilogue and
        the tail runs apply-only: Model A's residual-block ADD_RELU tails lose their reduce pass and their
        re-reads of four fp32 sources.  Returns the number of folded tails."""
        import os
        self.n_folded = 0
        if not self.FOLD_SOURCES or os.environ.get("MDA_FOLD", "1") != "1":
            return 0
        ls = self.bwd.launches
        recorded_at = {}  # event tag -> index of the launch that records it
        for i, l in enumerate(ls):
            if l.record is not None:
                recorded_at[l.record] = i
        last_dgrad = {}  # stream -> (index, launch) of its latest dgrad
        for i, l in enumerate(ls):
            if l.name == "conv_dgrad":
                last_dgrad[l.stream] = (i, l)
                continue
            if not l.name.startswith("tailbwd"):
                continue
            kind, G, nchunk, d = l.args
            g = d["g"]
            if kind not in (ACT_NONE, ACT_RELU, ADD_RELU) or not 2 <= len(g) <= 4 or l.stream not in last_dgrad:
                continue
            j, D = last_dgrad[l.stream]
            if any(k.stream == l.stream and k.name not in ("conv_wgrad",) for k in ls[j + 1:i]):
                continue  # something else runs between the dgrad and the tail
            mode, cfg, PG, pd = D.args
            mine = [q for q, (p, gs, ld) in enumerate(g) if p == pd["out"] and gs == pd["ogs"] and ld == pd["ldo"]]
            if (len(mine) != 1 or PG != G or pd.get("add") or pd["N"] != d["C"]
                    or (pd["Ho"], pd["Wo"]) != (d["H"], d["W"]) or pd["B"] != d["B"]):
                continue
            # the tail's waits move onto the earlier dgrad: each awaited event must be recorded before it in
            # launch order (else Phase.run would meet the wait before the record -- or a reused tag would
            # make the dgrad wait on a stale event and race the added sources)
            if any(recorded_at.get(self.bwd.alias.get(w, w), len(ls)) >= j for w in l.waits):
                continue
            pd["add"] = [{"p": p, "gs": gs, "ld": ld} for q, (p, gs, ld) in enumerate(g) if q != mine[0]]
            d["g"] = [g[mine[0]]]
            for k in ("dzbuf", "dzgs", "lddz"):
                d.pop(k, None)
            D.waits = tuple(D.waits) + tuple(l.waits)
            l.waits = ()
            self.n_folded += 1
        return self.n_folded

    def fuse_dgrad_bn_stats(self) -> int:
        """Move the BN-backward reduction of single-source elementwise tails into the producing dgrad.

        A BN tail whose activation is elementwise (none / ReLU / sigmoid) and whose output gradient has
        exactly ONE source -- the data gradient of the next conv, written once as fp32 on the tail's own
        pixel grid -- gets its per-channel sum(dz), sum(dz * xhat) from that dgrad's epilogue
        (csrc/conv.hip, ConvArgs::bpart), and its backward runs the apply pass only (``fused = 2``): one
        launch and one full pass over the gradient less per such layer (Model A: the 8 residual-block
        inner BNs and the 4 attention-generator BNs; Model C: every BasicConv2d feeding exactly one
        other).  Returns the number of fused layers."""
        self.n_dgrad_bnstats = 0
        producers = {}
        for l in self.bwd.launches:
            if l.name == "conv_dgrad":
                producers[l.args[3]["out"]] = l
            elif l.name.startswith("tailbwd"):
                kind, G, nchunk, d = l.args
                if kind not in (ACT_NONE, ACT_RELU, ACT_SIGMOID, ADD_RELU) or len(d["g"]) != 1 or d.get("dzbuf"):
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
                if kind == ADD_RELU:  # the residual (and its BN for a projection shortcut) enters the dz mask
                    pd["bnb"].update({"r": d["r"], "rgs": d["rgs"], "ldr": d["ldr"]})
                    if "bn2" in d:
                        pd["bnb"]["bn2"] = d["bn2"]
                d["fused"] = 2
                self.n_dgrad_bnstats += 1
        return self.n_dgrad_bnstats

    def set_source(self, X: torch.Tensor, labels: torch.Tensor, idx: torch.Tensor):
        """Bind the dataset tensors the gather launch reads (X [N,C,H,W] fp32, labels [N,2], idx [B])."""
        self.src = (X, labels, idx)

    stem_pack = (0, 0)  # (taps, offset) of the gather's vertical tap packing (core.stem_pack_geom)

    def gather_phase(self, X, labels, idx, clear: bool = False, cursor=None) -> Phase:
        """The batch gather; ``clear``: the same launch also zeroes the arena's zeroed region (what
        ``arena.clear`` does at the start of a training step), unless the guard allocator keeps every zeroed
        view in its own banded buffer -- then ``arena.clear`` runs first.  ``cursor``: ``idx`` is a
        [nrows][B] batch-index schedule and the gather takes row ``cursor`` mod nrows (the optimizer's
        step-counter kernel advances the cursor: set_step_cursor)."""
        if cursor is not None and (idx.dim() != 2 or idx.shape[1] != self.B):
            raise ValueError(f"index schedule must be [nrows][{self.B}], got {tuple(idx.shape)}")
        ph = Phase("gather")
        if self.stem_pack[0] and X.shape[1] != 1:
            raise ValueError("stem tap packing needs a single-channel input")
        zero = []
        if clear:
            zero = self.arena.zero_ranges()
            if zero is None:
                ph.add("clear", lambda st: self.arena.clear())
                zero = []
        ph.add("gather", k_gather, X, idx, labels, self.label_width, self.x, self.labels, self.B, X.shape[1], self.H0,
               self.W0, *self.stem_pack, zero, cursor)
        return ph

    def _wgfin_args(self, convs=None):
        t, nd, nblocks = build_wgfin_table([d for c in (self.convs if convs is None else convs) for d in c.finalize_descs()],
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
        self.bucket_anchors = None
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

    def stream_buckets(self, max_buckets: int) -> List[tuple]:
        """Gradient buckets for the eager-collective data-parallel step (backward_with_ext_events) WITHOUT cutting
        the backward: a bucket is a prefix range of the flat gradient whose every writer runs on ONE side stream
        no later than that stream's own finalize (batch_wgrads' SIDE_FINALIZE), so it is complete when that
        finalize is -- while stream 0 still runs its data-gradient chain -- and its all-reduce overlaps the rest
        of the backward with no extra join of the streams (segment_backward's cut joins every stream at the
        bucket boundary: A 30.0 k vs 33.3 k samples/s at 2 vs 1 buckets on the per-rank program of 8 GPUs).
        The remainder is the last bucket, complete at the tail finalize.  Model A: the level parameters lead the
        flat buffer and are written on stream 1 only.  Call after autotune_program (batched weight gradients)
        on a backward that segment_backward left whole.  Returns the buckets [(lo, hi)] in completion order."""
        f = self.flat
        ls = self.bwd.launches
        if any(l.name == "cut" for l in ls):
            raise ValueError("stream_buckets needs an uncut backward (segment_backward(1))")
        writers, side_fin = self._grad_writers()
        buckets, anchors, k, lo = [], [], 0, 0
        order = f.order
        # (a parameter with no writer -- a conv bias feeding a BN, whose gradient is identically 0 -- is never
        # written during the step: complete in any bucket)
        while k < len(order) and len(buckets) < max_buckets - 1:
            w = next((writers[f.off(q)] for q in order[k:] if f.off(q) in writers), None)
            st = next(iter(w))[0] if w else None
            if st not in side_fin:
                break
            j = k
            while j < len(order):
                w = writers.get(f.off(order[j]))
                if w and any(s2 != st or i2 > side_fin[st] for s2, i2 in w):
                    break
                j += 1
            hi = f.off(order[j]) if j < len(order) else f.numel
            if hi <= lo:
                break
            buckets.append((lo, hi))
            anchors.append(ls[side_fin[st]])
            lo, k = hi, j
        fins = [l for l in ls if l.name == "wgrad_finalize"]
        buckets.append((lo, f.numel))
        # the remainder is complete once every stream has joined stream 0 after its finalize (batch_wgrads)
        after = ls[ls.index(fins[-1]) + 1] if ls.index(fins[-1]) + 1 < len(ls) else None
        anchors.append(after if after is not None and after.name == "join_side" else fins[-1])
        self.buckets, self.bucket_anchors = buckets, anchors
        return buckets

    def _grad_writers(self):
        """(flat offset of a parameter's gradient -> {(stream, backward launch index)} of every launch writing
        it, side stream -> index of its own weight-gradient finalize).  A batched launch (engine/inception.py
        batch_tails: a device job table) writes what its ``owner`` launches would have."""
        f = self.flat
        gbase = P(f.grads)
        writers: Dict[int, set] = {}
        for i, l in enumerate(self.bwd.launches):
            if l.name == "wgrad_finalize":
                for c in (l.owner or self.convs):  # (no owner: the finalize covers every conv)
                    for m in c.mods:
                        writers.setdefault(f.off(m.weight), set()).add((l.stream, i))
            elif l.fn is not None:
                srcs = [l] + [o for o in (l.owner if isinstance(l.owner, (list, tuple)) else ())
                              if isinstance(o, Launch)]
                for src in srcs:
                    for off in _grad_offsets(src, gbase, f.numel):
                        writers.setdefault(off, set()).add((l.stream, i))
        side_fin = {l.stream: i for i, l in enumerate(self.bwd.launches)
                    if l.name == "wgrad_finalize" and l.stream != 0}
        return writers, side_fin

    def stream_param_order(self) -> Optional[list]:
        """A parameter order for the flat buffers (FlatState ``param_groups``) under which stream_buckets finds
        one bucket per side stream: first the parameters whose gradient only that side stream writes, no later
        than its own finalize, side streams in finalize order; then the rest in module order.  A program built
        with it (Model C: ``InceptionProgram(param_order=...)``, build_for_stream_buckets) all-reduces those
        buckets while stream 0 still runs the rest of the backward.  Call on a program lowered like the one to
        be built (autotuned, uncut).  None: no side stream finalizes a parameter of its own."""
        f = self.flat
        writers, side_fin = self._grad_writers()
        cls = {}
        for q in f.order:
            w = writers.get(f.off(q))
            sts = {s for s, _ in w} if w else set()
            st = next(iter(sts)) if len(sts) == 1 else None
            ok = st in side_fin and all(i <= side_fin[st] for _, i in w)
            cls[id(q)] = st if ok else 0
        sides = sorted((s for s in side_fin if any(c == s for c in cls.values())), key=lambda s: side_fin[s])
        if not sides:
            return None
        return [q for s in sides for q in f.order if cls[id(q)] == s] + [q for q in f.order if cls[id(q)] == 0]

    def backward_with_allreduce(self, allreduce) -> Phase:
        """The backward with every gradient bucket's all-reduce embedded in it, so the whole
        data-parallel step -- forward, backward, collectives, optimizer -- is one HIP graph.  Each bucket's
        finalize (segment_backward: one per bucket, at the end of its piece) records an event, and an
        ``allreduce(grads[lo:hi])`` launch on the communication stream waits for it: bucket k's collective
        overlaps pieces k+1.. of the backward, and the optimizer, the next phase, waits for every collective
        through the phase-end join of the communication stream.  ``allreduce`` must be stream-ordered
        (DistContext.all_reduce_ordered_; captured on RCCL)."""
        f = self.flat
        buckets = getattr(self, "buckets", None) or [(0, f.numel)]
        ph = Phase("backward_dp")
        ph.alias = dict(self.bwd.alias)
        fins = [l for l in self.bwd.launches if l.name == "wgrad_finalize"]
        last = {l.bucket: l for l in fins}  # a bucket may be finalized by several streams (SIDE_FINALIZE)
        done = {}
        for l in self.bwd.launches:
            if l.name == "cut":
                continue
            if l.name != "wgrad_finalize":
                ph.launches.append(l)
                continue
            tag = l.record or f"bucket{l.bucket}_grads_{len(done.get(l.bucket, []))}"
            ph.launches.append(Launch(l.name, l.fn, *l.args, owner=l.owner, stream=l.stream, waits=l.waits,
                                      record=tag, bucket=l.bucket))
            done.setdefault(l.bucket, []).append(tag)
            if l is last[l.bucket]:
                lo, hi = buckets[l.bucket]
                ph.launches.append(Launch("allreduce_grads", k_allreduce, allreduce, f.grads[lo:hi],
                                          stream=COMM_STREAM, waits=tuple(done[l.bucket]), bucket=l.bucket))
        if sorted(done) != list(range(len(buckets))):
            raise ValueError(f"finalize launches for buckets {sorted(done)}, expected {len(buckets)} buckets")
        return ph

    def backward_with_ext_events(self, events) -> Phase:
        """The backward with an EXTERNAL event recorded where each gradient bucket is complete: ``events[k]`` is
        an ExtEvent (engine/program.py), so in the captured step graph it is an event-record node.  The
        data-parallel step at world > 1 (engine/step.py "train_ext") replays forward + this backward as one
        graph and then, on the host, makes the communication stream wait for ``events[k]`` and issues bucket
        k's eager RCCL all-reduce there: bucket k's collective runs while the graph computes the rest of the
        backward -- overlap without capturing multi-rank collectives.  Buckets from stream_buckets: the event
        follows the bucket's side-stream finalize; from segment_backward: it follows the bucket's last finalize,
        joined over the finalizes' streams."""
        f = self.flat
        buckets = getattr(self, "buckets", None) or [(0, f.numel)]
        if len(events) != len(buckets):
            raise ValueError(f"{len(events)} events for {len(buckets)} buckets")
        ph = Phase("backward_ext")
        ph.alias = dict(self.bwd.alias)
        anchors = getattr(self, "bucket_anchors", None)
        if anchors is not None and len(anchors) == len(buckets):
            at = {id(a): k for k, a in enumerate(anchors)}
            for l in self.bwd.launches:
                ph.launches.append(l)
                if id(l) in at:
                    ph.launches.append(Launch("ext_record", k_ext_record, events[at[id(l)]], stream=l.stream))
            return ph
        fins = [l for l in self.bwd.launches if l.name == "wgrad_finalize"]
        last = {l.bucket: l for l in fins}
        done = {}
        for l in self.bwd.launches:
            if l.name == "cut":
                continue
            if l.name != "wgrad_finalize":
                ph.launches.append(l)
                continue
            tag = l.record or f"bucket{l.bucket}_grads_{len(done.get(l.bucket, []))}"
            ph.launches.append(Launch(l.name, l.fn, *l.args, owner=l.owner, stream=l.stream, waits=l.waits,
                                      record=tag, bucket=l.bucket))
            done.setdefault(l.bucket, []).append(tag)
            if l is last[l.bucket]:
                ph.launches.append(Launch("ext_record", k_ext_record, events[l.bucket], stream=l.stream,
                                          waits=tuple(t for t in done[l.bucket] if t != tag), bucket=l.bucket))
        if sorted(done) != list(range(len(buckets))):
            raise ValueError(f"finalize launches for buckets {sorted(done)}, expected {len(buckets)} buckets")
        return ph

    WGRAD_MAX_BATCHES = 3
    # the same cap for stream 0 only (its batches run serially after the data-gradient chain); None: as above
    WGRAD_MAX_BATCHES_S0 = None
    # hardware blocks of a side stream's batched weight-gradient launch (0: one per virtual block): a capped,
    # persistent grid leaves CU slots free for the critical chain's kernels (csrc/conv.hip WGRAD_FOR_VBLOCKS)
    SIDE_WGRAD_GRID = 0

    def merge_wgrad_cfgs(self, max_batches: Optional[int] = None) -> int:
        """Cap the number of distinct weight-gradient tile configs per stream (= batched launches, which run
        back to back at the end of the stream's backward): repeatedly move the cheapest config group whose
        convs are all valid under another config of the stream into the most expensive such config.  The
        autotuner picks each conv's config from its isolated time, but a batch that holds one small conv
        still costs a full dependent launch on the step's tail (~20 us each on Model A's main stream).
        The cap is WGRAD_MAX_BATCHES (swept 1/2/3/4/none in docs/PERF.md).  Returns the number of convs moved."""
        if max_batches is None:
            max_batches = self.WGRAD_MAX_BATCHES
        wg = [l for l in self.bwd.launches if l.name == "conv_wgrad" and l.owner is not None]
        moved = 0
        # one batch set per (gradient bucket, stream): a segmented backward batches each bucket separately
        for bk, st in sorted({(l.bucket, l.stream) for l in wg}):
            mine = [l for l in wg if l.stream == st and l.bucket == bk]
            cap = self.WGRAD_MAX_BATCHES_S0 if st == 0 and self.WGRAD_MAX_BATCHES_S0 else max_batches
            while True:
                groups = {}
                for l in mine:
                    groups.setdefault(l.args[0], []).append(l)
                if len(groups) <= cap:
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

    def batch_tails(self) -> int:
        """Batch independent BN-tail backward passes into shared launches after tuning (models whose lowering
        knows such groups override this; engine/inception.py)."""
        return 0

    def spill_wgrads(self, frac: float) -> int:
        """Move the weight gradients of stream 0's EARLIEST convs (in backward order; about ``frac`` of stream
        0's weight-gradient work) to their own batches on the spill stream, which start as soon as the last
        of them has its dy -- while stream 0 still runs the rest of its data-gradient chain.

        batch_wgrads otherwise puts every stream-0 weight gradient after stream 0's last kernel, and stream
        0 ends the backward (the stem / first residual blocks, serial dgrads of a few us each that leave most
        of the GPU idle).  Measured: Model C +1-2 % at frac 0.7 (the stem's wide-map weight gradients stay
        at the end, the Inception blocks' move); Model A -2..-8 % at any fraction, also with the spilled
        blocks capped at one per CU -- its stream-0 chain of small dgrads slows by more than the ~110 us of
        batches it sheds (tools/timeline.py: +150 us).  Chosen per model in the step by tune_in_context
        (table entry wgspill|..., percent; 0 = off).  Must run before merge_wgrad_cfgs / batch_wgrads; a
        backward cut into gradient-bucket pieces is left alone.  Returns the number of convs moved."""
        ls = self.bwd.launches
        if frac <= 0 or any(l.name == "cut" for l in ls):
            return 0
        wg0 = [l for l in ls if l.name == "conv_wgrad" and l.stream == 0]
        # a launch recording an event (other than the per-conv "wgrads" tag) ends the movable prefix
        cut = next((i for i, l in enumerate(wg0) if l.record not in (None, "wgrads")), len(wg0))
        wg0 = wg0[:cut]
        cost = [_wgrad_cost(l.args[0], l.args[1], l.args[2]) for l in wg0]
        total, acc, n = sum(cost), 0, 0
        while n < len(wg0) and acc + cost[n] <= frac * total:
            acc += cost[n]
            n += 1
        if n == 0:
            return 0
        last = next(i for i, l in enumerate(ls) if l is wg0[n - 1])
        ls.insert(last + 1, Launch("fork:wgspill", None, stream=0, record="wgspill"))
        for l in wg0[:n]:
            l.stream = SPILL_STREAM
            l.waits = tuple(l.waits) + ("wgspill",)
        self.n_wgrad_spilled = n
        return n

    # side streams finalize their own weight gradients (batch_wgrads) and, in a single process, update them:
    # C +0.6-7.5 % / A neutral, and A +0.3-0.6 % / C neutral (docs/PERF.md round 4); class switches for A/B runs
    SIDE_FINALIZE = True
    EARLY_ADAM = True
    # stream 0's tail finalize waits for every side stream's last launch (the round-5 form; class switch)
    JOIN_AT_FINALIZE = False

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
        for l in ls[:fin]:
            if l.name != "conv_wgrad":
                keep.append(l)
                continue
            if l.record is not None and l.record != "wgrads":
                # an event recorded on a removed launch now stands for the stream's previous kept launch
                prev = next((k for k in reversed(keep) if k.stream == l.stream), None)
                if prev is None:
                    raise RuntimeError(f"cannot re-anchor event {l.record}")
                if prev.record is None:
                    prev.record = l.record
                else:
                    self.bwd.alias[l.record] = prev.record
        self.wgrad_tables = []
        inserts, tags = [], []
        for st in sorted({l.stream for l in wg}):
            batched = []
            for cfg in sorted({l.args[0] for l in wg if l.stream == st}):
                group = [l for l in wg if l.stream == st and l.args[0] == cfg]
                batched.append(self._wgrad_batch_launch(cfg, group, st))
            # the jobs' own waits (spilled weight gradients: the spill point) go on the stream's first batch
            batched[0].waits = tuple(dict.fromkeys(w for l in wg if l.stream == st for w in l.waits))
            # list position = capture order, which the graph executor follows when it dispatches: a batch
            # goes right after its stream's last kernel or the launch recording what it waits for (a spilled
            # batch appended at the end of the list started after stream 0's whole chain)
            pos = max([i for i, k in enumerate(keep) if k.stream == st or (k.record and k.record in batched[0].waits)],
                      default=len(keep) - 1) + 1
            batched[-1].record = f"wgrads_s{st}"
            tags.append(batched[-1].record)
            inserts.append((pos, batched))
        if self.SIDE_FINALIZE:
            # every side stream reduces its own convs' split slabs right after its batches (overlapping
            # stream 0's remaining chain); the tail finalize keeps stream 0's convs
            side = {}
            for l in wg:
                if l.stream != 0 and l.owner is not None:
                    side.setdefault(l.stream, []).append(l.owner)
            for pos_batched in inserts:
                batched = pos_batched[1]
                st = batched[-1].stream
                if st in side:
                    convs = list(dict.fromkeys(side[st]))
                    tag = f"wgfin_s{st}"
                    batched.append(Launch("wgrad_finalize", k_wgfin, *self._wgfin_args(convs), owner=convs, stream=st,
                                          record=tag))
                    tags = [t for t in tags if t != batched[-2].record] + [tag]
            early_ok = self.EARLY_ADAM and not self.data_parallel and self._opt_hparams.get("grad_scale", 1.0) == 1.0
            done = [c for v in side.values() for c in v]
            rest = [c for c in self.convs if c not in done]
            if side and rest:
                ls[fin].owner = rest
                ls[fin].args = self._wgfin_args(rest)
            if side and early_ok:
                # single process: the side convs' Adam + re-pack right after their finalize, on their stream
                # (the optimizer phase then covers the rest); with gradient averaging (DP, set_optimizer's
                # data_parallel) the update must wait for the all-reduce, so it stays in the optimizer phase
                early = set()
                for pos_batched in inserts:
                    batched = pos_batched[1]
                    st = batched[-1].stream
                    if st not in side:
                        continue
                    offs = {self.flat.off(m.weight) for c in side[st] for m in c.mods}
                    segs = [g for g in self.opt_segs if g["kind"] == 3 and g["off"] in offs]
                    early |= offs
                    table, ns, nb = build_optseg_table(segs, self.device)
                    self._opt_tables = getattr(self, "_opt_tables", []) + [table]
                    d = dict(self._opt_base, segs=P(table), nsegs=ns, nblocks=nb, update=1, inc_step=0,
                             t_pre=int(self._step_early is not None), **self._opt_hparams)
                    tag = f"adam_s{st}"
                    batched.append(Launch("adam_pack_early", k_adam, d, stream=st, record=tag))
                    tags = [t for t in tags if t != f"wgfin_s{st}"] + [tag]
                    self._early_adam = getattr(self, "_early_adam", []) + [d]
                segs = [g for g in self.opt_segs if not (g["kind"] == 3 and g["off"] in early)]
                table, ns, nb = build_optseg_table(segs, self.device)
                self._opt_tables = getattr(self, "_opt_tables", []) + [table]
                self._opt_base = dict(self._opt_base, segs=P(table), nsegs=ns, nblocks=nb)
                self.set_optimizer(**self._opt_kwargs)
        for pos, batched in sorted(inserts, key=lambda x: -x[0]):
            keep[pos:pos] = batched
        for l in keep:  # the per-conv "wgrads" event is gone
            if l.record == "wgrads":
                l.record = None
        side_tags = tuple(t for t in tags if t != "wgrads_s0")
        if self.SIDE_FINALIZE and side and not self.JOIN_AT_FINALIZE:
            # stream 0's finalize reduces stream 0's convs only: it follows its own batches in stream order, and
            # the side streams (their finalize, early Adam) join stream 0 after it -- a pseudo-launch, the last
            # bucket's anchor (stream_buckets) -- instead of delaying it (A: the tail finalize waited ~20 us
            # for stream 1's early Adam, profiles/r6_timeline_modelA_end.txt)
            ls[fin].waits = ()
            self.bwd.launches = keep + ls[fin:fin + 1] + [Launch("join_side", None, stream=0, waits=side_tags)] \
                + ls[fin + 1:]
        else:
            ls[fin].waits = tuple(tags)
            self.bwd.launches = keep + ls[fin:]
        self.wgrads_batched = True

    def _wgrad_batch_launch(self, cfg: int, group: List[Launch], st: int, bucket: int = 0) -> Launch:
        raw, nblocks = lib().wgrad_table(cfg, [l.args[2] for l in group], [l.args[1] for l in group])
        table = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device)
        self.wgrad_tables.append(table)
        cap = self.SIDE_WGRAD_GRID if st != 0 else 0
        return Launch("wgrad_batched", k_wgrad_batched, cfg, table, len(group), nblocks, cap, stream=st, bucket=bucket)

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
                batched = [self._wgrad_batch_launch(cfg, [l for l in mine if l.stream == st and l.args[0] == cfg],
                                                    st, k)
                           for cfg in sorted({l.args[0] for l in mine if l.stream == st})]
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

    def _emit_optimizer(self, grad_scale: float = 1.0) -> Dict[str, Phase]:
        f = self.flat
        segs = optimizer_segments([s for c in self.convs for s in c.opt_segments()], f.numel)
        self.opt_segs = segs
        self.optseg_table, ns, nblocks = build_optseg_table(segs, self.device)
        base = {"p": P(f.params), "g": P(f.grads), "m": P(f.exp_avg), "v": P(f.exp_avg_sq), "n": f.numel,
                "lr": P(f.lr), "step": P(f.step), "segs": P(self.optseg_table), "nsegs": ns, "nblocks": nblocks}
        self._opt_base = base
        self._opt_hparams = dict(b1=0.9, b2=0.999, eps=1e-8, wd=0.0, grad_scale=grad_scale)
        self._opt_kwargs = dict(betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, grad_scale=grad_scale)
        self.data_parallel = False
        upd = Phase("adam")
        upd.add("adam_pack", k_adam, dict(base, update=1, **self._opt_hparams))
        pack = Phase("pack")
        pack.add("pack", k_adam, dict(base, update=0))
        return {"adam": upd, "pack": pack}

    def set_optimizer(self, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, grad_scale: float = 1.0,
                      data_parallel: bool = False):
        """Adam hyper-parameters.  ``data_parallel``: the gradients are all-reduced across processes before the
        update (any DP group, also a 1-rank one), so no weight may be updated inside the backward (early Adam
        is then never emitted; ``grad_scale`` = 1/world folds the averaging into the update)."""
        self._opt_kwargs = dict(betas=betas, eps=eps, weight_decay=weight_decay, grad_scale=grad_scale,
                                data_parallel=data_parallel)
        self._opt_hparams = dict(b1=betas[0], b2=betas[1], eps=eps, wd=weight_decay, grad_scale=grad_scale)
        self.data_parallel = bool(data_parallel)
        if getattr(self, "_early_adam", None) and (grad_scale != 1.0 or data_parallel):
            raise RuntimeError("the weight updates already run inside the backward: gradient averaging would miss them")
        for d in getattr(self, "_early_adam", []):  # the side streams' partial updates (batch_wgrads)
            d.update(self._opt_hparams)
        upd = Phase("adam")
        upd.add("adam_pack", k_adam, dict(self._opt_base, update=1, **self._opt_hparams, **self._step_mode()))
        self.opt["adam"] = upd
        self.set_step_cursor(getattr(self, "_step_cursor", None))

    _step_early = None  # the step-counter launch's args once use_early_step_counter moved it into the forward
    EARLY_STEP_COUNTER = True  # class switch for A/B runs (tools/variant.py)

    def _step_mode(self) -> dict:
        return {"t_pre": 1, "inc_step": 0} if self._step_early is not None else {}

    def use_early_step_counter(self) -> bool:
        """Advance the Adam step counter (and a schedule cursor) at the START of the training step, by a one-
        thread launch on the forward's first side stream, instead of after the last Adam launch, where it ended
        the step's critical tail (rocprof, Model A: 4 us kernel + its dependency gap; profiles/r6_kernels_*).
        Every Adam launch then uses t = step (AdamArgs::t_pre).  The launch waits for what the side stream's
        first forward launch waits for (after the gather phase, which reads the cursor), and every Adam launch
        follows it through the forward -> backward joins.  For the step runner (engine/step.py), which always
        runs the forward before the update; phases run by hand keep the old form.  Idempotent; False (no
        change) when the forward has no side stream."""
        if self._step_early is not None:
            return True
        if not self.EARLY_STEP_COUNTER:
            return False
        ls = self.fwd_train.launches
        i = next((i for i, l in enumerate(ls) if l.stream != 0), None)
        if i is None:
            return False
        self._step_early = {"step": self.flat.step.data_ptr()}
        ls.insert(i, Launch("step_inc", k_step_inc, self._step_early, stream=ls[i].stream, waits=tuple(ls[i].waits)))
        for d in getattr(self, "_early_adam", []):
            d.update(t_pre=1, inc_step=0)
        self.set_optimizer(**self._opt_kwargs)
        return True

    def set_step_cursor(self, cursor: Optional[torch.Tensor]):
        """The device int64 cursor of a batch-index schedule (gather_phase ``cursor``): the step-counter kernel
        advances it together with the Adam step count (csrc/optim.hip step_inc_kernel) -- after the last Adam
        launch, or early in the step (use_early_step_counter) -- after every gather block has read it.  None
        detaches it."""
        self._step_cursor = cursor
        ds = [l.args[0] for l in self.opt["adam"].launches if l.name == "adam_pack"]
        if self._step_early is not None:
            ds = [self._step_early]
        for d in ds:
            if cursor is None:
                d.pop("cursor", None)
            else:
                d["cursor"] = cursor.data_ptr()
    # -------------------------------------------------------------------------------------------
    def num_launches(self) -> dict:
        return {"forward_train": len(self.fwd_train), "backward": len(self.bwd), "adam": len(self.opt["adam"]) + 1}


def build_for_stream_buckets(make: Callable, n_buckets: int):
    """The eager-collective data-parallel program with up to ``n_buckets`` side-stream gradient buckets
    (LoweredProgram.stream_buckets).  ``make(param_order)`` builds, configures and autotunes a program on an
    uncut backward.  Where the parameter order the model's constructor gives has no side-stream prefix (Model C:
    the stem comes first in module order, so its one bucket completed at the very end), the program is built a
    second time with stream_param_order(), which groups each side stream's parameters.  Returns (program,
    buckets)."""
    prog = make(None)
    if n_buckets > 1 and getattr(prog, "REORDER_FOR_STREAM_BUCKETS", False):
        order = prog.stream_param_order()
        if order is not None:
            del prog
            import gc
            gc.collect()
            torch.cuda.empty_cache()
            prog = make(order)
    return prog, prog.stream_buckets(n_buckets)
