"""The MI355X lowering is pure bookkeeping until launch time: build it on the CPU and check the program
structure, the grouped (per-task) parameter layout and the descriptor tables."""
import pytest
import torch

from mtl_das_pytorch_amd.engine.mtl import MTLProgram
from mtl_das_pytorch_amd.models import MTL_Net, Single_Task_Net


def test_mtl_program_structure():
    m = MTL_Net()
    sd_before = {k: v.clone() for k, v in m.state_dict().items()}
    p = MTLProgram(m, 32, "cpu")
    # parameters now live in the flat buffer but keep their values and keys
    for k, v in m.state_dict().items():
        assert torch.equal(v, sd_before[k]), k
    assert p.flat.numel >= sum(x.numel() for x in m.parameters())
    n = p.num_launches()
    # forward: 9 BN+ReLU tails are folded into their consumer conv (normalise-on-load; the three on the 33x83
    # maps stay separate launches, MTLProgram.NOL_MAX_PX), and RB3/5/7's conv a and projection shortcut are
    # one fused conv each (one forward, one data gradient, one wgrad job)
    assert n["forward_train"] == 48 and n["backward"] == 84
    for R in (p.rbs[2], p.rbs[4], p.rbs[6]):
        cas = R["cas"]
        assert R["fused"] and cas.concat and cas.Co == 2 * R["ya"].C and [t for _, _, t in cas.members] == [0, 4]
        assert R["ys"].off == R["ya"].C and R["ys"].ld == cas.Co and R["bns"].sld == cas.Co
        assert "dxs" not in R and "cs" not in R
    # the residual tails have 2-4 gradient sources: the last producing dgrad sums them (fold_tail_sources)
    # and fuses the tail's statistics, so 7 of 8 run apply-only; RB8's tail has no dgrad before it
    tails = [l for l in p.bwd.launches if l.name == "tailbwd4"]
    assert len(tails) == 8 and p.n_folded == 8
    assert [l.args[3].get("fused", 0) == 2 for l in tails] == [False] + [True] * 7
    assert all(len(l.args[3]["g"]) == 1 and not l.waits for l in tails[1:])
    folded = [l for l in p.bwd.launches if l.name == "conv_dgrad" and l.args[3].get("add")]
    assert len(folded) == 8 and all(1 <= len(l.args[3]["add"]) <= 3 for l in folded)
    # both task branches of a level are ONE grouped launch with an even parameter stride
    L = p.levels[1]
    assert L["c0"].G == 2 and L["c0"].wstride > 0
    g0, g1 = m.att_mask_generato2[0][0].weight, m.att_mask_generato2[1][0].weight
    assert p.flat.off(g1) - p.flat.off(g0) == L["c0"].wstride
    # shared backbone input read with group stride 0, per-task prev level with stride > 0
    assert L["Fa"].gs == 0 and L["prevB"].gs > 0
    assert p.wgfin_table.numel() == (len(p.convs) + 3) * 88  # one finalize descriptor per fused member
    # fused optimizer: one segment per conv weight (both images), plain ranges for the rest; exact cover
    assert sum(s["kind"] == 3 for s in p.opt_segs) == sum(c.G for c in p.convs) + 3
    assert sum(s["n"] for s in p.opt_segs) == p.flat.numel and p.optseg_table.numel() == len(p.opt_segs) * 88
    assert all(a["off"] + a["n"] == b["off"] for a, b in zip(p.opt_segs, p.opt_segs[1:]))


def test_single_task_program():
    p = MTLProgram(Single_Task_Net("event"), 8, "cpu")
    assert p.T == 1 and p.lab_off == [1]
    assert all(c.G == 1 for c in p.convs)


def test_flat_state_views_track_module():
    m = MTL_Net()
    p = MTLProgram(m, 4, "cpu")
    with torch.no_grad():
        m.conv1[0].weight.fill_(0.5)
    o = p.flat.off(m.conv1[0].weight)
    assert torch.all(p.flat.params[o:o + m.conv1[0].weight.numel()] == 0.5)
    m.conv1[1].running_mean.fill_(2.0)
    assert p.flat.bn_mean[p.flat.bn_offsets[id(m.conv1[1])]].item() == 2.0


def test_inception_program_structure():
    """Model C lowers to 94 conv+BN+ReLU units and 13 pools; branch outputs are channel slices of the
    block buffers (no concatenation), and every value has 1..6 gradient sources."""
    from mtl_das_pytorch_amd.engine.inception import CBR, HConv, InceptionProgram, Pool
    from mtl_das_pytorch_amd.models import Multi_Classifier
    m = Multi_Classifier()
    sd_keys = list(m.state_dict())
    p = InceptionProgram(m, 4, "cpu")
    cbr = [o for o in p.ops if isinstance(o, CBR)]
    pools = [o for o in p.ops if isinstance(o, Pool)]
    hcs = [o for o in p.ops if isinstance(o, HConv)]
    assert len(cbr) == sum(1 for x in m.modules() if isinstance(x, torch.nn.Conv2d)) == 94
    assert len(pools) == 13
    assert (p.feat.act.H, p.feat.act.W, p.feat.act.C) == (1, 6, 2048)
    # horizontal fusion of the sibling 1x1 heads: InceptionA (5b-5d) and C (6b-6e) three each, D (7a) two,
    # E (7b, 7c) three -- InceptionB (6a) has none
    assert [len(h.members) for h in hcs] == [3, 3, 3, 3, 3, 3, 3, 2, 3, 3]
    assert hcs[0].conv.Co == 64 + 48 + 64 and hcs[-1].conv.Co == 320 + 384 + 448
    n_conv = 94 - sum(len(h.members) - 1 for h in hcs)  # conv launches: one per fused group
    assert n_conv == 94 - 19 == len(p.convs)
    kernels = lambda ph: sum(1 for l in ph.launches if l.fn is not None)  # not the fork points
    # tails folded into their consumer conv; the blocks' branch-output tails batched one launch per block
    assert kernels(p.fwd_train) == n_conv + 94 + 13 + 1 - p.n_nol - p.n_tail_batched + 11
    assert kernels(p.bwd) == 94 + 2 * n_conv - 1 + 13 + 1   # the stem conv has no data gradient
    # Mixed_5b's 1x1 branch writes channels [0, 64) of the 256-wide block buffer in place; its pre-BN y is a
    # slice of the fused group's output, its BN sums a slice of the group's combined replica rows
    blk = [o for o in cbr if o.module is m.Mixed_5b.branch1x1][0]
    assert blk.out.act.ld == 256 and blk.out.coff == 0 and blk.out.parent is not None
    assert blk.fused[0] is hcs[0] and blk.y.ld == hcs[0].conv.Co and blk.bn.sld == hcs[0].conv.Co
    b5 = [o for o in cbr if o.module is m.Mixed_5b.branch5x5_1][0]
    assert b5.y.off == 64 and b5.bn.args(True)["stats"] == hcs[0].stats.data_ptr() + 64 * 8
    for o in p.ops:
        if isinstance(o, (CBR, Pool)):
            assert 1 <= len(o.out.grad_sources()) <= 6
    # Mixed_5b's input gets ONE gradient source from the three fused heads (plus the pool branch's)
    assert len(hcs[0].src.grads) == 2
    # every parameter has a gradient producer: conv weights (finalize: one descriptor per fused member), BN
    # (tails), fc (head); the checkpoint key space is unchanged
    assert p.wgfin_table.numel() == 94 * 88
    assert list(p.model.state_dict()) == sd_keys and len(sd_keys) == 566
    _check_event_order(p.fwd_train)
    _check_event_order(p.bwd)


def test_wgrad_batching_structure():
    """All per-conv weight-gradient launches collapse into one launch per (stream, tile config); every conv
    appears in exactly one job table and exactly one finalize."""
    p = MTLProgram(MTL_Net(), 32, "cpu")
    n_wg = sum(1 for l in p.bwd.launches if l.name == "conv_wgrad")
    p.batch_wgrads()
    b = [l for l in p.bwd.launches if l.name == "wgrad_batched"]
    assert sum(l.args[2] for l in b) == n_wg
    fin, join = p.bwd.launches[-2:]
    assert fin.name == "wgrad_finalize" and fin.stream == 0 and join.name == "join_side" and join.fn is None
    fins = [l for l in p.bwd.launches if l.name == "wgrad_finalize"]
    # side streams finalize their own convs right after their batches; the tail finalize keeps stream 0's
    # and follows stream 0's batches in stream order, then every side stream joins stream 0; every conv is
    # finalized exactly once
    side = [l for l in fins if l.stream != 0]
    assert {l.stream for l in side} == {l.stream for l in b} - {0}
    # (with EARLY_ADAM each side stream's last launch is its partial Adam update, which the join waits for)
    last = {st: [l for l in p.bwd.launches if l.stream == st][-1] for st in {l.stream for l in side}}
    assert fin.waits == () and set(join.waits) == {l.record for l in last.values()}
    assert all(l.name == ("adam_pack_early" if p.EARLY_ADAM else "wgrad_finalize") for l in last.values())
    owners = [c for l in fins for c in l.owner]
    assert len(owners) == len(set(map(id, owners))) == len(p.convs)
    _check_event_order(p.bwd)


def test_dgrad_fused_bn_stats_wiring():
    """Single-source BN tails take their backward sums from the producing dgrad's epilogue (Model A: 8
    residual-block inner BNs + 4 grouped attention-generator BNs, and -- their sources folded into the last
    dgrad -- 7 residual ADD_RELU tails and conv1's tail)."""
    from mtl_das_pytorch_amd.engine.inception import InceptionProgram
    from mtl_das_pytorch_amd.models import Multi_Classifier
    p = MTLProgram(MTL_Net(), 8, "cpu")
    assert p.n_dgrad_bnstats == 20
    fused = [l for l in p.bwd.launches if l.name.startswith("tailbwd") and l.args[3].get("fused") == 2]
    bnb = [l for l in p.bwd.launches if l.name == "conv_dgrad" and "bnb" in l.args[3]]
    assert len(fused) == len(bnb) == 20
    res = [x for x in bnb if x.args[3]["bnb"]["kind"] == 4]  # ADD_RELU: residual (+ its BN) in the mask
    assert len(res) == 7 and sum("bn2" in x.args[3]["bnb"] for x in res) == 3
    for l in fused:
        kind, G, nchunk, d = l.args
        prod = [x for x in bnb if x.args[3]["out"] == d["g"][0][0]]
        assert len(prod) == 1 and prod[0].args[3]["bnb"]["part"] == d["part"] and prod[0].args[2] == G
        assert p.bwd.launches.index(prod[0]) < p.bwd.launches.index(l)
    c = InceptionProgram(Multi_Classifier(), 4, "cpu")
    assert c.n_dgrad_bnstats >= 40


def test_stem_tap_packing_geometry():
    """Single-channel stems run as 1 x KW convs over KH packed taps (the gather writes x[h - ph + j] into
    channel j): Model A's reduction shrinks from 416 to 64, Model C's from 96 to 32; output shapes and the
    weight layout seen by pack / finalize are the real ones."""
    from mtl_das_pytorch_amd.engine.core import stem_pack_geom
    from mtl_das_pytorch_amd.engine.inception import InceptionProgram
    from mtl_das_pytorch_amd.models import Multi_Classifier
    p = MTLProgram(MTL_Net(), 4, "cpu")
    c1 = p.conv1
    assert p.stem_pack == (7, 2)
    assert (c1.Ci, c1.KH, c1.KW, c1.Cs, c1.ph, c1.pw, c1.Ho, c1.Wo, c1.Kpad) == (7, 1, 7, 8, 0, 2, 33, 83, 64)
    d = c1.finalize_desc()
    assert d["elems"] == 16 * 7 * 7 and (d["Ci"], d["KH"], d["KW"]) == (7, 1, 7)
    c = InceptionProgram(Multi_Classifier(), 4, "cpu")
    s = c.ops[0].conv
    assert c.stem_pack == (3, 0) and (s.Ho, s.Wo, s.Kpad) == (49, 124, 32)
    assert stem_pack_geom(MTL_Net(in_channels=2).conv1[0], 100, 250) is None
    p2 = MTLProgram(MTL_Net(in_channels=2), 4, "cpu")
    assert p2.stem_pack == (0, 0) and p2.conv1.Kpad == 416  # 7*7*8 padded to 32


def _check_event_order(ph):
    seen = set()
    for l in ph.launches:
        for w in l.waits:
            assert ph.alias.get(w, w) in seen, (ph.name, l.name, w)
        if l.record:
            seen.add(l.record)


def test_stream_events_are_recorded_before_they_are_awaited():
    """Multi-stream programs (levels || backbone in A, Inception branches on streams 0..3 in C): every
    event a launch waits on is recorded by an earlier launch, before and after wgrad batching."""
    from mtl_das_pytorch_amd.engine.inception import InceptionProgram
    from mtl_das_pytorch_amd.models import Multi_Classifier
    for prog in (MTLProgram(MTL_Net(), 4, "cpu"), InceptionProgram(Multi_Classifier(), 4, "cpu")):
        for batched in (False, True):
            if batched:
                prog.batch_wgrads()
            for ph in (prog.fwd_train, prog.fwd_eval, prog.bwd):
                _check_event_order(ph)
    streams = {l.stream for l in prog.fwd_train.launches}
    assert streams == {0, 1, 2, 3}  # Inception branches spread over four streams


def test_merge_wgrad_cfgs_caps_batches_per_stream():
    """After tuning, small weight-gradient config groups are folded into a valid config of the same
    stream so that each stream's tail holds at most WGRAD_MAX_BATCHES batched launches."""
    from mtl_das_pytorch_amd.ops.functional import WGRAD_PATCH, WGRAD_TILES
    p = MTLProgram(MTL_Net(), 32, "cpu")
    wg = [l for l in p.bwd.launches if l.name == "conv_wgrad"]
    cfgs = sorted(WGRAD_TILES) + sorted(WGRAD_PATCH)
    for i, l in enumerate(wg):  # scatter the convs over every config valid for them
        valid = [c for c in cfgs if l.owner.wgrad_valid(c)]
        c = valid[i % len(valid)]
        l.owner.set_wgrad_cfg(c)
        l.args = (c,) + tuple(l.args[1:])
    before = {st: len({l.args[0] for l in wg if l.stream == st}) for st in {l.stream for l in wg}}
    assert max(before.values()) > 3
    assert p.merge_wgrad_cfgs(3) > 0
    for st in before:
        assert len({l.args[0] for l in wg if l.stream == st}) <= 3
    for l in wg:
        assert l.owner.wgrad_valid(l.args[0]) and l.args[2]["splits"] == l.owner.splits
    p.batch_wgrads()
    _check_event_order(p.bwd)


def test_inception_aux_logits_shape_error():
    """aux_logits at the DAS input: the reference's own InceptionAux cannot run (avg_pool 5/3 on 4 x 13); the
    engine says so instead of lowering a configuration that does not exist."""
    import torch
    from mtl_das_pytorch_amd.engine.inception import InceptionProgram, _mixed6_hw
    from mtl_das_pytorch_amd.models.multi_classifier import Multi_Classifier
    assert _mixed6_hw((100, 250)) == (4, 13)
    assert _mixed6_hw((299, 299)) == (17, 17)  # torchvision's comment sizes
    m = Multi_Classifier(aux_logits=True).train()
    with pytest.raises(RuntimeError, match="too small"):
        m(torch.randn(2, 1, 100, 250))
    with pytest.raises(ValueError, match="4 x 13"):
        InceptionProgram(m, 2, "cpu")


def test_guard_allocator_cpu_fallback():
    """On the CPU (or with the guard off) the guard allocator is plain torch.zeros / torch.empty."""
    from mtl_das_pytorch_amd.engine import guard
    t = guard.alloc((3, 4), torch.float32, "cpu", zero=True)
    assert t.shape == (3, 4) and not t.any()
    guard.enable(True)
    try:
        t = guard.alloc(5, torch.int64, "cpu", zero=True)  # CPU tensors are never guarded
        assert t.shape == (5,) and guard.count() == 0 and guard.check() == []
    finally:
        guard.enable(False)
        guard.reset()


@pytest.mark.parametrize("nb", [1, 2])
def test_backward_with_allreduce_structure(nb):
    """Data-parallel step as one graph (engine/step.py train_full_dp): every gradient bucket's finalize records
    an event and one all-reduce of exactly that bucket's flat range waits for it on the communication stream;
    the buckets cover the flat buffer once, and the program's own backward is left untouched."""
    from mtl_das_pytorch_amd.engine.program import COMM_STREAM
    p = MTLProgram(MTL_Net(), 32, "cpu")
    buckets = p.segment_backward(nb)
    assert len(buckets) == nb
    before = [(l.name, l.record) for l in p.bwd.launches]
    seen = []
    ph = p.backward_with_allreduce(lambda t: seen.append(t))
    assert [(l.name, l.record) for l in p.bwd.launches] == before
    fins = [l for l in ph.launches if l.name == "wgrad_finalize"]
    ars = [l for l in ph.launches if l.name == "allreduce_grads"]
    assert len(fins) == len(ars) == nb and not any(l.name == "cut" for l in ph.launches)
    covered = 0
    for f, a in zip(fins, ars):
        assert a.stream == COMM_STREAM and a.waits == (f.record,)
        lo, hi = buckets[f.bucket]
        t = a.args[1]
        assert t.data_ptr() == p.flat.grads[lo:hi].data_ptr() and t.numel() == hi - lo
        covered += t.numel()
        assert ph.launches.index(a) > ph.launches.index(f)
    assert covered == p.flat.numel


@pytest.mark.parametrize("model", ["MTL", "multi_classifier"])
def test_spill_wgrads(model):
    """The earliest stream-0 weight gradients move to the spill stream: their batch waits for the spill
    point, sits right after it in capture order, and the finalize waits for it."""
    from mtl_das_pytorch_amd.engine.program import SPILL_STREAM
    from mtl_das_pytorch_amd.models import build_model
    m = build_model(model)
    if model == "multi_classifier":
        from mtl_das_pytorch_amd.engine.inception import InceptionProgram
        p = InceptionProgram(m, 32, "cpu")
    else:
        p = MTLProgram(m, 32, "cpu")
    n0 = sum(1 for l in p.bwd.launches if l.name == "conv_wgrad" and l.stream == 0)
    n = p.spill_wgrads(0.7)
    assert 0 < n < n0
    p.merge_wgrad_cfgs()
    p.batch_wgrads()
    _check_event_order(p.bwd)
    ls = p.bwd.launches
    fork = next(i for i, l in enumerate(ls) if l.record == "wgspill")
    sp = [i for i, l in enumerate(ls) if l.stream == SPILL_STREAM]
    assert sp and sp[0] == fork + 1 and ls[sp[0]].waits == ("wgspill",)
    tail = 2 if p.EARLY_ADAM else 1  # the stream's finalize (and partial Adam) follow its batches
    assert all(l.name == "wgrad_batched" for l in (ls[i] for i in sp[:-tail]))
    # the spill stream finalizes (and with EARLY_ADAM updates) its own convs after its batches; the tail
    # finalize waits for that
    assert ls[sp[-1]].name == ("adam_pack_early" if p.EARLY_ADAM else "wgrad_finalize")
    assert ls[sp[-1]].record in ls[-1].waits


def test_inception_tail_batches_structure():
    """Model C's forward: every Inception block's branch-output tails in one launch after the join."""
    from mtl_das_pytorch_amd.engine.inception import InceptionProgram
    from mtl_das_pytorch_amd.models import build_model
    p = InceptionProgram(build_model("multi_classifier"), 32, "cpu")
    names = [l.name for l in p.fwd_train.launches]
    assert names.count("tailbatch1") == 11 and names.count("tail1") + names.count("tailbatch1") <= 30
    assert sum(len(l.owner) for l in p.fwd_train.launches if l.name == "tailbatch1") == p.n_tail_batched == 44
    for ph in (p.fwd_train, p.fwd_eval):
        _check_event_order(ph)
        for l in ph.launches:
            if l.name == "tailbatch1":
                assert l.stream == 0


@pytest.mark.parametrize("model", ["single_event", "multi_classifier"])
def test_optimizer_segments_cover_flat(model):
    """The fused Adam + pack covers every flat element exactly once: one tile segment per conv weight
    (both of its bf16 images), plain ranges in between."""
    from mtl_das_pytorch_amd.models import build_model
    m = build_model(model)
    if model == "multi_classifier":
        from mtl_das_pytorch_amd.engine.inception import InceptionProgram
        p = InceptionProgram(m, 8, "cpu")
    else:
        p = MTLProgram(m, 8, "cpu")
    segs = p.opt_segs
    assert segs[0]["off"] == 0 and sum(s["n"] for s in segs) == p.flat.numel
    assert all(a["off"] + a["n"] == b["off"] for a, b in zip(segs, segs[1:]))
    convw = {p.flat.off(mod.weight) for c in p.convs for mod in c.mods}
    assert {s["off"] for s in segs if s["kind"] == 3} == convw


def test_stream_slots_count_comm_and_spill_in_the_queue_budget():
    """the communication and spill streams share the hardware-queue budget with the compute
    streams (more streams than queues crashes graph replay, tools/hwq_repro.py)."""
    from mtl_das_pytorch_amd.engine.program import COMM_STREAM, MAX_STREAMS, SPILL_STREAM, Launch, stream_slots

    def ls(*ids):
        return [Launch("x", None, stream=s) for s in ids]

    for hwq in (1, 2, 3, 4, 8):
        for ids in ((0, 1, 2, 3), (0, 1, 2, 3, COMM_STREAM), (0, 1, 2, 3, COMM_STREAM, SPILL_STREAM),
                    (0, 1, SPILL_STREAM), (0, COMM_STREAM)):
            m = stream_slots(ls(*ids), hw_queues=hwq)
            assert len(set(m.values())) <= max(1, hwq), (hwq, ids, m)
            assert m[0] == 0 and all(0 <= v <= MAX_STREAMS + 1 for v in m.values())
            if COMM_STREAM in ids and hwq >= 2:
                assert m[COMM_STREAM] == MAX_STREAMS  # the collective keeps a stream of its own when it can
    # the round-4 Model C DP case: 4 compute branches + the comm stream on 4 queues -> 3 compute streams
    m = stream_slots(ls(0, 1, 2, 3, COMM_STREAM), hw_queues=4)
    assert sorted(set(m.values())) == [0, 1, 2, MAX_STREAMS]


def test_executor_schedule_rule_on_a_recorded_dot():
    """graphsched.schedule reproduces the HIP graph executor's StreamId of every node of a recorded
    DEBUG_HIP_GRAPH_DOT_PRINT dump (tools/hwq_repro.py --streams 3 --layers 2 on MI355X: 16 nodes; the
    Model A / C step dumps of round 5 match as well, profiles/r5_graph_streams.md)."""
    from mtl_das_pytorch_amd.engine import graphsched as gs
    edges = [(0, 1), (1, 8), (1, 10), (1, 12), (2, 3), (3, 6), (4, 5), (5, 6), (5, 8), (5, 10), (5, 12), (6, 7),
             (7, 8), (7, 10), (7, 12), (8, 9), (10, 11), (11, 14), (12, 13), (13, 14), (14, 15)]
    truth = [0, 0, 1, 1, 2, 2, 1, 1, 0, 0, 1, 1, 2, 2, 1, 1]
    ch = [[] for _ in range(16)]
    for a, b in edges:
        ch[a].append(b)
    assert gs.schedule(ch, 4) == truth  # recorded with the runtime's default 4 executor streams


@pytest.mark.parametrize("model", ["A", "C"])
def test_executor_schedule_rule_on_recorded_step_dumps_at_two_streams(model):
    """The executor rule at the package's 2 executor streams: every node's StreamId of the recorded Model A
    (120 nodes) and Model C (292 nodes) step graphs (tests/data/graph_dot_2streams.json, recorded on MI355X
    with tools/graph_dot.py) -- and the 4-stream rule does NOT reproduce C's dump, so the dump really is
    the 2-stream executor."""
    import json
    import os
    from mtl_das_pytorch_amd.engine import graphsched as gs
    d = json.load(open(os.path.join(os.path.dirname(__file__), "data", "graph_dot_2streams.json")))[model]
    assert gs.schedule(d["children"], 2) == d["stream"]
    if model == "C":
        assert gs.schedule(d["children"], 4) != d["stream"]


@pytest.mark.parametrize("model", ["MTL", "single_distance"])
def test_stream_buckets_need_no_cut(model):
    """The multi-rank DP step's buckets (LoweredProgram.stream_buckets): the first is a prefix of the flat
    gradient written only on stream 1, complete at stream 1's own finalize (its external event follows that
    launch, no stream join); the remainder completes at the tail finalize.  Model A: the level parameters."""
    from mtl_das_pytorch_amd.engine.core import P
    from mtl_das_pytorch_amd.engine.lowering import _grad_offsets
    from mtl_das_pytorch_amd.models import build_model
    m = build_model(model)
    p = MTLProgram(m, 32, "cpu")
    p.set_optimizer(weight_decay=1e-5, data_parallel=True)
    p.segment_backward(1)
    p.merge_wgrad_cfgs()
    p.refresh_wgrad_finalize()
    p.batch_wgrads()
    b = p.stream_buckets(2)
    f, ls = p.flat, p.bwd.launches
    assert len(b) == 2 and b[0][0] == 0 and b[0][1] == b[1][0] and b[1][1] == f.numel and b[0][1] > f.numel // 5
    a0, a1 = p.bucket_anchors
    assert a0.name == "wgrad_finalize" and a0.stream == 1 and a1.name == "join_side" and a1 is ls[-1]
    i0 = next(i for i, l in enumerate(ls) if l is a0)
    gbase = P(f.grads)
    for i, l in enumerate(ls):  # nothing writes bucket 0 after stream 1's finalize, or on another stream
        offs = _grad_offsets(l, gbase, f.numel) if l.name != "wgrad_finalize" else \
            [f.off(mm.weight) for c in (l.owner or p.convs) for mm in c.mods]
        if any(o < b[0][1] for o in offs):
            assert l.stream == 1 and i <= i0, (i, l.name, l.stream)
    ph = p.backward_with_ext_events(["e0", "e1"])
    recs = [(i, l.args[0]) for i, l in enumerate(ph.launches) if l.name == "ext_record"]
    assert [e for _, e in recs] == ["e0", "e1"]
    assert ph.launches[recs[0][0] - 1] is a0 and ph.launches[recs[0][0]].stream == 1


def test_early_step_counter_placement():
    """use_early_step_counter: the one-thread step-counter launch moves from after the last Adam launch to the
    forward's first side-stream position (same stream and waits), every Adam launch then uses t = step and never
    advances the counter itself, and a schedule cursor rides on the moved launch.  Off for Model C."""
    from mtl_das_pytorch_amd.engine.inception import InceptionProgram
    from mtl_das_pytorch_amd.models import Multi_Classifier
    p = MTLProgram(MTL_Net(), 8, "cpu")
    ls = p.fwd_train.launches
    i = next(k for k, l in enumerate(ls) if l.stream != 0)
    first = ls[i]
    assert p.use_early_step_counter() and p.use_early_step_counter()  # idempotent
    inc = [l for l in p.fwd_train.launches if l.name == "step_inc"]
    assert len(inc) == 1 and p.fwd_train.launches[i] is inc[0] and p.fwd_train.launches[i + 1] is first
    assert inc[0].stream == first.stream and inc[0].waits == first.waits
    d = p.opt["adam"].launches[0].args[0]
    assert d["t_pre"] == 1 and d["inc_step"] == 0
    cur = torch.zeros(1, dtype=torch.int64)
    p.set_step_cursor(cur)
    assert inc[0].args[0]["cursor"] == cur.data_ptr() and "cursor" not in d
    p.set_optimizer(weight_decay=1e-5)  # a rebuilt optimizer phase keeps the form
    d = p.opt["adam"].launches[0].args[0]
    assert d["t_pre"] == 1 and d["inc_step"] == 0 and "cursor" not in d
    c = InceptionProgram(Multi_Classifier(init_weights=False), 4, "cpu")
    assert not c.use_early_step_counter() and not any(l.name == "step_inc" for l in c.fwd_train.launches)


def test_stream_param_order_gives_model_c_side_stream_buckets():
    """Model C's module order starts with the stem (stream 0), so stream_buckets finds no side-stream prefix;
    rebuilt with stream_param_order (the parameters each side stream alone writes, grouped, in finalize order)
    the multi-rank DP step gets one bucket per side stream, each complete at that stream's own finalize --
    nothing writes it later or elsewhere, batched BN-tail launches (device job tables) included."""
    from mtl_das_pytorch_amd.engine.inception import InceptionProgram
    from mtl_das_pytorch_amd.models import build_model

    def make(order):
        torch.manual_seed(0)
        p = InceptionProgram(model, 8, "cpu", param_order=order)
        p.set_optimizer(weight_decay=1e-5, data_parallel=True)
        p.segment_backward(1)
        p.merge_wgrad_cfgs()
        p.refresh_wgrad_finalize()
        p.batch_wgrads()
        p.batch_tails()
        return p

    model = build_model("multi_classifier")
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    p0 = make(None)
    assert len(p0.stream_buckets(4)) == 1  # module order: no side-stream prefix
    order = p0.stream_param_order()
    assert sorted(map(id, order)) == sorted(map(id, p0.flat.order))
    del p0
    p = make(order)
    for k, v in model.state_dict().items():  # the rebuild keeps every value
        assert torch.equal(v, sd[k]), k
    b = p.stream_buckets(4)
    f, ls = p.flat, p.bwd.launches
    assert len(b) == 4 and b[0][0] == 0 and b[-1][1] == f.numel and all(b[i][1] == b[i + 1][0] for i in range(3))
    assert sum(hi - lo for lo, hi in b[:3]) > f.numel // 2  # the Inception blocks' branch parameters
    writers, side_fin = p._grad_writers()
    anchors = p.bucket_anchors
    assert [a.stream for a in anchors[:3]] == sorted(side_fin, key=side_fin.get) and anchors[3].stream == 0
    for (lo, hi), a in zip(b[:3], anchors[:3]):
        i0 = ls.index(a)
        for q in f.order:
            if lo <= f.off(q) < hi:
                assert all(s == a.stream and i <= i0 for s, i in writers.get(f.off(q), ())), q.shape
