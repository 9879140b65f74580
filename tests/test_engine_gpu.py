"""End-to-end parity of the lowered MI355X engine against the reference-math PyTorch module (fp32 autograd).

One training step of Model A (and B) on the same weights and batch: log-probabilities, every parameter
gradient, BN running statistics, Adam update, and HIP-graph replay == eager execution."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def _setup(model_cls, B=8, seed=0, **kw):
    from mtl_das_pytorch_amd.data.synthetic import generate
    from mtl_das_pytorch_amd.engine.mtl import MTLProgram
    torch.manual_seed(seed)
    model = model_cls(**kw)
    ref = copy.deepcopy(model).cuda()
    prog = MTLProgram(model, B, "cuda")
    # torch-op generator: the whole-network bounds below were calibrated on this input (at init the
    # network amplifies rounding differences input-dependently; the HIP generator's noise is another draw)
    X, d, e = generate(2 * B, seed=seed + 1, device="cuda", backend="torch")
    labels = torch.stack([d, e], 1)
    return model, ref, prog, X, labels


def _engine_step(prog, X, labels, idx, with_opt=False):
    prog.opt["pack"].run()
    prog.arena.clear()
    prog.gather_phase(X, labels, idx).run()
    prog.fwd_train.run()
    prog.bwd.run()
    if with_opt:
        prog.opt["adam"].run()
    torch.cuda.synchronize()


def _ref_step(ref, X, labels, idx):
    ref.train()
    x = X[idx].bfloat16().float()
    out = ref(x)
    out = out if isinstance(out, tuple) else (out,)
    return out


def _ref_grads(m, x, labels, idx, cols):
    m.zero_grad()
    outs = m(x)
    outs = outs if isinstance(outs, tuple) else (outs,)
    sum(F.nll_loss(o, labels[idx, c]) for o, c in zip(outs, cols)).backward()
    return outs, {n: p.grad.detach().clone() for n, p in m.named_parameters()}


@pytest.mark.parametrize("which", ["MTL", "single_distance", "single_event"])
def test_engine_train_step_matches_autograd(which):
    """The engine's gradients are compared with fp32 autograd on the SAME bf16-rounded weights.  The
    reference network at random init is ill-conditioned (0.1% weight noise moves early-layer gradients
    by ~15-20%, measured with a launch-by-launch comparison), so the bound for each tensor is derived from the reference's
    own sensitivity to a bf16-sized (4e-3) weight perturbation; well-conditioned tensors (head, level 4) are held
    to a tight absolute bound."""
    from mtl_das_pytorch_amd.engine.mtl import MTLProgram
    from mtl_das_pytorch_amd.models import MTL_Net, Single_Task_Net
    if which == "MTL":
        model, ref, prog, X, labels = _setup(MTL_Net)
        cols = [0, 1]
    else:
        task = which.split("_")[1]
        model, ref, prog, X, labels = _setup(Single_Task_Net, task=task)
        cols = [0 if task == "distance" else 1]
    B = prog.B
    idx = torch.arange(B, device="cuda")
    with torch.no_grad():
        for p in ref.parameters():
            p.copy_(p.bfloat16().float())  # the engine computes with the bf16 image of the masters
    _engine_step(prog, X, labels, idx)
    ref.train()
    x = X[idx].bfloat16().float()
    noisy = copy.deepcopy(ref)
    outs, g_ref = _ref_grads(ref, x, labels, idx, cols)
    torch.manual_seed(123)
    with torch.no_grad():
        for p in noisy.parameters():
            p.mul_(1 + 4e-3 * torch.randn_like(p))  # ~ one bf16 ulp of relative noise
    _, g_noise = _ref_grads(noisy, x, labels, idx, cols)
    for t, o in enumerate(outs):
        k = o.shape[1]
        err = (prog.logp[t, :, :k] - o.detach()).abs().max().item()
        assert err < 5e-2, f"task {t} logp max err {err}"
        assert prog.metrics[t, 2].item() == B
        assert abs(prog.metrics[t, 0].item() / B - F.nll_loss(o, labels[idx, cols[t]]).item()) < 5e-2
    prog.flat.sync_module_grads()
    flat_e, flat_r = [], []
    bad = []
    for name, p in model.named_parameters():
        gr = g_ref[name]
        if name.split(".")[-2] in ("0", "3") and name.endswith("bias") and "generat" in name:
            # conv bias feeding a training-mode BN: analytically zero gradient (engine writes exactly 0)
            assert gr.abs().max().item() < 1e-3
            continue
        e = rel(p.grad, gr)
        bound = 1.5 * rel(g_noise[name], gr) + 0.05
        flat_e.append(p.grad.flatten()); flat_r.append(gr.flatten())
        if e > bound:
            bad.append((name, round(e, 4), round(bound, 4)))
    ge, gr = torch.cat(flat_e), torch.cat(flat_r)
    cos = F.cosine_similarity(ge, gr, dim=0).item()
    print(f"global gradient cosine {cos:.4f}; over-bound tensors {bad}")
    assert not bad, bad
    assert cos > 0.9, cos
    # running statistics
    ref_bufs = dict(ref.named_buffers())
    for name, b in model.named_buffers():
        if name.endswith("num_batches_tracked"):
            assert int(b.item()) == int(ref_bufs[name].item()) == 1, name
        else:
            assert rel(b, ref_bufs[name]) < 3e-2, name


def test_adam_matches_torch():
    """Flat Adam + bf16 re-pack against torch.optim.Adam; the update must also leave bf16 weight images
    equal to a fresh pack of the updated masters."""
    from mtl_das_pytorch_amd.models import MTL_Net
    model, ref, prog, X, labels = _setup(MTL_Net)
    g = torch.Generator(device="cpu").manual_seed(5)
    for p in ref.parameters():
        p.grad = torch.randn(p.shape, generator=g).cuda() * 1e-2
    for (name, p), (_, rp) in zip(model.named_parameters(), ref.named_parameters()):
        prog.flat.grad_of(p).copy_(rp.grad)
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3, weight_decay=1e-5, foreach=False)
    prog.set_optimizer(weight_decay=1e-5)
    prog.flat.lr.fill_(1e-3)
    for _ in range(3):
        opt.step()
        prog.opt["adam"].run()
    torch.cuda.synchronize()
    assert prog.flat.step.item() == 3
    for (name, p), (_, rp) in zip(model.named_parameters(), ref.named_parameters()):
        assert torch.allclose(p, rp, atol=2e-6, rtol=1e-5), name
    images = [(c.wf.clone(), c.wd.clone()) for c in prog.convs]
    prog.opt["pack"].run()
    torch.cuda.synchronize()
    for c, (wf, wd) in zip(prog.convs, images):
        assert torch.equal(c.wf, wf) and torch.equal(c.wd, wd)


def test_graph_replay_matches_eager():
    """HIP-graph replay must reproduce eager execution BITWISE, and so must two eager runs: the only
    cross-block reductions are the BN replica sums, accumulated in fp64 so their atomic order cannot
    change a rounded result (with fp32 sums the chaotic-at-init network turned order noise into run-to-run
    gradient differences of up to 12%)."""
    from mtl_das_pytorch_amd.engine.step import StepRunner
    from mtl_das_pytorch_amd.models import MTL_Net
    model, ref, prog, X, labels = _setup(MTL_Net)
    prog.set_optimizer(weight_decay=1e-5)
    init = prog.flat.params.clone()

    def reset():
        prog.flat.params.copy_(init)
        prog.flat.exp_avg.zero_(); prog.flat.exp_avg_sq.zero_(); prog.flat.step.zero_()
        prog.flat.bn_mean.zero_(); prog.flat.bn_var.fill_(1.0); prog.flat.bn_nbt.zero_()

    grads, params = [], []
    for use_graph in (False, False, True):
        reset()
        # a no-op "all-reduce" splits the step into compute graph + optimizer graph
        r = StepRunner(prog, X, labels, use_graph=use_graph, allreduce=lambda g: None)
        r.set_lr(1e-3)
        r.pack_weights()
        r.train_step(torch.arange(prog.B, device="cuda"))
        torch.cuda.synchronize()
        grads.append(prog.flat.grads.clone())
        for i in range(2):
            r.train_step(torch.arange(prog.B, device="cuda") + ((i + 1) % 2) * prog.B)
        torch.cuda.synchronize()
        params.append((prog.flat.params.clone(), prog.flat.step.item()))
    base = rel(grads[1], grads[0])
    d = rel(grads[2], grads[0])
    print(f"one-step gradients: eager-vs-eager {base:.3e}  graph-vs-eager {d:.3e}")
    assert torch.equal(grads[1], grads[0]) and torch.equal(grads[2], grads[0])
    assert params[2][1] == 3.0
    assert torch.equal(params[2][0], params[0][0]) and torch.equal(params[1][0], params[0][0])


def _force_big_wgrad(prog):
    """Every conv whose reduction allows it on a large-tile weight-gradient config (32-35, rotating)."""
    i = 0
    for l in prog.bwd.launches:
        if l.name == "conv_wgrad":
            c = 32 + i % 4
            i += 1
            if l.owner.wgrad_valid(c):
                l.owner.set_wgrad_cfg(c)
                l.args = (c,) + tuple(l.args[1:])
    prog.refresh_wgrad_finalize()  # the split counts changed with the configs (as autotune_program does)
    return i


@pytest.mark.parametrize("model_name", ["MTL", "multi_classifier"])
@pytest.mark.parametrize("big", [False, True])
def test_batched_wgrad_bitwise_equal(model_name, big):
    """One launch per tile config computes exactly what the per-conv launches compute (also with every
    conv on the large-tile configs, whose gradients must match the default configs' to fp32 order), and so
    does a side stream's batch on a capped persistent grid (LoweredProgram.SIDE_WGRAD_GRID: 7 hardware
    blocks walking all virtual blocks)."""
    from mtl_das_pytorch_amd.models import build_model, encode_joint
    from mtl_das_pytorch_amd.data.synthetic import generate
    grads = []
    for batched in (False, True, "capped"):
        torch.manual_seed(0)
        m = build_model(model_name)
        if model_name == "multi_classifier":
            from mtl_das_pytorch_amd.engine.inception import InceptionProgram
            prog = InceptionProgram(m, 8, "cuda", p_drop=0.0)
        else:
            from mtl_das_pytorch_amd.engine.mtl import MTLProgram
            prog = MTLProgram(m, 8, "cuda")
        if big:
            assert _force_big_wgrad(prog) > 0
        prog.SIDE_WGRAD_GRID = 7 if batched == "capped" else 0  # (Model A ships 512)
        if batched:
            prog.batch_wgrads()
        X, d, e = generate(16, seed=1, device="cuda")
        lab = encode_joint(d, e) if model_name == "multi_classifier" else torch.stack([d, e], 1)
        _engine_step(prog, X, lab, torch.arange(8, device="cuda"))
        grads.append(prog.flat.grads.clone())
        if batched == "capped":
            assert any(l.name == "wgrad_batched" and l.args[4] == 7 for l in prog.bwd.launches)
    for g in grads[1:]:
        assert torch.equal(grads[0], g)


@pytest.mark.parametrize("model_name", ["MTL", "multi_classifier"])
def test_pack_images_match_layouts(model_name):
    """The optimizer's pack (forward image per 8 elements, data-gradient image through LDS-transposed
    tiles) writes exactly the bf16 layouts of ops.functional.pack_weight_fwd / pack_weight_dgrad, with
    zero padding, for every conv of the program (after perturbing the masters so no stale image passes)."""
    from mtl_das_pytorch_amd.engine.inception import InceptionProgram
    from mtl_das_pytorch_amd.engine.mtl import MTLProgram
    from mtl_das_pytorch_amd.models import MTL_Net, Multi_Classifier
    from mtl_das_pytorch_amd.ops.functional import pack_weight_dgrad, pack_weight_fwd
    torch.manual_seed(3)
    prog = MTLProgram(MTL_Net(), 4, "cuda") if model_name == "MTL" else InceptionProgram(Multi_Classifier(), 4, "cuda")
    with torch.no_grad():
        prog.flat.params.add_(torch.randn_like(prog.flat.params) * 1e-2)
    prog.opt["pack"].run()
    torch.cuda.synchronize()
    n = 0
    for c in prog.convs:
        # a horizontally fused group (Model C's sibling 1x1 heads, Model A's conv a + centre-tap 1x1 shortcut) is
        # ONE conv over the concatenated weights, a 1x1 member zero-padded to the group's kernel at its centre
        def embed(w):
            out = torch.zeros(w.shape[0], w.shape[1], c.KH, c.KW, device=w.device)
            dh, dw = (c.KH - w.shape[2]) // 2, (c.KW - w.shape[3]) // 2
            out[:, :, dh:dh + w.shape[2], dw:dw + w.shape[3]] = w
            return out
        groups = [torch.cat([embed(m.weight) for m in c.mods])] if c.concat else [m.weight for m in c.mods]
        for g, w in enumerate(groups):
            w = w.detach().float()
            if c.KH * c.KW == w.shape[2] * w.shape[3]:  # the packed-tap stem has its own (virtual) layout
                ef = pack_weight_fwd(w, c.Cs)
                got = c.wf[g]
                assert torch.equal(got[:ef.shape[0], :ef.shape[1]], ef)
                assert not got[ef.shape[0]:].any() and not got[:, ef.shape[1]:].any()
            ed = pack_weight_dgrad(w, c.Cs)
            gd = c.wd[g]
            if c.KH * c.KW != w.shape[2] * w.shape[3]:
                continue
            assert torch.equal(gd[:ed.shape[0], :ed.shape[1]], ed), (c.Co, c.Ci, c.KH, c.KW)
            assert not gd[ed.shape[0]:].any() and not gd[:, ed.shape[1]:].any()
            n += 1
    assert n > 10




def test_training_trajectory_matches_fp32_oracle():
    """Three full training steps of Model A (forward, backward, Adam with the reference's lr 1e-3 / coupled
    weight decay 1e-5 as torch.optim.Adam applies them) on the engine and on the fp32 reference module from
    the same bf16-rounded weights and batches.  Tolerances are the oracle's own sensitivity: a copy of the
    fp32 reference whose weights carry one bf16 ulp of relative noise (4e-3) is stepped alongside, and the
    engine must stay within 1.5x that copy's distance from the oracle (plus a small floor) -- per step for
    both task losses, and for the accumulated parameter update after the last step."""
    from mtl_das_pytorch_amd.engine.step import StepRunner
    from mtl_das_pytorch_amd.models import MTL_Net
    model, ref, prog, X, labels = _setup(MTL_Net, B=16)
    B, steps, lr, wd = prog.B, 3, 1e-3, 1e-5
    with torch.no_grad():
        for p in ref.parameters():
            p.copy_(p.bfloat16().float())
        prog.flat.params.copy_(prog.flat.params.bfloat16().float())  # the same rounded masters
    noisy = copy.deepcopy(ref)
    torch.manual_seed(321)
    with torch.no_grad():
        for p in noisy.parameters():
            p.mul_(1 + 4e-3 * torch.randn_like(p))
    p0 = {n: p.detach().clone() for n, p in ref.named_parameters()}
    pn0 = {n: p.detach().clone() for n, p in noisy.named_parameters()}
    prog.set_optimizer(betas=(0.9, 0.999), eps=1e-8, weight_decay=wd)
    runner = StepRunner(prog, X, labels, use_graph=False)
    runner.set_lr(lr)
    opts = [torch.optim.Adam(m.parameters(), lr=lr, weight_decay=wd, foreach=False) for m in (ref, noisy)]
    for s in range(steps):
        idx = torch.arange(s * B, (s + 1) * B, device="cuda") % X.shape[0]
        runner.reset_metrics()
        runner.train_step(idx)
        torch.cuda.synchronize()
        eng = [prog.metrics[t, 0].item() / B for t in range(2)]
        losses = []
        for m, opt in zip((ref, noisy), opts):
            m.train()
            opt.zero_grad()
            outs = m(X[idx].bfloat16().float())
            ls = [F.nll_loss(o, labels[idx, t]) for t, o in enumerate(outs)]
            sum(ls).backward()
            opt.step()
            losses.append([l.item() for l in ls])
        for t in range(2):
            tol = 1.5 * abs(losses[1][t] - losses[0][t]) + 0.02 * abs(losses[0][t]) + 1e-3
            assert abs(eng[t] - losses[0][t]) <= tol, (s, t, eng[t], losses[0][t], losses[1][t])
    upd_e = torch.cat([(p.detach() - p0[n]).flatten() for n, p in model.named_parameters()])
    upd_r = torch.cat([(p.detach() - p0[n]).flatten() for n, p in ref.named_parameters()])
    upd_n = torch.cat([(p.detach() - pn0[n]).flatten() for n, p in noisy.named_parameters()])
    e, bound = rel(upd_e, upd_r), 1.5 * rel(upd_n, upd_r) + 0.05
    print(f"3-step update: engine vs oracle {e:.3f}, noisy oracle vs oracle {rel(upd_n, upd_r):.3f}")
    assert e <= bound, (e, bound)


@pytest.mark.parametrize("model_name", ["MTL", "multi_classifier"])
def test_early_adam_matches_optimizer_phase(model_name, monkeypatch):
    """Side streams finalize AND update their convs right after their weight-gradient batches
    (LoweredProgram.SIDE_FINALIZE / EARLY_ADAM); two training steps give bitwise the parameters, moments and
    bf16 weight images of the program whose optimizer phase updates everything."""
    from mtl_das_pytorch_amd.data.synthetic import generate
    from mtl_das_pytorch_amd.engine.lowering import LoweredProgram
    from mtl_das_pytorch_amd.engine.tune import autotune_program
    from mtl_das_pytorch_amd.models import build_model, encode_joint
    res = []
    for early in (False, True):
        monkeypatch.setattr(LoweredProgram, "EARLY_ADAM", early)
        torch.manual_seed(0)
        m = build_model(model_name)
        if model_name == "multi_classifier":
            from mtl_das_pytorch_amd.engine.inception import InceptionProgram
            prog = InceptionProgram(m, 8, "cuda", p_drop=0.0)
        else:
            from mtl_das_pytorch_amd.engine.mtl import MTLProgram
            prog = MTLProgram(m, 8, "cuda")
        prog.set_optimizer(weight_decay=1e-5)
        autotune_program(prog, measure=False)
        assert any(l.name == "adam_pack_early" for l in prog.bwd.launches) == early
        prog.flat.lr.fill_(1e-3)
        X, d, e = generate(16, seed=1, device="cuda")
        lab = encode_joint(d, e) if model_name == "multi_classifier" else torch.stack([d, e], 1)
        prog.opt["pack"].run()
        for s in range(2):
            prog.gather_phase(X, lab, torch.arange(8, device="cuda") + 8 * s, clear=True).run()
            prog.fwd_train.run()
            prog.bwd.run()
            prog.opt["adam"].run()
        torch.cuda.synchronize()
        f = prog.flat
        res.append([f.params.clone(), f.exp_avg.clone(), f.exp_avg_sq.clone(), f.step.clone()]
                   + [c.wf.clone() for c in prog.convs] + [c.wd.clone() for c in prog.convs])
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_early_step_counter_matches_tail_counter():
    """LoweredProgram.use_early_step_counter (the step runner's form for Model A): the Adam step counter advanced
    by a launch on the forward's first side stream, every update using t = step, trains bitwise like the
    phases run by hand with the counter advanced after the last Adam launch; the counter ends equal."""
    from mtl_das_pytorch_amd.data.synthetic import generate
    from mtl_das_pytorch_amd.engine.mtl import MTLProgram
    from mtl_das_pytorch_amd.engine.step import StepRunner
    from mtl_das_pytorch_amd.engine.tune import autotune_program
    from mtl_das_pytorch_amd.models import build_model
    X, d, e = generate(32, seed=6, device="cuda")
    lab = torch.stack([d, e], 1)
    out = []
    for early in (False, True):
        torch.manual_seed(0)
        prog = MTLProgram(build_model("MTL"), 8, "cuda")
        prog.set_optimizer(weight_decay=1e-5)
        autotune_program(prog, measure=False)
        prog.flat.lr.fill_(1e-3)
        idx = [torch.arange(8, device="cuda") + 8 * (s % 4) for s in range(3)]
        if early:
            r = StepRunner(prog, X, lab, use_graph=False)
            assert any(l.name == "step_inc" for l in prog.fwd_train.launches)
            for i in idx:
                r.train_step(i)
        else:
            assert not any(l.name == "step_inc" for l in prog.fwd_train.launches)
            prog.opt["pack"].run()
            for i in idx:
                prog.gather_phase(X, lab, i, clear=True).run()
                prog.fwd_train.run()
                prog.bwd.run()
                prog.opt["adam"].run()
        torch.cuda.synchronize()
        f = prog.flat
        out.append([f.params.clone(), f.exp_avg.clone(), f.exp_avg_sq.clone(), f.step.clone()])
    assert float(out[1][3][0]) == 3.0
    for a, b in zip(*out):
        assert torch.equal(a, b)


@pytest.mark.parametrize("model_name", ["MTL", "multi_classifier"])
def test_index_schedule_matches_per_step_indices(model_name):
    """StepRunner.set_index_schedule: steps that gather the next row of a device-resident [nrows][B] index table
    (cursor advanced by the optimizer's step-counter kernel) train exactly like steps handed the same indices
    one by one -- bitwise equal weights and moments after more steps than the table has rows, equal metric
    counts (the loss sums are fp32 atomics over blocks: order-dependent in the last bits, also between two
    runs of the same path)."""
    from mtl_das_pytorch_amd.data.synthetic import generate
    from mtl_das_pytorch_amd.engine.step import StepRunner
    from mtl_das_pytorch_amd.engine.tune import autotune_program
    from mtl_das_pytorch_amd.models import build_model, encode_joint
    X, d, e = generate(64, seed=4, device="cuda")
    joint = model_name == "multi_classifier"
    lab = encode_joint(d, e) if joint else torch.stack([d, e], 1)
    sched = torch.randperm(64, device="cuda")[:24].view(3, 8)
    out = []
    for use_sched in (False, True):
        torch.manual_seed(0)
        m = build_model(model_name)
        if joint:
            from mtl_das_pytorch_amd.engine.inception import InceptionProgram
            prog = InceptionProgram(m, 8, "cuda", p_drop=0.0)
        else:
            from mtl_das_pytorch_amd.engine.mtl import MTLProgram
            prog = MTLProgram(m, 8, "cuda")
        prog.set_optimizer(weight_decay=1e-5)
        autotune_program(prog, measure=False)
        r = StepRunner(prog, X, lab)
        r.set_lr(1e-3)
        if use_sched:
            r.set_index_schedule(sched)
        for i in range(5):
            r.train_step() if use_sched else r.train_step(sched[i % 3])
        torch.cuda.synchronize()
        f = prog.flat
        out.append([f.params.clone(), f.exp_avg.clone(), f.exp_avg_sq.clone(), prog.metrics.clone()])
        if use_sched:
            assert int(r.cursor.item()) == 5
        r.close()
    for a, b in zip(out[0][:3], out[1][:3]):
        assert torch.equal(a, b)
    ma, mb = out[0][3], out[1][3]
    assert torch.equal(ma[:, 1:3], mb[:, 1:3])  # correct / count
    assert torch.allclose(ma, mb, rtol=1e-5, atol=1e-4)
