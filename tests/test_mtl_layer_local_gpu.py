"""Model A (MTL_Net) backward, layer by layer, against the closed-form / autograd math of each single op.

Every op of the lowered backward (engine/mtl.py ``_emit_backward``: residual tails ADD_RELU with identity
or projection shortcut, the inner BN+ReLU tails, every conv's data and weight gradient, the level
branches' max-pool / sigmoid-mask tails, the two-segment attention-generator input and the MTL head) is
fed with the ENGINE's own inputs -- its stored bf16 activations, its published BN constants and the sum of
its gradient sources -- and compared per tensor with fp32 PyTorch math at tolerances set by bf16 output
rounding, independent of the network's error amplification at init.  The program runs at the bench's
batch (32) with the tuned kernel configs the bench uses (LDS-staged convs, split-K, fused statistics,
normalise-on-load).  Reference: model/modelA_MTL.py:7-174.

Parametrized over the model -- A, and B (``Single_Task_Net``, one task branch; reference
model/modelB_singleTask.py) for each task -- and over A's input channels: 1 (the reference; the stem runs as a
1 x 7 conv over 7 packed taps) and 2 (BASELINE's 2-channel north star, ``--in_channels 2``: gather of two channels into the 8-channel
stored input, the unpacked 7x7 stem at K = 392 padded to 416 and its weight gradient / finalize); plus A's
data-parallel backward program (2 gradient buckets: the backward cut into pieces, weight gradients and
finalize per piece), run here without collectives.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

# Every activation gradient the engine stores is bf16 (one rounding of an fp32 accumulation, as under
# autocast), so dy / dx / side / dhead are compared at the bf16 output rounding: a relative L2 error of one
# rounding of N(0,1)-like data is 2^-9 / sqrt(3) ~ 1.1e-3; 6e-3 leaves the margin of the fp32 references'
# accumulation order.  dW / dgamma / dbeta are fp32 sums over the engine's own bf16 operands (tight).
# measured worst (MI355X, B = 32, fp32 gradient storage of round 3): dy 1.7e-3, dW 3.9e-5, dgamma 5.5e-7
TOL = {"dy": 6e-3, "dx": 6e-3, "dW": 2e-4, "dgamma": 1e-5, "dbeta": 1e-5, "side": 6e-3, "dhead": 6e-3}


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-20)).item()


def q(t):
    return t.bfloat16().float()


def nchw(a, z=0, c0=0, C=None):
    """Group z, channels [c0, c0 + C) of an engine NHWC activation as dense fp32 NCHW."""
    C = a.C - c0 if C is None else C
    t = a.t.reshape(-1)[a.off + z * a.gs + c0:]
    M = a.B * a.H * a.W
    idx = torch.arange(M, device=t.device)[:, None] * a.ld + torch.arange(C, device=t.device)[None]
    return t[idx].float().view(a.B, a.H, a.W, C).permute(0, 3, 1, 2)


def k4(bn, z=0):
    """(scale, shift, mean, invstd) the forward published for BN layer ``bn`` (group z), NCHW-broadcastable."""
    return [v.view(1, -1, 1, 1) for v in bn.consts[z]]


def bn_backward(dz, y, bn, z=0):
    """Closed-form training-BN backward on the stored bf16 y with the forward's constants."""
    _, _, mu, inv = k4(bn, z)
    gam = bn.mods[z].weight.detach().view(1, -1, 1, 1)
    xh = (y - mu) * inv
    dy = gam * inv * (dz - dz.mean((0, 2, 3), keepdim=True) - xh * (dz * xh).mean((0, 2, 3), keepdim=True))
    return dy, (dz * xh).sum((0, 2, 3)), dz.sum((0, 2, 3))


@pytest.fixture(scope="module", params=[("MTL", 1, 1), ("MTL", 2, 1), ("single_event", 1, 1),
                                        ("single_distance", 1, 1), ("MTL", 1, 2)],
                ids=["cin1", "cin2", "B_event", "B_distance", "dp_buckets2"])
def engine_step(request):
    from mtl_das_pytorch_amd.data.synthetic import generate
    from mtl_das_pytorch_amd.engine.mtl import MTLProgram
    from mtl_das_pytorch_amd.engine.tune import autotune_program
    from mtl_das_pytorch_amd.models import build_model
    # the single-op fp32 references run on PyTorch's native im2col + GEMM convolution, not MIOpen: one run
    # of this module hit an illegal address inside the reference conv backward (MIOpen solver choice)
    flags = (torch.backends.cudnn.enabled, torch.backends.cudnn.allow_tf32, torch.backends.cuda.matmul.allow_tf32)
    torch.backends.cudnn.enabled = False
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.manual_seed(0)
    B = 32
    name, cin, nbuckets = request.param
    model = build_model(name, in_channels=cin)  # Model A, or Model B (Single_Task_Net: one task branch)
    prog = MTLProgram(model, B, "cuda")
    assert (prog.stem_pack[0] > 0) == (cin == 1)
    if nbuckets > 1:  # the data-parallel backward: cut into gradient-bucket pieces, wgrads batched per piece
        assert len(prog.segment_backward(nbuckets)) == nbuckets
    autotune_program(prog, measure=False)  # the bench's tuned kernel configs
    X, d, e = generate(B, seed=11, device="cuda", in_channels=cin)
    labels = torch.stack([d, e], 1)
    idx = torch.arange(B, device="cuda")
    prog.opt["pack"].run()
    prog.arena.clear()
    prog.gather_phase(X, labels, idx).run()
    prog.fwd_train.run()
    prog.bwd.run()
    torch.cuda.synchronize()
    prog.flat.sync_module_grads()
    yield model, prog, X, labels
    torch.backends.cudnn.enabled, torch.backends.cudnn.allow_tf32, torch.backends.cuda.matmul.allow_tf32 = flags


class Checker:
    def __init__(self):
        self.worst, self.bad = {}, []

    def __call__(self, kind, what, e, r):
        err = rel(e, r)
        self.worst[kind] = max(self.worst.get(kind, 0.0), err)
        if not err < TOL[kind]:
            self.bad.append((what, kind, f"{err:.2e}"))

    def exact_zero(self, what, e, ref_noise):
        self.worst["db_ref_noise"] = max(self.worst.get("db_ref_noise", 0.0), ref_noise)
        if e.abs().max().item() != 0.0 or not ref_noise < 1e-3:  # noise of sum(dy) over bf16-rounded dy
            self.bad.append((what, "db", f"engine max {e.abs().max().item():.1e}, reference noise {ref_noise:.1e}"))

    def done(self):
        print("worst layer-local errors", {k: f"{v:.1e}" for k, v in self.worst.items()})
        assert not self.bad, self.bad


def conv_check(chk, name, conv, z, x, dy, dx_act=None, x_requires=True, dx_extra=None):
    """Autograd of the single conv (bf16-rounded weights, the engine's input and dy).  ``dx_extra``: the
    gradient sources the engine's dgrad epilogue added to its output (fold_tail_sources)."""
    m = conv.mods[z]
    x = x.clone().requires_grad_(x_requires and dx_act is not None)
    w = q(m.weight.detach()).requires_grad_(True)
    y = F.conv2d(x, w, None, m.stride, m.padding)
    y.backward(dy)
    chk("dW", f"{name}.weight", m.weight.grad, w.grad)
    if m.bias is not None:
        # every biased conv of Model A feeds a training-mode BN, so d(bias) = sum(dy) = 0 exactly (the BN
        # backward removes the mean); the engine writes exact zeros, autograd leaves rounding noise
        db = dy.sum((0, 2, 3))
        chk.exact_zero(f"{name}.bias", m.bias.grad, db.norm().item() / dy.abs().sum((0, 2, 3)).norm().item())
    if dx_act is not None:
        chk("dx", f"{name} dx", dx_act, x.grad if dx_extra is None else x.grad + dx_extra)


def fused_conv_check(chk, names, conv, x, dys, dx_act, dx_extra=None):
    """A horizontally fused conv (engine ConvLayer concat: RB3/5/7's conv a with its centre-tap 1x1 projection
    shortcut): each member's weight gradient from its own dy slice, and the ONE data gradient against the sum
    of the members' autograd input gradients."""
    x = x.clone().requires_grad_(True)
    for (m, _, _), name, dy in zip(conv.members, names, dys):
        w = q(m.weight.detach()).requires_grad_(True)
        F.conv2d(x, w, None, m.stride, m.padding).backward(dy)
        chk("dW", f"{name}.weight", m.weight.grad, w.grad)
    chk("dx", f"{names[0]}+shortcut dx", dx_act, x.grad if dx_extra is None else x.grad + dx_extra)


def bn_grads_check(chk, name, bn, z, dgam, dbet):
    chk("dgamma", f"{name}.weight", bn.mods[z].weight.grad, dgam)
    chk("dbeta", f"{name}.bias", bn.mods[z].bias.grad, dbet)


def test_mtl_backward_layer_local(engine_step):
    model, prog, X, labels = engine_step
    chk = Checker()
    T, lv, rbs = prog.T, prog.levels, prog.rbs

    def folded(R):  # which data gradient of block R summed all gradient sources of its input (or None)
        # (a fused conv a + shortcut writes "dxa": the one data gradient of the block's input)
        for key in ("dxs", "dxa"):
            if key in R and any(l.name == "conv_dgrad" and l.args[3].get("add") and l.args[3]["out"] == R[key].p
                                for l in prog.bwd.launches):
                return key
        return None

    def level_sources(k):
        g = 0
        if k >= 1:
            L = lv[(k - 1) // 2]
            for t in range(T):
                g = g + (nchw(L["dcat"], t, 0, L["C"]) if k % 2 == 1 else nchw(L["dF"], t))
        return g

    def sources(k):  # gradient sources of F_k (mirrors MTLProgram._emit_backward)
        g = level_sources(k)
        if k < 8:
            R = rbs[k]
            if folded(R):
                return nchw(R[folded(R)])
            g = g + nchw(R["dxa"])
            if not R.get("fused"):
                g = g + (nchw(R["dxs"]) if R["proj"] else nchw(R["side"]))
        return g

    def folded_extra(i, key):  # what the folded dgrad of block i (consuming F_i) added to its own output
        R = rbs[i]
        if folded(R) != key:
            return None
        if R.get("fused"):
            return level_sources(i)
        return level_sources(i) + (nchw(R["dxa"]) if key == "dxs" else nchw(R["side"]))

    # ---- task levels (per task t, group z = t)
    for li in range(3, -1, -1):
        L = lv[li]
        for t in range(T):
            nm = f"level{li + 1}.task{t}"
            if "co" in L:
                nxt = lv[li + 1]
                g = nchw(nxt["dcat"], t, nxt["Fa"].C, L["co"].Co)   # B_l part of d cat[F, B_l]
                yo = nchw(L["yo"], t)
                sc, sh, _, _ = k4(L["bno"], t)
                zin = (yo * sc + sh).requires_grad_(True)
                F.max_pool2d(torch.relu(zin), 2, 2, ceil_mode=True).backward(g)
                dyo, dgam, dbet = bn_backward(zin.grad, yo, L["bno"], t)
                chk("dy", f"{nm} pool tail dy", nchw(L["dyo"], t), dyo)
                bn_grads_check(chk, f"{nm}.out_bn", L["bno"], t, dgam, dbet)
                conv_check(chk, f"{nm}.out_conv", L["co"], t, nchw(L["Aout"], t), nchw(L["dyo"], t), nchw(L["dA"], t))
            g = nchw(L["dA"], t)
            ym2, Fb = nchw(L["ym2"], t), nchw(L["Fb"])
            sc, sh, _, _ = k4(L["bn3"], t)
            s = torch.sigmoid(ym2 * sc + sh)
            chk("side", f"{nm} dF", nchw(L["dF"], t), g * s)
            dym2, dgam, dbet = bn_backward(g * Fb * s * (1 - s), ym2, L["bn3"], t)
            chk("dy", f"{nm} mask tail dy", nchw(L["dym2"], t), dym2)
            bn_grads_check(chk, f"{nm}.gen_bn3", L["bn3"], t, dgam, dbet)
            ym1 = nchw(L["ym1"], t)
            sc0, sh0, _, _ = k4(L["bn0"], t)
            hm = q(torch.relu(ym1 * sc0 + sh0))  # normalise-on-load operand of c3
            conv_check(chk, f"{nm}.gen_conv3", L["c3"], t, hm, nchw(L["dym2"], t), nchw(L["dhm"], t))
            dym1, dgam, dbet = bn_backward(nchw(L["dhm"], t) * ((ym1 * sc0 + sh0) > 0), ym1, L["bn0"], t)
            chk("dy", f"{nm} gen tail dy", nchw(L["dym1"], t), dym1)
            bn_grads_check(chk, f"{nm}.gen_bn0", L["bn0"], t, dgam, dbet)
            x = nchw(L["Fa"]) if L["prevB"] is None else torch.cat([nchw(L["Fa"]), nchw(L["prevB"], t)], 1)
            conv_check(chk, f"{nm}.gen_conv0", L["c0"], t, x, nchw(L["dym1"], t), nchw(L["dcat"], t))

    # ---- residual blocks RB8 -> RB1
    for i in range(7, -1, -1):
        R = rbs[i]
        nm = f"resblock{i + 1}"
        g = sources(i + 1)
        yb = nchw(R["yb"])
        sc, sh, _, _ = k4(R["bnb"])
        if R["proj"]:
            ys = nchw(R["ys"])
            sc2, sh2, _, _ = k4(R["bns"])
            rr = ys * sc2 + sh2
        else:
            rr = nchw(R["in"])
        dz = g * ((yb * sc + sh + rr) > 0)
        dyb, dgam, dbet = bn_backward(dz, yb, R["bnb"])
        chk("dy", f"{nm} tail dy", nchw(R["dyb"]), dyb)
        bn_grads_check(chk, f"{nm}.left.4", R["bnb"], 0, dgam, dbet)
        if R["proj"]:
            dys, dgam2, dbet2 = bn_backward(dz, ys, R["bns"])
            chk("dy", f"{nm} shortcut dy", nchw(R["dys"]), dys)
            bn_grads_check(chk, f"{nm}.shortcut.1", R["bns"], 0, dgam2, dbet2)
        else:
            chk("side", f"{nm} shortcut grad", nchw(R["side"]), dz)
        ya = nchw(R["ya"])
        sca, sha, _, _ = k4(R["bna"])
        ha = q(torch.relu(ya * sca + sha))  # normalise-on-load operand of conv b
        conv_check(chk, f"{nm}.left.3", R["cb"], 0, ha, nchw(R["dyb"]), nchw(R["dha"]))
        dya, dgam, dbet = bn_backward(nchw(R["dha"]) * ((ya * sca + sha) > 0), ya, R["bna"])
        chk("dy", f"{nm} inner tail dy", nchw(R["dya"]), dya)
        bn_grads_check(chk, f"{nm}.left.1", R["bna"], 0, dgam, dbet)
        if R.get("fused"):
            fused_conv_check(chk, [f"{nm}.left.0", f"{nm}.shortcut.0"], R["cas"], nchw(R["in"]),
                             [nchw(R["dya"]), nchw(R["dys"])], nchw(R["dxa"]), dx_extra=folded_extra(i, "dxa"))
            continue
        conv_check(chk, f"{nm}.left.0", R["ca"], 0, nchw(R["in"]), nchw(R["dya"]), nchw(R["dxa"]),
                   dx_extra=folded_extra(i, "dxa"))
        if R["proj"]:
            conv_check(chk, f"{nm}.shortcut.0", R["cs"], 0, nchw(R["in"]), nchw(R["dys"]), nchw(R["dxs"]),
                       dx_extra=folded_extra(i, "dxs"))

    # ---- stem: conv1 tail (sources of f0) and the conv1 weight gradient on the real (unpacked) input
    y0 = nchw(prog.y0)
    sc, sh, _, _ = k4(prog.bn1)
    dy0, dgam, dbet = bn_backward(sources(0) * ((y0 * sc + sh) > 0), y0, prog.bn1)
    chk("dy", "conv1 tail dy", nchw(prog.dy0), dy0)
    bn_grads_check(chk, "conv1.1", prog.bn1, 0, dgam, dbet)
    if not prog.stem_pack[0]:  # the gathered NHWC input: the dataset rows, bf16, channels padded to 8 with 0
        xin = prog.x.float()
        assert torch.equal(xin[..., :X.shape[1]], q(X).permute(0, 2, 3, 1)) and not xin[..., X.shape[1]:].any()
    conv_check(chk, "conv1.0", prog.conv1, 0, q(X), nchw(prog.dy0))

    # ---- head: d loss / d A4 = w_t (softmax - onehot) / (B * group size * HW), broadcast per channel group
    A4 = lv[3]["Aout"]
    for t in range(T):
        K = model.task_cate_num[t]
        p = prog.logp[t, :, :K].exp()
        p[torch.arange(prog.B), labels[:, prog.lab_off[t]]] -= 1
        gsz = A4.C // K
        scale = prog.loss_weights[t] / (prog.B * gsz * A4.H * A4.W)
        ref = (p * scale).repeat_interleave(gsz, 1)[:, :, None, None].expand(-1, -1, A4.H, A4.W)
        chk("dhead", f"head task{t} dA4", nchw(prog.dA4, t), ref)
    chk.done()
