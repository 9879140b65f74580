"""Numerics of every HIP kernel against a plain fp32 PyTorch reference of the same op (MI355X only).

Inputs are rounded to bf16 first and the reference is computed in fp32 from those rounded values, so
the tolerances only absorb fp32-vs-MFMA accumulation order and the bf16 rounding of outputs."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

NREP = 32  # must match csrc/common.h


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def nchw(x):
    return x.permute(0, 3, 1, 2).contiguous()


@pytest.fixture(scope="module")
def fn():
    from mtl_das_pytorch_amd.ops import functional as Fn
    from mtl_das_pytorch_amd.ops.hip import lib
    lib()  # fail loudly if the extension is missing
    return Fn


CONV_CASES = [
    # B, H, W, Ci, Co, k, s, p
    (2, 33, 83, 16, 16, 3, 1, 1),
    (2, 33, 83, 16, 32, 1, 2, 0),
    (2, 33, 83, 16, 32, 3, 2, 1),
    (2, 17, 42, 32, 64, 3, 2, 1),
    (2, 9, 21, 64, 128, 3, 1, 1),
    (2, 5, 11, 256, 64, 1, 1, 0),
    (2, 33, 83, 8, 16, 3, 1, 1),
    (2, 10, 28, 48, 64, (5, 5), 1, (2, 2)),
    (2, 4, 13, 128, 128, (1, 7), 1, (0, 3)),
    (2, 4, 13, 128, 192, (7, 1), 1, (3, 0)),
    (2, 23, 60, 80, 192, 3, 1, 0),
    (1, 9, 27, 288, 384, 3, 2, 0),
]


def _mk(case, dev="cuda", seed=0):
    B, H, W, Ci, Co, k, s, p = case
    kh, kw = (k, k) if isinstance(k, int) else k
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(B, Ci, H, W, generator=g).bfloat16().float().to(dev)
    w = (torch.randn(Co, Ci, kh, kw, generator=g) / math.sqrt(Ci * kh * kw)).bfloat16().float().to(dev)
    b = torch.randn(Co, generator=g).to(dev)
    return x, w, b, s, p


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_forward_and_stats(fn, case):
    x, w, b, s, p = _mk(case)
    ref = F.conv2d(x, w, b, stride=s, padding=p)
    stats = torch.zeros(NREP, 2, w.shape[0], device="cuda", dtype=torch.float64)
    y = fn.conv2d(nhwc(x).bfloat16(), w, b, stride=s, padding=p, stats=stats)
    assert y.shape == nhwc(ref).shape
    assert rel(nchw(y), ref) < 6e-3
    st = stats.sum(0)
    assert rel(st[0], ref.sum((0, 2, 3))) < 1e-3
    assert rel(st[1], (ref * ref).sum((0, 2, 3))) < 1e-3


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_dgrad(fn, case):
    x, w, b, s, p = _mk(case, seed=1)
    x.requires_grad_(True)
    ref = F.conv2d(x, w, None, stride=s, padding=p)
    dy = torch.randn_like(ref).bfloat16().float()
    ref.backward(dy)
    dx = fn.conv2d_dgrad(nhwc(dy).bfloat16(), w, x.shape[2:], stride=s, padding=p)
    assert rel(nchw(dx), x.grad) < 5e-3


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_wgrad(fn, case):
    x, w, b, s, p = _mk(case, seed=2)
    w.requires_grad_(True)
    ref = F.conv2d(x, w, None, stride=s, padding=p)
    dy = torch.randn_like(ref).bfloat16().float()
    ref.backward(dy)
    dw = fn.conv2d_wgrad(nhwc(x).bfloat16(), nhwc(dy).bfloat16(), w.shape, stride=s, padding=p)
    assert rel(dw, w.grad) < 5e-3


@pytest.mark.parametrize("case,cfg", [((2, 33, 83, 16, 16, 3, 1, 1), 8), ((2, 33, 83, 16, 16, 3, 1, 1), 10),
                                      ((2, 33, 83, 8, 16, 3, 1, 1), 9), ((2, 17, 42, 32, 32, 3, 1, 1), 11),
                                      ((2, 33, 83, 16, 32, 3, 2, 1), 10), ((4, 9, 21, 32, 32, 3, 1, 1), 11)])
def test_conv_wgrad_whole_k_tiles(fn, case, cfg):
    """Whole-reduction weight-gradient tiles (configs 8-11) and the multi-lane finalize of many splits."""
    x, w, b, s, p = _mk(case, seed=3)
    w.requires_grad_(True)
    ref = F.conv2d(x, w, None, stride=s, padding=p)
    dy = torch.randn_like(ref).bfloat16().float()
    ref.backward(dy)
    dw = fn.conv2d_wgrad(nhwc(x).bfloat16(), nhwc(dy).bfloat16(), w.shape, stride=s, padding=p, cfg=cfg)
    assert rel(dw, w.grad) < 5e-3


@pytest.mark.parametrize("case,cfg", [((2, 33, 83, 16, 16, 3, 1, 1), 12), ((3, 33, 83, 16, 32, 3, 1, 1), 13),
                                      ((2, 17, 42, 16, 32, 3, 1, 1), 12), ((4, 17, 42, 32, 32, 3, 1, 1), 14),
                                      ((4, 17, 42, 32, 64, 3, 1, 1), 14), ((4, 9, 21, 64, 64, 3, 1, 1), 15),
                                      ((4, 5, 11, 128, 128, 3, 1, 1), 15), ((2, 7, 13, 32, 48, 3, 1, 1), 14),
                                      # "valid" 3x3 (padding 0) and the wide stem maps (configs 16-19, 2-row strips)
                                      ((2, 23, 60, 80, 192, 3, 1, 0), 13), ((2, 23, 60, 80, 48, 3, 1, 0), 12),
                                      ((2, 47, 122, 32, 64, 3, 1, 1), 17), ((2, 49, 124, 32, 32, 3, 1, 0), 16),
                                      ((2, 47, 122, 32, 64, 3, 1, 1), 18), ((3, 47, 122, 32, 40, 3, 1, 1), 19),
                                      ((2, 33, 96, 16, 16, 3, 1, 0), 19)])
@pytest.mark.parametrize("nol", [False, True])
def test_conv_wgrad_patch(fn, case, cfg, nol):
    """3x3 / stride-1 patch weight gradients (configs 12-19: the input strip staged once in LDS, all 9 taps
    read from it): widths that are not multiples of 8, heights that are not multiples of the strip,
    Cout not a multiple of the tile, several channel slices, padding 1 and 0, and normalise-on-load of
    the input."""
    B, H, W, C, Co, k, s, p = case
    x, w, _, _, _ = _mk(case, seed=cfg)
    g = torch.Generator().manual_seed(cfg + 7)
    dy = torch.randn(B, Co, H + 2 * p - 2, W + 2 * p - 2, generator=g).bfloat16().float().cuda()
    if nol:
        consts = torch.zeros(1, 4, C, device="cuda")
        consts[0, 0] = torch.rand(C, generator=g).cuda() + 0.5
        consts[0, 1] = torch.randn(C, generator=g).cuda() * 0.3
        act = F.relu(x * consts[0, 0].view(1, -1, 1, 1) + consts[0, 1].view(1, -1, 1, 1)).bfloat16().float()
    else:
        act = x
    wr = w.clone().requires_grad_(True)
    F.conv2d(act, wr, stride=s, padding=p).backward(dy)
    kw = {"nol": (consts, 1)} if nol else {}
    dw = fn.conv2d_wgrad(nhwc(x).bfloat16(), nhwc(dy).bfloat16(), w.shape, stride=s, padding=p, cfg=cfg, **kw)
    assert rel(dw, wr.grad) < 5e-3
    ref = fn.conv2d_wgrad(nhwc(x).bfloat16(), nhwc(dy).bfloat16(), w.shape, stride=s, padding=p, **kw)
    assert rel(dw, ref) < 1e-5  # same bf16 operands, fp32 accumulation: only the summation order differs


@pytest.mark.parametrize("case", [(2, 4, 13, 128, 128, (1, 7), 1, (0, 3)), (2, 4, 13, 128, 192, (7, 1), 1, (3, 0)),
                                  (2, 23, 60, 80, 192, 3, 1, 0), (1, 9, 27, 288, 384, 3, 2, 0),
                                  (2, 17, 42, 32, 48, 3, 2, 1), (2, 5, 11, 256, 64, 1, 1, 0), (2, 33, 83, 16, 40, 3, 1, 1)])
@pytest.mark.parametrize("cfg", [32, 33, 34, 35])
@pytest.mark.parametrize("nol", [False, True])
def test_conv_wgrad_big_tiles(fn, case, cfg, nol):
    """Large-tile weight gradients on the 32x32x16 MFMA (configs 32-35): a last K tile that runs past the
    padded reduction (Kpad = 896, 1344, 768, 2624 are no multiples of 128), Cout below / not a multiple of
    the 64- or 128-row tile, strided convs, and normalise-on-load of the input."""
    B, H, W, C, Co, k, s, p = case
    x, w, _, _, _ = _mk(case, seed=cfg + 11)
    g = torch.Generator().manual_seed(cfg + 13)
    ref_y = F.conv2d(x, w, stride=s, padding=p)
    dy = torch.randn(ref_y.shape, generator=g).bfloat16().float().cuda()
    if nol:
        consts = torch.zeros(1, 4, C, device="cuda")
        consts[0, 0] = torch.rand(C, generator=g).cuda() + 0.5
        consts[0, 1] = torch.randn(C, generator=g).cuda() * 0.3
        act = F.relu(x * consts[0, 0].view(1, -1, 1, 1) + consts[0, 1].view(1, -1, 1, 1)).bfloat16().float()
    else:
        act = x
    wr = w.clone().requires_grad_(True)
    F.conv2d(act, wr, stride=s, padding=p).backward(dy)
    kw = {"nol": (consts, 1)} if nol else {}
    dw = fn.conv2d_wgrad(nhwc(x).bfloat16(), nhwc(dy).bfloat16(), w.shape, stride=s, padding=p, cfg=cfg, **kw)
    assert rel(dw, wr.grad) < 5e-3
    ref = fn.conv2d_wgrad(nhwc(x).bfloat16(), nhwc(dy).bfloat16(), w.shape, stride=s, padding=p, **kw)
    assert rel(dw, ref) < 1e-5  # same bf16 operands, fp32 accumulation: only the summation order differs


@pytest.mark.parametrize("cfg", [32, 35])
def test_conv_wgrad_big_two_segment(fn, cfg):
    """Large-tile weight gradient of a conv reading two concatenated inputs (the Inception concat)."""
    g = torch.Generator().manual_seed(5)
    a = torch.randn(2, 96, 9, 21, generator=g).bfloat16().float().cuda()
    bb = torch.randn(2, 64, 9, 21, generator=g).bfloat16().float().cuda()
    w = (torch.randn(80, 160, 3, 3, generator=g) / 36).bfloat16().float().cuda()
    ref = F.conv2d(torch.cat([a, bb], 1), w, padding=1)
    dy = torch.randn(ref.shape, generator=g).bfloat16().float().cuda()
    dw = fn.conv2d_wgrad(nhwc(a).bfloat16(), nhwc(dy).bfloat16(), w.shape, padding=1, x2=nhwc(bb).bfloat16(), cfg=cfg)
    wr = w.clone().requires_grad_(True)
    F.conv2d(torch.cat([a, bb], 1), wr, padding=1).backward(dy)
    assert rel(dw, wr.grad) < 5e-3


@pytest.mark.parametrize("case", [(2, 33, 83, 16, 16, 3, 1, 1), (2, 17, 42, 32, 32, 3, 1, 1), (2, 33, 83, 16, 64, 3, 2, 1),
                                  (2, 5, 11, 128, 128, 3, 1, 1), (2, 4, 13, 64, 96, (1, 7), 1, (0, 3)),
                                  (2, 4, 13, 64, 48, (7, 1), 1, (3, 0)), (2, 23, 60, 80, 192, 3, 1, 0),
                                  (2, 5, 11, 256, 64, 1, 1, 0), (2, 33, 83, 8, 16, 1, 1, 0), (3, 9, 21, 32, 24, 3, 2, 1)])
@pytest.mark.parametrize("cfg", list(range(36, 48)))
@pytest.mark.parametrize("nol", [False, True])
def test_conv_wgrad_lean(fn, case, cfg, nol):
    """Lean-staging weight gradients (configs 36-47, csrc/wgrad_lean.hip: per-chunk pixel table in LDS,
    per-thread staging constants, branch-free loads; 44-47 on the 32x32x16 MFMA): 16-128-row tiles with Cout
    below / not a multiple of the tile, K tiles past the padded reduction (144-wide tiles over Kpad 192 / 320
    ...), strided and rectangular kernels, valid padding, 1x1 convs, pixel counts that end mid-chunk, and
    normalise-on-load of the input."""
    B, H, W, C, Co, k, s, p = case
    x, w, _, _, _ = _mk(case, seed=cfg + 21)
    g = torch.Generator().manual_seed(cfg + 23)
    ref_y = F.conv2d(x, w, stride=s, padding=p)
    dy = torch.randn(ref_y.shape, generator=g).bfloat16().float().cuda()
    if nol:
        consts = torch.zeros(1, 4, C, device="cuda")
        consts[0, 0] = torch.rand(C, generator=g).cuda() + 0.5
        consts[0, 1] = torch.randn(C, generator=g).cuda() * 0.3
        act = F.relu(x * consts[0, 0].view(1, -1, 1, 1) + consts[0, 1].view(1, -1, 1, 1)).bfloat16().float()
    else:
        act = x
    wr = w.clone().requires_grad_(True)
    F.conv2d(act, wr, stride=s, padding=p).backward(dy)
    kw = {"nol": (consts, 1)} if nol else {}
    dw = fn.conv2d_wgrad(nhwc(x).bfloat16(), nhwc(dy).bfloat16(), w.shape, stride=s, padding=p, cfg=cfg, **kw)
    assert rel(dw, wr.grad) < 5e-3
    ref = fn.conv2d_wgrad(nhwc(x).bfloat16(), nhwc(dy).bfloat16(), w.shape, stride=s, padding=p, **kw)
    assert rel(dw, ref) < 1e-5  # same bf16 operands, fp32 accumulation: only the summation order differs


@pytest.mark.parametrize("cfg", [38, 43, 47])
def test_conv_wgrad_lean_two_segment(fn, cfg):
    """Lean weight gradient of a conv reading two concatenated inputs (the Inception concat)."""
    g = torch.Generator().manual_seed(6)
    a = torch.randn(2, 96, 9, 21, generator=g).bfloat16().float().cuda()
    bb = torch.randn(2, 64, 9, 21, generator=g).bfloat16().float().cuda()
    w = (torch.randn(80, 160, 3, 3, generator=g) / 36).bfloat16().float().cuda()
    ref = F.conv2d(torch.cat([a, bb], 1), w, padding=1)
    dy = torch.randn(ref.shape, generator=g).bfloat16().float().cuda()
    dw = fn.conv2d_wgrad(nhwc(a).bfloat16(), nhwc(dy).bfloat16(), w.shape, padding=1, x2=nhwc(bb).bfloat16(), cfg=cfg)
    wr = w.clone().requires_grad_(True)
    F.conv2d(torch.cat([a, bb], 1), wr, padding=1).backward(dy)
    assert rel(dw, wr.grad) < 5e-3


# conv.hip default tile, and conv_lds.hip LDS-staged configs (tile, K chunk, K split) -- see test_conv_lds_gpu.py
# heuristic, three LDS-staged configs, and two depth-4 register-pipelined tiles (conv.hip, cfg 128 + tile)
LDS_SAMPLE = [None, 16 + 8 * 0 + 0 + 0, 16 + 8 * 1 + 4 + 2, 16 + 8 * 7 + 0 + 3, 128 + 8, 128 + 11]


@pytest.mark.parametrize("cfg", LDS_SAMPLE)
@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("case", [(4, 17, 42, 32, 32, 3, 1, 1), (2, 33, 83, 16, 16, 3, 1, 1), (4, 9, 21, 64, 128, 3, 2, 1),
                                  (4, 5, 11, 64, 128, 3, 1, 1)])
def test_conv_normalise_on_load(fn, kind, case, cfg):
    """Forward conv reading a pre-BN y and applying act(BN(y)) to its operand (training statistics from the
    replicas; running statistics updated and batch constants published by block 0), and the matching
    weight gradient that rebuilds the operand from the published constants."""
    B, H, W, C, Co, k, s, p = case
    g = torch.Generator().manual_seed(40 + kind)
    y = (torch.randn(B, C, H, W, generator=g) * 2 + 0.3).bfloat16().float().cuda()
    bn, gamma, beta, rm, rv, nbt = _bn_setup(fn, y, C, seed=kind)
    consts = torch.zeros(1, 4, C, device="cuda")
    bn["consts"] = consts.data_ptr()
    w = (torch.randn(Co, C, k, k, generator=g) / math.sqrt(C * k * k)).bfloat16().float().cuda()
    z = _torch_bn(y, gamma, beta)
    act = (z if kind == 0 else F.relu(z)).bfloat16().float()  # the engine's operand is bf16
    ref = F.conv2d(act, w, stride=s, padding=p)
    out = fn.conv2d(nhwc(y).bfloat16(), w, stride=s, padding=p, nol=(bn, kind), cfg=cfg)
    assert rel(nchw(out), ref) < 6e-3
    assert torch.allclose(rm, 0.1 * y.mean((0, 2, 3)), atol=1e-4, rtol=1e-3) and int(nbt.item()) == 1
    inv = torch.rsqrt(y.var((0, 2, 3), unbiased=False) + 1e-5)
    assert torch.allclose(consts[0, 0], gamma * inv, rtol=1e-4, atol=1e-5)
    dy = torch.randn(ref.shape, generator=g).bfloat16().float().cuda()
    wr = w.clone().requires_grad_(True)
    F.conv2d(act, wr, stride=s, padding=p).backward(dy)
    dw = fn.conv2d_wgrad(nhwc(y).bfloat16(), nhwc(dy).bfloat16(), w.shape, stride=s, padding=p, nol=(consts, kind))
    assert rel(dw, wr.grad) < 5e-3


@pytest.mark.parametrize("cfg", LDS_SAMPLE)
def test_conv_two_segment_input(fn, cfg):
    g = torch.Generator().manual_seed(3)
    a = torch.randn(2, 32, 17, 42, generator=g).bfloat16().float().cuda()
    bb = torch.randn(2, 32, 17, 42, generator=g).bfloat16().float().cuda()
    w = (torch.randn(16, 64, 1, 1, generator=g) / 8).bfloat16().float().cuda()
    ref = F.conv2d(torch.cat([a, bb], 1), w)
    y = fn.conv2d(nhwc(a).bfloat16(), w, x2=nhwc(bb).bfloat16(), cfg=cfg)
    assert rel(nchw(y), ref) < 6e-3
    dy = torch.randn_like(ref).bfloat16().float()
    dw = fn.conv2d_wgrad(nhwc(a).bfloat16(), nhwc(dy).bfloat16(), w.shape, x2=nhwc(bb).bfloat16())
    wr = w.clone().requires_grad_(True)
    F.conv2d(torch.cat([a, bb], 1), wr).backward(dy)
    assert rel(dw, wr.grad) < 5e-3


def test_stem_conv_channel_padding(fn):
    """1-channel input stored as 8 zero-padded channels (the gather layout)."""
    g = torch.Generator().manual_seed(4)
    x = torch.randn(2, 1, 100, 250, generator=g).bfloat16().float().cuda()
    w = (torch.randn(16, 1, 7, 7, generator=g) / 7).bfloat16().float().cuda()
    ref = F.conv2d(x, w, stride=3, padding=2)
    x8 = torch.zeros(2, 100, 250, 8, device="cuda", dtype=torch.bfloat16)
    x8[..., 0] = x[:, 0].bfloat16()
    y = fn.conv2d(x8, w, stride=3, padding=2)
    assert rel(nchw(y), ref) < 6e-3
    dy = torch.randn_like(ref).bfloat16().float()
    wr = w.clone().requires_grad_(True)
    F.conv2d(x, wr, stride=3, padding=2).backward(dy)
    dw = fn.conv2d_wgrad(x8, nhwc(dy).bfloat16(), w.shape, stride=3, padding=2)
    assert rel(dw, wr.grad) < 5e-3


# ---------------------------------------------------------------------------------------------------
def _bn_setup(fn, y_ref, C, eps=1e-5, seed=0):
    g = torch.Generator().manual_seed(seed)
    gamma = (1 + 0.2 * torch.randn(C, generator=g)).cuda()
    beta = (0.2 * torch.randn(C, generator=g)).cuda()
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    nbt = torch.zeros(1, device="cuda", dtype=torch.int64)
    stats = torch.zeros(NREP, 2, C, device="cuda", dtype=torch.float64)
    stats[0, 0] = y_ref.sum((0, 2, 3))
    stats[0, 1] = (y_ref * y_ref).sum((0, 2, 3))
    cnt = y_ref.numel() // C
    bn = fn.bn_args(stats, gamma, beta, rm, rv, nbt, cnt, eps=eps)
    bn["_keepalive"] = stats  # the dict only holds raw pointers
    return bn, gamma, beta, rm, rv, nbt


def _torch_bn(y, gamma, beta, eps=1e-5):
    return F.batch_norm(y, None, None, gamma, beta, training=True, eps=eps)


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("C", [8, 16, 48, 128])
def test_bn_tail_forward_backward(fn, kind, C, fused):
    g = torch.Generator().manual_seed(10 + kind)
    B, H, W = 4, 9, 21
    y = (torch.randn(B, C, H, W, generator=g) * 2 + 0.5).bfloat16().float().cuda()
    r = torch.randn(B, C, H, W, generator=g).bfloat16().float().cuda()
    bn, gamma, beta, rm, rv, nbt = _bn_setup(fn, y, C, seed=kind)
    yr = y.clone().requires_grad_(True)
    rr = r.clone().requires_grad_(True)
    gam = gamma.clone().requires_grad_(True)
    bet = beta.clone().requires_grad_(True)
    z = _torch_bn(yr, gam, bet)
    if kind == 0:
        out = z
    elif kind == 1:
        out = F.relu(z)
    elif kind == 2:
        out = torch.sigmoid(z)
    elif kind == 3:
        out = torch.sigmoid(z) * rr
    elif kind == 4:
        out = F.relu(z + rr)
    else:
        out = F.max_pool2d(F.relu(z), 2, 2, ceil_mode=True)
    ours = fn.bn_tail(kind, nhwc(y).bfloat16(), bn, r=nhwc(r).bfloat16() if kind in (3, 4) else None)
    assert rel(nchw(ours), out) < 6e-3
    # running statistics (momentum 0.1, unbiased variance)
    var = y.var(dim=(0, 2, 3), unbiased=True)
    assert torch.allclose(rm, 0.1 * y.mean((0, 2, 3)), atol=1e-4, rtol=1e-3)
    assert torch.allclose(rv, 0.9 + 0.1 * var, atol=1e-4, rtol=1e-3)
    assert int(nbt.item()) == 1
    # backward
    go = torch.randn_like(out)
    out.backward(go)
    dg, db = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
    dy, side, _ = fn.bn_tail_backward(kind, nhwc(y).bfloat16(), bn, [nhwc(go).contiguous()], dg, db,
                                      r=nhwc(r).bfloat16() if kind in (3, 4) else None, fused=fused)
    assert rel(nchw(dy), yr.grad) < 1e-2
    assert rel(dg, gam.grad) < 1e-2
    assert rel(db, bet.grad) < 1e-2
    if kind in (3, 4):
        assert rel(nchw(side), rr.grad) < 1e-2


@pytest.mark.parametrize("cfg", LDS_SAMPLE)
@pytest.mark.parametrize("kind", [0, 1, 2])
@pytest.mark.parametrize("case", [(4, 17, 42, 32, 16, 3, 1, 1), (4, 9, 21, 64, 128, 3, 2, 1),
                                  (2, 33, 83, 16, 16, 3, 1, 1), (4, 5, 11, 128, 64, 1, 1, 0)])
def test_dgrad_fused_bn_backward_stats(fn, kind, case, cfg):
    """conv(act(BN(y))): the dgrad epilogue accumulates the BN-backward sums, the tail runs its apply pass
    only; dy / dgamma / dbeta against autograd, and against the two-pass (reduce + apply) backward."""
    B, H, W, C, Co, k, s, p = case
    g = torch.Generator().manual_seed(30 + kind)
    y = (torch.randn(B, C, H, W, generator=g) * 2 + 0.3).bfloat16().float().cuda()
    bn, gamma, beta, rm, rv, nbt = _bn_setup(fn, y, C, seed=kind)
    w = (torch.randn(Co, C, k, k, generator=g) / math.sqrt(C * k * k)).bfloat16().float().cuda()
    yr = y.clone().requires_grad_(True)
    gam = gamma.clone().requires_grad_(True)
    bet = beta.clone().requires_grad_(True)
    z = _torch_bn(yr, gam, bet)
    act = z if kind == 0 else (F.relu(z) if kind == 1 else torch.sigmoid(z))
    out = F.conv2d(act, w, stride=s, padding=p)
    go = torch.randn(out.shape, generator=g).bfloat16().float().cuda()
    out.backward(go)
    yb = nhwc(y).bfloat16()
    part = torch.zeros(NREP, 3, C, device="cuda", dtype=torch.float64)
    dx = fn.conv2d_dgrad(nhwc(go).bfloat16(), w, (H, W), stride=s, padding=p, bn_stats=(yb, bn, part, kind), cfg=cfg)
    dg, db = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
    dy, _, _ = fn.bn_tail_backward(kind, yb, bn, [dx], dg, db, part=part)
    assert rel(nchw(dy), yr.grad) < 1e-2
    # the BN sums are cancelling sums (|sum| << sum |terms|): check them in fp64 on the ENGINE's own dx
    yd, gx = y.double(), nchw(dx).double()
    mu = yd.mean((0, 2, 3), keepdim=True)
    inv = torch.rsqrt(yd.var((0, 2, 3), unbiased=False, keepdim=True) + 1e-5)
    xh = (yd - mu) * inv
    zz = gamma.double().view(1, -1, 1, 1) * xh + beta.double().view(1, -1, 1, 1)
    dz = gx if kind == 0 else (gx * (zz > 0) if kind == 1 else gx * torch.sigmoid(zz) * (1 - torch.sigmoid(zz)))
    assert rel(dg, (dz * xh).sum((0, 2, 3))) < 1e-4
    assert rel(db, dz.sum((0, 2, 3))) < 1e-4
    dg2, db2 = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
    dy2, _, _ = fn.bn_tail_backward(kind, yb, bn, [dx], dg2, db2)
    assert rel(dy, dy2) < 1e-4 and rel(dg, dg2) < 1e-5 and rel(db, db2) < 1e-5


@pytest.mark.parametrize("fused", [False, True])
def test_bn_residual_projection(fn, fused):
    g = torch.Generator().manual_seed(20)
    B, C, H, W = (4, 32, 9, 21) if fused else (4, 32, 17, 42)  # single launch: <= 2048 pixels
    y = torch.randn(B, C, H, W, generator=g).bfloat16().float().cuda()
    y2 = (torch.randn(B, C, H, W, generator=g) + 1).bfloat16().float().cuda()
    bn, gamma, beta, *_ = _bn_setup(fn, y, C, seed=1)
    bn2, gamma2, beta2, *_ = _bn_setup(fn, y2, C, seed=2)
    yr, y2r = y.clone().requires_grad_(True), y2.clone().requires_grad_(True)
    gs = [t.clone().requires_grad_(True) for t in (gamma, beta, gamma2, beta2)]
    out = F.relu(_torch_bn(yr, gs[0], gs[1]) + _torch_bn(y2r, gs[2], gs[3]))
    ours = fn.bn_tail(4, nhwc(y).bfloat16(), bn, r=nhwc(y2).bfloat16(), bn2=bn2)
    assert rel(nchw(ours), out) < 6e-3
    go = torch.randn_like(out)
    out.backward(go)
    d = [torch.zeros(C, device="cuda") for _ in range(4)]
    dy, _, dy2 = fn.bn_tail_backward(4, nhwc(y).bfloat16(), bn, [nhwc(go)], d[0], d[1], r=nhwc(y2).bfloat16(),
                                     bn2=bn2, dgamma2=d[2], dbeta2=d[3], fused=fused)
    assert rel(nchw(dy), yr.grad) < 1e-2
    assert rel(nchw(dy2), y2r.grad) < 1e-2
    for a, b in zip(d, gs):
        assert rel(a, b.grad) < 1e-2


def test_bn_eval_mode(fn):
    g = torch.Generator().manual_seed(21)
    C = 16
    y = torch.randn(2, C, 9, 21, generator=g).bfloat16().float().cuda()
    gamma, beta = torch.rand(C).cuda() + 0.5, torch.randn(C).cuda()
    rm, rv = torch.randn(C).cuda(), torch.rand(C).cuda() + 0.5
    st = torch.zeros(NREP, 2, C, device="cuda", dtype=torch.float64)
    bn = fn.bn_args(st, gamma, beta, rm, rv, None, 1, training=False)
    out = fn.bn_tail(1, nhwc(y).bfloat16(), bn)
    ref = F.relu(F.batch_norm(y, rm, rv, gamma, beta, training=False))
    assert rel(nchw(out), ref) < 6e-3


@pytest.mark.parametrize("is_max", [True, False])
def test_inception_pools(fn, is_max):
    g = torch.Generator().manual_seed(30)
    x = torch.randn(2, 64, 23, 60, generator=g).bfloat16().float().cuda().requires_grad_(True)
    ref = F.max_pool2d(x, 3, 2) if is_max else F.avg_pool2d(x, 3, 1, 1)
    y = fn.pool3(nhwc(x.detach()).bfloat16(), is_max)
    assert rel(nchw(y), ref) < 6e-3
    go = torch.randn_like(ref).bfloat16().float()  # gradients are stored bf16
    ref.backward(go)
    dx = fn.pool3_backward(nhwc(x.detach()).bfloat16(), nhwc(go), is_max)
    assert dx.dtype == torch.bfloat16
    assert rel(nchw(dx), x.grad) < 4e-3  # fp32 sum of the bf16 window gradients, one bf16 rounding
    if is_max:  # argmax stored by the forward: identical gradient (same first-max tie rule), windows not re-read
        am = torch.full((y.numel(),), 255, dtype=torch.uint8, device="cuda")
        y2 = fn.pool3(nhwc(x.detach()).bfloat16(), is_max, am=am)
        assert torch.equal(y2, y) and int(am.max()) <= 8
        # ties: a constant patch must route the gradient to the first window position, as torch does
        xt = x.detach().clone()
        xt[:, :, :6, :6] = 0.5
        xt.requires_grad_(True)
        F.max_pool2d(xt, 3, 2).backward(go)
        fn.pool3(nhwc(xt.detach()).bfloat16(), is_max, am=am)
        dx2 = fn.pool3_backward(nhwc(xt.detach()).bfloat16(), nhwc(go), is_max, am=am)
        assert torch.equal(dx2, fn.pool3_backward(nhwc(xt.detach()).bfloat16(), nhwc(go), is_max))
        assert rel(nchw(dx2), xt.grad) < 4e-3
        # NaN propagates like torch: the output is NaN and the gradient goes to the NaN's position
        xn = x.detach().clone()
        xn[0, 3, 4, 5] = float("nan")
        xn.requires_grad_(True)
        rn = F.max_pool2d(xn, 3, 2)
        rn.backward(go)
        yn = nchw(fn.pool3(nhwc(xn.detach()).bfloat16(), is_max, am=am))
        assert torch.equal(torch.isnan(yn), torch.isnan(rn))
        dxn = nchw(fn.pool3_backward(nhwc(xn.detach()).bfloat16(), nhwc(go), is_max, am=am))
        assert rel(dxn, xn.grad) < 4e-3
        with pytest.raises(ValueError):  # the argmax buffer is validated before the kernel reads it
            fn.pool3_backward(nhwc(x.detach()).bfloat16(), nhwc(go), is_max, am=am[:-8])


def test_gather_batch(fn):
    X = torch.randn(10, 1, 100, 250, device="cuda")
    lab = torch.randint(0, 16, (10, 2), device="cuda")
    idx = torch.tensor([3, 7, 1], device="cuda")
    xb, lb = fn.gather_batch(X, lab, idx)
    assert torch.equal(lb, lab[idx])
    assert torch.equal(xb[..., 0], X[idx, 0].bfloat16())
    assert (xb[..., 1:] == 0).all()


def test_mtl_head(fn):
    from mtl_das_pytorch_amd.ops.hip import lib, ptr, stream
    T, B, H, W, C = 2, 6, 5, 11, 128
    g = torch.Generator().manual_seed(40)
    feat = torch.randn(T, B, C, H, W, generator=g).bfloat16().float().cuda()
    labels = torch.stack([torch.randint(0, 16, (B,)), torch.randint(0, 2, (B,))], 1).cuda()
    logp = torch.zeros(T, B, 16, device="cuda")
    dfeat = torch.zeros(T, B * H * W, C, device="cuda", dtype=torch.bfloat16)
    metrics = torch.zeros(T, 4, device="cuda")
    conf = torch.zeros(T, 16, 16, device="cuda", dtype=torch.int32)
    fb = torch.stack([nhwc(feat[t]) for t in range(T)]).bfloat16().contiguous()
    d = {"feat": ptr(fb), "fgs": B * H * W * C, "ldf": C, "labels": ptr(labels), "lab_stride": 2, "lab_off": 0,
         "T": T, "B": B, "HW": H * W, "C": C, "ncls": [16, 2], "w": [1.0, 0.5], "logp": ptr(logp),
         "dfeat": ptr(dfeat), "dgs": B * H * W * C, "metrics": ptr(metrics), "confusion": ptr(conf)}
    lib().mtl_head(stream(), d)
    fr = feat.clone().requires_grad_(True)
    loss = 0
    for t, (k, wt) in enumerate(zip([16, 2], [1.0, 0.5])):
        gap = fr[t].mean((2, 3))
        lg = F.avg_pool1d(gap.unsqueeze(1), C // k, C // k).squeeze(1)
        lp = F.log_softmax(lg, 1)
        assert torch.allclose(logp[t, :, :k], lp.detach(), atol=1e-4)
        nll = F.nll_loss(lp, labels[:, t])
        loss = loss + wt * nll
        assert abs(metrics[t, 0].item() - nll.item() * B) < 1e-3
        assert metrics[t, 1].item() == (lp.argmax(1) == labels[:, t]).sum().item()
        assert conf[t].sum().item() == B
    loss.backward()
    ref = torch.stack([nhwc(fr.grad[t]).reshape(B * H * W, C) for t in range(T)])
    assert rel(dfeat, ref) < 4e-3  # bf16 gradient storage
