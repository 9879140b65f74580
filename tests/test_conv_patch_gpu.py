"""The 3x3 / stride-1 patch conv kernel (csrc/conv_lds.hip conv_patch_kernel: a block stages R whole output
rows' input strip with halo and a channel slice of the weights in LDS, every tap's MFMA operand a shifted
read of the strip) against fp32 PyTorch: every tile x channel-slice config that accepts the shape, forward
(+bias, +fused BN sums, +normalise-on-load, two-segment input), data gradient ("same" and "valid" convs,
i.e. transposed-conv halos 1 and 2) and the fused BN-backward statistics epilogue."""
import math

import pytest
import torch
import torch.nn.functional as F

from test_conv_lds_gpu import NREP, nchw, nhwc, rel

pytestmark = pytest.mark.gpu

# (B, H, W, Ci, Co, padding): the geometries the kernel is for, shrunk in batch
PCASES = [
    (2, 47, 122, 32, 64, 1),   # Model C Conv2d_2b (R = 2 rows of 122 per block)
    (2, 49, 124, 32, 32, 0),   # Conv2d_2a ("valid": dgrad halo 2)
    (2, 23, 60, 80, 192, 0),   # Conv2d_4a (Cs = 80: slices of 16)
    (2, 33, 83, 16, 16, 1),    # Model A stage 1 (R = 3)
    (3, 17, 42, 32, 32, 1),    # Model A stage 2 (R = 6, last strip partial)
    (2, 9, 21, 64, 128, 1),    # Model A stage 3 (two slices of 32, N > BN)
    (2, 10, 28, 64, 96, 1),    # Inception Mixed_5b 3x3
]


def _cfgs():  # both forms: one strip per block, and persistent (DMA-pipelined strips, Cs == cb only)
    from mtl_das_pytorch_amd.ops import functional as fn
    return [fn.patch_cfg(t, cb, pers) for pers in (False, True) for t in range(len(fn.PATCH_TILES))
            for cb in fn.PATCH_CB]


def _mk(case, seed):
    B, H, W, Ci, Co, p = case
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, Ci, H, W, generator=g).bfloat16().float().cuda()
    w = (torch.randn(Co, Ci, 3, 3, generator=g) / math.sqrt(Ci * 9)).bfloat16().float().cuda()
    b = torch.randn(Co, generator=g).cuda()
    return x, w, b, p


def test_patch_forward_all_configs():
    from mtl_das_pytorch_amd.ops import functional as fn
    ran = 0
    for ci, case in enumerate(PCASES):
        x, w, b, p = _mk(case, ci)
        ref = F.conv2d(x, w, b, padding=p)
        for cfg in _cfgs():
            stats = torch.zeros(NREP, 2, w.shape[0], device="cuda", dtype=torch.float64)
            try:
                call = fn.prepare_conv2d(nhwc(x).bfloat16(), w, b, padding=p, stats=stats, cfg=cfg)
            except (ValueError, RuntimeError):
                continue  # this tile / slice does not take the shape (row wider than the strip, Cs % CB, LDS)
            y = call.run()
            ran += 1
            assert rel(nchw(y), ref) < 6e-3, (case, cfg)
            st = stats.sum(0)
            assert rel(st[0], ref.sum((0, 2, 3))) < 1e-3, (case, cfg)
            assert rel(st[1], (ref * ref).sum((0, 2, 3))) < 1e-3, (case, cfg)
    assert ran >= 50


def test_patch_persistent_matches_strip_form():
    """The persistent form (strips looped per block, DMA-prefetched, statistics summed in registers over a
    block's strips) gives the same output as the one-strip-per-block form up to the fp32 order of the BN sums."""
    from mtl_das_pytorch_amd.ops import functional as fn
    x, w, b, p = _mk((3, 47, 122, 32, 64, 1), 9)
    outs = []
    for pers in (False, True):
        stats = torch.zeros(NREP, 2, 64, device="cuda", dtype=torch.float64)
        y = fn.conv2d(nhwc(x).bfloat16(), w, b, padding=p, stats=stats, cfg=fn.patch_cfg(1, 32, pers))
        outs.append((y, stats.sum(0)))
    assert torch.equal(outs[0][0], outs[1][0])
    assert rel(outs[0][1], outs[1][1]) < 1e-6


def test_patch_dgrad_all_configs():
    from mtl_das_pytorch_amd.ops import functional as fn
    ran = 0
    for ci, case in enumerate(PCASES):
        x, w, b, p = _mk(case, 100 + ci)
        xr = x.clone().requires_grad_(True)
        out = F.conv2d(xr, w, None, padding=p)
        dy = torch.randn_like(out).bfloat16().float()
        out.backward(dy)
        for cfg in _cfgs():
            try:
                call = fn.prepare_conv2d_dgrad(nhwc(dy).bfloat16(), w, x.shape[2:], padding=p, cfg=cfg)
            except (ValueError, RuntimeError):
                continue
            dx = call.run()
            ran += 1
            assert rel(nchw(dx), xr.grad) < 5e-3, (case, cfg)
    assert ran >= 40


@pytest.mark.parametrize("kind", [0, 1])
def test_patch_normalise_on_load(kind):
    """MODE_FWD_NOL: the strip holds act(BN(y)) computed once per element while staging; padding stays 0."""
    from mtl_das_pytorch_amd.ops import functional as fn
    from test_kernels_gpu import _bn_setup, _torch_bn
    for case in [(2, 33, 83, 16, 16, 1), (2, 47, 122, 32, 64, 1), (2, 23, 60, 80, 96, 0)]:
        B, H, W, C, Co, p = case
        g = torch.Generator().manual_seed(40 + kind)
        y = (torch.randn(B, C, H, W, generator=g) * 2 + 0.3).bfloat16().float().cuda()
        w = (torch.randn(Co, C, 3, 3, generator=g) / math.sqrt(C * 9)).bfloat16().float().cuda()
        z = _torch_bn(y, *_bn_setup(fn, y, C, seed=kind)[1:3])
        act = (z if kind == 0 else F.relu(z)).bfloat16().float()
        ref = F.conv2d(act, w, padding=p)
        ran = 0
        for cfg in _cfgs():
            bn, gamma, beta, rm, rv, nbt = _bn_setup(fn, y, C, seed=kind)
            try:
                call = fn.prepare_conv2d(nhwc(y).bfloat16(), w, padding=p, nol=(bn, kind), cfg=cfg)
            except (ValueError, RuntimeError):
                continue
            out = call.run()
            ran += 1
            assert rel(nchw(out), ref) < 6e-3, (case, cfg)
            assert int(nbt.item()) == 1 and torch.allclose(rm, 0.1 * y.mean((0, 2, 3)), atol=1e-4, rtol=1e-3)
        assert ran >= 3, case


@pytest.mark.parametrize("Co", [48, 32])
@pytest.mark.parametrize("kind", [0, 1, 2])
def test_patch_dgrad_fused_bn_stats(kind, Co):
    from mtl_das_pytorch_amd.ops import functional as fn
    B, H, W, C = 2, 17, 42, 32
    g = torch.Generator().manual_seed(7 + kind)
    y = (torch.randn(B, C, H, W, generator=g) * 1.5 + 0.2).bfloat16().float().cuda()
    st = torch.zeros(NREP, 2, C, device="cuda", dtype=torch.float64)
    st[0, 0] = y.sum((0, 2, 3)).double()
    st[0, 1] = (y * y).sum((0, 2, 3)).double()
    gamma = (torch.rand(C, generator=g) + 0.5).cuda()
    beta = (torch.randn(C, generator=g) * 0.1).cuda()
    bn = fn.bn_args(st, gamma, beta, torch.zeros(C, device="cuda"), torch.ones(C, device="cuda"),
                    torch.zeros((), dtype=torch.int64, device="cuda"), count=B * H * W)
    yb = nhwc(y).bfloat16()
    w = (torch.randn(Co, C, 3, 3, generator=g) / 17).bfloat16().float().cuda()
    go = torch.randn(B, H, W, Co, generator=g).bfloat16().cuda()
    dx_ref = fn.conv2d_dgrad(go, w, (H, W), stride=1, padding=1)
    dg, db = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
    fn.bn_tail_backward(kind, yb, bn, [dx_ref], dg, db)
    ran = 0
    for cfg in _cfgs():
        part = torch.zeros(NREP, 3, C, device="cuda", dtype=torch.float64)
        try:
            call = fn.prepare_conv2d_dgrad(go, w, (H, W), stride=1, padding=1, cfg=cfg, bn_stats=(yb, bn, part, kind))
        except (ValueError, RuntimeError):
            continue
        dx = call.run()
        ran += 1
        assert rel(dx, dx_ref) < 2e-4, cfg  # bf16 outputs of two accumulation orders (one-ulp flips)
        got = part.sum(0)
        assert rel(got[0], db.double()) < 1e-4 and rel(got[1], dg.double()) < 1e-4, cfg
    assert ran >= (5 if Co == 48 else 15)  # dy channels 48: 16-channel slices only; 32: persistent forms too


def test_patch_two_segment_input():
    from mtl_das_pytorch_amd.ops import functional as fn
    g = torch.Generator().manual_seed(3)
    a = torch.randn(2, 32, 17, 42, generator=g).bfloat16().float().cuda()
    bb = torch.randn(2, 32, 17, 42, generator=g).bfloat16().float().cuda()
    w = (torch.randn(48, 64, 3, 3, generator=g) / 24).bfloat16().float().cuda()
    ref = F.conv2d(torch.cat([a, bb], 1), w, padding=1)
    for cfg in (fn.patch_cfg(1, 16), fn.patch_cfg(1, 32), fn.patch_cfg(3, 32)):
        y = fn.conv2d(nhwc(a).bfloat16(), w, padding=1, x2=nhwc(bb).bfloat16(), cfg=cfg)
        assert rel(nchw(y), ref) < 6e-3, cfg


def test_patch_rejects_other_convs():
    from mtl_das_pytorch_amd.ops import functional as fn
    x = torch.zeros(2, 17, 42, 32, device="cuda", dtype=torch.bfloat16)
    for w, s in [(torch.zeros(32, 32, 3, 3, device="cuda"), 2), (torch.zeros(32, 32, 1, 1, device="cuda"), 1)]:
        with pytest.raises((ValueError, RuntimeError)):
            fn.conv2d(x, w, stride=s, padding=1 if w.shape[2] == 3 else 0, cfg=fn.patch_cfg(1, 32))
    with pytest.raises((ValueError, RuntimeError)):  # row wider than the strip capacity of a 128-pixel tile
        fn.conv2d(torch.zeros(1, 4, 200, 32, device="cuda", dtype=torch.bfloat16),
                  torch.zeros(32, 32, 3, 3, device="cuda"), padding=1, cfg=fn.patch_cfg(3, 32))
