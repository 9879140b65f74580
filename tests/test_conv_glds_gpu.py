"""The LDS-DMA implicit-GEMM conv kernel (csrc/conv_lds.hip conv_glds_kernel: global_load_lds_dwordx4 into a
swizzled 3-stage LDS ring, or a deep ring of up to 8 stages, counted vmcnt + raw barrier) against fp32
PyTorch: every tile config (both rings) x cross-block K split, forward (+bias, +fused BN sums), data gradient (stride 1 and the stride-2 sub-pixel phases) and the
fused BN-backward statistics epilogue, on the Model A / Model C layer classes of tests/test_conv_lds_gpu.py
plus the stem geometries this kernel is meant for."""
import pytest
import torch
import torch.nn.functional as F

from test_conv_lds_gpu import CASES, NREP, _mk, nchw, nhwc, rel

pytestmark = pytest.mark.gpu

GCASES = CASES + [
    (2, 47, 122, 32, 64, 3, 1, 1),   # Model C Conv2d_2b (stem, 183k px at B = 32)
    (2, 23, 60, 64, 80, 1, 1, 0),    # Conv2d_3b
    (2, 100, 250, 8, 16, 3, 2, 1),   # a 2-channel-input style stem (Cs = 8)
]


RINGS = [(t, False) for t in range(8)] + [(t, True) for t in (0, 1, 2, 3, 5, 7)]  # (tile, deep ring)


@pytest.mark.parametrize("tile,deep", RINGS)
def test_glds_forward_all_configs(tile, deep):
    from mtl_das_pytorch_amd.ops import functional as fn
    for ci, case in enumerate(GCASES):
        x, w, b, s, p = _mk(case, ci)
        ref = F.conv2d(x, w, b, stride=s, padding=p)
        for splits in (1, 2, 8):
            cfg = fn.glds_cfg(tile, splits, deep)
            stats = torch.zeros(NREP, 2, w.shape[0], device="cuda", dtype=torch.float64)
            y = fn.conv2d(nhwc(x).bfloat16(), w, b, stride=s, padding=p, stats=stats, cfg=cfg)
            assert rel(nchw(y), ref) < 6e-3, (case, cfg)
            st = stats.sum(0)
            assert rel(st[0], ref.sum((0, 2, 3))) < 1e-3, (case, cfg)
            assert rel(st[1], (ref * ref).sum((0, 2, 3))) < 1e-3, (case, cfg)


@pytest.mark.parametrize("tile,deep", RINGS)
def test_glds_dgrad_all_configs(tile, deep):
    from mtl_das_pytorch_amd.ops import functional as fn
    for ci, case in enumerate(GCASES):
        x, w, b, s, p = _mk(case, 100 + ci)
        xr = x.clone().requires_grad_(True)
        out = F.conv2d(xr, w, None, stride=s, padding=p)
        dy = torch.randn_like(out).bfloat16().float()
        out.backward(dy)
        for splits in (1, 4):
            cfg = fn.glds_cfg(tile, splits, deep)
            dx = fn.conv2d_dgrad(nhwc(dy).bfloat16(), w, x.shape[2:], stride=s, padding=p, cfg=cfg)
            assert rel(nchw(dx), xr.grad) < 5e-3, (case, cfg)


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_glds_dgrad_fused_bn_stats(kind):
    """MODE_DGRAD_BNS on the LDS-DMA kernel: the dgrad output is the gradient of act(BN(y)) and the epilogue
    accumulates sum(dz), sum(dz * xhat) of that BN; against the reduce pass of bn_tail_backward."""
    from mtl_das_pytorch_amd.ops import functional as fn
    B, H, W, C, Co = 2, 17, 42, 32, 48
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
    for tile, deep in RINGS:
        for splits in (1, 2):
            part = torch.zeros(NREP, 3, C, device="cuda", dtype=torch.float64)
            cfg = fn.glds_cfg(tile, splits, deep)
            dx = fn.conv2d_dgrad(go, w, (H, W), stride=1, padding=1, cfg=cfg, bn_stats=(yb, bn, part, kind))
            dx_ref = fn.conv2d_dgrad(go, w, (H, W), stride=1, padding=1)
            # bf16 outputs of two fp32 accumulation orders: an element whose sums straddle a rounding boundary
            # differs by one bf16 ulp (~4e-3 relative), a few 1e-5 of them
            assert rel(dx, dx_ref) < 2e-4, (tile, splits)
            dg, db = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
            fn.bn_tail_backward(kind, yb, bn, [dx_ref], dg, db)
            got = part.sum(0)
            assert rel(got[0], db.double()) < 1e-4 and rel(got[1], dg.double()) < 1e-4, (tile, splits)
