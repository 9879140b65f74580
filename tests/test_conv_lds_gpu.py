"""The LDS-staged implicit-GEMM conv kernels (csrc/conv_lds.hip) against fp32 PyTorch: every tile config x
K chunk x cross-block K split, forward (+bias, +fused BN sums) and data gradient (stride 1 and the
sub-pixel phase decomposition of stride 2) on Model A and Model C layer geometries; plus split-K
determinism and the reuse of the arrival tickets across launches."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

NREP = 32

# B, H, W, Ci, Co, k, s, p -- Model A / Model C classes (kernel shapes, strides, paddings), odd sizes
CASES = [
    (2, 33, 83, 16, 16, 3, 1, 1),
    (2, 33, 83, 16, 32, 1, 2, 0),
    (2, 33, 83, 16, 32, 3, 2, 1),
    (2, 17, 42, 32, 64, 3, 2, 1),
    (2, 9, 21, 64, 128, 3, 1, 1),
    (2, 5, 11, 256, 64, 1, 1, 0),
    (2, 10, 28, 48, 64, (5, 5), 1, (2, 2)),
    (2, 4, 13, 128, 192, (1, 7), 1, (0, 3)),
    (2, 4, 13, 128, 160, (7, 1), 1, (3, 0)),
    (2, 23, 60, 80, 192, 3, 1, 0),
    (1, 9, 27, 288, 384, 3, 2, 0),
    (3, 1, 6, 448, 384, 3, 1, 1),
    (2, 7, 9, 40, 24, 3, 2, 0),
]
TILES = [(t, kc) for t in range(8) for kc in (64, 128) if not (kc == 128 and t == 3)]


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def nchw(x):
    return x.permute(0, 3, 1, 2).contiguous()


def _mk(case, seed):
    B, H, W, Ci, Co, k, s, p = case
    kh, kw = (k, k) if isinstance(k, int) else k
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, Ci, H, W, generator=g).bfloat16().float().cuda()
    w = (torch.randn(Co, Ci, kh, kw, generator=g) / math.sqrt(Ci * kh * kw)).bfloat16().float().cuda()
    b = torch.randn(Co, generator=g).cuda()
    return x, w, b, s, p


@pytest.mark.parametrize("tile,kc", TILES)
def test_lds_forward_all_configs(tile, kc):
    from mtl_das_pytorch_amd.ops import functional as fn
    for ci, case in enumerate(CASES):
        x, w, b, s, p = _mk(case, ci)
        ref = F.conv2d(x, w, b, stride=s, padding=p)
        for splits in (1, 2, 8):
            cfg = fn.lds_cfg(tile, kc, splits)
            stats = torch.zeros(NREP, 2, w.shape[0], device="cuda", dtype=torch.float64)
            y = fn.conv2d(nhwc(x).bfloat16(), w, b, stride=s, padding=p, stats=stats, cfg=cfg)
            assert rel(nchw(y), ref) < 6e-3, (case, cfg)
            st = stats.sum(0)
            assert rel(st[0], ref.sum((0, 2, 3))) < 1e-3, (case, cfg)
            assert rel(st[1], (ref * ref).sum((0, 2, 3))) < 1e-3, (case, cfg)


@pytest.mark.parametrize("tile,kc", TILES)
def test_lds_dgrad_all_configs(tile, kc):
    from mtl_das_pytorch_amd.ops import functional as fn
    for ci, case in enumerate(CASES):
        x, w, b, s, p = _mk(case, 100 + ci)
        xr = x.clone().requires_grad_(True)
        out = F.conv2d(xr, w, None, stride=s, padding=p)
        dy = torch.randn_like(out).bfloat16().float()
        out.backward(dy)
        for splits in (1, 4):
            cfg = fn.lds_cfg(tile, kc, splits)
            dx = fn.conv2d_dgrad(nhwc(dy).bfloat16(), w, x.shape[2:], stride=s, padding=p, cfg=cfg)
            assert rel(nchw(dx), xr.grad) < 5e-3, (case, cfg)


def test_lds_split_k_deterministic_and_tickets_reset():
    """A split-K launch re-run many times gives bitwise-identical results (the reducer sums the partial
    tiles in split order whatever block arrives last) and leaves every arrival ticket at zero."""
    from mtl_das_pytorch_amd.ops import functional as fn
    x, w, b, s, p = _mk((4, 4, 13, 192, 192, (1, 7), 1, (0, 3)), 7)
    call = fn.prepare_conv2d(nhwc(x).bfloat16(), w, b, stride=s, padding=p, cfg=fn.lds_cfg(0, 64, 8))
    first = call.run().clone()
    for _ in range(20):
        assert torch.equal(call.run(), first)
    w_, cnt = call._ws
    torch.cuda.synchronize()
    assert int(cnt.abs().sum()) == 0
    ref = F.conv2d(x, w, b, stride=s, padding=p)
    assert rel(nchw(first), ref) < 6e-3


def test_lds_invalid_configs_rejected():
    from mtl_das_pytorch_amd.ops import functional as fn
    x, w, b, s, p = _mk(CASES[0], 0)
    with pytest.raises(ValueError):  # 128 x 128 tile with a 128-deep chunk exceeds the LDS plan
        fn.prepare_conv2d(nhwc(x).bfloat16(), w, b, stride=s, padding=p, cfg=16 + 8 * 3 + 4)
