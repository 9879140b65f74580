"""Every register-pipelined implicit-GEMM tile config of csrc/conv.hip (tiles 0-13 at pipeline depth 2, and the
same tiles at depth 4, cfg 128 + tile) against fp32 PyTorch: forward with bias and fused BN sums, and
data gradient (stride 1 and 2) -- on Model A and Model C layer classes whose K loops are long, short and odd (remainder steps of the deeper pipeline).  Normalise-on-load, two-segment inputs and
the fused BN-backward statistics run on depth-4 tiles in tests/test_kernels_gpu.py (LDS_SAMPLE)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

NREP = 32
CFGS = list(range(14)) + [128 + t for t in range(14)]
CASES = [
    # B, H, W, Ci, Co, k, s, p
    (2, 33, 83, 16, 16, 3, 1, 1),          # K = 144: 5 K-steps
    (2, 4, 13, 128, 192, (1, 7), 1, (0, 3)),  # K = 896: 28 K-steps (Model C 1x7)
    (2, 17, 42, 32, 64, 3, 2, 1),          # strided
    (3, 1, 6, 448, 384, 3, 1, 1),          # K = 4032, M = 18
]


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


@pytest.fixture(scope="module")
def fn():
    from mtl_das_pytorch_amd.ops import functional as Fn
    from mtl_das_pytorch_amd.ops.hip import lib
    lib()
    return Fn


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("cfg", CFGS)
def test_igemm_forward_stats(fn, cfg, case):
    x, w, b, s, p = _mk(case, cfg)
    ref = F.conv2d(x, w, b, stride=s, padding=p)
    stats = torch.zeros(NREP, 2, w.shape[0], device="cuda", dtype=torch.float64)
    y = fn.conv2d(nhwc(x).bfloat16(), w, b, stride=s, padding=p, stats=stats, cfg=cfg)
    assert rel(nchw(y), ref) < 6e-3
    st = stats.sum(0)
    assert rel(st[0], ref.sum((0, 2, 3))) < 1e-3
    assert rel(st[1], (ref * ref).sum((0, 2, 3))) < 1e-3


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("cfg", CFGS)
def test_igemm_dgrad(fn, cfg, case):
    x, w, b, s, p = _mk(case, cfg + 1)
    x.requires_grad_(True)
    ref = F.conv2d(x, w, None, stride=s, padding=p)
    dy = torch.randn_like(ref).bfloat16().float()
    ref.backward(dy)
    dx = fn.conv2d_dgrad(nhwc(dy).bfloat16(), w, x.shape[2:], stride=s, padding=p, cfg=cfg)
    assert rel(nchw(dx), x.grad) < 5e-3
