"""Functional (tensor-in / tensor-out) entry points to the HIP kernels.

These are the stand-alone versions of what the engine launches from prebuilt programs; they are used by
the kernel numerics tests and are convenient for experimentation.  All activations are NHWC
(``[B, H, W, C]``) on the GPU; weights use the reference PyTorch layout ``[Co, Ci, KH, KW]`` (fp32).
Every function requires a CUDA (ROCm) tensor and the built extension -- there is no silent fallback.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from .hip import lib, ptr, stream

NREP = 32  # must match csrc/common.h


def _pad(x, m):
    return (x + m - 1) // m * m


def _grad(g: torch.Tensor) -> torch.Tensor:
    """An activation gradient as the kernels read it: contiguous bf16 (csrc/common.h GradSrcs)."""
    if not g.is_cuda:
        raise RuntimeError("HIP ops need a GPU tensor")
    return g.to(torch.bfloat16).contiguous()


def _check(t: torch.Tensor, dtype=None):
    if not t.is_cuda:
        raise RuntimeError("HIP ops need a GPU tensor")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError("expected a contiguous tensor")


def pack_weight_fwd(w: torch.Tensor, cin_stored: Optional[int] = None) -> torch.Tensor:
    Co, Ci, KH, KW = w.shape
    Cs = cin_stored or Ci
    t = torch.zeros(Co, KH, KW, Cs, device=w.device)
    t[..., :Ci] = w.permute(0, 2, 3, 1)
    K = KH * KW * Cs
    out = torch.zeros(_pad(Co, 16), _pad(K, 32), device=w.device, dtype=torch.bfloat16)
    out[:Co, :K] = t.reshape(Co, K).to(torch.bfloat16)
    return out


def pack_weight_dgrad(w: torch.Tensor, cin_stored: Optional[int] = None) -> torch.Tensor:
    Co, Ci, KH, KW = w.shape
    Cs = cin_stored or Ci
    K = KH * KW * Co
    out = torch.zeros(_pad(Cs, 16), _pad(K, 32), device=w.device, dtype=torch.bfloat16)
    out[:Ci, :K] = w.permute(1, 2, 3, 0).reshape(Ci, K).to(torch.bfloat16)
    return out


def _geom(x_shape, w_shape, stride, padding):
    B, H, W, _ = x_shape
    Co, Ci, KH, KW = w_shape
    sh, sw = (stride, stride) if isinstance(stride, int) else stride
    ph, pw = (padding, padding) if isinstance(padding, int) else padding
    Ho = (H + 2 * ph - KH) // sh + 1
    Wo = (W + 2 * pw - KW) // sw + 1
    return B, H, W, Co, Ci, KH, KW, sh, sw, ph, pw, Ho, Wo


def _fwd_cfg(N, M):
    if N <= 16:
        return 0
    if N <= 32:
        return 1
    if N <= 64:
        return 2 if M >= 64 * 256 else 4
    return 3 if M >= 64 * 128 else 4


CONV_LDS_CFG0, CONV_LDS_NCFG = 16, 64  # csrc/kernels.h: LDS-staged conv configs (conv_lds.hip)
CONV_DEEP_CFG0, CONV_DEEP_NCFG = 128, 14  # conv_igemm tiles 0-13 at register-pipeline depth 4 (conv.hip)
LDS_TILES = [(64, 64), (128, 64), (64, 128), (128, 128), (32, 64), (64, 32), (32, 32), (128, 16)]
CONV_GLDS_CFG0, CONV_GLDS_NCFG = 160, 32  # LDS-DMA conv configs (conv_lds.hip conv_glds_kernel)
GLDS_TILES = [(64, 64), (128, 64), (64, 128), (128, 128), (256, 64), (128, 32), (256, 128), (64, 32)]
CONV_PATCH_CFG0, CONV_PATCH_NCFG = 192, 15  # 3x3 / stride-1 patch conv configs (conv_lds.hip conv_patch_kernel)
PATCH_TILES = [(256, 16), (256, 32), (256, 64), (128, 32), (128, 64)]  # strip capacity (pixels) x BN channels
PATCH_CB = [16, 32, 64]  # channel slice staged per pass
CONV_GDEEP_CFG0, CONV_GDEEP_NCFG = 208, 32  # LDS-DMA configs with a deep ring (up to 8 K chunks in flight)
CONV_PATCHP_CFG0, CONV_PATCHP_NCFG = 240, 15  # persistent, DMA-pipelined patch conv (one channel slice)
GDEEP_TILES = [0, 1, 2, 3, 5, 7]  # GLDS_TILES entries that have a deep ring (conv_lds.hip GL_NST_DEEP)
CONV_XCD = 4096  # flag on any conv config: XCD-contiguous tile order (csrc/common.h block_coords)


def lds_cfg(tile: int, kc: int = 64, splits: int = 1) -> int:
    """Config id of the LDS-staged conv kernel: tile index into LDS_TILES (BM pixels x BN channels), K chunk
    64 / 128, cross-block split of K into 1 / 2 / 4 / 8."""
    return CONV_LDS_CFG0 + 8 * tile + 4 * (kc == 128) + {1: 0, 2: 1, 4: 2, 8: 3}[splits]


def glds_cfg(tile: int, splits: int = 1, deep: bool = False) -> int:
    """Config id of the LDS-DMA conv kernel: tile index into GLDS_TILES (BM pixels x BN channels, K chunk 64,
    3-stage ring, or with ``deep`` the tile's deepest ring), cross-block split of K into 1 / 2 / 4 / 8."""
    return (CONV_GDEEP_CFG0 if deep else CONV_GLDS_CFG0) + 4 * tile + {1: 0, 2: 1, 4: 2, 8: 3}[splits]


def patch_cfg(tile: int, cb: int, persistent: bool = False) -> int:
    """Config id of the patch conv kernel: tile index into PATCH_TILES (a block owns R = BM // Wout whole
    output rows x BN channels), channel slice cb (16 / 32 / 64; Cs must be a multiple).  ``persistent``: the
    block loops over strips with the next one in flight by LDS-DMA (Cs == cb, no normalise-on-load)."""
    return (CONV_PATCHP_CFG0 if persistent else CONV_PATCH_CFG0) + 3 * tile + PATCH_CB.index(cb)


def conv_workspace(mode: int, cfg: int, G: int, d: dict, device) -> Optional[tuple]:
    """Attach the split-K workspace an LDS-staged conv config needs (fp32 partial tiles + zeroed arrival
    tickets) to the argument dict ``d``; returns the tensors to keep alive, or None when ``cfg`` cannot run
    these arguments."""
    if (cfg & ~CONV_XCD) < CONV_LDS_CFG0:
        return ()
    rc, ws, nt = lib().conv_workspace(mode, cfg, G, d)
    if rc != 0:
        return None
    if ws == 0:
        d.pop("ws", None)
        d.pop("cnt", None)
        return ()
    from ..engine import guard
    w = guard.alloc(ws, torch.float32, device, label=f"split-K workspace cfg {cfg}")
    c = guard.alloc(nt, torch.int32, device, zero=True, label=f"split-K tickets cfg {cfg}")
    d["ws"], d["cnt"] = w.data_ptr(), c.data_ptr()
    return (w, c)


class ConvCall:
    """A prepared convolution launch (packed weights + argument dict); ``run()`` enqueues it again."""

    def __init__(self, mode, cfg, d, out, keep):
        self.mode, self.cfg, self.d, self.out, self._keep = mode, cfg, d, out, keep
        ws = conv_workspace(mode, cfg, 1, d, out.device)
        if ws is None:
            raise ValueError(f"conv config {cfg} cannot run this geometry")
        self._ws = ws

    def run(self):
        lib().conv(self.mode, self.cfg, 1, stream(), self.d)
        return self.out


class WgradCall:
    def __init__(self, cfg, d, slab, post, keep):
        self.cfg, self.d, self.slab, self.post, self._keep = cfg, d, slab, post, keep

    def run(self):
        lib().wgrad(self.cfg, 1, stream(), self.d)
        return self.post(self.slab)


def prepare_conv2d(x, w, bias=None, stride=1, padding=0, stats=None, x2=None, cfg=None, nol=None) -> ConvCall:
    if stats is not None and stats.dtype != torch.float64:
        raise TypeError("BN statistic replicas are fp64 ([NREP, 2, Co])")
    _check(x, torch.bfloat16)
    C1 = x2.shape[-1] if x2 is not None else 0
    Cs = x.shape[-1] + C1
    B, H, W, Co, Ci, KH, KW, sh, sw, ph, pw, Ho, Wo = _geom(x.shape, w.shape, stride, padding)
    if Ci > Cs:
        raise ValueError("weight has more input channels than the input")
    wf = pack_weight_fwd(w.float(), Cs)
    from ..engine import guard
    y = guard.alloc((B, Ho, Wo, Co), torch.bfloat16, x.device, label=f"conv out cfg {cfg}")
    src = {"p0": ptr(x), "ld0": x.shape[-1], "C0": x.shape[-1], "C1": C1}
    if x2 is not None:
        _check(x2, torch.bfloat16)
        src.update({"p1": ptr(x2), "ld1": C1})
    d = {"src": src, "w": ptr(wf), "bias": ptr(bias) if bias is not None else 0, "out": ptr(y), "ldo": Co,
         "stats": ptr(stats) if stats is not None else 0, "B": B, "Hs": H, "Ws": W, "Ho": Ho, "Wo": Wo, "N": Co,
         "Npad": wf.shape[0], "Cs": Cs, "KH": KH, "KW": KW, "sh": sh, "sw": sw, "ph": ph, "pw": pw, "Kpad": wf.shape[1]}
    if nol is not None:  # (bn dict of x's BN, kind): x is a pre-BN y, the operand is act(BN(x)) on load
        d["nol"] = {"bn": nol[0], "kind": nol[1]}
    return ConvCall(0, _fwd_cfg(Co, B * Ho * Wo) if cfg is None else cfg, d, y, (x, x2, wf, bias, stats, nol))


def conv2d(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, stride=1, padding=0,
           stats: Optional[torch.Tensor] = None, x2: Optional[torch.Tensor] = None, cfg: Optional[int] = None,
           nol=None):
    """NHWC bf16 convolution.  ``x2`` (optional) is a second input whose channels are concatenated after
    ``x``'s (the kernel reads both without materialising the concat).  ``stats`` ([NREP, 2, Co] fp64,
    zero-initialised by the caller) receives per-channel sums of the output and its square.  ``nol``
    ((bn dict, kind)): normalise-on-load -- ``x`` is a pre-BN tensor and the conv input is act(BN(x))."""
    return prepare_conv2d(x, w, bias, stride, padding, stats, x2, cfg, nol).run()


def prepare_conv2d_dgrad(dy, w, in_hw, stride=1, padding=0, cin_stored=None, cfg=None, bn_stats=None) -> ConvCall:
    """``bn_stats`` (optional): ``(y, bn, part, kind)`` -- the dgrad output is the gradient of
    ``act(BN(y))`` and the epilogue accumulates that BN's backward sums sum(dz), sum(dz*xhat) into rows 0/1
    of ``part`` ([NREP, 3, C] fp64, zero-initialised); see :func:`bn_tail_backward` ``stats_done``."""
    _check(dy, torch.bfloat16)
    B, Ho, Wo, Co = dy.shape
    _, Ci, KH, KW = w.shape
    Cs = cin_stored or Ci
    H, W = in_hw
    sh, sw = (stride, stride) if isinstance(stride, int) else stride
    ph, pw = (padding, padding) if isinstance(padding, int) else padding
    wd = pack_weight_dgrad(w.float(), Cs)
    from ..engine import guard
    dx = guard.alloc((B, H, W, Cs), torch.bfloat16, dy.device, label=f"dgrad out cfg {cfg}")
    d = {"src": {"p0": ptr(dy), "ld0": Co, "C0": Co, "C1": 0}, "w": ptr(wd), "out": ptr(dx), "ldo": Cs,
         "B": B, "Hs": Ho, "Ws": Wo, "Ho": H, "Wo": W, "N": Cs, "Npad": wd.shape[0], "Cs": Co, "KH": KH, "KW": KW,
         "sh": sh, "sw": sw, "ph": ph, "pw": pw, "Kpad": wd.shape[1]}
    keep = (dy, wd)
    if bn_stats is not None:
        y, bn, part, kind = bn_stats
        _check(y, torch.bfloat16)
        if part.dtype != torch.float64 or tuple(y.shape) != (B, H, W, Cs):
            raise ValueError("bn_stats: y must be the [B, H, W, C] bf16 BN input and part fp64 [NREP, 3, C]")
        d["bnb"] = {"y": ptr(y), "ldy": Cs, "bn": bn, "part": ptr(part), "kind": kind}
        keep = keep + (y, part)
    return ConvCall(1, _fwd_cfg(Cs, B * H * W) if cfg is None else cfg, d, dx, keep)


def conv2d_dgrad(dy: torch.Tensor, w: torch.Tensor, in_hw: Tuple[int, int], stride=1, padding=0,
                 cin_stored: Optional[int] = None, cfg: Optional[int] = None, bn_stats=None):
    """Gradient w.r.t. the NHWC input: bf16 ``[B, H, W, Cin_stored]`` (fp32 accumulation, one rounding)."""
    return prepare_conv2d_dgrad(dy, w, in_hw, stride, padding, cin_stored, cfg, bn_stats).run()


WGRAD_TILES = {0: (16, 32, 128), 1: (32, 32, 128), 2: (32, 64, 64), 3: (64, 64, 64), 4: (16, 64, 128),
               5: (16, 32, 256), 6: (32, 32, 256), 7: (64, 32, 64),
               # whole-reduction tiles for small-Cout layers (csrc/conv.hip WGRAD_CFG_CASES)
               8: (16, 192, 64), 9: (16, 128, 64), 10: (32, 192, 64), 11: (32, 320, 32),  # (TN, TK, MCH)
               # large tiles on the 32x32x16 MFMA (csrc/conv.hip wgrad_big_block); their last K tile may be
               # partial
               32: (64, 64, 64), 33: (64, 128, 64), 34: (128, 64, 64), 35: (128, 128, 64),
               # lean-staging im2col tiles (csrc/wgrad_lean.hip: per-chunk pixel table in LDS, per-thread staging
               # constants, branch-free loads); partial last K tile
               36: (16, 64, 256), 37: (16, 144, 128), 38: (32, 64, 256), 39: (32, 144, 128), 40: (64, 64, 128),
               41: (64, 128, 128), 42: (128, 64, 128), 43: (128, 128, 64),
               # the same staging under the large tiles' 32x32x16 MFMA compute and M split (cfg 32-35 + 12)
               44: (64, 64, 64), 45: (64, 128, 64), 46: (128, 64, 64), 47: (128, 128, 64)}
WGRAD_BIG0 = 32
WGRAD_LEAN0, WGRAD_LEAN_N = 36, 8   # lean 16x16x32 configs (their own M split: engine/core.py wgrad_plan)
WGRAD_LEANBIG0 = 44                 # lean large tiles 44-47: WGRAD_BIG0 + i -> WGRAD_LEANBIG0 + i


def wgrad_ktiles(cfg: int, Kpad: int) -> int:
    """K tiles of an im2col weight-gradient config over a padded reduction of ``Kpad`` columns; 0 if the
    config cannot cover it (the small-tile kernels need TK | Kpad)."""
    TK = WGRAD_TILES[cfg][1]
    if cfg >= WGRAD_BIG0:
        return math.ceil(Kpad / TK)
    return 0 if Kpad % TK else Kpad // TK


# 3x3 / stride-1 patch kernels, padding 1 or 0 (csrc/conv.hip wgrad_patch_block):
# (TN, CB, max padded width, output rows per strip)
WGRAD_PATCH = {12: (16, 16, 88, 4), 13: (32, 16, 88, 4), 14: (32, 32, 48, 4), 15: (64, 32, 24, 4),
               16: (32, 32, 128, 2), 17: (64, 32, 128, 2), 18: (64, 16, 128, 2), 19: (32, 16, 128, 2)}


def patch_valid(cfg, Cs, KH, KW, stride, padding, Hi, Wi, Ho, Wo, C0=None, C1=0) -> bool:
    TN, CB, W8, R = WGRAD_PATCH[cfg]
    s = (stride, stride) if isinstance(stride, int) else tuple(stride)
    p = (padding, padding) if isinstance(padding, int) else tuple(padding)
    return ((KH, KW) == (3, 3) and s == (1, 1) and p[0] in (0, 1) and p[1] in (0, 1)
            and (Ho, Wo) == (Hi + 2 * p[0] - 2, Wi + 2 * p[1] - 2) and Cs % CB == 0
            and _pad(Wo, 8) <= W8 and (R * _pad(Wo, 8)) % 32 == 0 and (C1 == 0 or C0 % CB == 0))


def patch_plan(cfg, B, Ho, Npad, Cs, G=1, target=512):
    """(splits, units per split) of a patch wgrad: unit = (image, strip of R output rows).  (Capping the
    units per block at 3 to even out the blocks of a batched launch measured 4 % slower on Model A: the
    extra splits cost more slab traffic in the finalize than the shorter blocks saved.)"""
    TN, CB, _, R = WGRAD_PATCH[cfg]
    U = B * math.ceil(Ho / R)
    tiles = math.ceil(Npad / TN) * (Cs // CB) * G
    splits = max(1, min(U, math.ceil(target / tiles)))
    ups = math.ceil(U / splits)
    return math.ceil(U / ups), ups


def wgrad_cfg(Co: int, Kpad: int) -> int:
    return 0 if Co <= 16 else ((1 if Kpad <= 64 else 2) if Co <= 32 else 3)


def prepare_conv2d_wgrad(x, dy, w_shape, stride=1, padding=0, x2=None, splits=None, cfg=None, nol=None) -> WgradCall:
    _check(x, torch.bfloat16)
    _check(dy, torch.bfloat16)
    Co, Ci, KH, KW = w_shape
    C1 = x2.shape[-1] if x2 is not None else 0
    Cs = x.shape[-1] + C1
    B, H, W, _ = x.shape
    _, Ho, Wo, _ = dy.shape
    sh, sw = (stride, stride) if isinstance(stride, int) else stride
    ph, pw = (padding, padding) if isinstance(padding, int) else padding
    Kpad = _pad(KH * KW * Cs, 64)
    Npad = _pad(Co, 16)
    if cfg is None:
        cfg = wgrad_cfg(Co, Kpad)
    if cfg in WGRAD_PATCH:
        if not patch_valid(cfg, Cs, KH, KW, (sh, sw), (ph, pw), H, W, Ho, Wo, x.shape[-1], C1):
            raise ValueError(f"wgrad patch config {cfg} does not fit this convolution")
        splits, mps = patch_plan(cfg, B, Ho, Npad, Cs)
    else:
        TN, TK, MCH = WGRAD_TILES[cfg]
        if not wgrad_ktiles(cfg, Kpad):
            raise ValueError(f"wgrad config {cfg} (TK={TK}) does not tile the padded reduction {Kpad}")
        M = B * Ho * Wo
        tiles = math.ceil(Npad / TN) * wgrad_ktiles(cfg, Kpad)
        if splits is None:
            splits = max(1, min(math.ceil(M / MCH), math.ceil(512 / tiles)))
        mps = _pad(math.ceil(M / splits), MCH)
        splits = math.ceil(M / mps)
    from ..engine import guard
    slab = guard.alloc((1, splits, Npad, Kpad), torch.float32, x.device, label=f"wgrad slab cfg {cfg}")
    src = {"p0": ptr(x), "ld0": x.shape[-1], "C0": x.shape[-1], "C1": C1}
    if x2 is not None:
        src.update({"p1": ptr(x2), "ld1": C1})
    d = {"src": src, "dy": ptr(dy), "ldd": Co, "slab": ptr(slab), "splits": splits, "m_per_split": mps,
         "B": B, "Hi": H, "Wi": W, "Ho": Ho, "Wo": Wo, "Co": Co, "Npad": Npad, "Cs": Cs, "KH": KH, "KW": KW,
         "sh": sh, "sw": sw, "ph": ph, "pw": pw, "Kpad": Kpad}

    if nol is not None:  # (consts [1, 4, Cs] fp32: scale, shift, mean, invstd; kind)
        d["nol"] = {"consts": ptr(nol[0]), "kind": nol[1]}

    def post(sl):
        dWp = sl.sum(dim=1)[0, :Co, :KH * KW * Cs].view(Co, KH, KW, Cs)[..., :Ci]
        return dWp.permute(0, 3, 1, 2).contiguous()
    return WgradCall(cfg, d, slab, post, (x, x2, dy, nol))


def conv2d_wgrad(x: torch.Tensor, dy: torch.Tensor, w_shape, stride=1, padding=0, x2: Optional[torch.Tensor] = None,
                 splits: Optional[int] = None, cfg: Optional[int] = None, nol=None):
    """Weight gradient in the reference layout ``[Co, Ci, KH, KW]`` (fp32).  ``nol`` ((consts, kind)): ``x``
    is pre-BN and the operand is act(x * consts[0,0] + consts[0,1]), as in a normalise-on-load forward."""
    return prepare_conv2d_wgrad(x, dy, w_shape, stride, padding, x2, splits, cfg, nol).run()


# ---------------------------------------------------------------------------------------------------
ACT_NONE, ACT_RELU, ACT_SIGMOID, SIGMUL, ADD_RELU, POOL_RELU = range(6)


def bn_args(stats, gamma, beta, run_mean, run_var, nbt, count, eps=1e-5, momentum=0.1, training=True):
    """Kernel BN descriptor.  The dict keeps references to the tensors it points at (``_keep``) so that
    they cannot be freed while a launch may still use them."""
    if stats.dtype != torch.float64:
        raise TypeError("BN statistic replicas are fp64 ([NREP, 2, C])")
    return {"_keep": (stats, gamma, beta, run_mean, run_var, nbt),"stats": ptr(stats), "gamma": ptr(gamma), "beta": ptr(beta), "run_mean": ptr(run_mean),
            "run_var": ptr(run_var), "nbt": ptr(nbt) if nbt is not None else 0, "pstride": 0, "C": gamma.numel(),
            "count": count, "eps": eps, "momentum": momentum, "training": 1 if training else 0}


def bn_tail(kind: int, y: torch.Tensor, bn: dict, r: Optional[torch.Tensor] = None, bn2: Optional[dict] = None,
            blocks: int = 64):
    """Fused BN(+act/+mul/+residual/+pool) forward on NHWC bf16 ``y``; returns the bf16 output."""
    B, H, W, C = y.shape
    if kind == POOL_RELU:
        out = torch.empty(B, (H + 1) // 2, (W + 1) // 2, C, device=y.device, dtype=torch.bfloat16)
    else:
        out = torch.empty_like(y)
    d = {"y": ptr(y), "ldy": C, "bn": bn, "out": ptr(out), "ldo": C, "B": B, "H": H, "W": W, "C": C}
    if r is not None:
        d.update({"r": ptr(r), "ldr": r.shape[-1]})
    if bn2 is not None:
        d["bn2"] = bn2
    lib().tail_fwd(kind, 1, blocks, stream(), d)
    return out


def bnb_cgb(C: int) -> int:
    """Channel groups of 8 per block of the 2-D tiled BN backward (csrc/bn.hip bnb_cgb)."""
    cg = C // 8
    for g in (8, 4, 2):
        if cg % g == 0:
            return g
    return 1


def bnb_plan(M: int, C: int, G: int = 1, target_blocks: int = 1024):
    """Chunking of the 2-D tiled BN backward (csrc/bn.hip bnb_*): blocks of 256 threads cover 8*CGB
    channels x 256/CGB pixel lanes; chunks are sized so that chunks x channel blocks x G ~ target_blocks
    (at most 8 pixel steps per thread).  Returns (nchunk, pixels per chunk)."""
    cgb = bnb_cgb(C)
    pl = 256 // cgb
    steps = max(1, math.ceil(M / pl))
    cblocks = (C // (8 * cgb)) * G
    per = max(1, min(8, math.ceil(steps * cblocks / target_blocks)))
    chunk_px = pl * per
    return math.ceil(M / chunk_px), chunk_px


def bn_tail_backward(kind: int, y: torch.Tensor, bn: dict, grads: Sequence[torch.Tensor], dgamma, dbeta,
                     r: Optional[torch.Tensor] = None, bn2: Optional[dict] = None, dgamma2=None, dbeta2=None,
                     fused: bool = False, store_dz: bool = False, part: Optional[torch.Tensor] = None):
    """Returns ``(dy bf16, side bf16 | None, dy2 bf16 | None)``; writes dgamma/dbeta (and 2) in place.
    ``grads``: the upstream gradient sources (bf16, as the engine stores them; other dtypes are rounded);
    ``fused``: single-launch variant (block per 8 channels over all pixels) instead of reduce + apply;
    ``store_dz``: the reduce stores dz and the apply reads it instead of recomputing it;
    ``part``: the statistics were already accumulated (by a dgrad with ``bn_stats``): apply pass only."""
    B, H, W, C = y.shape
    nchunk, chunk_px = bnb_plan(B * H * W, C)
    mode = int(fused)
    if part is not None:
        mode = 2
    else:
        part = torch.zeros(NREP, 3, C, device=y.device, dtype=torch.float64)
    dy = torch.empty_like(y)
    grads = [_grad(g) for g in grads]
    d = {"y": ptr(y), "ldy": C, "bn": bn, "B": B, "H": H, "W": W, "C": C,
         "g": [(ptr(g), 0, g.shape[-1]) for g in grads], "part": ptr(part), "chunk_px": chunk_px,
         "dy": ptr(dy), "ldd": C, "dgamma": ptr(dgamma), "dbeta": ptr(dbeta), "fused": mode}
    dzbuf = None
    if store_dz:
        dzbuf = torch.empty(B, H, W, C, device=y.device, dtype=torch.bfloat16)
        d.update({"dzbuf": ptr(dzbuf), "lddz": C})
    side = dy2 = None
    if r is not None:
        d.update({"r": ptr(r), "ldr": r.shape[-1]})
    if kind in (SIGMUL,) or (kind == ADD_RELU and bn2 is None):
        side = torch.empty(B, H, W, C, device=y.device, dtype=torch.bfloat16)
        d.update({"side": ptr(side), "lds": C})
    if bn2 is not None:
        dy2 = torch.empty_like(y)
        d.update({"bn2": bn2, "dy2": ptr(dy2), "ldd2": C, "dgamma2": ptr(dgamma2),
                  "dbeta2": ptr(dbeta2)})
    lib().tail_bwd(kind, 1, nchunk, stream(), d)
    return dy, side, dy2


def pool3(x: torch.Tensor, is_max: bool, am: Optional[torch.Tensor] = None):
    """Inception pools on NHWC bf16: max 3x3/s2 (valid) or avg 3x3/s1/p1 (count_include_pad).  ``am``
    (max only, uint8 [B, Ho, Wo, C]): receives each output's window argmax for :func:`pool3_backward`."""
    B, H, W, C = x.shape
    Ho, Wo = ((H - 3) // 2 + 1, (W - 3) // 2 + 1) if is_max else (H, W)
    y = torch.empty(B, Ho, Wo, C, device=x.device, dtype=torch.bfloat16)
    d = {"x": ptr(x), "ldx": C, "y": ptr(y), "ldy": C, "B": B, "H": H, "W": W, "C": C, "Ho": Ho, "Wo": Wo}
    if am is not None:
        if am.dtype != torch.uint8 or am.numel() != B * Ho * Wo * C:
            raise ValueError("am must be uint8 with one entry per output element")
        d["am"] = ptr(am)
    lib().pool3(int(is_max), 0, stream(), d)
    return y


def pool3_backward(x: torch.Tensor, g: torch.Tensor, is_max: bool, am: Optional[torch.Tensor] = None):
    """Input gradient (bf16) of :func:`pool3` from the output gradient ``g`` (bf16; other dtypes are rounded)."""
    B, H, W, C = x.shape
    _, Ho, Wo, _ = g.shape
    g = _grad(g)
    dx = torch.empty(B, H, W, C, device=x.device, dtype=torch.bfloat16)
    d = {"x": ptr(x), "ldx": C, "g": ptr(g), "ldg": C, "dx": ptr(dx), "lddx": C, "B": B, "H": H, "W": W, "C": C,
         "Ho": Ho, "Wo": Wo}
    if am is not None:  # the kernel reads the argmax with 8-byte loads per 8-channel group
        if am.dtype != torch.uint8 or am.numel() != B * Ho * Wo * C or C % 8 or not is_max:
            raise ValueError("am must be the uint8 [B, Ho, Wo, C] argmax of a max pool with C % 8 == 0")
        d["am"] = ptr(am)
    lib().pool3(int(is_max), 1, stream(), d)
    return dx


def gather_batch(X: torch.Tensor, labels: torch.Tensor, idx: torch.Tensor):
    """HBM-resident dataset rows -> (bf16 NHWC batch with C padded to 8, labels)."""
    N, Cin, H, W = X.shape
    B = idx.numel()
    lw = labels.shape[1] if labels.dim() == 2 else 1
    out = torch.empty(B, H, W, 8, device=X.device, dtype=torch.bfloat16)
    lab = torch.empty(B, lw, device=X.device, dtype=torch.int64)
    lib().gather_batch(ptr(X), ptr(idx), ptr(labels), lw, ptr(out), ptr(lab), B, Cin, H, W, stream())
    return out, lab
