"""Probe one conv geometry across kernel configs and epilogue options (isolated graph-replay timing).

    python tools/conv_probe.py B H W Ci Co KH KW s p [--dgrad]

Prints, per config: plain, +fused BN sums (forward) / +fused BN-backward sums (dgrad), +normalise-on-load
(forward; training statistics from the replicas) and +normalise-on-load with eval statistics (no replica reduction), so fixed costs (BN-constant preparation, fp64 replica atomics) can be told apart from the
main loop.
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.engine.tune import CONV_CFGS, _time  # noqa: E402
from mtl_das_pytorch_amd.ops import functional as fn  # noqa: E402

NREP = 32


def main():
    ap = argparse.ArgumentParser()
    for k in ("B", "H", "W", "Ci", "Co", "KH", "KW", "s", "p"):
        ap.add_argument(k, type=int)
    ap.add_argument("--pw", type=int, default=None)
    ap.add_argument("--dgrad", action="store_true")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--cfgs", default="", help="comma-separated configs to run (default: every tuner config)")
    a = ap.parse_args()
    cfgs = [int(c) for c in a.cfgs.split(",")] if a.cfgs else CONV_CFGS
    pad = (a.p, a.p if a.pw is None else a.pw)
    dev = "cuda"
    g = torch.Generator().manual_seed(0)
    x = torch.randn(a.B, a.H, a.W, a.Ci, generator=g).bfloat16().to(dev)
    w = (torch.randn(a.Co, a.Ci, a.KH, a.KW, generator=g) / math.sqrt(a.Ci * a.KH * a.KW)).to(dev)
    Ho = (a.H + 2 * pad[0] - a.KH) // a.s + 1
    Wo = (a.W + 2 * pad[1] - a.KW) // a.s + 1
    stats = torch.zeros(NREP, 2, a.Co, device=dev, dtype=torch.float64)
    st_in = torch.rand(NREP, 2, a.Ci, device=dev, dtype=torch.float64)
    gam, bet = torch.ones(a.Ci, device=dev), torch.zeros(a.Ci, device=dev)
    rm, rv = torch.zeros(a.Ci, device=dev), torch.ones(a.Ci, device=dev)
    nbt = torch.zeros(1, device=dev, dtype=torch.int64)
    bn = fn.bn_args(st_in, gam, bet, rm, rv, nbt, a.B * a.H * a.W)
    dy = torch.randn(a.B, Ho, Wo, a.Co, generator=g).bfloat16().to(dev)
    yb = torch.randn(a.B, a.H, a.W, a.Ci, generator=g).bfloat16().to(dev)
    part = torch.zeros(NREP, 3, a.Ci, device=dev, dtype=torch.float64)
    res = []
    for c in cfgs:
        row = [c]
        variants = ([{}, {"bn_stats": (yb, bn, part, 1)}] if a.dgrad else
                    [{}, {"stats": stats}, {"stats": stats, "nol": (bn, 1)},
                     {"stats": stats, "nol": (dict(bn, training=0), 1)}])
        ok = True
        for kw in variants:
            try:
                if a.dgrad:
                    call = fn.prepare_conv2d_dgrad(dy, w, (a.H, a.W), stride=a.s, padding=pad, cfg=c, **kw)
                else:
                    call = fn.prepare_conv2d(x, w, None, stride=a.s, padding=pad, cfg=c, **kw)
                row.append(_time(call.run) * 1e3)
            except (ValueError, RuntimeError):  # a variant this config does not support (e.g. normalise-on-load by LDS-DMA)
                if len(row) == 1:
                    ok = False
                    break
                row.append(float("nan"))
        if ok:
            res.append(row)
    fl = 2 * a.B * Ho * Wo * a.Co * a.Ci * a.KH * a.KW
    print(f"M={a.B * Ho * Wo} N={a.Co if not a.dgrad else a.Ci} K={a.Ci * a.KH * a.KW if not a.dgrad else a.Co * a.KH * a.KW}"
          f" {fl / 1e9:.3f} GFLOP")
    hdr = ["cfg", "plain", "+bnb"] if a.dgrad else ["cfg", "plain", "+stats", "+nol", "+nol_ev"]
    print("  ".join(f"{h:>8s}" for h in hdr))
    for r in sorted(res, key=lambda r: r[1])[:a.top]:
        print("  ".join([f"{r[0]:8d}"] + [f"{v:8.2f}" for v in r[1:]]))


if __name__ == "__main__":
    main()
