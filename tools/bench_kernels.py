"""Micro-benchmark of the conv kernels on Model A's layer shapes (bs 32): every tile config, fwd with and
without the fused BN-statistics epilogue, dgrad and wgrad.  Interleaved repetitions in one process."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.ops import functional as fn  # noqa: E402
from mtl_das_pytorch_amd.ops.hip import lib, stream  # noqa: E402

B = 32
SHAPES = {  # name: (H, W, Ci, Co, k, s, p)
    "rb1_3x3_16_16": (33, 83, 16, 16, 3, 1, 1),
    "ol1_3x3_16_32": (33, 83, 16, 32, 3, 1, 1),
    "amg1_3x3_8_16": (33, 83, 8, 16, 3, 1, 1),
    "rb4_3x3_32_32": (17, 42, 32, 32, 3, 1, 1),
    "ol2_3x3_32_64": (17, 42, 32, 64, 3, 1, 1),
    "rb6_3x3_64_64": (9, 21, 64, 64, 3, 1, 1),
    "rb8_3x3_128": (5, 11, 128, 128, 3, 1, 1),
    "amg4_1x1_256_64": (5, 11, 256, 64, 1, 1, 0),
}


def timeit(f, reps=20, inner=20):
    """Per-launch device time from a HIP graph of ``inner`` back-to-back launches (no host overhead)."""
    f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(inner):
            f()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (reps * inner) * 1e3  # us


res = {}
for name, (H, W, Ci, Co, k, s, p) in SHAPES.items():
    x = torch.randn(B, H, W, Ci, device="cuda").bfloat16()
    w = torch.randn(Co, Ci, k, k, device="cuda") * 0.1
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = torch.randn(B, Ho, Wo, Co, device="cuda").bfloat16()
    stats = torch.zeros(32, 2, Co, device="cuda", dtype=torch.float64)
    r = {}
    for cfg in range(int(os.environ.get("NCFG", 5))):
        try:
            c0 = fn.prepare_conv2d(x, w, stride=s, padding=p, cfg=cfg)
            c1 = fn.prepare_conv2d(x, w, stride=s, padding=p, stats=stats, cfg=cfg)
            c2 = fn.prepare_conv2d_dgrad(dy, w, (H, W), stride=s, padding=p, cfg=cfg)
            r[f"fwd{cfg}"] = timeit(c0.run)
            r[f"fwd{cfg}_stats"] = timeit(c1.run)
            r[f"dgrad{cfg}"] = timeit(c2.run)
        except Exception as ex:  # noqa: BLE001
            r[f"cfg{cfg}"] = str(ex)[:80]
    for cfg in range(8):
        try:
            c3 = fn.prepare_conv2d_wgrad(x, dy, w.shape, stride=s, padding=p, cfg=cfg)
            r[f"wgrad{cfg}"] = timeit(lambda: lib().wgrad(c3.cfg, 1, stream(), c3.d))
        except Exception as ex:  # noqa: BLE001
            r[f"wg{cfg}"] = str(ex)[:80]
    flop = 2 * B * Ho * Wo * Co * Ci * k * k
    r["gflop"] = flop / 1e9
    res[name] = r
    print(name, json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/bench_kernels.json", "w"), indent=1)
