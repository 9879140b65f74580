"""Time the synthetic generator: one HIP launch (csrc/synth.hip) vs the torch-op implementation."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.data.synthetic import generate  # noqa: E402

for n in (256, 2048, 8192):
    for be in ("hip", "torch"):
        generate(64, seed=0, device="cuda", backend=be)
        torch.cuda.synchronize()
        t = time.perf_counter()
        generate(n, seed=1, device="cuda", backend=be)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        print(f"n={n:5d} {be:5s}: {dt * 1e3:8.1f} ms ({n / dt:,.0f} samples/s)", flush=True)
