"""Isolated time of every valid weight-gradient config on Model A / C 3x3 stride-1 layer shapes (graph of
back-to-back replays, engine.tune._time), to compare the patch kernels (12-15) with the im2col tiles."""
import sys

import torch

sys.path.insert(0, ".")
from mtl_das_pytorch_amd.engine.tune import _time  # noqa: E402
from mtl_das_pytorch_amd.ops import functional as fn  # noqa: E402

# (B, H, W, Cin, Cout, padding): input H x W; "valid" (p 0) convs have a (H-2) x (W-2) output
SHAPES = [(32, 33, 83, 16, 16, 1), (32, 33, 83, 16, 32, 1), (32, 17, 42, 32, 32, 1), (32, 17, 42, 16, 32, 1),
          (32, 17, 42, 32, 64, 1), (32, 9, 21, 64, 64, 1), (32, 9, 21, 64, 128, 1), (32, 5, 11, 128, 128, 1),
          (32, 47, 122, 32, 64, 1), (32, 49, 124, 32, 32, 0), (32, 23, 60, 80, 192, 0), (32, 10, 28, 96, 96, 1),
          (32, 10, 28, 64, 96, 1)]


def main():
    torch.manual_seed(0)
    for B, H, W, C, Co, p in SHAPES:
        x = torch.randn(B, H, W, C, device="cuda").bfloat16()
        dy = torch.randn(B, H + 2 * p - 2, W + 2 * p - 2, Co, device="cuda").bfloat16()
        res = []
        for cfg in sorted(fn.WGRAD_TILES) + sorted(fn.WGRAD_PATCH):
            try:
                call = fn.prepare_conv2d_wgrad(x, dy, (Co, C, 3, 3), 1, p, cfg=cfg)
            except ValueError:
                continue
            t = _time(lambda: fn.lib().wgrad(call.cfg, 1, torch.cuda.current_stream().cuda_stream, call.d))
            res.append((t * 1e3, cfg, call.d["splits"]))
        res.sort()
        print(f"{B}x{H}x{W} {C}->{Co} p{p}: " + "  ".join(f"c{c}:{t:.1f}us(s{s})" for t, c, s in res[:6]), flush=True)


if __name__ == "__main__":
    main()
