"""Reference-style eager PyTorch training step on one GPU (fp32, NCHW, torch.optim.Adam), i.e. what the
reference's train loop does per batch (utils.py:346-374 for Models A/B, 746-771 for Model C), for any
of the four model types.  Prints one JSON line; used as the like-for-like comparison for bench.py.

    python tools/eager_baseline.py --model multi_classifier --batch 32 --steps 30
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="MTL")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--cudnn-benchmark", action="store_true")
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32",
                    help="bf16: torch.autocast(bfloat16) around the forward (fp32 master weights, like the engine)")
    ap.add_argument("--no-miopen", action="store_true",
                    help="torch.backends.cudnn.enabled = False: PyTorch's own convolutions (im2col + rocBLAS GEMM) "
                         "instead of MIOpen -- the bf16 path that avoids the MIOpen fault of "
                         "profiles/r1_eager_reference_probe.log")
    args = ap.parse_args()
    import contextlib
    import torch
    import torch.nn.functional as F
    from mtl_das_pytorch_amd.models import build_model
    torch.backends.cudnn.benchmark = args.cudnn_benchmark
    torch.backends.cudnn.enabled = not args.no_miopen
    amp = (lambda: torch.autocast("cuda", dtype=torch.bfloat16)) if args.dtype == "bf16" else contextlib.nullcontext
    torch.manual_seed(0)
    model = build_model(args.model).cuda().train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-5)
    B = args.batch
    x = torch.randn(B, 1, 100, 250, device="cuda")
    d = torch.randint(0, 16, (B,), device="cuda")
    e = torch.randint(0, 2, (B,), device="cuda")

    def step():
        with amp():
            out = model(x)
            if args.model == "multi_classifier":
                loss = F.cross_entropy(out, d + 16 * e)
            elif args.model == "MTL":
                loss = F.nll_loss(out[0], d) + F.nll_loss(out[1], e)
            else:
                loss = F.nll_loss(out, d if args.model == "single_distance" else e)
        opt.zero_grad()
        loss.backward()
        opt.step()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / args.steps
    print(json.dumps({"model": args.model, "batch": B, "dtype": args.dtype, "ms_per_step": round(dt * 1e3, 3),
                      "samples_per_s": round(B / dt, 1), "cudnn_benchmark": args.cudnn_benchmark,
                      "miopen": not args.no_miopen}), flush=True)


if __name__ == "__main__":
    main()
