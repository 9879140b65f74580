"""Weight-gradient tile assignment policies, timed in the captured training step.

The autotuner picks a conv's weight-gradient config from its ISOLATED time, but every conv's weight
gradient runs inside a batched launch (one per stream and config) beside dozens of others: there the
aggregate bytes staged through LDS matter, not one job's latency, and the small tiles that win alone
(more blocks for one small conv) lose to the large 32x32x16 tiles (2-4x fewer staged bytes per output).
This tool applies a policy to every conv, merges / batches as the bench does, and reports the step time
(HIP graph replays) and the batched weight-gradient launches' isolated times.

    python tools/wgrad_assign.py [MTL|multi_classifier] [policy,...] [--min-px 256,512]

policies: table (the shipped table), big (every im2col conv on the large tile its Cout / reduction
suit; patch configs kept), bigall (patch configs replaced too).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.data.synthetic import generate  # noqa: E402
from mtl_das_pytorch_amd.engine.core import ConvLayer  # noqa: E402
from mtl_das_pytorch_amd.engine.tune import _time, autotune_program, step_time_us  # noqa: E402
from mtl_das_pytorch_amd.models import build_model, encode_joint  # noqa: E402
from mtl_das_pytorch_amd.ops.functional import WGRAD_BIG0, WGRAD_PATCH  # noqa: E402


def big_cfg(conv) -> int:
    """Large tile for a conv: 128 rows when Cout fills them, 128 columns when the reduction does."""
    return WGRAD_BIG0 + 2 * (conv.Npad > 64) + (conv.Kpad_w > 64)


def build(model_type: str, policy: str):
    torch.manual_seed(0)
    m = build_model(model_type)
    if model_type == "multi_classifier":
        from mtl_das_pytorch_amd.engine.inception import InceptionProgram
        p = InceptionProgram(m, 32, "cuda")
    else:
        from mtl_das_pytorch_amd.engine.mtl import MTLProgram
        p = MTLProgram(m, 32, "cuda")
    p.set_optimizer(betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-5)
    autotune_program(p, measure=False, batch_wgrads=False)
    if policy != "table":
        for l in p.bwd.launches:
            if l.name != "conv_wgrad":
                continue
            if policy == "big" and l.args[0] in WGRAD_PATCH:
                continue
            c = big_cfg(l.owner)
            if l.owner.wgrad_valid(c):
                l.owner.set_wgrad_cfg(c)
                l.args = (c,) + tuple(l.args[1:])
    p.merge_wgrad_cfgs()
    p.refresh_wgrad_finalize()
    p.batch_wgrads()
    return p


def measure(p, model_type: str, reps: int):
    X, d, e = generate(256, seed=1, device="cuda")
    lab = encode_joint(d, e) if model_type == "multi_classifier" else torch.stack([d, e], 1)
    step_us = step_time_us(p, X, lab, reps)
    batches = []  # operands hold the last replay's data
    for l in p.bwd.launches:
        if l.name in ("wgrad_batched", "wgrad_finalize"):
            t = _time(lambda l=l: l.fn(*l.args, torch.cuda.current_stream().cuda_stream))  # the capture stream
            batches.append((l.name, l.args[0] if l.name == "wgrad_batched" else -1, l.stream, 1e3 * t))
    return step_us, batches


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("model", nargs="?", default="multi_classifier")
    ap.add_argument("policies", nargs="?", default="table,big,bigall")
    ap.add_argument("--min-px", default="256")
    ap.add_argument("--reps", type=int, default=100)
    args = ap.parse_args()
    for mp in [int(x) for x in args.min_px.split(",")]:
        ConvLayer.MIN_SPLIT_PX_BIG = mp
        for pol in args.policies.split(","):
            p = build(args.model, pol)
            step_us, batches = measure(p, args.model, args.reps)
            wg = sum(t for n, _, _, t in batches if n == "wgrad_batched")
            fin = sum(t for n, _, _, t in batches if n == "wgrad_finalize")
            print(f"{args.model} policy {pol:7s} min_px {mp:5d}: step {step_us:8.1f} us  wgrad batches "
                  f"{wg:7.1f} us (sum of {sum(1 for b in batches if b[0] == 'wgrad_batched')})  finalize {fin:6.1f} us",
                  flush=True)
            for n, c, s, t in batches:
                print(f"    {n:15s} cfg {c:3d} stream {s}: {t:7.1f} us")
            del p
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
