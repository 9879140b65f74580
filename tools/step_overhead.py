#!/usr/bin/env python3
"""What a training step costs around its graph: bench.py's loop (StepRunner.train_step: the batch-index copy
into the graph's index buffer, then the replay) against bare replays of the same captured step graph with
the index buffer left as it is, interleaved rounds, device-event timed.

    python tools/step_overhead.py [MTL|multi_classifier] [--steps 300]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.data.synthetic import generate  # noqa: E402
from mtl_das_pytorch_amd.engine.step import StepRunner  # noqa: E402
from mtl_das_pytorch_amd.engine.tune import autotune_program  # noqa: E402
from mtl_das_pytorch_amd.models import build_model, encode_joint  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("model", nargs="?", default="MTL")
    ap.add_argument("--steps", type=int, default=300)
    args = ap.parse_args()
    torch.manual_seed(1234)
    joint = args.model == "multi_classifier"
    m = build_model(args.model)
    if joint:
        from mtl_das_pytorch_amd.engine.inception import InceptionProgram
        p = InceptionProgram(m, 32, "cuda")
    else:
        from mtl_das_pytorch_amd.engine.mtl import MTLProgram
        p = MTLProgram(m, 32, "cuda")
    p.set_optimizer(weight_decay=1e-5)
    autotune_program(p, measure=False)
    X, d, e = generate(4096, seed=1, device="cuda")
    labels = encode_joint(d, e) if joint else torch.stack([d, e], 1)
    runner = StepRunner(p, X, labels, use_graph=True)
    runner.set_lr(1e-3)
    perm = torch.randperm(4096, device="cuda")
    batches = [perm[i * 32:(i + 1) * 32] for i in range(4096 // 32)]
    for i in range(20):
        runner.train_step(batches[i % len(batches)])
    torch.cuda.synchronize()

    def timed(fn) -> float:
        s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for i in range(args.steps):
            fn(i)
        t.record()
        torch.cuda.synchronize()
        return 1e3 * s.elapsed_time(t) / args.steps

    g = runner.graphs["train_full"]
    res = {"train_step (index copy + replay)": [], "replay only": []}
    for _ in range(3):
        res["train_step (index copy + replay)"].append(timed(lambda i: runner.train_step(batches[i % len(batches)])))
        res["replay only"].append(timed(lambda i: g.replay()))
    for k, v in res.items():
        print(f"{args.model}: {k}: {' / '.join(f'{x:.1f}' for x in v)} us per step", flush=True)
    runner.close()


if __name__ == "__main__":
    main()
