#!/usr/bin/env python3
"""Cost of the graph-launch boundary between training steps: the captured step (gather, forward, backward,
Adam) replayed once per step, against K steps captured back to back into ONE graph and replayed once per K
steps (same operands; learning rate 0, state restored afterwards).

    python tools/multistep_graph.py [MTL|multi_classifier] [--k 1,2,4] [--reps 60]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.data.synthetic import generate  # noqa: E402
from mtl_das_pytorch_amd.engine.step import StateSnapshot, capture_graph  # noqa: E402
from mtl_das_pytorch_amd.engine.tune import autotune_program  # noqa: E402
from mtl_das_pytorch_amd.models import build_model, encode_joint  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("model", nargs="?", default="MTL")
    ap.add_argument("--k", default="1,2,4")
    ap.add_argument("--reps", type=int, default=60)
    args = ap.parse_args()
    torch.manual_seed(0)
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
    X, d, e = generate(128, seed=3, device="cuda")
    labels = encode_joint(d, e) if joint else torch.stack([d, e], 1)
    f = p.flat
    snap = StateSnapshot([f.params, f.grads, f.exp_avg, f.exp_avg_sq, f.bn_mean, f.bn_var, f.bn_nbt, f.step,
                          f.lr, p.metrics, p.confusion, p.logp] + list(getattr(p, "extra_state", [])))
    f.lr.zero_()
    p.opt["pack"].run()
    gather = p.gather_phase(X, labels, torch.arange(32, device="cuda"), clear=True)
    step = [gather.run, p.fwd_train.run, p.bwd.run, p.opt["adam"].run]
    for fn in step:
        fn()
    torch.cuda.synchronize()
    res = {}
    for _ in range(2):  # two interleaved rounds
        for k in [int(v) for v in args.k.split(",")]:
            g, keep = capture_graph(step * k)
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            n = max(1, args.reps // k)
            s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(n):
                g.replay()
            t.record()
            torch.cuda.synchronize()
            us = 1e3 * s.elapsed_time(t) / (n * k)
            res.setdefault(k, []).append(us)
            g.reset()
            del g, keep
    snap.restore()
    p.opt["pack"].run()
    base = min(res[min(res)])
    for k, v in sorted(res.items()):
        print(f"{args.model}: {k} step(s) per graph: {' / '.join(f'{x:.1f}' for x in v)} us per step "
              f"({100 * (min(v) / base - 1):+.1f} % vs {min(res)} per graph)", flush=True)


if __name__ == "__main__":
    main()
