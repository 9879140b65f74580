#!/usr/bin/env python3
"""Where the SyncBN all-reduces of a training step come from: builds the program as ``bench.py --sync_bn``
does (with a collective that is never executed) and lists every all-reduce launch -- phase, stream, element
count and the launch it follows -- with a per-kind summary.

    python tools/syncbn_breakdown.py [multi_classifier|MTL]
"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.engine.tune import autotune_program  # noqa: E402
from mtl_das_pytorch_amd.models import build_model  # noqa: E402


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "multi_classifier"
    torch.manual_seed(0)
    m = build_model(model)
    if model == "multi_classifier":
        from mtl_das_pytorch_amd.engine.inception import InceptionProgram
        p = InceptionProgram(m, 32, "cuda", sync_world=2)
    else:
        from mtl_das_pytorch_amd.engine.mtl import MTLProgram
        p = MTLProgram(m, 32, "cuda", sync_world=2)
    n = p.enable_sync_bn(lambda t: t)
    p.set_optimizer(weight_decay=1e-5, grad_scale=0.5, data_parallel=True)
    p.segment_backward(1)
    autotune_program(p, measure=False)
    kinds = collections.Counter()
    total = 0
    for tag, ph in (("fwd", p.fwd_train), ("bwd", p.bwd)):
        prev = None
        for l in ph.launches:
            if l.name == "allreduce_bn":
                t = l.args[1]
                t = t.t if hasattr(t, "bind") else t
                after = prev.name if prev is not None else "-"
                kind = f"{tag} after {after.split(':')[0] if not after.startswith('fork') else 'fork'}"
                kinds[kind] += 1
                total += 1
                print(f"{tag} s{l.stream} {t.numel():7d} fp64  after {after}")
            elif l.fn is not None:
                prev = l
    print(f"\n{model}: enable_sync_bn returned {n}; all-reduce launches in the step: {total}")
    for k, v in kinds.most_common():
        print(f"  {v:4d}  {k}")


if __name__ == "__main__":
    main()
