#!/usr/bin/env python3
"""Two tuned tables on one program, in one process: builds the model's program the way bench.py does from each
table (engine/tune.py autotune_program, cached entries only), times the captured training step of each
(engine/tune.py step_time_us, interleaved rounds) and lists the launches whose kernel configuration differs.

    python tools/table_ab.py TABLE_A TABLE_B [--model MTL] [--rounds 3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.data.synthetic import generate  # noqa: E402
from mtl_das_pytorch_amd.engine.tune import autotune_program, load_cache, step_time_us  # noqa: E402
from mtl_das_pytorch_amd.models import build_model, encode_joint  # noqa: E402


def build(model: str, table: str):
    torch.manual_seed(0)
    m = build_model(model)
    if model == "multi_classifier":
        from mtl_das_pytorch_amd.engine.inception import InceptionProgram
        p = InceptionProgram(m, 32, "cuda")
    else:
        from mtl_das_pytorch_amd.engine.mtl import MTLProgram
        p = MTLProgram(m, 32, "cuda")
    p.set_optimizer(betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-5)
    p.segment_backward(1)
    cache = load_cache(table)
    n = len(cache)
    autotune_program(p, cache=cache, measure=True)
    return p, len(cache) - n


def listing(p):
    out = []
    for tag, ph in (("fwd", p.fwd_train), ("bwd", p.bwd)):
        for l in ph.launches:
            cfg = l.args[1] if l.name in ("conv_fwd", "conv_dgrad") else (
                l.args[0] if l.name == "wgrad_batched" else None)
            d = next((a for a in l.args if isinstance(a, dict)), {})
            shape = ",".join(str(d[k]) for k in ("Ho", "Wo", "N", "Cs", "KH", "KW", "H", "W", "C") if k in d)
            out.append((tag, l.stream, l.name, shape, cfg, d.get("fused")))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--model", default="MTL")
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    joint = args.model == "multi_classifier"
    X, d, e = generate(128, seed=3, device="cuda")
    labels = encode_joint(d, e) if joint else torch.stack([d, e], 1)
    progs = {}
    for k in ("a", "b"):
        progs[k], nmeas = build(args.model, getattr(args, k))
        print(f"table {k} = {getattr(args, k)}: {nmeas} entries measured (missing from the table)", flush=True)
    for r in range(args.rounds):
        ta = step_time_us(progs["a"], X, labels)
        tb = step_time_us(progs["b"], X, labels)
        print(f"round {r}: step a {ta:.1f} us, b {tb:.1f} us ({100 * (tb / ta - 1):+.1f} %)", flush=True)
    la, lb = listing(progs["a"]), listing(progs["b"])
    print(f"launches: a {len(la)}, b {len(lb)}")
    if len(la) == len(lb):
        for x, y in zip(la, lb):
            if x != y:
                print(f"  {x}\n  -> {y}")
    else:
        for name, L in (("a", la), ("b", lb)):
            print(f"--- {name}")
            for x in L:
                print("  ", x)


if __name__ == "__main__":
    main()
