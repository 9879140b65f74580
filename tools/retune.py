"""Re-measure the per-layer kernel choices of every model at the benchmark batch and write the tuned table.

    python tools/retune.py [--batch 32] [--models MTL,single_event,single_distance,multi_classifier]
                           [--out gpurun_out/tuned_cfgs.json] [--keep]

Starts from an empty table (``--keep`` starts from the shipped one and only fills missing layers), tunes
every conv forward / data-gradient / weight-gradient launch and BN-backward variant of each model's
program (engine/tune.py), and writes the merged table.  Copy it over
mtl_das_pytorch_amd/engine/tuned_cfgs.json to ship it.
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.engine.inception import InceptionProgram  # noqa: E402
from mtl_das_pytorch_amd.engine.mtl import MTLProgram  # noqa: E402
from mtl_das_pytorch_amd.engine.tune import autotune_phases, load_cache, save_cache  # noqa: E402
from mtl_das_pytorch_amd.models import build_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--models", default="MTL,single_event,single_distance,multi_classifier")
    ap.add_argument("--out", default=os.path.join("gpurun_out", "tuned_cfgs.json"))
    ap.add_argument("--keep", action="store_true")
    args = ap.parse_args()
    cache = load_cache() if args.keep else {}
    for name in args.models.split(","):
        t0 = time.time()
        torch.manual_seed(0)
        m = build_model(name)
        prog = InceptionProgram(m, args.batch, "cuda") if name == "multi_classifier" else MTLProgram(m, args.batch, "cuda")
        n0 = len(cache)
        autotune_phases([prog.fwd_train, prog.fwd_eval, prog.bwd], cache, verbose=True, measure=True)
        print(f"{name}: {len(cache) - n0} new entries in {time.time() - t0:.1f} s", flush=True)
        del prog, m
        torch.cuda.empty_cache()
    save_cache(cache, args.out)
    print(f"wrote {len(cache)} entries to {args.out}")


if __name__ == "__main__":
    main()
