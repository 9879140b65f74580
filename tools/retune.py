"""Re-measure the per-layer kernel choices of every model at the benchmark batch and write the tuned table.

    python tools/retune.py [--batch 32] [--models MTL,single_event,single_distance,multi_classifier]
                           [--out gpurun_out/tuned_cfgs.json] [--keep [--drop wgrad,...]] [--wgrad-batches]
                           [--spill] [--in-context [--topk 3]]

Starts from an empty table (``--keep`` starts from the shipped one and only fills missing layers), tunes
every conv forward / data-gradient / weight-gradient launch and BN-backward variant of each model's
program by isolated timing (engine/tune.py autotune_phases); ``--wgrad-batches`` re-chooses the weight-
gradient configs of A and C by the time of the batched launches they run in (tune_wgrad_batches; Model B
shares A's backbone signatures and keeps A's choices); ``--wgrad-in-step`` then re-times the heaviest of them
in the captured step (tune_wgrad_in_step); ``--spill`` picks the weight-gradient spill fraction
of A and C in the captured step (tune_spill); ``--in-context`` then refines the conv choices by
timing the whole captured training step per candidate (engine/tune.py tune_in_context; the tuned set is kept
only if it beats the starting choices in interleaved re-timings).
Writes the merged table; copy it over mtl_das_pytorch_amd/engine/tuned_cfgs.json to ship it.
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.engine.inception import InceptionProgram  # noqa: E402
from mtl_das_pytorch_amd.engine.mtl import MTLProgram  # noqa: E402
from mtl_das_pytorch_amd.data.synthetic import generate  # noqa: E402
from mtl_das_pytorch_amd.engine.tune import (autotune_phases, autotune_program, conv_signature, load_cache,  # noqa: E402
                                             save_cache, tune_in_context, tune_spill, tune_wgrad_batches,
                                             tune_wgrad_in_step)
from mtl_das_pytorch_amd.ops.functional import CONV_XCD  # noqa: E402
from mtl_das_pytorch_amd.models import build_model, encode_joint  # noqa: E402


def _make(name: str, batch: int):
    torch.manual_seed(0)
    m = build_model(name)
    prog = InceptionProgram(m, batch, "cuda") if name == "multi_classifier" else MTLProgram(m, batch, "cuda")
    prog.set_optimizer(weight_decay=1e-5)
    return prog


def _warm_step(prog, name: str, batch: int):
    """One eager training step (learning rate 0) so that every operand the weight gradients read holds data."""
    X, d, e = generate(batch, seed=5, device="cuda")
    labels = encode_joint(d, e) if name == "multi_classifier" else torch.stack([d, e], 1)
    prog.opt["pack"].run()
    prog.arena.clear()
    prog.gather_phase(X, labels, torch.arange(batch, device="cuda")).run()
    prog.fwd_train.run()
    prog.bwd.run()
    torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--models", default="MTL,single_event,single_distance,multi_classifier")
    ap.add_argument("--out", default=os.path.join("gpurun_out", "tuned_cfgs.json"))
    ap.add_argument("--keep", action="store_true")
    ap.add_argument("--in-context", action="store_true")
    ap.add_argument("--topk", type=int, default=3)
    ap.add_argument("--in-context-models", default="MTL,multi_classifier",
                    help="models whose conv choices --in-context refines (Model B shares A's signatures)")
    ap.add_argument("--margin", type=float, default=0.002, help="in-context: relative step-time gain to keep a config")
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--drop", default="", help="with --keep: comma-separated key prefixes to re-measure (e.g. wgrad)")
    ap.add_argument("--wgrad-big-init", action="store_true",
                    help="--wgrad-batches starts from every im2col conv on its large tile")
    ap.add_argument("--wgrad-lean-init", default="",
                    help="--wgrad-batches starts from the convs of these streams (comma-separated, 'all': every "
                         "stream) on their fastest lean-staging config (36-43)")
    ap.add_argument("--wgrad-passes", type=int, default=2, help="--wgrad-batches: coordinate-descent passes")
    ap.add_argument("--wgrad-batches", action="store_true",
                    help="re-choose the weight-gradient configs by their batched launches' time (tune_wgrad_batches)")
    ap.add_argument("--wgrad-in-step", action="store_true",
                    help="then re-choose the heaviest weight-gradient configs by the captured step's time "
                         "(tune_wgrad_in_step; A and C)")
    ap.add_argument("--wgrad-top", type=int, default=10, help="--wgrad-in-step: signatures to re-time")
    ap.add_argument("--wgrad-topk", type=int, default=3,
                    help="--wgrad-in-step: candidates per signature from its isolated ranking (+ its large tile)")
    ap.add_argument("--spill", action="store_true",
                    help="choose the weight-gradient spill fraction in the step (tune_spill)")
    ap.add_argument("--passes", default="cfg,xcd,tail", help="in-context passes: conv configs, tile order, BN tails")
    ap.add_argument("--xcd-init", default="keep", choices=("keep", "on", "off"),
                    help="in-context: the tile order every conv signature of the model starts from")
    args = ap.parse_args()
    cache = load_cache() if args.keep else {}
    for pre in filter(None, args.drop.split(",")):
        for k in [k for k in cache if k.startswith(pre)]:
            del cache[k]
    for name in args.models.split(","):
        t0 = time.time()
        prog = _make(name, args.batch)
        n0 = len(cache)
        autotune_phases([prog.fwd_train, prog.fwd_eval, prog.bwd], cache, verbose=True, measure=True)
        print(f"{name}: {len(cache) - n0} new entries in {time.time() - t0:.1f} s", flush=True)
        if args.wgrad_batches and name in ("MTL", "multi_classifier"):
            _warm_step(prog, name, args.batch)
            tune_wgrad_batches(prog, cache, verbose=True, passes=args.wgrad_passes, init_big=args.wgrad_big_init,
                               init_lean=(True if args.wgrad_lean_init == "all" else
                                          {int(x) for x in args.wgrad_lean_init.split(",") if x}))
            print(f"{name}: weight-gradient batches tuned at {time.time() - t0:.1f} s", flush=True)
        if args.wgrad_in_step and name in ("MTL", "multi_classifier"):
            X, d, e = generate(4 * args.batch, seed=3, device="cuda")
            labels = encode_joint(d, e) if name == "multi_classifier" else torch.stack([d, e], 1)
            tune_wgrad_in_step(lambda: _make(name, args.batch), X, labels, cache, top=args.wgrad_top,
                               topk=args.wgrad_topk)
            save_cache(cache, args.out)
            print(f"{name}: weight gradients tuned in the step at {time.time() - t0:.1f} s", flush=True)
        if args.spill and name in ("MTL", "multi_classifier"):
            X, d, e = generate(4 * args.batch, seed=3, device="cuda")
            labels = encode_joint(d, e) if name == "multi_classifier" else torch.stack([d, e], 1)
            tune_spill(lambda: _make(name, args.batch), X, labels, cache)
        if args.in_context and name in args.in_context_models.split(","):
            autotune_program(prog, cache=cache, measure=False)  # batch the weight gradients as the bench does
            X, d, e = generate(4 * args.batch, seed=3, device="cuda")
            labels = encode_joint(d, e) if name == "multi_classifier" else torch.stack([d, e], 1)
            if args.xcd_init != "keep":
                for ph in (prog.fwd_train, prog.fwd_eval, prog.bwd):
                    for l in ph.launches:
                        if l.name in ("conv_fwd", "conv_dgrad"):
                            mode, cfg, G, d = l.args
                            cfg = (cfg | CONV_XCD) if args.xcd_init == "on" else (cfg & ~CONV_XCD)
                            cache[conv_signature(mode, G, d)] = cfg
                            l.args = (mode, cfg, G, d)
            ps = args.passes.split(",")
            tune_in_context(prog, X, labels, cache, topk=args.topk, margin=args.margin, reps=args.reps,
                            on_change=lambda c: save_cache(c, args.out),  # progress survives a crash
                            cfg_pass="cfg" in ps, xcd_pass="xcd" in ps, tail_pass="tail" in ps)
            print(f"{name}: in-context refinement done at {time.time() - t0:.1f} s", flush=True)
        del prog
        torch.cuda.empty_cache()
    save_cache(cache, args.out)
    print(f"wrote {len(cache)} entries to {args.out}")


if __name__ == "__main__":
    main()
