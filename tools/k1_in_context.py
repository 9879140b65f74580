#!/usr/bin/env python3
"""K1 decided in context: for each forward conv signature of Model A on the wide maps
(33x83 and 17x42, the layers the north star names for LDS-staged input tiles), the best isolated config of
EVERY kernel family -- register-direct implicit GEMM (conv_igemm, incl. the depth-4 pipeline), LDS-staged
im2col (conv_lds), LDS-DMA ring (conv_glds), patch conv (a strip with halo staged once per channel slice,
conv_patch / persistent conv_patchp), gdeep -- is put on every launch of that signature and the WHOLE
captured training step is timed (best of 3 x 15 replays, each candidate bracketed by the shipped table's
step time measured right before it).  Prints the per-family table: isolated launch time and the step-time
change against the shipped choice.

    python tools/k1_in_context.py [MTL] [--maps 33x83,17x42] [--reps 15]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.data.synthetic import generate  # noqa: E402
from mtl_das_pytorch_amd.engine.step import StateSnapshot, capture_graph  # noqa: E402
from mtl_das_pytorch_amd.engine.tune import _isolated, _set_conv_cfg, autotune_program, conv_signature  # noqa: E402
from mtl_das_pytorch_amd.models import build_model  # noqa: E402
from mtl_das_pytorch_amd.ops.functional import CONV_XCD  # noqa: E402

FAMILIES = [("igemm", lambda c: c < 16 or 128 <= c < 142), ("lds", lambda c: 16 <= c < 80),
            ("glds", lambda c: 160 <= c < 192), ("patch", lambda c: 192 <= c < 207),
            ("gdeep", lambda c: 208 <= c < 240), ("patchp", lambda c: 240 <= c < 255)]


def family(cfg: int) -> str:
    c = cfg & ~CONV_XCD
    return next((n for n, f in FAMILIES if f(c)), "?")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("model", nargs="?", default="MTL")
    ap.add_argument("--maps", default="33x83,17x42")
    ap.add_argument("--reps", type=int, default=15)
    args = ap.parse_args()
    maps = {tuple(int(v) for v in m.split("x")) for m in args.maps.split(",")}
    torch.manual_seed(0)
    from mtl_das_pytorch_amd.engine.mtl import MTLProgram
    p = MTLProgram(build_model(args.model), 32, "cuda")
    p.set_optimizer(weight_decay=1e-5)
    autotune_program(p, measure=False)
    X, d, e = generate(256, seed=1, device="cuda")
    lab = torch.stack([d, e], 1)
    idx = torch.arange(32, device="cuda")
    f = p.flat
    snap = StateSnapshot([f.params, f.grads, f.exp_avg, f.exp_avg_sq, f.bn_mean, f.bn_var, f.bn_nbt, f.step,
                          f.lr, p.metrics, p.confusion, p.logp])
    f.lr.zero_()
    p.opt["pack"].run()
    gather = p.gather_phase(X, lab, idx, clear=True)
    fns = [gather.run, p.fwd_train.run, p.bwd.run, p.opt["adam"].run]

    def step_us() -> float:
        for fn in fns:
            fn()
        torch.cuda.synchronize()
        g, keep = capture_graph(fns)
        g.replay()
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(3):
            s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.reps):
                g.replay()
            t.record()
            torch.cuda.synchronize()
            best = min(best, 1e3 * s.elapsed_time(t) / args.reps)
        g.reset()
        del g, keep
        return best

    groups = {}
    for l in p.fwd_train.launches:
        if l.name == "conv_fwd":
            mode, cfg, G, dd = l.args
            if (dd["Ho"], dd["Wo"]) in maps:
                groups.setdefault(conv_signature(mode, G, dd), []).append(l)
    keep = {}
    print(f"{args.model}: {len(groups)} forward conv signatures on {sorted(maps)}; step time of the shipped table "
          f"{step_us():.1f} us")
    print(f"{'layer (Ho x Wo, Cs -> N, KHxKW, nol)':42s} {'family':7s} {'cfg':>5s} {'isolated us':>11s} "
          f"{'step us':>8s} {'vs shipped':>10s}")
    for sig, ls in groups.items():
        mode, cur, G, dd = ls[0].args
        iso = _isolated(mode, G, dd, sig)
        best_of = {}
        for ms, c in iso:
            best_of.setdefault(family(c), (ms, c))
        layer = (f"{dd['Ho']}x{dd['Wo']}, {dd['Cs']}->{dd['N']}, {dd['KH']}x{dd['KW']}"
                 f"{', nol' if dd.get('nol') else ''}  x{len(ls)}")
        for fam, (ms, c) in sorted(best_of.items(), key=lambda kv: kv[1][0]):
            base = step_us()
            if not all(_set_conv_cfg(l, c, keep) for l in ls):
                for l in ls:
                    _set_conv_cfg(l, cur, keep)
                continue
            t = step_us()
            for l in ls:
                _set_conv_cfg(l, cur, keep)
            mark = " (shipped family)" if family(cur) == fam else ""
            print(f"{layer:42s} {fam:7s} {c:5d} {1e3 * ms:11.2f} {t:8.1f} {t - base:+10.1f}{mark}", flush=True)
    snap.restore()
    p.opt["pack"].run()


if __name__ == "__main__":
    main()
