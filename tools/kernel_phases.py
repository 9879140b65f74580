#!/usr/bin/env python3
"""In-kernel phase timers of the critical-chain kernels, inside the captured training step.

Every conv_igemm launch (forward, normalise-on-load forward, data gradient with and without fused BN-backward
statistics), every forward BN tail and every apply pass of a BN-tail backward gets a per-block timer buffer
(``ptm``, csrc/common.h ``ptick``): thread 0 of each block stores the 100 MHz wall clock at kernel entry (0),
after the prologue (1: BN constants / replica reduction / k-group table, ``__syncthreads``), after the main
loop (2: the conv's K loop; tails have none) and at exit (3: epilogue stores + fp64 statistic atomics).  The
step is captured as one HIP graph and replayed; the last replay's stamps give, per launch:

  gap      first block's entry - previous launch's (on the same stream) last block's exit: dispatch latency
           of a dependent kernel inside the graph (barrier packet, end-of-kernel cache release, launch)
  ramp     last block's entry - first block's entry: how long the grid takes to get all its blocks started
  prolog   median block: entry -> prologue done
  main     median block: prologue -> K loop done (conv)
  epi      median block: K loop (tail: prologue) -> exit
  span     first entry -> last exit

and the same launch replayed ALONE (its own graph, 20 replays, same operands): the difference is what the
concurrent step does to it.

    python tools/kernel_phases.py [MTL|multi_classifier] [--all]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.data.synthetic import generate  # noqa: E402
from mtl_das_pytorch_amd.engine.step import StateSnapshot, capture_graph  # noqa: E402
from mtl_das_pytorch_amd.engine.tune import autotune_program  # noqa: E402
from mtl_das_pytorch_amd.models import build_model, encode_joint  # noqa: E402

PT_MAX_BLOCKS = 16384
TIMED = ("conv_fwd", "conv_dgrad")


def _dict_of(l):
    return next((a for a in l.args if isinstance(a, dict)), None)


def _shape(d):
    keys = ("Ho", "Wo", "H", "W", "N", "Cs", "C", "KH", "KW")
    s = ",".join(f"{k}={d[k]}" for k in keys if k in d)
    if "nol" in d and d["nol"]:
        s += ",nol"
    if "bnb" in d and d["bnb"]:
        s += ",bns"
    if "fused" in d:
        s += f",fused={d['fused']}"
    return s


def instrumentable(l) -> bool:
    d = _dict_of(l)
    if d is None or l.fn is None:
        return False
    if l.name in TIMED:
        return True
    if l.name.startswith("tail") and not l.name.startswith("tailbatch") and not l.name.startswith("tailbwd"):
        return True  # forward tails (tail_fwd_kernel)
    return l.name.startswith("tailbwd") and d.get("fused", 0) == 2  # apply-only backward (bnb_apply)


def phases_of(buf: torch.Tensor):
    t = buf.view(-1, 4).cpu()
    used = t[:, 0] != 0
    t = t[used].tolist()
    if not t:
        return None
    to_us = lambda x: x / 100.0  # noqa: E731  (100 MHz)
    start = min(r[0] for r in t)
    last_start = max(r[0] for r in t)
    end = max(max(r) for r in t)  # a kernel path without the exit stamp (e.g. an early return) ends at its last
    pro = [r[1] - r[0] for r in t if r[1]]
    main = [r[2] - r[1] for r in t if r[2] and r[1]]
    epi = [r[3] - (r[2] if r[2] else r[1]) for r in t if r[3] and r[1]]
    med = lambda v: to_us(statistics.median(v)) if v else 0.0  # noqa: E731
    return {"blocks": len(t), "start": start, "end": end, "ramp": to_us(last_start - start),
            "prolog": med(pro), "main": med(main), "epi": med(epi), "span": to_us(end - start)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("model", nargs="?", default="MTL")
    ap.add_argument("--all", action="store_true", help="print every stream, not only stream 0")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    torch.manual_seed(0)
    m = build_model(args.model)
    joint = args.model == "multi_classifier"
    if joint:
        from mtl_das_pytorch_amd.engine.inception import InceptionProgram
        p = InceptionProgram(m, 32, "cuda")
    else:
        from mtl_das_pytorch_amd.engine.mtl import MTLProgram
        p = MTLProgram(m, 32, "cuda")
    p.set_optimizer(weight_decay=1e-5)
    autotune_program(p, measure=False)
    X, d, e = generate(256, seed=1, device="cuda")
    lab = encode_joint(d, e) if joint else torch.stack([d, e], 1)
    idx = torch.arange(32, device="cuda")
    p.flat.lr.fill_(1e-3)
    p.opt["pack"].run()
    gather = p.gather_phase(X, lab, idx, clear=True)
    phases = [("fwd", p.fwd_train), ("bwd", p.bwd)]
    timed = []
    for tag, ph in phases:
        for i, l in enumerate(ph.launches):
            if instrumentable(l):
                buf = torch.zeros(PT_MAX_BLOCKS * 4, dtype=torch.int64, device="cuda")
                _dict_of(l)["ptm"] = buf.data_ptr()
                timed.append((tag, i, l, buf))
    fns = [gather.run, p.fwd_train.run, p.bwd.run, p.opt["adam"].run]
    f = p.flat
    snap = StateSnapshot([f.params, f.grads, f.exp_avg, f.exp_avg_sq, f.bn_mean, f.bn_var, f.bn_nbt, f.step,
                          p.metrics, p.confusion, p.logp] + list(getattr(p, "extra_state", [])))
    for fn in fns:
        fn()
    torch.cuda.synchronize()
    g, keep = capture_graph(fns)
    for _ in range(args.reps):
        g.replay()
    torch.cuda.synchronize()
    instep = [phases_of(buf) for _, _, _, buf in timed]
    # each launch alone: a graph of just that launch, same operands (state rolled back afterwards)
    alone = []
    for (tag, i, l, buf), ps in zip(timed, instep):
        buf.zero_()
        st = torch.cuda.current_stream().cuda_stream
        l(st)
        torch.cuda.synchronize()
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1):
            l(torch.cuda.current_stream().cuda_stream)
        for _ in range(args.reps):
            g1.replay()
        torch.cuda.synchronize()
        alone.append(phases_of(buf))
        g1.reset()
    snap.restore()
    g.reset()
    del g, keep
    print(f"{args.model}: {len(timed)} instrumented launches (us; 'alone' = the launch replayed by itself)")
    hdr = (f"{'phase':5s} s {'launch':12s} {'shape':44s} {'blk':>5s} {'gap':>6s} {'ramp':>5s} {'prolog':>6s} "
           f"{'main':>6s} {'epi':>6s} {'span':>6s} | {'alone: ramp':>11s} {'prolog':>6s} {'main':>6s} {'epi':>6s} {'span':>6s}")
    print(hdr)
    last_end = {}
    tot = {"gap": 0.0, "span": 0.0, "span_alone": 0.0, "prolog": 0.0, "main": 0.0, "epi": 0.0, "n": 0}
    for (tag, i, l, buf), ps, pa in zip(timed, instep, alone):
        if ps is None:
            continue
        key = (tag if tag == "fwd" else "bwd", l.stream)
        gap = (ps["start"] - last_end[key]) / 100.0 if key in last_end else float("nan")
        last_end[key] = ps["end"]
        if l.stream == 0:
            if gap == gap:
                tot["gap"] += gap
            tot["span"] += ps["span"]
            tot["prolog"] += ps["prolog"]
            tot["main"] += ps["main"]
            tot["epi"] += ps["epi"]
            tot["span_alone"] += pa["span"] if pa else 0.0
            tot["n"] += 1
        if l.stream != 0 and not args.all:
            continue
        a = pa or {"ramp": 0, "prolog": 0, "main": 0, "epi": 0, "span": 0}
        print(f"{tag:5s} {l.stream} {l.name:12s} {_shape(_dict_of(l))[:44]:44s} {ps['blocks']:5d} {gap:6.1f} "
              f"{ps['ramp']:5.1f} {ps['prolog']:6.2f} {ps['main']:6.2f} {ps['epi']:6.2f} {ps['span']:6.2f} | "
              f"{a['ramp']:11.1f} {a['prolog']:6.2f} {a['main']:6.2f} {a['epi']:6.2f} {a['span']:6.2f}")
    n = max(tot["n"], 1)
    print(f"stream 0, {tot['n']} timed launches: sum gap {tot['gap']:.1f} us, sum span {tot['span']:.1f} us "
          f"(alone {tot['span_alone']:.1f}); per launch: gap {tot['gap'] / n:.2f}, prolog {tot['prolog'] / n:.2f}, "
          f"main {tot['main'] / n:.2f}, epi {tot['epi'] / n:.2f}, span {tot['span'] / n:.2f} us")


if __name__ == "__main__":
    main()
