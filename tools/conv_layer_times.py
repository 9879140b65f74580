"""Isolated device time of every conv launch (forward / data gradient / weight gradient) of a lowered
program at its tuned configuration, with the layer's implicit-GEMM shape and achieved TFLOP/s.

    python tools/conv_layer_times.py [MTL|multi_classifier] [--batch 32] [--top 40] [--json out.json]

Each launch is timed from a HIP graph of back-to-back launches (engine/tune.py _time), so the number is
the kernel's own latency/throughput with no neighbours on other streams.  Used to rank the layers whose
kernels deserve work and to build the roofline table in docs/PERF.md.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.engine.inception import InceptionProgram  # noqa: E402
from mtl_das_pytorch_amd.engine.mtl import MTLProgram  # noqa: E402
from mtl_das_pytorch_amd.engine.tune import _time, autotune_program  # noqa: E402
from mtl_das_pytorch_amd.models import build_model  # noqa: E402
from mtl_das_pytorch_amd.ops.hip import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("model", nargs="?", default="multi_classifier")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    torch.manual_seed(0)
    m = build_model(args.model)
    prog = InceptionProgram(m, args.batch, "cuda") if args.model == "multi_classifier" else MTLProgram(m, args.batch, "cuda")
    autotune_program(prog, measure=False, batch_wgrads=False)
    cs = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731 (the capture stream)
    L = lib()
    rows = []
    for ph in (prog.fwd_train, prog.bwd):
        for l in ph.launches:
            if l.name in ("conv_fwd", "conv_dgrad"):
                mode, cfg, G, d = l.args
                t = _time(lambda: L.conv(mode, cfg, G, cs(), d))
                M, N, K = d["B"] * d["Ho"] * d["Wo"], d["N"], d["KH"] * d["KW"] * d["Cs"]
                kind = "fwd" if mode == 0 else "dgrad"
            elif l.name == "conv_wgrad":
                cfg, G, d = l.args
                t = _time(lambda: L.wgrad(cfg, G, cs(), d))
                M, N, K = d["B"] * d["Ho"] * d["Wo"], d["Co"], d["KH"] * d["KW"] * d["Cs"]
                kind = "wgrad"
            else:
                continue
            fl = 2.0 * M * N * K * G
            rows.append({"kind": kind, "cfg": cfg, "G": G, "M": M, "N": N, "K": K, "KH": d["KH"], "KW": d["KW"],
                         "sh": d["sh"], "HWo": f"{d['Ho']}x{d['Wo']}", "us": t * 1e3, "gflop": fl / 1e9,
                         "tflops": fl / (t * 1e-3) / 1e12, "nol": bool(d.get("nol")), "bns": bool(d.get("bnb"))})
    tot = sum(r["us"] for r in rows)
    for k in ("fwd", "dgrad", "wgrad"):
        rk = [r for r in rows if r["kind"] == k]
        print(f"{k:6s} {len(rk):3d} launches {sum(r['us'] for r in rk):8.1f} us  "
              f"{sum(r['gflop'] for r in rk):7.2f} GFLOP")
    print(f"total  {tot:.1f} us (isolated sum)")
    print(f"{'kind':6s} {'cfg':>3s} {'G':>2s} {'out':>8s} {'k':>5s} {'s':>2s} {'M':>7s} {'N':>4s} {'K':>5s} "
          f"{'us':>7s} {'GF':>6s} {'TF/s':>6s}")
    for r in sorted(rows, key=lambda r: -r["us"])[:args.top]:
        print(f"{r['kind']:6s} {r['cfg']:3d} {r['G']:2d} {r['HWo']:>8s} {r['KH']}x{r['KW']:<3d} {r['sh']:2d} "
              f"{r['M']:7d} {r['N']:4d} {r['K']:5d} {r['us']:7.1f} {r['gflop']:6.2f} {r['tflops']:6.1f}"
              f"{' nol' if r['nol'] else ''}{' bns' if r['bns'] else ''}")
    if args.json:
        with open(args.json, "w") as f:
            json.dump(rows, f, indent=0)


if __name__ == "__main__":
    main()
