"""Micro-benchmark of the fused BN tails (forward, backward reduce+apply) on Model A / C shapes: cost of
re-reducing the NREP statistic replicas in every block vs reading finalized statistics, and the effect
of the grid size.  Graph-timed (no host overhead)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.ops.hip import lib  # noqa: E402

NREP = 32
SHAPES = {  # name: (M, C)
    "A_l1_33x83x16": (32 * 33 * 83, 16),
    "A_l1_33x83x32": (32 * 33 * 83, 32),
    "A_l2_17x42x64": (32 * 17 * 42, 64),
    "A_l4_5x11x256": (32 * 5 * 11, 256),
    "C_stem_47x122x64": (32 * 47 * 122, 64),
    "C_5x_10x28x64": (32 * 10 * 28, 64),
    "C_6x_4x13x192": (32 * 4 * 13, 192),
    "C_7x_1x6x384": (32 * 1 * 6, 384),
}


def timeit(f, reps=20, inner=20):
    f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(inner):
            f()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (reps * inner) * 1e3


def blocks(M, C, cap=1024, per_thread=2):
    cg = max(1, C // 8)
    pl = max(1, 256 // cg)
    return int(max(1, min(cap, math.ceil(M / (pl * per_thread)))))


def main():
    L = lib()
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    for name, (M, C) in SHAPES.items():
        y = (torch.randn(M, C, device="cuda")).bfloat16()
        out = torch.empty_like(y)
        stats = torch.rand(NREP, 2, C, device="cuda", dtype=torch.float64) * 10
        fin = torch.rand(4, C, device="cuda")
        gam, bet = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        nbt = torch.zeros(1, dtype=torch.int64, device="cuda")
        g = torch.randn(M, C, device="cuda", dtype=torch.bfloat16)
        dy = torch.empty_like(y)
        from mtl_das_pytorch_amd.ops.functional import bnb_plan
        nchunk, chunk_px = bnb_plan(M, C)
        part = torch.empty(nchunk, 3, C, device="cuda")
        dgam, dbet = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")

        def bn(with_fin):
            d = {"stats": stats.data_ptr(), "gamma": gam.data_ptr(), "beta": bet.data_ptr(), "run_mean": rm.data_ptr(),
                 "run_var": rv.data_ptr(), "nbt": nbt.data_ptr(), "pstride": 0, "C": C, "count": M, "eps": 1e-5,
                 "momentum": 0.1, "training": 1}
            if with_fin:
                d.update(fin=fin.data_ptr(), cnt=cnt.data_ptr())
            return d

        cnt = torch.zeros(2, dtype=torch.int32, device="cuda")
        r = {}
        for pt in (2,):
            nb = blocks(M, C, per_thread=pt)
            for wf in (0,):
                d = {"y": y.data_ptr(), "ygs": 0, "ldy": C, "bn": bn(wf), "out": out.data_ptr(), "ogs": 0, "ldo": C,
                     "B": 1, "H": M, "W": 1, "C": C}
                r[f"fwd_pt{pt}_fin{wf}"] = timeit(lambda: L.tail_fwd(1, 1, nb, torch.cuda.current_stream().cuda_stream, d))
                db = {"y": y.data_ptr(), "ygs": 0, "ldy": C, "bn": bn(wf), "B": 1, "H": M, "W": 1, "C": C,
                      "g": [(g.data_ptr(), 0, C)], "part": part.data_ptr(), "chunk_px": chunk_px, "dy": dy.data_ptr(), "dgs": 0, "ldd": C,
                      "dgamma": dgam.data_ptr(), "dbeta": dbet.data_ptr(), "pgs": 0}
                r[f"bwd_pt{pt}_fin{wf}"] = timeit(lambda: L.tail_bwd(1, 1, nchunk, torch.cuda.current_stream().cuda_stream, db))
                if pt == 2 and wf == 0 and M <= 4096:
                    dbf = dict(db, fused=1)
                    r["bwd_fused"] = timeit(lambda: L.tail_bwd(1, 1, nb, torch.cuda.current_stream().cuda_stream, dbf))
            r[f"blocks_pt{pt}"] = nb
        res[name] = r
        print(name, {k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}, flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/bench_tails.json", "w"), indent=1)


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def phases():
    """Phase breakdown of the single-launch BN backward (block 0's timestamps, wall_clock64 = 100 MHz)."""
    L = lib()
    for kind, (M, C) in [(1, (192, 384)), (1, (1664, 192)), (4, (1760, 128))]:
        y = torch.randn(M, C, device="cuda").bfloat16()
        r = torch.randn(M, C, device="cuda").bfloat16()
        stats = torch.rand(NREP, 2, C, device="cuda", dtype=torch.float64) * 10
        gam, bet = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        g = torch.randn(M, C, device="cuda", dtype=torch.bfloat16)
        dy, dy2 = torch.empty_like(y), torch.empty_like(y)
        dgam, dbet = torch.zeros(2, C, device="cuda"), torch.zeros(2, C, device="cuda")
        tsc = torch.zeros(8, dtype=torch.int64, device="cuda")
        bn = {"stats": stats.data_ptr(), "gamma": gam.data_ptr(), "beta": bet.data_ptr(), "run_mean": rm.data_ptr(),
              "run_var": rv.data_ptr(), "pstride": 0, "C": C, "count": M, "eps": 1e-5, "momentum": 0.1, "training": 1}
        d = {"y": y.data_ptr(), "ldy": C, "bn": bn, "B": 1, "H": M, "W": 1, "C": C, "g": [(g.data_ptr(), 0, C)],
             "dy": dy.data_ptr(), "ldd": C, "dgamma": dgam[0].data_ptr(), "dbeta": dbet[0].data_ptr(), "fused": 1,
             "tsc": tsc.data_ptr()}
        if kind == 4:
            d.update({"r": r.data_ptr(), "ldr": C, "bn2": bn, "dy2": dy2.data_ptr(), "ldd2": C,
                      "dgamma2": dgam[1].data_ptr(), "dbeta2": dbet[1].data_ptr()})
        for _ in range(3):
            L.tail_bwd(kind, 1, 1, torch.cuda.current_stream().cuda_stream, d)
            torch.cuda.synchronize()
        t = tsc.cpu().tolist()
        ph = [(t[i + 1] - t[i]) * 10 for i in range(5)]
        d2 = dict(d); d2.pop("tsc")
        tot = timeit(lambda: L.tail_bwd(kind, 1, 1, torch.cuda.current_stream().cuda_stream, d2))
        print(f"kind {kind} M={M} C={C}: graph-timed {tot:.1f} us; block-0 phases (ns): stats {ph[0]}, pass1 {ph[1]}, "
              f"wave-reduce {ph[2]}, coef {ph[3]}, pass2 {ph[4]}; block0 total {(t[5] - t[0]) * 10} ns", flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "phases":
    phases()
