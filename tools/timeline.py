"""Profiler-free timeline of one training step replayed from a HIP graph.

rocprofv3's kernel tracing serialises the cross-stream edges of a captured multi-stream graph (tens of
microseconds of artificial gaps per edge), so it cannot show where a multi-stream step really spends its
time.  This tool inserts a one-thread ``tick`` kernel (csrc/misc.hip, stores the 100 MHz wall clock)
after every launch, on that launch's stream, captures the whole step into one graph, replays it, and
prints when each launch finished on its stream, and the time since the stream's previous tick (the
launch's duration plus one dependent-kernel boundary).  The ticks add ~1.5 us per launch to each stream,
so absolute times are inflated, but waits between streams and the relative cost of every launch in its
real concurrent context are visible.

    python tools/timeline.py [MTL|multi_classifier] [phases: fwd,bwd,adam]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.data.synthetic import generate  # noqa: E402
from mtl_das_pytorch_amd.engine.program import Launch  # noqa: E402
from mtl_das_pytorch_amd.engine.step import StateSnapshot, StepRunner, capture_graph  # noqa: E402
from mtl_das_pytorch_amd.engine.tune import autotune_program  # noqa: E402
from mtl_das_pytorch_amd.models import build_model, encode_joint  # noqa: E402
from mtl_das_pytorch_amd.ops.hip import lib  # noqa: E402


NSTAMP = 4096  # launches a timeline can stamp (the queue-id buffer has one slot per stamp)


def k_tick(buf, qbuf, i, st):
    lib().tick(buf, i, st, NSTAMP + 2, qbuf)


def shape_of(l):
    d = next((a for a in l.args if isinstance(a, dict)), {})
    keys = ("H", "W", "C", "Ho", "Wo", "N", "Cs", "KH", "KW")
    s = ",".join(f"{k}={d[k]}" for k in keys if k in d)
    if isinstance(d.get("g"), list):
        s += f",nsrc={len(d['g'])}"
    if "fused" in d:
        s += f",fused={d['fused']}"
    if "bnb" in d:
        s += ",bnstats"
    return s


def main():
    model_type = sys.argv[1] if len(sys.argv) > 1 else "MTL"
    torch.manual_seed(0)
    m = build_model(model_type)
    if model_type == "multi_classifier":
        from mtl_das_pytorch_amd.engine.inception import InceptionProgram
        p = InceptionProgram(m, 32, "cuda")
    else:
        from mtl_das_pytorch_amd.engine.mtl import MTLProgram
        p = MTLProgram(m, 32, "cuda")
    p.set_optimizer(weight_decay=1e-5)
    autotune_program(p, measure=False)
    X, d, e = generate(256, seed=1, device="cuda")
    lab = encode_joint(d, e) if model_type == "multi_classifier" else torch.stack([d, e], 1)
    idx = torch.arange(32, device="cuda")
    p.flat.lr.fill_(1e-3)
    p.opt["pack"].run()
    buf = torch.zeros(NSTAMP + 2, dtype=torch.int64, device="cuda")  # + 2 clock-calibration stamps
    qbuf = torch.zeros(NSTAMP, dtype=torch.int64, device="cuda")
    labels = []

    def instrument(ph, tag):
        new = []
        for l in ph.launches:
            new.append(l)
            if l.fn is None:
                continue
            labels.append((tag, l.name, l.stream, shape_of(l)))
            if len(labels) > NSTAMP:
                raise SystemExit(f"timeline: more than {NSTAMP} launches to stamp")
            new.append(Launch("tick", k_tick, buf.data_ptr(), qbuf.data_ptr(), len(labels) - 1, stream=l.stream))
        ph.launches = new

    gather = p.gather_phase(X, lab, idx)
    phases = [("gather", gather), ("fwd", p.fwd_train), ("bwd", p.bwd), ("adam", p.opt["adam"])]
    for tag, ph in phases:
        instrument(ph, tag)
    fns = [p.arena.clear] + [ph.run for _, ph in phases]
    f = p.flat
    snap = StateSnapshot([f.params, f.grads, f.exp_avg, f.exp_avg_sq, f.bn_mean, f.bn_var, f.bn_nbt, f.step])
    for fn in fns:
        fn()
    torch.cuda.synchronize()
    g, keep = capture_graph(fns)  # noqa: F841 (the events live as long as the graph)
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    snap.restore()
    # clock calibration
    st = torch.cuda.current_stream().cuda_stream
    lib().tick(buf.data_ptr(), NSTAMP, st, NSTAMP + 2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    time.sleep(0.2)
    lib().tick(buf.data_ptr(), NSTAMP + 1, st, NSTAMP + 2)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t = buf.cpu().tolist()
    mhz = (t[NSTAMP + 1] - t[NSTAMP]) / dt / 1e6
    n = len(labels)
    base = min(t[:n])
    us = [(t[i] - base) / mhz for i in range(n)]
    print(f"{model_type}: {n} launches, clock {mhz:.1f} MHz, last tick at {max(us):.1f} us")
    # the HSA queue each tick was dispatched from: how the graph executor mapped the captured (logical)
    # streams onto its own streams / hardware queues
    qids = {}
    tq = qbuf.cpu().tolist()
    q = [qids.setdefault(tq[i], len(qids)) for i in range(n)]
    per = {}
    for i in range(n):
        per.setdefault(labels[i][2], {}).setdefault(q[i], 0)
        per[labels[i][2]][q[i]] += 1
    print("queues per logical stream (queue: launches): " +
          "; ".join(f"s{s_}: " + ", ".join(f"q{k}:{v}" for k, v in sorted(d.items())) for s_, d in sorted(per.items())))
    last = {}
    order = sorted(range(n), key=lambda i: us[i])
    for i in order:
        tag, name, s, shp = labels[i]
        key = s
        prev = last.get(key, 0.0)
        last[key] = us[i]
        print(f"{us[i]:8.1f} s{s} q{q[i]} +{us[i] - prev:6.1f}  {tag:5s} {name:16s} {shp}")


if __name__ == "__main__":
    main()
