"""Worker of tests/test_rccl_gpu.py: the RCCL code path on ONE MI355X through a real 1-rank RCCL group.

Run with MDA_DIST_BACKEND=nccl and WORLD_SIZE unset/1: ``init_distributed`` then builds a 1-rank RCCL
communicator on cuda:0 (``torch.distributed`` backend "nccl" is RCCL on ROCm), so every collective below is
an actual RCCL launch on the GPU -- only its peer count is 1.  Checks, for the model given on the command
line (bench.py's flagship step at per-GPU batch 32, tuned kernel configs):

  dp         the DP step in both forms, against the same lowered program replayed as ONE graph without
             collectives -- bitwise equal after 3 steps (a 1-rank sum is exact), for 1 and 2 (A) / 4 (C) buckets:
             * captured (the 1-rank default, DistContext.capture_group): the buckets' all-reduces inside the
               step graph on the communication stream;
             * ext (the world > 1 default; ``FlatGradAllReducer.capturable = False`` here): forward + backward
               as ONE graph recording an external event per gradient bucket; after the replay is enqueued
               the communication stream waits for bucket k's event and issues its async RCCL all-reduce
               (``FlatGradAllReducer.start``), ``finish`` makes the compute stream wait (Work.wait), then
               the optimizer graph;
  syncbn     ``enable_sync_bn``: every BN's replica sums all-reduced by RCCL inside the step, CAPTURED in the
             step's HIP graph (no eager fallback on RCCL): graph == eager bitwise; after one step the BN running
             statistics equal plain BN's bitwise and the gradients agree to summation order;
  misc       ``barrier`` (device_ids form), metric reduction, BN-statistic averaging.

Prints one JSON line.
"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.data.synthetic import generate  # noqa: E402
from mtl_das_pytorch_amd.engine.backends import Metrics, reduce_metrics  # noqa: E402
from mtl_das_pytorch_amd.engine.inception import InceptionProgram  # noqa: E402
from mtl_das_pytorch_amd.engine.mtl import MTLProgram  # noqa: E402
from mtl_das_pytorch_amd.engine.step import StepRunner  # noqa: E402
from mtl_das_pytorch_amd.engine.tune import autotune_program  # noqa: E402
from mtl_das_pytorch_amd.models import build_model, encode_joint  # noqa: E402
from mtl_das_pytorch_amd.parallel.dist import FlatGradAllReducer, average_, init_distributed, shutdown  # noqa: E402

B = 32


def run(ctx, model_type, X, labels, *, buckets=1, dp=False, sync_bn=False, graph=True, steps=3, time_steps=0,
        capture_dp=True):
    torch.manual_seed(1234)
    m = build_model(model_type)
    joint = model_type == "multi_classifier"
    prog = (InceptionProgram(m, B, ctx.device) if joint else MTLProgram(m, B, ctx.device))
    n_ar = prog.enable_sync_bn(ctx.all_reduce_ordered_) if sync_bn else 0
    prog.set_optimizer(betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-5, grad_scale=1.0 / ctx.world,
                       data_parallel=dp)
    if joint:
        prog.set_rng_stream(0, ctx.rank)
    nb = len(prog.segment_backward(buckets))
    autotune_program(prog, measure=False)
    ar = FlatGradAllReducer(ctx) if dp else None
    if ar is not None and not capture_dp:
        # the multi-rank default (collectives not capturable): one forward + backward graph with an external
        # event per bucket, each bucket's RCCL all-reduce issued asynchronously behind its event
        ar.capturable = False
    runner = StepRunner(prog, X, labels, use_graph=graph, allreduce=ar)
    runner.set_lr(1e-3)
    for i in range(steps):
        runner.train_step(torch.arange(B * i, B * (i + 1), device=ctx.device) % X.shape[0])
    torch.cuda.synchronize()
    ms = None
    if time_steps:
        t0 = time.perf_counter()
        for i in range(time_steps):
            runner.train_step(torch.arange(B * i, B * (i + 1), device=ctx.device) % X.shape[0])
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / time_steps
    f = prog.flat
    state = {k: t.detach().clone() for k, t in (("params", f.params), ("grads", f.grads), ("exp_avg", f.exp_avg),
                                                ("exp_avg_sq", f.exp_avg_sq), ("bn_mean", f.bn_mean),
                                                ("bn_var", f.bn_var), ("step", f.step))}
    info = {"buckets": nb, "collectives_per_step": n_ar, "ms_per_step": ms, "graphs": sorted(runner.graphs),
            "captured_dp": runner.capture_dp, "ext_dp": runner.ext_dp}
    runner.close()
    return state, info


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def main():
    model_type = sys.argv[1] if len(sys.argv) > 1 else "MTL"
    ctx = init_distributed()
    out = {"model": model_type, "enabled": ctx.enabled, "backend": dist.get_backend() if dist.is_initialized() else None,
           "world": dist.get_world_size() if dist.is_initialized() else 0}
    X, d, e = generate(4 * B, seed=11, device=ctx.device)
    labels = encode_joint(d, e) if model_type == "multi_classifier" else torch.stack([d, e], 1)
    nbk = 4 if model_type == "multi_classifier" else 2
    for buckets in (1, nbk):
        ref, _ = run(ctx, model_type, X, labels, buckets=buckets, dp=False)
        got, info = run(ctx, model_type, X, labels, buckets=buckets, dp=True)
        out[f"dp{buckets}"] = dict(info, bitwise={k: bool(torch.equal(ref[k], got[k])) for k in ref})
        # the world > 1 default path on RCCL: one graph with external bucket events + async bucket all-reduces
        got, info = run(ctx, model_type, X, labels, buckets=buckets, dp=True, capture_dp=False)
        out[f"dp{buckets}_ext"] = dict(info, bitwise={k: bool(torch.equal(ref[k], got[k])) for k in ref})
    # SyncBN: collectives inside the step's graph
    eager, _ = run(ctx, model_type, X, labels, sync_bn=True, graph=False, steps=2)
    graph, info = run(ctx, model_type, X, labels, sync_bn=True, graph=True, steps=2)
    # one step: the forward (and so the BN running statistics) is bitwise the same with a 1-rank all-reduce;
    # the backward differs from plain BN only by the summation order of the reduce passes (the tails split
    # into reduce + all-reduce + apply instead of the tuned single-launch variants)
    sync1, _ = run(ctx, model_type, X, labels, sync_bn=True, graph=True, steps=1)
    plain, _ = run(ctx, model_type, X, labels, steps=1)
    _, tinfo = run(ctx, model_type, X, labels, sync_bn=True, graph=True, steps=2, time_steps=30)
    _, pinfo = run(ctx, model_type, X, labels, steps=2, time_steps=30)
    info["ms_per_step"] = tinfo["ms_per_step"]
    out["syncbn"] = dict(info, plain_ms_per_step=pinfo["ms_per_step"],
                         graph_eq_eager={k: bool(torch.equal(eager[k], graph[k])) for k in eager},
                         rel_vs_plain={k: rel(sync1[k], plain[k]) for k in ("params", "bn_mean", "bn_var", "grads")})
    # C3 / C4 / C5
    ctx.barrier()
    m = Metrics(["distance", "event"], [16, 2])
    m.loss[:] = [1.5, 2.5]
    m.correct[:] = [3, 4]
    m.count[:] = [8, 8]
    m.cm[0][1, 2] = 5
    r = reduce_metrics(ctx, m)
    t = torch.arange(6, dtype=torch.float32, device=ctx.device)
    average_(ctx, [t])
    out["misc"] = {"metrics_ok": bool(list(r.loss) == [1.5, 2.5] and int(r.cm[0][1, 2]) == 5),
                   "average_ok": bool(torch.equal(t, torch.arange(6, dtype=torch.float32, device=ctx.device)))}
    print(json.dumps(out), flush=True)
    shutdown(ctx)


if __name__ == "__main__":
    main()
