#!/usr/bin/env python3
"""Headline benchmark: Model A (MTL_Net) training throughput, per-GPU batch 32, bf16, on N MI355X.

Metric (BASELINE.json): "samples/sec (whole node) MTL train bs=32 at 1/2/4/8 MI355X; event-cls accuracy".
One step = gather batch from an HBM-resident synthetic dataset -> forward -> backward -> (N>1: RCCL
all-reduce of the flat gradient bucket) -> fused Adam (+bf16 weight re-pack), i.e. the complete
reference training step (utils.py:346-374), nothing skipped.  Weights are random-init of the exact
reference architecture; data is synthetic DAS time-space matrices of the paper's shape (1x100x250).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

``--gpus N > 1`` without a launcher (no WORLD_SIZE in the environment) starts the N rank processes itself
(``_self_launch``: child processes, one per GPU, rendezvous on 127.0.0.1, before anything touches the GPU)
and exits with the first failing rank's status; under torchrun each process is one rank.

Weak scaling: per-GPU batch fixed at 32, global batch 32*N.  Rank 0 prints one JSON line; the time is
the max over ranks of K steps bracketed by barrier + device synchronize.

Without a GPU (CPU container, tests) the same contract runs the reference-math fp32 PyTorch step over gloo
(``_cpu_bench``): it checks the launch / rendezvous / one-JSON-line plumbing, not performance.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "samples/sec (whole node) MTL train bs=32 at 1/2/4/8 MI355X; event-cls accuracy"
# the only throughput number for this metric is the survey's CPU plumbing measurement of the
# reference (176.1 samples/s, Model A train step, bs 32).  The reference-style eager PyTorch step on one
# MI355X measured 4,037 samples/s (profiles/r1_eager_reference_probe.log) and is reported alongside.
BASELINE_VALUE = 176.1
EAGER_MI355X_PER_GPU = 4037.0
# reference-style eager fp32 PyTorch on one MI355X per model (docs/PERF.md headline table,
# profiles/r1_eager_reference_probe.log, profiles/r1_modelB_C_engine_vs_eager.log)
EAGER_BY_MODEL = {"MTL": EAGER_MI355X_PER_GPU, "single_event": 5292.0, "multi_classifier": 1876.0}
MODEL_NAMES = {"MTL": "modelA_MTL", "single_distance": "modelB_singleTask_distance",
               "single_event": "modelB_singleTask_event", "multi_classifier": "modelC_multiClassifier"}


def _accs(m, joint):
    """distance / event accuracy from the head's metric rows (Model C: decoded joint rows 1, 2)."""
    if joint:
        return {"distance": round(float(m[1, 1] / m[1, 2]), 4), "event": round(float(m[2, 1] / m[2, 2]), 4)}
    return {"distance": round(float(m[0, 1] / m[0, 2]), 4), "event": round(float(m[-1, 1] / m[-1, 2]), 4)}


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _self_launch(n: int) -> int:
    """Run this script as ``n`` rank processes (RANK = LOCAL_RANK = i, WORLD_SIZE = n, rendezvous on
    127.0.0.1) and return the first non-zero exit status (0 if every rank succeeded).  The parent never
    imports torch or touches the GPU: the ranks are fresh interpreters, not forks of a HIP process.  When a
    rank fails the others are terminated, so a dead peer cannot leave the rest waiting in a collective."""
    port = _free_port()
    procs = []
    for i in range(n):
        env = dict(os.environ, RANK=str(i), LOCAL_RANK=str(i), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc if rc >= 0 else 128 - rc


def _cpu_bench(args, ctx):
    """The bench contract without a GPU: the reference-math fp32 PyTorch training step (forward, the model's
    losses, backward, gradient all-reduce over gloo with 1/world averaging, torch Adam) on synthetic data,
    K timed steps, rank 0 prints one JSON line.  Plumbing only (multi-process launch, rendezvous, timing,
    the JSON contract): the numbers say nothing about MI355X."""
    import torch
    import torch.nn.functional as F
    from mtl_das_pytorch_amd.data.synthetic import generate
    from mtl_das_pytorch_amd.models import build_model, encode_joint
    from mtl_das_pytorch_amd.parallel.dist import FlatGradAllReducer, broadcast_module_state

    torch.set_num_threads(max(1, (os.cpu_count() or 1) // ctx.world))  # the ranks share the host's cores
    torch.manual_seed(1234)
    model = build_model(args.model, in_channels=args.in_channels)
    with torch.no_grad():
        broadcast_module_state(ctx, list(model.parameters()) + list(model.buffers()))
    opt = torch.optim.Adam(model.parameters(), lr=1e-3 / 1.5, weight_decay=1e-5)
    n = max(args.batch, min(args.dataset_size, 4 * args.batch))
    X, d, e = generate(n, seed=1000 + ctx.rank, in_channels=args.in_channels)
    joint = args.model == "multi_classifier"
    red = FlatGradAllReducer(ctx)
    g = torch.Generator().manual_seed(7 + ctx.rank)

    def step():
        idx = torch.randint(0, n, (args.batch,), generator=g)
        out = model(X[idx])
        if joint:
            loss = F.cross_entropy(out[0] if isinstance(out, tuple) else out, encode_joint(d[idx], e[idx]))
        elif args.model == "MTL":
            loss = F.nll_loss(out[0], d[idx]) + F.nll_loss(out[1], e[idx])
        else:
            loss = F.nll_loss(out, d[idx] if args.model == "single_distance" else e[idx])
        opt.zero_grad(set_to_none=False)
        loss.backward()
        params = [p for p in model.parameters() if p.grad is not None]
        flat = torch.cat([p.grad.reshape(-1) for p in params])
        red(flat)
        flat /= ctx.world
        o = 0
        for p in params:
            p.grad.copy_(flat[o:o + p.numel()].view_as(p))
            o += p.numel()
        opt.step()

    model.train()
    for _ in range(args.warmup):
        step()
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.barrier()
    dt = ctx.max_scalar(time.perf_counter() - t0)
    value = ctx.world * args.batch * args.steps / dt
    return {
        "metric": METRIC, "value": round(value, 2), "unit": "samples/s", "n_gpus": ctx.world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1e3 * dt / args.steps, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": round(value / BASELINE_VALUE, 3), "dtype": "fp32",
        "data": f"synthetic (DAS time-space matrices {args.in_channels}x100x250, random-init weights)",
        "config": {"model": MODEL_NAMES.get(args.model, args.model), "global_batch": args.batch * ctx.world,
                   "seq_len": 250, "input_shape": [args.in_channels, 100, 250], "parallelism": f"dp{ctx.world}"},
        "device": "cpu", "engine": "torch-eager fp32 (no GPU: launch / rendezvous plumbing only)",
        "dist_backend": ctx.backend,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32, help="per-GPU batch")
    ap.add_argument("--model", default="MTL", choices=["MTL", "single_distance", "single_event", "multi_classifier"])
    ap.add_argument("--dataset-size", type=int, default=2048, help="synthetic samples resident per GPU")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of one HIP graph per step")
    ap.add_argument("--buckets", type=int, default=None,
                    help="DP gradient buckets overlapped with the backward (default: the model's, 1 on one GPU)")
    ap.add_argument("--heldout", type=int, default=1024, help="held-out samples per GPU evaluated after timing")
    ap.add_argument("--no-tune", action="store_true", help="skip per-layer kernel autotuning (cached table only)")
    ap.add_argument("--in_channels", type=int, default=1,
                    help="input channels of the synthetic DAS matrices (reference 1; BASELINE north star 2)")
    ap.add_argument("--sync_bn", action="store_true",
                    help="SyncBN: BN statistics all-reduced inside the step (one GPU: run with MDA_DIST_BACKEND=nccl "
                         "for a 1-rank RCCL group, so the collectives execute)")
    ap.add_argument("--dp-shape", type=int, default=0,
                    help="rehearse the per-rank program of an N-GPU data-parallel run on this rank's group (run with "
                         "MDA_DIST_BACKEND=nccl for a 1-rank RCCL group): N's gradient buckets, updates only after "
                         "the all-reduce, and the world > 1 collective path (per-bucket piece graphs, async RCCL)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_self_launch(args.gpus))
    # HIP graph executor streams (read by the runtime when it initialises, i.e. before the first HIP call):
    # the engine's latency-bound steps run best on 2 (docs/PERF.md round 5); an explicit setting wins
    from mtl_das_pytorch_amd import use_engine_graph_queues
    graph_queues = use_engine_graph_queues()

    import torch
    import torch.distributed as dist
    from mtl_das_pytorch_amd.data.synthetic import generate
    from mtl_das_pytorch_amd.engine.inception import InceptionProgram
    from mtl_das_pytorch_amd.engine.mtl import MTLProgram
    from mtl_das_pytorch_amd.engine.lowering import build_for_stream_buckets
    from mtl_das_pytorch_amd.engine.step import StepRunner
    from mtl_das_pytorch_amd.engine.tune import autotune_program
    from mtl_das_pytorch_amd.models import build_model, encode_joint
    from mtl_das_pytorch_amd.parallel.dist import (FlatGradAllReducer, ShardedIndexSampler, broadcast_module_state,
                                                   calibrate_allreduce, init_distributed, shutdown)

    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws != args.gpus:  # fail before touching the GPU: a mislaunch would report the wrong n_gpus
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}; launch one rank per GPU with "
                 f"torch.distributed.run --nproc-per-node {args.gpus}")
    ctx = init_distributed()
    world = ctx.world
    dev = ctx.device
    if dev.type != "cuda":
        out = _cpu_bench(args, ctx)
        if ctx.is_main:
            print(json.dumps(out), flush=True)
        shutdown(ctx)
        return
    torch.manual_seed(1234)  # identical init on every rank (then broadcast for certainty)
    model = build_model(args.model, in_channels=args.in_channels)
    joint = args.model == "multi_classifier"
    sync = args.sync_bn and ctx.enabled
    sw = world if sync else 1
    n_sync = 0

    def make_prog(order=None):
        nonlocal n_sync
        p = (InceptionProgram(model, args.batch, dev, sync_world=sw, param_order=order) if joint
             else MTLProgram(model, args.batch, dev, sync_world=sw))
        if sync:  # the statistics collectives are captured into the step's HIP graph (RCCL)
            n_sync = p.enable_sync_bn(ctx.all_reduce_ordered_)
        p.set_optimizer(betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-5, grad_scale=1.0 / world,
                        data_parallel=ctx.enabled or args.dp_shape > 1)
        if hasattr(p, "set_rng_stream"):  # Model C dropout: an independent mask stream per rank
            p.set_rng_stream(0, ctx.rank)
        return p

    def tuned(p, n_seg):
        segs = p.segment_backward(n_seg)
        autotune_program(p, out_path=os.path.join("gpurun_out", "tuned_cfgs.json") if ctx.is_main else None,
                         measure=not args.no_tune)
        return p, segs

    prog = make_prog()
    # DP: gradient buckets whose all-reduces overlap the rest of the backward (engine/step.py), sized from the
    # all-reduce time of the whole flat gradient on the live group (a 1-rank rehearsal of N ranks, --dp-shape,
    # cannot measure N's all-reduce: it takes the model's default bucket count)
    # (--buckets K on one GPU runs the same bucketed graph with no-op collectives: measures the split's cost)
    shape = max(world, args.dp_shape)
    # the form the step's collectives take: captured in the step graph (one-rank groups; SyncBN, whose in-step
    # collectives are always captured where the group can -- the gradient buckets then share the capture
    # communicator), else eager behind the graph's external bucket events (the multi-rank default)
    captured = ctx.capturable_collectives and (sync or (ctx.capture_gradients and args.dp_shape <= 1))
    ar_ms = calibrate_allreduce(ctx, prog.flat.numel)
    nb = prog.dp_buckets(shape, ar_ms if world > 1 else None) if args.buckets is None else args.buckets
    # captured collectives: the backward cut at the bucket boundaries (segment_backward); eager RCCL behind the
    # graph's external events (the multi-rank default): buckets completed by side streams, no cut (stream_buckets)
    ext_form = not captured and (ctx.enabled or nb > 1)
    if ext_form and nb > 1:
        # side-stream buckets; Model C is rebuilt with its side streams' parameters grouped (stream_param_order)
        first = [prog]
        del prog
        prog, buckets = build_for_stream_buckets(lambda order: tuned(first.pop() if (order is None and first)
                                                                     else make_prog(order), 1)[0], nb)
    else:
        prog, buckets = tuned(prog, 1 if ext_form else nb)
    f = prog.flat
    broadcast_module_state(ctx, [f.params, f.bn_mean, f.bn_var, f.bn_nbt])
    X, d, e = generate(args.dataset_size, seed=1000 + ctx.rank, device=dev, in_channels=args.in_channels)
    labels = encode_joint(d, e) if joint else torch.stack([d, e], 1)
    reducer = FlatGradAllReducer(ctx, capture=captured) if (ctx.enabled or len(buckets) > 1) else None
    runner = StepRunner(prog, X, labels, use_graph=not args.no_graph and (not sync or captured), allreduce=reducer)
    runner.set_lr(1e-3 / 1.5)  # reference: lr/1.5 applied at the epoch-0 validation
    sampler = ShardedIndexSampler(args.dataset_size * world, args.batch, ctx, seed=7)
    # indices address this rank's resident shard
    batches = [b % args.dataset_size for b in sampler.epoch(0, dev)]

    # the epoch's batch indices stay on the device: each step's gather reads the next row of the schedule
    # (StepRunner.set_index_schedule), no host-issued index copy before a replay
    runner.set_index_schedule(torch.stack(batches))

    def step(i):
        runner.train_step()

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    runner.reset_metrics()
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    ctx.barrier()
    dt = time.perf_counter() - t0
    dt = ctx.max_scalar(dt)
    m = prog.metrics.clone()
    ctx.all_reduce_(m)
    # after the timed region: held-out accuracy of the model the timed steps produced (the metric's
    # "event-cls accuracy" half) on samples no rank trained on, BN in eval mode (running statistics)
    mh = None
    if args.heldout >= args.batch:
        Xh, dh, eh = generate(args.heldout, seed=500000 + ctx.rank, device=dev, in_channels=args.in_channels)
        runner.set_eval_source(Xh, encode_joint(dh, eh) if joint else torch.stack([dh, eh], 1))
        runner.reset_metrics()
        for i in range(0, args.heldout - args.batch + 1, args.batch):
            runner.eval_step(torch.arange(i, i + args.batch, device=dev))
        mh = prog.metrics.clone()
        ctx.all_reduce_(mh)
    value = world * args.batch * args.steps / dt
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * dt / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / BASELINE_VALUE, 3),
        "dtype": "bf16",
        "data": f"synthetic (DAS time-space matrices {args.in_channels}x100x250 from the on-device generator, "
                "HBM-resident, random-init weights)",
        "config": {"model": MODEL_NAMES.get(args.model, args.model),
                   "global_batch": args.batch * world, "seq_len": 250, "input_shape": [args.in_channels, 100, 250],
                   "parallelism": f"dp{world}"},
        "train_acc_timed_steps": _accs(m, joint),
        "heldout_acc_after_timed_steps": _accs(mh, joint) if mh is not None else None,
        "heldout_note": "held-out accuracy after only warmup + timed steps of training (near initialisation), "
                        "not a converged accuracy; converged numbers: docs/ACCURACY.md",
        "heldout_samples": (args.heldout // args.batch) * args.batch * world,
        "train_steps_before_heldout": args.warmup + args.steps,
        "vs_eager_pytorch_mi355x": (round(value / (EAGER_BY_MODEL[args.model] * world), 3)
                                    if args.model in EAGER_BY_MODEL else None),
        "hip_graph": runner.use_graph,
        "hip_graph_executor_streams": int(graph_queues),  # DEBUG_HIP_FORCE_GRAPH_QUEUES in effect at HIP init
        "sync_bn": sync,
        "sync_bn_collectives_per_step": n_sync if sync else 0,
        "grad_buckets_mb": [round((hi - lo) * 4 / 2 ** 20, 2) for lo, hi in buckets],
        "dist_backend": ctx.backend,
        "dp_shape": shape,
        "captured_collectives": runner.capture_dp,
        # how the bucket all-reduces overlap the backward: captured in the step graph, or eager RCCL behind the
        # graph's external bucket events (the multi-rank default)
        "dp_overlap": "captured" if runner.capture_dp else ("ext_events" if runner.ext_dp else None),
        "allreduce_ms": None if ar_ms is None else round(ar_ms, 4),
        "rccl_ranks": dist.get_world_size() if ctx.backend == "nccl" else 0,
        "baseline_note": "vs_baseline divides by BASELINE.md's 176.1 samples/s (reference on CPU, the only "
                         "throughput number it has); vs_eager_pytorch_mi355x divides by the reference-style "
                         "eager fp32 PyTorch step of the same model measured on MI355X (A: 4037 samples/s/GPU)",
    }
    if ctx.is_main:
        print(json.dumps(out), flush=True)
    runner.close()  # graphs, streams and events released while the HIP runtime is alive
    shutdown(ctx)


if __name__ == "__main__":
    main()
