"""Worker of tests/test_dp_engine_gpu.py: one rank of a 2-rank data-parallel engine job on ONE GPU.

Launched by torch.distributed.run with MDA_SINGLE_DEVICE=1 (every rank on cuda:0) and MDA_DIST_BACKEND=gloo
(RCCL refuses two ranks on one device): the exact engine DP path of bench.py / the trainer -- split
backward graphs per gradient bucket, asynchronous bucket all-reduces overlapping the next piece, 1/world
folded into the fused Adam -- with gloo carrying the collectives.  Per step it checks

  * the all-reduced gradient equals the sum of the two ranks' single-process engine gradients (each rank
    recomputes its gradient with an unsegmented, unreduced program from the same weights);
  * the fused Adam applied exactly that averaged gradient (reference Adam in fp64 from the saved state);
  * every rank holds bitwise-identical parameters and Adam moments afterwards.

Prints one JSON line per rank: {"rank", "steps", "max_grad_rel", "max_adam_abs", "buckets"}.
    python -m torch.distributed.run --nproc-per-node 2 ... tests/dp_engine_worker.py MODEL NBUCKETS
"""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.data.synthetic import generate  # noqa: E402
from mtl_das_pytorch_amd.engine.inception import InceptionProgram  # noqa: E402
from mtl_das_pytorch_amd.engine.mtl import MTLProgram  # noqa: E402
from mtl_das_pytorch_amd.engine.step import StepRunner  # noqa: E402
from mtl_das_pytorch_amd.engine.tune import autotune_program  # noqa: E402
from mtl_das_pytorch_amd.models import build_model, encode_joint  # noqa: E402
from mtl_das_pytorch_amd.parallel.dist import (FlatGradAllReducer, broadcast_module_state,  # noqa: E402
                                               init_distributed, shutdown)

WD, LR, B1, B2, EPS = 1e-5, 1e-3, 0.9, 0.999, 1e-8


def build(model_type, B, dev, nbuckets):
    torch.manual_seed(1234)
    m = build_model(model_type)
    joint = model_type == "multi_classifier"
    prog = InceptionProgram(m, B, dev) if joint else MTLProgram(m, B, dev)
    if joint:  # both programs of a rank draw this rank's dropout masks
        prog.set_rng_stream(0, int(os.environ.get("RANK", "0")))
    return prog, joint


def gather_cpu(t):
    """all_gather of a device tensor through gloo (on CPU copies)."""
    c = t.detach().cpu()
    out = [torch.empty_like(c) for _ in range(dist.get_world_size())]
    dist.all_gather(out, c)
    return out


def main():
    model_type, nbuckets = sys.argv[1], int(sys.argv[2])
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    # "stream": the multi-rank production form (uncut backward, side-stream buckets: stream_buckets);
    # "cut": segment_backward's cut backward
    form = sys.argv[4] if len(sys.argv) > 4 else "stream"
    ctx = init_distributed()
    world, dev = ctx.world, ctx.device
    B = 32
    prog, joint = build(model_type, B, dev, nbuckets)
    prog.set_optimizer(betas=(B1, B2), eps=EPS, weight_decay=WD, grad_scale=1.0 / world, data_parallel=True)
    buckets = prog.segment_backward(nbuckets if form == "cut" else 1)
    autotune_program(prog, measure=False)
    if form == "stream" and nbuckets > 1:
        buckets = prog.stream_buckets(nbuckets)
    f = prog.flat
    broadcast_module_state(ctx, [f.params, f.bn_mean, f.bn_var, f.bn_nbt])
    X, d, e = generate(4 * B, seed=100 + ctx.rank, device=dev)  # different data on every rank
    lab = encode_joint(d, e) if joint else torch.stack([d, e], 1)
    runner = StepRunner(prog, X, lab, use_graph=True, allreduce=FlatGradAllReducer(ctx))
    runner.set_lr(LR)
    # reference: the same network, one bucket, no collectives -- this rank's own gradient
    ref, _ = build(model_type, B, dev, 1)
    ref.set_optimizer(betas=(B1, B2), eps=EPS, weight_decay=WD)
    autotune_program(ref, measure=False)
    rrun = StepRunner(ref, X, lab, use_graph=True)
    worst_g, worst_a = 0.0, 0.0
    for s in range(steps):
        idx = (torch.arange(B, device=dev) + s * B) % X.shape[0]
        # this rank's single-process gradient at the current (shared) weights
        ref.flat.params.copy_(f.params)
        rrun.pack_weights()
        rrun.idx.copy_(idx)
        rrun._run("train_compute")
        torch.cuda.synchronize()
        g_sum = sum(gather_cpu(ref.flat.grads)).to(torch.float64)
        p0, m0, v0 = (t.detach().clone().double() for t in (f.params, f.exp_avg, f.exp_avg_sq))
        step0 = float(f.step.item())
        runner.train_step(idx)
        torch.cuda.synchronize()
        g = f.grads.detach().double().cpu()
        scale = float(g_sum.abs().max())
        worst_g = max(worst_g, float((g - g_sum).abs().max()) / scale)
        # reference Adam (torch 1.8 math, coupled L2) on the averaged gradient the engine reduced
        ga = g.to(dev) / world + WD * p0
        m1 = B1 * m0 + (1 - B1) * ga
        v1 = B2 * v0 + (1 - B2) * ga * ga
        t = step0 + 1
        bc1, bc2 = 1 - B1 ** t, 1 - B2 ** t
        p1 = p0 - (LR / bc1) * m1 / (v1.sqrt() / bc2 ** 0.5 + EPS)
        worst_a = max(worst_a, float((p1 - f.params.double()).abs().max()))
        # ranks agree bitwise on everything the step mutates
        # (BN running statistics legitimately differ: each rank normalises its own batch, as without
        # SyncBN; the trainer averages them before validation)
        for name, tt in (("params", f.params), ("exp_avg", f.exp_avg), ("exp_avg_sq", f.exp_avg_sq)):
            parts = gather_cpu(tt)
            if not all(torch.equal(parts[0], q) for q in parts[1:]):
                raise AssertionError(f"step {s}: ranks disagree on {name}")
    print(json.dumps({"rank": ctx.rank, "steps": steps, "max_grad_rel": worst_g, "max_adam_abs": worst_a,
                      "buckets": [list(b) for b in buckets], "ext_dp": runner.ext_dp}), flush=True)
    shutdown(ctx)


if __name__ == "__main__":
    main()
