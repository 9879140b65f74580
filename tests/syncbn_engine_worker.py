"""Worker of tests/test_dp_engine_gpu.py::test_engine_sync_bn: one rank of a 2-rank SyncBN engine job on ONE
GPU (MDA_SINGLE_DEVICE=1, gloo), checked against ONE process training the union of both ranks' batches.

With SyncBN every BN normalises with the statistics of the global batch, so two ranks training B samples
each must reproduce a single process training the same 2B samples: the same BN running statistics on
every rank, and (after the data-parallel average) the same parameter gradient -- up to fp32 summation
order, which the ill-conditioned network at init amplifies in the backward.  ``sync`` = 0 runs the plain
DP path as the negative control (each rank normalises its own half).

Prints one JSON line per rank: {"rank", "sync", "grad_rel", "bn_rel", "bn_rank_rel", "loss_rel"}.
    python -m torch.distributed.run --nproc-per-node 2 ... tests/syncbn_engine_worker.py MODEL SYNC
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
from mtl_das_pytorch_amd.parallel.dist import FlatGradAllReducer, init_distributed, shutdown  # noqa: E402


def build(model_type, B, dev, sync_world):
    torch.manual_seed(1234)  # identical init everywhere
    m = build_model(model_type)
    if model_type == "multi_classifier":
        prog = InceptionProgram(m, B, dev, p_drop=0.0, sync_world=sync_world)  # no dropout: exact comparison
    else:
        prog = MTLProgram(m, B, dev, sync_world=sync_world)
    return prog


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def main():
    model_type, sync = sys.argv[1], int(sys.argv[2])
    ctx = init_distributed()
    world, dev = ctx.world, ctx.device
    B = 16
    joint = model_type == "multi_classifier"
    X, d, e = generate(world * B, seed=77, device=dev)  # the same global batch on every rank
    lab = encode_joint(d, e) if joint else torch.stack([d, e], 1)
    mine = torch.arange(ctx.rank * B, (ctx.rank + 1) * B, device=dev)
    prog = build(model_type, B, dev, world if sync else 1)
    prog.set_optimizer(weight_decay=0.0, grad_scale=1.0 / world)
    if sync:
        prog.enable_sync_bn(lambda t: ctx.all_reduce_(t))
    autotune_program(prog, measure=False)
    runner = StepRunner(prog, X, lab, use_graph=not sync, allreduce=FlatGradAllReducer(ctx))
    runner.set_lr(0.0)  # gradients and statistics only
    runner.train_step(mine)
    torch.cuda.synchronize()
    g = prog.flat.grads.detach().clone() / world  # the data-parallel average
    # reference: one process, the whole 2B batch
    ref = build(model_type, world * B, dev, 1)
    ref.set_optimizer(weight_decay=0.0)
    autotune_program(ref, measure=False)
    rrun = StepRunner(ref, X, lab, use_graph=False)
    rrun.set_lr(0.0)
    rrun.train_step(torch.arange(world * B, device=dev))
    torch.cuda.synchronize()
    # one step from the init (mean 0, var 1, momentum 0.1): running mean = 0.1 mu, var = 0.9 + 0.1 sigma^2
    bn_mine = torch.cat([prog.flat.bn_mean, prog.flat.bn_var - 0.9])
    bn_ref = torch.cat([ref.flat.bn_mean, ref.flat.bn_var - 0.9])
    parts = [torch.empty_like(bn_mine.cpu()) for _ in range(world)]
    dist.all_gather(parts, bn_mine.cpu())
    # summed loss of the first metric row (Model C: joint CE; A: distance NLL)
    loss_mine = prog.metrics[0, 0].reshape(1).clone().cpu()
    dist.all_reduce(loss_mine)
    out = {"rank": ctx.rank, "sync": sync, "grad_rel": rel(g, ref.flat.grads),
           "bn_rel": rel(bn_mine, bn_ref), "bn_rank_rel": rel(parts[1], parts[0]),
           "loss_rel": rel(loss_mine, ref.metrics[0, 0].reshape(1).cpu())}
    print(json.dumps(out), flush=True)
    shutdown(ctx)


if __name__ == "__main__":
    main()
