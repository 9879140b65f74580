"""Worker of tests/test_dp_engine_gpu.py::test_engine_sync_bn: one rank of a 2-rank SyncBN engine job on ONE
GPU (MDA_SINGLE_DEVICE=1, gloo), checked against ONE process training the union of both ranks' batches.

With SyncBN every BN normalises with the statistics of the global batch, so two ranks training B samples
each must reproduce a single process training the same 2B samples: the same BN running statistics on
every rank, and (after the data-parallel average) the same parameter gradient -- up to fp32 summation
order, which the ill-conditioned network at init amplifies in the backward.  ``sync`` = 0 runs the plain
DP path as the negative control (each rank normalises its own half).

The whole-network gradient comparison is loose by nature (a 1e-5 forward difference between the B = 16
and B = 32 kernel configurations grows to ~10% in the backward at init); the layer-local check
(``local_dy_rel``) is exact: every BN tail's dy on this rank (Model A: the backbone's; Model C: all ~94
BasicConv2d tails) against the closed-form backward with the globally all-reduced sums.

Prints one JSON line per rank: {"rank", "sync", "grad_rel", "bn_rel", "bn_rank_rel", "loss_rel", "local_dy_rel"}.
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


def local_syncbn_check(prog, world):
    """Chaos-free SyncBN check (Model A backbone): for every backbone BN tail, the engine's dy on this rank
    against the closed-form backward with GLOBAL batch sums -- this rank's dz from its own gradient
    sources, sum(dz) and sum(dz xhat) all-reduced over the ranks.  Returns the worst relative error."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_mtl_layer_local_gpu import k4, nchw
    lv, rbs, T = prog.levels, prog.rbs, prog.T

    def sources(k):
        g = 0
        if k >= 1:
            L = lv[(k - 1) // 2]
            for t in range(T):
                g = g + (nchw(L["dcat"], t, 0, L["C"]) if k % 2 == 1 else nchw(L["dF"], t))
        if k < 8:
            R = rbs[k]
            for key in ("dxs", "dxa"):  # a dgrad that summed every source of F_k (fold_tail_sources)
                if key in R and any(l.name == "conv_dgrad" and l.args[3].get("add") and l.args[3]["out"] == R[key].p
                                    for l in prog.bwd.launches):
                    return nchw(R[key])
            g = g + nchw(R["dxa"])
            if not R.get("fused"):  # (a fused conv a + shortcut: "dxa" is the block input's one data gradient)
                g = g + (nchw(R["dxs"]) if R["proj"] else nchw(R["side"]))
        return g

    def sync_dy(dz, y, bn):
        _, _, mu, inv = k4(bn)
        xh = (y - mu) * inv
        sums = torch.stack([dz.sum((0, 2, 3)), (dz * xh).sum((0, 2, 3))]).double().cpu()
        dist.all_reduce(sums)
        n = world * dz.shape[0] * dz.shape[2] * dz.shape[3]
        m1, m2 = (sums / n).float().to(dz.device).view(2, 1, -1, 1, 1)
        gam = bn.mods[0].weight.detach().view(1, -1, 1, 1)
        return gam * inv * (dz - m1 - xh * m2)

    errs = {}
    for i in range(8):
        R = rbs[i]
        yb = nchw(R["yb"])
        sc, sh, _, _ = k4(R["bnb"])
        if R["proj"]:
            sc2, sh2, _, _ = k4(R["bns"])
            rr = nchw(R["ys"]) * sc2 + sh2
        else:
            rr = nchw(R["in"])
        dz = sources(i + 1) * ((yb * sc + sh + rr) > 0)
        errs[f"rb{i + 1}.tail"] = rel(nchw(R["dyb"]), sync_dy(dz, yb, R["bnb"]))
        if R["proj"]:
            errs[f"rb{i + 1}.short"] = rel(nchw(R["dys"]), sync_dy(dz, nchw(R["ys"]), R["bns"]))
        ya = nchw(R["ya"])
        sca, sha, _, _ = k4(R["bna"])
        errs[f"rb{i + 1}.inner"] = rel(nchw(R["dya"]), sync_dy(nchw(R["dha"]) * ((ya * sca + sha) > 0), ya, R["bna"]))
    y0 = nchw(prog.y0)
    sc, sh, _, _ = k4(prog.bn1)
    errs["conv1"] = rel(nchw(prog.dy0), sync_dy(sources(0) * ((y0 * sc + sh) > 0), y0, prog.bn1))
    print(json.dumps({k: round(v, 5) for k, v in errs.items()}), file=sys.stderr, flush=True)
    return max(errs.values())


def local_syncbn_check_inception(prog, world):
    """The same chaos-free check for Model C: every BasicConv2d's BN-ReLU tail backward on this rank (its dz
    from the engine's own gradient sources and stored y) against the closed form with the all-reduced
    sum(dz), sum(dz xhat).  Returns the worst relative error over the ~94 layers."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_inception_gpu import _nchw
    from test_mtl_layer_local_gpu import k4
    from mtl_das_pytorch_amd.engine.inception import CBR
    errs = []
    for op in prog.ops:
        if not isinstance(op, CBR):
            continue
        g = sum(_nchw(a) for a in op.out.grad_sources())
        y = _nchw(op.y)
        sc, sh, mu, inv = k4(op.bn)
        dz = g * ((y * sc + sh) > 0)
        xh = (y - mu) * inv
        sums = torch.stack([dz.sum((0, 2, 3)), (dz * xh).sum((0, 2, 3))]).double().cpu()
        dist.all_reduce(sums)
        n = world * dz.shape[0] * dz.shape[2] * dz.shape[3]
        m1, m2 = (sums / n).float().to(dz.device).view(2, 1, -1, 1, 1)
        gam = op.bn.mods[0].weight.detach().view(1, -1, 1, 1)
        errs.append(rel(_nchw(op.dy), gam * inv * (dz - m1 - xh * m2)))
    print(json.dumps({"layers": len(errs), "worst": max(errs), "median": sorted(errs)[len(errs) // 2]}),
          file=sys.stderr, flush=True)
    return max(errs)


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
    prog.set_optimizer(weight_decay=0.0, grad_scale=1.0 / world, data_parallel=True)
    if sync:
        prog.enable_sync_bn(ctx.all_reduce_ordered_)
    autotune_program(prog, measure=False)
    runner = StepRunner(prog, X, lab, use_graph=not sync, allreduce=FlatGradAllReducer(ctx))
    runner.set_lr(0.0)  # gradients and statistics only
    runner.train_step(mine)
    torch.cuda.synchronize()
    g = prog.flat.grads.detach().clone() / world  # the data-parallel average
    local = local_syncbn_check(prog, world) if not joint else local_syncbn_check_inception(prog, world)
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
    # per BN layer in module order: the first layers see no amplification of the B = 16 / B = 32 kernel
    # configuration differences (Model C is ~90 layers deep; its last blocks drift chaotically either way)
    per = []
    for name, m in prog.model.named_modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            o, c = prog.flat.bn_offsets[id(m)], m.num_features
            per.append(rel(prog.flat.bn_mean[o:o + c], ref.flat.bn_mean[o:o + c]))
    parts = [torch.empty_like(bn_mine.cpu()) for _ in range(world)]
    dist.all_gather(parts, bn_mine.cpu())
    # summed loss of the first metric row (Model C: joint CE; A: distance NLL)
    loss_mine = prog.metrics[0, 0].reshape(1).clone().cpu()
    dist.all_reduce(loss_mine)
    loss_ref = ref.metrics[0, 0].reshape(1).cpu()
    # the same step again from the same weights (lr 0): bitwise-identical gradients (determinism)
    runner.train_step(mine)
    torch.cuda.synchronize()
    repeat_equal = bool(torch.equal(prog.flat.grads / world, g))
    out = {"rank": ctx.rank, "sync": sync, "grad_rel": rel(g, ref.flat.grads),
           "bn_rel": rel(bn_mine, bn_ref), "bn_rel_first8": max(per[:8]), "bn_rank_rel": rel(parts[1], parts[0]),
           "loss_rel": rel(loss_mine, loss_ref), "local_dy_rel": local,
           "repeat_equal": repeat_equal}
    print(json.dumps(out), flush=True)
    shutdown(ctx)


if __name__ == "__main__":
    main()
