"""Data-parallel logic on CPU with the gloo backend and world_size 2 (the RCCL path on MI355X is the same
code with backend 'nccl')."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from mtl_das_pytorch_amd.parallel.dist import init_distributed
    return init_distributed(backend="gloo")


def _worker_grads(rank, world, port, q):
    import torch.nn.functional as F
    from mtl_das_pytorch_amd.models import MTL_Net
    from mtl_das_pytorch_amd.parallel.dist import FlatGradAllReducer, broadcast_module_state
    ctx = _init(rank, world, port)
    torch.manual_seed(rank)  # different init per rank: broadcast must fix it
    m = MTL_Net().eval()  # BN in eval mode: per-sample independent -> DP grads == full-batch grads
    broadcast_module_state(ctx, list(m.parameters()) + list(m.buffers()))
    g = torch.Generator().manual_seed(0)
    x = torch.randn(4, 1, 100, 250, generator=g)
    lab = torch.randint(0, 2, (4,), generator=g)
    sl = slice(2 * rank, 2 * rank + 2)
    o1, o2 = m(x[sl])
    F.nll_loss(o2, lab[sl]).backward()
    flat = torch.cat([p.grad.reshape(-1) for p in m.parameters() if p.grad is not None])
    FlatGradAllReducer(ctx, bucket_mb=0.5)(flat)  # chunked buckets
    flat /= world
    # full-batch reference on rank 0's (broadcast) weights
    m.zero_grad()
    o1, o2 = m(x)
    F.nll_loss(o2, lab).backward()
    ref = torch.cat([p.grad.reshape(-1) for p in m.parameters() if p.grad is not None])
    q.put((rank, float((flat - ref).norm() / ref.norm()), float(next(m.parameters()).sum())))
    dist.destroy_process_group()


def test_dp_gradients_equal_full_batch():
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker_grads, args=(r, 2, port, q)) for r in range(2)]
    [p.start() for p in ps]
    res = sorted(q.get(timeout=300) for _ in range(2))
    [p.join(60) for p in ps]
    for rank, err, wsum in res:
        assert err < 1e-5, err
    assert res[0][2] == res[1][2]  # identical (broadcast) weights


def _worker_sampler(rank, world, port, q):
    from mtl_das_pytorch_amd.parallel.dist import ShardedIndexSampler, sum_
    ctx = _init(rank, world, port)
    s = ShardedIndexSampler(21, 4, ctx, seed=3)
    b = s.epoch(0, "cpu")
    t = torch.tensor([float(len(b))])
    sum_(ctx, [t])
    q.put((rank, [x.tolist() for x in b], float(t)))
    dist.destroy_process_group()


def test_sharded_sampler_covers_dataset():
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker_sampler, args=(r, 2, port, q)) for r in range(2)]
    [p.start() for p in ps]
    res = sorted(q.get(timeout=300) for _ in range(2))
    [p.join(60) for p in ps]
    a, b = res[0][1], res[1][1]
    assert len(a) == len(b) == 3  # ceil(21 / 8) full batches on every rank
    seen = set(sum(a, []) + sum(b, []))
    assert seen == set(range(21))
    assert res[0][2] == 6.0


def _worker_train(rank, world, port, out, q):
    from mtl_das_pytorch_amd.engine.trainer import Trainer
    from mtl_das_pytorch_amd.utils.config import TrainConfig
    ctx = _init(rank, world, port)
    cfg = TrainConfig(model="MTL", synthetic=2, batch_size=4, epoch_num=1, output_savedir=out, GPU_device=False,
                      save_threshold=0.0, log_every=2)
    tr = Trainer(cfg, ctx)
    tr.run()
    p = torch.cat([x.detach().reshape(-1) for x in tr.model.parameters()])
    q.put((rank, float(p.sum()), float(p.abs().sum()), tr.save_dir))
    dist.destroy_process_group()


def test_dp_trainer_ranks_stay_in_sync(tmp_path):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker_train, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    [p.start() for p in ps]
    res = sorted(q.get(timeout=600) for _ in range(2))
    [p.join(60) for p in ps]
    assert res[0][1] == pytest.approx(res[1][1], rel=1e-6)
    assert res[0][2] == pytest.approx(res[1][2], rel=1e-6)
    assert res[0][3] == res[1][3]
    dirs = [d for d in os.listdir(tmp_path)]
    assert len(dirs) == 1  # only rank 0 writes, one run directory
    files = os.listdir(os.path.join(tmp_path, dirs[0]))
    assert "console output.log" in files and any(f.endswith(".pth") for f in files)


def _worker_one_rank(q):
    os.environ.pop("WORLD_SIZE", None)
    os.environ["MDA_DIST_BACKEND"] = "gloo"
    from mtl_das_pytorch_amd.parallel.dist import FlatGradAllReducer, init_distributed, shutdown
    ctx = init_distributed()
    t = torch.arange(8, dtype=torch.float32)
    red = FlatGradAllReducer(ctx)
    red.start(t[:4])
    red.start(t[4:])
    red.finish()
    ctx.barrier()
    q.put((ctx.enabled, ctx.world, dist.is_initialized(), dist.get_world_size(), t.tolist()))
    shutdown(ctx)


def test_one_rank_process_group():
    """MDA_DIST_BACKEND with WORLD_SIZE=1 builds a real 1-rank process group (in-process store): the
    collective code path runs and a 1-rank sum is the identity (the GPU test does the same over RCCL)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker_one_rank, args=(q,))
    p.start()
    res = q.get(timeout=120)
    p.join(60)
    assert res == (True, 1, True, 1, [float(i) for i in range(8)])
