"""Data-parallel training over RCCL (torch.distributed backend "nccl" is RCCL on ROCm) across xGMI.

The reference has no distributed code at all; this module adds, MI355X-first:

  C1  broadcast of parameters + BN buffers from rank 0 (once, and after loading a checkpoint)
  C2  all-reduce(SUM) of the *flat* fp32 gradient buffer -- the engine's gradients already live in one
      contiguous, persistent buffer, so there is no pack/unpack; the 1/world averaging is folded into
      the fused Adam kernel (grad_scale).  Model A's whole gradient is 4.5 MB: one bucket.  Larger
      models are split into ``bucket_mb`` chunks issued back to back (xGMI is point-to-point, so one
      ring per collective is link-bound; RCCL spreads channels over the 7 links itself).
  C3  all-reduce of on-device metric counters / confusion matrices (validation)
  C4  averaging of BN running statistics before evaluation / checkpointing (ranks see different data)
  C5  barriers around rank-0 I/O

Launch with one process per GPU: ``torchrun --nproc-per-node N --master-addr 127.0.0.1 ...``.  The
same code runs on CPU with the gloo backend (tests use world_size 2).
"""
from __future__ import annotations

import datetime
import math
import os
from dataclasses import dataclass
from typing import Iterable, List, Optional

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: Optional[str] = None
    # RCCL: a second communicator that runs ONLY collectives captured into HIP graphs.  PyTorch's
    # process-group watchdog thread polls the completion events of every eager collective it still lists;
    # on ROCm that poll fails once the communicator's stream has joined a graph capture ("event last
    # recorded in a capturing stream") and the watchdog aborts the process.  Captured collectives are never
    # listed, so a communicator that never runs an eager collective never has anything to poll: capture is
    # safe by construction, with no dependence on the watchdog's timing.
    capture_group: object = None

    @property
    def enabled(self) -> bool:
        """A process group exists: collectives run (a 1-rank RCCL group included -- MDA_DIST_BACKEND=nccl with
        WORLD_SIZE=1 executes the whole RCCL code path on one GPU)."""
        return self.backend is not None

    @property
    def capturable_collectives(self) -> bool:
        """Collectives can be captured into a HIP graph (RCCL: stream-ordered device collectives, run on the
        capture-only communicator ``capture_group``); gloo's host round trip cannot.  SyncBN's in-step
        collectives are captured whenever this holds (the eager alternative is ~10x slower); the gradient
        buckets only where ``capture_gradients`` says so.  MDA_CAPTURE_COLLECTIVES=0 disables capture."""
        return self.capture_group is not None

    @property
    def capture_gradients(self) -> bool:
        """The gradient buckets' all-reduces are captured in the step graph: one-rank groups, or several ranks
        with MDA_CAPTURE_COLLECTIVES=1.  The multi-rank default keeps them eager behind the graph's external
        bucket events (engine/step.py "train_ext"): multi-rank RCCL graph capture could not be validated on
        the one-GPU machines this was built on, the eager RCCL path is the known-good one."""
        return self.capturable_collectives and (self.world == 1 or os.environ.get("MDA_CAPTURE_COLLECTIVES") == "1")

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    def barrier(self):
        if self.enabled:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.local_rank])
            else:
                dist.barrier()

    def all_reduce_(self, t: torch.Tensor, op=None):
        if self.enabled:
            dist.all_reduce(t, op=op or dist.ReduceOp.SUM)
        return t

    def all_reduce_ordered_(self, t: torch.Tensor):
        """All-reduce(SUM) of a device tensor ordered on the CURRENT stream: the kernels queued before on
        that stream are reduced, the ones queued after see the result.  RCCL gives exactly this; gloo (the
        one-GPU rehearsal of several ranks) goes through a host copy: ``.cpu()`` waits for the stream, the
        CPU all-reduce runs, and the copy back is queued on the stream."""
        if not self.enabled:
            return t
        if self.backend == "nccl":
            if torch.cuda.is_current_stream_capturing():  # the capture-only communicator (see ``capture_group``)
                dist.all_reduce(t, group=self.capture_group)
            else:
                # eager (the warm-up run before a capture among others): async on the group's own stream, the
                # current stream waits for it.  A synchronous all_reduce runs on -- and records its work's
                # events on -- the CURRENT stream, here an engine phase stream; the graph captured right after
                # the warm-up captures on those same phase streams, and the watchdog's poll of the not yet
                # retired eager work then queries an event of a stream that is capturing: "operation not
                # permitted on an event last recorded in a capturing stream", an abort whose timing depended on
                # the watchdog's 100 ms poll (the round-3 0.5 s sleep hid it; the 1-rank RCCL test failed ~1 in 3)
                dist.all_reduce(t, async_op=True).wait()
            return t
        if t.device.type != "cuda":
            dist.all_reduce(t)
            return t
        c = t.cpu()
        dist.all_reduce(c)
        t.copy_(c)
        return t

    def broadcast_(self, t: torch.Tensor, src: int = 0):
        if self.enabled:
            dist.broadcast(t, src=src)
        return t

    def max_scalar(self, x: float) -> float:
        if not self.enabled:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())


def init_distributed(backend: Optional[str] = None, timeout_s: Optional[int] = None) -> DistContext:
    """Initialise from torchrun's environment (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*).

    Failure detection: collectives time out after ``timeout_s`` (env ``MDA_PG_TIMEOUT``, default 600 s)
    instead of hanging when a peer dies, so the rank errors out and torchrun's elastic agent
    (``--max-restarts``) can restart the worker group, which resumes with ``--resume auto``."""
    if timeout_s is None:
        timeout_s = int(os.environ.get("MDA_PG_TIMEOUT", "600"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available()
    # MDA_SINGLE_DEVICE=1 puts every rank on cuda:0 and MDA_DIST_BACKEND overrides the backend: together
    # they rehearse the multi-rank GPU path (split graphs around the all-reduce, sharded sampler, metric
    # reduction) on a one-GPU machine with gloo (RCCL refuses two ranks on one device)
    dev_index = 0 if os.environ.get("MDA_SINGLE_DEVICE") == "1" else local_rank
    device = torch.device(f"cuda:{dev_index}") if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(device)
    backend = backend or os.environ.get("MDA_DIST_BACKEND")
    if world <= 1:
        if not backend:
            return DistContext(0, 1, 0, device, None)
        # a real 1-rank process group (MDA_DIST_BACKEND=nccl: a 1-rank RCCL communicator on this GPU), so
        # the collective code path -- async bucket all-reduces, stream-ordered SyncBN sums, barriers,
        # metric reduction -- executes on a one-GPU machine; rendezvous through an in-process store
        if not dist.is_initialized():
            kw = dict(backend=backend, store=dist.HashStore(), rank=0, world_size=1,
                      timeout=datetime.timedelta(seconds=timeout_s))
            if backend == "nccl":
                kw.update(device_id=device, pg_options=_rccl_options())
            dist.init_process_group(**kw)
        return _with_capture_group(DistContext(0, 1, 0, device, backend))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    backend = backend or ("nccl" if use_gpu else "gloo")
    if backend == "gloo" and os.environ["MASTER_ADDR"] in ("127.0.0.1", "localhost"):
        # single-node gloo over loopback: the host name may not resolve (containers), and gloo's
        # interface guess then makes a restarted group's full-mesh connect fail intermittently
        os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
    if not dist.is_initialized():
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw.update(device_id=device, pg_options=_rccl_options())
        dist.init_process_group(**kw)
    return _with_capture_group(DistContext(rank, world, local_rank, device, backend))


# communicator streams from torch's high-priority pool (see _rccl_options; a class-free switch for A/B runs)
RCCL_HIGH_PRIORITY = True


def _rccl_options():
    """RCCL communicators run on HIGH-priority pool streams (RCCL_HIGH_PRIORITY).  PyTorch hands out the normal-priority pool's 32
    streams round robin to every ``torch.cuda.Stream()`` -- the engine's phase streams and the graph-capture
    stream among them -- and to the process group's communication stream alike; once the pool wraps, a
    communicator's stream can BE a stream the step graph captures on, and the watchdog's poll of an eager
    collective's event recorded there fails during the capture ("event last recorded in a capturing stream",
    seen on Model C's 4-stream step).  A separate pool keeps them apart; priority also puts the collectives'
    kernels ahead of compute in the queues, as wanted for overlapped gradient buckets."""
    return dist.ProcessGroupNCCL.Options(is_high_priority_stream=RCCL_HIGH_PRIORITY)


def _with_capture_group(ctx: DistContext) -> DistContext:
    """Create the capture-only RCCL communicator (DistContext.capture_group) on RCCL groups (unless
    MDA_CAPTURE_COLLECTIVES=0).  Every rank makes the same call (new_group is collective); the default group is
    bound to the device, so the new communicator is initialised eagerly here -- never lazily inside a capture."""
    if ctx.backend == "nccl" and os.environ.get("MDA_CAPTURE_COLLECTIVES") != "0":
        ctx.capture_group = dist.new_group(backend="nccl", pg_options=_rccl_options())
    return ctx


def shutdown(ctx: DistContext):
    if ctx.enabled and dist.is_initialized():
        dist.destroy_process_group()


# ------------------------------------------------------------------------------------------------
class FlatGradAllReducer:
    """All-reduce(SUM) of a flat gradient buffer in ``bucket_mb`` chunks (0 = one bucket)."""

    def __init__(self, ctx: DistContext, bucket_mb: float = 0.0, capture: Optional[bool] = None):
        self.ctx = ctx
        self.bucket_elems = int(bucket_mb * 2 ** 20 / 4) if bucket_mb > 0 else 0
        self._pending = []
        # the bucket all-reduces may be embedded in the step's HIP graph (engine/step.py "train_full_dp"):
        # ``ordered`` is then the stream-ordered form the captured launches call.  Default: where the group
        # captures gradients (DistContext.capture_gradients); ``capture=True`` where every collective of the
        # step must share the capture communicator (SyncBN's captured collectives), if the group can capture
        want = ctx.capture_gradients if capture is None else (capture and ctx.capturable_collectives)
        self.capturable = want and os.environ.get("MDA_DP_CAPTURE", "1") == "1"
        self.ordered = ctx.all_reduce_ordered_

    # issue each bucket as a stream-ordered (async_op=False) collective while the communication stream is
    # current, and join that stream once in finish(), instead of async work on the process group's internal
    # stream that the caller then waits for per bucket: one stream hop less per bucket (per-rank program of 8
    # GPUs on a 1-rank RCCL group: A 33,368 / 33,345 -> 34,866 / 34,807, C 9,129 / 9,071 -> 9,261 / 9,363;
    # docs/PERF.md round 6).  Class switch for A/B runs.
    ON_COMM_STREAM = True

    def start(self, t: torch.Tensor):
        """Issue an asynchronous all-reduce(SUM) of one gradient bucket (a contiguous view of the flat
        buffer).  The communication stream waits for the work already queued on the current stream, so
        the bucket must be complete in stream order; the current stream is free to continue."""
        if not self.ctx.enabled:
            return
        if self.ON_COMM_STREAM:
            dist.all_reduce(t)
            self._pending.append(torch.cuda.current_stream() if t.is_cuda else None)
        else:
            self._pending.append(dist.all_reduce(t, async_op=True))

    def finish(self):
        """Make the current stream wait for every bucket issued by ``start`` (no host synchronisation on
        RCCL: Work.wait() inserts a stream dependency)."""
        joined = set()
        for h in self._pending:
            if isinstance(h, torch.cuda.Stream):
                if h not in joined:
                    torch.cuda.current_stream().wait_stream(h)
                    joined.add(h)
            elif h is not None:
                h.wait()
        self._pending = []

    def __call__(self, grads: torch.Tensor):
        if not self.ctx.enabled:
            return
        n = grads.numel()
        if self.bucket_elems <= 0 or n <= self.bucket_elems:
            dist.all_reduce(grads)
            return
        handles = [dist.all_reduce(grads[o:o + self.bucket_elems], async_op=True)
                   for o in range(0, n, self.bucket_elems)]
        for h in handles:
            h.wait()


def calibrate_allreduce(ctx: DistContext, numel: int, reps: int = 5) -> Optional[float]:
    """Milliseconds of one all-reduce(SUM) of ``numel`` fp32 elements on the live process group (median of
    ``reps`` after a warm-up, max over ranks so that every rank derives the same bucket count from it), or None
    without a group.  bench.py reports it (``allreduce_ms``) and LoweredProgram.dp_buckets sizes the gradient
    buckets from it: on xGMI the flat gradient's all-reduce is 10s of us (A, 4.3 MB) to ~0.5 ms (C, 83 MB)."""
    if not ctx.enabled:
        return None
    import time
    t = torch.zeros(numel, dtype=torch.float32, device=ctx.device)
    sync = torch.cuda.synchronize if t.is_cuda else (lambda: None)
    dist.all_reduce(t)
    sync()
    times = []
    for _ in range(reps):
        ctx.barrier()
        sync()
        t0 = time.perf_counter()
        dist.all_reduce(t)
        sync()
        times.append(time.perf_counter() - t0)
    del t
    return ctx.max_scalar(1e3 * sorted(times)[len(times) // 2])


def broadcast_module_state(ctx: DistContext, tensors: Iterable[torch.Tensor], src: int = 0):
    """C1: make every rank start from rank ``src``'s parameters and buffers."""
    if not ctx.enabled:
        return
    for t in tensors:
        dist.broadcast(t, src=src)


def average_(ctx: DistContext, tensors: Iterable[torch.Tensor]):
    """C4: average (float) tensors across ranks, e.g. BN running statistics before eval/checkpoint."""
    if not ctx.enabled:
        return
    for t in tensors:
        if t.is_floating_point():
            dist.all_reduce(t)
            t.div_(ctx.world)


def sum_(ctx: DistContext, tensors: Iterable[torch.Tensor]):
    """C3: sum metric counters / confusion matrices across ranks."""
    if not ctx.enabled:
        return
    for t in tensors:
        dist.all_reduce(t)


# ------------------------------------------------------------------------------------------------
class ShardedIndexSampler:
    """Per-epoch shuffled indices, sharded across ranks (rank r takes batches r, r+W, ...).

    Every rank receives the same number of full batches: the permutation is padded with a seeded random
    draw so that no rank runs a shorter epoch (the engine's HIP graph has a fixed batch size)."""

    def __init__(self, n: int, batch: int, ctx: DistContext, shuffle: bool = True, seed: int = 0,
                 pad_random: bool = True):
        self.n, self.batch, self.ctx, self.shuffle, self.seed = n, batch, ctx, shuffle, seed
        self.pad_random = pad_random

    def num_batches(self) -> int:
        return math.ceil(self.n / (self.batch * self.ctx.world))

    def epoch(self, epoch: int, device) -> List[torch.Tensor]:
        g = torch.Generator().manual_seed(self.seed * 1000003 + epoch)
        order = torch.randperm(self.n, generator=g) if self.shuffle else torch.arange(self.n)
        per_step = self.batch * self.ctx.world
        total = self.num_batches() * per_step
        if total > self.n:
            extra = torch.randint(0, self.n, (total - self.n,), generator=g) if self.pad_random else \
                order[torch.arange(total - self.n) % self.n]
            order = torch.cat([order, extra])
        order = order.view(self.num_batches(), self.ctx.world, self.batch)[:, self.ctx.rank]
        order = order.to(device)
        return [order[i] for i in range(order.shape[0])]
