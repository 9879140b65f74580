"""A lowered program: an ordered list of prebuilt HIP launches (forward, backward, optimizer).

Launch arguments (device pointers, geometry, descriptor tables) are resolved once at lowering time,
so executing a phase is a tight loop of pybind calls; on the GPU the loop is captured once into a
HIP graph and replayed (engine/step.py).

Launches carry a logical stream id: 0 is the caller's stream (the critical path), 1..3 are side streams
forked from it at phase start.  Dependencies between streams are explicit ``record``/``wait`` event
tags; every side stream is joined back into stream 0 at the end of the phase.  Under graph capture the
events become graph edges, so independent branches (task branches vs. backbone, weight gradients vs.
the data-gradient chain) run concurrently on the GPU."""
from __future__ import annotations

from typing import Callable, List

import os

from ..ops.hip import lib, stream

# Side streams are on by default (MDA_STREAMS=0 runs the list serially on one stream).  Measured on
# MI355X: independent branches captured on separate streams DO overlap in graph replay (two chains of
# small convs: 253 vs 320 us, tools/graph_concurrency.py); Model A levels || backbone: 21.2k -> 25.0k
# samples/s, Model C Inception branches on 4 streams: 5.7k -> 6.35k.  Cross-stream edges are kept few
# (join-then-fork points, wgrads on their producer's stream): denser event patterns crashed
# hipStreamEndCapture on ROCm 7.
MULTI_STREAM = os.environ.get("MDA_STREAMS", "1") == "1"
# streams used at most (ids above are folded onto the last one -- still a valid schedule); never more than
# the process's hardware queues: with GPU_MAX_HW_QUEUES=2 a 4-stream graph segfaults inside the HIP runtime
# at replay, engine-free repro in tools/hwq_repro.py (profiles/r4_runtime_faults.txt)
MAX_STREAMS = max(1, min(4, int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))))
# logical id of the communication stream: data-parallel gradient all-reduces embedded in the backward
# (LoweredProgram.backward_with_allreduce) run there, beside the compute streams, never folded onto them
COMM_STREAM = 7
# logical id of the weight-gradient spill stream (LoweredProgram.spill_wgrads): the early stream-0 weight
# gradients run there while stream 0 continues its data-gradient chain
SPILL_STREAM = 6


class Launch:
    __slots__ = ("name", "fn", "args", "owner", "stream", "waits", "record", "bucket")

    def __init__(self, name: str, fn: Callable, *args, owner=None, stream: int = 0, waits=(), record=None,
                 bucket: int = 0):
        self.name = name
        self.bucket = bucket  # gradient bucket whose finalize this launch feeds (segmented backward, DP)
        self.fn = fn
        self.args = args
        self.owner = owner  # the layer object that emitted it (used by the autotuner)
        self.stream = stream
        self.waits = tuple(waits)
        self.record = record

    def __call__(self, st: int, tstream=None):
        if self.fn is None:  # a pseudo-launch that only carries waits / a record (fork point)
            return
        if self.fn is k_allreduce:  # a host-issued collective: it runs with the launch's stream as current
            import torch
            if tstream is None or tstream == torch.cuda.current_stream():
                self.fn(*self.args, None)
            else:
                with torch.cuda.stream(tstream):
                    self.fn(*self.args, None)
            return
        self.fn(*self.args, st)


class Phase:
    def __init__(self, name: str):
        self.name = name
        self.launches: List[Launch] = []
        self._streams = None
        self.cur_stream = 0      # default stream id for add()
        self.pending_waits = []  # waits attached to the next add() on any stream
        self.alias = {}          # event tag -> tag it is recorded under (after launches were removed)

    def add(self, name, fn, *args, owner=None, stream=None, waits=(), record=None):
        sid = self.cur_stream if stream is None else stream
        w = tuple(waits) + tuple(self.pending_waits)
        self.pending_waits = []
        self.launches.append(Launch(name, fn, *args, owner=owner, stream=sid, waits=w, record=record))

    def fork_point(self, tag: str, waits=()):
        """A kernel-free launch on the current stream that waits for ``waits`` and records ``tag``:
        the join-then-fork point other streams wait on (eager: stream waits + an event record)."""
        self.launches.append(Launch(f"fork:{tag}", None, stream=self.cur_stream, waits=tuple(waits), record=tag))

    def mark(self, tag: str):
        """Record event ``tag`` after the last launch added on the current stream."""
        for l in reversed(self.launches):
            if l.stream == self.cur_stream:
                if l.record is not None and l.record != tag:
                    raise ValueError("launch already records an event")
                l.record = tag
                return
        raise ValueError("no launch to mark")

    def run(self, st=None):
        import torch
        if not MULTI_STREAM or all(l.stream == 0 and not l.waits for l in self.launches):
            st = stream() if st is None else st
            for l in self.launches:
                if l.fn is not None:
                    l(st)
            return
        main = torch.cuda.current_stream()
        if self._streams is None or self._streams[0].device != main.device:
            self._streams = [torch.cuda.Stream(device=main.device) for _ in range(MAX_STREAMS + 1)]
        streams = [main] + self._streams  # [MAX_STREAMS] communication, [MAX_STREAMS + 1] spill stream
        sid_of = lambda l: (MAX_STREAMS if l.stream == COMM_STREAM else MAX_STREAMS + 1 if l.stream == SPILL_STREAM  # noqa: E731
                            else min(l.stream, MAX_STREAMS - 1))
        used = {sid_of(l) for l in self.launches}
        start = main.record_event()
        for sid in used - {0}:
            streams[sid].wait_event(start)
        events = {}
        for l in self.launches:
            s = streams[sid_of(l)]
            for tag in l.waits:
                s.wait_event(events[self.alias.get(tag, tag)])
            l(s.cuda_stream, s)
            if l.record is not None:
                events[l.record] = s.record_event()
        for sid in used - {0}:
            main.wait_stream(streams[sid])
        # keep the events alive past this call: under HIP-graph capture they must outlive the capture
        # (destroying a recorded event while the capture is open crashed hipStreamEndCapture)
        self._live_events = (start, events)

    def __len__(self):
        return len(self.launches)

    def split(self) -> List["Phase"]:
        """Cut the phase at its pseudo-launches named ``cut`` into consecutive phases.

        Each piece is run (or captured) on its own: its side streams fork from stream 0 at its start and
        are joined back at its end, so an event recorded in an earlier piece is already ordered before
        the later one -- such waits are dropped.  Used to end the backward at gradient-bucket boundaries
        (DP: a bucket's all-reduce is issued between two pieces and overlaps the next one)."""
        pieces, cur = [], []
        for l in self.launches:
            if l.name == "cut":
                pieces.append(cur)
                cur = []
            else:
                cur.append(l)
        pieces.append(cur)
        out, recorded = [], set()
        for i, ls in enumerate(pieces):
            ph = Phase(f"{self.name}_{i}")
            ph.alias = dict(self.alias)
            for l in ls:
                w = tuple(t for t in l.waits if self.alias.get(t, t) not in recorded)
                ph.launches.append(Launch(l.name, l.fn, *l.args, owner=l.owner, stream=l.stream, waits=w,
                                          record=l.record, bucket=l.bucket))
            for l in ls:
                if l.record is not None:
                    recorded.add(l.record)
            out.append(ph)
        return out


# thin adapters giving every launch the signature fn(*args, stream)
def k_conv(mode, cfg, G, d, st):
    lib().conv(mode, cfg, G, st, d)


def k_wgrad(cfg, G, d, st):
    lib().wgrad(cfg, G, st, d)


def k_tail_fwd(kind, G, blocks, d, st):
    lib().tail_fwd(kind, G, blocks, st, d)


def k_tail_fwd_batched(kind, table, nj, nblocks, max_c, st):
    lib().tail_fwd_batched(kind, table.data_ptr(), nj, nblocks, max_c, st)


def k_tail_bwd_batched(kind, cgb, reduce, table, nj, nblocks, st):
    lib().tail_bwd_batched(kind, cgb, reduce, table.data_ptr(), nj, nblocks, st)


def k_tail_bwd(kind, G, blocks, d, st):
    lib().tail_bwd(kind, G, blocks, st, d)


def k_head(d, st):
    lib().mtl_head(st, d)


def k_cls_head(d, st):
    lib().cls_head(st, d)


def k_pool(is_max, bwd, d, st):
    lib().pool3(is_max, bwd, st, d)


def k_wgrad_batched(cfg, table, nj, nblocks, st):
    lib().wgrad_batched(cfg, table.data_ptr(), nj, nblocks, st)


def k_wgfin(table, nd, nblocks, st):
    lib().wgrad_finalize(table.data_ptr(), nd, nblocks, 1.0, st)


def k_adam(d, st):
    lib().adam_pack(st, d)


def k_allreduce(fn, t, st):
    """A collective inside a phase (SyncBN): Launch.__call__ makes the launch's stream current, so
    ``fn(tensor)`` (DistContext.all_reduce_ordered_) is ordered after that stream's previous launches and
    before its next ones."""
    fn(t.t if hasattr(t, "bind") else t)  # arena LazyView -> its bound tensor


def k_gather(X, idx, lab, lab_w, out, lab_out, B, Cin, H, W, taps, off, zero, st):
    lib().gather_batch(X.data_ptr(), idx.data_ptr(), lab.data_ptr(), lab_w, out.data_ptr(), lab_out.data_ptr(),
                       B, Cin, H, W, st, taps, off, zero)
