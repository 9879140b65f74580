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
# hardware queues of this process (HIP's default 4): the budget for ALL streams a phase touches -- caller,
# compute side streams, communication and spill streams.  With more streams than queues a multi-stream
# graph segfaults inside the HIP runtime at replay (engine-free repro: tools/hwq_repro.py,
# profiles/r4_runtime_faults.txt).
HW_QUEUES = max(1, int(os.environ.get("GPU_MAX_HW_QUEUES", "4")))
# compute streams used at most (logical ids above are folded onto the last one -- still a valid schedule)
MAX_STREAMS = max(1, min(4, HW_QUEUES))
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
        if self.fn is k_ext_record:  # an external event: a graph event-record node under capture
            import torch
            self.args[0].record(torch.cuda.current_stream() if tstream is None else tstream)
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


def stream_slots(launches, hw_queues: int = None) -> dict:
    """Logical stream id -> physical slot for one phase, within the hardware-queue budget: slot 0 is the
    caller's stream, 1..MAX_STREAMS-1 the compute side streams, MAX_STREAMS the communication stream and
    MAX_STREAMS+1 the spill stream (EngineStreams order).  The communication and spill streams count
    against the budget: the compute streams shrink first (never below 1), then the spill and finally the
    communication stream fold onto the last compute stream (a valid schedule, less overlap)."""
    hwq = HW_QUEUES if hw_queues is None else hw_queues
    ids = {l.stream for l in launches}
    comm, spill = COMM_STREAM in ids, SPILL_STREAM in ids
    ncomp = max(1, min(MAX_STREAMS, hwq - comm - spill))
    room = hwq - ncomp
    own_comm = comm and room >= 1
    own_spill = spill and room >= 1 + own_comm
    out = {}
    for s in ids:
        if s == COMM_STREAM:
            out[s] = MAX_STREAMS if own_comm else ncomp - 1
        elif s == SPILL_STREAM:
            out[s] = MAX_STREAMS + 1 if own_spill else ncomp - 1
        else:
            out[s] = min(s, ncomp - 1)
    return out


class EngineStreams:
    """The HIP streams the engine runs its side branches on: one fixed set per device for the whole process,
    created with ``hipStreamCreateWithPriority`` by the extension (not drawn from torch's 32-entry
    round-robin pool, whose streams a phase could share with the graph-capture stream or another phase's
    streams), and released by :func:`release_streams` (atexit).  Index 0..MAX_STREAMS-2 are the compute
    side streams, then the communication and the spill stream; ``capture`` is the stream graphs are captured
    on."""

    _by_device = {}

    def __init__(self, device):
        import torch
        self.device = device
        n = MAX_STREAMS - 1 + 2
        self.handles = [lib().stream_create(0) for _ in range(n + 1)]
        self.streams = [torch.cuda.ExternalStream(h, device=device) for h in self.handles[:n]]
        # the communication stream (slot MAX_STREAMS): captured bucket collectives run on it inside a phase,
        # and the world > 1 step issues its eager bucket all-reduces on it (engine/step.py)
        self.comm = self.streams[MAX_STREAMS - 1]
        # graph captures and their eager warm-up runs (StepRunner, capture_graph): never a pool stream, so a
        # communicator's pool stream can never be the stream a graph is captured on
        self.capture = torch.cuda.ExternalStream(self.handles[n], device=device)

    @classmethod
    def get(cls, device):
        s = cls._by_device.get(device)
        if s is None:
            s = cls._by_device[device] = cls(device)
        return s

    def destroy(self):
        for h in self.handles:
            lib().stream_destroy(h)
        self.handles, self.streams, self.capture, self.comm = [], [], None, None


def release_streams():
    """Synchronize and destroy the engine's streams (safe to call more than once; they are re-created on
    demand)."""
    import torch
    if not EngineStreams._by_device:
        return
    torch.cuda.synchronize()
    for s in EngineStreams._by_device.values():
        s.destroy()
    EngineStreams._by_device.clear()


import atexit  # noqa: E402

atexit.register(release_streams)


class EventKeeper:
    """Owner of the events a phase records while a HIP graph is captured: their lifetime is tied to the
    graph (StepRunner keeps the keeper next to the graph executable and drops both together), so no phase
    re-run -- eager or another capture -- can destroy an event a live graph was built from."""

    active = None  # the keeper of the capture in progress, if any

    def __init__(self):
        self.events = []

    def __enter__(self):
        if EventKeeper.active is not None:
            raise RuntimeError("nested EventKeeper")
        EventKeeper.active = self
        return self

    def __exit__(self, *exc):
        EventKeeper.active = None
        return False


class Phase:
    def __init__(self, name: str):
        self.name = name
        self.launches: List[Launch] = []
        self._live_events = None
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
        keeper = EventKeeper.active
        if not MULTI_STREAM or all(l.stream == 0 and not l.waits for l in self.launches):
            st = stream() if st is None else st
            for l in self.launches:
                if l.fn is not None:
                    l(st)
            return
        main = torch.cuda.current_stream()
        es = EngineStreams.get(main.device)
        slot = stream_slots(self.launches)
        phys = {0: main}
        for sid in set(slot.values()) - {0}:
            phys[sid] = es.streams[sid - 1]
        start = main.record_event()
        for sid in phys:
            if sid:
                phys[sid].wait_event(start)
        events = {}
        for l in self.launches:
            s = phys[slot[l.stream]]
            for tag in l.waits:
                s.wait_event(events[self.alias.get(tag, tag)])
            l(s.cuda_stream, s)
            if l.record is not None:
                events[l.record] = s.record_event()
        for sid in phys:
            if sid:
                main.wait_stream(phys[sid])
        # keep the events alive past this call: under HIP-graph capture they must live as long as the graph
        # (destroying a recorded event while the capture is open crashed hipStreamEndCapture), so a capture's
        # events go to its EventKeeper; an eager run's are held until the phase runs again
        if keeper is not None:
            keeper.events.append((start, events))
        else:
            self._live_events = (start, events)

    def __len__(self):
        return len(self.launches)

    def release(self):
        """Drop the events of the last eager run (the caller has synchronized)."""
        self._live_events = None


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


def k_wgrad_batched(cfg, table, nj, nblocks, cap, st):
    lib().wgrad_batched(cfg, table.data_ptr(), nj, nblocks, st, cap)


def k_wgfin(table, nd, nblocks, st):
    lib().wgrad_finalize(table.data_ptr(), nd, nblocks, 1.0, st)


def k_adam(d, st):
    lib().adam_pack(st, d)


def k_step_inc(d, st):
    lib().step_inc(d["step"], d.get("cursor", 0), st)


class ExtEvent:
    """A HIP event recorded with ``hipEventRecordExternal`` while its stream captures (an event-record node of
    the graph, re-recorded at every replay), plainly otherwise; ``wait(stream)`` makes a torch stream wait for
    its latest record.  (PyTorch refuses ``torch.cuda.Event(external=True)`` on ROCm.)  ``destroy`` after the
    device has finished every graph that records it."""

    def __init__(self):
        self.handle = lib().event_create()

    def record(self, stream):
        lib().event_record_external(self.handle, stream.cuda_stream)

    def wait(self, stream):
        lib().stream_wait_event(stream.cuda_stream, self.handle)

    def destroy(self):
        if self.handle:
            lib().event_destroy(self.handle)
            self.handle = 0


def k_ext_record(ev, st):
    """Marker launch: record the EXTERNAL event ``ev`` (ExtEvent) on the launch's stream (Launch.__call__).  Captured, it is an event-record node of the graph: the host can order work
    issued after the replay -- an eager RCCL all-reduce on another stream -- after that point of the graph
    (engine/step.py, the data-parallel step at world > 1)."""
    raise RuntimeError("k_ext_record is dispatched by Launch.__call__")


def k_allreduce(fn, t, st):
    """A collective inside a phase (SyncBN): Launch.__call__ makes the launch's stream current, so
    ``fn(tensor)`` (DistContext.all_reduce_ordered_) is ordered after that stream's previous launches and
    before its next ones."""
    fn(t.t if hasattr(t, "bind") else t)  # arena LazyView -> its bound tensor


def k_gather(X, idx, lab, lab_w, out, lab_out, B, Cin, H, W, taps, off, zero, cursor, st):
    """``cursor``: None, or the device int64 cursor of a [nrows][B] batch-index schedule ``idx`` (StepRunner
    set_index_schedule): the kernel gathers row cursor mod nrows."""
    lib().gather_batch(X.data_ptr(), idx.data_ptr(), lab.data_ptr(), lab_w, out.data_ptr(), lab_out.data_ptr(),
                       B, Cin, H, W, st, taps, off, zero, cursor.data_ptr() if cursor is not None else 0,
                       idx.shape[0] if cursor is not None else 0)
