"""Train / eval step execution for a lowered program, with HIP-graph capture.

A training step is

    [gather batch + zero the arena's accumulators] [forward] [backward]  ->  (DP: RCCL all-reduce of the flat
    gradient buckets)  ->  [fused Adam + bf16 re-pack] [step++]

Single GPU: the whole step is ONE captured HIP graph (``torch.cuda.CUDAGraph`` is a hipGraph on ROCm),
so a step costs one graph launch from the host.  Data parallel with capturable collectives (a 1-rank RCCL
group, see DistContext.capturable_collectives): still ONE graph -- the gradient buckets' all-reduces are
captured on a communication stream inside it (LoweredProgram.backward_with_allreduce), each waiting only for
its bucket's finalize.  Otherwise (the multi-rank default: RCCL collectives stay eager) forward + backward
are ONE graph that records an EXTERNAL event where each gradient bucket is complete
(LoweredProgram.backward_with_ext_events); after enqueuing its replay the host makes the communication
stream wait for bucket k's event and issues bucket k's asynchronous RCCL all-reduce there, so it runs while
the graph computes the rest of the backward; the optimizer graph waits for every bucket (Work.wait).

The batch indices come from a device-resident schedule (set_index_schedule: the gather reads the next row,
the optimizer kernel advances the cursor) or from a persistent device buffer the host refreshes before each
replay; the learning rate is a device scalar, so the reference's LR schedule never forces a re-capture.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional

import torch

from .program import EngineStreams, EventKeeper, ExtEvent, Phase


class StateSnapshot:
    """Save/restore every tensor a step mutates (used to make warm-up runs side-effect free)."""

    def __init__(self, tensors: List[torch.Tensor]):
        self.tensors = tensors
        self.saved = [t.detach().clone() for t in tensors]

    def restore(self):
        for t, s in zip(self.tensors, self.saved):
            t.copy_(s)


def capture_graph(fns, error_mode: str = "global"):
    """Capture ``fns`` (phase runs) into one HIP graph on the engine's capture stream.  Returns (graph,
    EventKeeper): the keeper holds the events the capture recorded and must live as long as the graph."""
    keeper = EventKeeper()
    g = torch.cuda.CUDAGraph()
    cap = EngineStreams.get(torch.cuda.current_stream().device).capture
    with keeper, torch.cuda.graph(g, stream=cap, capture_error_mode=error_mode):
        for f in fns:
            f()
    return g, keeper


class StepRunner:
    # Graphs are captured (and warmed up) on the engine's own capture stream (EngineStreams.capture), never on
    # torch's pool streams: the world > 1 data-parallel step ran 2.7x slower with pool capture streams (bench.py
    # --dp-shape 8 on Model A: 11.3 k -> 30.3 k samples/s, docs/PERF.md round 5).

    def __init__(self, program, X: torch.Tensor, labels: torch.Tensor, use_graph: bool = True,
                 allreduce: Optional[Callable[[torch.Tensor], None]] = None, X_eval: torch.Tensor = None,
                 labels_eval: torch.Tensor = None):
        self.p = program
        self.use_graph = use_graph and program.device.type == "cuda"
        self.allreduce = allreduce
        B = program.B
        self.idx = torch.zeros(B, dtype=torch.int64, device=program.device)
        self.sources = {"train": (X, labels)}
        if X_eval is not None:
            self.sources["eval"] = (X_eval, labels_eval)
        self.graphs: Dict[str, torch.cuda.CUDAGraph] = {}
        self.keepers: Dict[str, EventKeeper] = {}  # events each graph was captured with (same lifetime)
        self._packed = False
        self._bwd_dp = None
        self._bwd_ext = None
        # the DP step as one graph with the bucket collectives captured in it (FlatGradAllReducer.capturable)
        self.capture_dp = self.use_graph and allreduce is not None and getattr(allreduce, "capturable", False)
        # otherwise forward + backward as one graph with an external event per gradient bucket, the bucket
        # all-reduces issued eagerly on the communication stream after those events (train_step)
        self.ext_dp = self.use_graph and allreduce is not None and not self.capture_dp
        self.ext_events = None
        reducing = allreduce is not None and getattr(getattr(allreduce, "ctx", None), "enabled", False)
        if reducing and any(l.name == "adam_pack_early" for l in program.bwd.launches):
            # an update inside the backward would use local, un-reduced gradients
            raise ValueError("data-parallel step with weight updates inside the backward: call "
                             "set_optimizer(data_parallel=True) before autotune_program")
        if hasattr(program, "use_early_step_counter"):
            program.use_early_step_counter()  # the step counter off the step's tail (every step runs the forward)
        if hasattr(program, "check_sync_bn"):
            program.check_sync_bn()  # every SyncBN collective the program promised is in its launch lists
        self.buckets = list(getattr(program, "buckets", None) or [(0, program.flat.numel)])
        self.schedule = None  # [nrows][B] batch-index schedule (set_index_schedule)
        self.cursor = None

    def set_index_schedule(self, schedule: Optional[torch.Tensor]):
        """Train from a device-resident [nrows][B] batch-index schedule: ``train_step()`` without indices then
        gathers row (cursor mod nrows) and the step's optimizer kernel advances the cursor, so a replay is not
        preceded by a host-issued index copy (A: 6 us per step, tools/step_overhead.py).  The cursor restarts at
        row 0; None returns to per-call indices.  The training graphs are re-captured."""
        for kind in [k for k in self.graphs if k.startswith("train")]:
            self._drop_graph(kind)
        if schedule is None:
            self.schedule = self.cursor = None
            self.p.set_step_cursor(None)
            return
        if schedule.dim() != 2 or schedule.shape[1] != self.p.B or schedule.dtype != torch.int64:
            raise ValueError(f"index schedule must be int64 [nrows][{self.p.B}]")
        self.schedule = schedule.to(self.p.device).contiguous()
        self.cursor = torch.zeros(1, dtype=torch.int64, device=self.p.device)
        self.p.set_step_cursor(self.cursor)

    def restart_schedule(self, schedule: torch.Tensor):
        """Start the schedule over with new rows of the same shape (the next epoch): copied into the buffer the
        captured graphs read, cursor back to row 0, no re-capture."""
        if self.schedule is None or self.schedule.shape != schedule.shape:
            return self.set_index_schedule(schedule)
        self.schedule.copy_(schedule)
        self.cursor.zero_()

    # -------------------------------------------------------------------------------------------
    def _mutable_state(self) -> List[torch.Tensor]:
        f = self.p.flat
        return ([f.params, f.grads, f.exp_avg, f.exp_avg_sq, f.bn_mean, f.bn_var, f.bn_nbt, f.step, self.p.metrics,
                 self.p.confusion, self.p.logp] + list(getattr(self.p, "extra_state", []))
                + ([self.cursor] if self.cursor is not None else []))

    def pack_weights(self):
        """(Re)build the bf16 MFMA weight images from the fp32 masters (after init / load_state_dict)."""
        self.p.opt["pack"].run()
        self._packed = True

    def _phases(self, kind: str) -> List[Callable[[], None]]:
        p = self.p
        X, lab = self.sources["train" if kind.startswith("train") else "eval"]
        # a training step's gather also zeroes the arena's accumulators (one launch; arena.clear otherwise)
        sched = self.schedule is not None and kind.startswith("train")
        gather = p.gather_phase(X, lab, self.schedule if sched else self.idx, clear=kind.startswith("train"),
                                cursor=self.cursor if sched else None)
        if kind == "train_ext":
            if self._bwd_ext is None:
                self.ext_events = [ExtEvent() for _ in self.buckets]
                self._bwd_ext = p.backward_with_ext_events(self.ext_events)
            return [gather.run, p.fwd_train.run, self._bwd_ext.run]
        if kind == "train_compute":
            return [gather.run, p.fwd_train.run, p.bwd.run]
        if kind == "train_opt":
            return [p.opt["adam"].run]
        if kind == "train_full":
            return [gather.run, p.fwd_train.run, p.bwd.run, p.opt["adam"].run]
        if kind == "train_full_dp":
            if self._bwd_dp is None:
                self._bwd_dp = p.backward_with_allreduce(self.allreduce.ordered)
            return [gather.run, p.fwd_train.run, self._bwd_dp.run, p.opt["adam"].run]
        if kind == "eval":
            return [gather.run, p.fwd_eval.run]
        raise ValueError(kind)

    def _run(self, kind: str):
        if not self.use_graph:
            for f in self._phases(kind):
                f()
            return
        self._ensure_graph(kind)
        self.graphs[kind].replay()

    def _drop_graph(self, kind: str):
        """Release one captured graph and the events it was captured with, after the device has finished
        every replay of it (destroying an executable that may still run is undefined)."""
        g = self.graphs.pop(kind, None)
        if g is None:
            return
        torch.cuda.synchronize()
        g.reset()
        self.keepers.pop(kind, None)

    def _ensure_graph(self, kind: str):
        """Warm up (side effects rolled back) and capture the graph of ``kind`` once."""
        g = self.graphs.get(kind)
        if g is None:
            fns = self._phases(kind)
            snap = StateSnapshot(self._mutable_state())
            s = EngineStreams.get(torch.cuda.current_stream().device).capture
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):  # warm-up (loads code objects); side effects are rolled back
                for f in fns:
                    f()
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            snap.restore()
            self.p.opt["pack"].run()  # the bf16 weight images are derived state: rebuild from restored masters
            # Collectives captured here run on the capture-only RCCL communicator (DistContext.capture_group),
            # which never has eager work for the process-group watchdog to poll; the capture is thread-local
            # so that the watchdog's polls of the default communicator's eager work stay legal meanwhile.
            g, keeper = capture_graph(fns, "thread_local")
            torch.cuda.synchronize()
            self.graphs[kind] = g
            self.keepers[kind] = keeper

    # -------------------------------------------------------------------------------------------
    def set_lr(self, lr: float):
        self.p.flat.lr.fill_(float(lr))

    def train_step(self, idx: Optional[torch.Tensor] = None):
        """One training step on the batch ``idx`` -- or, with an index schedule set (set_index_schedule) and
        no ``idx``, on the schedule's next row."""
        if not self._packed:
            self.pack_weights()
        if idx is not None:
            if self.schedule is not None:
                raise ValueError("an index schedule is set: call train_step() without indices")
            self.idx.copy_(idx, non_blocking=True)
        elif self.schedule is None:
            raise ValueError("train_step() without indices needs set_index_schedule")
        if self.allreduce is None:
            self._run("train_full")
        elif self.capture_dp:
            self._run("train_full_dp")
        elif self.ext_dp:
            # one graph for forward + backward; bucket k's all-reduce is issued on the communication stream
            # behind the graph's external event k, so it overlaps the rest of the backward
            if not self.graphs.get("train_ext") or not self.graphs.get("train_opt"):
                self._ensure_graph("train_ext")  # both captured before any collective is in flight (the
                self._ensure_graph("train_opt")  # capture's state snapshot/restore must not race an all-reduce)
            self._run("train_ext")
            g = self.p.flat.grads
            if hasattr(self.allreduce, "start"):
                comm = EngineStreams.get(self.p.device).comm
                for ev, (lo, hi) in zip(self.ext_events, self.buckets):
                    ev.wait(comm)
                    with torch.cuda.stream(comm):
                        self.allreduce.start(g[lo:hi])
                self.allreduce.finish()
            else:  # a plain callable: the whole gradient, in stream order after the graph
                self.allreduce(g)
            self._run("train_opt")
        else:  # eager launches (no graphs): the whole gradient after the backward
            self._run("train_compute")
            self.allreduce(self.p.flat.grads)
            self._run("train_opt")

    def set_eval_source(self, X: torch.Tensor, labels: torch.Tensor):
        """Point the eval step at another resident set (the captured eval graph is rebuilt when the
        tensors differ: its gather launch holds their device pointers)."""
        cur = self.sources.get("eval")
        if cur is not None and cur[0] is X and cur[1] is labels:
            return
        self.sources["eval"] = (X, labels)
        self._drop_graph("eval")

    def eval_step(self, idx: torch.Tensor):
        if not self._packed:
            self.pack_weights()
        self.idx.copy_(idx, non_blocking=True)
        self._run("eval")

    def reset_metrics(self):
        self.p.metrics.zero_()
        self.p.confusion.zero_()

    def close(self):
        """Release every HIP object the runner and its program's phases hold -- graph executables with the
        events they were captured with, the phases' last eager events, the replay stream -- while the HIP runtime is certainly alive (at interpreter exit the
        order in which module globals, the runtime and these objects are finalised is not defined).  The
        runner can be used again afterwards (graphs are re-captured on demand)."""
        torch.cuda.synchronize()
        for k in list(self.graphs):
            self._drop_graph(k)
        p = self.p
        phases = [p.fwd_train, p.fwd_eval, p.bwd] + list(p.opt.values())
        phases += [ph for ph in (self._bwd_dp, self._bwd_ext) if ph is not None]
        for ph in phases:
            ph.release()
        self._bwd_dp = self._bwd_ext = None
        for ev in self.ext_events or []:
            ev.destroy()
        self.ext_events = None
        torch.cuda.synchronize()
