"""Run-to-run determinism check used as a race detector.

The engine's training step is bitwise reproducible: every buffer is written by exactly one launch, the
only cross-block reductions are the BN replica sums (accumulated in fp64, so their atomic order cannot
change a rounded result) and the weight gradients go through a fixed-order split-M finalize.  A racing
kernel therefore shows up as a bitwise difference between two executions of the same step from the same
state.  ``check_step`` runs the step twice (eagerly, or as the captured graph) and reports the first
parameter-gradient tensor that differs; ``first_divergent_launch`` bisects down to the launch.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch


def check_step(prog, X: torch.Tensor, labels: torch.Tensor, idx: torch.Tensor, use_graph: bool = False,
               runs: int = 2) -> Dict[str, object]:
    from .step import StepRunner
    f = prog.flat
    state = [f.params, f.exp_avg, f.exp_avg_sq, f.bn_mean, f.bn_var, f.bn_nbt, f.step] + \
        list(getattr(prog, "extra_state", []))  # e.g. Model C's dropout RNG counter
    saved = [t.clone() for t in state]
    grads, outs = [], []
    for _ in range(runs):
        for t, s in zip(state, saved):
            t.copy_(s)
        r = StepRunner(prog, X, labels, use_graph=use_graph, allreduce=lambda g: None)
        r.pack_weights()
        r.train_step(idx)
        torch.cuda.synchronize()
        grads.append(f.grads.clone())
        outs.append(prog.logp.clone())
    for t, s in zip(state, saved):
        t.copy_(s)
    first_diff: Optional[str] = None
    for p in f.order:
        o, n = f.off(p), p.numel()
        if any(not torch.equal(g[o:o + n], grads[0][o:o + n]) for g in grads[1:]):
            first_diff = next(name for name, q in f.module.named_parameters() if q is p)
            break
    return {"bitwise_equal": first_diff is None and all(torch.equal(o, outs[0]) for o in outs[1:]),
            "first_differing_parameter": first_diff,
            "max_abs_grad_diff": max(float((g - grads[0]).abs().max()) for g in grads[1:])}


# argument keys of a launch that point at buffers it WRITES (program launch dicts, engine/lowering.py)
_OUT_KEYS = ("out", "dy", "dy2", "side", "slab", "stats", "dfeat", "logp", "part", "dzbuf", "dx", "dlogits")


def _written_buffers(prog):
    """(base pointer, byte size, tensor) of every device buffer the program owns, for pointer lookup."""
    from .core import Act, LazyView
    acc, seen = [], set()

    def walk(o):
        if id(o) in seen:
            return
        seen.add(id(o))
        if isinstance(o, torch.Tensor):
            if o.is_cuda:
                acc.append(o)
        elif isinstance(o, LazyView):
            if o.t is not None:
                acc.append(o.t)
        elif isinstance(o, Act):
            walk(o.t)
        elif isinstance(o, dict):
            for v in o.values():
                walk(v)
        elif isinstance(o, (list, tuple)):
            for v in o:
                walk(v)
        elif hasattr(o, "__dict__") and type(o).__module__.startswith("mtl_das_pytorch_amd"):
            for v in vars(o).values():
                walk(v)

    walk(prog)
    regs = {}
    for t in acc + [prog.flat.grads]:
        st = t.untyped_storage()
        regs[st.data_ptr()] = (st.nbytes(), t)
    return sorted((b, n, t) for b, (n, t) in regs.items())


def first_divergent_launch(prog, X: torch.Tensor, labels: torch.Tensor, idx: torch.Tensor) -> Optional[dict]:
    """Race bisection: execute the forward + backward twice (after a warm-up) from the same state, eagerly and one launch at a
    time (serialised on one stream), snapshot every buffer each launch writes, and return the first launch
    whose output bytes differ between the two executions -- ``{"phase", "index", "launch", "arg"}`` -- or
    None when the step is bitwise reproducible.  The first divergence is the racing kernel (later launches
    only propagate it)."""
    from ..ops.hip import stream
    f = prog.flat
    regs = _written_buffers(prog)

    def region(p):
        for base, nb, t in regs:
            if base <= p < base + nb:
                return base, nb, t
        return None

    launches = [(ph.name, i, l) for ph in (prog.fwd_train, prog.bwd) for i, l in enumerate(ph.launches)]
    state = [f.params, f.exp_avg, f.exp_avg_sq, f.bn_mean, f.bn_var, f.bn_nbt, f.step] + \
        list(getattr(prog, "extra_state", []))
    saved = [t.clone() for t in state]

    def execute():
        for t, s in zip(state, saved):
            t.copy_(s)
        prog.opt["pack"].run()
        prog.arena.clear()
        prog.gather_phase(X, labels, idx).run()
        st, snaps = stream(), []
        for _, _, l in launches:
            if l.fn is None:
                snaps.append([])
                continue
            l(st)
            torch.cuda.synchronize()
            d = next((a for a in l.args if isinstance(a, dict)), {})
            out = []
            for k in _OUT_KEYS:
                v = d.get(k)
                r = region(v) if isinstance(v, int) and not isinstance(v, bool) and v else None
                if r is not None:
                    base, nb, t = r
                    out.append((k, torch.empty(0, dtype=torch.uint8, device=t.device).set_(t.untyped_storage()).clone()))
            if l.name == "wgrad_finalize":
                out.append(("grads", f.grads.clone()))
            snaps.append(out)
        return snaps

    # three executions, the first discarded: a buffer several launches write in parts (a fused conv's combined
    # dy, written slice by slice) holds the previous execution's bytes in its unwritten parts at a snapshot --
    # after a warm-up execution those are the same in both compared runs
    execute()
    a, b = execute(), execute()
    for t, s in zip(state, saved):
        t.copy_(s)
    for (phase, i, l), sa, sb in zip(launches, a, b):
        for (k, x), (_, y) in zip(sa, sb):
            if not torch.equal(x, y):
                return {"phase": phase, "index": i, "launch": l.name, "arg": k}
    return None
