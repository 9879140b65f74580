"""Run-to-run determinism check used as a race detector.

The engine's training step is bitwise reproducible: every buffer is written by exactly one launch, the
only cross-block reductions are the BN replica sums (accumulated in fp64, so their atomic order cannot
change a rounded result) and the weight gradients go through a fixed-order split-M finalize.  A racing
kernel therefore shows up as a bitwise difference between two executions of the same step from the same
state.  ``check_step`` runs the step twice (eagerly, or as the captured graph) and reports the first
parameter-gradient tensor that differs; tools/dbg_race.py bisects down to the launch.
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
