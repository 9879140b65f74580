"""Sliding-window inference over long DAS recordings.

A recording is a (fiber position x time) matrix, usually much larger than the 100 x 250 window the
models are trained on.  It is cut into windows with a configurable stride; the windows are sharded over
the data-parallel ranks, evaluated, and the per-window predictions (distance bin, event type and class
probabilities) are gathered on every rank.  This is batch growth, served by data parallelism, not a
sequence-parallel scheme (there is no sequence dimension in these models).

Execution: on a GPU the window batches run through the lowered HIP engine's eval program (bf16 MFMA,
BN with running statistics, one HIP graph per batch); elsewhere through the PyTorch module in fp32.
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .models import decode_joint
from .parallel.dist import DistContext

WINDOW = (100, 250)


def window_starts(length: int, win: int, stride: int) -> np.ndarray:
    """Window start offsets covering ``[0, length)``; the last window is aligned to the end so every
    sample is covered (no partial windows)."""
    if length < win:
        raise ValueError(f"recording dimension {length} is shorter than the window {win}")
    starts = list(range(0, length - win + 1, stride))
    if starts[-1] != length - win:
        starts.append(length - win)
    return np.asarray(starts, dtype=np.int64)


def sliding_windows(rec: torch.Tensor, window: Tuple[int, int] = WINDOW, stride: Tuple[int, int] = (100, 125)):
    """``rec``: [F, T] or [C, F, T].  Returns (tiles [N, C, wf, wt], positions [N, 2] = (f0, t0))."""
    if rec.dim() == 2:
        rec = rec.unsqueeze(0)
    C, Fn, Tn = rec.shape
    fs, ts = window_starts(Fn, window[0], stride[0]), window_starts(Tn, window[1], stride[1])
    tiles = rec.unfold(1, window[0], 1).unfold(2, window[1], 1)  # [C, F', T', wf, wt] (views)
    sel = tiles[:, fs][:, :, ts]                                      # [C, nf, nt, wf, wt]
    out = sel.permute(1, 2, 0, 3, 4).reshape(len(fs) * len(ts), C, window[0], window[1]).contiguous()
    pos = np.stack(np.meshgrid(fs, ts, indexing="ij"), -1).reshape(-1, 2)
    return out, pos


def _shard(n: int, ctx: Optional[DistContext]) -> Tuple[int, int]:
    if ctx is None or not ctx.enabled:
        return 0, n
    per = (n + ctx.world - 1) // ctx.world
    return min(n, ctx.rank * per), min(n, (ctx.rank + 1) * per)


def _torch_probs(model: nn.Module, model_type: str, x: torch.Tensor) -> Sequence[torch.Tensor]:
    out = model(x)
    if model_type == "multi_classifier":
        return [torch.softmax(out[0] if isinstance(out, tuple) else out, 1)]
    outs = out if isinstance(out, tuple) else (out,)
    return [o.exp() for o in outs]  # A/B heads emit log-probabilities


@torch.no_grad()
def predict_recording(model: nn.Module, model_type: str, rec: torch.Tensor, stride=(100, 125), batch: int = 32,
                      ctx: Optional[DistContext] = None, device=None, use_engine: Optional[bool] = None) -> Dict:
    """Per-window predictions for one recording.  Returns numpy arrays: ``positions`` [N, 2], and per task
    (``distance`` / ``event`` as the model provides) ``<task>_pred`` [N] and ``<task>_prob`` [N, k]."""
    device = torch.device(device) if device is not None else (ctx.device if ctx else torch.device("cpu"))
    tiles, pos = sliding_windows(rec.float(), stride=stride)
    n = len(tiles)
    lo, hi = _shard(n, ctx)
    mine = tiles[lo:hi].to(device)
    if use_engine is None:
        use_engine = device.type == "cuda"
    names = {"MTL": ["distance", "event"], "single_distance": ["distance"], "single_event": ["event"],
             "multi_classifier": ["joint"]}[model_type]
    ncls = {"distance": 16, "event": 2, "joint": model.num_classes if model_type == "multi_classifier" else 0}
    probs = [torch.zeros(n, ncls[t], device=device) for t in names]
    if len(mine):
        if use_engine:
            chunks = _engine_probs(model, model_type, mine, batch, device)
        else:
            model.eval().to(device)
            chunks = [[] for _ in names]
            for i in range(0, len(mine), batch):
                for t, p in enumerate(_torch_probs(model, model_type, mine[i:i + batch])):
                    chunks[t].append(p)
            chunks = [torch.cat(c) for c in chunks]
        for t in range(len(names)):
            probs[t][lo:hi] = chunks[t].float()
    if ctx is not None and ctx.enabled:  # every rank wrote its own rows; the sum is the gather
        for p in probs:
            ctx.all_reduce_(p)
    res = {"positions": pos}
    if model_type == "multi_classifier":
        joint = probs[0].argmax(1)
        d, e = decode_joint(joint)
        res.update(joint_pred=joint.cpu().numpy(), joint_prob=probs[0].cpu().numpy(), distance_pred=d.cpu().numpy(),
                   event_pred=e.cpu().numpy())
    else:
        for t, name in enumerate(names):
            res[f"{name}_pred"] = probs[t].argmax(1).cpu().numpy()
            res[f"{name}_prob"] = probs[t].cpu().numpy()
    return res


def _engine_probs(model: nn.Module, model_type: str, x: torch.Tensor, batch: int, device) -> Sequence[torch.Tensor]:
    """Eval-mode forward of the lowered program over window batches (the last batch padded)."""
    from .engine.step import StepRunner
    n = len(x)
    if model_type == "multi_classifier":
        from .engine.inception import InceptionProgram
        prog = InceptionProgram(model, batch, device, in_hw=tuple(x.shape[2:]), p_drop=0.0)
        labels = torch.zeros(n, dtype=torch.int64, device=device)
    else:
        from .engine.mtl import MTLProgram
        prog = MTLProgram(model, batch, device, in_hw=tuple(x.shape[2:]))
        labels = torch.zeros(n, 2, dtype=torch.int64, device=device)
    from .engine.tune import autotune_program
    autotune_program(prog, measure=False)
    runner = StepRunner(prog, x, labels, use_graph=True, X_eval=x, labels_eval=labels)
    outs = [[] for _ in range(1 if model_type == "multi_classifier" else prog.T)]
    for i in range(0, n, batch):
        idx = torch.arange(i, min(n, i + batch), device=device)
        m = idx.numel()
        if m < batch:
            idx = torch.cat([idx, idx[:1].expand(batch - m)])
        runner.eval_step(idx)
        if model_type == "multi_classifier":
            outs[0].append(torch.softmax(prog.logp[:m], 1).clone())
        else:
            for t in range(prog.T):
                k = 16 if prog.lab_off[t] == 0 else 2
                outs[t].append(prog.logp[t, :m, :k].exp().clone())
    return [torch.cat(o) for o in outs]
