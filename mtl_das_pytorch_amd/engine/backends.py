"""Execution backends used by the trainer.

``EngineBackend``  the MI355X path: the model lowered onto the HIP kernels (engine/mtl.py), bf16 MFMA
                   compute with fp32 masters, one HIP graph per step, fused Adam, on-device metrics.
``TorchBackend``   the reference-math path in plain PyTorch (fp32 autograd + torch.optim.Adam): runs on
                   the CPU (tests, BASELINE config #1 plumbing) and serves models not yet lowered.

Both expose the same interface: train/eval a batch given device indices into a resident dataset,
accumulate per-task loss sums / correct counts / confusion matrices, read them back only when the
trainer logs, and keep the reference ``state_dict`` format for checkpoints.

Reported tasks: Model A -> distance (16) + event (2); Model B -> its single task; Model C -> the joint
32-way label decoded into distance + event (plus the joint loss), as in reference utils.py:597-793.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..models import decode_joint, model_tasks
from ..parallel.dist import (DistContext, FlatGradAllReducer, average_, broadcast_module_state, calibrate_allreduce,
                             sum_)

N_DIST, N_EVENT = 16, 2


class Metrics:
    """Host-side view of the per-task accumulators."""

    def __init__(self, names: Sequence[str], ncls: Sequence[int]):
        self.names = list(names)
        self.ncls = list(ncls)
        self.loss = np.zeros(len(names))
        self.correct = np.zeros(len(names))
        self.count = np.zeros(len(names))
        self.cm = [np.zeros((n, n), dtype=np.int64) for n in ncls]

    def acc(self, t: int) -> float:
        return float(self.correct[t] / self.count[t]) if self.count[t] else 0.0

    def __sub__(self, o: "Metrics") -> "Metrics":
        m = Metrics(self.names, self.ncls)
        m.loss, m.correct, m.count = self.loss - o.loss, self.correct - o.correct, self.count - o.count
        m.cm = [a - b for a, b in zip(self.cm, o.cm)]
        return m


class Backend:
    model_type: str
    names: List[str]
    ncls: List[int]

    def set_lr(self, lr: float): ...
    def train_batch(self, idx: torch.Tensor): ...
    def eval_batch(self, idx: torch.Tensor, nvalid: int): ...
    def read_metrics(self) -> Metrics: ...
    def reset_metrics(self): ...
    def sync_bn_stats(self): ...
    def optimizer_state(self) -> dict: ...
    def load_optimizer_state(self, st: dict): ...
    def close(self): ...


def _report_tasks(model_type: str):
    if model_type == "MTL":
        return ["distance", "event"], [N_DIST, N_EVENT]
    if model_type == "single_distance":
        return ["distance"], [N_DIST]
    if model_type == "single_event":
        return ["event"], [N_EVENT]
    return ["distance", "event"], [N_DIST, N_EVENT]  # multi_classifier: decoded joint prediction


class TorchBackend(Backend):
    """Reference-math training in plain PyTorch (fp32)."""

    def __init__(self, model: nn.Module, model_type: str, X: torch.Tensor, labels: torch.Tensor,
                 X_eval: torch.Tensor, labels_eval: torch.Tensor, ctx: DistContext, batch: int, lr: float,
                 weight_decay: float, loss_weights: Sequence[float] = (1.0, 1.0)):
        self.model = model
        self.model_type = model_type
        self.ctx = ctx
        self.device = X.device
        self.X, self.labels, self.X_eval, self.labels_eval = X, labels, X_eval, labels_eval
        self.B = batch
        self.names, self.ncls = _report_tasks(model_type)
        self.loss_weights = list(loss_weights)
        self.opt = torch.optim.Adam(model.parameters(), lr=lr, weight_decay=weight_decay)
        self._m = Metrics(self.names, self.ncls)
        self._joint_loss = 0.0
        self._flat_grads = None
        broadcast_module_state(ctx, list(model.parameters()) + list(model.buffers()))

    def set_lr(self, lr: float):
        for g in self.opt.param_groups:
            g["lr"] = lr

    def _targets(self, lab: torch.Tensor):
        """Per-reported-task label vectors from the stored labels ([N,2] or joint [N])."""
        if self.model_type == "multi_classifier":
            d, e = decode_joint(lab)
            return [d, e], lab
        if self.model_type == "MTL":
            return [lab[:, 0], lab[:, 1]], None
        return [lab[:, 0] if self.model_type == "single_distance" else lab[:, 1]], None

    def _forward_losses(self, x, lab, train: bool, nvalid: Optional[int] = None):
        targets, joint = self._targets(lab)
        out = self.model(x)
        if self.model_type == "multi_classifier":
            if isinstance(out, tuple):
                out = out[0]
            loss_vec = F.cross_entropy(out, joint, reduction="none")
            pred = out.argmax(1)
            preds = list(decode_joint(pred))
            losses = [loss_vec, loss_vec]
            total = loss_vec.mean()
        else:
            outs = out if isinstance(out, tuple) else (out,)
            losses = [F.nll_loss(o, t, reduction="none") for o, t in zip(outs, targets)]
            preds = [o.argmax(1) for o in outs]
            w = self.loss_weights if len(outs) > 1 else [1.0]
            total = sum(wi * l.mean() for wi, l in zip(w, losses))
        n = len(lab) if nvalid is None else nvalid
        with torch.no_grad():
            for t in range(len(self.names)):
                self._m.loss[t] += float(losses[t][:n].sum())
                self._m.correct[t] += float((preds[t][:n] == targets[t][:n]).sum())
                self._m.count[t] += n
                np.add.at(self._m.cm[t], (targets[t][:n].cpu().numpy(), preds[t][:n].cpu().numpy()), 1)
        return total

    def train_batch(self, idx: torch.Tensor):
        self.model.train()
        x, lab = self.X[idx], self.labels[idx]
        loss = self._forward_losses(x, lab, True)
        self.opt.zero_grad(set_to_none=False)
        loss.backward()
        if self.ctx.enabled:
            params = [p for p in self.model.parameters() if p.grad is not None]
            flat = torch.cat([p.grad.reshape(-1) for p in params])
            FlatGradAllReducer(self.ctx)(flat)
            flat /= self.ctx.world
            o = 0
            for p in params:
                n = p.numel()
                p.grad.copy_(flat[o:o + n].view_as(p))
                o += n
        self.opt.step()

    def set_eval_data(self, X: torch.Tensor, labels: torch.Tensor):
        self.X_eval, self.labels_eval = X, labels

    @torch.no_grad()
    def eval_batch(self, idx: torch.Tensor, nvalid: int):
        self.model.eval()
        self._forward_losses(self.X_eval[idx], self.labels_eval[idx], False, nvalid)

    def read_metrics(self) -> Metrics:
        m = Metrics(self.names, self.ncls)
        m.loss, m.correct, m.count = self._m.loss.copy(), self._m.correct.copy(), self._m.count.copy()
        m.cm = [c.copy() for c in self._m.cm]
        return m

    def reset_metrics(self):
        self._m = Metrics(self.names, self.ncls)

    def sync_bn_stats(self):
        average_(self.ctx, [b for n, b in self.model.named_buffers() if b.is_floating_point()])

    def optimizer_state(self) -> dict:
        names = {id(p): n for n, p in self.model.named_parameters()}
        moments, step = {}, 0.0
        for p in self.model.parameters():
            s = self.opt.state.get(p)
            if s:
                moments[names[id(p)]] = (s["exp_avg"].detach().cpu().clone(), s["exp_avg_sq"].detach().cpu().clone())
                step = float(s["step"])
        return {"adam_by_name": moments, "adam_step": step}

    def load_optimizer_state(self, st: dict):
        moments, step = portable_adam_state(st, self.model)
        for n, p in self.model.named_parameters():
            if n in moments:
                m, v = moments[n]
                self.opt.state[p] = {"step": torch.tensor(step), "exp_avg": m.to(p.device).view_as(p).clone(),
                                     "exp_avg_sq": v.to(p.device).view_as(p).clone()}


class EngineBackend(Backend):
    """The MI355X HIP engine: Models A/B lowered by engine/mtl.py, Model C by engine/inception.py."""

    def __init__(self, model: nn.Module, model_type: str, X: torch.Tensor, labels: torch.Tensor,
                 X_eval: torch.Tensor, labels_eval: torch.Tensor, ctx: DistContext, batch: int, lr: float,
                 weight_decay: float, loss_weights: Sequence[float] = (1.0, 1.0), use_graph: bool = True,
                 tune: bool = False, seed: int = 0, sync_bn: bool = False):
        from .inception import InceptionProgram
        from .lowering import build_for_stream_buckets
        from .mtl import MTLProgram
        from .step import StepRunner
        from .tune import autotune_program
        self.model_type = model_type
        self.ctx = ctx
        self.names, self.ncls = _report_tasks(model_type)
        sync = sync_bn and ctx.enabled
        sw = ctx.world if sync else 1

        def make(order=None):
            if model_type == "multi_classifier":
                p = InceptionProgram(model, batch, ctx.device, in_hw=tuple(X.shape[2:]), sync_world=sw,
                                     param_order=order)
            else:
                w = list(loss_weights) if model_type == "MTL" else [1.0]
                p = MTLProgram(model, batch, ctx.device, in_hw=tuple(X.shape[2:]), loss_weights=w, sync_world=sw)
            if sync:  # SyncBN: BN statistics all-reduced inside the step (captured into the HIP graph on RCCL)
                p.enable_sync_bn(ctx.all_reduce_ordered_)
            p.set_optimizer(betas=(0.9, 0.999), eps=1e-8, weight_decay=weight_decay, grad_scale=1.0 / ctx.world,
                            data_parallel=ctx.enabled)
            if hasattr(p, "set_rng_stream"):
                p.set_rng_stream(seed, ctx.rank)
            return p

        self.prog = make()
        if sync and not ctx.capturable_collectives:
            # gloo (or MDA_CAPTURE_COLLECTIVES=0): the step runs its launches and collectives eagerly -- say so,
            # this is several times slower
            if ctx.is_main:
                print("SyncBN: collectives are not captured on this process group; the training step runs "
                      "eagerly", flush=True)
            use_graph = False
        nb = self.prog.dp_buckets(ctx.world, calibrate_allreduce(ctx, self.prog.flat.numel))
        # captured collectives (a 1-rank RCCL group): the backward cut at the bucket boundaries; several ranks
        # (eager RCCL behind the step graph's external bucket events): side-stream buckets, no cut (Model C
        # rebuilt with its side streams' parameters grouped, build_for_stream_buckets)
        captured = ctx.capturable_collectives and (sync or ctx.capture_gradients)
        ext_form = ctx.enabled and not captured and use_graph
        if ext_form and nb > 1:
            first = [self.prog]
            self.prog = None

            def tuned(order):
                p = first.pop() if (order is None and first) else make(order)
                p.segment_backward(1)
                autotune_program(p, measure=tune)
                return p

            self.prog, _ = build_for_stream_buckets(tuned, nb)
        else:
            self.prog.segment_backward(1 if ext_form else nb)
            autotune_program(self.prog, measure=tune)
        f = self.prog.flat
        broadcast_module_state(ctx, [f.params, f.bn_mean, f.bn_var, f.bn_nbt])
        lab_eval = labels_eval if labels_eval is not None else labels
        self.runner = StepRunner(self.prog, X, labels, use_graph=use_graph,
                                 allreduce=FlatGradAllReducer(ctx, capture=captured) if ctx.enabled else None,
                                 X_eval=X_eval if X_eval is not None else X, labels_eval=lab_eval)
        self.runner.set_lr(lr)
        self.B = batch

    def set_lr(self, lr: float):
        self.runner.set_lr(lr)

    def train_batch(self, idx: Optional[torch.Tensor]):
        """One step on the batch ``idx`` -- or, after set_epoch_schedule and with ``idx`` None, on the schedule's
        next row."""
        self.runner.train_step(idx)

    def set_epoch_schedule(self, schedule: torch.Tensor):
        """Train the coming steps from the device-resident [nbatches][B] index schedule (StepRunner.
        set_index_schedule).  An epoch of the same shape reuses the schedule buffer the captured graph reads
        (copy + cursor reset, no re-capture)."""
        self.runner.restart_schedule(schedule.to(torch.int64))

    def set_eval_data(self, X: torch.Tensor, labels: torch.Tensor):
        self.runner.set_eval_source(X, labels)

    def eval_batch(self, idx: torch.Tensor, nvalid: int):
        if idx.numel() < self.B:  # pad the last batch (BN uses running stats in eval: padding is inert)
            idx = torch.cat([idx, idx[:1].expand(self.B - idx.numel())])
        self.prog.nvalid.fill_(nvalid)
        self.runner.eval_step(idx)
        self.prog.nvalid.fill_(self.B)

    def read_metrics(self) -> Metrics:
        met = self.prog.metrics.detach().double().cpu().numpy()
        conf = self.prog.confusion.detach().cpu().numpy().astype(np.int64)
        m = Metrics(self.names, self.ncls)
        if self.model_type == "multi_classifier":
            # rows: joint, distance, event; the joint CE loss is reported for both decoded tasks
            for t in range(2):
                m.loss[t], m.correct[t], m.count[t] = met[0, 0], met[1 + t, 1], met[1 + t, 2]
                n = self.ncls[t]
                m.cm[t] = conf[t, :n, :n].copy()
            return m
        for t in range(len(self.names)):
            m.loss[t], m.correct[t], m.count[t] = met[t, 0], met[t, 1], met[t, 2]
            n = self.ncls[t]
            m.cm[t] = conf[t, :n, :n].copy()
        return m

    def reset_metrics(self):
        self.runner.reset_metrics()

    def sync_bn_stats(self):
        f = self.prog.flat
        average_(self.ctx, [f.bn_mean, f.bn_var])

    def optimizer_state(self) -> dict:
        f = self.prog.flat
        moments = {}
        for n, p in self.prog.model.named_parameters():
            o = f.off(p)
            moments[n] = (f.exp_avg[o:o + p.numel()].detach().cpu().clone().view_as(p),
                          f.exp_avg_sq[o:o + p.numel()].detach().cpu().clone().view_as(p))
        st = {"adam_by_name": moments, "adam_step": float(f.step.item())}
        if hasattr(self.prog, "seed"):  # Model C's dropout RNG counter (stream + step)
            st["dropout_counter"] = int(self.prog.seed.item())
        return st

    def load_optimizer_state(self, st: dict):
        f = self.prog.flat
        moments, step = portable_adam_state(st, self.prog.model)
        for n, p in self.prog.model.named_parameters():
            if n in moments:
                o = f.off(p)
                f.exp_avg[o:o + p.numel()].copy_(moments[n][0].reshape(-1))
                f.exp_avg_sq[o:o + p.numel()].copy_(moments[n][1].reshape(-1))
        f.step.fill_(step)
        if "dropout_counter" in st and hasattr(self.prog, "seed"):
            # keep this rank's stream (high word), continue the saved step count (low word)
            cur = int(self.prog.seed.item())
            self.prog.seed.fill_((cur & ~0xFFFFFFFF) | (int(st["dropout_counter"]) & 0xFFFFFFFF))

    def after_load(self):
        """Re-pack bf16 weight images after the fp32 masters were overwritten (checkpoint load)."""
        self.runner.pack_weights()

    def close(self):
        """Release the step runner's graphs, captured events and replay stream (Trainer.run's exit)."""
        self.runner.close()


def portable_adam_state(st: dict, model: nn.Module):
    """Adam moments keyed by parameter name + the step count, from a resume sidecar written by either
    backend (so an engine run resumes under --dtype fp32 and vice versa).  Raises when the sidecar holds no
    optimizer state this model can use, instead of silently restarting the moments."""
    names = [n for n, _ in model.named_parameters()]
    if "adam_by_name" in st:
        moments, step = st["adam_by_name"], float(st["adam_step"])
    else:
        raise ValueError(f"resume sidecar has no portable Adam state (keys: {sorted(st)})")
    missing = [n for n in names if n not in moments]
    if missing and moments:
        raise ValueError(f"resume sidecar lacks Adam moments for {len(missing)} parameters, e.g. {missing[:3]}")
    return moments, step


def reduce_metrics(ctx: DistContext, m: Metrics) -> Metrics:
    """C3: sum counters and confusion matrices over ranks."""
    if not ctx.enabled:
        return m
    t = torch.tensor(np.concatenate([m.loss, m.correct, m.count] + [c.reshape(-1) for c in m.cm]),
                     dtype=torch.float64, device=ctx.device)
    sum_(ctx, [t])
    a = t.cpu().numpy()
    k = len(m.names)
    out = Metrics(m.names, m.ncls)
    out.loss, out.correct, out.count = a[:k], a[k:2 * k], a[2 * k:3 * k]
    o = 3 * k
    for i, n in enumerate(m.ncls):
        out.cm[i] = a[o:o + n * n].reshape(n, n).round().astype(np.int64)
        o += n * n
    return out
