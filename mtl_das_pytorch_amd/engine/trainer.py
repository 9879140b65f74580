"""The generic multi-task trainer behind train.py / test.py.

One trainer replaces the reference's three near-identical loops (trainer_MTL, trainer_single_task,
trainer_multiClassifier; utils.py:226-793) and its orchestrator (main_process, utils.py:78-223):

  * model factory, output directory ``<out>/<%m-%d-%H_%M_%S> model_type=X is_test=Y/`` and console tee;
  * optional ``load_state_dict(strict=True)`` of a reference-format ``.pth``;
  * Adam(lr 1e-3, wd 1e-5); LR divided by 1.5 at every validation epoch (also epoch 0 for A/B, not for C);
  * epoch loop ``0..epoch_num``: validation every 5 epochs (before training that epoch), training for
    epochs ``< epoch_num``; every 100 batches the running loss/accuracy line and the ``train*Line.npy``
    curves; after each validation the ``test*Line.npy`` curves, and -- when the validation distance
    accuracy reaches 0.98 (A/B) / 0.95 (C) -- a ``{time}__{acc:.5f}_{epoch}.pth`` state_dict checkpoint
    plus ``confusion matrix <task> <acc> <epoch>.npy`` files;
  * after training the four curve PNGs, after testing the confusion-matrix SVGs.

Console lines and artefact names/formats follow the reference.  Documented fixes: runs with fewer than
100 batches per epoch no longer crash (curve files always exist); the single-task accuracy line prints
its value and the event-task matrix is saved under "event"; Model C's matrices get formatted names;
every validation also reports the distance MAE in metres (new metric).

Data parallel: one process per GPU (torchrun); each rank trains on its shard of every epoch's
permutation, gradients are all-reduced over RCCL, validation counters and confusion matrices are
summed, BN running statistics are averaged before validation, and only rank 0 writes files.
"""
from __future__ import annotations

import datetime
import os
import sys
import time
from typing import List, Optional

import numpy as np
import torch

from ..data.mat_dataset import Dataset_mat_MTL
from ..data.stream import DiskBatchStream
from ..data.synthetic import N_DIST, generate
from ..models import build_model
from ..parallel.dist import DistContext, ShardedIndexSampler, init_distributed
from ..utils.config import TrainConfig
from ..utils.logger import Logger
from ..utils.metrics import format_task_report, mae_from_confusion, metrics_from_confusion
from ..utils.plots import plot_confusion_files, plot_curves
from ..utils.profiling import phase_range
from .backends import EngineBackend, Metrics, TorchBackend, reduce_metrics


# ------------------------------------------------------------------------------------------------
def _labels_tensor(label_list, joint: bool) -> torch.Tensor:
    return torch.as_tensor(np.asarray(label_list, dtype=np.int64))


class ResidentSource:
    """A split resident in device memory (HBM on the GPU): batches are index tensors into ``X``."""

    def __init__(self, X: torch.Tensor, labels: torch.Tensor):
        self.X, self.labels = X, labels

    def __len__(self):
        return len(self.X)

    def batches(self, index_batches):
        """Yield (device index batch, size).  The whole epoch's indices go to the device in ONE copy
        (pinned host memory, non_blocking) and the batches are device slices: a per-batch pageable copy
        would make the host wait for the previous step's graph before it could launch the next one."""
        index_batches = list(index_batches)
        if not index_batches:
            return
        sizes = [int(b.numel()) for b in index_batches]
        flat = torch.cat([b.reshape(-1).to("cpu", torch.int64) for b in index_batches])
        if self.X.device.type == "cuda":
            flat = flat.pin_memory().to(self.X.device, non_blocking=True)
        o = 0
        for n in sizes:
            yield flat[o:o + n], n
            o += n

    def close(self):
        pass


def load_datasets(cfg: TrainConfig, device):
    """``(train, val)`` data sources (``ResidentSource`` or, with ``--dataset_ram False``, a
    ``DiskBatchStream``); labels are ``[N,2]`` (distance, event) or joint ``[N]``.  Test mode returns
    ``(None, test_set)``."""
    joint = cfg.model == "multi_classifier"
    if cfg.synthetic > 0:
        per = cfg.synthetic
        d = torch.arange(N_DIST).repeat_interleave(2 * per)
        e = torch.arange(2).repeat_interleave(per).repeat(N_DIST)
        seed = cfg.synthetic_seed + (7919 if cfg.is_test else 0)
        X, d_, e_ = generate(len(d), seed=seed, device="cpu", in_channels=cfg.in_channels, distance=d, event=e)
        lab = (d_ + N_DIST * e_) if joint else torch.stack([d_, e_], 1)
        if cfg.is_test:
            return None, ResidentSource(X.to(device), lab.to(device))
        # per-class KFold-like split: every 5th sample of each class goes to validation
        g = torch.Generator().manual_seed(cfg.random_state)
        perm = torch.randperm(len(d), generator=g)
        nval = max(1, len(d) // 5)
        val_idx, tr_idx = perm[:nval], perm[nval:]
        return (ResidentSource(X[tr_idx].to(device), lab[tr_idx].to(device)),
                ResidentSource(X[val_idx].to(device), lab[val_idx].to(device)))
    if cfg.is_test:
        dirs = (cfg.test_set_striking, cfg.test_set_excavating)
    else:
        dirs = (cfg.trainVal_set_striking, cfg.trainVal_set_excavating)
    ds = Dataset_mat_MTL(dirs[0], dirs[1], random_state=cfg.random_state, ram=cfg.dataset_ram, is_test=cfg.is_test,
                         fold_index=cfg.fold_index, multi_categories=joint, snr_db=cfg.snr_db, progress=False)
    if not cfg.dataset_ram:  # reference DatasetDisk: stream every epoch from disk through a bounded ring
        mk = lambda split: DiskBatchStream(ds.dataset[split], cfg.batch_size, device, ring=cfg.stream_ring,
                                           threads=cfg.loader_threads)
        return (None if cfg.is_test else mk("train")), mk("val")
    sources = []
    for split in ("train", "val"):
        x, y = ds.dataset[split].as_arrays()
        sources.append(ResidentSource(torch.as_tensor(x).to(device), torch.as_tensor(y).to(device)))
    return (None if cfg.is_test else sources[0]), sources[1]


class Trainer:
    def __init__(self, cfg: TrainConfig, ctx: Optional[DistContext] = None):
        self.cfg = cfg
        self.ctx = ctx or init_distributed()
        self.is_main = self.ctx.is_main
        use_gpu = cfg.GPU_device and torch.cuda.is_available()
        self.device = self.ctx.device if use_gpu else torch.device("cpu")
        torch.manual_seed(cfg.seed)
        self.model = build_model(cfg.model, in_channels=cfg.in_channels, head=cfg.head)
        note = "model_type={} is_test={}".format(cfg.model, cfg.is_test)
        stamp = datetime.datetime.now().strftime("%m-%d-%H_%M_%S")
        if self.ctx.enabled:  # every rank must agree on the directory name
            t = torch.tensor([float(datetime.datetime.now().timestamp())], dtype=torch.float64, device=self.ctx.device)
            self.ctx.broadcast_(t)
            stamp = datetime.datetime.fromtimestamp(float(t.item())).strftime("%m-%d-%H_%M_%S")
        self.save_dir = os.path.join(cfg.output_savedir, "{} {}".format(stamp, note)) + "/"
        self.resume_path = None
        if cfg.resume == "auto":
            # elastic restart: continue the newest run of this model type in the same directory
            self.resume_path = find_latest_resume(cfg.output_savedir, cfg.model)
            if self.resume_path:
                self.save_dir = os.path.dirname(self.resume_path) + "/"
        elif cfg.resume:
            self.resume_path = cfg.resume
        if self.is_main:
            os.makedirs(self.save_dir, exist_ok=True)
        self.logger = Logger("console output.log", self.save_dir, enabled=self.is_main,
                             append=self.resume_path is not None)
        if cfg.model_path and cfg.is_test:
            sd = torch.load(cfg.model_path, map_location="cpu", weights_only=True)
            self.model.load_state_dict(sd, strict=True)
        self.backend_name = self._pick_backend()

    def _pick_backend(self) -> str:
        c = self.cfg
        if c.head != "group_mean":  # the engine lowers the reference's parameter-free head only
            if c.backend == "engine":
                raise ValueError("--head fc runs on the plain-PyTorch backend (--backend torch / auto)")
            return "torch"
        if c.backend == "torch" or self.device.type != "cuda":
            return "torch"
        return "engine"

    def print(self, *a, **k):
        if self.is_main:
            print(*a, **k, file=self.logger)

    # --------------------------------------------------------------------------------------------
    def run(self):
        cfg = self.cfg
        self.print(os.path.abspath(__file__))
        self.train_src, self.val_src = load_datasets(cfg, self.device)
        if self.train_src is None:  # test mode evaluates the (whole) test set
            self.train_src = self.val_src
        X, Y, Xv, Yv = self.train_src.X, self.train_src.labels, self.val_src.X, self.val_src.labels
        kw = dict(ctx=self.ctx, batch=cfg.batch_size, lr=cfg.lr, weight_decay=cfg.weight_decay,
                  loss_weights=cfg.loss_weights)
        if self.backend_name == "engine":
            self.model.to(self.device)
            self.backend = EngineBackend(self.model, cfg.model, X, Y, Xv, Yv, use_graph=cfg.graph, tune=cfg.tune,
                                         seed=cfg.seed, sync_bn=cfg.sync_bn, **kw)
        else:
            if cfg.sync_bn and self.ctx.enabled:
                self.model = torch.nn.SyncBatchNorm.convert_sync_batchnorm(self.model)
            self.model.to(self.device)
            self.backend = TorchBackend(self.model, cfg.model, X, Y, Xv, Yv, **kw)
        self.n_train, self.n_val = len(self.train_src), len(self.val_src)
        self.print(f"backend: {self.backend_name}  device: {self.device}  world: {self.ctx.world}  "
                   f"train samples: {0 if cfg.is_test else self.n_train}  val samples: {self.n_val}")
        start_epoch, lr, val_done = 0, cfg.lr, False
        self.curves = {"trainAccLine": [[], []], "trainLossLine": [[], []], "testAccLine": [[], []],
                       "testLossLine": [[], []]}
        if self.resume_path:
            start_epoch, lr, val_done = self._load_resume(self.resume_path)
        self.lr = lr
        self.backend.set_lr(lr)
        self.global_step = 0
        self.fault = parse_fault_injection(self.ctx.rank)
        self.start_time = datetime.datetime.now()
        if cfg.model == "multi_classifier":
            self.print("{}：{}".format("Start Test" if cfg.is_test else "Start Training", self.start_time))
        sampler = ShardedIndexSampler(self.n_train, cfg.batch_size, self.ctx, shuffle=True, seed=cfg.seed)
        E = cfg.epoch_num
        for epoch in range(start_epoch, E + 1):
            if epoch % cfg.val_every == 0 and not (epoch == start_epoch and val_done):
                if cfg.model != "multi_classifier" or epoch != 0:
                    self.lr /= cfg.lr_decay
                    self.backend.set_lr(self.lr)
                self.validate(epoch)
                self._save_resume(epoch, val_done=True)
                if cfg.is_test:
                    break
            if epoch < E:
                self.train_epoch(epoch, sampler)
                self.print("Epoch {} finished！".format(epoch + 1))
                self._save_resume(epoch + 1, val_done=False)
        if self.is_main:
            if cfg.is_test:
                plot_confusion_files(self.save_dir)
            else:
                for name in ("trainAccLine", "trainLossLine"):
                    p = os.path.join(self.save_dir, name + ".npy")
                    if not os.path.exists(p):  # fewer than log_every batches ran: keep the artefact set complete
                        np.save(p, self._train_line(name))
                plot_curves(self.save_dir, cfg.model)
        self.ctx.barrier()
        self.close()
        return self.save_dir

    def close(self):
        """Release the backend's device objects (graphs, events, streams), the data sources and the log.
        ``run`` calls it at its end; ``evaluate`` still works afterwards (it re-captures its graph; call ``close``
        again when done)."""
        if getattr(self, "backend", None) is not None:
            self.backend.close()  # idempotent; graphs captured by a later ``evaluate`` are released again
        if getattr(self, "_closed", False):
            return
        self._closed = True
        for src in {id(self.train_src): self.train_src, id(self.val_src): self.val_src}.values():
            src.close()
        self.logger.save()
        self.logger.close()

    # --------------------------------------------------------------------------------------------
    def _train_line(self, name):
        rows = self.curves[name]
        if self.cfg.model in ("single_distance", "single_event"):
            return np.asarray([rows[0]], dtype=np.float64)
        return np.asarray(rows, dtype=np.float64)

    def train_epoch(self, epoch: int, sampler: ShardedIndexSampler):
        cfg, be = self.cfg, self.backend
        batches = sampler.epoch(epoch, "cpu")
        be.reset_metrics()
        last = be.read_metrics()
        prof = self._maybe_profiler(epoch)
        t_log = time.perf_counter()
        if hasattr(be, "set_epoch_schedule") and isinstance(self.train_src, ResidentSource) and batches:
            # the engine trains from a device-resident schedule of the epoch's batch indices (one copy per epoch;
            # the step's gather reads the next row, its optimizer kernel advances the cursor): the step bench.py
            # times, with no host-issued index copy before each graph replay
            be.set_epoch_schedule(torch.stack(batches).to(self.device))
            steps = ((None, len(b)) for b in batches)
        else:
            steps = self.train_src.batches(batches)
        for bi, (idx, _) in enumerate(steps):
            if self.fault is not None and self.global_step == self.fault:
                print(f"fault injection: rank {self.ctx.rank} exits at global step {self.global_step}",
                      file=sys.stderr, flush=True)
                self.logger.flush()
                os._exit(13)
            with phase_range("train_step"):
                be.train_batch(idx)
            self.global_step += 1
            if prof is not None:
                prof.step()
                if bi + 1 >= cfg.profile_steps:
                    prof.stop()
                    prof = None
                    self.print(f"profiler trace written to {self.save_dir}")
            if (bi + 1) % cfg.log_every == 0:
                now = be.read_metrics()
                delta = reduce_metrics(self.ctx, now - last)
                last = now
                nt = len(delta.names)
                acc = [float(delta.correct[t] / max(delta.count[t], 1)) for t in range(nt)]
                # reference: mean over the 100 batches of (batch-mean loss / batch size)
                loss = [float(delta.loss[t] / max(delta.count[t], 1) / cfg.batch_size) for t in range(nt)]
                if cfg.model == "multi_classifier":
                    loss = [loss[0], loss[0]]
                self.print("epoch-iteration:{}-{}, loss:{}, accuracy:{}".format(epoch + 1, bi + 1, loss, acc))
                self.print("time:{}".format(datetime.datetime.now() - self.start_time))
                if self.device.type == "cuda":
                    torch.cuda.synchronize()
                dt = time.perf_counter() - t_log
                t_log = time.perf_counter()
                self.print("throughput: {:.1f} samples/s ({} GPU(s), {:.3f} ms/step)".format(
                    cfg.log_every * cfg.batch_size * self.ctx.world / dt, self.ctx.world, 1e3 * dt / cfg.log_every))
                for t in range(2):
                    self.curves["trainLossLine"][t].append(loss[min(t, nt - 1)])
                    self.curves["trainAccLine"][t].append(acc[min(t, nt - 1)])
                if self.is_main:
                    np.save(os.path.join(self.save_dir, "trainLossLine"), self._train_line("trainLossLine"))
                    np.save(os.path.join(self.save_dir, "trainAccLine"), self._train_line("trainAccLine"))

    @torch.no_grad()
    def _eval_pass(self, src):
        """Evaluate a whole data source (sharded over ranks); returns the rank-summed metrics and the
        reference's validation loss numerator (sum of batch-mean losses, per task)."""
        cfg, be = self.cfg, self.backend
        be.reset_metrics()
        n = len(src)
        B = cfg.batch_size
        order = torch.arange(n)
        per = (n + self.ctx.world - 1) // self.ctx.world
        mine = order[self.ctx.rank * per:min(n, (self.ctx.rank + 1) * per)]
        chunks = [mine[i:i + B] for i in range(0, len(mine), B)]
        # reference loss: sum over batches of the batch-mean loss.  Every batch but the last is full, so
        # the sum is (loss over the full batches) / B + (last batch's loss) / its size: the metrics are read
        # back twice per validation instead of once per batch
        batch_means = np.zeros(len(be.names))
        before_tail = None
        for idx, nv in src.batches(chunks):
            if nv < B:
                before_tail = be.read_metrics()
            be.eval_batch(idx, nv)
        cur = be.read_metrics()
        if before_tail is None:
            batch_means += cur.loss / B
        else:
            batch_means += before_tail.loss / B + (cur.loss - before_tail.loss) / max(len(chunks[-1]), 1)
        m = reduce_metrics(self.ctx, cur)
        if self.ctx.enabled:
            bm = torch.tensor(batch_means, dtype=torch.float64, device=self.ctx.device)
            self.ctx.all_reduce_(bm)
            batch_means = bm.cpu().numpy()
        return m, batch_means

    @torch.no_grad()
    def evaluate(self, X: torch.Tensor, labels: torch.Tensor) -> dict:
        """Accuracy / MAE / loss of the current model on an arbitrary resident set (e.g. a held-out test
        set, or one at a given SNR) without touching curves, checkpoints or the LR schedule."""
        self.backend.sync_bn_stats()
        self.backend.set_eval_data(X, labels)
        try:
            m, batch_means = self._eval_pass(ResidentSource(X, labels))
        finally:
            self.backend.set_eval_data(self.val_src.X, self.val_src.labels)
        n = len(X)
        out = {"acc": {m.names[t]: m.acc(t) for t in range(len(m.names))},
               "loss": {m.names[t]: float(batch_means[t] / n) for t in range(len(m.names))}}
        if "distance" in m.names:
            cm = m.cm[m.names.index("distance")]
            out["mae_m"] = mae_from_confusion(cm)
            out["distance_cm"] = cm.tolist()
        return out

    @torch.no_grad()
    def validate(self, epoch: int):
        cfg, be = self.cfg, self.backend
        be.sync_bn_stats()
        n = self.n_val
        m, batch_means = self._eval_pass(self.val_src)
        nt = len(m.names)
        accs = [m.acc(t) for t in range(nt)]
        if cfg.model == "multi_classifier":
            val_loss = [batch_means[0] / n] * 2
        else:
            val_loss = [batch_means[t] / n for t in range(nt)]
        for t in range(2):
            self.curves["testLossLine"][t].append(float(val_loss[min(t, nt - 1)]))
            self.curves["testAccLine"][t].append(accs[min(t, nt - 1)])
        star = "*" * 50
        if cfg.model == "MTL":
            self.print("{}\nepoch:{}  Validation Accuracy: distance:{}  event:{}".format(star, epoch, accs[0], accs[1]))
        elif cfg.model == "multi_classifier":
            self.print("{}\nepoch:{}  Accuracy: distance:{}  event:{}".format(star, epoch + 1, accs[0], accs[1]))
        else:
            self.print("{}\nepoch:{}  Validation Accuracy: {}:{}".format(star, epoch, m.names[0], accs[0]))
        for t in range(nt):
            self.print(format_task_report("Task {}：{}".format(t + 1, m.names[t]), m.cm[t]))
        if "distance" in m.names:
            self.print("Distance MAE (m)：{}".format(mae_from_confusion(m.cm[m.names.index("distance")])))
        if self.is_main:
            if not cfg.is_test:
                np.save(os.path.join(self.save_dir, "testAccLine"), np.asarray(self.curves["testAccLine"]))
                np.save(os.path.join(self.save_dir, "testLossLine"), np.asarray(self.curves["testLossLine"]))
            acc1 = accs[0]
            if acc1 >= cfg.threshold:
                sd = {k: v.detach().cpu().clone() for k, v in self.model.state_dict().items()}
                name = "{}__{:.5f}_{}.pth".format(datetime.datetime.now().strftime("%Y_%m_%d__%H_%M_%S"), acc1, epoch)
                torch.save(sd, os.path.join(self.save_dir, name))
                for t in range(nt):
                    np.save(os.path.join(self.save_dir, "confusion matrix {} {:.5f} {}.npy".format(
                        m.names[t], accs[t], epoch)), m.cm[t])
        self.last_val = {"epoch": epoch, "acc": dict(zip(m.names, accs)), "loss": val_loss,
                         "mae_m": mae_from_confusion(m.cm[0]) if m.names[0] == "distance" else None}
        self.ctx.barrier()

    # --------------------------------------------------------------------------------------------
    def _maybe_profiler(self, epoch: int):
        """--profile_steps N: torch.profiler (Kineto/roctracer on ROCm) over the first N train steps of
        the first trained epoch, exported as a chrome trace into the run directory (rank 0)."""
        n = self.cfg.profile_steps
        if n <= 0 or not self.is_main or getattr(self, "_profiled", False):
            return None
        self._profiled = True
        acts = [torch.profiler.ProfilerActivity.CPU]
        if self.device.type == "cuda":
            acts.append(torch.profiler.ProfilerActivity.CUDA)
        path = os.path.join(self.save_dir, f"trace_epoch{epoch}.json")
        prof = torch.profiler.profile(activities=acts, on_trace_ready=lambda p: p.export_chrome_trace(path))
        prof.start()
        return prof

    def _save_resume(self, epoch: int, val_done: bool):
        """Resumable sidecar (never inside the reference-format .pth): weights, optimizer moments, next
        epoch, whether that epoch's validation (and LR decay) already ran, LR, RNG state and curves.
        Written atomically by rank 0 after every validation and every training epoch."""
        if not self.is_main or self.cfg.is_test:
            return
        st = {"epoch": epoch, "val_done": val_done, "lr": self.lr,
              "model": {k: v.detach().cpu().clone() for k, v in self.model.state_dict().items()},
              "optimizer": self.backend.optimizer_state(), "rng": torch.get_rng_state(),
              "curves": self.curves, "model_type": self.cfg.model, "global_step": self.global_step}
        tmp = os.path.join(self.save_dir, "last.resume.pt.tmp")
        torch.save(st, tmp)
        os.replace(tmp, os.path.join(self.save_dir, RESUME_NAME))

    def _load_resume(self, path: str):
        st = torch.load(path, map_location="cpu", weights_only=True)
        if st.get("model_type", self.cfg.model) != self.cfg.model:
            raise ValueError(f"{path} holds a {st['model_type']} run, not {self.cfg.model}")
        self.model.load_state_dict(st["model"], strict=True)
        self.backend.load_optimizer_state(st["optimizer"])
        if hasattr(self.backend, "after_load"):
            self.backend.after_load()
        torch.set_rng_state(st["rng"])
        if "curves" in st:
            self.curves = st["curves"]
        self.print(f"resumed from {path} at epoch {st['epoch']} (lr {st['lr']})")
        return int(st["epoch"]), float(st["lr"]), bool(st.get("val_done", True))


RESUME_NAME = "last.resume.pt"


def find_latest_resume(root: str, model_type: str) -> Optional[str]:
    """Newest ``last.resume.pt`` of a ``model_type`` run directly under ``root`` (training runs only)."""
    best, best_t = None, -1.0
    if not os.path.isdir(root):
        return None
    for d in os.listdir(root):
        p = os.path.join(root, d, RESUME_NAME)
        if f"model_type={model_type} is_test=False" in d and os.path.isfile(p):
            t = os.path.getmtime(p)
            if t > best_t:
                best, best_t = p, t
    return best


def parse_fault_injection(rank: int) -> Optional[int]:
    """MDA_FAULT_INJECT="rank=R,step=S": rank R exits (status 13) before global train step S -- only in
    the first attempt of an elastic job (TORCHELASTIC_RESTART_COUNT 0), so a restarted job runs through
    (SURVEY 5.3)."""
    spec = os.environ.get("MDA_FAULT_INJECT")
    if not spec or int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")) > 0:
        return None
    kv = dict(item.split("=") for item in spec.split(","))
    return int(kv["step"]) if int(kv.get("rank", 0)) == rank else None


def main_process(cfg: TrainConfig) -> str:
    """Reference-compatible orchestrator entry point (utils.main_process)."""
    return Trainer(cfg).run()
