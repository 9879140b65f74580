"""Run configuration and the train.py / test.py command lines.

Flag names and defaults are identical to the reference (train.py:7-26, test.py:7-26).  Documented
deviations:
  * boolean flags are parsed (``--GPU_device False`` means False; the reference's ``type=bool`` turns
    every non-empty string into True);
  * test.py's ``--test_set_striking`` default typo ('E:./dataset/striking_test') is fixed;
  * every hyper-parameter the reference hard-codes is a flag with the reference value as default.
"""
from __future__ import annotations

import argparse
from dataclasses import dataclass, field
from typing import List, Optional


def str2bool(v) -> bool:
    if isinstance(v, bool):
        return v
    s = str(v).strip().lower()
    if s in ("1", "true", "t", "yes", "y", "on"):
        return True
    if s in ("0", "false", "f", "no", "n", "off", ""):
        return False
    raise argparse.ArgumentTypeError(f"not a boolean: {v!r}")


@dataclass
class TrainConfig:
    model: str = "MTL"
    running_mode: Optional[str] = None
    GPU_device: bool = True
    batch_size: int = 32
    epoch_num: int = 40
    random_state: int = 1
    fold_index: Optional[int] = 0
    output_savedir: str = "./"
    model_path: Optional[str] = None
    dataset_ram: bool = True
    trainVal_set_striking: str = "./dataset/striking_train"
    trainVal_set_excavating: str = "./dataset/excavating_train"
    test_set_striking: str = "./dataset/striking_test"
    test_set_excavating: str = "./dataset/excavating_test"
    # --- extensions (reference values as defaults) ---
    lr: float = 1e-3                      # utils.py:133
    weight_decay: float = 1e-5            # utils.py:134
    lr_decay: float = 1.5                 # utils.py:232
    val_every: int = 5                    # utils.py:245
    log_every: int = 100                  # utils.py:382
    save_threshold: Optional[float] = None  # 0.98 (A/B) / 0.95 (C), utils.py:329,716
    loss_weights: List[float] = field(default_factory=lambda: [1.0, 1.0])  # utils.py:367 (unweighted sum)
    in_channels: int = 1
    head: str = "group_mean"              # group_mean (reference) | fc (ablation, plain-PyTorch backend only)
    backend: str = "auto"                 # auto | engine | torch
    synthetic: int = 0                    # >0: N synthetic samples per (distance, event) class, no dataset needed
    synthetic_seed: int = 0
    snr_db: Optional[float] = None        # optional SNR noise injection (reference add_gaussian, disabled there)
    seed: int = 0
    graph: bool = True
    tune: bool = False
    resume: Optional[str] = None          # path to a *.resume.pt sidecar, or "auto" (newest under output_savedir)
    dtype: Optional[str] = None           # bf16 -> HIP engine, fp32 -> plain PyTorch (alias of --backend)
    sync_bn: bool = False                 # all-reduce BN batch statistics across ranks (engine and torch backends)
    profile_steps: int = 0                # >0: torch.profiler trace of that many train steps (rank 0)
    debug: bool = False                   # serialised kernels + blocking launches, no HIP graphs
    stream_ring: int = 4                  # --dataset_ram False: batches in flight (disk -> pinned -> HBM ring)
    loader_threads: int = 8               # native .mat reader threads (csrc/matio.cpp)
    is_test: bool = False

    @property
    def threshold(self) -> float:
        if self.save_threshold is not None:
            return self.save_threshold
        return 0.95 if self.model == "multi_classifier" else 0.98


def build_parser(is_test: bool) -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="Model test" if is_test else "Model Training")
    ap.add_argument("--model", type=str, default="MTL",
                    help="The used model type: MTL, single_event, single_distance, multi_classifier")
    ap.add_argument("--running_mode", type=str, help="running mode: train, test")
    ap.add_argument("--GPU_device", default=True, type=str2bool, help="Whether to use GPU")
    ap.add_argument("--batch_size", default=32, type=int, help="The batch size for training or test")
    ap.add_argument("--epoch_num", default=40, type=int, help="The Training epoch")
    ap.add_argument("--random_state", default=1, type=int, help="The random state for dataset divison")
    ap.add_argument("--fold_index", default=0, type=int,
                    help="The fold index in five-fold cross validation (-1: 70/15 train_test_split)")
    ap.add_argument("--output_savedir", default="./", type=str, help="The saving directory for output files")
    ap.add_argument("--model_path", default="./", type=str, help="The path of saved model")
    ap.add_argument("--dataset_ram", default=True, type=str2bool,
                    help="Whether to put all the dataset into the memory during training")
    ap.add_argument("--trainVal_set_striking", default="./dataset/striking_train", type=str,
                    help="Path of Training and validation dataset for striking event")
    ap.add_argument("--trainVal_set_excavating", default="./dataset/excavating_train", type=str,
                    help="Path of Training and validation dataset for excavating event")
    ap.add_argument("--test_set_striking", default="./dataset/striking_test", type=str,
                    help="Path of test dataset for striking event")
    ap.add_argument("--test_set_excavating", default="./dataset/excavating_test", type=str,
                    help="Path of test dataset for excavating event")
    g = ap.add_argument_group("extensions")
    g.add_argument("--lr", type=float, default=1e-3)
    g.add_argument("--weight_decay", type=float, default=1e-5)
    g.add_argument("--lr_decay", type=float, default=1.5, help="LR divisor applied at every validation epoch")
    g.add_argument("--val_every", type=int, default=5)
    g.add_argument("--log_every", type=int, default=100)
    g.add_argument("--save_threshold", type=float, default=None)
    g.add_argument("--loss_weights", type=str, default="1,1", help="w_distance,w_event for the MTL loss")
    g.add_argument("--in_channels", type=int, default=1)
    g.add_argument("--head", choices=["group_mean", "fc"], default="group_mean",
                   help="A / B classifier head: the reference's group mean, or a learned linear layer per task "
                        "(backbone-vs-head ablation; trains on the plain-PyTorch backend)")
    g.add_argument("--backend", choices=["auto", "engine", "torch"], default="auto",
                   help="engine = MI355X HIP engine (bf16), torch = plain PyTorch (fp32, CPU capable)")
    g.add_argument("--synthetic", type=int, default=0, help="synthetic samples per (distance, event) class")
    g.add_argument("--synthetic_seed", type=int, default=0)
    g.add_argument("--snr_db", type=float, default=None)
    g.add_argument("--seed", type=int, default=0)
    g.add_argument("--graph", type=str2bool, default=True, help="capture each step into a HIP graph")
    g.add_argument("--tune", type=str2bool, default=False, help="autotune kernel configs at start-up")
    g.add_argument("--resume", type=str, default=None,
                   help="resume from a *.resume.pt sidecar; 'auto' = newest sidecar of this model under "
                        "--output_savedir (elastic restarts), fresh start if none")
    g.add_argument("--dtype", choices=["bf16", "fp32"], default=None,
                   help="compute dtype: bf16 = HIP engine, fp32 = plain PyTorch (overrides --backend)")
    g.add_argument("--sync_bn", type=str2bool, default=False,
                   help="synchronise BN batch statistics across ranks (engine: in-step all-reduces of the BN "
                        "sums, eager launches; torch: nn.SyncBatchNorm)")
    g.add_argument("--profile_steps", type=int, default=0, help="write a torch.profiler trace of N train steps")
    g.add_argument("--debug", type=str2bool, default=False,
                   help="debug mode: AMD_SERIALIZE_KERNEL=3, HIP_LAUNCH_BLOCKING=1, no HIP graphs")
    g.add_argument("--stream_ring", type=int, default=4,
                   help="--dataset_ram False: batches in flight in the disk -> pinned host -> HBM ring")
    g.add_argument("--loader_threads", type=int, default=8, help="threads of the native .mat batch reader")
    return ap


def config_from_args(args: argparse.Namespace, is_test: bool) -> TrainConfig:
    d = vars(args).copy()
    d["loss_weights"] = [float(x) for x in str(d["loss_weights"]).split(",")]
    if d.get("fold_index") is not None and d["fold_index"] < 0:
        d["fold_index"] = None
    if not is_test:
        d["model_path"] = None  # reference train.py passes pth_file=None (train.py:35)
    d["is_test"] = is_test
    if d.get("dtype") == "bf16":
        d["backend"] = "engine"
    elif d.get("dtype") == "fp32":
        d["backend"] = "torch"
    if d.get("debug"):
        d["graph"] = False
    return TrainConfig(**d)


def apply_debug_env(argv) -> None:
    """--debug must take effect before the HIP runtime initialises: called by train.py / test.py before
    importing torch.  Serialised kernels + blocking launches make a faulting kernel report at its own
    launch.  Also selects the engine's HIP graph executor stream count for the process
    (mtl_das_pytorch_amd.use_engine_graph_queues)."""
    import os
    from .. import use_engine_graph_queues
    use_engine_graph_queues()
    for i, a in enumerate(argv):
        val = a.split("=", 1)[1] if a.startswith("--debug=") else (argv[i + 1] if a == "--debug" and i + 1 < len(argv) else None)
        if val is not None and str2bool(val):
            os.environ.setdefault("AMD_SERIALIZE_KERNEL", "3")
            os.environ.setdefault("HIP_LAUNCH_BLOCKING", "1")
