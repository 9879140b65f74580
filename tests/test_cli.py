"""End-to-end train.py / test.py on CPU with a tiny synthetic .mat tree (BASELINE config #1 plumbing)."""
import glob
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def tree(tmp_path_factory):
    from mtl_das_pytorch_amd.data import write_mat_tree
    return write_mat_tree(str(tmp_path_factory.mktemp("das")), n_per_class=5, n_test_per_class=1, seed=11)


def _run(script, args, cwd):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", PYTHONHASHSEED="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, script)] + args, cwd=cwd, env=env,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


@pytest.mark.parametrize("model", ["MTL", "single_distance", "single_event", "multi_classifier"])
def test_train_then_test(tree, tmp_path, model):
    out = tmp_path / "out"
    args = ["--model", model, "--batch_size", "4", "--epoch_num", "1", "--output_savedir", str(out),
            "--trainVal_set_striking", tree["striking_train"], "--trainVal_set_excavating", tree["excavating_train"],
            "--save_threshold", "0.0", "--GPU_device", "False"]
    stdout = _run("train.py", args, str(tmp_path))
    runs = glob.glob(str(out / f"* model_type={model} is_test=False"))
    assert len(runs) == 1
    d = runs[0]
    # reference artefact set; 32 batches per epoch (< 100) used to crash the reference (utils.py:185)
    for name in ("trainAccLine", "trainLossLine", "testAccLine", "testLossLine"):
        assert os.path.exists(os.path.join(d, name + ".npy")) and os.path.exists(os.path.join(d, name + ".png"))
    assert os.path.exists(os.path.join(d, "console output.log"))
    log = open(os.path.join(d, "console output.log"), encoding="utf-8").read()
    assert "Validation Accuracy" in log or "Accuracy: distance" in log
    assert "Epoch 1 finished！" in log
    ta = np.load(os.path.join(d, "testAccLine.npy"))
    assert ta.shape == (2, 1)
    pths = sorted(glob.glob(os.path.join(d, "*.pth")))
    assert pths, "threshold 0 must save a checkpoint"
    sd = torch.load(pths[-1], map_location="cpu", weights_only=True)
    assert not any(k.startswith("module.") for k in sd)
    # test.py on the saved checkpoint
    targs = ["--model", model, "--model_path", pths[-1], "--batch_size", "4", "--output_savedir", str(out),
             "--test_set_striking", tree["striking_test"], "--test_set_excavating", tree["excavating_test"],
             "--save_threshold", "0.0", "--GPU_device", "False"]
    _run("test.py", targs, str(tmp_path))
    truns = glob.glob(str(out / f"* model_type={model} is_test=True"))
    assert len(truns) == 1
    svgs = glob.glob(os.path.join(truns[0], "*.svg"))
    assert svgs, "test mode draws the confusion matrices"


def test_bool_flags_are_parsed():
    from mtl_das_pytorch_amd.utils.config import build_parser, config_from_args
    a = build_parser(False).parse_args(["--GPU_device", "False", "--dataset_ram", "0"])
    c = config_from_args(a, False)
    assert c.GPU_device is False and c.dataset_ram is False and c.model_path is None
    t = build_parser(True).parse_args([])
    assert t.test_set_striking == "./dataset/striking_test"


def test_training_learns_synthetic(tmp_path):
    """A few epochs on separable synthetic data: event accuracy well above chance (CPU, torch backend)."""
    from mtl_das_pytorch_amd.engine.trainer import Trainer
    from mtl_das_pytorch_amd.utils.config import TrainConfig
    torch.manual_seed(0)
    cfg = TrainConfig(model="MTL", synthetic=6, batch_size=16, epoch_num=4, val_every=4, log_every=10,
                      output_savedir=str(tmp_path), GPU_device=False, save_threshold=2.0)
    tr = Trainer(cfg)
    tr.run()
    assert tr.last_val["epoch"] == 4
    assert tr.last_val["acc"]["event"] > 0.7
