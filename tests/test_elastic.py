"""Failure detection / elastic recovery on CPU: a 2-rank gloo job under torchrun with
``--max-restarts 1``; ``MDA_FAULT_INJECT`` kills rank 1 in the middle of the second epoch, the elastic
agent restarts the worker group, and ``--resume auto`` continues from the last sidecar in the SAME run
directory, finishing with the complete reference artefact set."""
import glob
import os
import socket
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_fault_injection_elastic_restart_resumes(tmp_path):
    out = tmp_path / "out"
    port = _free_port()
    # a short collective timeout turns "peer died mid-collective" into an error the agent restarts on;
    # three restarts absorb gloo's occasional refused connection while a restarted group re-forms
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", MDA_FAULT_INJECT="rank=1,step=9",
               OMP_NUM_THREADS="2", MDA_PG_TIMEOUT="30")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--rdzv-backend", "c10d", "--rdzv-endpoint", f"127.0.0.1:{port}", "--max-restarts", "3", "--monitor-interval", "1",
           os.path.join(ROOT, "train.py"), "--model", "single_event", "--synthetic", "2", "--batch_size", "4",
           "--epoch_num", "3", "--val_every", "1", "--log_every", "2", "--output_savedir", str(out),
           "--GPU_device", "False", "--resume", "auto", "--save_threshold", "0"]
    for attempt in range(2):
        r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=900)
        if r.returncode == 0 or "connectFullMesh failed" not in r.stdout + r.stderr:
            break
        # gloo's full-mesh connect of a restarted group occasionally fails under host load (refused /
        # timed-out TCP connect in gloo itself); that is not what this test checks: run the scenario again,
        # visibly (a warning in the test report), at most once
        import shutil
        import warnings
        warnings.warn("known gloo connectFullMesh flake in the restarted group: re-running the scenario once")
        shutil.rmtree(out, ignore_errors=True)
        port = _free_port()
        cmd[cmd.index("--rdzv-endpoint") + 1] = f"127.0.0.1:{port}"
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    runs = glob.glob(str(out / "* model_type=single_event is_test=False"))
    assert len(runs) == 1, runs  # the restarted job continued in the same directory
    log = open(os.path.join(runs[0], "console output.log"), encoding="utf-8").read()
    assert "fault injection: rank 1 exits at global step 9" in r.stdout + r.stderr + log
    assert "resumed from" in log
    # every epoch's validation ran exactly once across both attempts: epochs 0..3
    assert log.count("Validation Accuracy") == 4, log
    acc = np.load(os.path.join(runs[0], "testAccLine.npy"))
    assert acc.shape[-1] == 4
    for name in ("trainAccLine", "trainLossLine", "testAccLine", "testLossLine"):
        assert os.path.exists(os.path.join(runs[0], name + ".png"))
