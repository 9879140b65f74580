"""Sliding-window inference: tiling covers the recording, predictions equal direct model
evaluation of each window, DP sharding over 2 gloo ranks gives the single-rank result, and the CLI."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_window_starts_cover_the_recording():
    from mtl_das_pytorch_amd.inference import window_starts
    assert list(window_starts(250, 250, 125)) == [0]
    assert list(window_starts(600, 250, 125)) == [0, 125, 250, 350]   # last window aligned to the end
    with pytest.raises(ValueError):
        window_starts(99, 100, 50)


def test_sliding_windows_match_slices():
    from mtl_das_pytorch_amd.inference import sliding_windows
    rec = torch.randn(230, 700)
    tiles, pos = sliding_windows(rec, stride=(100, 200))
    assert tiles.shape == (len(pos), 1, 100, 250)
    for k in (0, len(pos) // 2, len(pos) - 1):
        f0, t0 = pos[k]
        assert torch.equal(tiles[k, 0], rec[f0:f0 + 100, t0:t0 + 250])


@pytest.mark.parametrize("model_type", ["MTL", "single_event", "multi_classifier"])
def test_predictions_equal_direct_evaluation(model_type):
    from mtl_das_pytorch_amd.inference import predict_recording, sliding_windows
    from mtl_das_pytorch_amd.models import build_model
    torch.manual_seed(0)
    m = build_model(model_type).eval()
    rec = torch.randn(200, 600)
    res = predict_recording(m, model_type, rec, stride=(100, 175), batch=3, use_engine=False)
    tiles, pos = sliding_windows(rec, stride=(100, 175))
    with torch.no_grad():
        out = m(tiles)
    if model_type == "MTL":
        assert np.array_equal(res["distance_pred"], out[0].argmax(1).numpy())
        assert np.array_equal(res["event_pred"], out[1].argmax(1).numpy())
    elif model_type == "single_event":
        assert np.array_equal(res["event_pred"], out.argmax(1).numpy())
    else:
        j = out.argmax(1).numpy()
        assert np.array_equal(res["joint_pred"], j) and np.array_equal(res["distance_pred"], j % 16)
    assert np.array_equal(res["positions"], pos)


def _dp_worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK=str(rank))
    from mtl_das_pytorch_amd.inference import predict_recording
    from mtl_das_pytorch_amd.models import build_model
    from mtl_das_pytorch_amd.parallel.dist import init_distributed, shutdown
    ctx = init_distributed(backend="gloo")
    torch.manual_seed(0)
    m = build_model("MTL").eval()
    rec = torch.randn(200, 600, generator=torch.Generator().manual_seed(3))
    res = predict_recording(m, "MTL", rec, stride=(100, 175), batch=4, ctx=ctx, use_engine=False)
    q.put((rank, res["distance_pred"].tolist(), res["event_prob"].tolist()))
    shutdown(ctx)


def test_dp_sharded_inference_matches_single_rank():
    import socket
    from mtl_das_pytorch_amd.inference import predict_recording
    from mtl_das_pytorch_amd.models import build_model
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_dp_worker, args=(r, port, q)) for r in range(2)]
    [p.start() for p in ps]
    res = sorted(q.get(timeout=300) for _ in range(2))
    [p.join(timeout=60) for p in ps]
    torch.manual_seed(0)
    m = build_model("MTL").eval()
    rec = torch.randn(200, 600, generator=torch.Generator().manual_seed(3))
    ref = predict_recording(m, "MTL", rec, stride=(100, 175), batch=4, use_engine=False)
    for _, dpred, eprob in res:
        assert dpred == ref["distance_pred"].tolist()
        assert np.allclose(eprob, ref["event_prob"], atol=1e-6)


def test_infer_cli(tmp_path):
    rec = np.random.default_rng(0).standard_normal((150, 500)).astype(np.float32)
    np.save(tmp_path / "rec.npy", rec)
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "infer.py"), "--model", "MTL", "--recording",
                        str(tmp_path / "rec.npy"), "--out", str(tmp_path / "p.csv")], env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    import pandas as pd
    df = pd.read_csv(tmp_path / "p.csv")
    assert len(df) == 2 * 3 and set(df.columns) >= {"fiber_start", "time_start", "distance_pred", "event_pred"}
