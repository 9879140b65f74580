"""bench.py's launch contract without a launcher: ``--gpus 2`` with no WORLD_SIZE in the
environment starts its two rank processes itself (gloo on the CPU here; one rank per GPU on an MI355X node),
and exactly one JSON line -- rank 0's -- reaches stdout."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_self_launches_two_ranks_and_prints_one_json_line():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["CUDA_VISIBLE_DEVICES"] = ""  # the CPU (gloo) form of the contract even on a GPU box
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--batch", "2"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    js = [l for l in lines if l.lstrip().startswith("{")]
    assert len(js) == 1, r.stdout  # (gloo itself prints its connection lines to stdout)
    out = json.loads(js[0])
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 4
    assert out["value"] > 0 and out["dist_backend"] == "gloo"


def test_bench_self_launch_propagates_a_failing_rank():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "nope"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and not r.stdout.strip()
