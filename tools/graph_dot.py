#!/usr/bin/env python3
"""Dump the HIP graph executor's view of one captured training step: run from an output directory with
DEBUG_HIP_GRAPH_DOT_PRINT=1 in the environment, it captures the ``train_full`` graph through StepRunner
(which makes the runtime write ``graph_<pid>_dot_print_<n>``: every node with the executor stream it was
scheduled on, and the edges in insertion order) and writes ``launches.json`` -- the engine's launches in
capture order with their logical stream, waits and recorded event -- for engine/graphsched.py to compare
against.

    mkdir -p gpurun_out/dot_A && cd gpurun_out/dot_A && \\
        DEBUG_HIP_GRAPH_DOT_PRINT=1 python ../../tools/graph_dot.py MTL
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.data.synthetic import generate  # noqa: E402
from mtl_das_pytorch_amd.engine.graphsched import launch_records  # noqa: E402
from mtl_das_pytorch_amd.engine.step import StepRunner  # noqa: E402
from mtl_das_pytorch_amd.engine.tune import autotune_program  # noqa: E402
from mtl_das_pytorch_amd.models import build_model, encode_joint  # noqa: E402


def main():
    model_type = sys.argv[1] if len(sys.argv) > 1 else "MTL"
    torch.manual_seed(0)
    m = build_model(model_type)
    joint = model_type == "multi_classifier"
    if joint:
        from mtl_das_pytorch_amd.engine.inception import InceptionProgram
        p = InceptionProgram(m, 32, "cuda")
    else:
        from mtl_das_pytorch_amd.engine.mtl import MTLProgram
        p = MTLProgram(m, 32, "cuda")
    p.set_optimizer(weight_decay=1e-5)
    autotune_program(p, measure=False)
    X, d, e = generate(64, seed=1, device="cuda")
    lab = encode_joint(d, e) if joint else torch.stack([d, e], 1)
    r = StepRunner(p, X, lab)
    r.train_step(torch.arange(32, device="cuda"))
    torch.cuda.synchronize()
    phases = [p.gather_phase(X, lab, r.idx, clear=True), p.fwd_train, p.bwd, p.opt["adam"]]
    with open("launches.json", "w") as f:
        json.dump(launch_records(phases), f)
    print("graphs:", sorted(r.graphs), "dot files:", sorted(x for x in os.listdir(".") if "dot_print" in x))
    r.close()


if __name__ == "__main__":
    main()
