#!/usr/bin/env python3
"""Model test (reference test.py): evaluates ``--model_path`` on the test set and writes the
confusion-matrix figures.  Note: like the reference, a checkpoint copy and the confusion-matrix .npy
files are written only when the distance accuracy reaches the save threshold (0.98 / 0.95)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from mtl_das_pytorch_amd.utils.config import apply_debug_env, build_parser, config_from_args  # noqa: E402

apply_debug_env(sys.argv)  # before anything initialises the HIP runtime

from mtl_das_pytorch_amd.engine.trainer import main_process  # noqa: E402

if __name__ == "__main__":
    args = build_parser(is_test=True).parse_args()
    main_process(config_from_args(args, is_test=True))
