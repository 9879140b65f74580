#!/usr/bin/env python3
"""Model training (reference train.py): same flags, same console output and artefacts.

    python train.py --model MTL --batch_size 32 --epoch_num 40 \
        --trainVal_set_striking ./dataset/striking_train --trainVal_set_excavating ./dataset/excavating_train
    python train.py --model MTL --synthetic 20 --epoch_num 5          # no dataset needed
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train.py ...   # data parallel over RCCL
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from mtl_das_pytorch_amd.utils.config import apply_debug_env, build_parser, config_from_args  # noqa: E402

apply_debug_env(sys.argv)  # before anything initialises the HIP runtime

from mtl_das_pytorch_amd.engine.trainer import main_process  # noqa: E402

if __name__ == "__main__":
    args = build_parser(is_test=False).parse_args()
    main_process(config_from_args(args, is_test=False))
