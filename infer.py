#!/usr/bin/env python3
"""Sliding-window inference over a long DAS recording (fiber x time matrix, .npy or .mat).

    python infer.py --model MTL --model_path run/<...>.pth --recording fiber.npy --stride 100,125 \
        --out predictions.csv
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 infer.py ...   # windows sharded over ranks
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser(description="Sliding-window DAS inference")
    ap.add_argument("--model", default="MTL", help="MTL, single_event, single_distance, multi_classifier")
    ap.add_argument("--model_path", default=None, help="reference-format state_dict (.pth)")
    ap.add_argument("--recording", required=True, help=".npy ([F, T] or [C, F, T]) or .mat (key --key)")
    ap.add_argument("--key", default="data")
    ap.add_argument("--stride", default="100,125", help="window stride (fiber, time)")
    ap.add_argument("--batch_size", type=int, default=32)
    ap.add_argument("--in_channels", type=int, default=1)
    ap.add_argument("--backend", choices=["auto", "engine", "torch"], default="auto")
    ap.add_argument("--out", default="predictions.csv")
    args = ap.parse_args()

    from mtl_das_pytorch_amd import use_engine_graph_queues
    use_engine_graph_queues()  # before the first HIP call
    import numpy as np
    import torch
    from mtl_das_pytorch_amd.data.mat_dataset import load_mat
    from mtl_das_pytorch_amd.inference import predict_recording
    from mtl_das_pytorch_amd.models import build_model
    from mtl_das_pytorch_amd.parallel.dist import init_distributed, shutdown

    ctx = init_distributed()
    model = build_model(args.model, in_channels=args.in_channels)
    if args.model_path:
        model.load_state_dict(torch.load(args.model_path, map_location="cpu", weights_only=True), strict=True)
    if args.recording.endswith(".mat"):
        rec = np.asarray(load_mat(args.recording, (args.key,)), dtype=np.float32)
    else:
        rec = np.load(args.recording, allow_pickle=False).astype(np.float32)
    use_engine = {"auto": None, "engine": True, "torch": False}[args.backend]
    res = predict_recording(model, args.model, torch.from_numpy(rec), stride=tuple(int(s) for s in args.stride.split(",")),
                            batch=args.batch_size, ctx=ctx, use_engine=use_engine)
    if ctx.is_main:
        import pandas as pd
        cols = {"fiber_start": res["positions"][:, 0], "time_start": res["positions"][:, 1]}
        for k in ("distance_pred", "event_pred", "joint_pred"):
            if k in res:
                cols[k] = res[k]
        pd.DataFrame(cols).to_csv(args.out, index=False)
        print(f"{len(res['positions'])} windows -> {args.out}")
    shutdown(ctx)


if __name__ == "__main__":
    main()
