"""Bitwise digest of a few captured training steps, for comparing two builds of the HIP extension.

    python tools/ext_digest.py [--model MTL|multi_classifier|...] [--steps 5]
    MDA_EXT_PATH=ab/_mda_hip_base.so python tools/ext_digest.py ...

Builds the model's program from the shipped tuned table (no measuring, so both builds run the same kernel
configurations), trains ``--steps`` graph-replayed steps on a fixed synthetic batch schedule and prints the
sha256 of the fp32 master weights, gradients, Adam moments and BN running statistics, and of the head's
correct / count metric columns.
Kernel changes that only reorder loads (no arithmetic change) must print the same digest as the baseline build.
"""
import argparse
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="MTL")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    args = ap.parse_args()
    from mtl_das_pytorch_amd import use_engine_graph_queues
    use_engine_graph_queues()
    import torch
    from mtl_das_pytorch_amd.data.synthetic import generate
    from mtl_das_pytorch_amd.engine.inception import InceptionProgram
    from mtl_das_pytorch_amd.engine.mtl import MTLProgram
    from mtl_das_pytorch_amd.engine.step import StepRunner
    from mtl_das_pytorch_amd.engine.tune import autotune_program
    from mtl_das_pytorch_amd.models import build_model, encode_joint
    from mtl_das_pytorch_amd.ops import hip

    hip.lib()
    dev = torch.device("cuda:0")
    torch.manual_seed(1234)
    model = build_model(args.model)
    joint = args.model == "multi_classifier"
    prog = (InceptionProgram(model, args.batch, dev) if joint else MTLProgram(model, args.batch, dev))
    prog.set_optimizer(betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-5)
    prog.segment_backward(1)
    autotune_program(prog, measure=False)
    n = 4 * args.batch
    X, d, e = generate(n, seed=1000, device=dev)
    labels = encode_joint(d, e) if joint else torch.stack([d, e], 1)
    runner = StepRunner(prog, X, labels, use_graph=True)
    runner.set_lr(1e-3 / 1.5)
    g = torch.Generator().manual_seed(7)
    sched = torch.stack([torch.randperm(n, generator=g)[:args.batch] for _ in range(args.steps)]).to(dev)
    runner.set_index_schedule(sched)
    for _ in range(args.steps):
        runner.train_step()
    torch.cuda.synchronize()
    f = prog.flat
    h = hashlib.sha256()
    for name in ("params", "grads", "exp_avg", "exp_avg_sq", "bn_mean", "bn_var"):
        t = getattr(f, name, None)
        if t is not None:
            h.update(t.detach().cpu().numpy().tobytes())
    # the metric rows' correct / count columns (the loss column is an fp32 atomic sum: its last bits follow the
    # order the blocks arrive in, run to run)
    hm = hashlib.sha256(prog.metrics[:, 1:3].detach().cpu().numpy().tobytes())
    print(f"DIGEST {args.model} steps={args.steps} state={h.hexdigest()[:16]} metrics={hm.hexdigest()[:16]} "
          f"ext={os.environ.get('MDA_EXT_PATH', 'in-tree')}", flush=True)
    runner.close()


if __name__ == "__main__":
    main()
