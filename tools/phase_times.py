"""Wall time of the step's phases without a profiler attached (rocprofv3 serialises cross-stream graph
edges and inflates multi-stream steps): captures one HIP graph per prefix of the step
([gather], [+forward], [+backward], [+Adam]) and times N replays of each with device events.

    python tools/phase_times.py [MTL|single_event|multi_classifier] [replays]
MDA_STREAMS=0 gives the single-stream numbers for comparison."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.data.synthetic import generate  # noqa: E402
from mtl_das_pytorch_amd.engine.step import StateSnapshot, capture_graph  # noqa: E402
from mtl_das_pytorch_amd.engine.tune import autotune_program  # noqa: E402
from mtl_das_pytorch_amd.models import build_model, encode_joint  # noqa: E402


def main():
    model_type = sys.argv[1] if len(sys.argv) > 1 else "MTL"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    torch.manual_seed(0)
    m = build_model(model_type)
    if model_type == "multi_classifier":
        from mtl_das_pytorch_amd.engine.inception import InceptionProgram
        p = InceptionProgram(m, 32, "cuda")
    else:
        from mtl_das_pytorch_amd.engine.mtl import MTLProgram
        p = MTLProgram(m, 32, "cuda")
    p.set_optimizer(betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-5)
    autotune_program(p, measure=False)
    X, d, e = generate(256, seed=1, device="cuda")
    lab = encode_joint(d, e) if model_type == "multi_classifier" else torch.stack([d, e], 1)
    idx = torch.arange(32, device="cuda")
    p.flat.lr.fill_(1e-3)
    p.opt["pack"].run()
    gather = p.gather_phase(X, lab, idx, clear=True)  # with the arena clear, as the step runs it
    f = p.flat
    state = [f.params, f.grads, f.exp_avg, f.exp_avg_sq, f.bn_mean, f.bn_var, f.bn_nbt, f.step, p.metrics,
             p.confusion, p.logp] + list(getattr(p, "extra_state", []))
    prefixes = {
        "gather": [gather.run],
        "+fwd": [gather.run, p.fwd_train.run],
        "+bwd": [gather.run, p.fwd_train.run, p.bwd.run],
        "+adam (full step)": [gather.run, p.fwd_train.run, p.bwd.run, p.opt["adam"].run],
        "eval fwd": [gather.run, p.fwd_eval.run],
    }
    counts = {"fwd": len(p.fwd_train), "bwd": len(p.bwd), "adam": len(p.opt["adam"]), "eval": len(p.fwd_eval)}
    print(f"{model_type}: launches {counts}, MDA_STREAMS={os.environ.get('MDA_STREAMS', '1')}")
    prev = 0.0
    for name, fns in prefixes.items():
        snap = StateSnapshot(state)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for fn in fns:
                fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g, keep = capture_graph(fns)
        for _ in range(20):
            g.replay()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(reps):
            g.replay()
        t1.record()
        torch.cuda.synchronize()
        us = 1e3 * t0.elapsed_time(t1) / reps
        delta = "" if name == "eval fwd" else f"  (+{us - prev:7.1f} us)"
        print(f"{name:20s} {us:8.1f} us/replay{delta}")
        if name != "eval fwd":
            prev = us
        snap.restore()
        g.reset()
        del g, keep
    p.opt["pack"].run()


if __name__ == "__main__":
    main()
