"""Time every launch of a lowered program in isolation (graph of 20 back-to-back replays of that launch)
and print them in program order with their shapes -- to compare against the in-step rocprof times."""
import sys

import torch

sys.path.insert(0, ".")
from mtl_das_pytorch_amd.data.synthetic import generate  # noqa: E402
from mtl_das_pytorch_amd.engine.tune import _time, autotune_program  # noqa: E402
from mtl_das_pytorch_amd.models import build_model, encode_joint  # noqa: E402


def shape_of(l):
    d = next((a for a in l.args if isinstance(a, dict)), {})
    keys = ("B", "H", "W", "C", "Hs", "Ws", "Ho", "Wo", "N", "Cs", "KH", "KW", "Co")
    s = ",".join(f"{k}={d[k]}" for k in keys if k in d)
    if "g" in d:
        s += f",nsrc={len(d['g'])}"
    if "fused" in d:
        s += f",fused={d['fused']}"
    return s


def main():
    model_type = sys.argv[1] if len(sys.argv) > 1 else "MTL"
    phase = sys.argv[2] if len(sys.argv) > 2 else "bwd"
    torch.manual_seed(0)
    m = build_model(model_type)
    if model_type == "multi_classifier":
        from mtl_das_pytorch_amd.engine.inception import InceptionProgram
        prog = InceptionProgram(m, 32, "cuda")
    else:
        from mtl_das_pytorch_amd.engine.mtl import MTLProgram
        prog = MTLProgram(m, 32, "cuda")
    autotune_program(prog, measure=False)
    X, d, e = generate(64, seed=1, device="cuda")
    lab = encode_joint(d, e) if model_type == "multi_classifier" else torch.stack([d, e], 1)
    prog.opt["pack"].run()
    prog.arena.clear()
    prog.gather_phase(X, lab, torch.arange(32, device="cuda")).run()
    prog.fwd_train.run()
    prog.bwd.run()
    torch.cuda.synchronize()
    ph = {"fwd": prog.fwd_train, "bwd": prog.bwd}[phase]
    tot = 0.0
    for i, l in enumerate(ph.launches):
        t = _time(lambda: l(torch.cuda.current_stream().cuda_stream), inner=10, reps=5) * 1e3
        tot += t
        print(f"{i:4d} {l.name:16s} {t:8.1f} us  {shape_of(l)}", flush=True)
    print(f"sum of isolated launch times: {tot:.1f} us")


if __name__ == "__main__":
    main()
