"""Weight-gradient batches of a lowered program, job by job: for every (stream, tile config) batch of the
backward, the isolated time of each of its conv jobs launched alone (with its tuned split count), of the
whole batched launch, and the jobs' shapes / split counts / block counts -- to see whether a batch runs its
jobs side by side (batch ~ max of the jobs) or one after another (batch ~ sum).

    python tools/wgrad_jobs.py [MTL|multi_classifier]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.data.synthetic import generate  # noqa: E402
from mtl_das_pytorch_amd.engine.tune import _time, autotune_program  # noqa: E402
from mtl_das_pytorch_amd.models import build_model, encode_joint  # noqa: E402
from mtl_das_pytorch_amd.ops.hip import lib  # noqa: E402


def main():
    model_type = sys.argv[1] if len(sys.argv) > 1 else "MTL"
    torch.manual_seed(0)
    m = build_model(model_type)
    if model_type == "multi_classifier":
        from mtl_das_pytorch_amd.engine.inception import InceptionProgram
        prog = InceptionProgram(m, 32, "cuda")
    else:
        from mtl_das_pytorch_amd.engine.mtl import MTLProgram
        prog = MTLProgram(m, 32, "cuda")
    autotune_program(prog, measure=False, batch_wgrads=False)
    prog.merge_wgrad_cfgs()
    prog.refresh_wgrad_finalize()
    X, d, e = generate(64, seed=1, device="cuda")
    lab = encode_joint(d, e) if model_type == "multi_classifier" else torch.stack([d, e], 1)
    prog.opt["pack"].run()
    prog.arena.clear()
    prog.gather_phase(X, lab, torch.arange(32, device="cuda")).run()
    prog.fwd_train.run()
    prog.bwd.run()
    torch.cuda.synchronize()
    L = lib()
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    wg = [l for l in prog.bwd.launches if l.name == "conv_wgrad"]
    prog.wgrad_tables = []
    total = 0.0
    for s in sorted({l.stream for l in wg}):
        for cfg in sorted({l.args[0] for l in wg if l.stream == s}):
            group = [l for l in wg if l.stream == s and l.args[0] == cfg]
            b = prog._wgrad_batch_launch(cfg, group, s)
            tb = _time(lambda: b(st()), inner=10, reps=5) * 1e3
            total += tb
            print(f"stream {s} cfg {cfg}: {len(group)} jobs, {b.args[3]} blocks, batched {tb:.1f} us", flush=True)
            tj = 0.0
            for l in group:
                c, G, dd = l.args
                t = _time(lambda: L.wgrad(c, G, st(), dd), inner=10, reps=5) * 1e3
                tj += t
                print(f"    {t:6.1f} us  G{G} {dd['B']}x{dd['Hi']}x{dd['Wi']}->{dd['Ho']}x{dd['Wo']} "
                      f"{dd['Cs']}->{dd['Co']} k{dd['KH']}x{dd['KW']} s{dd['sh']} splits {dd['splits']}", flush=True)
            print(f"    sum of jobs alone {tj:.1f} us", flush=True)
    print(f"sum of batched launches {total:.1f} us")


if __name__ == "__main__":
    main()
