"""Weight-gradient jobs of a model, one by one: the isolated time of the shipped tile config against every valid
lean-staging config (csrc/wgrad_lean.hip, configs 36-47) at the split counts ConvLayer.wgrad_plan gives them,
and the batched launches per stream with the shipped configs vs each job on its fastest lean config vs the shipped
table with its large tiles (32-35) on their lean-staging twins (44-47).

    python tools/wgrad_lean_probe.py [MTL|multi_classifier]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.data.synthetic import generate  # noqa: E402
from mtl_das_pytorch_amd.engine.tune import _time, autotune_program  # noqa: E402
from mtl_das_pytorch_amd.models import build_model, encode_joint  # noqa: E402
from mtl_das_pytorch_amd.ops.functional import WGRAD_BIG0, WGRAD_LEAN0, WGRAD_LEAN_N, WGRAD_LEANBIG0  # noqa: E402
from mtl_das_pytorch_amd.ops.hip import lib  # noqa: E402

LEAN = list(range(WGRAD_LEAN0, WGRAD_LEAN0 + WGRAD_LEAN_N)) + list(range(WGRAD_LEANBIG0, WGRAD_LEANBIG0 + 4))


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
    shipped = {id(l): l.args[0] for l in wg}
    best = {}
    for l in wg:
        conv, (c0, G, dd) = l.owner, l.args
        conv.set_wgrad_cfg(c0)
        t0 = _time(lambda: L.wgrad(c0, G, st(), dd), inner=10, reps=5) * 1e3
        row = [f"c{c0}:{t0:5.1f}"]
        cand = [(t0, c0)]
        for c in LEAN:
            if not conv.wgrad_valid(c):
                continue
            conv.set_wgrad_cfg(c)
            t = _time(lambda: L.wgrad(c, G, st(), dd), inner=10, reps=5) * 1e3
            cand.append((t, c))
            row.append(f"c{c}:{t:5.1f}/s{dd['splits']}")
        conv.set_wgrad_cfg(c0)
        tb, cb = min((t, c) for t, c in cand if c in LEAN) if len(cand) > 1 else (t0, c0)
        best[id(l)] = cb
        print(f"s{l.stream} G{G} {dd['B']}x{dd['Hi']}x{dd['Wi']}->{dd['Ho']}x{dd['Wo']} {dd['Cs']}->{dd['Co']} "
              f"k{dd['KH']}x{dd['KW']} s{dd['sh']}: shipped {t0:5.1f} us, best lean c{cb} {tb:5.1f} us | " + " ".join(row),
              flush=True)
    # batched launches per stream: shipped configs vs every job on its best lean config (one batch per config)
    prog.wgrad_tables = []
    # the shipped table with every large-tile job (32-35) on its lean-staging twin (44-47): same tiles and M split,
    # only the staging differs -- the throughput comparison of the two staging forms
    twin = {k: (c - WGRAD_BIG0 + WGRAD_LEANBIG0 if WGRAD_BIG0 <= c < WGRAD_BIG0 + 4 else c) for k, c in shipped.items()}
    for label, pick in (("shipped", shipped), ("lean", best), ("leanbig-twins", twin)):
        tot = 0.0
        for l in wg:
            l.owner.set_wgrad_cfg(pick[id(l)])
            l.args = (pick[id(l)],) + tuple(l.args[1:])
        for s in sorted({l.stream for l in wg}):
            for cfg in sorted({l.args[0] for l in wg if l.stream == s}):
                group = [l for l in wg if l.stream == s and l.args[0] == cfg]
                b = prog._wgrad_batch_launch(cfg, group, s)
                tb = _time(lambda: b(st()), inner=10, reps=5) * 1e3
                tot += tb
                print(f"  {label}: stream {s} cfg {cfg}: {len(group)} jobs, {b.args[3]} blocks, {tb:.1f} us", flush=True)
        print(f"{label}: sum of batched launches {tot:.1f} us", flush=True)


if __name__ == "__main__":
    main()
