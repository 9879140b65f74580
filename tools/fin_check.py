"""Producer-side BN finalize vs consumer-side replica reduction: one training step of each engine program
with MDA_BN_FIN=1 and =0 (two child processes, same seed), compared bitwise per BN layer and gradient."""
import os
import subprocess
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(model, B, out):
    from mtl_das_pytorch_amd.data.synthetic import generate
    from mtl_das_pytorch_amd.engine.inception import InceptionProgram
    from mtl_das_pytorch_amd.engine.mtl import MTLProgram
    from mtl_das_pytorch_amd.engine.step import StepRunner
    from mtl_das_pytorch_amd.engine.tune import autotune_program
    from mtl_das_pytorch_amd.models import build_model, encode_joint
    torch.manual_seed(0)
    m = build_model(model)
    joint = model == "multi_classifier"
    prog = InceptionProgram(m, B, "cuda", p_drop=0.0) if joint else MTLProgram(m, B, "cuda")
    prog.set_optimizer(weight_decay=0.0)
    autotune_program(prog, measure=False)
    X, d, e = generate(B, seed=1, device="cuda", backend="torch")
    lab = encode_joint(d, e) if joint else torch.stack([d, e], 1)
    run = StepRunner(prog, X, lab, use_graph=False)
    run.set_lr(0.0)
    run.train_step(torch.arange(B, device="cuda"))
    torch.cuda.synchronize()
    torch.save({"grads": prog.flat.grads.cpu(), "consts": [bn.consts.cpu() for bn in prog.flat.bn_layers],
                "rm": prog.flat.bn_mean.cpu(), "rv": prog.flat.bn_var.cpu(), "nbt": prog.flat.bn_nbt.cpu()}, out)


def main():
    model, B = sys.argv[1], int(sys.argv[2])
    res = {}
    for v in ("1", "0"):
        out = f"/tmp/fin_{model}_{v}.pt"
        subprocess.run([sys.executable, __file__, "child", model, str(B), out], check=True,
                       env=dict(os.environ, MDA_BN_FIN=v))
        res[v] = torch.load(out, weights_only=True)
    a, b = res["1"], res["0"]
    bad = [i for i, (x, y) in enumerate(zip(a["consts"], b["consts"])) if not torch.equal(x, y)]
    print(f"{model} B={B}: {len(a['consts'])} BN layers, consts differ in {bad[:10]} ({len(bad)})")
    if bad:
        i = bad[0]
        print("  first differing layer max abs diff", (a["consts"][i] - b["consts"][i]).abs().max().item())
    print("  grads equal", torch.equal(a["grads"], b["grads"]), "max diff", (a["grads"] - b["grads"]).abs().max().item())
    print("  running mean/var equal", torch.equal(a["rm"], b["rm"]), torch.equal(a["rv"], b["rv"]),
          "nbt", a["nbt"].tolist()[:4], b["nbt"].tolist()[:4])


if __name__ == "__main__":
    if sys.argv[1] == "child":
        child(sys.argv[2], int(sys.argv[3]), sys.argv[4])
    else:
        main()
