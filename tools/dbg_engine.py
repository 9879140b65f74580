"""Diagnostic: per-parameter and per-activation gradient errors of the MI355X engine vs fp32 autograd."""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.data.synthetic import generate  # noqa: E402
from mtl_das_pytorch_amd.engine.mtl import MTLProgram  # noqa: E402
from mtl_das_pytorch_amd.models import MTL_Net  # noqa: E402


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


torch.manual_seed(0)
B = int(os.environ.get("B", 8))
model = MTL_Net()
ref = copy.deepcopy(model).cuda()
prog = MTLProgram(model, B, "cuda")
X, d, e = generate(2 * B, seed=1, device="cuda")
labels = torch.stack([d, e], 1)
idx = torch.arange(B, device="cuda")
prog.opt["pack"].run()
prog.arena.clear()
prog.gather_phase(X, labels, idx).run()
prog.fwd_train.run()
prog.bwd.run()
torch.cuda.synchronize()

# reference with hooks on every resblock output and task-branch tensors
acts = {}
ref.train()
x = X[idx].bfloat16().float()
feat = ref.features(x)
for i, f in enumerate(feat):
    f.retain_grad()
    acts[f"F{i+1}"] = f
outs = []
for t in range(2):
    prev = None
    for lvl in range(4):
        gen = ref.att_generators[lvl][t]
        src = feat[2 * lvl] if prev is None else torch.cat((feat[2 * lvl], prev), 1)
        a = gen(src) * feat[2 * lvl + 1]
        a.retain_grad()
        acts[f"A{lvl+1}_t{t}"] = a
        if lvl < 3:
            prev = ref.down_sampling(ref.output_layers[lvl][t](a))
            prev.retain_grad()
            acts[f"B{lvl+1}_t{t}"] = prev
        else:
            prev = a
    gap, grp = ref.head_modules(t)
    outs.append(F.log_softmax(grp(gap(prev).flatten(1).unsqueeze(1)).squeeze(1), 1))
loss = F.nll_loss(outs[0], labels[idx, 0]) + F.nll_loss(outs[1], labels[idx, 1])
loss.backward()


def nchw(t, L):
    return t.view(L.B, L.H, L.W, L.C).permute(0, 3, 1, 2)


# forward activations
for i, Fk in enumerate(prog.F):
    print(f"fwd F{i+1}: rel {rel(nchw(Fk.t[0].float(), Fk), acts[f'F{i+1}']):.4f}")
for lvl, L in enumerate(prog.levels):
    for t in range(2):
        A = L["Aout"]
        print(f"fwd A{lvl+1}_t{t}: rel {rel(nchw(A.t[t].float(), A), acts[f'A{lvl+1}_t{t}']):.4f}")
        if "Bp" in L:
            Bp = L["Bp"]
            print(f"fwd B{lvl+1}_t{t}: rel {rel(nchw(Bp.t[t].float(), Bp), acts[f'B{lvl+1}_t{t}']):.4f}")

# backward: gradients w.r.t. A_l (dA) and B_l (from next level dcat)
for lvl, L in enumerate(prog.levels):
    for t in range(2):
        dA = L["dA"]
        print(f"grad A{lvl+1}_t{t}: rel {rel(nchw(dA.t[t], dA), acts[f'A{lvl+1}_t{t}'].grad):.4f}")
        if lvl < 3:
            nxt = prog.levels[lvl + 1]
            dcat = nxt["dcat"]
            Cn = nxt["Fa"].C
            g = dcat.t[t].view(B, nxt["H"], nxt["W"], 2 * Cn)[..., Cn:].permute(0, 3, 1, 2)
            print(f"grad B{lvl+1}_t{t}: rel {rel(g, acts[f'B{lvl+1}_t{t}'].grad):.4f}")

prog.flat.sync_module_grads()
rp = dict(ref.named_parameters())
for name, p in model.named_parameters():
    if rp[name].grad is None:
        continue
    print(f"{name:45s} rel {rel(p.grad, rp[name].grad):.4f}  |ref| {rp[name].grad.norm().item():.3e}")

# --- intrinsic sensitivity: fp32 reference with bf16-rounded weights vs fp32 reference ---
def ref_grads(m, xin):
    m.zero_grad()
    o1, o2 = m(xin)
    (F.nll_loss(o1, labels[idx, 0]) + F.nll_loss(o2, labels[idx, 1])).backward()
    return {n: p.grad.clone() for n, p in m.named_parameters()}


torch.manual_seed(0)
base = copy.deepcopy(ref)
g0 = ref_grads(base, x)
q = copy.deepcopy(base)
with torch.no_grad():
    for p in q.parameters():
        p.copy_(p.bfloat16().float())
g1 = ref_grads(q, x)
pert = copy.deepcopy(base)
with torch.no_grad():
    for p in pert.parameters():
        p.mul_(1 + 1e-3 * torch.randn_like(p))
g2 = ref_grads(pert, x)
print("\nintrinsic sensitivity (fp32 autograd):")
for n in ["conv1.0.weight", "resblock1.left.0.weight", "resblock4.left.0.weight", "resblock8.left.0.weight",
          "att_mask_generator1.0.0.weight", "att_mask_generator4.0.0.weight", "output_layer1.0.0.weight"]:
    print(f"{n:40s} bf16-weights {rel(g1[n], g0[n]):.4f}   1e-3 weight noise {rel(g2[n], g0[n]):.4f}   engine {rel(dict(model.named_parameters())[n].grad, g0[n]):.4f}")
