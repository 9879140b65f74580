"""Layer-local check of the Model C lowering: for every op, recompute its output in fp32 PyTorch from
the ENGINE's own input activation and report the relative error (isolates kernel/lowering bugs from
the network's error amplification)."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from mtl_das_pytorch_amd.data.synthetic import generate  # noqa: E402
from mtl_das_pytorch_amd.engine.inception import CBR, InceptionProgram, Pool  # noqa: E402
from mtl_das_pytorch_amd.models import Multi_Classifier, encode_joint  # noqa: E402


def nchw(a):
    t = a.t.view(-1)[a.off:]
    M = a.B * a.H * a.W
    idx = torch.arange(M, device=t.device)[:, None] * a.ld + torch.arange(a.C, device=t.device)[None]
    return t[idx].float().view(a.B, a.H, a.W, a.C).permute(0, 3, 1, 2)


def rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def main():
    torch.manual_seed(0)
    B = 8
    m = Multi_Classifier()
    prog = InceptionProgram(m, B, "cuda", p_drop=0.0)
    X, d, e = generate(2 * B, seed=1, device="cuda")
    lab = encode_joint(d, e)
    idx = torch.arange(B, device="cuda")
    prog.opt["pack"].run()
    prog.arena.clear()
    prog.gather_phase(X, lab, idx).run()
    prog.fwd_train.run()
    torch.cuda.synchronize()
    worst = []
    for i, op in enumerate(prog.ops):
        x = nchw(op.src.act)
        out = nchw(op.out.act)
        if isinstance(op, CBR):
            c = op.conv.mods[0]
            bn = op.bn.mods[0]
            w = c.weight.detach().bfloat16().float()
            if op.conv.Cs != c.in_channels:
                x = x[:, :c.in_channels]
            y = F.conv2d(x, w, None, c.stride, c.padding)
            ye = nchw(op.y)
            ey = rel(ye, y)
            mu = y.mean((0, 2, 3), keepdim=True)
            var = y.var((0, 2, 3), unbiased=False, keepdim=True)
            z = (ye - mu) / torch.sqrt(var + bn.eps) * bn.weight.view(1, -1, 1, 1) + bn.bias.view(1, -1, 1, 1)
            r = F.relu(z)
            eo = rel(out, r)
            name = [n for n, mm in m.named_modules() if mm is c][0]
            print(f"{i:3d} CBR {name:40s} y {tuple(y.shape)} err_conv {ey:.2e} err_tail {eo:.2e}")
            worst.append((max(ey, eo), name))
        else:
            r = F.max_pool2d(x, 3, 2) if op.is_max else F.avg_pool2d(x, 3, 1, 1)
            eo = rel(out, r)
            print(f"{i:3d} POOL max={op.is_max} {tuple(r.shape)} err {eo:.2e}")
            worst.append((eo, f"pool{i}"))
    feat = nchw(prog.feat.act).mean((2, 3))
    logits = feat @ m.fc.weight.t() + m.fc.bias
    print("head err", rel(prog.logp, logits))
    worst.sort(reverse=True)
    print("worst", worst[:8])


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def global_drift():
    """Engine activations vs an fp32 reference that rounds where the engine stores bf16, layer by layer,
    plus the reference's own sensitivity to a 1e-3 input perturbation (chaos check)."""
    import copy
    import types
    from mtl_das_pytorch_amd.models import multi_classifier as mc
    torch.manual_seed(0)
    B = 8
    m = Multi_Classifier()
    ref = copy.deepcopy(m).cuda()
    prog = InceptionProgram(m, B, "cuda", p_drop=0.0)
    X, d, e = generate(2 * B, seed=1, device="cuda")
    lab = encode_joint(d, e)
    idx = torch.arange(B, device="cuda")
    prog.opt["pack"].run()
    prog.arena.clear()
    prog.gather_phase(X, lab, idx).run()
    prog.fwd_train.run()
    torch.cuda.synchronize()
    q = lambda t: t.bfloat16().float()
    outs = {}

    def fwd(self, x):
        y = q(self.conv(x))
        z = q(F.relu(self.bn(y)))
        outs.setdefault(id(self), []).append(z)
        return z

    for mod in ref.modules():
        if isinstance(mod, mc.BasicConv2d):
            mod.forward = types.MethodType(fwd, mod)
    mc._avgpool3 = lambda x: q(F.avg_pool2d(x, 3, 1, 1))
    with torch.no_grad():
        for p in ref.parameters():
            p.copy_(q(p))
        ref.train()
        x = q(X[idx])
        out0 = ref(x)
        out1 = ref(x * (1 + 1e-3 * torch.randn_like(x)))
    print("ref logits sensitivity to 1e-3 input noise:", rel(out1, out0))
    for i, op in enumerate(prog.ops):
        if isinstance(op, CBR):
            bc = [mm for mm in m.modules() if isinstance(mm, mc.BasicConv2d) and mm.conv is op.conv.mods[0]][0]
            rb = [mm for mm in ref.modules() if isinstance(mm, mc.BasicConv2d)]
            names = [n for n, mm in m.named_modules() if mm is bc]
            rmod = dict(ref.named_modules())[names[0]]
            r = outs[id(rmod)][0]
            print(f"{i:3d} {names[0]:36s} drift {rel(nchw(op.out.act), r):.3e}  drift(rerun) {rel(outs[id(rmod)][1], r):.3e}")
    print("logits drift", rel(prog.logp, out0))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "drift":
    global_drift()


def pools():
    from mtl_das_pytorch_amd.engine.inception import Pool
    torch.manual_seed(0)
    B = 8
    m = Multi_Classifier()
    prog = InceptionProgram(m, B, "cuda", p_drop=0.0)
    X, d, e = generate(2 * B, seed=1, device="cuda")
    lab = encode_joint(d, e)
    idx = torch.arange(B, device="cuda")
    prog.opt["pack"].run()
    prog.arena.clear()
    prog.gather_phase(X, lab, idx).run()
    prog.fwd_train.run()
    prog.bwd.run()
    torch.cuda.synchronize()
    for i, op in enumerate(prog.ops):
        if not isinstance(op, Pool):
            continue
        srcs = op.out.grad_sources()
        g = sum(nchw(a) for a in srcs)
        x = nchw(op.src.act).contiguous().requires_grad_(True)
        yy = F.max_pool2d(x, 3, 2) if op.is_max else F.avg_pool2d(x, 3, 1, 1)
        yy.backward(g)
        dx = nchw(op.dx)
        ties = (x == 0).float().mean().item()
        print(f"{i:3d} max={op.is_max} x{tuple(x.shape)} nsrc={len(srcs)} zeros={ties:.2f} err={rel(dx, x.grad):.3e} "
              f"|dx|={dx.norm().item():.3e} |ref|={x.grad.norm().item():.3e} |g|={g.norm().item():.3e} "
              f"src ld={[a.ld for a in srcs]} off={[a.off for a in srcs]}")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "pools":
    pools()
