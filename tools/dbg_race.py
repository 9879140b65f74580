"""Find a nondeterministic launch: run the same training step twice from identical state, eagerly, one
launch at a time, snapshot each launch's output buffer(s) after it runs, and report launches whose
outputs differ between the runs (fp32 BN-statistic atomics only reorder sums -> ~1e-6 relative; a race
shows up as a large jump at the first culprit)."""
import sys

import torch

sys.path.insert(0, ".")
from mtl_das_pytorch_amd.data.synthetic import generate  # noqa: E402
from mtl_das_pytorch_amd.engine.core import Act, LazyView  # noqa: E402
from mtl_das_pytorch_amd.models import build_model, encode_joint  # noqa: E402
from mtl_das_pytorch_amd.ops.hip import stream  # noqa: E402

OUT_KEYS = ("out", "dy", "dy2", "side", "slab", "stats", "dfeat", "logp", "part", "dzbuf", "dx", "y", "dlogits")


def collect(obj, seen, acc):
    if id(obj) in seen:
        return
    seen.add(id(obj))
    if isinstance(obj, torch.Tensor):
        if obj.is_cuda:
            acc.append(obj)
    elif isinstance(obj, LazyView):
        if obj.t is not None:
            acc.append(obj.t)
    elif isinstance(obj, Act):
        collect(obj.t, seen, acc)
    elif isinstance(obj, dict):
        for v in obj.values():
            collect(v, seen, acc)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            collect(v, seen, acc)
    elif hasattr(obj, "__dict__") and type(obj).__module__.startswith("mtl_das_pytorch_amd"):
        for v in vars(obj).values():
            collect(v, seen, acc)


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
    X, d, e = generate(64, seed=1, device="cuda")
    lab = encode_joint(d, e) if model_type == "multi_classifier" else torch.stack([d, e], 1)
    idx = torch.arange(32, device="cuda")
    tensors = []
    collect(prog, set(), tensors)
    tensors += [prog.flat.params, prog.flat.grads]
    regs = sorted({(t.untyped_storage().data_ptr(), t.untyped_storage().nbytes()): t for t in tensors}.items())

    def find(p):
        for (base, nb), t in regs:
            if base <= p < base + nb:
                return base, nb
        return None

    launches = [(ph, l) for ph in (prog.fwd_train, prog.bwd) for l in ph.launches]
    f = prog.flat
    state = [f.params, f.exp_avg, f.exp_avg_sq, f.bn_mean, f.bn_var, f.bn_nbt, f.step]
    saved = [t.clone() for t in state]

    def run():
        for t, s in zip(state, saved):
            t.copy_(s)
        prog.opt["pack"].run()
        prog.arena.clear()
        prog.gather_phase(X, lab, idx).run()
        snaps = []
        st = stream()
        for ph, l in launches:
            l(st)
            torch.cuda.synchronize()
            d = next((a for a in l.args if isinstance(a, dict)), {})
            outs = []
            for k in OUT_KEYS:
                if l.name.startswith("tail") and k == "y":
                    continue
                v = d.get(k)
                if isinstance(v, int) and v:
                    r = find(v)
                    if r:
                        base, nb = r
                        buf = torch.empty(nb, dtype=torch.uint8, device="cuda")
                        src = torch.tensor([], dtype=torch.uint8, device="cuda").set_(
                            [t for (b, n), t in regs if b == base][0].untyped_storage())
                        buf.copy_(src[:nb])
                        outs.append((k, buf))
            if l.name == "wgrad_finalize":
                outs.append(("grads", f.grads.clone().view(torch.uint8)))
            snaps.append(outs)
        return snaps

    a = run()
    b = run()
    for i, ((ph, l), sa, sb) in enumerate(zip(launches, a, b)):
        for (k, x), (_, y) in zip(sa, sb):
            if k == "stats":
                xf, yf = x.view(torch.float64), y.view(torch.float64)
            elif x.numel() % 4 == 0 and k in ("slab", "part", "dzbuf", "dfeat", "logp", "dx", "grads", "side", "dlogits"):
                xf, yf = x.view(torch.float32), y.view(torch.float32)
            else:
                xf, yf = x.view(torch.bfloat16).float(), y.view(torch.bfloat16).float()
            diff = ((xf - yf).norm() / yf.norm().clamp_min(1e-30)).item()
            flag = " <<<<" if diff > 1e-3 else ""
            if diff > 1e-5:
                print(f"{i:4d} {ph.name:14s} {l.name:14s} {k:6s} rel diff {diff:.3e}{flag}", flush=True)
    print("done")


if __name__ == "__main__":
    main()
