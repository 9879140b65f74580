"""Built-in complexity counter (replaces the reference's commented-out ptflops call, utils.py:127-131).

Counts multiply-accumulates per sample with module forward hooks using the same conventions as
ptflops 0.6.x, which is what produced the README's complexity claims (README.md:8):

  Conv2d          out_elems * Cin/groups * kh * kw  (+ out_elems if bias)
  BatchNorm2d     in_elems * (2 if affine else 1)
  ReLU / Sigmoid  out_elems
  Max/Avg pools   in_elems (incl. adaptive and 1-d pools)
  Linear          in_elems * out_features (bias not counted)

Functional ops (``F.relu``, ``torch.cat``, ``*``, ``F.avg_pool2d``) and ``nn.Dropout`` are
not counted, exactly like ptflops' module-hook backend.  With these rules the
model zoo reproduces the published ratios: MACs(A) / (MACs(B_dist) + MACs(B_event)) = 0.677 (67.8%)
and MACs(A) / MACs(C) = 0.198 (19.8%).
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch
import torch.nn as nn

_POOLS = (nn.MaxPool1d, nn.MaxPool2d, nn.AvgPool1d, nn.AvgPool2d, nn.AdaptiveAvgPool1d, nn.AdaptiveAvgPool2d,
          nn.AdaptiveMaxPool2d)
_ACTS = (nn.ReLU, nn.ReLU6, nn.LeakyReLU, nn.ELU, nn.PReLU, nn.Sigmoid)


def _module_macs(m: nn.Module, inp: torch.Tensor, out: torch.Tensor) -> int:
    if isinstance(m, nn.Conv2d):
        kh, kw = m.kernel_size
        per_pos = kh * kw * (m.in_channels // m.groups) * m.out_channels
        positions = out.shape[0] * out.shape[2] * out.shape[3]
        return per_pos * positions + (m.out_channels * positions if m.bias is not None else 0)
    if isinstance(m, nn.BatchNorm2d):
        return inp.numel() * (2 if m.affine else 1)
    if isinstance(m, _ACTS):
        return out.numel()
    if isinstance(m, _POOLS):
        return inp.numel()
    if isinstance(m, nn.Linear):
        return inp.numel() * m.out_features
    return 0


@torch.no_grad()
def count_macs(model: nn.Module, input_res: Tuple[int, ...] = (1, 100, 250), per_layer: bool = False):
    """Return ``(macs_per_sample, n_params)`` (and a per-module dict when ``per_layer``)."""
    totals: Dict[str, int] = {}
    hooks = []
    names = {m: n for n, m in model.named_modules()}

    def hook(m, i, o):
        x = i[0] if isinstance(i, tuple) else i
        totals[names[m]] = totals.get(names[m], 0) + _module_macs(m, x, o)

    for m in model.modules():
        if len(list(m.children())) == 0:
            hooks.append(m.register_forward_hook(hook))
    was_training = model.training
    model.eval()
    try:
        dev = next(model.parameters()).device
        model(torch.zeros((1,) + tuple(input_res), device=dev))
    finally:
        for h in hooks:
            h.remove()
        model.train(was_training)
    macs = sum(totals.values())
    params = sum(p.numel() for p in model.parameters() if p.requires_grad)
    return (macs, params, totals) if per_layer else (macs, params)


def complexity_report(input_res=(1, 100, 250)) -> dict:
    """MACs / params of A, B_dist, B_event, C and the two published ratios."""
    from ..models import MTL_Net, Multi_Classifier, Single_Task_Net
    a, pa = count_macs(MTL_Net(), input_res)
    bd, pbd = count_macs(Single_Task_Net("distance"), input_res)
    be, pbe = count_macs(Single_Task_Net("event"), input_res)
    c, pc = count_macs(Multi_Classifier(init_weights=False), input_res)
    return {"macs": {"A": a, "B_distance": bd, "B_event": be, "C": c},
            "params": {"A": pa, "B_distance": pbd, "B_event": pbe, "C": pc},
            "ratio_A_over_2B": a / (bd + be), "ratio_A_over_C": a / c}


def main(argv=None):
    """``python -m mtl_das_pytorch_amd.utils.flops [--model M] [--per_layer]``: the ptflops-style report the
    reference prints (commented out at utils.py:127-131), plus the README's 67.8 % / 19.8 % ratios."""
    import argparse
    import json
    ap = argparse.ArgumentParser(description=main.__doc__)
    ap.add_argument("--model", default=None, help="MTL | single_distance | single_event | multi_classifier")
    ap.add_argument("--input_res", default="1,100,250")
    ap.add_argument("--per_layer", action="store_true")
    args = ap.parse_args(argv)
    res = tuple(int(x) for x in args.input_res.split(","))
    if args.model is None:
        print(json.dumps(complexity_report(res), indent=1))
        return
    from ..models import build_model
    m = build_model(args.model, in_channels=res[0])
    if args.per_layer:
        macs, params, per = count_macs(m, res, per_layer=True)
        for name, v in per.items():
            print(f"{name:60s} {v / 1e6:10.3f} MMac")
    else:
        macs, params = count_macs(m, res)
    print(f"Computational complexity: {macs / 1e9:.3f} GMac")
    print(f"Number of parameters: {params / 1e6:.3f} M")


if __name__ == "__main__":
    main()
