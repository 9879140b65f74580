"""Per-layer kernel autotuning on the device.

Every conv forward / data-gradient launch of a lowered program has 14 tile configurations
(csrc/conv.hip ``launch_conv_cfg``: wave layout channels x pixels x K-split).  The best one depends on
the layer's M (B*H*W), N (channels) and K (taps*Cin) and on MI355X's CU count, so it is *measured*:
each candidate is timed from a HIP graph of back-to-back launches (no host overhead), the fastest is
written into the launch, and the result is cached by shape signature in ``tuned_cfgs.json`` (shipped in
the package, so normal runs do not pay the tuning time).
"""
from __future__ import annotations

import json
import os
from typing import Dict, Iterable, Optional

import torch

from ..ops.functional import (CONV_DEEP_CFG0, CONV_DEEP_NCFG, CONV_LDS_CFG0, CONV_LDS_NCFG, WGRAD_PATCH, WGRAD_TILES,
                              conv_workspace)
from ..ops.hip import lib

# conv.hip register-pipelined tiles 0-13 (pipeline depth 2, and 4 at CONV_DEEP_CFG0 + tile), then
# conv_lds.hip LDS-staged tiles x K chunk x K split
CONV_CFGS = (list(range(14)) + list(range(CONV_LDS_CFG0, CONV_LDS_CFG0 + CONV_LDS_NCFG))
             + list(range(CONV_DEEP_CFG0, CONV_DEEP_CFG0 + CONV_DEEP_NCFG)))


def fused_max_m(kind: int) -> int:
    """csrc/bn.hip tail_bwd_fused_kernel: 1024 threads x <= 4 register-cached pixels (2 for ADD_RELU)."""
    return 1024 * (2 if kind == 4 else 4)
WGRAD_CFGS = sorted(WGRAD_TILES) + sorted(WGRAD_PATCH)
_CACHE_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned_cfgs.json")


def conv_signature(mode: int, G: int, d: dict) -> str:
    keys = ("B", "Hs", "Ws", "Ho", "Wo", "N", "Cs", "KH", "KW", "sh", "sw", "ph", "pw")
    src = d["src"]
    sig = f"conv{mode}|G{G}|" + ",".join(str(d[k]) for k in keys) + f"|seg{int(src.get('C1', 0) > 0)}" + \
          f"|st{int(bool(d.get('stats')))}"
    return sig


def load_cache(path: str = _CACHE_PATH) -> Dict[str, int]:
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def save_cache(cache: Dict[str, int], path: str):
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        json.dump(dict(sorted(cache.items())), f, indent=0)


def _time(fn, inner: int = 10, reps: int = 5) -> float:
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(inner):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (inner * reps)


def autotune_phases(phases: Iterable, cache: Optional[Dict[str, int]] = None, verbose: bool = False,
                    measure: bool = True) -> Dict[str, int]:
    """Choose the conv tile config of every conv launch in ``phases`` (mutates the launches).  With
    ``measure=False`` only cached choices are applied (layers missing from the cache keep the heuristic)."""
    cache = load_cache() if cache is None else cache
    L = lib()
    for ph in phases:
        keep = ph.__dict__.setdefault("ws_keep", {})  # split-K workspaces of the chosen LDS configs
        for launch in ph.launches:
            if launch.name not in ("conv_fwd", "conv_dgrad"):
                continue
            mode, cfg, G, d = launch.args
            sig = conv_signature(mode, G, d)
            if sig not in cache and not measure:
                continue
            if sig not in cache:
                best, best_t = cfg, float("inf")
                dev = torch.device("cuda", torch.cuda.current_device())
                for c in CONV_CFGS:
                    dc = dict(d)
                    ws = conv_workspace(mode, c, G, dc, dev)
                    if ws is None:
                        continue
                    t = _time(lambda: L.conv(mode, c, G, torch.cuda.current_stream().cuda_stream, dc))
                    del ws
                    if t < best_t:
                        best, best_t = c, t
                cache[sig] = best
                if verbose:
                    print(f"tuned {sig}: cfg {best} ({best_t * 1e3:.1f} us)", flush=True)
            cfg = cache[sig]
            ws = conv_workspace(mode, cfg, G, d, torch.device("cuda", torch.cuda.current_device()))
            if ws is None:
                raise RuntimeError(f"cached conv config {cfg} is invalid for {sig}")
            keep[id(launch)] = ws
            launch.args = (mode, cfg, G, d)
    for ph in phases:
        for launch in ph.launches:
            if launch.name != "conv_wgrad" or launch.owner is None:
                continue
            cfg, G, d = launch.args
            conv = launch.owner
            sig = "wgrad|" + conv_signature(0, G, dict(d, N=d["Co"], Hs=d["Hi"], Ws=d["Wi"], stats=0))
            if sig not in cache and not measure:
                continue
            if sig not in cache:
                best, best_t = cfg, float("inf")
                for c in WGRAD_CFGS:
                    if not conv.wgrad_valid(c):
                        continue
                    conv.set_wgrad_cfg(c)
                    t = _time(lambda: L.wgrad(c, G, torch.cuda.current_stream().cuda_stream, d))
                    if t < best_t:
                        best, best_t = c, t
                cache[sig] = best
                if verbose:
                    print(f"tuned {sig}: cfg {best} ({best_t * 1e3:.1f} us)", flush=True)
            conv.set_wgrad_cfg(cache[sig])
            launch.args = (cache[sig], G, d)
    # BN backward: reduce + apply (grid over pixels, replica atomics) vs the single-launch variant
    # (one block per 8 channels over all pixels) -- the crossover depends on M, C and the sources
    for ph in phases:
        for launch in ph.launches:
            if not launch.name.startswith("tailbwd"):
                continue
            kind, G, blocks, d = launch.args
            if d.get("fused") in (2, 3):  # statistics from the producers (apply only) / a partial reduce
                continue
            sig = tail_bwd_signature(kind, G, d)
            if sig not in cache and not measure:
                continue
            if sig not in cache:
                fusable = d["B"] * d["H"] * d["W"] <= fused_max_m(kind)
                ts = [_time(lambda: L.tail_bwd(kind, G, blocks, torch.cuda.current_stream().cuda_stream,
                                                dict(d, fused=f))) if (f == 0 or fusable) else float("inf")
                      for f in (0, 1)]
                cache[sig] = int(ts[1] < ts[0])
                if verbose:
                    print(f"tuned {sig}: fused={cache[sig]} ({ts[0] * 1e3:.1f} / {ts[1] * 1e3:.1f} us)", flush=True)
            d["fused"] = cache[sig]
    return cache


def tail_bwd_signature(kind: int, G: int, d: dict) -> str:
    return (f"tailbwd|k{kind}|G{G}|{d['B']},{d['H']},{d['W']},{d['C']}|src{len(d['g'])}"
            f"|bn2{int('bn2' in d)}|side{int(bool(d.get('side')))}")


def autotune_program(prog, out_path: Optional[str] = None, verbose: bool = False, measure: bool = True,
                     batch_wgrads: bool = True) -> Dict[str, int]:
    """Tune every conv launch of a lowered program (train forward, eval forward, backward), then batch the
    weight-gradient launches per tile config (``batch_wgrads``)."""
    if prog.device.type != "cuda":
        return {}
    cache = {} if os.environ.get("MDA_RETUNE") == "1" else load_cache()
    n0 = len(cache)
    autotune_phases([prog.fwd_train, prog.fwd_eval, prog.bwd], cache, verbose, measure)
    if batch_wgrads:
        prog.merge_wgrad_cfgs()
    prog.refresh_wgrad_finalize()
    if batch_wgrads:
        prog.batch_wgrads()
    if out_path and len(cache) != n0:
        save_cache(cache, out_path)
    return cache
