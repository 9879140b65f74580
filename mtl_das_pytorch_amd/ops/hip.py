"""Loader for the in-tree HIP extension ``_mda_hip`` (built from ``csrc/`` by ``csrc/build.py``).

``torch`` is imported first so that the process already holds torch's HIP runtime
(``libamdhip64.so.7``) when the extension is dlopen'ed; the extension then binds to that same runtime
and its kernels run on PyTorch's streams (graph capture included).

On a machine with a GPU the extension is mandatory: :func:`lib` raises if it is missing or fails to
load, so GPU code paths can never silently fall back to eager PyTorch.
"""
from __future__ import annotations

import importlib
import os
import sys

import torch

_LIB = None
_ERR = None


def _load():
    global _LIB, _ERR
    if _LIB is not None or _ERR is not None:
        return
    try:
        pkg_dir = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        if os.environ.get("MDA_AUTOBUILD", "1") == "1":
            from ..csrc import build as _b
            if _b.needs_build():
                _b.build(verbose=False)
        if pkg_dir not in sys.path:
            sys.path.insert(0, pkg_dir)
        alt = os.environ.get("MDA_EXT_PATH")  # A/B measurements: another build of the same extension
        if alt:
            from importlib import util as _ilu
            spec = _ilu.spec_from_file_location("mtl_das_pytorch_amd._mda_hip", alt)
            _LIB = _ilu.module_from_spec(spec)
            spec.loader.exec_module(_LIB)
            sys.modules["mtl_das_pytorch_amd._mda_hip"] = _LIB
            return
        _LIB = importlib.import_module("mtl_das_pytorch_amd._mda_hip")
    except Exception as e:  # pragma: no cover - exercised on broken installs
        _ERR = e


def available() -> bool:
    _load()
    return _LIB is not None


def lib():
    """The extension module; raises (loudly) when it cannot be loaded."""
    _load()
    if _LIB is None:
        raise RuntimeError(f"mtl_das_pytorch_amd HIP extension unavailable: {_ERR!r}. "
                           f"Build it with `python -m mtl_das_pytorch_amd.csrc.build`.")
    return _LIB


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t: torch.Tensor, offset_elems: int = 0) -> int:
    return t.data_ptr() + offset_elems * t.element_size() if t is not None else 0
