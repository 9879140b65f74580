#!/usr/bin/env python3
"""Run an entry script (default bench.py) with engine class switches or module constants overridden, for
same-call A/B measurements without per-feature environment knobs:

    python tools/variant.py engine.mtl.MTLProgram.SIDE_WGRAD_GRID=0 engine.core.BN_PX_PER_REP=256 \\
        -- --steps 300 --warmup 30
    python tools/variant.py --script tools/timeline.py engine.mtl.MTLProgram.SIDE_WGRAD_GRID=0 -- MTL

Each override is ``<module under mtl_das_pytorch_amd>.<Class>.<ATTR>=<python literal>`` (or
``<module>.<ATTR>=...`` for a module constant); values that are not Python literals are taken as strings.
The overrides are printed to stderr, so every log names the variant it measured."""
import ast
import importlib
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def apply(spec: str):
    path, val = spec.split("=", 1)
    try:
        v = ast.literal_eval(val)
    except (ValueError, SyntaxError):
        v = val
    parts = path.split(".")
    # longest importable module prefix, then attribute lookups
    for k in range(len(parts) - 1, 0, -1):
        try:
            obj = importlib.import_module("mtl_das_pytorch_amd." + ".".join(parts[:k]))
        except ImportError:
            continue
        for a in parts[k:-1]:
            obj = getattr(obj, a)
        if not hasattr(obj, parts[-1]):
            raise AttributeError(f"{path}: no attribute {parts[-1]}")
        setattr(obj, parts[-1], v)
        print(f"variant: {path} = {v!r}", file=sys.stderr, flush=True)
        return
    raise ImportError(path)


def main():
    argv = sys.argv[1:]
    script = os.path.join(ROOT, "bench.py")
    if argv[:1] == ["--script"]:
        script, argv = os.path.join(ROOT, argv[1]), argv[2:]
    rest = []
    if "--" in argv:
        i = argv.index("--")
        argv, rest = argv[:i], argv[i + 1:]
    for spec in argv:
        apply(spec)
    sys.argv = [script] + rest
    runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()
