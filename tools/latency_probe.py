"""Latency calibration (see latency_probe.hip).  Prints per-launch times from graph replays."""
import ctypes
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "latency_probe.so")


def build():
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", SO,
                           os.path.join(HERE, "latency_probe.hip")])


def timeit(f, reps=20, inner=20):
    f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(inner):
            f()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (reps * inner) * 1e3


def main():
    if not os.path.exists(SO) or "--build" in sys.argv:
        build()
    if "--build-only" in sys.argv:
        return
    lib = ctypes.CDLL(SO)
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for b, t in [(1, 64), (48, 256), (48, 1024), (256, 256), (1024, 256), (4096, 256)]:
        print(f"empty kernel {b}x{t}: {timeit(lambda: lib.launch_empty(b, t, st())):.2f} us", flush=True)
    for n in [1 << 10, 1 << 16, 1 << 20, 1 << 23]:
        x = torch.randn(n, device="cuda")
        y = torch.empty_like(x)
        for t in (256, 1024):
            us = timeit(lambda: lib.launch_copy(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()), n, t, st()))
            print(f"copy {n} floats, {t} thr/block: {us:.2f} us ({8 * n / us / 1e3:.0f} GB/s)", flush=True)
    out = torch.zeros(1, dtype=torch.int32, device="cuda")
    for ring, label in [(1 << 12, "16KB ring"), (1 << 24, "64MB ring")]:
        perm = torch.randperm(ring)
        nxt = torch.empty(ring, dtype=torch.int32)
        nxt[perm] = torch.roll(perm, -1).int()
        nxt = nxt.cuda()
        for cached in (1, 0):
            t0 = timeit(lambda: lib.launch_chase(ctypes.c_void_p(nxt.data_ptr()), 1, ctypes.c_void_p(out.data_ptr()), cached, st()), reps=5, inner=10)
            t1 = timeit(lambda: lib.launch_chase(ctypes.c_void_p(nxt.data_ptr()), 201, ctypes.c_void_p(out.data_ptr()), cached, st()), reps=5, inner=10)
            print(f"pointer chase {label} {'cached' if cached else 'nontemporal'}: {(t1 - t0) / 200 * 1e3:.0f} ns/hop", flush=True)


if __name__ == "__main__":
    main()
