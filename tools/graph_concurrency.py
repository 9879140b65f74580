"""Does a captured HIP graph execute independent branches (captured on two streams) concurrently?
Times N small conv launches in one stream vs split over two streams (fork/join inside the capture)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.ops import functional as fn  # noqa: E402
from mtl_das_pytorch_amd.ops.hip import lib  # noqa: E402


def make_calls(n):
    calls = []
    for i in range(n):
        x = torch.randn(32, 9, 21, 64, device="cuda").bfloat16()
        w = torch.randn(64, 64, 3, 3, device="cuda") * 0.05
        calls.append(fn.prepare_conv2d(x, w, padding=1, cfg=8))
    return calls


def run(calls, streams):
    main = torch.cuda.current_stream()
    if streams == 1:
        for c in calls:
            lib().conv(c.mode, c.cfg, 1, main.cuda_stream, c.d)
        return
    side = torch.cuda.Stream()
    side.wait_stream(main)
    half = len(calls) // 2
    for c in calls[:half]:
        lib().conv(c.mode, c.cfg, 1, main.cuda_stream, c.d)
    with torch.cuda.stream(side):
        for c in calls[half:]:
            lib().conv(c.mode, c.cfg, 1, side.cuda_stream, c.d)
    main.wait_stream(side)


def bench_eager(streams, n=40, reps=20):
    calls = make_calls(n)
    run(calls, streams)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        run(calls, streams)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def bench(streams, n=40, reps=20):
    calls = make_calls(n)
    run(calls, streams)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        run(calls, streams)
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for st in (1, 2, 1, 2):
    print(f"graph {st} stream(s): {bench(st):.1f} us per 40 launches", flush=True)
for st in (1, 2, 1, 2):
    print(f"eager {st} stream(s): {bench_eager(st):.1f} us per 40 launches", flush=True)
