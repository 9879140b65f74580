"""Minimal, engine-free reproduction attempt of the HIP-runtime segfault seen at graph launch with
GPU_MAX_HW_QUEUES=2 (docs/PERF.md, round 3: Model C's 4-stream step graph).

Only PyTorch ops: a graph is captured over ``--streams`` streams forked from the capture stream with the
join-then-fork event pattern of engine/program.py (every side stream waits for a fork event, records its
own events, some streams wait on other streams' events mid-phase, all are joined at the end), then
replayed ``--replays`` times.  Run it under the queue setting in question:

    GPU_MAX_HW_QUEUES=2 python -X faulthandler tools/hwq_repro.py --streams 4

If this crashes, the fault is in the runtime's mapping of graph branches onto fewer hardware queues than
streams (no engine code involved); if it does not, the engine's own launches are the next suspects.
"""
import argparse
import os

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--layers", type=int, default=40, help="fork / work / cross-wait / join rounds per graph")
    ap.add_argument("--replays", type=int, default=200)
    ap.add_argument("--numel", type=int, default=1 << 18)
    args = ap.parse_args()
    print("GPU_MAX_HW_QUEUES =", os.environ.get("GPU_MAX_HW_QUEUES", "(default)"), flush=True)
    dev = torch.device("cuda")
    bufs = [torch.zeros(args.numel, device=dev) for _ in range(args.streams)]
    side = [torch.cuda.Stream() for _ in range(args.streams - 1)]
    keep = []

    def body():
        main = torch.cuda.current_stream()
        streams = [main] + side
        for layer in range(args.layers):
            fork = main.record_event()
            keep.append(fork)
            for s in side:
                s.wait_event(fork)
            evs = []
            for i, s in enumerate(streams):
                with torch.cuda.stream(s):
                    bufs[i].mul_(0.5).add_(float(layer + i))
                    evs.append(s.record_event())
            keep.extend(evs)
            # a cross-stream edge mid-phase (as the Inception branches' collectives / concat joins)
            if args.streams > 2:
                side[0].wait_event(evs[-1])
                with torch.cuda.stream(side[0]):
                    bufs[1].add_(bufs[-1][:1].sum())
            for s in side:
                main.wait_stream(s)

    s0 = torch.cuda.Stream()
    s0.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s0):
        body()  # warm-up
    torch.cuda.current_stream().wait_stream(s0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    torch.cuda.synchronize()
    print("captured", flush=True)
    for i in range(args.replays):
        g.replay()
        if i % 50 == 0:
            torch.cuda.synchronize()
            print("replay", i, float(bufs[0][0]), flush=True)
    torch.cuda.synchronize()
    g.reset()
    print("ok", flush=True)


if __name__ == "__main__":
    main()
