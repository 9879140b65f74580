"""Round-5 crash bisection helper (profiles/r5_runtime_faults.md): tools/accuracy_table.py on the current engine
with ONE of the round-5 lifetime fixes reverted to its round-4 behaviour:

    --pool-streams   every phase draws its side streams from torch's round-robin pool (round 4) instead of
                     the engine's fixed stream set
    --no-keeper      a capture's events are kept by the phase until its next run (round 4) instead of living as
                     long as the graph
    --no-close       Trainer/EngineBackend.close disabled (graphs live until garbage collection)
"""
import os
import runpy
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mtl_das_pytorch_amd.engine import backends, program  # noqa: E402

args = sys.argv[1:]
if "--pool-streams" in args:
    args.remove("--pool-streams")

    class _Pool:
        def __init__(self, device):
            self.streams = [torch.cuda.Stream(device=device) for _ in range(program.MAX_STREAMS + 1)]

        def destroy(self):
            pass

    _run = program.Phase.run

    def run(self, st=None):
        dev = torch.cuda.current_stream().device
        if "_pool" not in self.__dict__:
            self.__dict__["_pool"] = _Pool(dev)
        program.EngineStreams._by_device[dev] = self.__dict__["_pool"]
        return _run(self, st)

    program.Phase.run = run
    print("bisect: pool streams per phase", flush=True)
if "--no-keeper" in args:
    args.remove("--no-keeper")
    program.EventKeeper.__enter__ = lambda self: self
    print("bisect: capture events kept by the phase", flush=True)
if "--no-close" in args:
    args.remove("--no-close")
    backends.EngineBackend.close = lambda self: None
    print("bisect: no close", flush=True)
sys.argv = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "accuracy_table.py")] + args
runpy.run_path(sys.argv[0], run_name="__main__")
