"""Which phase of the Inception program breaks multi-stream HIP-graph capture? Prints before each capture."""
import os
import sys

import torch

sys.path.insert(0, ".")
os.environ.setdefault("MDA_STREAMS", "1")
from mtl_das_pytorch_amd.data.synthetic import generate  # noqa: E402
from mtl_das_pytorch_amd.engine.inception import InceptionProgram  # noqa: E402
from mtl_das_pytorch_amd.models import Multi_Classifier, encode_joint  # noqa: E402

torch.manual_seed(0)
prog = InceptionProgram(Multi_Classifier(), 16, "cuda", p_drop=0.0)
if len(sys.argv) > 1 and sys.argv[1] == "batched":
    prog.batch_wgrads()
X, d, e = generate(32, seed=1, device="cuda")
lab = encode_joint(d, e)
idx = torch.arange(16, device="cuda")
gather = prog.gather_phase(X, lab, idx)
prog.opt["pack"].run()


def capture(name, fns):
    print("capturing", name, flush=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for f in fns:
            f()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for f in fns:
            f()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    print("ok", name, flush=True)


for ph in (prog.fwd_train, prog.bwd):
    streams = sorted({l.stream for l in ph.launches})
    print(ph.name, len(ph.launches), "launches, streams", streams,
          "records", sum(1 for l in ph.launches if l.record), "waits", sum(len(l.waits) for l in ph.launches),
          flush=True)
capture("gather+fwd", [prog.arena.clear, gather.run, prog.fwd_train.run])
capture("bwd", [prog.bwd.run])
capture("full", [prog.arena.clear, gather.run, prog.fwd_train.run, prog.bwd.run, prog.opt["adam"].run])
print("all ok")
