"""The world > 1 data-parallel step (engine/step.py "train_ext"): forward + backward as ONE
HIP graph that records an EXTERNAL event where each gradient bucket is complete; the host then makes the
communication stream wait for bucket k's event and issues bucket k's collective there, overlapping the rest of
the backward.  The collective here is a stand-in that ADDS 1 to its bucket on the communication stream: if the
external event did not order it after the bucket's finalize (a graph event-record node the runtime ignored, a
wait on a stale record), the finalize would overwrite the +1 and the step would differ from the eager reference
(forward + backward, then +1 on the whole gradient, then Adam) -- so bitwise equality after several steps
proves the ordering for every bucket of every step."""
import pytest
import torch

pytestmark = pytest.mark.gpu


class _AddOne:
    """FlatGradAllReducer's interface; ``start`` enqueues on the CURRENT stream (the communication stream)."""
    capturable = False

    class ctx:  # noqa: N801 (FlatGradAllReducer.ctx)
        enabled = False

    def __init__(self):
        self.pending = []

    def start(self, t):
        t.add_(1.0)
        self.pending.append(torch.cuda.current_stream())

    def finish(self):
        for s in self.pending:
            torch.cuda.current_stream().wait_stream(s)
        self.pending = []

    def __call__(self, g):
        g.add_(1.0)


def _run(model_type, buckets, graph, form, steps=3):
    from mtl_das_pytorch_amd.data.synthetic import generate
    from mtl_das_pytorch_amd.engine.inception import InceptionProgram
    from mtl_das_pytorch_amd.engine.lowering import build_for_stream_buckets
    from mtl_das_pytorch_amd.engine.mtl import MTLProgram
    from mtl_das_pytorch_amd.engine.step import StepRunner
    from mtl_das_pytorch_amd.engine.tune import autotune_program
    from mtl_das_pytorch_amd.models import build_model, encode_joint
    B = 32
    torch.manual_seed(1234)
    m = build_model(model_type)
    joint = model_type == "multi_classifier"

    def make(order, nseg=1):
        p = InceptionProgram(m, B, "cuda", param_order=order) if joint else MTLProgram(m, B, "cuda")
        p.set_optimizer(weight_decay=1e-5, data_parallel=True)
        p.segment_backward(nseg)
        autotune_program(p, measure=False)
        return p

    if form == "stream":  # the multi-rank default (Model C rebuilt with stream_param_order)
        prog, bl = build_for_stream_buckets(make, buckets)
        nb = len(bl)
    else:
        prog = make(None, buckets)
        nb = len(prog.buckets)
    X, d, e = generate(4 * B, seed=11, device="cuda")
    labels = encode_joint(d, e) if joint else torch.stack([d, e], 1)
    runner = StepRunner(prog, X, labels, use_graph=graph, allreduce=_AddOne())
    runner.set_lr(1e-3)
    for i in range(steps):
        runner.train_step(torch.arange(B * i, B * (i + 1), device="cuda") % X.shape[0])
    torch.cuda.synchronize()
    f = prog.flat
    out = {k: getattr(f, k).detach().clone() for k in ("params", "grads", "exp_avg", "exp_avg_sq", "bn_mean", "bn_var")}
    info = {"buckets": nb, "ext": runner.ext_dp, "graphs": sorted(runner.graphs)}
    runner.close()
    return out, info


@pytest.mark.parametrize("model_type,buckets,form", [("MTL", 2, "stream"), ("MTL", 2, "segmented"),
                                                     ("multi_classifier", 4, "segmented"),
                                                     ("multi_classifier", 4, "stream")])
def test_external_bucket_events_order_the_collectives(model_type, buckets, form):
    """form "stream": LoweredProgram.stream_buckets (the multi-rank default: buckets completed by a side stream's
    finalize, no cut); "segmented": segment_backward's cut backward (bucket events after each bucket's finalize)."""
    ref, rinfo = _run(model_type, buckets, graph=False, form=form)
    got, info = _run(model_type, buckets, graph=True, form=form)
    assert not rinfo["ext"] and info["ext"] and info["buckets"] == buckets, info
    assert "train_ext" in info["graphs"] and "train_opt" in info["graphs"]
    bad = [k for k in ref if not torch.equal(ref[k], got[k])]
    assert not bad, bad
