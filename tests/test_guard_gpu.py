"""Out-of-bounds write detector (engine/guard.py): every buffer the engine's kernels write
-- arena activations and gradients, BN replicas, weight-gradient slabs, dz buffers, the LDS conv kernels'
split-K workspaces and tickets, the flat parameter / gradient / moment buffers, the bf16 weight images, head
outputs -- sits between two 4 KiB canary bands.  After real training and evaluation steps of A, B and C at
the bench's batch with the tuned kernel configs (HIP graph), and after every conv / data-gradient / weight-
gradient kernel config on the layer classes of the kernel tests, no band may have changed."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def guarded():
    from mtl_das_pytorch_amd.engine import guard
    guard.reset()
    guard.enable(True)
    yield guard
    guard.enable(False)
    guard.reset()


@pytest.mark.parametrize("model", ["MTL", "single_event", "multi_classifier"])
def test_engine_step_canaries(guarded, model):
    from mtl_das_pytorch_amd.data.synthetic import generate
    from mtl_das_pytorch_amd.engine.inception import InceptionProgram
    from mtl_das_pytorch_amd.engine.mtl import MTLProgram
    from mtl_das_pytorch_amd.engine.step import StepRunner
    from mtl_das_pytorch_amd.engine.tune import autotune_program
    from mtl_das_pytorch_amd.models import build_model, encode_joint
    torch.manual_seed(0)
    B = 32
    joint = model == "multi_classifier"
    prog = InceptionProgram(build_model(model), B, "cuda") if joint else MTLProgram(build_model(model), B, "cuda")
    prog.set_optimizer(weight_decay=1e-5)
    autotune_program(prog, measure=False)  # the bench's configs: LDS split-K workspaces are guarded too
    X, d, e = generate(3 * B, seed=5, device="cuda")
    labels = encode_joint(d, e) if joint else torch.stack([d, e], 1)
    run = StepRunner(prog, X, labels, X_eval=X, labels_eval=labels)
    run.set_lr(1e-3)
    for i in range(2):
        run.train_step(torch.arange(B * i, B * (i + 1), device="cuda"))
    run.eval_step(torch.arange(2 * B, 3 * B, device="cuda"))
    torch.cuda.synchronize()
    assert guarded.count() > 100
    bad = guarded.check()
    assert not bad, bad[:10]
    assert torch.isfinite(prog.flat.params).all()


CASES = [(2, 33, 83, 16, 16, 3, 1, 1), (2, 17, 42, 32, 64, 3, 2, 1), (2, 5, 11, 256, 64, 1, 1, 0),
         (2, 4, 13, 128, 160, (7, 1), 1, (3, 0)), (1, 9, 27, 288, 384, 3, 2, 0), (3, 1, 6, 448, 384, 3, 1, 1),
         (2, 7, 9, 40, 24, 3, 2, 0), (2, 47, 122, 32, 64, 3, 1, 1)]


def test_every_conv_config_canaries(guarded):
    from mtl_das_pytorch_amd.engine.tune import CONV_CFGS
    from mtl_das_pytorch_amd.ops import functional as fn
    g = torch.Generator().manual_seed(0)
    n = 0
    for B, H, W, Ci, Co, k, s, p in CASES:
        kh, kw = (k, k) if isinstance(k, int) else k
        x = torch.randn(B, H, W, Ci, generator=g).bfloat16().cuda()
        w = (torch.randn(Co, Ci, kh, kw, generator=g) / math.sqrt(Ci * kh * kw)).cuda()
        ph, pw = (p, p) if isinstance(p, int) else p
        Ho, Wo = (H + 2 * ph - kh) // s + 1, (W + 2 * pw - kw) // s + 1
        dy = torch.randn(B, Ho, Wo, Co, generator=g).bfloat16().cuda()
        for cfg in CONV_CFGS:
            for mk in (lambda: fn.prepare_conv2d(x, w, None, stride=s, padding=p, cfg=cfg),
                       lambda: fn.prepare_conv2d_dgrad(dy, w, (H, W), stride=s, padding=p, cfg=cfg)):
                try:
                    call = mk()
                except (ValueError, RuntimeError):
                    continue
                call.run()
                n += 1
        for cfg in sorted(fn.WGRAD_TILES) + sorted(fn.WGRAD_PATCH):
            try:
                fn.conv2d_wgrad(x, dy, (Co, Ci, kh, kw), stride=s, padding=p, cfg=cfg)
            except ValueError:
                continue
            n += 1
    torch.cuda.synchronize()
    assert n > 300
    bad = guarded.check()
    assert not bad, bad[:10]
