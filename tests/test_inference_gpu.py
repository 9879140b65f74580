"""GPU: engine-path sliding-window inference vs the fp32 module; bitwise step determinism (race check)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("model_type", ["MTL", "multi_classifier"])
def test_engine_inference_matches_module(model_type):
    from mtl_das_pytorch_amd.inference import predict_recording
    from mtl_das_pytorch_amd.models import build_model
    torch.manual_seed(0)
    m = build_model(model_type)
    # give BN non-trivial running statistics so eval mode is exercised
    m.train()
    with torch.no_grad():
        m(torch.randn(8, 1, 100, 250))
    m.eval()
    ref_model = build_model(model_type)
    ref_model.load_state_dict(m.state_dict())
    ref_model.eval().cuda()
    rec = torch.randn(200, 700)
    eng = predict_recording(m, model_type, rec, stride=(100, 150), batch=8, device="cuda", use_engine=True)
    ref = predict_recording(ref_model, model_type, rec, stride=(100, 150), batch=8, device="cuda", use_engine=False)
    key = "joint_prob" if model_type == "multi_classifier" else "event_prob"
    err = np.abs(eng[key] - ref[key]).max()
    assert err < 5e-2, err
    pk = "joint_pred" if model_type == "multi_classifier" else "distance_pred"
    assert (eng[pk] == ref[pk]).mean() > 0.8


@pytest.mark.parametrize("model_type", ["MTL", "multi_classifier"])
@pytest.mark.parametrize("use_graph", [False, True])
def test_training_step_is_bitwise_deterministic(model_type, use_graph):
    from mtl_das_pytorch_amd.data.synthetic import generate
    from mtl_das_pytorch_amd.engine.determinism import check_step
    from mtl_das_pytorch_amd.models import build_model, encode_joint
    torch.manual_seed(0)
    m = build_model(model_type)
    X, d, e = generate(32, seed=2, device="cuda")
    if model_type == "multi_classifier":
        from mtl_das_pytorch_amd.engine.inception import InceptionProgram
        prog, lab = InceptionProgram(m, 16, "cuda"), encode_joint(d, e)
    else:
        from mtl_das_pytorch_amd.engine.mtl import MTLProgram
        prog, lab = MTLProgram(m, 16, "cuda"), torch.stack([d, e], 1)
    res = check_step(prog, X, lab, torch.arange(16, device="cuda"), use_graph=use_graph, runs=3)
    assert res["bitwise_equal"], res


def test_race_bisection_finds_nothing_on_a_deterministic_step():
    """The launch-level race bisection (engine/determinism.py first_divergent_launch) runs the step launch by
    launch twice and compares every written buffer bitwise: the engine's step has no divergent launch."""
    from mtl_das_pytorch_amd.data.synthetic import generate
    from mtl_das_pytorch_amd.engine.determinism import first_divergent_launch
    from mtl_das_pytorch_amd.engine.mtl import MTLProgram
    from mtl_das_pytorch_amd.models import build_model
    torch.manual_seed(0)
    prog = MTLProgram(build_model("MTL"), 16, "cuda")
    X, d, e = generate(16, seed=3, device="cuda")
    assert first_divergent_launch(prog, X, torch.stack([d, e], 1), torch.arange(16, device="cuda")) is None
