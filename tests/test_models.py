"""Model zoo parity: reference state_dict key spaces, parameter counts, shapes, complexity ratios."""
import pytest
import torch

from mtl_das_pytorch_amd.models import (MTL_Net, Multi_Classifier, Single_Task_Net, build_model, decode_joint,
                                        encode_joint)
from mtl_das_pytorch_amd.utils.flops import complexity_report, count_macs


@pytest.mark.parametrize("ctor,keys,params,tensors,buf", [
    (lambda: MTL_Net(), 268, 1136224, 142, 4778),
    (lambda: Single_Task_Net("distance"), 194, 918376, 101, 3599),
    (lambda: Single_Task_Net("event"), 194, 918376, 101, 3599),
    (lambda: Multi_Classifier(init_weights=False), 566, 21850560, 284, 34526),
])
def test_state_dict_census(ctor, keys, params, tensors, buf):
    m = ctor()
    sd = m.state_dict()
    assert len(sd) == keys
    assert sum(p.numel() for p in m.parameters()) == params
    assert len(list(m.parameters())) == tensors
    assert sum(b.numel() for b in m.buffers()) == buf


def test_reference_key_names():
    sd = MTL_Net().state_dict()
    for k in ["conv1.0.weight", "conv1.1.running_var", "resblock3.shortcut.0.weight", "resblock1.left.4.bias",
              "att_mask_generator1.1.3.bias", "att_mask_generato2.0.0.weight", "att_mask_generator4.1.4.num_batches_tracked",
              "output_layer3.1.0.weight", "output_layer1.0.1.running_mean"]:
        assert k in sd, k
    assert "resblock1.shortcut.0.weight" not in sd  # identity shortcut
    assert sd["conv1.0.weight"].shape == (16, 1, 7, 7)
    assert sd["att_mask_generato2.0.0.weight"].shape == (16, 64, 1, 1)
    csd = Multi_Classifier(init_weights=False).state_dict()
    for k in ["Conv2d_1a_3x3.conv.weight", "Mixed_5b.branch_pool.bn.running_var", "Mixed_6e.branch7x7dbl_5.conv.weight",
              "Mixed_7c.branch3x3dbl_3b.bn.weight", "fc.weight", "fc.bias"]:
        assert k in csd, k
    assert csd["Conv2d_1a_3x3.conv.weight"].shape == (32, 1, 3, 3)
    assert csd["fc.weight"].shape == (32, 2048)


def test_forward_shapes_and_logprobs():
    torch.manual_seed(0)
    x = torch.randn(2, 1, 100, 250)
    a = MTL_Net().eval()
    d, e = a(x)
    assert d.shape == (2, 16) and e.shape == (2, 2)
    assert torch.allclose(d.exp().sum(1), torch.ones(2), atol=1e-5)
    for task, n in (("distance", 16), ("event", 2)):
        o = Single_Task_Net(task).eval()(x)
        assert o.shape == (2, n)
    c = Multi_Classifier().eval()
    assert c(x).shape == (2, 32)


def test_checkpoint_roundtrip_strict(tmp_path):
    m = MTL_Net()
    p = tmp_path / "a.pth"
    torch.save(m.state_dict(), p)
    m2 = MTL_Net()
    m2.load_state_dict(torch.load(p, map_location="cpu", weights_only=True), strict=True)
    for (k, v), (_, v2) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(v, v2), k


def test_in_channels_changes_stem_only():
    m = MTL_Net(in_channels=2)
    assert m.state_dict()["conv1.0.weight"].shape == (16, 2, 7, 7)
    assert m(torch.randn(1, 2, 100, 250))[0].shape == (1, 16)


def test_complexity_ratios_reproduce_readme():
    r = complexity_report()
    assert r["macs"]["A"] == 220687584
    assert r["macs"]["B_distance"] == r["macs"]["B_event"] == 163077952
    assert r["macs"]["C"] == 1113630592
    assert round(r["ratio_A_over_2B"], 3) == 0.677
    assert round(r["ratio_A_over_C"], 3) == 0.198


def test_joint_label_codec():
    d = torch.arange(16).repeat(2)
    e = torch.arange(2).repeat_interleave(16)
    j = encode_joint(d, e)
    assert j.tolist() == list(range(32))
    d2, e2 = decode_joint(j)
    assert torch.equal(d2, d) and torch.equal(e2, e)


def test_factory():
    for t in ("MTL", "single_distance", "single_event"):
        assert build_model(t) is not None
    with pytest.raises(ValueError):
        build_model("nope")


def test_inception_init_is_truncated_normal():
    torch.manual_seed(0)
    c = Multi_Classifier()
    w = c.Mixed_6b.branch7x7_2.conv.weight
    assert w.abs().max() <= 0.2 + 1e-6 and 0.05 < w.std() < 0.1
    assert torch.all(c.Mixed_5b.branch1x1.bn.weight == 1)


def test_fc_head_ablation():
    """head="fc" (docs/ACCURACY.md backbone-vs-head ablation): a learned linear layer per task on the pooled
    features; the reference head's key space is untouched, the trainer keeps it off the engine."""
    from mtl_das_pytorch_amd.engine.trainer import Trainer
    from mtl_das_pytorch_amd.utils.config import TrainConfig
    m = build_model("MTL", head="fc")
    sd = m.state_dict()
    assert len(sd) == 268 + 4 and sd["task1fc.weight"].shape == (16, 128) and sd["task2fc.weight"].shape == (2, 128)
    d, e = m.eval()(torch.randn(2, 1, 100, 250))
    assert d.shape == (2, 16) and e.shape == (2, 2)
    assert torch.allclose(d.exp().sum(1), torch.ones(2), atol=1e-5)
    assert build_model("single_distance", head="fc")(torch.randn(1, 1, 100, 250)).shape == (1, 16)
    with pytest.raises(ValueError):
        build_model("multi_classifier", head="fc")
    with pytest.raises(ValueError):
        build_model("MTL", head="nope")
    tr = Trainer(TrainConfig(model="MTL", head="fc", synthetic=1, output_savedir="/tmp/mda_fc_head_test"))
    assert tr.backend_name == "torch"
    with pytest.raises(ValueError):
        Trainer(TrainConfig(model="MTL", head="fc", backend="engine", synthetic=1,
                            output_savedir="/tmp/mda_fc_head_test"))._pick_backend()
