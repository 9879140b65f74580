"""train.py / test.py semantics on the MI355X engine backend."""
import glob
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_engine_trainer_learns_and_checkpoints(tmp_path):
    """Same data, seed and schedule on the engine (bf16 HIP) and on the fp32 torch path: the engine must
    learn at least about as well."""
    from mtl_das_pytorch_amd.engine.trainer import Trainer
    from mtl_das_pytorch_amd.utils.config import TrainConfig
    last = {}
    for backend in ("torch", "engine"):
        cfg = TrainConfig(model="MTL", synthetic=16, batch_size=32, epoch_num=6, val_every=3, log_every=4,
                          output_savedir=str(tmp_path / backend), save_threshold=0.0, backend=backend, seed=1)
        tr = Trainer(cfg)
        assert tr.backend_name == backend
        tr.run()
        last[backend] = tr.last_val["acc"]
    print(last)
    assert last["engine"]["event"] > 0.6, last
    assert last["engine"]["event"] > last["torch"]["event"] - 0.15, last
    tmp_path = tmp_path / "engine"
    d = glob.glob(str(tmp_path / "* model_type=MTL is_test=False"))[0]
    pths = sorted(glob.glob(os.path.join(d, "*.pth")))
    assert pths
    # the engine checkpoint evaluates identically (up to bf16) on the fp32 torch path
    from mtl_das_pytorch_amd.engine.trainer import Trainer as T2
    res = {}
    for backend in ("engine", "torch"):
        c2 = TrainConfig(model="MTL", synthetic=4, batch_size=32, output_savedir=str(tmp_path / backend),
                         model_path=pths[-1], is_test=True, backend=backend, save_threshold=2.0)
        t2 = T2(c2)
        t2.run()
        res[backend] = t2.last_val["acc"]
    assert abs(res["engine"]["event"] - res["torch"]["event"]) < 0.1, res
    assert abs(res["engine"]["distance"] - res["torch"]["distance"]) < 0.15, res


def test_single_task_engine_trainer(tmp_path):
    from mtl_das_pytorch_amd.engine.trainer import Trainer
    from mtl_das_pytorch_amd.utils.config import TrainConfig
    cfg = TrainConfig(model="single_event", synthetic=4, batch_size=16, epoch_num=2, val_every=2,
                      output_savedir=str(tmp_path), backend="engine")
    tr = Trainer(cfg)
    tr.run()
    assert set(tr.last_val["acc"]) == {"event"}


def test_engine_disk_stream_matches_ram(tmp_path):
    """--dataset_ram False on the engine: batches arrive through the pinned host ring, the copy stream and
    the HBM ring (csrc/matio.cpp reader) and train bitwise like the HBM-resident dataset."""
    from mtl_das_pytorch_amd.data import write_mat_tree
    from mtl_das_pytorch_amd.engine.trainer import Trainer
    from mtl_das_pytorch_amd.utils.config import TrainConfig
    tree = write_mat_tree(str(tmp_path / "das"), n_per_class=5, n_test_per_class=1, seed=5, splits=("train",))
    res = {}
    for ram in (True, False):
        torch.manual_seed(0)
        cfg = TrainConfig(model="MTL", batch_size=8, epoch_num=2, val_every=2, log_every=4,
                          output_savedir=str(tmp_path / str(ram)), save_threshold=2.0, backend="engine",
                          dataset_ram=ram, stream_ring=3, trainVal_set_striking=tree["striking_train"],
                          trainVal_set_excavating=tree["excavating_train"])
        tr = Trainer(cfg)
        tr.run()
        res[ram] = (tr.last_val, tr.backend.prog.flat.params.detach().clone())
    assert res[True][0]["acc"] == res[False][0]["acc"]
    assert torch.equal(res[True][1], res[False][1])
