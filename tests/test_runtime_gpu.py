"""Process-lifetime behaviour of the engine's HIP objects (graphs, captured events, streams).

Round 4 (profiles/r4_runtime_faults.txt): one process that trained several Model C programs back to back
died with SIGSEGV inside the HIP runtime when the 6th program started training.  Since then
* the engine's side streams are a fixed, engine-owned set per device (program.EngineStreams), never drawn
  from torch's round-robin stream pool (where a phase's "side" stream could be the capture stream itself);
* the events a graph was captured with live exactly as long as that graph (program.EventKeeper), and a
  graph is only destroyed after the device finished its replays (StepRunner._drop_graph);
* Trainer.run releases its runner (EngineBackend.close) before the next program is built.
This test runs the crashing sequence -- six short Model C trainings with test-set evaluations in one
process -- once."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(600)
def test_six_model_c_programs_in_one_process(tmp_path):
    from mtl_das_pytorch_amd.data.synthetic import generate
    from mtl_das_pytorch_amd.engine.program import EngineStreams
    from mtl_das_pytorch_amd.engine.trainer import Trainer
    from mtl_das_pytorch_amd.models import encode_joint
    from mtl_das_pytorch_amd.utils.config import TrainConfig
    Xt, dt, et = generate(96, seed=77, device="cuda")
    lab = encode_joint(dt, et)
    streams = None
    for i in range(6):
        cfg = TrainConfig(model="multi_classifier", synthetic=3, batch_size=32, epoch_num=2, val_every=2,
                          log_every=4, output_savedir=str(tmp_path / f"c{i}"), save_threshold=2.0,
                          backend="engine", seed=i)
        tr = Trainer(cfg)
        tr.run()
        for sel in (slice(None), slice(0, 64)):  # re-captured eval graphs on other resident sets
            r = tr.evaluate(Xt[sel], lab[sel])
            assert 0.0 <= r["acc"]["event"] <= 1.0
        tr.close()
        assert not tr.backend.runner.graphs and not tr.backend.runner.keepers
        cur = [s.handles for s in EngineStreams._by_device.values()]
        assert streams is None or cur == streams, "engine streams must be one fixed set per device"
        streams = cur
        del tr
    torch.cuda.synchronize()
