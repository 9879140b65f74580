import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mtl_das_pytorch_amd  # noqa: E402

mtl_das_pytorch_amd.use_engine_graph_queues()  # the GPU suites run the executor setting the entry points use


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm) GPU and the built HIP extension")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU available")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True, scope="session")
def _no_miopen_references():
    """The fp32 PyTorch references (and the torch backend the trainer tests compare against) run on PyTorch's
    native im2col + GEMM convolutions instead of MIOpen: two round-1 full-suite runs on MI355X aborted inside
    MIOpen (an illegal address in a conv backward, an abort in an autograd worker thread) while every
    HIP-engine kernel had completed.  Round 3 re-ran the layer-local suites (Model A and C) with MIOpen
    (MDA_TEST_MIOPEN=1) and the engine's canary guard bands on (MDA_GUARD=1): 8/8 passed, and the session
    check below finds every band intact, so the engine's kernels do not corrupt memory MIOpen later touches.
    The references stay on the native path only so that a MIOpen fault cannot take the round-end GPU suite
    down; MDA_TEST_MIOPEN=1 keeps MIOpen."""
    import torch
    if not torch.cuda.is_available() or os.environ.get("MDA_TEST_MIOPEN") == "1":
        yield
        return
    prev = torch.backends.cudnn.enabled
    torch.backends.cudnn.enabled = False
    yield
    torch.backends.cudnn.enabled = prev


@pytest.fixture(autouse=True)
def _guard_bands_intact():
    """With MDA_GUARD=1 every engine buffer sits between canary bands (engine/guard.py); after each test none
    of them may have been written.  The registry is then cleared: it holds the buffers (strongly) only until
    the end of the test that allocated them, so a full-suite guard run does not accumulate device memory
    (buffers of module-scoped fixtures are checked after the first test that used them)."""
    yield
    from mtl_das_pytorch_amd.engine import guard
    if guard.enabled() and guard.count():
        import torch
        torch.cuda.synchronize()
        bad = guard.check()
        guard.reset()
        assert not bad, bad
