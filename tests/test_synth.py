"""On-device synthetic generator (csrc/synth.hip) against the torch implementation of the same
physical model (data/synthetic.py) and a NumPy Philox-4x32-10 reference."""
import numpy as np
import pytest
import torch

from mtl_das_pytorch_amd.data.synthetic import generate

M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85


def philox_np(ctr: np.ndarray, key: int) -> np.ndarray:
    """Philox-4x32-10 on uint32 counters [n, 4] (Salmon et al., SC'11), vectorised in NumPy."""
    c = ctr.astype(np.uint64)
    k0, k1 = np.uint64(key & 0xFFFFFFFF), np.uint64(key >> 32)
    mask = np.uint64(0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(M0) * c[:, 0]
        p1 = np.uint64(M1) * c[:, 2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & mask
        hi1, lo1 = p1 >> np.uint64(32), p1 & mask
        c = np.stack([hi1 ^ c[:, 1] ^ k0, lo1, hi0 ^ c[:, 3] ^ k1, lo0], 1)
        k0, k1 = (k0 + np.uint64(W0)) & mask, (k1 + np.uint64(W1)) & mask
    return c.astype(np.uint32)


def test_philox_known_answers():
    """Random123's published Philox-4x32-10 known-answer vectors."""
    ctr = np.array([[0, 0, 0, 0], [0xFFFFFFFF] * 4, [0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344]], np.uint32)
    keys = [0, 0xFFFFFFFFFFFFFFFF, (0x299F31D0 << 32) | 0xA4093822]
    want = [[0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8], [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD],
            [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]]
    for i in range(3):
        assert philox_np(ctr[i:i + 1], keys[i])[0].tolist() == want[i]


@pytest.mark.gpu
def test_philox_device_matches_numpy():
    from mtl_das_pytorch_amd.ops.hip import lib
    rng = np.random.default_rng(0)
    ctr = rng.integers(0, 2 ** 32, size=(1000, 4), dtype=np.uint64).astype(np.uint32)
    key = 0x1234567890ABCDEF
    c = torch.from_numpy(ctr.view(np.int32)).cuda()
    out = torch.empty_like(c)
    lib().philox_kat(c.data_ptr(), key, out.data_ptr(), 1000, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), philox_np(ctr, key))


@pytest.mark.gpu
@pytest.mark.parametrize("in_channels", [1, 3])
def test_hip_generator_clean_signal_matches_torch(in_channels):
    """Same seed -> same labels and per-sample scalars; the clean signal agrees with the torch model to fp32
    rounding (rare isolated points sit on the discontinuity of remainder(tau, period), where a last-bit
    difference of tau picks the other branch)."""
    n = 64
    xh, dh, eh = generate(n, seed=5, device="cuda", in_channels=in_channels, backend="hip", noise=False)
    xt, dt, et = generate(n, seed=5, device="cuda", in_channels=in_channels, backend="torch", noise=False)
    assert torch.equal(dh, dt) and torch.equal(eh, et)
    diff = (xh - xt).abs()
    scale = xt.abs().amax()
    frac_bad = (diff > 1e-3 * scale).float().mean().item()
    assert frac_bad < 1e-4, frac_bad
    assert (diff.median() / scale).item() < 1e-6


@pytest.mark.gpu
def test_hip_generator_noise_statistics_and_determinism():
    """The noise is N(0, sigma_s^2) with sigma_s set by the drawn SNR, reproducible and independent per sample."""
    n = 256
    x1, d, e = generate(n, seed=9, device="cuda")
    x2, _, _ = generate(n, seed=9, device="cuda")
    assert torch.equal(x1, x2)  # deterministic
    x3, _, _ = generate(n, seed=10, device="cuda")
    assert not torch.equal(x1, x3)
    clean, _, _ = generate(n, seed=9, device="cuda", noise=False)
    noise = (x1 - clean) / 100.0
    p_sig = (clean / 100.0).pow(2).mean((1, 2, 3)).clamp_min(1e-12)
    g = torch.Generator().manual_seed(9)  # replay the CPU draws up to the SNR
    torch.randint(0, 16, (n,), generator=g), torch.randint(0, 2, (n,), generator=g)
    torch.rand(n, generator=g), torch.rand(n, generator=g), torch.rand(n, 4, generator=g)
    snr = (torch.rand(n, generator=g) * 14.0 + 6.0).cuda()
    sigma = torch.sqrt(p_sig / 10.0 ** (snr / 10.0))
    z = noise / sigma.view(n, 1, 1, 1)
    assert abs(z.mean().item()) < 5e-3
    assert abs(z.std().item() - 1.0) < 5e-3
    zz = z.flatten().double()
    assert abs((zz ** 4).mean().item() - 3.0) < 0.05  # Gaussian kurtosis
    # neighbouring elements and samples uncorrelated
    assert abs((z[:, :, :, 1:] * z[:, :, :, :-1]).mean().item()) < 5e-3
    assert abs((z[1:] * z[:-1]).mean().item()) < 5e-3


@pytest.mark.gpu
def test_hip_generator_trains_like_torch_data():
    """The engine learns the event task from HIP-generated data as it does from torch-generated data."""
    from mtl_das_pytorch_amd.engine.mtl import MTLProgram
    from mtl_das_pytorch_amd.engine.step import StepRunner
    from mtl_das_pytorch_amd.models import MTL_Net
    torch.manual_seed(0)
    X, d, e = generate(512, seed=3, device="cuda")
    lab = torch.stack([d, e], 1)
    prog = MTLProgram(MTL_Net(), 32, "cuda")
    prog.set_optimizer(weight_decay=0.0)
    run = StepRunner(prog, X, lab)
    run.set_lr(1e-3)
    for ep in range(3):
        for i in range(16):
            run.train_step(torch.arange(32 * i, 32 * (i + 1), device="cuda"))
    Xt, dt, et = generate(256, seed=4, device="cuda")
    run.set_eval_source(Xt, torch.stack([dt, et], 1))
    run.reset_metrics()
    for i in range(8):
        run.eval_step(torch.arange(32 * i, 32 * (i + 1), device="cuda"))
    m = prog.metrics.cpu()
    assert m[-1, 2].item() == 256
    assert m[-1, 1].item() / 256 > 0.8  # held-out event accuracy
