"""Synthetic DAS time-space matrices with (radial distance, event type) labels.

There is no network access to the reference's field dataset (README.md:36), so every entry point can
run on synthetic data of the paper's shape: ``C x 100 x 250`` (C = 1 by default, ``in_channels``
configurable), 16 radial-distance classes (0..15 m, 1 m bins) and 2 event types (striking=0,
excavating=1).

Physical toy model (per sample; torch ops on the CPU, one HIP kernel -- csrc/synth.hip -- on the GPU):
  * a source at radial distance ``d`` metres from the fibre and along-fibre position ``x0`` emits a
    wavelet that reaches fibre point ``x`` at ``t0 + sqrt(d^2 + (x-x0)^2) / v`` (hyperbolic moveout);
  * amplitude decays as ``1 / (1 + d/4)``, the spatial footprint widens with ``d``;
  * striking = repeated short broadband impacts; excavating = longer, lower-frequency periodic bursts;
  * additive white noise at a random SNR.
Distance is therefore encoded in curvature/width/amplitude and event type in the temporal signature,
which makes both tasks learnable but not trivial.

``write_mat_tree`` materialises the reference's directory layout
``<root>/{striking,excavating}_{train,test}/<N>m/<i>.mat`` (key ``'data'``) so the reference-style
``DataCollector``/``Dataset_mat_MTL`` path is exercised end to end.  ``DeviceDataset`` keeps a whole
split resident in HBM and hands out batches by on-device index gather (no host collate, no pageable
H2D copies in the training loop).
"""
from __future__ import annotations

import math
import os
from typing import Optional, Tuple

import numpy as np
import torch

H, W = 100, 250
N_DIST, N_EVENT = 16, 2


def generate(n: int, seed: int = 0, device="cpu", in_channels: int = 1, height: int = H, width: int = W,
             distance: Optional[torch.Tensor] = None, event: Optional[torch.Tensor] = None,
             snr_db: Tuple[float, float] = (6.0, 20.0), dtype=torch.float32, backend: Optional[str] = None,
             noise: bool = True):
    """Return ``(x [n,C,H,W], distance [n], event [n])``; labels drawn uniformly unless given.

    ``backend``: "hip" evaluates the model in one HIP kernel (``csrc/synth.hip``, Philox noise; the default on
    a GPU), "torch" with torch ops (the default on the CPU).  Both draw the per-sample scalars from the same
    CPU generator, so their clean signals agree to fp32 rounding; the noise streams differ.  ``noise=False``
    returns the clean signal (x 100)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    if distance is None:
        distance = torch.randint(0, N_DIST, (n,), generator=g)
    if event is None:
        event = torch.randint(0, N_EVENT, (n,), generator=g)
    distance = distance.to("cpu").long()
    event = event.to("cpu").long()
    # per-sample random scalars drawn on CPU for determinism independent of the device
    x0 = torch.rand(n, generator=g) * 0.5 + 0.25                 # along-fibre position (fraction)
    t0 = torch.rand(n, generator=g) * 0.35 + 0.1                 # onset time (fraction)
    jitter = torch.rand(n, 4, generator=g)
    snr = torch.rand(n, generator=g) * (snr_db[1] - snr_db[0]) + snr_db[0]
    noise_seed = int(torch.randint(0, 2 ** 31 - 1, (1,), generator=g))

    dev = torch.device(device)
    if backend is None:
        backend = os.environ.get("MDA_SYNTH_BACKEND") or ("hip" if dev.type == "cuda" else "torch")
    if backend == "hip":
        return _generate_hip(n, dev, distance, event, x0, t0, jitter, snr, noise_seed, in_channels, height, width,
                             noise, dtype)
    if backend != "torch":
        raise ValueError(f"unknown backend {backend!r}")
    d = distance.to(dev, torch.float32)
    ev = event.to(dev, torch.float32)
    x0, t0, jitter, snr = x0.to(dev), t0.to(dev), jitter.to(dev), snr.to(dev)
    xs = torch.linspace(0, 1, height, device=dev).view(1, height, 1)     # fibre axis
    ts = torch.linspace(0, 1, width, device=dev).view(1, 1, width)       # time axis
    dist_m = (d + 0.5).view(n, 1, 1)
    # hyperbolic moveout: fibre span 100 points ~ 20 m; slowness chosen so curvature spans the window
    dx = (xs - x0.view(n, 1, 1)) * 20.0
    arrival = t0.view(n, 1, 1) + torch.sqrt(dist_m ** 2 + dx ** 2) / 110.0
    tau = ts - arrival                                                   # [n, H, W]
    footprint = torch.exp(-(dx ** 2) / (2.0 * (1.5 + 0.6 * dist_m) ** 2))
    amp = 1.0 / (1.0 + dist_m / 4.0)
    # event signatures
    f_strike = 38.0 + 6.0 * jitter[:, 0].view(n, 1, 1)
    period = 0.16 + 0.04 * jitter[:, 1].view(n, 1, 1)
    phase = torch.remainder(tau, period)
    strike = torch.exp(-phase / 0.012) * torch.cos(2 * math.pi * f_strike * phase) * (tau > 0)
    f_dig = 9.0 + 3.0 * jitter[:, 2].view(n, 1, 1)
    burst = torch.exp(-((tau - 0.18) ** 2) / (2 * 0.09 ** 2))
    dig = burst * torch.sin(2 * math.pi * f_dig * tau + 6.28 * jitter[:, 3].view(n, 1, 1))
    e = ev.view(n, 1, 1)
    clean = amp * footprint * ((1 - e) * strike + e * dig)               # [n, H, W]
    p_sig = clean.pow(2).mean(dim=(1, 2), keepdim=True).clamp_min(1e-12)
    sigma = torch.sqrt(p_sig / (10.0 ** (snr.view(n, 1, 1) / 10.0))) * float(noise)
    gn = torch.Generator(device=dev).manual_seed(noise_seed)
    chans = []
    for c in range(in_channels):
        noise = torch.randn(n, height, width, generator=gn, device=dev)
        sig = clean if c == 0 else torch.roll(clean, shifts=c, dims=2)   # extra channels: shifted copies
        chans.append(sig + sigma * noise)
    x = torch.stack(chans, dim=1) * 100.0                               # field units ~ O(1..10)
    return x.to(dtype), distance.to(dev), event.to(dev)


def _generate_hip(n, dev, distance, event, x0, t0, jitter, snr, noise_seed, in_channels, height, width, noise,
                  dtype):
    """One ``synth_das`` launch: block s evaluates sample s (csrc/synth.hip)."""
    from ..ops.hip import lib
    params = torch.cat([distance.float().view(n, 1), event.float().view(n, 1), x0.view(n, 1), t0.view(n, 1),
                        jitter.view(n, 4), snr.view(n, 1)], 1).contiguous().to(dev)
    x = torch.empty(n, in_channels, height, width, device=dev, dtype=torch.float32)
    with torch.cuda.device(dev):
        lib().synth_das(torch.cuda.current_stream(dev).cuda_stream,
                        {"params": params.data_ptr(), "out": x.data_ptr(), "n": n, "C": in_channels, "H": height,
                         "W": width, "noise": int(noise), "key": noise_seed, "sample0": 0})
    return x.to(dtype), distance.to(dev), event.to(dev)


def write_mat_tree(root: str, n_per_class: int = 8, n_test_per_class: int = 2, seed: int = 0,
                   in_channels: int = 1, splits=("train", "test")) -> dict:
    """Write ``<root>/{striking,excavating}_{train,test}/<N>m/<i>.mat`` and return the four paths."""
    import scipy.io as sio
    out = {}
    s = seed
    for split in splits:
        per = n_per_class if split == "train" else n_test_per_class
        for ev_id, ev_name in enumerate(("striking", "excavating")):
            base = os.path.join(root, f"{ev_name}_{split}")
            out[f"{ev_name}_{split}"] = base
            for dcls in range(N_DIST):
                cat = os.path.join(base, f"{dcls}m")
                os.makedirs(cat, exist_ok=True)
                x, _, _ = generate(per, seed=s, in_channels=in_channels,
                                   distance=torch.full((per,), dcls), event=torch.full((per,), ev_id))
                s += 1
                arr = x.numpy().astype(np.float64)
                for i in range(per):
                    data = arr[i, 0] if in_channels == 1 else arr[i]
                    sio.savemat(os.path.join(cat, f"{i}.mat"), {"data": data})
    return out


class DeviceDataset:
    """A whole split resident on one device: ``x`` ``[N,C,H,W]`` plus label tensors.

    ``labels`` is ``[N]`` (joint) or ``[N,2]`` (distance, event).  ``batches()`` yields index tensors
    drawn on-device (shuffled with a seeded generator); the engine gathers+casts the batch with one
    HIP kernel.
    """

    def __init__(self, x: torch.Tensor, labels: torch.Tensor):
        self.x = x
        self.labels = labels
        self.n = x.shape[0]

    def __len__(self):
        return self.n

    @classmethod
    def from_arrays(cls, x: np.ndarray, labels: np.ndarray, device):
        return cls(torch.as_tensor(x, dtype=torch.float32).to(device), torch.as_tensor(labels).to(device).long())

    @classmethod
    def synthetic(cls, n: int, device, seed: int = 0, in_channels: int = 1, joint: bool = False):
        x, d, e = generate(n, seed=seed, device=device, in_channels=in_channels)
        lab = (d + N_DIST * e) if joint else torch.stack([d, e], dim=1)
        return cls(x, lab.to(device))

    def batch_indices(self, batch_size: int, shuffle: bool, generator: Optional[torch.Generator] = None,
                      drop_last: bool = False):
        dev = self.x.device
        order = torch.randperm(self.n, device=dev, generator=generator) if shuffle else torch.arange(self.n, device=dev)
        stop = self.n - (self.n % batch_size) if drop_last else self.n
        return [order[i:i + batch_size] for i in range(0, stop, batch_size)]
