"""Building blocks shared by the MTL / single-task networks (reference Models A and B).

Parity notes (reference = sunmin123456/MTL-DAS.PyTorch):
  * residual block  -> model/modelA_MTL.py:7-32   (conv3x3-BN-ReLU-conv3x3-BN + shortcut, ReLU)
  * conv3x3 helper  -> model/modelA_MTL.py:35-39  (bias=False)
  * attention mask  -> model/modelA_MTL.py:42-50  (1x1 conv(+bias)-BN-ReLU-3x3 conv(+bias)-BN-Sigmoid)

The module *attribute names and Sequential indices* are part of the checkpoint key space
(``resblockN.left.{0,1,3,4}``, ``resblockN.shortcut.{0,1}``, ``att_mask_generator1.{t}.{0,1,3,4}``),
so every container here is laid out to reproduce those keys exactly.  The forward functions are the
plain-PyTorch (NCHW, fp32) definition of the math; they are used on CPU and as the numerical oracle
for the MI355X engine (``mtl_das_pytorch_amd.engine``), which lowers the same parameters onto the
HIP kernels in ``csrc/``.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


def conv3x3(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    """3x3, pad 1, no bias (reference ``conv3x3``)."""
    return nn.Conv2d(cin, cout, kernel_size=(3, 3), stride=(stride, stride), padding=(1, 1), bias=False)


class ResBlock(nn.Module):
    """Pre-activation-free residual block: ``relu(BN(conv(relu(BN(conv(x))))) + shortcut(x))``.

    ``left`` is a Sequential whose indices 0,1,3,4 carry parameters (2 is the in-place ReLU) so that
    the state_dict keys match ``resblockN.left.{0,1,3,4}.*``.  The projection shortcut exists only
    when the stride or channel count changes (reference modelA_MTL.py:21-26).
    """

    def __init__(self, inchannel: int, outchannel: int, stride: int = 1):
        super().__init__()
        self.left = nn.Sequential(
            conv3x3(inchannel, outchannel, stride),
            nn.BatchNorm2d(outchannel),
            nn.ReLU(inplace=True),
            conv3x3(outchannel, outchannel, 1),
            nn.BatchNorm2d(outchannel),
        )
        self.shortcut = nn.Sequential()
        if stride != 1 or inchannel != outchannel:
            self.shortcut = nn.Sequential(
                nn.Conv2d(inchannel, outchannel, kernel_size=(1, 1), stride=(stride, stride), bias=False),
                nn.BatchNorm2d(outchannel),
            )

    @property
    def has_projection(self) -> bool:
        return len(self.shortcut) > 0

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return F.relu(self.left(x) + self.shortcut(x))


def att_generator(cin: int, cmid: int, cout: int) -> nn.Sequential:
    """Sigmoid spatial/channel attention mask generator (1x1 reduce, 3x3 expand, both with bias)."""
    return nn.Sequential(
        nn.Conv2d(cin, cmid, kernel_size=(1, 1)),
        nn.BatchNorm2d(cmid),
        nn.ReLU(inplace=True),
        nn.Conv2d(cmid, cout, kernel_size=(3, 3), padding=(1, 1)),
        nn.BatchNorm2d(cout),
        nn.Sigmoid(),
    )


def encoder_block(cin: int, cout: int) -> nn.Sequential:
    """Task-branch "output layer": conv3x3 -> BN -> ReLU (reference modelA_MTL.py:101-113)."""
    return nn.Sequential(conv3x3(cin, cout), nn.BatchNorm2d(cout), nn.ReLU(inplace=True))
