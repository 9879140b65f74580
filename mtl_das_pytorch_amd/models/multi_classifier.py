"""Single-level 32-way multi-classifier baseline (reference Model C): Inception-v3, 1-channel stem.

Reference: model/modelC_multiClassifier.py:28-172.  The reference imports the Inception blocks from
torchvision (not available in this image, and not wanted as a dependency); they are re-implemented
here with the *same attribute names* so the 566-key state_dict (``Mixed_5b.branch1x1.conv.weight``,
``...bn.running_var``, ``fc.weight`` ...) is interchangeable with a reference checkpoint.

Joint label: ``label = distance + 16 * event`` (reference dataset_preparation.py:217-224); decoding
is vectorised in :func:`decode_joint` (reference utils.py:600,656-666 does it per sample in Python).
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

JOINT_CLASSES = 32
N_DISTANCE = 16


def encode_joint(distance: torch.Tensor, event: torch.Tensor) -> torch.Tensor:
    return distance + N_DISTANCE * event


def decode_joint(joint: torch.Tensor):
    """joint -> (distance, event) with ``hash_list[i] = [i % 16, i // 16]`` semantics."""
    return joint % N_DISTANCE, torch.div(joint, N_DISTANCE, rounding_mode="floor")


class BasicConv2d(nn.Module):
    """conv (no bias) -> BN(eps=1e-3) -> ReLU  (reference modelC_multiClassifier.py:10-25)."""

    def __init__(self, in_channels: int, out_channels: int, **kwargs):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, bias=False, **kwargs)
        self.bn = nn.BatchNorm2d(out_channels, eps=0.001)

    def forward(self, x):
        return F.relu(self.bn(self.conv(x)), inplace=True)


def _avgpool3(x):
    return F.avg_pool2d(x, kernel_size=3, stride=1, padding=1)


def _maxpool3s2(x):
    return F.max_pool2d(x, kernel_size=3, stride=2)


class InceptionA(nn.Module):
    """35x35-grid block: 1x1 | 1x1-5x5 | 1x1-3x3-3x3 | avgpool-1x1  -> 224 + pool_features ch."""

    def __init__(self, in_channels: int, pool_features: int, conv_block: Optional[Callable] = None):
        super().__init__()
        cb = conv_block or BasicConv2d
        self.branch1x1 = cb(in_channels, 64, kernel_size=1)
        self.branch5x5_1 = cb(in_channels, 48, kernel_size=1)
        self.branch5x5_2 = cb(48, 64, kernel_size=5, padding=2)
        self.branch3x3dbl_1 = cb(in_channels, 64, kernel_size=1)
        self.branch3x3dbl_2 = cb(64, 96, kernel_size=3, padding=1)
        self.branch3x3dbl_3 = cb(96, 96, kernel_size=3, padding=1)
        self.branch_pool = cb(in_channels, pool_features, kernel_size=1)

    def branches(self, x):
        b1 = self.branch1x1(x)
        b5 = self.branch5x5_2(self.branch5x5_1(x))
        b3 = self.branch3x3dbl_3(self.branch3x3dbl_2(self.branch3x3dbl_1(x)))
        bp = self.branch_pool(_avgpool3(x))
        return [b1, b5, b3, bp]

    def forward(self, x):
        return torch.cat(self.branches(x), 1)


class InceptionB(nn.Module):
    """Grid reduction 35->17: 3x3/s2 | 1x1-3x3-3x3/s2 | maxpool/s2  -> 480 + in ch."""

    def __init__(self, in_channels: int, conv_block: Optional[Callable] = None):
        super().__init__()
        cb = conv_block or BasicConv2d
        self.branch3x3 = cb(in_channels, 384, kernel_size=3, stride=2)
        self.branch3x3dbl_1 = cb(in_channels, 64, kernel_size=1)
        self.branch3x3dbl_2 = cb(64, 96, kernel_size=3, padding=1)
        self.branch3x3dbl_3 = cb(96, 96, kernel_size=3, stride=2)

    def branches(self, x):
        b3 = self.branch3x3(x)
        bd = self.branch3x3dbl_3(self.branch3x3dbl_2(self.branch3x3dbl_1(x)))
        return [b3, bd, _maxpool3s2(x)]

    def forward(self, x):
        return torch.cat(self.branches(x), 1)


class InceptionC(nn.Module):
    """17x17-grid block with factorised 7x7 convolutions -> 768 ch."""

    def __init__(self, in_channels: int, channels_7x7: int, conv_block: Optional[Callable] = None):
        super().__init__()
        cb = conv_block or BasicConv2d
        c7 = channels_7x7
        self.branch1x1 = cb(in_channels, 192, kernel_size=1)
        self.branch7x7_1 = cb(in_channels, c7, kernel_size=1)
        self.branch7x7_2 = cb(c7, c7, kernel_size=(1, 7), padding=(0, 3))
        self.branch7x7_3 = cb(c7, 192, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7dbl_1 = cb(in_channels, c7, kernel_size=1)
        self.branch7x7dbl_2 = cb(c7, c7, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7dbl_3 = cb(c7, c7, kernel_size=(1, 7), padding=(0, 3))
        self.branch7x7dbl_4 = cb(c7, c7, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7dbl_5 = cb(c7, 192, kernel_size=(1, 7), padding=(0, 3))
        self.branch_pool = cb(in_channels, 192, kernel_size=1)

    def branches(self, x):
        b1 = self.branch1x1(x)
        b7 = self.branch7x7_3(self.branch7x7_2(self.branch7x7_1(x)))
        bd = x
        for i in range(1, 6):
            bd = getattr(self, f"branch7x7dbl_{i}")(bd)
        bp = self.branch_pool(_avgpool3(x))
        return [b1, b7, bd, bp]

    def forward(self, x):
        return torch.cat(self.branches(x), 1)


class InceptionD(nn.Module):
    """Grid reduction 17->8: 1x1-3x3/s2 | 1x1-1x7-7x1-3x3/s2 | maxpool/s2  -> 512 + in ch."""

    def __init__(self, in_channels: int, conv_block: Optional[Callable] = None):
        super().__init__()
        cb = conv_block or BasicConv2d
        self.branch3x3_1 = cb(in_channels, 192, kernel_size=1)
        self.branch3x3_2 = cb(192, 320, kernel_size=3, stride=2)
        self.branch7x7x3_1 = cb(in_channels, 192, kernel_size=1)
        self.branch7x7x3_2 = cb(192, 192, kernel_size=(1, 7), padding=(0, 3))
        self.branch7x7x3_3 = cb(192, 192, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7x3_4 = cb(192, 192, kernel_size=3, stride=2)

    def branches(self, x):
        b3 = self.branch3x3_2(self.branch3x3_1(x))
        b7 = x
        for i in range(1, 5):
            b7 = getattr(self, f"branch7x7x3_{i}")(b7)
        return [b3, b7, _maxpool3s2(x)]

    def forward(self, x):
        return torch.cat(self.branches(x), 1)


class InceptionE(nn.Module):
    """8x8-grid block with split 1x3 / 3x1 outputs -> 2048 ch."""

    def __init__(self, in_channels: int, conv_block: Optional[Callable] = None):
        super().__init__()
        cb = conv_block or BasicConv2d
        self.branch1x1 = cb(in_channels, 320, kernel_size=1)
        self.branch3x3_1 = cb(in_channels, 384, kernel_size=1)
        self.branch3x3_2a = cb(384, 384, kernel_size=(1, 3), padding=(0, 1))
        self.branch3x3_2b = cb(384, 384, kernel_size=(3, 1), padding=(1, 0))
        self.branch3x3dbl_1 = cb(in_channels, 448, kernel_size=1)
        self.branch3x3dbl_2 = cb(448, 384, kernel_size=3, padding=1)
        self.branch3x3dbl_3a = cb(384, 384, kernel_size=(1, 3), padding=(0, 1))
        self.branch3x3dbl_3b = cb(384, 384, kernel_size=(3, 1), padding=(1, 0))
        self.branch_pool = cb(in_channels, 192, kernel_size=1)

    def branches(self, x):
        b1 = self.branch1x1(x)
        s = self.branch3x3_1(x)
        b3 = [self.branch3x3_2a(s), self.branch3x3_2b(s)]
        d = self.branch3x3dbl_2(self.branch3x3dbl_1(x))
        bd = [self.branch3x3dbl_3a(d), self.branch3x3dbl_3b(d)]
        bp = self.branch_pool(_avgpool3(x))
        return [b1] + b3 + bd + [bp]

    def forward(self, x):
        return torch.cat(self.branches(x), 1)


class InceptionAux(nn.Module):
    """Auxiliary classifier (only built when ``aux_logits=True``; off in the reference)."""

    def __init__(self, in_channels: int, num_classes: int, conv_block: Optional[Callable] = None):
        super().__init__()
        cb = conv_block or BasicConv2d
        self.conv0 = cb(in_channels, 128, kernel_size=1)
        self.conv1 = cb(128, 768, kernel_size=5)
        self.conv1.stddev = 0.01
        self.fc = nn.Linear(768, num_classes)
        self.fc.stddev = 0.001

    def forward(self, x):
        x = F.avg_pool2d(x, kernel_size=5, stride=3)
        x = self.conv1(self.conv0(x))
        x = F.adaptive_avg_pool2d(x, (1, 1))
        return self.fc(torch.flatten(x, 1))


class Multi_Classifier(nn.Module):
    """Inception-v3 with a ``in_channels``-channel stem and ``num_classes`` joint classes."""

    def __init__(self, num_classes: int = JOINT_CLASSES, aux_logits: bool = False, transform_input: bool = False,
                 inception_blocks=None, init_weights: bool = True, in_channels: int = 1):
        super().__init__()
        blocks = inception_blocks or [BasicConv2d, InceptionA, InceptionB, InceptionC, InceptionD, InceptionE,
                                      InceptionAux]
        assert len(blocks) == 7
        conv_block, inc_a, inc_b, inc_c, inc_d, inc_e, inc_aux = blocks
        self.aux_logits = aux_logits
        self.transform_input = transform_input
        self.num_classes = num_classes
        self.Conv2d_1a_3x3 = conv_block(in_channels, 32, kernel_size=3, stride=2)
        self.Conv2d_2a_3x3 = conv_block(32, 32, kernel_size=3)
        self.Conv2d_2b_3x3 = conv_block(32, 64, kernel_size=3, padding=1)
        self.maxpool1 = nn.MaxPool2d(kernel_size=3, stride=2)
        self.Conv2d_3b_1x1 = conv_block(64, 80, kernel_size=1)
        self.Conv2d_4a_3x3 = conv_block(80, 192, kernel_size=3)
        self.maxpool2 = nn.MaxPool2d(kernel_size=3, stride=2)
        self.Mixed_5b = inc_a(192, pool_features=32)
        self.Mixed_5c = inc_a(256, pool_features=64)
        self.Mixed_5d = inc_a(288, pool_features=64)
        self.Mixed_6a = inc_b(288)
        self.Mixed_6b = inc_c(768, channels_7x7=128)
        self.Mixed_6c = inc_c(768, channels_7x7=160)
        self.Mixed_6d = inc_c(768, channels_7x7=160)
        self.Mixed_6e = inc_c(768, channels_7x7=192)
        self.AuxLogits = inc_aux(768, num_classes) if aux_logits else None
        self.Mixed_7a = inc_d(768)
        self.Mixed_7b = inc_e(1280)
        self.Mixed_7c = inc_e(2048)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.dropout = nn.Dropout()
        self.fc = nn.Linear(2048, num_classes)
        if init_weights:
            self.reset_parameters()

    def reset_parameters(self):
        """Truncated-normal(+-2 sigma) weights.  As in the reference (modelC_multiClassifier.py:88-100)
        ``stddev`` is looked up on the raw Conv2d/Linear module, so every conv gets 0.1 (torchvision sets
        it on the BasicConv2d wrapper) while the aux ``fc`` keeps its 0.001."""
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.Linear)):
                std = float(getattr(m, "stddev", 0.1))
                with torch.no_grad():
                    nn.init.trunc_normal_(m.weight, mean=0.0, std=std, a=-2 * std, b=2 * std)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    @property
    def stem(self):
        return [self.Conv2d_1a_3x3, self.Conv2d_2a_3x3, self.Conv2d_2b_3x3, self.maxpool1, self.Conv2d_3b_1x1,
                self.Conv2d_4a_3x3, self.maxpool2]

    @property
    def mixed(self):
        return [self.Mixed_5b, self.Mixed_5c, self.Mixed_5d, self.Mixed_6a, self.Mixed_6b, self.Mixed_6c,
                self.Mixed_6d, self.Mixed_6e, self.Mixed_7a, self.Mixed_7b, self.Mixed_7c]

    def forward(self, x):
        for m in self.stem:
            x = m(x)
        aux = None
        for name in ("Mixed_5b", "Mixed_5c", "Mixed_5d", "Mixed_6a", "Mixed_6b", "Mixed_6c", "Mixed_6d",
                     "Mixed_6e"):
            x = getattr(self, name)(x)
        if self.AuxLogits is not None and self.training:
            aux = self.AuxLogits(x)
        for name in ("Mixed_7a", "Mixed_7b", "Mixed_7c"):
            x = getattr(self, name)(x)
        x = torch.flatten(self.dropout(self.avgpool(x)), 1)
        x = self.fc(x)
        if self.training and self.aux_logits:
            return x, aux
        return x
