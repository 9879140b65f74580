"""Two-level multi-task network (reference Model A) and its single-task variant (Model B).

Reference: model/modelA_MTL.py:53-174 (``MTL_Net``) and model/modelB_singleTask.py:53-178
(``Single_Task_Net``).  Both are the same architecture parametrised by the list of tasks:

  shared backbone   conv7x7/s3 -> BN -> ReLU -> 8 residual blocks (channels 16,16,32,32,64,64,128,128)
  per task, level k (k=1..4):
      mask_k  = att_gen_k( F_{2k-1}            )   if k == 1
              = att_gen_k( cat[F_{2k-1}, B_{k-1}] )  otherwise (shared feature first)
      A_k     = mask_k * F_{2k}
      B_k     = maxpool2x2_ceil( relu(BN(conv3x3(A_k))) )     for k = 1..3
  head      GAP(A_4) -> mean over groups of 128/n_classes channels -> log_softmax
            (``head="fc"``: GAP(A_4) -> Linear(128, n_classes) -> log_softmax -- NOT in the reference: the
            backbone-vs-head ablation of docs/ACCURACY.md, trained on the plain-PyTorch backend only)

``MTLNet`` is generic in the task list; ``MTL_Net()`` and ``Single_Task_Net(task)`` are thin
constructors that reproduce the reference class names, default arguments and the *exact*
state_dict key space (including the misspelt ``att_mask_generato2`` ModuleList).
"""
from __future__ import annotations

from typing import Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from .layers import ResBlock, att_generator, encoder_block

#: number of classes of every task the framework knows about (reference modelA_MTL.py:68-69)
TASK_CLASSES = {"distance": 16, "event": 2}


class MTLNet(nn.Module):
    """Shared residual backbone + one attention branch per task.

    Args:
        tasks: task names, subset/ordering of :data:`TASK_CLASSES` keys.
        in_channels: input channels (reference: 1; ``--in_channels 2`` changes conv1's weight shape).
        first_ch: channels of the first stage (reference: 16; doubles every two residual blocks).
        head: ``"group_mean"`` (the reference's parameter-free head) or ``"fc"`` (ablation: a learned linear
            layer per task on the pooled features, as Model C's classifier; adds ``task{1,2}fc`` keys).
    """

    HEADS = ("group_mean", "fc")

    def __init__(self, tasks: Sequence[str] = ("distance", "event"), in_channels: int = 1, first_ch: int = 16,
                 num_classes: Sequence[int] | None = None, head: str = "group_mean"):
        super().__init__()
        if head not in self.HEADS:
            raise ValueError(f"unknown head {head!r}; expected one of {self.HEADS}")
        self.head = head
        self.tasks = list(tasks)
        for t in self.tasks:
            if t not in TASK_CLASSES and num_classes is None:
                raise ValueError(f"unknown task {t!r}")
        self.task_cate_num = list(num_classes) if num_classes is not None else [TASK_CLASSES[t] for t in self.tasks]
        self.in_channels = in_channels
        self.res_num = 8
        self.first_ch = first_ch
        # channel schedule [16, 16, 32, 64, 128]
        self.ch = [first_ch, first_ch] + [first_ch * 2 ** (i + 1) for i in range(self.res_num // 2 - 1)]
        ch = self.ch
        T = len(self.tasks)

        self.conv1 = nn.Sequential(
            nn.Conv2d(in_channels, ch[0], kernel_size=(7, 7), stride=(3, 3), padding=(2, 2), bias=False),
            nn.BatchNorm2d(ch[0]),
            nn.ReLU(),
        )
        # (in, out, stride) for resblock1..8
        plan = [(ch[0], ch[1], 1), (ch[1], ch[1], 1)]
        for s in range(2, 5):
            plan += [(ch[s - 1], ch[s], 2), (ch[s], ch[s], 1)]
        for i, (cin, cout, stride) in enumerate(plan, start=1):
            setattr(self, f"resblock{i}", ResBlock(cin, cout, stride))

        # attention mask generators; attribute name of level 2 is misspelt in the reference
        self.att_mask_generator1 = nn.ModuleList([att_generator(ch[1], ch[1] // 2, ch[1]) for _ in range(T)])
        self.att_mask_generato2 = nn.ModuleList([att_generator(2 * ch[2], ch[2] // 2, ch[2]) for _ in range(T)])
        self.att_mask_generator3 = nn.ModuleList([att_generator(2 * ch[3], ch[3] // 2, ch[3]) for _ in range(T)])
        self.att_mask_generator4 = nn.ModuleList([att_generator(2 * ch[4], ch[4] // 2, ch[4]) for _ in range(T)])
        self.output_layer1 = nn.ModuleList([encoder_block(ch[1], ch[2]) for _ in range(T)])
        self.output_layer2 = nn.ModuleList([encoder_block(ch[2], ch[3]) for _ in range(T)])
        self.output_layer3 = nn.ModuleList([encoder_block(ch[3], ch[4]) for _ in range(T)])
        self.down_sampling = nn.MaxPool2d(kernel_size=2, stride=2, ceil_mode=True)

        # parameter-free heads (kept as modules so FLOP counting sees them, like the reference)
        for t, ncls in zip(self.tasks, self.task_cate_num):
            if ch[-1] % ncls:
                raise ValueError(f"{ch[-1]} channels are not divisible into {ncls} classes")
            idx = 1 if t == "distance" else 2
            setattr(self, f"task{idx}pool", nn.AdaptiveAvgPool2d((1, 1)))
            setattr(self, f"task{idx}pool1d", nn.AvgPool1d(kernel_size=ch[-1] // ncls, stride=ch[-1] // ncls))
            if head == "fc":
                setattr(self, f"task{idx}fc", nn.Linear(ch[-1], ncls))

    # ---- structure accessors used by the engine -------------------------------------------------
    @property
    def resblocks(self):
        return [getattr(self, f"resblock{i}") for i in range(1, self.res_num + 1)]

    @property
    def att_generators(self):
        return [self.att_mask_generator1, self.att_mask_generato2, self.att_mask_generator3, self.att_mask_generator4]

    @property
    def output_layers(self):
        return [self.output_layer1, self.output_layer2, self.output_layer3]

    def head_modules(self, t: int):
        idx = 1 if self.tasks[t] == "distance" else 2
        return getattr(self, f"task{idx}pool"), getattr(self, f"task{idx}pool1d")

    # ---- reference-math forward (NCHW, any dtype) ------------------------------------------------
    def features(self, x: torch.Tensor):
        x = self.conv1(x)
        shared = []
        for rb in self.resblocks:
            x = rb(x)
            shared.append(x)
        return shared

    def forward(self, x: torch.Tensor):
        shared = self.features(x)
        outs = []
        for t in range(len(self.tasks)):
            prev = None
            for lvl in range(4):
                gen = self.att_generators[lvl][t]
                src = shared[2 * lvl] if prev is None else torch.cat((shared[2 * lvl], prev), dim=1)
                a = gen(src) * shared[2 * lvl + 1]
                if lvl < 3:
                    prev = self.down_sampling(self.output_layers[lvl][t](a))
                else:
                    prev = a
            gap, grp = self.head_modules(t)
            if self.head == "fc":
                logits = getattr(self, f"task{1 if self.tasks[t] == 'distance' else 2}fc")(gap(prev).flatten(1))
            else:
                logits = grp(gap(prev).flatten(1).unsqueeze(1)).squeeze(1)
            outs.append(F.log_softmax(logits, dim=1))
        return tuple(outs) if len(outs) > 1 else outs[0]


class MTL_Net(MTLNet):
    """Reference-compatible constructor: ``MTL_Net()`` (Model A, tasks distance+event)."""

    def __init__(self, in_channels: int = 1, head: str = "group_mean"):
        super().__init__(tasks=("distance", "event"), in_channels=in_channels, head=head)


class Single_Task_Net(MTLNet):
    """Reference-compatible constructor: ``Single_Task_Net(task)`` (Model B)."""

    def __init__(self, task: str = "distance", in_channels: int = 1, head: str = "group_mean"):
        if task not in ("distance", "event"):
            raise ValueError(task)
        super().__init__(tasks=(task,), in_channels=in_channels, head=head)
