"""ResNet-50 on synthetic ImageNet (BASELINE.json config 5: "ResNet-50
synthetic-ImageNet RayAccelerator num_workers=8 bf16 -- large-grad-bucket xGMI
allreduce stress").  Not part of the reference tree (SURVEY.md §2.8 last row);
torchvision is not available in this image, so the architecture is defined
here (He et al. 2015, v1.5: stride on the 3x3 conv of each bottleneck).

MI355X choices:
  * channels_last activations + bf16 autocast: MIOpen's NHWC bf16 convolutions
    run on the MFMA units; BatchNorm statistics stay fp32;
  * parameters live in a flat fp32 arena (25,557,032 params = 97.5 MiB), the
    SGD-momentum step is ONE fused HIP launch over it, and DDP buckets are
    arena slices allreduced in place (no flatten/unflatten copies);
  * zero-init of the last BN gamma in each residual branch (standard large-batch
    recipe) is optional (``zero_init_residual``).
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.nn.functional as F
from torch import nn
from torch.utils.data import Dataset

from ..lightning import LightningModule
from ..ops.bn import BatchNormAct2d
from ..ops.conv import BNStats, Conv1x1NHWC, GradFork
from ..ops.pool import MaxPool2dNHWC, global_avg_pool_nhwc
from ..ops.shadow import ConvBF16


def _conv3x3(cin: int, cout: int, stride: int = 1, fused: bool = False) -> nn.Conv2d:
    # fused: reads the arena's bf16 weight shadow under autocast (ops/shadow.py)
    return (ConvBF16 if fused else nn.Conv2d)(cin, cout, 3, stride, 1, bias=False)


def _conv1x1(cin: int, cout: int, stride: int = 1, fused: bool = False) -> nn.Conv2d:
    # fused: stride-1 1x1 convs pick MIOpen or a GEMM per operation (ops/conv.py);
    # same parameter / state-dict key as nn.Conv2d either way
    if fused and stride == 1:
        return Conv1x1NHWC(cin, cout)
    return (ConvBF16 if fused else nn.Conv2d)(cin, cout, 1, stride, bias=False)


def _bn(c: int, fused: bool, act: Optional[str] = "relu") -> nn.BatchNorm2d:
    # fused: BatchNorm + ReLU (+ residual add) in the gfx950 kernels of csrc/bn_act.hip;
    # same parameters / buffers / state-dict keys as nn.BatchNorm2d either way
    return BatchNormAct2d(c, act=act) if fused else nn.BatchNorm2d(c)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, width: int, stride: int = 1, downsample: Optional[nn.Module] = None,
                 fused_bn: bool = False):
        super().__init__()
        cout = width * self.expansion
        self.fused_bn = fused_bn
        self.conv1 = _conv1x1(cin, width, fused=fused_bn)
        self.bn1 = _bn(width, fused_bn)
        self.conv2 = _conv3x3(width, width, stride, fused=fused_bn)
        self.bn2 = _bn(width, fused_bn)
        self.conv3 = _conv1x1(width, cout, fused=fused_bn)
        self.bn3 = _bn(cout, fused_bn)  # fused: relu(bn3(x) + identity) in one pass
        self.downsample = downsample
        if fused_bn and downsample is None and isinstance(self.conv1, Conv1x1NHWC):
            # identity block: x (the previous bn3's output) reaches autograd only through
            # conv1 -- the shortcut's gradient is folded into bn3 -- so conv1's input
            # gradient may compute the previous bn3's backward partial (ops/conv.py)
            self.conv1.fuse_bn_dgrad = True

    @staticmethod
    def _conv_bn(conv, bn, x, **kw):
        """bn(conv(x)): a stride-1 1x1 or 3x3 conv may compute bn's batch statistics in
        its epilogue (ops.conv.BNStats; bn then skips its partial pass over the output)."""
        fork = kw.pop("fork", None)
        if isinstance(conv, (Conv1x1NHWC, ConvBF16)) and bn.training:
            st = BNStats()
            return bn(conv(x, fork=fork, bn_stats=st), bn_stats=st, **kw)
        return bn(conv(x, fork=fork) if fork is not None else conv(x), **kw)

    def forward(self, x):
        # bn2's output feeds conv3 only, bn1's conv2 only: the conv may apply the
        # BatchNorm + ReLU to its own operands (ops/bn.py DeferredApply), so that
        # activation is never written (bn1: stride-1 conv2, where the 3x3 kernel runs)
        defer = isinstance(self.conv3, Conv1x1NHWC)
        defer1 = isinstance(self.conv2, ConvBF16) and tuple(self.conv2.stride) == (1, 1)
        if self.fused_bn and self.downsample is not None:
            # conv1 and the downsample conv both read x: their input gradients meet in
            # one tensor (ops.conv.GradFork) instead of an autograd add of two
            fork = GradFork()
            idt = self._conv_bn(self.downsample[0], self.downsample[1], x, fork=fork)
            out = self._conv_bn(self.conv2, self.bn2, self._conv_bn(self.conv1, self.bn1, x, fork=fork, defer=defer1),
                                defer=defer)
            return self._conv_bn(self.conv3, self.bn3, out, residual=idt, residual_is_ancestor=False)
        idt = x if self.downsample is None else self.downsample(x)
        if self.fused_bn:
            out = self._conv_bn(self.conv2, self.bn2, self._conv_bn(self.conv1, self.bn1, x, defer=defer1), defer=defer)
            # identity shortcut: x is an ancestor of conv3's output, so bn3 may fold
            # its residual gradient into the previous block's bn3 backward (ops/bn.py)
            return self._conv_bn(self.conv3, self.bn3, out, residual=idt,
                                 residual_is_ancestor=self.downsample is None)
        out = F.relu(self.bn1(self.conv1(x)), inplace=True)
        out = F.relu(self.bn2(self.conv2(out)), inplace=True)
        out = self.bn3(self.conv3(out))
        return F.relu(out + idt, inplace=True)


class ResNet(nn.Module):
    def __init__(self, layers: List[int], num_classes: int = 1000, zero_init_residual: bool = False,
                 fused_bn: bool = False):
        super().__init__()
        self.inplanes = 64
        self.fused_bn = fused_bn
        self.conv1 = (ConvBF16 if fused_bn else nn.Conv2d)(3, 64, 7, 2, 3, bias=False)
        self.bn1 = _bn(64, fused_bn)
        # fused path: NHWC bf16 kernels with a one-byte argmax (ops/pool.py)
        self.maxpool = MaxPool2dNHWC(3, 2, 1) if fused_bn else nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make(64, layers[0])
        self.layer2 = self._make(128, layers[1], 2)
        self.layer3 = self._make(256, layers[2], 2)
        self.layer4 = self._make(512, layers[3], 2)
        self.fc = nn.Linear(512 * Bottleneck.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)

    def _make(self, width: int, blocks: int, stride: int = 1) -> nn.Sequential:
        down = None
        cout = width * Bottleneck.expansion
        if stride != 1 or self.inplanes != cout:
            down = nn.Sequential(_conv1x1(self.inplanes, cout, stride, fused=self.fused_bn),
                                 _bn(cout, self.fused_bn, act=None))
        layers = [Bottleneck(self.inplanes, width, stride, down, self.fused_bn)]
        self.inplanes = cout
        layers += [Bottleneck(cout, width, fused_bn=self.fused_bn) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        if self.fused_bn and self.bn1.training:
            # the stem kernel may compute bn1's batch statistics in its epilogue, and
            # bn1 + ReLU run inside the max pool's pass (ops/bn.py ``pool``)
            st = BNStats()
            x = self.bn1(self.conv1(x, bn_stats=st), bn_stats=st, pool=self.maxpool)
        else:
            x = self.bn1(self.conv1(x))
            x = self.maxpool(x if self.fused_bn else F.relu(x, inplace=True))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        if self.fused_bn:
            return self.fc(global_avg_pool_nhwc(x))  # NHWC backward kernel (ops/pool.py)
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


def resnet50(num_classes: int = 1000, zero_init_residual: bool = False, fused_bn: bool = False) -> ResNet:
    """``fused_bn``: BatchNorm+ReLU(+residual add) layers run the gfx950 fused kernels
    (``ops.bn.BatchNormAct2d``) -- identical parameters and state-dict keys."""
    return ResNet([3, 4, 6, 3], num_classes, zero_init_residual, fused_bn)


RESNET50_PARAMS = 25_557_032


_RESIDENT: dict = {}  # (spec, device) -> device columns, per process (recycled workers reuse them)


class SyntheticImageNet(Dataset):
    """Random images / labels of ImageNet shape, generated per index (deterministic).

    ``resident_tensors(device)`` is the GPU data path (``lightning/sampling.py``):
    the whole set generated once -- the SAME per-index values ``__getitem__``
    returns, on a thread pool -- and held in HBM as a channels_last image tensor
    plus int64 labels (3,200 images at 224 px = 1.9 GB of 288 GB).  The
    graph-captured Trainer step then gathers each batch on the device from the
    DistributedSampler order: no per-image CPU ``randn``, no pageable H2D copy."""

    def __init__(self, length: int = 1281, image_size: int = 224, num_classes: int = 1000, seed: int = 0):
        self.length, self.size, self.nc, self.seed = length, image_size, num_classes, seed

    def __len__(self) -> int:
        return self.length

    def __getitem__(self, i: int):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        return torch.randn(3, self.size, self.size, generator=g), int(torch.randint(0, self.nc, (1,), generator=g))

    def resident_tensors(self, device) -> List[torch.Tensor]:
        device = torch.device(device)
        key = (self.length, self.size, self.nc, self.seed, str(device))
        cols = _RESIDENT.get(key)
        if cols is not None:
            return cols
        from concurrent.futures import ThreadPoolExecutor

        n, s = self.length, self.size
        host = torch.empty(n, s, s, 3, pin_memory=device.type == "cuda")  # NHWC rows
        labels = torch.empty(n, dtype=torch.int64)

        def fill(lo_hi):
            for i in range(*lo_hi):
                x, y = self[i]
                host[i].copy_(x.permute(1, 2, 0))
                labels[i] = y

        workers = max(1, min(8, (os.cpu_count() or 1), n // 64 or 1))
        step = -(-n // workers)
        with ThreadPoolExecutor(workers) as ex:
            list(ex.map(fill, [(a, min(n, a + step)) for a in range(0, n, step)]))
        x = host.to(device, non_blocking=True).permute(0, 3, 1, 2)  # [N, 3, S, S] channels_last
        y = labels.to(device, non_blocking=True)
        if device.type == "cuda":
            torch.cuda.current_stream(device).synchronize()  # the pinned source is freed below
        while len(_RESIDENT) >= 2:  # a train and a validation set per process (recycled workers)
            _RESIDENT.pop(next(iter(_RESIDENT)))
        _RESIDENT[key] = [x, y]
        return _RESIDENT[key]


class LightningResNet50(LightningModule):
    """ResNet-50 as a LightningModule (SGD momentum, cross-entropy) -- BASELINE.json
    config 5 through ``RayAccelerator`` + ``Trainer.fit``.

    ``hip_graph_step = True``: the Trainer captures the whole training step
    (forward, backward, DDP bucket all-reduce, fused SGD) in one hipGraph and
    replays it (``lightning/graph_step.py``); with the resident synthetic set the
    batches are gathered on the device inside that graph.  Parameters are
    channels_last (NHWC convolutions on MFMA, no per-use weight re-layout)."""

    hip_graph_step = True

    def __init__(self, config: Optional[dict] = None):
        super().__init__()
        cfg = dict(lr=0.1, momentum=0.9, weight_decay=5e-5, batch_size=64, num_classes=1000,
                   image_size=224, n_train=512, n_val=0, fused_bn=True, num_workers=0)
        cfg.update(config or {})
        self.cfg = cfg
        self.model = resnet50(cfg["num_classes"], fused_bn=cfg["fused_bn"]).to(memory_format=torch.channels_last)

    def forward(self, x):
        return self.model(x)

    def training_step(self, batch, batch_idx):
        x, y = batch
        x = x.contiguous(memory_format=torch.channels_last)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=x.is_cuda):
            logits = self(x)
        loss = F.cross_entropy(logits.float(), y)
        self.log("train_loss", loss)
        return loss

    def validation_step(self, batch, batch_idx):
        """Loss and top-1 of one held-out batch (BatchNorm in eval mode: running stats)."""
        x, y = batch
        x = x.contiguous(memory_format=torch.channels_last)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=x.is_cuda):
            logits = self(x)
        loss = F.cross_entropy(logits.float(), y)
        return {"val_loss": loss, "val_acc": (logits.argmax(1) == y).float().mean()}

    def validation_epoch_end(self, outputs):
        if outputs:
            self.log("val_loss", torch.stack([o["val_loss"] for o in outputs]).mean())
            self.log("val_acc", torch.stack([o["val_acc"] for o in outputs]).mean())

    def configure_optimizers(self):
        return torch.optim.SGD(self.parameters(), lr=self.cfg["lr"], momentum=self.cfg["momentum"],
                               weight_decay=self.cfg["weight_decay"])

    def val_dataloader(self):
        """``n_val`` held-out synthetic images (seed 1: disjoint from the training
        draws); none when ``n_val`` is 0."""
        if not self.cfg["n_val"]:
            return None
        from torch.utils.data import DataLoader

        ds = SyntheticImageNet(self.cfg["n_val"], self.cfg["image_size"], self.cfg["num_classes"], seed=1)
        return DataLoader(ds, batch_size=self.cfg["batch_size"], num_workers=self.cfg["num_workers"])

    def train_dataloader(self):
        from torch.utils.data import DataLoader

        ds = SyntheticImageNet(self.cfg["n_train"], self.cfg["image_size"], self.cfg["num_classes"])
        return DataLoader(ds, batch_size=self.cfg["batch_size"], num_workers=self.cfg["num_workers"],
                          drop_last=True)
