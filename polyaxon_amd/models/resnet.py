"""ResNet-50 (v1.5: stride on the 3x3 conv) for the Hyperband/ASHA north-star sweep (BASELINE.json config 3).

The reference ships no models; the north-star workload names a ResNet-50 sweep on
synthetic ImageNet-shape data, so the framework carries its own architecture definition.  It is laid out
for MI355X: channels_last (NHWC) activations so MIOpen picks its NHWC implicit-GEMM convolutions that
map onto MFMA, bf16 autocast compute, fp32 master weights living in one flat buffer (see
``polyaxon_amd.ops.flat``) so the whole optimizer step is one fused HIP kernel.
"""
from __future__ import annotations

from typing import List, Optional, Type

import torch
import torch.nn as nn

from polyaxon_amd.ops.conv1x1 import Conv1x1, GradMailbox
from polyaxon_amd.ops.conv import Conv3x3, ConvKxK
from polyaxon_amd.ops.norm import BatchNormAct
from polyaxon_amd.ops.pool import MaxPool3s2, global_avg_pool
from polyaxon_amd.ops.stem import StemConv, stem_bn_relu_pool


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, in_ch: int, width: int, stride: int = 1, downsample: Optional[nn.Module] = None,
                 fused: bool = True, native_conv: bool = True):
        super().__init__()
        out_ch = width * self.expansion
        # every conv but the stem runs as an (implicit) MFMA GEMM on the NHWC rows (ops/conv1x1.py, ops/conv.py)
        self.conv1 = Conv1x1(in_ch, width, native=native_conv)
        self.bn1 = BatchNormAct(width, act=True, fused=fused)
        self.conv2 = Conv3x3(width, width, stride, native=native_conv)
        self.bn2 = BatchNormAct(width, act=True, fused=fused)
        self.conv3 = Conv1x1(width, out_ch, native=native_conv)
        # bn3 fuses the residual add and the final ReLU: y = relu(bn(x) + identity)
        self.bn3 = BatchNormAct(out_ch, act=True, fused=fused, residual=True)
        self.downsample = downsample

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        train = self.training and torch.is_grad_enabled() and x.requires_grad
        box = GradMailbox() if train else None
        if self.downsample is None:
            # identity block: bn3's residual gradient is added inside conv1's dgrad GEMM (ops.conv1x1.GradMailbox),
            # so conv1's dgrad is x's whole gradient and serves the previous block's bn3 its backward partials
            out = self.bn1(self.conv1(x, grad_box=box, bn_link=True))
            out = self.bn2(self.conv2(out, bn_link=True))
            return self.bn3(self.conv3(out, bn_link=True), x, residual_grad_box=box)
        # downsampling block: conv1's data gradient is deferred into the downsample conv's dgrad epilogue, and the
        # downsample BatchNorm's output feeds only bn3, so bn3's dx pass reduces that BatchNorm's backward partials
        identity = self.downsample(x, grad_box=box)
        out = self.bn1(self.conv1(x, grad_sink=box, bn_link=True))
        out = self.bn2(self.conv2(out, bn_link=True))
        return self.bn3(self.conv3(out, bn_link=True), identity, residual_link=True)




class Downsample(nn.Module):
    def __init__(self, in_ch: int, out_ch: int, stride: int, fused: bool = True, native_conv: bool = True):
        super().__init__()
        self.conv = (Conv1x1(in_ch, out_ch, native=native_conv) if stride == 1
                     else ConvKxK(in_ch, out_ch, 1, stride, native=native_conv))
        self.bn = BatchNormAct(out_ch, act=False, fused=fused)

    def forward(self, x: torch.Tensor, grad_box: Optional[GradMailbox] = None) -> torch.Tensor:
        # the output feeds only bn3's residual add, which applies this BatchNorm's scale/bias itself
        # bn_link: the conv's dgrad (+ the box's conv1 gradient) is x's whole gradient -- it serves the BatchNorm that
        # produced x its backward partials (with conv1's dgrad when strided, ops.conv1x1.BnLink.request_split)
        return self.bn(self.conv(x, grad_box=grad_box, bn_link=True), defer_apply=True)


class ResNet(nn.Module):
    def __init__(self, layers: List[int], num_classes: int = 1000, width: int = 64,
                 zero_init_residual: bool = True, fused: bool = True, native_conv: bool = True):
        super().__init__()
        # 3 -> 64: the MFMA stem GEMM with BN-stats epilogue (ops/stem.py); other widths: the library convolution
        self.stem = (StemConv(3, width, native=native_conv) if width == 64
                     else nn.Conv2d(3, width, 7, stride=2, padding=3, bias=False))
        self.stem_bn = BatchNormAct(width, act=True, fused=fused)
        self.pool = MaxPool3s2(native=native_conv)
        stages = []
        in_ch = width
        for i, n in enumerate(layers):
            w = width * (2 ** i)
            stride = 1 if i == 0 else 2
            blocks = []
            for j in range(n):
                ds = None
                if j == 0 and (stride != 1 or in_ch != w * Bottleneck.expansion):
                    ds = Downsample(in_ch, w * Bottleneck.expansion, stride, fused=fused, native_conv=native_conv)
                blocks.append(Bottleneck(in_ch, w, stride if j == 0 else 1, ds, fused=fused, native_conv=native_conv))
                in_ch = w * Bottleneck.expansion
            stages.append(nn.Sequential(*blocks))
        self.stages = nn.Sequential(*stages)
        self.fc = nn.Linear(in_ch, num_classes)
        self.zero_init_residual = zero_init_residual
        self.reset_parameters()

    def init_spec(self):
        """(param, kind, scale) triples describing the per-tensor random init (used by the fused
        in-place re-initialiser, ``plx_init_flat``): kaiming-normal fan_out for convs, BN gamma=1
        (0 for the last BN of each residual branch when zero_init_residual), beta=0, fc uniform."""
        spec = []
        for name, mod in self.named_modules():
            if isinstance(mod, nn.Conv2d):
                fan_out = mod.out_channels * mod.kernel_size[0] * mod.kernel_size[1]
                spec.append((mod.weight, "normal", (2.0 / fan_out) ** 0.5))
            elif isinstance(mod, BatchNormAct):
                gamma = 0.0 if (self.zero_init_residual and mod.residual) else 1.0
                spec.append((mod.weight, "const", gamma))
                spec.append((mod.bias, "const", 0.0))
            elif isinstance(mod, nn.Linear):
                bound = 1.0 / mod.in_features ** 0.5
                spec.append((mod.weight, "uniform", bound))
                spec.append((mod.bias, "uniform", bound))
        return spec

    @torch.no_grad()
    def reset_parameters(self) -> None:
        for p, kind, scale in self.init_spec():
            if kind == "normal":
                p.normal_(0.0, scale)
            elif kind == "const":
                p.fill_(scale)
            else:
                p.uniform_(-scale, scale)
        for mod in self.modules():
            if isinstance(mod, BatchNormAct):
                mod.reset_running_stats()

    def forward_features(self, x: torch.Tensor) -> torch.Tensor:
        """Everything before the classifier head: the last stage's [N, C, H, W] output (channels_last on the GPU)."""
        x = self.stem(x)
        # BN + ReLU + max-pool fused (ops/stem.py): the 112x112 BatchNorm output is never materialised
        x = stem_bn_relu_pool(x, self.stem_bn, self.pool)
        return self.stages(x)

    def forward_head(self, x: torch.Tensor) -> torch.Tensor:
        """Global average pool (NHWC kernel, ops/pool.py) + fc."""
        x = torch.flatten(x.mean((2, 3)), 1) if x.is_contiguous() else global_avg_pool(x)
        return self.fc(x)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.forward_head(self.forward_features(x))


def resnet50(num_classes: int = 1000, fused: bool = True, **kw) -> ResNet:
    return ResNet([3, 4, 6, 3], num_classes=num_classes, fused=fused, **kw)


def resnet18ish(num_classes: int = 10, fused: bool = True, **kw) -> ResNet:
    """Small bottleneck ResNet used by CPU tests (same code path, fewer blocks and channels)."""
    return ResNet([1, 1, 1, 1], num_classes=num_classes, width=8, fused=fused, **kw)
