"""BatchNorm (+ optional residual add) (+ optional ReLU) as one op.

In a ResNet-50 training step every convolution is followed by BN→ReLU, and the last BN of each bottleneck
by BN→add→ReLU.  Executed as separate PyTorch ops that is 3–4 full passes over every activation in the
forward and as many again in the backward.  ``BatchNormAct`` exposes the fused form; on a GPU it dispatches
to the hand-written NHWC bf16 HIP kernels in ``csrc/bn_kernels.hip`` (stats pass + one fused
normalise/affine/add/ReLU pass forward; one fused dgamma/dbeta reduction + one dx pass backward).  On CPU
(tests, no GPU in the build container) it runs the PyTorch composition, which is also the numerics
reference the GPU tests compare against.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F


def bn_act_reference(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor,
                     running_mean: Optional[torch.Tensor], running_var: Optional[torch.Tensor],
                     training: bool, momentum: float, eps: float, residual: Optional[torch.Tensor],
                     act: bool) -> torch.Tensor:
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    if residual is not None:
        y = y + residual
    if act:
        y = F.relu(y)
    return y


class BatchNormAct(nn.Module):
    def __init__(self, num_features: int, act: bool = True, residual: bool = False, fused: bool = True,
                 eps: float = 1e-5, momentum: float = 0.1):
        super().__init__()
        self.num_features = num_features
        self.act = act
        self.residual = residual
        self.fused = fused
        self.eps = eps
        self.momentum = momentum
        self.weight = nn.Parameter(torch.ones(num_features))
        self.bias = nn.Parameter(torch.zeros(num_features))
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features))

    def reset_running_stats(self) -> None:
        with torch.no_grad():
            self.running_mean.zero_()
            self.running_var.fill_(1.0)

    def forward(self, x: torch.Tensor, identity: Optional[torch.Tensor] = None, residual_grad_box=None,
                residual_link: bool = False, defer_apply: bool = False) -> torch.Tensor:
        """``defer_apply``: the caller guarantees the output feeds only the residual add of another
        BatchNormAct (see ``ops.bn_fused.bn_act``)."""
        if self.residual and identity is None:
            raise ValueError("BatchNormAct(residual=True) needs the identity tensor")
        if self.fused and x.is_cuda:
            from polyaxon_amd.ops import bn_fused
            if bn_fused.supported(x):
                ext = getattr(x, "_plx_channel_stats", None)  # set by ops.conv1x1 on its output
                return bn_fused.bn_act(x, self.weight, self.bias, self.running_mean, self.running_var,
                                       self.training, self.momentum, self.eps, identity, self.act, ext,
                                       residual_grad_box, residual_link, defer_apply)
        if identity is not None and identity.is_cuda:
            from polyaxon_amd.ops.bn_fused import materialize
            identity = materialize(identity)
        return bn_act_reference(x, self.weight, self.bias, self.running_mean, self.running_var,
                                self.training, self.momentum, self.eps, identity, self.act)

    def extra_repr(self) -> str:
        return f"{self.num_features}, act={self.act}, residual={self.residual}, fused={self.fused}"
