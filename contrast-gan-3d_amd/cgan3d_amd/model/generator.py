"""ResnetGenerator — reference ``contrast_gan_3D/model/generator.py:9-90``, HIP compute.

Same constructor, same module tree (``model.first``, ``model.downsampling.i``,
``model.resnet_backbone.r.block{0,1}``, ``model.upsampling.j``, ``model.last_conv``,
``model.tanh``) and therefore the same ``state_dict``.  ``forward`` runs the fused generator plan
(``cgan3d_amd.engine.GeneratorPlan``): channels-last implicit-GEMM convs with the BatchNorm
statistics produced in the conv epilogue, BN+ReLU(+residual) apply kernels, and the last
reflect-padded conv with bias + tanh.  Under autograd, ``backward`` is the hand-derived
generator backward of the same plan (first-order; inputs are data and get no gradient).
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass

import torch
import torch.nn as nn

from .. import ops
from .blocks import ConvBlock, ResNetBlock


@dataclass(frozen=True)
class GenConfig:
    n_resnet_blocks: int = 4
    n_updownsample_blocks: int = 2
    init_channels_out: int = 16
    is_2D: bool = False  # the 2-D variants (experiments/conf_2D.py): planar kernels, f32


class ResnetGenerator(nn.Module):
    def __init__(self, n_resnet_blocks: int, n_updownsample_blocks: int, init_channels_out: int,
                 is_2D: bool = False, resnet_dropout_prob: float = 0.0, resnet_padding_mode: str = "zeros"):
        assert n_resnet_blocks > 0
        super().__init__()
        self.config = GenConfig(n_resnet_blocks, n_updownsample_blocks, init_channels_out, bool(is_2D))
        self.is_2D = is_2D
        if resnet_dropout_prob > 0 or resnet_padding_mode != "zeros":
            self._unsupported = "dropout / non-zero resnet padding variants are not used by any reference config"
        else:
            self._unsupported = None
        common = {"kernel_size": 7, "padding_mode": "reflect", "padding": 3}
        model = [("first", ConvBlock(is_2D, 1, init_channels_out, **common))]
        down = []
        for i in range(n_updownsample_blocks):
            dim_in = init_channels_out * 2**i
            dim_out = dim_in * 2
            down.append(ConvBlock(is_2D, dim_in, dim_out, kernel_size=3, stride=2, padding=1))
        model.append(("downsampling", nn.Sequential(*down)))
        model.append(("resnet_backbone", nn.Sequential(*[
            ResNetBlock(is_2D, dim_out, dim_out, dropout_prob=resnet_dropout_prob, padding_mode=resnet_padding_mode)
            for _ in range(n_resnet_blocks)])))
        up = []
        for i in range(n_updownsample_blocks, 0, -1):
            dim_in = init_channels_out * 2**i
            up.append(ConvBlock(is_2D, dim_in, dim_in // 2, kernel_size=3, stride=2, padding=1, output_padding=1,
                                upsample=True))
        model.append(("upsampling", nn.Sequential(*up)))
        model.append(("last_conv", (nn.Conv2d if is_2D else nn.Conv3d)(init_channels_out, 1, **common, bias=True)))
        model.append(("tanh", nn.Tanh()))
        self.model = nn.Sequential(OrderedDict(model))
        self._plan = None

    def _tensors(self):
        d = dict(self.named_parameters())
        d.update(dict(self.named_buffers()))
        return d

    def plan_for(self, n, dims, fresh=False):
        from ..engine import GeneratorPlan
        # the plan's packed-weight descriptors hold raw parameter addresses: rebuild if they moved
        key = (n, tuple(dims), self.model.first.conv.weight.device, tuple(p.data_ptr() for p in self.parameters()))
        if fresh or self._plan is None or self._plan[0] != key:
            plan = GeneratorPlan(self.config, n, tuple(dims), key[2], self._tensors(), allow_resize=not fresh)
            if fresh:
                return plan
            self._plan = (key, plan)
        return self._plan[1]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self._unsupported:
            raise NotImplementedError(self._unsupported)
        if x.dim() != (4 if self.is_2D else 5) or x.shape[1] != 1:
            raise ValueError(f"ResnetGenerator expects [N,1,{'H,W' if self.is_2D else 'D,H,W'}], got {tuple(x.shape)}")
        params = [p for p in self.parameters()]
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            return _GeneratorFn.apply(x, self, *params)
        n, _, *dims = x.shape
        plan = self.plan_for(n, dims)
        plan.pack()  # weights may have changed since the plan was built
        xc = x.detach().float().contiguous().view(n, *dims, 1)
        plan.forward(self._tensors(), xc, training=self.training)
        # dims that are not multiples of 4 come out at other dims (the reference's conv arithmetic)
        out = plan.out_dims[1:] if self.is_2D else plan.out_dims
        return plan.att.clone().view(n, 1, *out)


class _GeneratorFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, module, *params):
        if not module.training:
            raise NotImplementedError("generator backward with eval-mode BatchNorm is not a reference path")
        n, _, *dims = x.shape
        plan = module.plan_for(n, dims, fresh=True)  # buffers live until backward
        xc = x.detach().float().contiguous().view(n, *dims, 1)
        plan.forward(module._tensors(), xc, training=True)
        ctx.plan, ctx.module, ctx.xc = plan, module, xc
        return plan.att.clone().view(n, 1, *dims)

    @staticmethod
    def backward(ctx, grad_out):
        if torch.is_grad_enabled():
            raise NotImplementedError("double backward through the HIP generator is not implemented")
        plan, module = ctx.plan, ctx.module
        ops.tanh_backward(plan.att, grad_out.contiguous().view_as(plan.att), plan.dz_last)
        names = [n for n, _ in module.named_parameters()]
        grads = {n: torch.zeros_like(p) for n, p in module.named_parameters()}
        plan.backward(module._tensors(), grads, ctx.xc)
        return (None, None, *[grads[n] for n in names])
