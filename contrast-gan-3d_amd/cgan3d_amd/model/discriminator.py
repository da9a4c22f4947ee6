"""PatchGANDiscriminator — reference ``contrast_gan_3D/model/discriminator.py:9-84``, HIP compute.

Same constructor and module tree (``model.first``, ``model.middle.n``, ``model.last``) hence the
same ``state_dict``.  The hot-path configuration is the gradient-penalty critic
(``norm_layer=nn.Identity``, ``experiments/gradient_penalty_conf.py:14``): k4 s2 p1 convs with
bias + LeakyReLU(0.2) fused in the conv epilogue, last k4 s1 p1 conv to one channel.  Under
autograd ``backward`` runs the critic input-grad chain (LeakyReLU masks fused into the
input-grad conv epilogues) and the weight-grad kernels.  The GP's double backward is done by the
Trainer's step engine (``cgan3d_amd.engine``), not through autograd.  Also built: the weight-clip
conf's BatchNorm critic and the gp_layernorm conf's LayerNorm critic (``norm_layer=nn.LayerNorm``,
``patch_size=(1, *patch)``, ``elementwise_affine=False``: ``experiments/gp_layernorm.py:9-11``).
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass

import torch
from torch import Tensor, nn

from .. import ops
from .blocks import ConvBlock
from .utils import convolution_output_shape


@dataclass(frozen=True)
class CriticConfig:
    channels_in: int = 1
    init_channels_out: int = 8
    discriminator_depth: int = 3
    negative_slope: float = 0.2
    norm: str = "identity"


class PatchGANDiscriminator(nn.Module):
    def __init__(self, channels_in: int, init_channels_out: int, discriminator_depth: int, is_2D: bool = False,
                 kernel_size: int = 4, padding: int = 1, norm_layer: type | None = None, **kwargs):
        super().__init__()
        stride = 2
        slope = kwargs.get("negative_slope", 0.01)
        norm = {None: "batch", nn.BatchNorm3d: "batch", nn.BatchNorm2d: "batch", nn.Identity: "identity",
                nn.LayerNorm: "layer"}.get(norm_layer, "other")
        self.config = CriticConfig(channels_in, init_channels_out, discriminator_depth, slope, norm)
        self._unsupported = None
        if is_2D or kernel_size != 4 or padding != 1 or norm not in ("identity", "batch", "layer"):
            self._unsupported = ("the HIP critic implements the 3-D k4 p1 critic with Identity norm (GP conf), "
                                 "BatchNorm (weight-clip conf) or LayerNorm (gp_layernorm conf); 2-D critics are "
                                 "SURVEY.md §8f row 4")
        elif norm == "layer" and kwargs.get("elementwise_affine", True):
            self._unsupported = ("the HIP LayerNorm critic implements the gp_layernorm conf's LayerNorm without "
                                 "affine parameters (gp_layernorm.py:9-11: elementwise_affine=False)")
        model = [("first", ConvBlock(is_2D, channels_in, init_channels_out, kernel_size, stride=stride,
                                     padding=padding, norm_layer=nn.Identity, activation_fn=nn.LeakyReLU, **kwargs))]
        middle = []
        kwargs = kwargs.copy()
        if ps := kwargs.get("patch_size"):
            kwargs["patch_size"] = convolution_output_shape(ps, init_channels_out, kernel_size, padding, stride)
        out_ = init_channels_out
        for n in range(discriminator_depth):
            in_ = min(2**n, 8) * init_channels_out
            out_ = min(2 ** (n + 1), 8) * init_channels_out
            if ps := kwargs.get("patch_size"):
                kwargs["patch_size"] = convolution_output_shape(ps, out_, kernel_size, padding, stride)
            middle.append(ConvBlock(is_2D, in_, out_, kernel_size, stride=stride, padding=padding,
                                    norm_layer=norm_layer, activation_fn=nn.LeakyReLU, **kwargs))
        model.append(("middle", nn.Sequential(*middle)))
        if norm == "layer" and self._unsupported is None and any(
                len(m.normalization.normalized_shape) != 4 for m in middle):
            self._unsupported = ("the HIP LayerNorm critic normalises each sample over (C, D, H, W): pass "
                                 "patch_size=(1, D, H, W) as gp_layernorm.py:9-11 does")
        model.append(("last", (nn.Conv2d if is_2D else nn.Conv3d)(out_, 1, kernel_size=kernel_size, stride=1,
                                                                   padding=padding)))
        self.model = nn.Sequential(OrderedDict(model))

    def _check_layernorm_shape(self, dims):
        """nn.LayerNorm's normalized_shape is fixed at construction (the patch size): reject
        other patch sizes as torch would."""
        if self.config.norm != "layer":
            return
        d = [(x + 2 - 4) // 2 + 1 for x in dims]  # the first k4 s2 p1 conv
        for m in self.model.middle:
            d = [(x + 2 - 4) // 2 + 1 for x in d]
            want = (m.conv.out_channels, *d)
            if tuple(m.normalization.normalized_shape) != want:
                raise RuntimeError(f"LayerNorm normalized_shape {tuple(m.normalization.normalized_shape)} does not "
                                   f"match the block output {want} (patch size {tuple(dims)})")

    def _tensors(self):
        return dict(self.state_dict(keep_vars=True))  # parameters and BatchNorm buffers

    def plan_for(self, n, dims, fresh: bool = False):
        """The critic plan for an ``n``-sample batch of ``dims`` patches: cached per shape (buffers
        are allocated once; the packed weight copies are refreshed on every call, the weights may
        have changed).  ``fresh`` plans own their buffers until the caller drops them (the autograd
        paths keep activations for their backward)."""
        from ..engine import CriticPlan
        dev = self.model.first.conv.weight.device
        key = (n, tuple(dims), dev, tuple(p.data_ptr() for p in self.parameters()))
        if fresh:
            return CriticPlan(self.config, n, tuple(dims), dev, self._tensors())
        if getattr(self, "_plan", None) is None or self._plan[0] != key:
            self._plan = (key, CriticPlan(self.config, n, tuple(dims), dev, self._tensors()))
        else:
            self._plan[1].pack()
        return self._plan[1]

    def forward(self, x: Tensor) -> Tensor:
        if self._unsupported:
            raise NotImplementedError(self._unsupported)
        if x.dim() != 5 or x.shape[1] != self.config.channels_in or self.config.channels_in != 1:
            raise ValueError(f"PatchGANDiscriminator expects [N,1,D,H,W], got {tuple(x.shape)}")
        params = list(self.parameters())
        if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params)):
            return _CriticFn.apply(x, self, *params)
        n, _, *dims = x.shape
        self._check_layernorm_shape(dims)
        plan = self.plan_for(n, dims)
        logits = plan.forward(self._tensors(), x.detach().float().contiguous().view(n, *dims, 1), 0, n,
                              training=self.training)
        return logits.clone().view(n, 1, *logits.shape[1:4])


class _CriticFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, module, *params):
        n, _, *dims = x.shape
        module._check_layernorm_shape(dims)
        plan = module.plan_for(n, dims, fresh=True)  # activations live until backward
        xc = x.detach().float().contiguous().view(n, *dims, 1)
        logits = plan.forward(module._tensors(), xc, 0, n, training=module.training)
        ctx.plan, ctx.module, ctx.xc, ctx.needs_x = plan, module, xc, x.requires_grad
        return logits.clone().view(n, 1, *logits.shape[1:4])

    @staticmethod
    def backward(ctx, grad_out):
        if torch.is_grad_enabled():
            raise NotImplementedError("create_graph through the HIP critic: the gradient penalty's double backward "
                                      "runs in the Trainer step engine (cgan3d_amd.engine.StepEngine)")
        plan, module, xc = ctx.plan, ctx.module, ctx.xc
        n = xc.shape[0]
        plan.dz[-1].view(-1).copy_(grad_out.reshape(-1))
        dx = torch.empty_like(xc) if ctx.needs_x else None
        names = [nm for nm, _ in module.named_parameters()]
        grads = {nm: torch.zeros_like(p) for nm, p in module.named_parameters()}
        if plan.bn and not module.training:
            raise NotImplementedError("backward through the eval-mode BatchNorm critic")
        plan.input_grad(module._tensors(), 0, n, dx if dx is not None else xc, 0, n if dx is not None else 0,
                        G=grads)
        plan.weight_grads(module._tensors(), grads, xc, n, n)
        dxo = dx.view(n, 1, *xc.shape[1:4]) if dx is not None else None
        return (dxo, None, *[grads[nm] for nm in names])
