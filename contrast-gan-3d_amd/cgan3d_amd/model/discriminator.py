"""PatchGANDiscriminator — reference ``contrast_gan_3D/model/discriminator.py:9-84``, HIP compute.

Same constructor and module tree (``model.first``, ``model.middle.n``, ``model.last``) hence the
same ``state_dict``.  The hot-path configuration is the gradient-penalty critic
(``norm_layer=nn.Identity``, ``experiments/gradient_penalty_conf.py:14``): k4 s2 p1 convs with
bias + LeakyReLU(0.2) fused in the conv epilogue, last k4 s1 p1 conv to one channel.  Under
autograd ``backward`` runs the critic input-grad chain (LeakyReLU masks fused into the
input-grad conv epilogues) and the weight-grad kernels.  The GP's double backward runs fused in
the Trainer's step engine (``cgan3d_amd.engine``); for the Identity-norm critic it is also
available through autograd (``torch.autograd.grad(..., create_graph=True)`` then ``backward``, as
the reference's ``wgan_gradient_penalty`` does, model/utils.py:34-41) via ``_CriticInputGradFn``.  Also built: the weight-clip
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
    is_2D: bool = False  # the 2-D variants (experiments/conf_2D.py): planar kernels, f32


class PatchGANDiscriminator(nn.Module):
    def __init__(self, channels_in: int, init_channels_out: int, discriminator_depth: int, is_2D: bool = False,
                 kernel_size: int = 4, padding: int = 1, norm_layer: type | None = None, **kwargs):
        super().__init__()
        stride = 2
        slope = kwargs.get("negative_slope", 0.01)
        norm = {None: "batch", nn.BatchNorm3d: "batch", nn.BatchNorm2d: "batch", nn.Identity: "identity",
                nn.LayerNorm: "layer"}.get(norm_layer, "other")
        self.config = CriticConfig(channels_in, init_channels_out, discriminator_depth, slope, norm, bool(is_2D))
        self.is_2D = is_2D
        self._unsupported = None
        if kernel_size != 4 or padding != 1 or norm not in ("identity", "batch", "layer") or (is_2D and norm == "layer"):
            self._unsupported = ("the HIP critic implements the k4 p1 critic with Identity norm (GP conf), "
                                 "BatchNorm (weight-clip conf, 3-D and conf_2D) or LayerNorm (gp_layernorm conf, 3-D)")
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
        if x.dim() != (4 if self.is_2D else 5) or x.shape[1] != self.config.channels_in or self.config.channels_in != 1:
            raise ValueError(f"PatchGANDiscriminator expects [N,1,{'H,W' if self.is_2D else 'D,H,W'}], "
                             f"got {tuple(x.shape)}")
        params = list(self.parameters())
        if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params)):
            return _CriticFn.apply(x, self, *params)
        n, _, *dims = x.shape
        self._check_layernorm_shape(dims)
        plan = self.plan_for(n, dims)
        logits = plan.forward(self._tensors(), x.detach().float().contiguous().view(n, *dims, 1), 0, n,
                              training=self.training)
        return logits.clone().view(n, 1, *logits.shape[(2 if self.is_2D else 1):4])


class _CriticFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, module, *params):
        n, _, *dims = x.shape
        module._check_layernorm_shape(dims)
        plan = module.plan_for(n, dims, fresh=True)  # activations live until backward
        xc = x.detach().float().contiguous().view(n, *dims, 1)
        logits = plan.forward(module._tensors(), xc, 0, n, training=module.training)
        ctx.plan, ctx.module, ctx.xc, ctx.needs_x = plan, module, xc, x.requires_grad
        ctx.x_shape = x.shape
        return logits.clone().view(n, 1, *logits.shape[(2 if module.is_2D else 1):4])

    @staticmethod
    def backward(ctx, grad_out):
        create_graph = torch.is_grad_enabled()  # autograd.grad(..., create_graph=True): model/utils.py:34-39
        plan, module, xc = ctx.plan, ctx.module, ctx.xc
        if create_graph and (plan.bn or plan.ln):
            raise NotImplementedError("create_graph through the HIP critic is built for the GP conf's Identity-norm "
                                      "critic; the LayerNorm critic's penalty runs in the Trainer step engine "
                                      "(cgan3d_amd.engine.StepEngine)")
        n = xc.shape[0]
        names = [nm for nm, _ in module.named_parameters()]
        with torch.no_grad():
            plan.dz[-1].view(-1).copy_(grad_out.reshape(-1))
            dx = torch.empty_like(xc) if ctx.needs_x else None
            grads = {nm: torch.zeros_like(p) for nm, p in module.named_parameters()}
            if plan.bn and not module.training:
                raise NotImplementedError("backward through the eval-mode BatchNorm critic")
            plan.input_grad(module._tensors(), 0, n, dx if dx is not None else xc, 0, n if dx is not None else 0,
                            G=grads)
            plan.weight_grads(module._tensors(), grads, xc, n, n)
        dxo = dx.view(ctx.x_shape) if dx is not None else None
        if create_graph and dxo is not None:
            # dx as a differentiable function of the parameters (and of grad_out): the penalty's
            # double backward, _CriticInputGradFn.backward
            dxo = _CriticInputGradFn.apply(dxo, grad_out, _PlanRef(plan, module), *module.parameters())
        return (dxo, None, *[grads[nm] for nm in names])


class _PlanRef:
    """Carries a fresh CriticPlan (activations, masks and the dz chain of one forward / backward)
    into the second-order Function without making it an autograd input."""

    def __init__(self, plan, module):
        self.plan, self.module = plan, module


class _CriticInputGradFn(torch.autograd.Function):
    """dx = dD/dx . grad_out of the Identity-norm critic (convs + LeakyReLU, gradient_penalty_conf.py:14),
    differentiable w.r.t. the parameters and grad_out: what ``torch.autograd.grad(critic(x), x,
    create_graph=True)`` provides the reference's wgan_gradient_penalty (model/utils.py:34-41).

    For s = <dx, gamma>: ds/dW_l = wgrad(nu_{l-1}, dz_l) with the forward-mode tangent
    nu_0 = gamma, nu_l = m_l * conv_l(nu_{l-1}) along the fixed LeakyReLU masks m_l and dz_l the
    first backward's chain; ds/db_l = 0; ds/dgrad_out = conv_last(nu_{L-1}); ds/dx = 0 (the masks
    are piecewise constant in x).  The same chain as the Trainer's fused penalty (engine.py)."""

    @staticmethod
    def forward(ctx, dx, grad_out, ref, *params):
        ctx.ref = ref
        ctx.go_shape = grad_out.shape
        return dx.view_as(dx)

    @staticmethod
    def backward(ctx, gamma):
        plan, module = ctx.ref.plan, ctx.ref.module
        ctx.ref = None  # the plan's activations are overwritten below: one double backward per forward
        n = gamma.shape[0]
        names = [nm for nm, _ in module.named_parameters()]
        with torch.no_grad():
            P = module._tensors()
            g = gamma.detach().float().contiguous().view(n, *plan.dims, 1)
            plan.gp_forward_mode(P, g, 0, n)  # nu_l over a_l (the masks are consumed as it goes)
            grads = {nm: torch.zeros_like(p) for nm, p in module.named_parameters()}
            sink = {nm: torch.zeros_like(p) for nm, p in module.named_parameters() if nm.endswith("bias")}
            plan.weight_grads(P, {**grads, **sink}, g, n, n)
            d_go = None
            if ctx.needs_input_grad[1]:  # J gamma: the last conv (no bias) over nu_{L-1}
                ly = plan.layers[-1]
                geo = plan._geo(ops.conv_fwd_geom(n, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p, planar=plan.pl),
                                plan.wf[-1])
                w = plan.wf[-1] if plan.wf[-1] is not None else P[f"{ly.name}.weight"]
                out = torch.empty((n, *ly.dout, 1), device=gamma.device)
                ops.conv(geo, plan.a[-2][:n], w, out)
                d_go = out.view(ctx.go_shape)
        return (None, d_go, None, *[grads[nm] for nm in names])
