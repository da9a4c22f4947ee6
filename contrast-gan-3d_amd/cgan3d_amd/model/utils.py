"""Shape helpers and the WGAN gradient penalty — reference ``contrast_gan_3D/model/utils.py``.

``convolution_output_shape`` / ``compute_convolution_filters_shape`` / ``count_parameters`` are
host-side bookkeeping (utils.py:47-105).  ``wgan_gradient_penalty`` (utils.py:12-41) keeps the
reference signature; with this package's critic it is computed by the HIP critic plan: g = dD/dx
at the interpolation (forward + input-grad chain seeded with ones), the per-sample norm
reduction, and — for ``backward`` — the forward-mode chain that yields the critic
weight-gradients of the penalty without a double-backward graph (see cgan3d_amd.engine).
"""
from __future__ import annotations

import builtins
from typing import List, Optional, Union

import numpy as np
import torch
from torch import Tensor, nn


def wgan_gradient_penalty(real_batch: Tensor, fake_batch: Tensor, critic: nn.Module,
                          device: Union[torch.device, str] = "cpu", lambda_: float = 10,
                          rng: Optional[np.random.Generator] = None, eps: Optional[Tensor] = None) -> Tensor:
    interp_sample_size, *t_shape = real_batch.shape
    if len(real_batch) != len(fake_batch):  # utils.py:21-25
        interp_sample_size = min(len(real_batch), len(fake_batch))
        rng = rng or np.random.default_rng()
        real_batch = real_batch[rng.integers(len(real_batch), size=interp_sample_size)]
        fake_batch = fake_batch[rng.integers(len(fake_batch), size=interp_sample_size)]
    if eps is None:
        eps = torch.rand((interp_sample_size,) + (1,) * len(t_shape), device=device)
    params = list(critic.parameters())
    return _GradientPenaltyFn.apply(real_batch.detach(), fake_batch.detach(), eps.detach(), critic, float(lambda_),
                                    *params)


class _GradientPenaltyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, real, fake, eps, critic, lambda_, *params):
        from .. import ops
        n, _, *dims = real.shape
        plan = critic.plan_for(n, dims, fresh=True)  # kept until backward
        P = critic._tensors()
        V = dims[0] * dims[1] * dims[2]
        x = torch.empty((n, *dims, 1), device=real.device)
        ops.gp_interpolate(real.contiguous(), fake.contiguous(), eps.contiguous(), x, n, V)
        plan.forward(P, x, 0, n)
        plan.dz[-1].fill_(1.0)
        g = torch.empty_like(x)
        plan.input_grad(P, 0, n, g, 0, n)
        losses = torch.zeros(8, device=real.device)
        ws = torch.empty(ops.loss_ws_floats(), device=real.device)
        gamma = torch.empty_like(x)
        ops.gradient_penalty(g, n, V, lambda_, gamma, losses, ws)
        ctx.state = (plan, critic, x, gamma, n)
        return losses[2].clone()

    @staticmethod
    def backward(ctx, grad_out):
        plan, critic, x, gamma, n = ctx.state
        P = critic._tensors()
        gamma = gamma * grad_out
        plan.gp_forward_mode(P, gamma, 0, n)
        names = [nm for nm, _ in critic.named_parameters()]
        grads = {nm: torch.zeros_like(p) for nm, p in critic.named_parameters()}
        # biases receive no gradient from the penalty (LeakyReLU masks are piecewise constant)
        bias_sink = {nm: torch.zeros_like(p) for nm, p in critic.named_parameters()}
        plan.weight_grads(P, {**grads, **{k: v for k, v in bias_sink.items() if k.endswith("bias")}}, gamma, n, n)
        return (None, None, None, None, None, *[grads[nm] for nm in names])


# simplified versions of torch's Conv3d / ConvTranspose3d output-shape formulas (utils.py:47-67)
def convolution_output_shape(dims: List[int], c_out: int, kernel_size: int, padding: int, stride: int,
                             dilation: int = 1, transpose_output_padding: Optional[int] = None) -> List[int]:
    def fwd(x):
        return int((x + 2 * padding - dilation * (kernel_size - 1) - 1) / stride + 1)

    def tr(x):
        return int((x - 1) * stride - 2 * padding + dilation * (kernel_size - 1) + transpose_output_padding + 1)

    f = tr if transpose_output_padding is not None else fwd
    return [c_out] + [f(d) for d in dims[1:]]


def compute_convolution_filters_shape(model: nn.Module, input_shape, show: bool = True) -> List[int]:
    lines = [f"Input shape: {list(input_shape)}"]
    for n, m in model.named_modules():
        if type(m) in (nn.Conv3d, nn.Conv2d, nn.ConvTranspose3d, nn.ConvTranspose2d):
            kw = {}
            if isinstance(m, (nn.ConvTranspose3d, nn.ConvTranspose2d)):
                kw = {"transpose_output_padding": m.output_padding[0]}
            input_shape = convolution_output_shape(input_shape, m.out_channels, m.kernel_size[0], m.padding[0],
                                                   m.stride[0], **kw)
            bias = "" if m.bias is None else f" bias: {list(m.bias.shape)}"
            lines.append(f"{n:<40} -> {str(input_shape):<22} {'# params: ' + str(count_parameters(m)):<20} "
                         f"weight: {str(list(m.weight.shape)):<20}{bias}")
    if show:
        for ln in lines:
            print(ln)
    return input_shape


def count_parameters(model: nn.Module, print: bool = False) -> int:  # noqa: A002 (reference signature)
    tot = 0
    for n, p in model.named_parameters():
        if p.requires_grad:
            tot += p.numel()
            if print:
                builtins.print(n, p.numel())
    return tot
