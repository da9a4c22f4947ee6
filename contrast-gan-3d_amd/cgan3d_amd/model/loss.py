"""Losses — reference ``contrast_gan_3D/model/loss.py:11-80``, HIP compute.

Standalone modules with the reference's call signatures.  Each forward runs the fused loss
kernels of ``csrc/loss.hip`` and keeps the input-gradient it produces for ``backward``
(the reference's custom ``StableStd`` gradient, ``loss.py:25-29``, included).  Inside the
Trainer these reductions are fused into the step engine instead.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import Tensor, nn

from .. import _lib as L
from .. import ops


def _zncc_hu(source: Tensor, target: Tensor, mask: Optional[Tensor], lo: float, hi: float, sim_w: float,
             hu_w: float):
    """One launch sequence of cgan3d_generator_output_grad; returns (losses[8], d loss/d source)."""
    s = source.detach().float().contiguous().view(-1)
    t = target.detach().float().contiguous().view(-1)
    n = s.numel()
    m = (mask.detach().reshape(-1).to(torch.uint8).contiguous() if mask is not None
         else torch.zeros(n, dtype=torch.uint8, device=s.device))
    att = torch.zeros_like(s)  # (1 - att^2) = 1: the kernel then returns -dL/ds
    dz = torch.empty_like(s)
    losses = torch.zeros(8, device=s.device)
    ws = torch.empty(ops.loss_ws_floats(), device=s.device)
    ops.generator_output_grad(s, t, att, m, None, n, lo, hi, sim_w, hu_w, dz, losses, ws)
    return losses, (-dz).view_as(source)


class _LossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, source, value, grad):
        ctx.save_for_backward(grad)
        return value

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        return g * grad, None, None


class ZNCCLoss(nn.Module):
    """``-cc / (std_s * std_t + 1e-8)`` over the whole batch tensor (loss.py:32-41)."""

    def forward(self, source: Tensor, target: Tensor) -> Tensor:
        losses, grad = _zncc_hu(source, target, None, 0.0, 0.0, 1.0, 0.0)
        value = losses[L.L_SIM].clone()
        if torch.is_grad_enabled() and source.requires_grad:
            return _LossFn.apply(source, value, grad)
        return value


class HULoss(nn.Module):
    """Masked squared distance to the [min, max] HU band (loss.py:44-71)."""

    def __init__(self, min_HU_contstraint: float, max_HU_constraint: float, patch_size=None):
        super().__init__()
        self.lo, self.hi = float(min_HU_contstraint), float(max_HU_constraint)
        self.patch_size = patch_size

    def forward(self, batch: Tensor, mask: torch.BoolTensor) -> Tensor:
        losses, grad = _zncc_hu(batch, batch, mask, self.lo, self.hi, 0.0, 1.0)
        value = losses[L.L_HU].clone()
        if torch.is_grad_enabled() and batch.requires_grad:
            return _LossFn.apply(batch, value, grad)
        return value


class WassersteinLoss(nn.Module):
    """``mean(fake) [- mean(real)]`` (loss.py:74-80)."""

    @staticmethod
    def forward(fake: Tensor, real: Optional[Tensor] = None) -> Tensor:
        def mean(x):
            xf = x.detach().float().contiguous().view(-1)
            losses = torch.zeros(8, device=xf.device)
            dl = torch.empty_like(xf)
            ops.generator_logits_grad(xf, xf.numel(), -1.0, dl, losses)  # losses[G] = mean(x), dl = 1/n
            v = losses[L.L_G].clone()
            if torch.is_grad_enabled() and x.requires_grad:
                return _LossFn.apply(x, v, dl.view_as(x))
            return v

        ret = mean(fake)
        if real is not None:
            ret = ret - mean(real)
        return ret
