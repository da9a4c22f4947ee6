"""ConvBlock / ResNetBlock with the reference's constructor signatures and parameter layout.

Mirror of ``contrast_gan_3D/model/blocks.py:4-88``: the submodules are the same torch containers
(``conv``: ``nn.Conv3d`` / ``nn.ConvTranspose3d``; ``normalization``: ``nn.BatchNorm3d`` by
default, ``nn.Identity`` or ``nn.LayerNorm``; ``activation_fn``) so ``state_dict`` keys match
and checkpoints interchange.  The compute is the HIP library: ``forward`` runs the conv /
BatchNorm / activation kernels on channels-last activations (standalone use; the networks and
the Trainer drive the fused plans in ``cgan3d_amd.engine`` instead).
"""
from __future__ import annotations

import torch
from torch import Tensor, nn

from .. import _lib as L
from .. import ops


def _act_code(mod: nn.Module):
    if isinstance(mod, nn.ReLU):
        return L.ACT_RELU, 0.0
    if isinstance(mod, nn.LeakyReLU):
        return L.ACT_LRELU, float(mod.negative_slope)
    if isinstance(mod, nn.Identity):
        return L.ACT_NONE, 0.0
    raise NotImplementedError(f"activation {type(mod).__name__} has no HIP kernel")


class ConvBlock(nn.Module):
    """``act(norm(conv(x)))`` — reference ``model/blocks.py:4-53``."""

    def __init__(self, is_2D: bool, channels_in: int, channels_out: int, kernel_size: int, upsample: bool = False,
                 output_padding: int = 0, padding_mode: str = "zeros", padding: int = 0, stride: int = 1,
                 activation_fn: type = nn.ReLU, norm_layer: type | None = None, **kwargs):
        super().__init__()
        conv_class, args = (nn.Conv2d if is_2D else nn.Conv3d), {}
        if upsample:
            args = {"output_padding": output_padding}
            conv_class = nn.ConvTranspose2d if is_2D else nn.ConvTranspose3d
        if norm_layer is None:
            norm_layer = nn.BatchNorm2d if is_2D else nn.BatchNorm3d
        self.is_2D = is_2D
        self.conv = conv_class(channels_in, channels_out, kernel_size, stride=stride, bias=norm_layer == nn.Identity,
                               padding_mode=padding_mode, padding=padding, **args)
        norm_shape, norm_args = channels_out, {}
        if norm_layer == nn.LayerNorm and (ps := kwargs.get("patch_size")):
            norm_shape = ps
            if (affine := kwargs.get("elementwise_affine")) is not None:
                norm_args["elementwise_affine"] = affine
        self.normalization = norm_layer(norm_shape, **norm_args)
        act_kwargs = {}
        if (ns := kwargs.get("negative_slope")) is not None:
            act_kwargs["negative_slope"] = ns
        self.activation_fn = activation_fn(inplace=True, **act_kwargs)

    # -- standalone HIP forward (channels-first API tensors) -------------------------------
    def forward(self, x: Tensor) -> Tensor:
        if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters())):
            raise NotImplementedError("ConvBlock.forward with autograd: use ResnetGenerator / "
                                      "PatchGANDiscriminator or the Trainer step engine")
        conv = self.conv
        pl = self.is_2D  # 2-D variants: planar geometries on (1, H, W) grids
        if x.dim() != (4 if pl else 5):
            raise ValueError(f"ConvBlock expects [N, C, {'H, W' if pl else 'D, H, W'}], got {tuple(x.shape)}")
        n, cin, *sp = x.shape
        din = (1, *sp) if pl else tuple(sp)
        k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
        xc = x.movedim(1, -1).contiguous()
        reflect = conv.padding_mode == "reflect"
        keep = lambda a, v: v if not (pl and a == 0) else 1  # noqa: E731 (depth passes through in 2-D)
        if isinstance(conv, (nn.ConvTranspose3d, nn.ConvTranspose2d)):
            op = conv.output_padding[0]
            dout = tuple(keep(a, (d - 1) * s - 2 * p + k + op) for a, d in enumerate(din))
            g = ops.convt_fwd_geom(n, din, dout, cin, conv.out_channels, k, s, p, planar=pl)
        else:
            dout = tuple(keep(a, (d + 2 * p - k) // s + 1) for a, d in enumerate(din))
            g = ops.conv_fwd_geom(n, din, dout, cin, conv.out_channels, k, s, p, reflect, planar=pl)
        cout = conv.out_channels
        z = torch.empty((n, *dout, cout), device=x.device)
        act, slope = _act_code(self.activation_fn)
        norm = self.normalization
        out_shape = (n, cout, *(dout[1:] if pl else dout))

        def channels_first(t):
            return t.view(n, *(dout[1:] if pl else dout), cout).movedim(-1, 1).contiguous()
        if isinstance(norm, nn.Identity):
            ops.conv(g, xc, conv.weight, z, ops.epilogue(bias=conv.bias, act=act, slope=slope))
            return channels_first(z)
        if not isinstance(norm, (nn.BatchNorm3d, nn.BatchNorm2d)):
            raise NotImplementedError("LayerNorm critic (gp_layernorm.py) is outside this build's hot path")
        nvox = n * dout[0] * dout[1] * dout[2]
        ss = torch.empty(2 * cout, device=x.device)
        if norm.training:
            stats = torch.empty(ops.stats_floats(g), device=x.device)
            ops.conv(g, xc, conv.weight, z, ops.epilogue(stats=stats))
            mi = torch.empty(2 * cout, device=x.device)
            ops.bn_finalize(stats, stats.numel() // (2 * cout + 1), cout, norm.weight, norm.bias, norm.running_mean,
                            norm.running_var, norm.num_batches_tracked, ss, mi, momentum=norm.momentum, eps=norm.eps)
        else:
            ops.conv(g, xc, conv.weight, z)
            inv = torch.rsqrt(norm.running_var + norm.eps)
            ss[:cout] = norm.weight * inv
            ss[cout:] = norm.bias - norm.running_mean * ss[:cout]
        y = torch.empty_like(z)
        ops.bn_apply(z, nvox, cout, ss, act, y, slope=slope)
        assert channels_first(y).shape == out_shape
        return channels_first(y)


class ResNetBlock(nn.Module):
    """``x + block1(dropout(block0(x)))`` — reference ``model/blocks.py:56-88``."""

    def __init__(self, is_2D: bool, channels_in: int, channels_out: int, kernel_size: int = 3,
                 dropout_prob: float = 0.0, padding_mode: str = "zeros"):
        super().__init__()
        padding_amount = 1
        self.block0 = ConvBlock(is_2D, channels_in, channels_out, kernel_size, padding_mode=padding_mode,
                                padding=padding_amount, activation_fn=nn.Identity)
        self.dropout = nn.Dropout(p=dropout_prob) if dropout_prob > 0 else nn.Identity()
        self.block1 = ConvBlock(is_2D, channels_out, channels_out, kernel_size, padding_mode=padding_mode,
                                padding=padding_amount)

    def forward(self, x: Tensor) -> Tensor:
        if not isinstance(self.dropout, nn.Identity):
            raise NotImplementedError("dropout > 0 is not used by any reference config")
        return x + self.block1(self.block0(x))
