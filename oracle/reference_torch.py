"""ORACLE — CPU fp32 restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / the timed CPU baseline.  The product path
(``contrast-gan-3d_amd/cgan3d_amd``) never imports it and fails loudly without its HIP library.

A from-scratch functional restatement (``torch.nn.functional`` + torch autograd, CPU, fp32) of
xqz-u/contrast-gan-3D's G+D training step, written from the reference's behaviour, not copied:

* generator  — ``contrast_gan_3D/model/generator.py:9-90`` built from ``model/blocks.py:4-88``
* critic     — ``contrast_gan_3D/model/discriminator.py:9-84``
* losses     — ``contrast_gan_3D/model/loss.py:11-80`` (ZNCC with the StableStd custom backward,
               masked HU-range loss, Wasserstein)
* GP         — ``contrast_gan_3D/model/utils.py:12-41``
* step       — ``contrast_gan_3D/trainer/Trainer.py:108-203`` with ``torch.optim.Adam`` semantics
               (``experiments/basic_conf.py:55,67``; GP conf ``gradient_penalty_conf.py:7-15``)

Parity of THIS module is pinned by the fixtures in ``tests/golden/`` which were produced by
running the reference itself in the build container (``tests/golden/make_golden.py``);
``tests/test_oracle.py`` checks it against them on CPU.

Parameters live in plain dicts keyed by the reference's ``state_dict`` names, e.g.
``model.first.conv.weight`` or ``model.resnet_backbone.3.block1.normalization.bias``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

Tensor = torch.Tensor


# ----------------------------------------------------------------------------- architecture
@dataclass
class GenConfig:
    n_resnet_blocks: int = 4
    n_updownsample_blocks: int = 2
    init_channels_out: int = 16
    is_2D: bool = False  # experiments/conf_2D.py: Conv2d / ConvTranspose2d / BatchNorm2d (blocks.py:22-27)


@dataclass
class CriticConfig:
    channels_in: int = 1
    init_channels_out: int = 8
    discriminator_depth: int = 3
    negative_slope: float = 0.2
    norm: str = "identity"  # "identity" (GP conf), "batch" (basic conf) or "layer" (gp_layernorm conf)
    is_2D: bool = False  # experiments/conf_2D.py


def gen_param_shapes(cfg: GenConfig) -> "Dict[str, tuple]":
    """state_dict layout of ResnetGenerator (generator.py:24-88)."""
    c0 = cfg.init_channels_out
    shp = {}
    K3, K7 = ((3, 3), (7, 7)) if cfg.is_2D else ((3, 3, 3), (7, 7, 7))

    def bn(prefix, c):
        shp[f"{prefix}.normalization.weight"] = (c,)
        shp[f"{prefix}.normalization.bias"] = (c,)
        shp[f"{prefix}.normalization.running_mean"] = (c,)
        shp[f"{prefix}.normalization.running_var"] = (c,)
        shp[f"{prefix}.normalization.num_batches_tracked"] = ()

    shp["model.first.conv.weight"] = (c0, 1, *K7)
    bn("model.first", c0)
    for i in range(cfg.n_updownsample_blocks):
        ci = c0 * 2**i
        shp[f"model.downsampling.{i}.conv.weight"] = (2 * ci, ci, *K3)
        bn(f"model.downsampling.{i}", 2 * ci)
    cr = c0 * 2**cfg.n_updownsample_blocks
    for r in range(cfg.n_resnet_blocks):
        for b in (0, 1):
            shp[f"model.resnet_backbone.{r}.block{b}.conv.weight"] = (cr, cr, *K3)
            bn(f"model.resnet_backbone.{r}.block{b}", cr)
    for j, i in enumerate(range(cfg.n_updownsample_blocks, 0, -1)):
        ci = c0 * 2**i
        shp[f"model.upsampling.{j}.conv.weight"] = (ci, ci // 2, *K3)  # ConvTranspose: [Cin, Cout, ...]
        bn(f"model.upsampling.{j}", ci // 2)
    shp["model.last_conv.weight"] = (1, c0, *K7)
    shp["model.last_conv.bias"] = (1,)
    return shp


def critic_param_shapes(cfg: CriticConfig) -> "Dict[str, tuple]":
    """state_dict layout of PatchGANDiscriminator (discriminator.py:19-80)."""
    c0, shp = cfg.init_channels_out, {}
    K4 = (4, 4) if cfg.is_2D else (4, 4, 4)
    shp["model.first.conv.weight"] = (c0, cfg.channels_in, *K4)
    shp["model.first.conv.bias"] = (c0,)
    out_ = c0
    for n in range(cfg.discriminator_depth):
        in_, out_ = min(2**n, 8) * c0, min(2 ** (n + 1), 8) * c0
        shp[f"model.middle.{n}.conv.weight"] = (out_, in_, *K4)
        if cfg.norm == "identity":
            shp[f"model.middle.{n}.conv.bias"] = (out_,)
        elif cfg.norm == "layer":
            pass  # conv without bias (blocks.py:34), LayerNorm without affine parameters (gp_layernorm.py:9-11)
        else:
            p = f"model.middle.{n}.normalization"
            shp[f"{p}.weight"], shp[f"{p}.bias"] = (out_,), (out_,)
            shp[f"{p}.running_mean"], shp[f"{p}.running_var"] = (out_,), (out_,)
            shp[f"{p}.num_batches_tracked"] = ()
    shp["model.last.weight"] = (1, out_, *K4)
    shp["model.last.bias"] = (1,)
    return shp


# ----------------------------------------------------------------------------- bf16 yardstick
# BF16_OPERANDS (tests only): every generator conv and the critic's middle convs take their
# operands rounded to bf16 (round-to-nearest-even) — forward (input, weight), input-grad (the
# incoming gradient, weight) and weight-grad (input, incoming gradient) — with exact accumulation,
# which is what a bf16 MFMA path with fp32 accumulation does.  Run in float64 it measures how far
# a bf16-operand reference lands from the exact step: the yardstick for the device's bf16 path
# (tests/test_gpu_configs.py).  The critic's first (1 -> 8) and last (64 -> 1) layers stay exact,
# as the device runs them in fp32.
BF16_OPERANDS = False


def _bf16(t: Tensor) -> Tensor:
    """t rounded to bf16 in the forward pass, identity gradient (straight-through)."""
    return t + (t.to(torch.bfloat16).to(t.dtype) - t).detach()


class _GradToBf16(torch.autograd.Function):
    """Identity forward; the incoming gradient is rounded to bf16 (differentiable, so the
    gradient penalty's double backward sees the same rounding)."""

    @staticmethod
    def forward(ctx, t):
        return t.view_as(t)

    @staticmethod
    def backward(ctx, g):
        return _bf16(g)


_COLS_MAX = 1 << 30


def _fft_len(n: int) -> int:
    """The smallest 5-smooth length >= n (a reflect-padded extent like 262 = 2 * 131 is ~2x slower)."""
    while True:
        m = n
        for p in (2, 3, 5):
            while m % p == 0:
                m //= p
        if m == 1:
            return n
        n += 1


def _conv3d_fft(x: Tensor, w: Tensor) -> Tensor:
    """Valid (unpadded, stride-1) cross-correlation through a float64 FFT: the circular
    convolution of x with the flipped kernel over any length L >= the input's extent equals the
    valid correlation at indices k-1 .. D-1 (no wrap reaches them).  Differentiable (torch.fft)."""
    k = w.shape[2:]
    s = x.shape[2:]
    fs = [_fft_len(v) for v in s]
    dims = tuple(range(2, x.dim()))
    X = torch.fft.rfftn(x, s=fs, dim=dims)
    Wf = torch.fft.rfftn(torch.flip(w, dims=dims), s=fs, dim=dims)
    Y = torch.einsum("nc...,oc...->no...", X, Wf)
    y = torch.fft.irfftn(Y, s=fs, dim=dims)
    return y[(slice(None), slice(None)) + tuple(slice(kk - 1, v) for kk, v in zip(k, s))]


def _conv3d_unfold(x: Tensor, w: Tensor, stride: int = 1, padding: int = 0) -> Tensor:
    """Cross-correlation as one GEMM over windows (Tensor.unfold views + einsum): the backward is
    an unfold adjoint plus GEMMs, ~15x faster than the CPU's float64 slow_conv3d backward."""
    nd = x.dim() - 2
    if padding:
        x = F.pad(x, (padding,) * (2 * nd))
    k = w.shape[2]
    u = x
    for a in range(2, 2 + nd):
        u = u.unfold(a, k, stride)  # [n, c, (do,) ho, wo, (k,) k, k]
    if nd == 2:
        return torch.einsum("nchwjk,ocjk->nohw", u, w)
    return torch.einsum("ncdhwijk,ocijk->nodhw", u, w)


def _conv3d_cpu(x: Tensor, w: Tensor, b: Optional[Tensor], **kw) -> Tensor:
    """F.conv3d.  float64 on the CPU (the exact-arithmetic stand-in, where torch's only kernel is
    the unfold-based slow_conv3d at a few GFLOP/s): the generator's k7 convs through an FFT, the
    k3 / k4 convs as one windowed GEMM — the same sums to float64 rounding.  Otherwise a stride-1
    unpadded conv whose unfolded operand (Cin k^3 x output voxels) would pass 2^30 elements runs
    over slabs of output depth (same sums)."""
    k = w.shape[2]
    if x.dtype == torch.float64 and not x.is_cuda:
        if k >= 7 and not kw:
            y = _conv3d_fft(x, w)
        else:
            y = _conv3d_unfold(x, w, kw.get("stride", 1), kw.get("padding", 0))
        return y if b is None else y + b.view(1, -1, *([1] * (x.dim() - 2)))
    if x.dim() == 4:  # the 2-D variants
        return F.conv2d(x, w, b, **kw)
    do = x.shape[2] - k + 1
    cols = w.shape[1] * k ** 3 * x.shape[0] * do * (x.shape[3] - k + 1) * (x.shape[4] - k + 1)
    if kw or x.is_cuda or cols <= _COLS_MAX:
        return F.conv3d(x, w, b, **kw)
    per = max(1, do * _COLS_MAX // cols)
    return torch.cat([F.conv3d(x[:, :, d0:min(do, d0 + per) + k - 1], w, b) for d0 in range(0, do, per)], dim=2)


def _conv3d(x: Tensor, w: Tensor, b: Optional[Tensor] = None, rounded: bool = True, **kw) -> Tensor:
    if not (BF16_OPERANDS and rounded):
        return _conv3d_cpu(x, w, b, **kw)
    return _GradToBf16.apply(_conv3d_cpu(_bf16(x), _bf16(w), b, **kw))


def _conv_transpose3d(x: Tensor, w: Tensor, **kw) -> Tensor:
    f = F.conv_transpose2d if x.dim() == 4 else F.conv_transpose3d  # 2-D variants: ConvTranspose2d
    if not BF16_OPERANDS:
        return f(x, w, **kw)
    return _GradToBf16.apply(f(_bf16(x), _bf16(w), **kw))


# ----------------------------------------------------------------------------- layers
def batch_norm(x: Tensor, p: Dict[str, Tensor], prefix: str, training: bool, momentum=0.1, eps=1e-5):
    """nn.BatchNorm3d / nn.BatchNorm2d (blocks.py:26-27,45): in train mode batch statistics over
    N·(D·)H·W (biased variance to normalise, unbiased for running_var, momentum 0.1), eval mode the
    running statistics.  torch's own batch_norm, as the reference's module calls it: its fused
    backward keeps the float32 gradients within ~1e-5 of float64, where differentiating an explicit
    (x - mean) / sqrt(var + eps) formula in float32 drifts by ~1e-3 on ill-conditioned layers."""
    if training:
        with torch.no_grad():
            p[f"{prefix}.num_batches_tracked"].add_(1)
    return F.batch_norm(x, p[f"{prefix}.running_mean"], p[f"{prefix}.running_var"], p[f"{prefix}.weight"],
                        p[f"{prefix}.bias"], training, momentum, eps)


def generator_forward(p: Dict[str, Tensor], x: Tensor, cfg: GenConfig, training=True) -> Tensor:
    """ResnetGenerator.forward (generator.py:89-90)."""
    npad = 2 * (x.dim() - 2)
    h = F.pad(x, (3,) * npad, mode="reflect")  # padding_mode="reflect", padding=3 (generator.py:19-23)
    h = F.relu(batch_norm(_conv3d(h, p["model.first.conv.weight"]), p, "model.first.normalization", training))
    for i in range(cfg.n_updownsample_blocks):
        pre = f"model.downsampling.{i}"
        h = _conv3d(h, p[f"{pre}.conv.weight"], stride=2, padding=1)
        h = F.relu(batch_norm(h, p, f"{pre}.normalization", training))
    for r in range(cfg.n_resnet_blocks):  # ResNetBlock.forward: x + block1(block0(x)) (blocks.py:87-88)
        pre = f"model.resnet_backbone.{r}"
        t = _conv3d(h, p[f"{pre}.block0.conv.weight"], padding=1)
        t = batch_norm(t, p, f"{pre}.block0.normalization", training)  # activation Identity
        t = _conv3d(t, p[f"{pre}.block1.conv.weight"], padding=1)
        t = F.relu(batch_norm(t, p, f"{pre}.block1.normalization", training))
        h = h + t
    for j in range(cfg.n_updownsample_blocks):
        pre = f"model.upsampling.{j}"
        h = _conv_transpose3d(h, p[f"{pre}.conv.weight"], stride=2, padding=1, output_padding=1)
        h = F.relu(batch_norm(h, p, f"{pre}.normalization", training))
    h = F.pad(h, (3,) * npad, mode="reflect")
    h = _conv3d(h, p["model.last_conv.weight"], p["model.last_conv.bias"])
    return torch.tanh(h)


def critic_forward(p: Dict[str, Tensor], x: Tensor, cfg: CriticConfig, training=True) -> Tensor:
    """PatchGANDiscriminator.forward (discriminator.py:83-84)."""
    s = cfg.negative_slope
    h = F.leaky_relu(_conv3d(x, p["model.first.conv.weight"], p["model.first.conv.bias"], rounded=False, stride=2,
                             padding=1), s)
    for n in range(cfg.discriminator_depth):
        pre = f"model.middle.{n}"
        if cfg.norm == "identity":
            h = _conv3d(h, p[f"{pre}.conv.weight"], p[f"{pre}.conv.bias"], stride=2, padding=1)
        elif cfg.norm == "layer":  # LayerNorm over (C, D, H, W) per sample (blocks.py:40-45, gp_layernorm.py:9-11)
            h = _conv3d(h, p[f"{pre}.conv.weight"], stride=2, padding=1)
            h = F.layer_norm(h, h.shape[1:], eps=1e-5)
        else:
            h = batch_norm(_conv3d(h, p[f"{pre}.conv.weight"], stride=2, padding=1), p, f"{pre}.normalization", training)
        h = F.leaky_relu(h, s)
    return _conv3d(h, p["model.last.weight"], p["model.last.bias"], rounded=False, stride=1, padding=1)


# ----------------------------------------------------------------------------- losses
class _StableStd(torch.autograd.Function):
    """torch.std with the reference's custom gradient (loss.py:11-29)."""

    @staticmethod
    def forward(ctx, t):
        ctx.save_for_backward(t)
        r = torch.std(t)
        ctx.r = r.detach()
        return r

    @staticmethod
    def backward(ctx, g):
        (t,) = ctx.saved_tensors
        return (2.0 / (t.numel() - 1.0)) * (g / (ctx.r * 2 + 1e-6)) * (t - t.mean())


def zncc_loss(source: Tensor, target: Tensor) -> Tensor:
    """ZNCCLoss.forward (loss.py:37-41): batch-global, not per sample."""
    cc = ((source - source.mean()) * (target - target.mean())).mean()
    std = _StableStd.apply(source) * _StableStd.apply(target)
    return -(cc / (std + 1e-8))


def hu_loss(x: Tensor, mask: Tensor, lo: float, hi: float) -> Tensor:
    """HULoss.forward (loss.py:64-71)."""
    lo_t, hi_t = torch.full_like(x, lo), torch.full_like(x, hi)
    below = (torch.minimum(x, lo_t) - lo_t).square()
    above = (torch.maximum(x, hi_t) - hi_t).square()
    return ((below + above) * mask).sum() / (mask.sum() + 1e-8)


def wasserstein(fake: Tensor, real: Optional[Tensor] = None) -> Tensor:
    """WassersteinLoss.forward (loss.py:76-80)."""
    r = fake.mean()
    return r - real.mean() if real is not None else r


def gradient_penalty(p, real, fake, eps, cfg: CriticConfig, lambda_=10.0, gp_idx=None):
    """wgan_gradient_penalty (model/utils.py:12-41) with ``eps`` [B,1,1,1,1] injected; ``gp_idx`` =
    (real rows, fake rows) of the resampling when |real| != |fake| (model/utils.py:21-25), injected."""
    if gp_idx is not None:
        real = real[torch.as_tensor(gp_idx[0], dtype=torch.long)]
        fake = fake[torch.as_tensor(gp_idx[1], dtype=torch.long)]
    interp = eps * real + (1 - eps) * fake
    if not interp.requires_grad:
        interp.requires_grad_(True)
    logits = critic_forward(p, interp, cfg)
    (g,) = torch.autograd.grad(logits, interp, torch.ones_like(logits), create_graph=True)
    return lambda_ * (g.reshape(g.shape[0], -1).norm(2, dim=-1) - 1).square().mean()


# ----------------------------------------------------------------------------- optimiser
@dataclass
class AdamState:
    lr: float
    beta1: float
    beta2: float
    eps: float = 1e-8
    step: int = 0
    exp_avg: Dict[str, Tensor] = field(default_factory=dict)
    exp_avg_sq: Dict[str, Tensor] = field(default_factory=dict)


def adam_step(params: Dict[str, Tensor], grads: Dict[str, Tensor], st: AdamState):
    """torch.optim.Adam single-tensor update (no weight decay, no amsgrad)."""
    st.step += 1
    bc1 = 1 - st.beta1**st.step
    bc2 = 1 - st.beta2**st.step
    for k, g in grads.items():
        if g is None:
            continue
        m = st.exp_avg.setdefault(k, torch.zeros_like(g))
        v = st.exp_avg_sq.setdefault(k, torch.zeros_like(g))
        m.lerp_(g, 1 - st.beta1)
        v.mul_(st.beta2).addcmul_(g, g, value=1 - st.beta2)
        denom = (v.sqrt() / math.sqrt(bc2)).add_(st.eps)
        params[k].data.addcdiv_(m, denom, value=-st.lr / bc1)


# ----------------------------------------------------------------------------- the step
@dataclass
class StepConfig:
    gen: GenConfig = field(default_factory=GenConfig)
    critic: CriticConfig = field(default_factory=CriticConfig)
    gp_weight: Optional[float] = 10.0  # None => weight clipping (basic_conf.py:37)
    weight_clip: Optional[float] = None
    hu_lo: float = 112.0 / 600.0
    hu_hi: float = 212.0 / 600.0
    hu_w: float = 1.0
    sim_w: float = 1.0
    gan_w: float = 1.0


def trainable(p: Dict[str, Tensor]) -> List[str]:
    return [k for k in p if not ("running" in k or "tracked" in k)]


def train_step(gp_: Dict[str, Tensor], dp: Dict[str, Tensor], g_opt: AdamState, d_opt: AdamState,
               opt: Tensor, subopt: Tensor, mask: Tensor, eps: Optional[Tensor], cfg: StepConfig,
               record: Optional[dict] = None, after_critic=None, gp_idx=None) -> Dict[str, float]:
    """Trainer.train_step (Trainer.py:163-203) with both updates on this iteration.

    ``gp_``/``dp``: generator / critic state dicts (modified in place: params, BN buffers).
    Returns the reference's log_dict values {"D", "G", "G-full", "sim", "HU"}.
    ``record`` (optional) receives the gradients each optimiser step consumed.
    ``after_critic`` (optional, tests) is called with the critic state dict after its update, so a
    checker can substitute the device's updated critic and compare the generator update alone
    (Adam's first steps are ~lr*sign(g), which amplifies last-bit gradient differences).
    """
    gkeys, dkeys = trainable(gp_), trainable(dp)
    for k in gkeys:
        gp_[k].requires_grad_(True)
    for k in dkeys:
        dp[k].requires_grad_(True)
    # generate (Trainer.py:170-171)
    attenuation = generator_forward(gp_, subopt, cfg.gen, training=True)
    opt_hat = subopt - attenuation
    # critic update (Trainer.py:108-142)
    real_logits = critic_forward(dp, opt, cfg.critic)
    fake_logits = critic_forward(dp, opt_hat.detach(), cfg.critic)
    loss_d = cfg.gan_w * wasserstein(fake_logits, real_logits)
    if cfg.weight_clip is None:
        # the interpolation's gradient w.r.t. the generator is identically zero;
        # the critic-parameter gradients are what the reference computes
        loss_d = loss_d + gradient_penalty(dp, opt, opt_hat.detach(), eps, cfg.critic, cfg.gp_weight, gp_idx)
    d_grads = torch.autograd.grad(loss_d, [dp[k] for k in dkeys], allow_unused=True)
    d_grads = dict(zip(dkeys, d_grads))
    if record is not None:
        record["D"] = {k: v.detach().clone() for k, v in d_grads.items() if v is not None}
    with torch.no_grad():
        adam_step(dp, d_grads, d_opt)
        if cfg.weight_clip is not None:
            for k in dkeys:
                dp[k].clamp_(-cfg.weight_clip, cfg.weight_clip)
        if after_critic is not None:
            after_critic(dp)
    # generator update (Trainer.py:144-161), with the updated critic
    loss_g = cfg.gan_w * -wasserstein(critic_forward(dp, opt_hat, cfg.critic))
    loss_sim = cfg.sim_w * zncc_loss(opt_hat, subopt)
    loss_hu = cfg.hu_w * hu_loss(opt_hat, mask, cfg.hu_lo, cfg.hu_hi)
    full = loss_g + loss_sim + loss_hu
    g_grads = torch.autograd.grad(full, [gp_[k] for k in gkeys], allow_unused=True)
    g_grads = dict(zip(gkeys, g_grads))
    if record is not None:
        record["G"] = {k: v.detach().clone() for k, v in g_grads.items() if v is not None}
    with torch.no_grad():
        adam_step(gp_, g_grads, g_opt)
    for k in gkeys:
        gp_[k].requires_grad_(False)
    for k in dkeys:
        dp[k].requires_grad_(False)
    return {"D": float(loss_d.detach()), "G": float(loss_g.detach()), "G-full": float(full.detach()), "sim": float(loss_sim.detach()),
            "HU": float(loss_hu.detach())}
