"""The standalone modules of the drop-in API on the GPU, against the reference's own fixtures and the
oracle: the losses (contrast_gan_3D/model/loss.py:11-80), the gradient penalty
(model/utils.py:12-41), the generator / critic autograd backward, and eval-mode forwards
(Trainer.validate, Trainer.py:247-308).

These are the entry points a user of the reference calls directly (outside Trainer.train_step);
inside the step engine the same arithmetic runs fused.  Tolerance: north_star's 1e-3 relative
(conftest.assert_close: max-abs error <= 1e-3 x max|ref| and relative L2 <= 1e-3).
"""
import numpy as np
import pytest
import torch

from conftest import assert_close, assert_parity

pytestmark = pytest.mark.gpu

D_ARGS = dict(channels_in=1, init_channels_out=8, discriminator_depth=3, negative_slope=0.2)


def test_zncc_hu_wasserstein_match_reference_fixture(golden):
    """ZNCCLoss (with the StableStd custom backward), HULoss and WassersteinLoss: values and input
    gradients against the reference's outputs (tests/golden/losses.npz)."""
    from cgan3d_amd.model.loss import HULoss, WassersteinLoss, ZNCCLoss
    f = golden("losses")
    s = torch.from_numpy(f["s"]).cuda().requires_grad_()
    z = ZNCCLoss()(s, torch.from_numpy(f["x"]).cuda())
    (gs,) = torch.autograd.grad(z, s)
    assert_close(z.detach().cpu().numpy(), f["zncc"], 1e-3, "zncc")
    assert_close(gs.cpu().numpy(), f["zncc_grad"], 1e-3, "zncc grad")
    h = torch.from_numpy(f["x"]).cuda().requires_grad_()
    hu = HULoss(float(f["hu_lo"]), float(f["hu_hi"]), tuple(f["x"].shape))(h, torch.from_numpy(f["seg"]).cuda())
    (gh,) = torch.autograd.grad(hu, h)
    assert_close(hu.detach().cpu().numpy(), f["hu"], 1e-3, "HU")
    assert_close(gh.cpu().numpy(), f["hu_grad"], 1e-3, "HU grad")
    fk = torch.from_numpy(f["w_fake"]).cuda().requires_grad_()
    rl = torch.from_numpy(f["w_real"]).cuda().requires_grad_()
    w2 = WassersteinLoss()(fk, rl)
    gf, gr = torch.autograd.grad(w2, (fk, rl))
    assert_close(w2.detach().cpu().numpy(), f["w2"], 1e-6, "W2")
    n = fk.numel()
    assert_close(gf.cpu().numpy(), np.full(fk.shape, 1.0 / n, np.float32), 1e-6, "dW2/dfake")
    assert_close(gr.cpu().numpy(), np.full(rl.shape, -1.0 / n, np.float32), 1e-6, "dW2/dreal")
    assert_close(WassersteinLoss()(fk.detach()).cpu().numpy(), f["w1"], 1e-6, "W1")


def test_gradient_penalty_matches_reference_fixture(golden):
    """wgan_gradient_penalty with the reference's eps (injected): the penalty and the critic's
    parameter gradients of its backward (the reference's create_graph double backward) against
    tests/golden/gp.npz."""
    from torch import nn
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.init import pcg64_init_
    from cgan3d_amd.model.utils import wgan_gradient_penalty
    f = golden("gp")
    d = pcg64_init_(PatchGANDiscriminator(**D_ARGS, norm_layer=nn.Identity), 1).cuda()
    gp = wgan_gradient_penalty(torch.from_numpy(f["real"]).cuda(), torch.from_numpy(f["fake"]).cuda(), d,
                               device="cuda", lambda_=10, eps=torch.from_numpy(f["eps"]).cuda())
    gp.backward()
    assert_close(gp.detach().cpu().numpy(), f["gp"], 1e-3, "GP")
    wmax = float(np.abs(f["grad/model.first.conv.weight"]).max())
    for name, p in d.named_parameters():
        key = f"grad/{name}"
        if key in f:
            # the penalty's bias gradients are exactly zero in real arithmetic (LeakyReLU masks are
            # piecewise constant); the reference's double backward leaves rounding-level values
            atol = 1e-6 * wmax if name.endswith("bias") else 0.0
            assert_close(p.grad.cpu().numpy(), f[key], 1e-3, key, atol=atol)


def _oracle_params(module):
    return {k: v.detach().cpu().clone().double() if v.is_floating_point() else v.detach().cpu().clone()
            for k, v in module.state_dict().items()}


def test_generator_autograd_backward_matches_oracle():
    """ResnetGenerator used as a plain module (forward + loss.backward(), as a user outside the
    Trainer would): parameter gradients against the oracle's autograd in float64, with its float32
    run as the yardstick of the BatchNorm-amplified tensors (conftest.assert_parity)."""
    from oracle import reference_torch as R
    from cgan3d_amd.data.synthetic import synth_patches
    from cgan3d_amd.model.generator import ResnetGenerator
    from cgan3d_amd.model.init import pcg64_init_
    # (the 16-channel generator at 32^3 B=2 is ill-conditioned under this random loss: the reference's own
    # float32 weight gradients deviate from float64 by ~1e-2 there; this width is conditioned to ~5e-6)
    g_args = dict(n_resnet_blocks=1, n_updownsample_blocks=2, init_channels_out=8)
    g = pcg64_init_(ResnetGenerator(**g_args), 0).cuda().train()
    par = _oracle_params(g)
    x, _ = synth_patches(2, 32, 5)
    r = np.random.Generator(np.random.PCG64(6)).standard_normal(x.shape).astype(np.float32)
    y = g(torch.from_numpy(x).cuda())
    (y * torch.from_numpy(r).cuda()).sum().backward()
    keys = [k for k, _ in g.named_parameters()]
    # the oracle in float64 (exact stand-in) and float32 (the reference's precision: the yardstick for
    # the BatchNorm-amplified weight gradients, conftest.assert_parity)
    res = {}
    for dt in (torch.float64, torch.float32):
        pp = {k: (v.to(dt).detach().requires_grad_(k in keys) if v.is_floating_point() else v.clone())
              for k, v in par.items()}
        yr = R.generator_forward(pp, torch.from_numpy(x).to(dt), R.GenConfig(**g_args), training=True)
        res[dt] = (yr.detach(), torch.autograd.grad((yr * torch.from_numpy(r).to(dt)).sum(), [pp[k] for k in keys]))
    assert_close(y.detach().cpu().numpy(), res[torch.float64][0].numpy(), 1e-3, "G(x)")
    for i, (k, p) in enumerate(g.named_parameters()):
        assert_parity(p.grad.cpu().numpy(), res[torch.float32][1][i].numpy(), res[torch.float64][1][i].numpy(),
                      f"dG/d{k}")


@pytest.mark.parametrize("norm", ["identity", "layer"])
def test_critic_autograd_backward_matches_oracle(norm):
    """PatchGANDiscriminator (GP conf; gp_layernorm conf's LayerNorm critic) as a plain module:
    input and parameter gradients of sum(D(x) * r) against the oracle's autograd in float64."""
    from torch import nn
    from oracle import reference_torch as R
    from cgan3d_amd.data.synthetic import synth_patches
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.init import pcg64_init_
    kw = dict(norm_layer=nn.Identity)
    if norm == "layer":  # experiments/gp_layernorm.py:9-11
        kw = dict(norm_layer=nn.LayerNorm, patch_size=(1, 32, 32, 32), elementwise_affine=False)
    d = pcg64_init_(PatchGANDiscriminator(**D_ARGS, **kw), 1).cuda()
    par = _oracle_params(d)
    x, _ = synth_patches(3, 32, 7)
    xd = torch.from_numpy(x).cuda().requires_grad_()
    y = d(xd)
    r = np.random.Generator(np.random.PCG64(8)).standard_normal(tuple(y.shape)).astype(np.float32)
    (y * torch.from_numpy(r).cuda()).sum().backward()
    keys = [k for k, _ in d.named_parameters()]
    for k in keys:
        par[k].requires_grad_(True)
    xr = torch.from_numpy(x).double().requires_grad_()
    yr = R.critic_forward(par, xr, R.CriticConfig(norm=norm))
    assert_close(y.detach().cpu().numpy(), yr.detach().numpy(), 1e-3, "D(x)")
    grads = torch.autograd.grad((yr * torch.from_numpy(r).double()).sum(), [xr] + [par[k] for k in keys])
    assert_close(xd.grad.cpu().numpy(), grads[0].numpy(), 1e-3, "dD/dx")
    for (k, p), gr in zip(d.named_parameters(), grads[1:]):
        assert_close(p.grad.cpu().numpy(), gr.numpy(), 1e-3, f"dD/d{k}")


def test_reference_style_gradient_penalty_double_backward():
    """The reference's own penalty code path over the HIP critic (model/utils.py:26-41: interpolate,
    torch.autograd.grad(D(x_hat), x_hat, ones, create_graph=True), lambda * mean((||g|| - 1)^2),
    then backward): critic parameter gradients against the same code over the oracle's float64
    critic.  Biases get no penalty gradient (exactly 0 in real arithmetic, atol 1e-9)."""
    from torch import nn
    from oracle import reference_torch as R
    from cgan3d_amd.data.synthetic import synth_patches
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.init import pcg64_init_

    def penalty(critic_fn, real, fake, eps):
        xh = (eps * real + (1 - eps) * fake).requires_grad_(True)
        out = critic_fn(xh)
        g = torch.autograd.grad(outputs=out, inputs=xh, grad_outputs=torch.ones_like(out), create_graph=True,
                                retain_graph=True)[0]
        return 10.0 * ((g.flatten(1).norm(2, dim=1) - 1) ** 2).mean()

    d = pcg64_init_(PatchGANDiscriminator(**D_ARGS, norm_layer=nn.Identity), 1).cuda()
    par = _oracle_params(d)
    real, _ = synth_patches(2, 32, 21)
    fake, _ = synth_patches(2, 32, 22)
    eps = np.array([0.3, 0.8], dtype=np.float32).reshape(2, 1, 1, 1, 1)
    gp = penalty(d, *(torch.from_numpy(a).cuda() for a in (real, fake, eps)))
    gp.backward()
    keys = [k for k, _ in d.named_parameters()]
    for k in keys:
        par[k].requires_grad_(True)
    gpr = penalty(lambda x: R.critic_forward(par, x, R.CriticConfig(norm="identity")),
                  *(torch.from_numpy(a).double() for a in (real, fake, eps)))
    grads = torch.autograd.grad(gpr, [par[k] for k in keys], allow_unused=True)  # (the last bias is unused)
    grads = [torch.zeros_like(par[k]) if gr is None else gr for k, gr in zip(keys, grads)]
    assert_close(float(gp.detach()), float(gpr.detach()), 1e-3, "GP value")
    for (k, p), gr in zip(d.named_parameters(), grads):
        assert_close(p.grad.cpu().numpy(), gr.numpy(), 1e-3, f"dGP/d{k}", atol=1e-9 if k.endswith("bias") else 0.0)


def _random_running_stats(module, rng):
    with torch.no_grad():
        for k, b in module.named_buffers():
            if k.endswith("running_mean"):
                b.copy_(torch.from_numpy(rng.normal(0.0, 0.3, b.shape).astype(np.float32)))
            elif k.endswith("running_var"):
                b.copy_(torch.from_numpy(rng.uniform(0.5, 2.0, b.shape).astype(np.float32)))


def test_eval_mode_forwards_match_oracle():
    """Eval-mode (running-statistics) BatchNorm forwards, as Trainer.validate runs them
    (Trainer.py:248-249): the generator with non-trivial running buffers and the BatchNorm critic
    of the weight-clip conf, against the oracle with training=False."""
    from oracle import reference_torch as R
    from cgan3d_amd.data.synthetic import synth_patches
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.generator import ResnetGenerator
    from cgan3d_amd.model.init import pcg64_init_
    g_args = dict(n_resnet_blocks=4, n_updownsample_blocks=2, init_channels_out=16)
    rng = np.random.Generator(np.random.PCG64(11))
    g = pcg64_init_(ResnetGenerator(**g_args), 0).cuda()
    _random_running_stats(g, rng)
    g.eval()
    x, _ = synth_patches(2, 32, 12)
    with torch.no_grad():
        y = g(torch.from_numpy(x).cuda())
    yr = R.generator_forward(_oracle_params(g), torch.from_numpy(x).double(), R.GenConfig(**g_args), training=False)
    assert_close(y.cpu().numpy(), yr.numpy(), 1e-3, "G_eval(x)")
    d = pcg64_init_(PatchGANDiscriminator(**D_ARGS), 1).cuda()
    _random_running_stats(d, rng)
    d.eval()
    with torch.no_grad():
        yd = d(torch.from_numpy(x).cuda())
    ydr = R.critic_forward(_oracle_params(d), torch.from_numpy(x).double(), R.CriticConfig(norm="batch"),
                           training=False)
    assert_close(yd.cpu().numpy(), ydr.numpy(), 1e-3, "D_eval(x)")


def test_critic_module_reuses_its_plan():
    """A no-grad critic forward on the same shape reuses one CriticPlan (buffers allocated once)
    and still sees weight updates (the packed copies are refreshed per call)."""
    from torch import nn
    from cgan3d_amd.data.synthetic import synth_patches
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.init import pcg64_init_
    d = pcg64_init_(PatchGANDiscriminator(**D_ARGS, norm_layer=nn.Identity), 1).cuda()
    x = torch.from_numpy(synth_patches(2, 32, 3)[0]).cuda()
    with torch.no_grad():
        y1 = d(x)
        p1 = d.plan_for(2, (32, 32, 32))
        y2 = d(x)
        assert d.plan_for(2, (32, 32, 32)) is p1
        torch.testing.assert_close(y1, y2, rtol=0, atol=0)
        for p in d.parameters():
            p.mul_(1.5)
        y3 = d(x)
    assert not torch.allclose(y3, y1)
