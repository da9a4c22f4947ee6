"""Generate the parity fixtures in tests/golden/ by running the REFERENCE implementation.

Run in the build container only (needs /root/reference; nothing here runs on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference (xqz-u/contrast-gan-3D @ 2024-08-07) is pure Python on torch; it is imported
read-only with stubs for the absent third-party modules it names only for typing
(``batchgenerators``, used at ``contrast_gan_3D/alias.py:7-21``), for
``trainer/utils.py`` (whose import chain reaches Python-3.11-only syntax in
``data/CCTADataLoader.py:69``) and for the wandb logger.  Nothing of the
reference is copied: only inputs and outputs are written, as .npz fixtures.

Fixtures (all fp32, CPU, torch as installed here — recorded in each file's ``torch_version``):
  g_fwd_*.npz     ResnetGenerator forward (train-mode BN) + running stats
  d_fwd_*.npz     PatchGANDiscriminator forward (GP conf: Identity norm; BN conf)
  losses.npz      ZNCCLoss / HULoss / WassersteinLoss values and input gradients
  gp.npz          wgan_gradient_penalty value + critic parameter gradients (eps injected)
  step_*.npz      Trainer.train_step over 1-3 iterations (GP conf, weight-clip conf, and the
                  gp_layernorm conf's LayerNorm critic with the GP):
                  losses, gradients seen by each optimizer step, final params & buffers; per
                  iteration the entering state and a float64 re-run of that iteration
"""
from __future__ import annotations

import contextlib
import os
import sys
import types
from functools import partial
from pathlib import Path

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True

import numpy as np
import torch

REF = "/root/reference"
HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO / "contrast-gan-3d_amd"))
sys.path.insert(0, REF)

from cgan3d_amd.data.synthetic import scaled_hu_bounds, synth_patches  # noqa: E402
from cgan3d_amd.model.init import pcg64_init_  # noqa: E402


def _install_stubs():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    class _Dummy:  # typing-only placeholders
        def __init__(self, *a, **k):
            pass

    mod("batchgenerators")
    mod("batchgenerators.dataloading")
    mod("batchgenerators.dataloading.multi_threaded_augmenter", MultiThreadedAugmenter=_Dummy)
    mod("batchgenerators.dataloading.nondet_multi_threaded_augmenter",
        NonDetMultiThreadedAugmenter=_Dummy)
    mod("batchgenerators.dataloading.single_threaded_augmenter", SingleThreadedAugmenter=_Dummy)
    import contrast_gan_3D.trainer  # noqa: F401  (package __init__ is empty)
    mod("contrast_gan_3D.trainer.utils", find_latest_checkpoint=lambda d: None)
    mod("contrast_gan_3D.trainer.logger")
    mod("contrast_gan_3D.trainer.logger.LoggerInterface",
        SingleThreadedLogger=_Dummy, MultiThreadedLogger=_Dummy)


_install_stubs()
from contrast_gan_3D.model.discriminator import PatchGANDiscriminator  # noqa: E402
from contrast_gan_3D.model.generator import ResnetGenerator  # noqa: E402
from contrast_gan_3D.model import loss as ref_loss  # noqa: E402
from contrast_gan_3D.model import utils as ref_utils  # noqa: E402
from contrast_gan_3D.trainer.Trainer import Trainer  # noqa: E402

G_ARGS = dict(n_resnet_blocks=4, n_updownsample_blocks=2, init_channels_out=16)  # basic_conf.py:49-53
G_SMALL = dict(n_resnet_blocks=1, n_updownsample_blocks=2, init_channels_out=8)
D_ARGS = dict(channels_in=1, init_channels_out=8, discriminator_depth=3, negative_slope=0.2)  # :60-65


@contextlib.contextmanager
def injected_rand(values):
    """Make ``torch.rand`` inside wgan_gradient_penalty (model/utils.py:26) return ``values``."""
    orig = torch.rand
    queue = list(values)

    def fake_rand(size, *a, **k):
        v = queue.pop(0)
        assert tuple(v.shape) == tuple(size), (v.shape, size)
        return v.clone()

    torch.rand = fake_rand
    try:
        yield
    finally:
        torch.rand = orig


def sd_np(module, prefix):
    return {f"{prefix}{k}": v.detach().cpu().numpy().copy() for k, v in module.state_dict().items()}


def gen_forward(S, B, seed):
    g = pcg64_init_(ResnetGenerator(**G_ARGS), 0)
    x, _ = synth_patches(B, S, seed)
    g.train()
    with torch.no_grad():
        y = g(torch.from_numpy(x))
    out = {"x": x, "y": y.numpy()}
    # weights are regenerated from the PCG64 recipe; keep only the BN buffers the step updates
    out.update({k: v for k, v in sd_np(g, "sd/").items() if "running" in k or "tracked" in k})
    np.savez_compressed(HERE / f"g_fwd_{S}.npz", torch_version=torch.__version__, **out)


def disc_forward(S, B, seed):
    out = {}
    x, _ = synth_patches(B, S, seed)
    out["x"] = x
    for tag, extra in (("gp", dict(norm_layer=torch.nn.Identity)), ("bn", {})):
        d = pcg64_init_(PatchGANDiscriminator(**D_ARGS, **extra), 1)
        d.train()
        with torch.no_grad():
            out[f"{tag}/y"] = d(torch.from_numpy(x)).numpy()
        out.update({k: v for k, v in sd_np(d, f"{tag}/sd/").items() if "running" in k})
    np.savez_compressed(HERE / f"d_fwd_{S}.npz", torch_version=torch.__version__, **out)


def losses(S, B, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    x, seg = synth_patches(B, S, seed)
    s = torch.from_numpy(x + 0.1 * rng.standard_normal(x.shape).astype(np.float32)).requires_grad_()
    t = torch.from_numpy(x)
    zncc = ref_loss.ZNCCLoss()(s, t)
    (gs,) = torch.autograd.grad(zncc, s)
    lo, hi = scaled_hu_bounds()
    h = torch.from_numpy(x).requires_grad_()
    hu = ref_loss.HULoss(lo, hi, tuple(x.shape))(h, torch.from_numpy(seg))
    (gh,) = torch.autograd.grad(hu, h)
    f = torch.from_numpy(rng.standard_normal((B, 1, 3, 3, 3)).astype(np.float32))
    r = torch.from_numpy(rng.standard_normal((B, 1, 3, 3, 3)).astype(np.float32))
    w2 = ref_loss.WassersteinLoss()(f, r)
    w1 = ref_loss.WassersteinLoss()(f)
    np.savez_compressed(
        HERE / "losses.npz", torch_version=torch.__version__,
        x=x, seg=seg, s=s.detach().numpy(), zncc=zncc.detach().numpy(), zncc_grad=gs.numpy(),
        hu=hu.detach().numpy(), hu_grad=gh.numpy(), hu_lo=np.float32(lo), hu_hi=np.float32(hi),
        w_fake=f.numpy(), w_real=r.numpy(), w2=w2.numpy(), w1=w1.numpy())


def gradient_penalty(S, B, seed):
    d = pcg64_init_(PatchGANDiscriminator(**D_ARGS, norm_layer=torch.nn.Identity), 1)
    real, _ = synth_patches(B, S, seed)
    fake, _ = synth_patches(B, S, seed + 1)
    fake = 0.5 * fake
    eps = torch.from_numpy(np.random.Generator(np.random.PCG64(seed + 2)).random((B, 1, 1, 1, 1)).astype(np.float32))
    d.zero_grad(set_to_none=True)
    # as in train_critic (Trainer.py:123-130) the fake batch is the generator output, which
    # requires grad; interpolation then requires grad and autograd.grad accepts it
    fake_t = torch.from_numpy(fake).requires_grad_()
    with injected_rand([eps]):
        gp = ref_utils.wgan_gradient_penalty(torch.from_numpy(real), fake_t, d,
                                             device="cpu", lambda_=10)
    gp.backward()
    out = {f"grad/{n}": p.grad.numpy() for n, p in d.named_parameters() if p.grad is not None}
    out["fake_grad_absmax"] = np.float32(fake_t.grad.abs().max())  # the dead path: exactly 0
    np.savez_compressed(HERE / "gp.npz", torch_version=torch.__version__, real=real, fake=fake,
                        eps=eps.numpy(), gp=gp.detach().numpy(), **out)


class _NullLogger:
    class logger:  # noqa: N801  (mirrors logger_interface.logger.log_loss)
        @staticmethod
        def log_loss(*a, **k):
            pass

    def __call__(self, *a, **k):
        pass

    def end_hook(self):
        pass


def _make_trainer(g_args, gp: bool, S, b_low, b_high, iters, dtype, critic_norm="identity", d_args=None):
    """A reference Trainer for the fixture runs; ``dtype=torch.float64`` converts the modules, the
    optimisers and the HU constants to double (the exact-arithmetic yardstick).  ``critic_norm``
    "layer": the gp_layernorm conf's critic (experiments/gp_layernorm.py:9-11: LayerNorm over
    (C, D, H, W) of every middle block, no affine parameters)."""
    shape = tuple(S) if isinstance(S, (tuple, list)) else (S, S, S)
    d_extra = dict(norm_layer=torch.nn.Identity) if gp else {}
    if critic_norm == "layer":
        d_extra = dict(norm_layer=torch.nn.LayerNorm, patch_size=(1, *shape), elementwise_affine=False)
    lr, betas = (1e-4, (0.0, 0.9)) if gp else (2e-4, (0.5, 0.999))
    lo, hi = scaled_hu_bounds()
    tr = Trainer(
        train_iterations=iters, val_iterations=1, validate_every=None,
        train_generator_every=1, train_critic_every=1, log_every=10**9, log_images_every=10**9,
        generator_class=partial(ResnetGenerator, **g_args),
        critic_class=partial(PatchGANDiscriminator, **(d_args or D_ARGS), **d_extra),
        generator_optim_class=partial(torch.optim.Adam, lr=lr, betas=betas),
        critic_optim_class=partial(torch.optim.Adam, lr=lr, betas=betas),
        hu_loss_instance=ref_loss.HULoss(lo, hi, (b_low + b_high, 1, *shape)),
        logger_interface=_NullLogger(), device=torch.device("cpu"), checkpoint_dir=None,
        weight_clip=None if gp else 0.01, checkpoint_every=None)
    pcg64_init_(tr.generator, 0)
    pcg64_init_(tr.critic, 1)
    if dtype != torch.float32:
        tr.generator.to(dtype)
        tr.critic.to(dtype)
        tr.optimizer_G = partial(torch.optim.Adam, lr=lr, betas=betas)(tr.generator.parameters())
        tr.optimizer_D = partial(torch.optim.Adam, lr=lr, betas=betas)(tr.critic.parameters())
        tr.loss_HU.min_HU = tr.loss_HU.min_HU.to(dtype)  # loss.py:51-56 constants
        tr.loss_HU.max_HU = tr.loss_HU.max_HU.to(dtype)
    tr.generator.train()
    tr.critic.train()
    return tr, lr, betas


def _snapshot(tr):
    """Everything the next iteration depends on: both state_dicts (parameters + BatchNorm buffers)
    and both Adam states (deep copies)."""
    import copy
    return {"G": copy.deepcopy(tr.generator.state_dict()), "D": copy.deepcopy(tr.critic.state_dict()),
            "optG": copy.deepcopy(tr.optimizer_G.state_dict()), "optD": copy.deepcopy(tr.optimizer_D.state_dict())}


def _restore(tr, snap):
    tr.generator.load_state_dict(snap["G"])
    tr.critic.load_state_dict(snap["D"])
    tr.optimizer_G.load_state_dict(snap["optG"])  # moments cast to the parameters' dtype by torch
    tr.optimizer_D.load_state_dict(snap["optD"])


def _state_arrays(tr, snap, it):
    """Fixture entries of the state entering iteration ``it``: the GPU test loads it, so every
    iteration's gradients are checked from the reference's own state (not from a state the device
    reached by itself, which differs by Adam's sign flips of sub-noise gradient elements)."""
    out = {}
    for net, mod, optk in (("G", tr.generator, "optG"), ("D", tr.critic, "optD")):
        for k, v in snap[net].items():
            out[f"it{it}/state/{net}/{k}"] = v.detach().cpu().numpy().copy()
        st = snap[optk]["state"]
        for idx, (n, _) in enumerate(mod.named_parameters()):
            if idx in st:
                out[f"it{it}/adam/{net}/{n}/exp_avg"] = st[idx]["exp_avg"].detach().cpu().numpy().copy()
                out[f"it{it}/adam/{net}/{n}/exp_avg_sq"] = st[idx]["exp_avg_sq"].detach().cpu().numpy().copy()
                out[f"it{it}/adam/{net}/step"] = np.float32(float(st[idx]["step"]))
    return out


def _run_iteration(tr, gp, inputs, it, dtype):
    """One Trainer.train_step on ``inputs``; returns (logged losses, {"G": grads, "D": grads}) with
    the gradients each optimiser step consumed."""
    opt, low, low_seg, high, high_seg, eps = inputs
    grads = {}

    def snap(optim, model, key):
        orig = optim.step

        def step(*a, **k):
            grads[key] = {n: p.grad.detach().clone().numpy() for n, p in model.named_parameters()
                          if p.grad is not None}
            return orig(*a, **k)
        optim.step = step
        return orig

    og = snap(tr.optimizer_G, tr.generator, "G")
    od = snap(tr.optimizer_D, tr.critic, "D")
    patches = [{"data": torch.from_numpy(opt).to(dtype)},
               {"data": torch.from_numpy(low).to(dtype), "seg": torch.from_numpy(low_seg)},
               {"data": torch.from_numpy(high).to(dtype), "seg": torch.from_numpy(high_seg)}]
    logged = {}
    orig_c, orig_g = tr.train_critic, tr.train_generator

    def tc(*a, **k):
        r = orig_c(*a, **k)
        logged.update(r)
        return r

    def tg(*a, **k):
        r = orig_g(*a, **k)
        logged.update(r)
        return r
    tr.train_critic, tr.train_generator = tc, tg
    ctx = injected_rand([torch.from_numpy(eps).to(dtype)]) if gp else contextlib.nullcontext()
    with ctx:
        tr.train_step(patches, it)
    tr.train_critic, tr.train_generator = orig_c, orig_g
    tr.optimizer_G.step, tr.optimizer_D.step = og, od
    return {k: v.detach().numpy() for k, v in logged.items()}, grads


def _patches(n, shape, seed):
    """synth_patches of a 3-D shape, or of a 2-D (H, W) shape as [n, 1, H, W]."""
    if len(shape) == 2:
        x, m = synth_patches(n, (1, *shape), seed)
        return x[:, :, 0], m[:, :, 0]
    return synth_patches(n, shape, seed)


def train_steps(tag, g_args, gp: bool, S, b_opt, b_low, b_high, iters, seed, save_final_g=True,
                critic_norm="identity", d_args=None):
    """Trainer.train_step (Trainer.py:163-203) with train_{critic,generator}_every = 1, ``iters``
    iterations in float32 (the reference's precision).

    For every iteration the fixture also holds the state entering it (``it{k}/state``,
    ``it{k}/adam``, k > 0) and the same iteration re-run in float64 from that state
    (``it{k}/grad64``, ``it{k}/loss64``): the exact-arithmetic yardstick the GPU test holds each
    iteration to."""
    shape = tuple(S) if isinstance(S, (tuple, list)) else (S, S, S)
    tr, lr, betas = _make_trainer(g_args, gp, shape, b_low, b_high, iters, torch.float32, critic_norm, d_args)
    out = {}
    rngs = np.random.Generator(np.random.PCG64(seed + 100))
    for it in range(iters):
        opt, _ = _patches(b_opt, shape, seed + 10 * it)
        low, low_seg = _patches(b_low, shape, seed + 10 * it + 1)
        high, high_seg = _patches(b_high, shape, seed + 10 * it + 2)
        low = low - 0.3  # hypo-enhanced (LOW) / hyper-enhanced (HIGH) flavour
        high = high + 0.3
        eps = rngs.random((min(b_opt, b_low + b_high),) + (1,) * (len(shape) + 1)).astype(np.float32)
        inputs = (opt, low, low_seg, high, high_seg, eps)
        snap = _snapshot(tr)
        if it > 0:
            out.update(_state_arrays(tr, snap, it))
        losses, grads = _run_iteration(tr, gp, inputs, it, torch.float32)
        # the same iteration in float64 from the same state
        tr64, _, _ = _make_trainer(g_args, gp, shape, b_low, b_high, iters, torch.float64, critic_norm, d_args)
        _restore(tr64, snap)
        losses64, grads64 = _run_iteration(tr64, gp, inputs, it, torch.float64)
        out[f"it{it}/opt"] = opt
        out[f"it{it}/low"] = low
        out[f"it{it}/high"] = high
        out[f"it{it}/low_seg"] = low_seg
        out[f"it{it}/high_seg"] = high_seg
        out[f"it{it}/eps"] = eps
        for k, v in losses.items():
            out[f"it{it}/loss/{k}"] = v
            out[f"it{it}/loss64/{k}"] = np.asarray(losses64[k], dtype=np.float32)
        for key in ("G", "D"):
            for n, g in grads[key].items():
                out[f"it{it}/grad/{key}/{n}"] = g
                out[f"it{it}/grad64/{key}/{n}"] = np.asarray(grads64[key][n], dtype=np.float32)
    if save_final_g:
        out.update(sd_np(tr.generator, "final/G/"))
    out.update(sd_np(tr.critic, "final/D/"))
    meta = dict(S=shape[0] if len(set(shape)) == 1 and len(shape) == 3 else None, shape=shape, b_opt=b_opt,
                b_low=b_low, b_high=b_high, iters=iters, gp=int(gp), lr=lr, critic_norm=critic_norm,
                beta1=betas[0], beta2=betas[1], teacher_forced=1,
                d_init_channels_out=(d_args or D_ARGS)["init_channels_out"],
                **{f"g_{k}": v for k, v in g_args.items()})
    np.savez_compressed(HERE / f"step_{tag}.npz", torch_version=torch.__version__,
                        meta=np.array(repr(meta)), **out)


def clip_2d():
    """experiments/conf_2D.py: the 2-D variants on top of basic_conf (weight clip 0.01, BatchNorm
    critic, Adam lr 2e-4 betas (0.5, 0.999)) — generator with 6 ResNet blocks (is_2D), critic with
    16 initial channels (16 -> 32 -> 64 -> 128), at 32 x 32 (the 2-D conf trains 128 x 128).  The
    generator's width is halved (8 initial channels) to keep the fixture small; the full conf_2D
    widths run against the oracle in tests/test_gpu_2d.py."""
    g2 = dict(n_resnet_blocks=6, n_updownsample_blocks=2, init_channels_out=8, is_2D=True)
    d2 = dict(channels_in=1, init_channels_out=16, discriminator_depth=3, negative_slope=0.2, is_2D=True)
    train_steps("clip_2d", g2, False, S=(32, 32), b_opt=2, b_low=1, b_high=1, iters=2, seed=900, d_args=d2)


def ln_aniso():
    """gp_layernorm conf on an anisotropic patch (experiments/small_patch_size.py:4 trains
    128 x 128 x 32 with it; here 32 x 40 x 48, every axis >= 32 for the critic's k4 pyramid)."""
    train_steps("ln_aniso", G_SMALL, True, S=(32, 40, 48), b_opt=2, b_low=1, b_high=1, iters=2, seed=1000,
                critic_norm="layer")


if __name__ == "__main__":
    torch.set_num_threads(8)
    torch.use_deterministic_algorithms(True)
    only = sys.argv[1:]  # optional fixture tags to (re)generate, e.g. gp_layernorm
    if only:
        if "gp_layernorm" in only:
            train_steps("gp_layernorm", G_SMALL, True, S=32, b_opt=2, b_low=1, b_high=1, iters=2, seed=800,
                        critic_norm="layer")
        if "clip_2d" in only:
            clip_2d()
        if "ln_aniso" in only:
            ln_aniso()
        sys.exit(0)
    gen_forward(32, 2, seed=1234)
    disc_forward(32, 3, seed=1234)
    losses(32, 2, seed=77)
    gradient_penalty(32, 2, seed=99)
    # the critic's k4/s2 pyramid needs S >= 32 (4 halvings, then a k4 s1 p1 layer)
    train_steps("gp_small", G_SMALL, True, S=32, b_opt=2, b_low=1, b_high=1, iters=3, seed=500)
    train_steps("gp_full", G_ARGS, True, S=32, b_opt=2, b_low=1, b_high=1, iters=1, seed=600,
                save_final_g=False)
    train_steps("clip_small", G_SMALL, False, S=32, b_opt=2, b_low=1, b_high=1, iters=2, seed=700)
    # gp_layernorm conf (experiments/gp_layernorm.py): LayerNorm critic with the gradient penalty
    train_steps("gp_layernorm", G_SMALL, True, S=32, b_opt=2, b_low=1, b_high=1, iters=2, seed=800,
                critic_norm="layer")
    clip_2d()
    ln_aniso()
    for f in sorted(HERE.glob("*.npz")):
        print(f.name, f.stat().st_size)
