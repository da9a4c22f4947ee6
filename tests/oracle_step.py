"""Shared checker for full-step GPU tests: the HIP step engine against the CPU oracle
(``oracle/reference_torch.py``, test infrastructure) on identical synthetic inputs.

``run_vs_oracle`` drives ``iters`` steps of a ``StepEngine`` and, for every step, the same step
through the oracle in float32 (the reference's precision) and float64 (exact-arithmetic stand-in),
each iteration starting from the device's state (parameters, BatchNorm buffers, Adam moments).
The generator update is compared against an oracle that uses the device's updated critic
(``after_critic``), so the generator gradients are judged from identical inputs.  It returns the
per-tensor records; the caller states and applies its tolerance.
"""
import numpy as np
import torch

D_ARGS = dict(channels_in=1, init_channels_out=8, discriminator_depth=3, negative_slope=0.2)


def models(g_args, critic_bn=False):
    from torch import nn
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.generator import ResnetGenerator
    from cgan3d_amd.model.init import pcg64_init_
    g = pcg64_init_(ResnetGenerator(**g_args), 0).cuda()
    norm = {} if critic_bn else dict(norm_layer=nn.Identity)  # BatchNorm critic: basic_conf.py:60-66
    d = pcg64_init_(PatchGANDiscriminator(**D_ARGS, **norm), 1).cuda()
    return g, d


def step_inputs(b, S, it, seed=0):
    from cgan3d_amd.data.synthetic import synth_patches
    opt, _ = synth_patches(b, S, seed + 10 + it)
    sub, seg = synth_patches(b, S, seed + 20 + it)
    eps = np.random.Generator(np.random.PCG64(seed + 30 + it)).random((b, 1, 1, 1, 1)).astype(np.float32)
    return opt, sub, seg, eps


def rel_errors(actual, ref):
    """(max-abs error / max|ref|, L2 error / ||ref||) in float64."""
    a = np.asarray(actual, dtype=np.float64)
    e = np.asarray(ref, dtype=np.float64)
    emax, enrm = max(float(np.abs(e).max()), 1e-30), max(float(np.linalg.norm(e)), 1e-30)
    return float(np.abs(a - e).max()) / emax, float(np.linalg.norm(a - e)) / enrm


def run_vs_oracle(S, b, iters, precision="f32", g_args=None, with_fp32=True, threads=None, yard="fp32", exact=True):
    """Yield, per iteration, ``(it, losses, ref32, ref64, grads, rec32, rec64, params)``:
    device losses (engine slot layout), the oracle's float32 / float64 losses, the device gradient
    arenas {net: {name: ndarray}}, the oracle's float32 / float64 gradient records, and
    ``params`` = {net: (before, device_after, oracle64_after, grads64, yard_after)} for the post-Adam
    comparison (``yard_after``: the float32 / bf16-operand yardstick run's own post-Adam parameters).
    ``with_fp32=False`` skips the float32 oracle (``ref32`` / ``rec32`` are then None).
    ``yard="bf16"``: the yardstick run (``ref32`` / ``rec32``) is the oracle in float64 with every
    bf16-MFMA convolution's operands rounded to bf16 (``reference_torch.BF16_OPERANDS``) instead of
    the float32 oracle.  ``exact=False`` skips the exact float64 run (``ref64`` / ``rec64`` and the
    oracle's post-Adam parameters are then None)."""
    from oracle import reference_torch as R
    from cgan3d_amd.engine import StepEngine
    if threads:
        torch.set_num_threads(threads)
    g_args = g_args or dict(n_resnet_blocks=4, n_updownsample_blocks=2, init_channels_out=16)
    g, d = models(g_args)
    dbl = lambda v: v.detach().cpu().clone().double() if v.is_floating_point() else v.detach().cpu().clone()  # noqa
    gpar = {k: dbl(v) for k, v in g.state_dict().items()}
    dpar = {k: dbl(v) for k, v in d.state_dict().items()}
    eng = StepEngine(g, d, g.config, d.config, b, b, (S, S, S), g_hyper=(1e-4, 0.0, 0.9, 1e-8),
                     d_hyper=(1e-4, 0.0, 0.9, 1e-8), precision=precision)
    cfg = R.StepConfig(gen=R.GenConfig(**g_args), critic=R.CriticConfig())
    gopt, dopt = R.AdamState(1e-4, 0.0, 0.9), R.AdamState(1e-4, 0.0, 0.9)
    for it in range(iters):
        opt, sub, seg, eps = step_inputs(b, S, it)
        before = {"G": {k: v.detach().cpu().clone() for k, v in g.state_dict().items()},
                  "D": {k: v.detach().cpu().clone() for k, v in d.state_dict().items()}}
        eng.load_inputs(torch.from_numpy(opt).cuda(), torch.from_numpy(sub).cuda(), torch.from_numpy(seg).cuda(),
                        torch.from_numpy(eps).cuda())
        eng.generator_forward()
        eng.critic_update()
        d_after = {k: v.detach().cpu().clone() for k, v in d.state_dict().items()}
        eng.generator_update()

        d_oracle_after = {}

        def use_device_critic(dp):
            if not d_oracle_after:  # the first (float64 or float32) oracle's own post-Adam critic
                d_oracle_after.update({k: v.detach().clone() for k, v in dp.items()})
            for k in dp:
                dp[k].data.copy_(d_after[k])

        ref32 = rec32 = None
        if with_fp32:
            dt = torch.float64 if yard == "bf16" else torch.float32
            cp = lambda v: v.to(dt, copy=True) if v.is_floating_point() else v.clone()  # noqa: E731 (never aliases)
            g32 = {k: cp(v) for k, v in gpar.items()}
            d32 = {k: cp(v) for k, v in dpar.items()}
            o32 = R.AdamState(1e-4, 0.0, 0.9, exp_avg={k: cp(v) for k, v in gopt.exp_avg.items()},
                              exp_avg_sq={k: cp(v) for k, v in gopt.exp_avg_sq.items()}, step=gopt.step)
            od32 = R.AdamState(1e-4, 0.0, 0.9, exp_avg={k: cp(v) for k, v in dopt.exp_avg.items()},
                               exp_avg_sq={k: cp(v) for k, v in dopt.exp_avg_sq.items()}, step=dopt.step)
            rec32 = {}
            R.BF16_OPERANDS = yard == "bf16"
            try:
                ref32 = R.train_step(g32, d32, o32, od32, torch.from_numpy(opt).to(dt), torch.from_numpy(sub).to(dt),
                                     torch.from_numpy(seg), torch.from_numpy(eps).to(dt), cfg, record=rec32,
                                     after_critic=use_device_critic)
            finally:
                R.BF16_OPERANDS = False
        yard_after = {"G": {k: v.detach().clone() for k, v in g32.items()}, "D": dict(d_oracle_after)} if with_fp32 else None
        d_oracle_after.clear()
        rec64 = ref64 = None
        if exact:
            rec64 = {}
            ref64 = R.train_step(gpar, dpar, gopt, dopt, torch.from_numpy(opt).double(), torch.from_numpy(sub).double(),
                                 torch.from_numpy(seg), torch.from_numpy(eps).double(), cfg, record=rec64,
                                 after_critic=use_device_critic)
        losses = eng.losses.cpu().numpy()
        grads = {net: {k: gv.cpu().numpy() for k, gv in arena.gviews.items()}
                 for net, arena in (("G", eng.g_arena), ("D", eng.d_arena))}
        after = {"G": {k: v.detach().cpu().clone() for k, v in g.state_dict().items()},
                 "D": d_after}
        oracle_after = {"G": {k: v.detach().clone() for k, v in gpar.items()}, "D": dict(d_oracle_after)}
        params = {net: (before[net], after[net], oracle_after[net] if exact else None, rec64[net] if exact else None,
                        yard_after[net] if with_fp32 else None) for net in ("G", "D")}
        yield it, losses, ref32, ref64, grads, rec32, rec64, params
        # the next iteration starts from the device's state (params, BN buffers, Adam moments)
        for k, v in g.state_dict().items():
            gpar[k].copy_(v.detach().cpu())
        for k, v in d.state_dict().items():
            dpar[k].copy_(v.detach().cpu())
        for st, opt_ in ((gopt, eng.g_optim), (dopt, eng.d_optim)):
            for k, p in zip(opt_.arena.names, opt_.arena.params):
                st.exp_avg[k] = opt_.state[p]["exp_avg"].detach().cpu().double()
                st.exp_avg_sq[k] = opt_.state[p]["exp_avg_sq"].detach().cpu().double()


LOSS_SLOTS = (("D", 0), ("G", 3), ("sim", 4), ("HU", 5), ("G-full", 6))
