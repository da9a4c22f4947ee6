"""Pin the oracle (oracle/reference_torch.py) to the reference's own outputs (tests/golden/).

CPU only.  The fixtures were produced by running xqz-u/contrast-gan-3D itself
(tests/golden/make_golden.py); the oracle is a from-scratch restatement, so agreement here is
what makes the oracle a trustworthy checker for the HIP path.
"""
import ast

import numpy as np
import pytest
import torch

from conftest import assert_close, assert_parity
from oracle import reference_torch as R
from cgan3d_amd.model.init import pcg64_state_dict

GEN = R.GenConfig()
GEN_SMALL = R.GenConfig(n_resnet_blocks=1, n_updownsample_blocks=2, init_channels_out=8)


def params(shapes, seed):
    sd = pcg64_state_dict(list(shapes.items()), seed)
    return {k: torch.from_numpy(v.copy()) for k, v in sd.items()}


def test_generator_forward(golden):
    f = golden("g_fwd_32")
    p = params(R.gen_param_shapes(GEN), 0)
    with torch.no_grad():
        y = R.generator_forward(p, torch.from_numpy(f["x"]), GEN, training=True)
    assert_close(y.numpy(), f["y"], 1e-4, "G(x)")
    for k in p:
        if "running" in k or "tracked" in k:
            assert_close(p[k].numpy(), f[f"sd/{k}"], 1e-4, k)


@pytest.mark.parametrize("tag", ["gp", "bn"])
def test_critic_forward(golden, tag):
    f = golden("d_fwd_32")
    cfg = R.CriticConfig(norm="identity" if tag == "gp" else "batch")
    p = params(R.critic_param_shapes(cfg), 1)
    with torch.no_grad():
        y = R.critic_forward(p, torch.from_numpy(f["x"]), cfg)
    assert_close(y.numpy(), f[f"{tag}/y"], 1e-4, "D(x)")


def test_losses(golden):
    f = golden("losses")
    s = torch.from_numpy(f["s"]).requires_grad_()
    z = R.zncc_loss(s, torch.from_numpy(f["x"]))
    (gs,) = torch.autograd.grad(z, s)
    assert_close(z.detach().numpy(), f["zncc"], 1e-5, "zncc")
    assert_close(gs.numpy(), f["zncc_grad"], 1e-4, "zncc grad")
    h = torch.from_numpy(f["x"]).requires_grad_()
    hu = R.hu_loss(h, torch.from_numpy(f["seg"]), float(f["hu_lo"]), float(f["hu_hi"]))
    (gh,) = torch.autograd.grad(hu, h)
    assert_close(hu.detach().numpy(), f["hu"], 1e-5, "HU")
    assert_close(gh.numpy(), f["hu_grad"], 1e-5, "HU grad")
    fk, rl = torch.from_numpy(f["w_fake"]), torch.from_numpy(f["w_real"])
    assert_close(R.wasserstein(fk, rl).numpy(), f["w2"], 1e-6, "W2")
    assert_close(R.wasserstein(fk).numpy(), f["w1"], 1e-6, "W1")


def test_gradient_penalty(golden):
    f = golden("gp")
    cfg = R.CriticConfig()
    p = params(R.critic_param_shapes(cfg), 1)
    for k in p:
        p[k].requires_grad_(True)
    gp = R.gradient_penalty(p, torch.from_numpy(f["real"]), torch.from_numpy(f["fake"]),
                            torch.from_numpy(f["eps"]), cfg)
    keys = [k for k in p if f"grad/{k}" in f]
    grads = torch.autograd.grad(gp, [p[k] for k in keys], allow_unused=True)
    assert_close(gp.detach().numpy(), f["gp"], 1e-5, "GP")
    for k, g in zip(keys, grads):
        assert_close(g.numpy(), f[f"grad/{k}"], 1e-4, k)
    assert float(f["fake_grad_absmax"]) == 0.0  # the G path of the GP is dead


def _critic_norm(meta):
    return meta.get("critic_norm", "identity") if meta["gp"] else "batch"


def _configs(meta):
    """Oracle configs of a step fixture (3-D confs, the anisotropic LayerNorm conf, conf_2D)."""
    is2d = bool(meta.get("g_is_2D", False))
    gen = R.GenConfig(meta["g_n_resnet_blocks"], meta["g_n_updownsample_blocks"], meta["g_init_channels_out"], is2d)
    crit = R.CriticConfig(init_channels_out=meta.get("d_init_channels_out", 8), norm=_critic_norm(meta), is_2D=is2d)
    return gen, crit


@pytest.mark.parametrize("tag", ["gp_small", "gp_full", "clip_small", "gp_layernorm", "clip_2d", "ln_aniso"])
def test_train_step(golden, tag):
    f = golden(f"step_{tag}")
    meta = ast.literal_eval(str(f["meta"]))
    gen, crit = _configs(meta)
    gp = bool(meta["gp"])
    cfg = R.StepConfig(gen=gen, critic=crit, gp_weight=10.0 if gp else None,
                       weight_clip=None if gp else 0.01)
    gpar, dpar = params(R.gen_param_shapes(gen), 0), params(R.critic_param_shapes(crit), 1)
    gopt = R.AdamState(meta["lr"], meta["beta1"], meta["beta2"])
    dopt = R.AdamState(meta["lr"], meta["beta1"], meta["beta2"])
    for it in range(meta["iters"]):
        opt = torch.from_numpy(f[f"it{it}/opt"])
        sub = torch.from_numpy(np.concatenate([f[f"it{it}/low"], f[f"it{it}/high"]]))
        mask = torch.from_numpy(np.concatenate([f[f"it{it}/low_seg"], f[f"it{it}/high_seg"]]))
        rec = {}
        logs = R.train_step(gpar, dpar, gopt, dopt, opt, sub, mask,
                            torch.from_numpy(f[f"it{it}/eps"]), cfg, record=rec)
        for k, v in logs.items():
            assert_close(v, f[f"it{it}/loss/{k}"], 1e-4, f"it{it} loss {k}")
        for net in ("G", "D"):
            for k, g in rec[net].items():
                # fp32 against fp32 in another summation order: the reference's own float32
                # deviation from its float64 run is the yardstick (conftest.assert_parity)
                key = f"it{it}/grad/{net}/{k}"
                assert_parity(g.numpy(), f[key], f[key.replace("/grad/", "/grad64/")], f"it{it} grad {net} {k}",
                              atol=1e-7 if k == "model.last.bias" else 0.0)
    for net, p in (("G", gpar), ("D", dpar)):
        keys = [k for k in f if k.startswith(f"final/{net}/")]
        if not keys:
            continue
        assert [k.split("/", 2)[2] for k in keys] == list(p.keys())  # same state_dict layout & order
        for k in keys:
            assert_close(p[k.split("/", 2)[2]].numpy(), f[k], 1e-3, k)


@pytest.mark.parametrize("tag", ["gp_small", "clip_small", "gp_layernorm", "clip_2d", "ln_aniso"])
def test_teacher_forced_fixture_state_is_consistent(golden, tag):
    """The per-iteration fixture entries the GPU test is held to: from the stored state entering
    iteration k (parameters, BatchNorm buffers, Adam moments), the oracle in float64 reproduces the
    reference's float64 gradients of that iteration (it{k}/grad64)."""
    f = golden(f"step_{tag}")
    meta = ast.literal_eval(str(f["meta"]))
    gen, crit = _configs(meta)
    gp = bool(meta["gp"])
    cfg = R.StepConfig(gen=gen, critic=crit, gp_weight=10.0 if gp else None, weight_clip=None if gp else 0.01)
    it = meta["iters"] - 1
    pars = {}
    for net in ("G", "D"):
        pars[net] = {k.split("/", 3)[3]: torch.from_numpy(f[k].copy()) for k in f if k.startswith(f"it{it}/state/{net}/")}
        pars[net] = {k: v.double() if v.is_floating_point() else v for k, v in pars[net].items()}
    opts = {}
    for net in ("G", "D"):
        st = R.AdamState(meta["lr"], meta["beta1"], meta["beta2"], step=int(f[f"it{it}/adam/{net}/step"]))
        for k in R.trainable(pars[net]):
            st.exp_avg[k] = torch.from_numpy(f[f"it{it}/adam/{net}/{k}/exp_avg"]).double()
            st.exp_avg_sq[k] = torch.from_numpy(f[f"it{it}/adam/{net}/{k}/exp_avg_sq"]).double()
        opts[net] = st
    opt = torch.from_numpy(f[f"it{it}/opt"]).double()
    sub = torch.from_numpy(np.concatenate([f[f"it{it}/low"], f[f"it{it}/high"]])).double()
    mask = torch.from_numpy(np.concatenate([f[f"it{it}/low_seg"], f[f"it{it}/high_seg"]]))
    rec = {}
    logs = R.train_step(pars["G"], pars["D"], opts["G"], opts["D"], opt, sub, mask,
                        torch.from_numpy(f[f"it{it}/eps"]).double(), cfg, record=rec)
    for k, v in logs.items():
        assert_close(v, f[f"it{it}/loss64/{k}"], 1e-5, f"it{it} loss64 {k}")
    for net in ("G", "D"):
        for k, g in rec[net].items():
            assert_close(g.numpy(), f[f"it{it}/grad64/{net}/{k}"], 1e-4, f"it{it} grad64 {net} {k}", atol=1e-9)
