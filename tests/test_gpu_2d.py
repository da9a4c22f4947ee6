"""The 2-D variants (experiments/conf_2D.py) on the HIP path: planar geometries (include/cgan3d.h
cgan3d_conv_geom.planar) through the generic f32 implicit-GEMM / VALU kernels.

conf_2D builds on basic_conf: a 2-D ResnetGenerator with 6 ResNet blocks (16 initial channels), a
2-D PatchGAN critic with 16 initial channels (16 -> 32 -> 64 -> 128, BatchNorm2d, LeakyReLU 0.2),
weight clipping at 0.01, Adam lr 2e-4 betas (0.5, 0.999).  The reference fixture (32 x 32, the
generator at half width) is matched in test_gpu_step.py::test_step_matches_reference_fixture[clip_2d];
here the full conf_2D widths run one step at 64 x 64 against the float64 oracle at north_star's
1e-3 (conftest.assert_parity: the oracle's own float32 deviation as the yardstick, ceiling 5e-3),
plus the modules' standalone forwards."""
import numpy as np
import pytest
import torch

from conftest import assert_close, assert_parity

pytestmark = pytest.mark.gpu

G2 = dict(n_resnet_blocks=6, n_updownsample_blocks=2, init_channels_out=16, is_2D=True)
D2 = dict(channels_in=1, init_channels_out=16, discriminator_depth=3, negative_slope=0.2, is_2D=True)
LR, BETAS = 2e-4, (0.5, 0.999)


def _models():
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.generator import ResnetGenerator
    from cgan3d_amd.model.init import pcg64_init_
    return pcg64_init_(ResnetGenerator(**G2), 0).cuda(), pcg64_init_(PatchGANDiscriminator(**D2), 1).cuda()


def _inputs(b, H, W, seed):
    from cgan3d_amd.data.synthetic import synth_patches
    opt, _ = synth_patches(b, (1, H, W), seed)
    sub, seg = synth_patches(b, (1, H, W), seed + 1)
    return opt[:, :, 0], sub[:, :, 0], seg[:, :, 0]


def test_conf_2d_step_matches_oracle():
    from oracle import reference_torch as R
    from cgan3d_amd.engine import StepEngine
    H = W = 64
    b = 4
    g, d = _models()
    gpar = {k: v.detach().cpu().clone() for k, v in g.state_dict().items()}
    dpar = {k: v.detach().cpu().clone() for k, v in d.state_dict().items()}
    eng = StepEngine(g, d, g.config, d.config, b, b, (H, W), g_hyper=(LR, *BETAS, 1e-8), d_hyper=(LR, *BETAS, 1e-8),
                     weight_clip=0.01)
    assert eng.planar and eng.dims == (1, H, W)
    opt, sub, seg = _inputs(b, H, W, 40)
    eng.load_inputs(torch.from_numpy(opt).cuda(), torch.from_numpy(sub).cuda(), torch.from_numpy(seg).cuda(),
                    torch.zeros(b, device="cuda"))
    eng.generator_forward()
    eng.critic_update()
    d_after = {k: v.detach().cpu().clone() for k, v in d.state_dict().items()}
    eng.generator_update()

    def use_device_critic(dp):
        for k in dp:
            dp[k].data.copy_(d_after[k])
    cfg = R.StepConfig(gen=R.GenConfig(6, 2, 16, is_2D=True),
                       critic=R.CriticConfig(init_channels_out=16, norm="batch", is_2D=True),
                       gp_weight=None, weight_clip=0.01)
    recs, refs = {}, {}
    for dt in (torch.float32, torch.float64):
        # copies (the oracle updates its parameters and BatchNorm buffers in place)
        cp = {k: v.to(dt, copy=True) if v.is_floating_point() else v.clone() for k, v in gpar.items()}
        cd = {k: v.to(dt, copy=True) if v.is_floating_point() else v.clone() for k, v in dpar.items()}
        rec = {}
        refs[dt] = R.train_step(cp, cd, R.AdamState(LR, *BETAS), R.AdamState(LR, *BETAS),
                                torch.from_numpy(opt).to(dt), torch.from_numpy(sub).to(dt), torch.from_numpy(seg),
                                None, cfg, record=rec, after_critic=use_device_critic)
        recs[dt] = rec
    losses = eng.losses.cpu().numpy()
    for k, slot in (("D", 0), ("G", 3), ("sim", 4), ("HU", 5), ("G-full", 6)):
        assert_parity(losses[slot], refs[torch.float32][k], refs[torch.float64][k], f"loss {k}")
    for net, arena in (("G", eng.g_arena), ("D", eng.d_arena)):
        for k, gv in arena.gviews.items():
            atol = 1e-7 if k == "model.last.bias" else 0.0  # exactly 0 in real arithmetic
            assert_parity(gv.cpu().numpy(), recs[torch.float32][net][k].numpy(), recs[torch.float64][net][k].numpy(),
                          f"grad {net} {k}", atol=atol)


def test_conf_2d_module_forwards_match_oracle():
    """ResnetGenerator(is_2D) / PatchGANDiscriminator(is_2D) forwards (train-mode BatchNorm: batch
    statistics and running buffers) and eval-mode forwards against the float64 oracle."""
    from oracle import reference_torch as R
    g, d = _models()
    gs = {k: v.detach().cpu().double().clone() if v.is_floating_point() else v.clone() for k, v in g.state_dict().items()}
    ds = {k: v.detach().cpu().double().clone() if v.is_floating_point() else v.clone() for k, v in d.state_dict().items()}
    x, _, _ = _inputs(3, 48, 64, 7)
    xt = torch.from_numpy(x).cuda()
    with torch.no_grad():
        yg, yd = g(xt), d(xt)
    eg = R.generator_forward(gs, torch.from_numpy(x).double(), R.GenConfig(6, 2, 16, is_2D=True), training=True)
    ed = R.critic_forward(ds, torch.from_numpy(x).double(), R.CriticConfig(init_channels_out=16, norm="batch",
                                                                           is_2D=True), training=True)
    assert tuple(yg.shape) == tuple(eg.shape) == (3, 1, 48, 64) and tuple(yd.shape) == tuple(ed.shape)
    assert_close(yg.cpu().numpy(), eg.numpy(), 1e-3, "G_2d(x)")
    assert_close(yd.cpu().numpy(), ed.numpy(), 1e-3, "D_2d(x)")
    for k, v in g.state_dict().items():
        if k.endswith(("running_mean", "running_var")):
            assert_close(v.cpu().numpy(), gs[k].numpy(), 1e-3, k)
    g.eval()
    d.eval()
    with torch.no_grad():
        yg, yd = g(xt), d(xt)
    eg = R.generator_forward(gs, torch.from_numpy(x).double(), R.GenConfig(6, 2, 16, is_2D=True), training=False)
    ed = R.critic_forward(ds, torch.from_numpy(x).double(), R.CriticConfig(init_channels_out=16, norm="batch",
                                                                           is_2D=True), training=False)
    assert_close(yg.cpu().numpy(), eg.numpy(), 1e-3, "G_2d(x) eval")
    assert_close(yd.cpu().numpy(), ed.numpy(), 1e-3, "D_2d(x) eval")


@pytest.mark.parametrize("transposed", [False, True])
def test_planar_conv_matches_torch_conv2d(transposed):
    """One planar geometry per role against torch's float64 conv2d: forward / input-grad / weight-grad,
    cout above 64 (the critic's 128 channels: several channel blocks)."""
    from cgan3d_amd import ops
    rng = np.random.default_rng(3)
    n, cin, cout, k, s, p, H = 2, 64, 128, 4, 2, 1, 20
    if transposed:  # ConvTranspose2d(cin, cout, 3, 2, 1, output_padding=1)
        cin, cout, k, s, p, H = 64, 32, 3, 2, 1, 10
        Ho = 2 * H
        w = rng.standard_normal((cin, cout, k, k)).astype(np.float32) * 0.05
        geo = ops.convt_fwd_geom(n, (1, H, H), (1, Ho, Ho), cin, cout, k, s, p, planar=True)
    else:
        Ho = (H + 2 * p - k) // s + 1
        w = rng.standard_normal((cout, cin, k, k)).astype(np.float32) * 0.05
        geo = ops.conv_fwd_geom(n, (1, H, H), (1, Ho, Ho), cin, cout, k, s, p, planar=True)
    x = rng.standard_normal((n, cin, H, H)).astype(np.float32)
    xt = torch.from_numpy(x).double()
    wt = torch.from_numpy(w).double()
    if transposed:
        ref = torch.nn.functional.conv_transpose2d(xt, wt, stride=s, padding=p, output_padding=1)
    else:
        ref = torch.nn.functional.conv2d(xt, wt, stride=s, padding=p)
    xd = torch.from_numpy(x).cuda().permute(0, 2, 3, 1).contiguous()
    wd = torch.from_numpy(w).cuda()
    y = torch.empty((n, Ho, Ho, cout), device="cuda")
    ops.conv(geo, xd, wd, y)
    assert_close(y.permute(0, 3, 1, 2).cpu().numpy(), ref.numpy(), 1e-4, "planar fwd")
    if transposed:
        return
    # input-grad and weight-grad of the same Conv2d from a random output gradient
    gy = rng.standard_normal(tuple(ref.shape)).astype(np.float32)
    gyt = torch.from_numpy(gy).double()
    dx_ref = torch.nn.grad.conv2d_input(xt.shape, wt, gyt, stride=s, padding=p)
    dw_ref = torch.nn.grad.conv2d_weight(xt, wt.shape, gyt, stride=s, padding=p)
    gyd = torch.from_numpy(gy).cuda().permute(0, 2, 3, 1).contiguous()
    gd = ops.conv_dgrad_geom(n, (1, H, H), (1, Ho, Ho), cin, cout, k, s, p, planar=True)
    dx = torch.empty((n, H, H, cin), device="cuda")
    ops.conv(gd, gyd, wd, dx)
    assert_close(dx.permute(0, 3, 1, 2).cpu().numpy(), dx_ref.numpy(), 1e-4, "planar dgrad")
    gw = ops.conv_wgrad_geom(n, (1, H, H), (1, Ho, Ho), cin, cout, k, s, p, planar=True)
    dw = torch.empty_like(wd)
    ws = torch.empty(ops.wgrad_ws_floats(gw), device="cuda")
    ops.wgrad(gw, xd, gyd, dw, ws)
    assert_close(dw.cpu().numpy(), dw_ref.numpy(), 1e-4, "planar wgrad")
