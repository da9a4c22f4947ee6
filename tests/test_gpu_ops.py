"""Per-op parity of the HIP convolution kernels against torch (CPU, float64), every role and shape
family the step uses (forward / input-grad / weight-grad of Conv3d and ConvTranspose3d, reflect and
zero padding, the k7 single-channel kernels), including sizes that leave partial tiles.

Tolerance 1e-3 relative (north_star); the kernels accumulate in fp32.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import assert_close

pytestmark = pytest.mark.gpu

CONV_CASES = [
    # cin, cout, k, s, p, reflect, spatial
    (1, 16, 7, 1, 3, True, (12, 20, 36)),    # generator first conv (k7 n2w kernel)
    (16, 1, 7, 1, 3, True, (12, 20, 36)),    # generator last conv (k7 w2n kernel)
    (1, 8, 7, 1, 3, True, (8, 8, 8)),
    (8, 1, 7, 1, 3, True, (8, 8, 8)),
    (16, 32, 3, 2, 1, False, (12, 16, 20)),  # downsampling
    (64, 64, 3, 1, 1, False, (6, 8, 10)),    # resnet block
    (1, 8, 4, 2, 1, False, (16, 16, 16)),    # critic first (conv_c1.hip)
    (1, 8, 4, 2, 1, False, (10, 12, 36)),    # critic first, partial 2 x 8 x 16 tiles
    (8, 16, 4, 2, 1, False, (16, 16, 16)),   # critic middle
    (64, 1, 4, 1, 1, False, (4, 4, 4)),      # critic last
    (12, 20, 3, 1, 1, False, (5, 6, 7)),     # odd channel counts (generic path)
]


def _ref_conv(x, w, s, p, reflect):
    if reflect:
        return F.conv3d(F.pad(x, (p,) * 6, mode="reflect"), w, stride=s)
    return F.conv3d(x, w, stride=s, padding=p)


def _cl(t):  # NCDHW -> NDHWC contiguous fp32 on the GPU
    return t.permute(0, 2, 3, 4, 1).contiguous().float().cuda()


def _ncdhw(t):
    return t.permute(0, 4, 1, 2, 3).double().cpu()


@pytest.mark.parametrize("cin,cout,k,s,p,reflect,sp", CONV_CASES)
def test_conv3d_fwd_dgrad_wgrad(cin, cout, k, s, p, reflect, sp):
    from cgan3d_amd import ops
    g = torch.Generator().manual_seed(cin * 100 + cout + k)
    n = 2
    x = torch.randn(n, cin, *sp, generator=g, dtype=torch.float64)
    w = torch.randn(cout, cin, k, k, k, generator=g, dtype=torch.float64) / np.sqrt(cin * k**3)
    x.requires_grad_(True)
    w.requires_grad_(True)
    y = _ref_conv(x, w, s, p, reflect)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    dx, dw = torch.autograd.grad(y, (x, w), gy)
    din, dout = tuple(sp), tuple(y.shape[2:])
    wd = w.detach().float().cuda()
    # forward
    yo = torch.empty(n, *dout, cout, device="cuda")
    ops.conv(ops.conv_fwd_geom(n, din, dout, cin, cout, k, s, p, reflect), _cl(x.detach()), wd, yo)
    assert_close(_ncdhw(yo).numpy(), y.detach().numpy(), 1e-3, "fwd")
    # weight grad
    dwo = torch.empty_like(wd)
    gw = ops.conv_wgrad_geom(n, din, dout, cin, cout, k, s, p, reflect)
    ws = torch.empty(ops.wgrad_ws_floats(gw), device="cuda")
    ops.wgrad(gw, _cl(x.detach()), _cl(gy), dwo, ws)
    assert_close(dwo.double().cpu().numpy(), dw.numpy(), 1e-3, "wgrad")
    # input grad (zero padding directly; reflect via the padded grid + fold, as the engine does)
    if reflect:
        pd = tuple(d + 2 * p for d in din)
        gd = ops.conv_dgrad_geom(n, pd, dout, cin, cout, k, s, 0)
        dpad = torch.empty(n, *pd, cin, device="cuda")
        ops.conv(gd, _cl(gy), wd, dpad)
        dxo = torch.empty(n, *din, cin, device="cuda")
        ops.reflect_fold(dpad, dxo, n, din, cin, p)
    else:
        gd = ops.conv_dgrad_geom(n, din, dout, cin, cout, k, s, p)
        if any(d % s for d in din):
            pytest.skip("input-grad in the transposed mapping needs dims divisible by the stride")
        dxo = torch.empty(n, *din, cin, device="cuda")
        ops.conv(gd, _cl(gy), wd, dxo)
    assert_close(_ncdhw(dxo).numpy(), dx.numpy(), 1e-3, "dgrad")


@pytest.mark.parametrize("cin,cout,sp", [(64, 32, (4, 6, 8)), (32, 16, (8, 8, 8)), (12, 8, (3, 5, 4))])
def test_conv_transpose3d_fwd_dgrad_wgrad(cin, cout, sp):
    from cgan3d_amd import ops
    g = torch.Generator().manual_seed(cin + cout)
    n, k, s, p, op = 2, 3, 2, 1, 1
    x = torch.randn(n, cin, *sp, generator=g, dtype=torch.float64, requires_grad=True)
    w = (torch.randn(cin, cout, k, k, k, generator=g, dtype=torch.float64) / np.sqrt(cout * k**3)).requires_grad_()
    y = F.conv_transpose3d(x, w, stride=s, padding=p, output_padding=op)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    dx, dw = torch.autograd.grad(y, (x, w), gy)
    din, dout = tuple(sp), tuple(y.shape[2:])
    wd = w.detach().float().cuda()
    yo = torch.empty(n, *dout, cout, device="cuda")
    ops.conv(ops.convt_fwd_geom(n, din, dout, cin, cout, k, s, p), _cl(x.detach()), wd, yo)
    assert_close(_ncdhw(yo).numpy(), y.detach().numpy(), 1e-3, "convT fwd")
    dxo = torch.empty(n, *din, cin, device="cuda")
    ops.conv(ops.convt_dgrad_geom(n, din, dout, cin, cout, k, s, p), _cl(gy), wd, dxo)
    assert_close(_ncdhw(dxo).numpy(), dx.numpy(), 1e-3, "convT dgrad")
    gw = ops.convt_wgrad_geom(n, din, dout, cin, cout, k, s, p)
    ws = torch.empty(ops.wgrad_ws_floats(gw), device="cuda")
    dwo = torch.empty_like(wd)
    ops.wgrad(gw, _cl(gy), _cl(x.detach()), dwo, ws)
    assert_close(dwo.double().cpu().numpy(), dw.numpy(), 1e-3, "convT wgrad")


@pytest.mark.parametrize("c", [16, 32])
def test_batchnorm_train_forward_backward(c):
    """BN fwd (stats from the conv epilogue) + ReLU + backward vs torch autograd."""
    from cgan3d_amd import ops, _lib as L
    g = torch.Generator().manual_seed(c)
    n, sp = 2, (8, 12, 16)
    x = torch.randn(n, 8, *sp, generator=g, dtype=torch.float64)
    w = torch.randn(c, 8, 3, 3, 3, generator=g, dtype=torch.float64) / 10
    gamma = torch.rand(c, generator=g, dtype=torch.float64) + 0.5
    beta = torch.randn(c, generator=g, dtype=torch.float64) * 0.1
    z = F.conv3d(x, w, padding=1).requires_grad_()
    gm, bt = gamma.clone().requires_grad_(), beta.clone().requires_grad_()
    rm, rv = torch.zeros(c, dtype=torch.float64), torch.ones(c, dtype=torch.float64)
    y = F.relu(F.batch_norm(z, rm, rv, gm, bt, training=True, momentum=0.1, eps=1e-5))
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    dz, dgm, dbt = torch.autograd.grad(y, (z, gm, bt), gy)
    geo = ops.conv_fwd_geom(n, sp, sp, 8, c, 3, 1, 1)
    zd = torch.empty(n, *sp, c, device="cuda")
    stats = torch.empty(ops.stats_floats(geo), device="cuda")
    ops.conv(geo, _cl(x), w.float().cuda(), zd, ops.epilogue(stats=stats))
    ss, mi = torch.empty(2 * c, device="cuda"), torch.empty(2 * c, device="cuda")
    rmd, rvd = torch.zeros(c, device="cuda"), torch.ones(c, device="cuda")
    nbt = torch.zeros((), dtype=torch.int64, device="cuda")
    gmd, btd = gamma.float().cuda(), beta.float().cuda()
    ops.bn_finalize(stats, stats.numel() // (2 * c + 1), c, gmd, btd, rmd, rvd, nbt, ss, mi)
    nvox = n * sp[0] * sp[1] * sp[2]
    yd = torch.empty_like(zd)
    y16 = torch.empty(zd.shape, device="cuda", dtype=torch.bfloat16)
    ops.bn_apply(zd, nvox, c, ss, L.ACT_RELU, yd, y16=y16)
    assert_close(_ncdhw(yd).numpy(), y.detach().numpy(), 1e-3, "bn fwd")
    assert torch.equal(y16, yd.bfloat16()), "bf16 shadow of the BN output"
    assert_close(rmd.cpu().numpy(), rm.numpy(), 1e-3, "running_mean")
    assert_close(rvd.cpu().numpy(), rv.numpy(), 1e-3, "running_var")
    assert int(nbt.item()) == 1
    dzd, dgd, dbd = torch.empty_like(zd), torch.empty(c, device="cuda"), torch.empty(c, device="cuda")
    ws = torch.empty(ops.bn_backward_ws_floats(nvox, c), device="cuda")
    ops.bn_backward(_cl(gy), zd, nvox, c, ss, mi, gmd, L.ACT_RELU, dgd, dbd, dzd, ws)
    assert_close(_ncdhw(dzd).numpy(), dz.numpy(), 1e-3, "bn dz")
    assert_close(dgd.double().cpu().numpy(), dgm.numpy(), 1e-3, "bn dgamma")
    assert_close(dbd.double().cpu().numpy(), dbt.numpy(), 1e-3, "bn dbeta")


def test_generator_forward_partial_tiles():
    """Generator forward at sizes that leave partial tiles in every kernel (vs the fp64 oracle)."""
    from oracle import reference_torch as R
    from cgan3d_amd.model.generator import ResnetGenerator
    from cgan3d_amd.model.init import pcg64_init_
    g = pcg64_init_(ResnetGenerator(2, 2, 8), 0).cuda().train()
    p = {k: (v.detach().cpu().double() if v.is_floating_point() else v.detach().cpu().clone())
         for k, v in g.state_dict().items()}
    x = torch.randn(2, 1, 12, 20, 36, generator=torch.Generator().manual_seed(5))
    with torch.no_grad():
        y = g(x.cuda())
        yr = R.generator_forward(p, x.double(), R.GenConfig(2, 2, 8), training=True)
    assert_close(y.double().cpu().numpy(), yr.numpy(), 1e-3, "G(x) partial tiles")


GEMM_CASES = [(16, 32, 3, 2, 1, (12, 16, 20)), (64, 64, 3, 1, 1, (6, 8, 10)), (1, 8, 4, 2, 1, (16, 16, 16)),
              (32, 64, 4, 2, 1, (8, 8, 8)), (12, 20, 3, 1, 1, (5, 6, 7))]


@pytest.mark.parametrize("cin,cout,k,s,p,sp", GEMM_CASES)
@pytest.mark.parametrize("prec", ["f32", "bf16"])
def test_conv_gemm_packed(cin, cout, k, s, p, sp, prec, monkeypatch):
    """Implicit-GEMM path with packed weights: f32 within 1e-3; bf16 operands (f32 accumulate)
    within 2e-2 (8-bit mantissa inputs), against torch float64."""
    from cgan3d_amd import ops, _lib as L
    monkeypatch.setattr(ops, "HALO", False)  # the halo-tiled kernel has its own test below
    g = torch.Generator().manual_seed(7 + cin + cout)
    n = 2
    x = torch.randn(n, cin, *sp, generator=g, dtype=torch.float64)
    w = torch.randn(cout, cin, k, k, k, generator=g, dtype=torch.float64) / np.sqrt(cin * k**3)
    y = F.conv3d(x, w, stride=s, padding=p)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    dx = torch.nn.grad.conv3d_input(x.shape, w, gy, stride=s, padding=p)
    din, dout = tuple(sp), tuple(y.shape[2:])
    pc = L.PREC_BF16 if prec == "bf16" else L.PREC_F32
    tol = 2e-2 if prec == "bf16" else 1e-3
    wd = w.float().cuda()
    ps = ops.PackSet(torch.device("cuda"))
    gf, wf = ps.add(ops.conv_fwd_geom(n, din, dout, cin, cout, k, s, p), wd, pc)
    ps.pack()
    # the critic's single-channel first layer reads torch-layout weights (conv_c1.hip)
    assert gf.w_packed == (0 if (cin == 1 and k == 4) else 1)
    yo = torch.empty(n, *dout, cout, device="cuda")
    ops.conv(gf, _cl(x), wf, yo)
    assert_close(_ncdhw(yo).numpy(), y.numpy(), tol, f"{prec} fwd")
    if all(d % s == 0 for d in din) and cin >= 2:
        ps2 = ops.PackSet(torch.device("cuda"))
        gd, wdp = ps2.add(ops.conv_dgrad_geom(n, din, dout, cin, cout, k, s, p), wd, pc)
        ps2.pack()
        dxo = torch.empty(n, *din, cin, device="cuda")
        ops.conv(gd, _cl(gy), wdp, dxo)
        assert_close(_ncdhw(dxo).numpy(), dx.numpy(), tol, f"{prec} dgrad")


def test_bf16_step_tracks_f32_step():
    """One full engine step in bf16 vs f32 from identical state: losses within 2 %."""
    from torch import nn
    from cgan3d_amd.data.synthetic import synth_patches
    from cgan3d_amd.engine import StepEngine
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.generator import ResnetGenerator
    from cgan3d_amd.model.init import pcg64_init_
    S, b = 32, 2
    opt, _ = synth_patches(b, S, 1)
    sub, seg = synth_patches(b, S, 2)
    out = {}
    for prec in ("f32", "bf16"):
        g = pcg64_init_(ResnetGenerator(4, 2, 16), 0).cuda()
        d = pcg64_init_(PatchGANDiscriminator(1, 8, 3, negative_slope=0.2, norm_layer=nn.Identity), 1).cuda()
        eng = StepEngine(g, d, g.config, d.config, b, b, (S, S, S), precision=prec)
        eng.load_inputs(torch.from_numpy(opt).cuda(), torch.from_numpy(sub).cuda(), torch.from_numpy(seg).cuda(),
                        torch.full((b,), 0.4, device="cuda"))
        eng.step()
        out[prec] = eng.losses.cpu().numpy()
    for slot in (0, 2, 4, 5, 6):  # D, GP, sim, HU, G-full
        a, e = float(out["bf16"][slot]), float(out["f32"][slot])
        assert abs(a - e) <= 2e-2 * max(abs(e), 1e-3), (slot, a, e)


HALO_CASES = [
    # transposed-module?, cin, cout, k, s, p, spatial (input of the module)
    (False, 64, 64, 3, 1, 1, (6, 8, 10)),     # ResNet block conv (partial 4^3 tiles)
    (False, 64, 64, 3, 1, 1, (16, 16, 16)),
    (False, 32, 64, 3, 2, 1, (12, 16, 20)),   # downsampling 32 -> 64
    (False, 32, 64, 4, 2, 1, (16, 16, 16)),   # critic middle layer (k4 s2, 10^3 halo)
    (False, 64, 32, 3, 1, 1, (5, 7, 9)),      # 32-channel output tiles
    (True, 64, 32, 3, 2, 1, (4, 6, 8)),       # upsampling ConvTranspose3d 64 -> 32
]


@pytest.mark.parametrize("transposed,cin,cout,k,s,p,sp", HALO_CASES)
def test_conv_halo_bf16(transposed, cin, cout, k, s, p, sp):
    """Halo-tiled bf16 kernel (conv_halo.hip): forward with a residual + ReLU + BN-statistics
    epilogue and the input-grad launch, each against torch float64 within 2e-2 (bf16 operands,
    f32 accumulate); the BN partials against the kernel's own output within 1e-4."""
    from cgan3d_amd import ops, _lib as L
    g = torch.Generator().manual_seed(11 + cin + cout + k)
    n = 2
    x = torch.randn(n, cin, *sp, generator=g, dtype=torch.float64)
    if transposed:
        w = torch.randn(cin, cout, k, k, k, generator=g, dtype=torch.float64) / np.sqrt(cout * k**3)
        y = F.conv_transpose3d(x, w, stride=s, padding=p, output_padding=s - 1)
    else:
        w = torch.randn(cout, cin, k, k, k, generator=g, dtype=torch.float64) / np.sqrt(cin * k**3)
        y = F.conv3d(x, w, stride=s, padding=p)
    res = torch.randn(y.shape, generator=g, dtype=torch.float64)
    yref = torch.relu(y) + res
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    if transposed:
        dx = F.conv3d(gy, w, stride=s, padding=p)
    else:
        dx = torch.nn.grad.conv3d_input(x.shape, w, gy, stride=s, padding=p)
    din, dout = tuple(sp), tuple(y.shape[2:])
    wd = w.float().cuda()
    ps = ops.PackSet(torch.device("cuda"))
    if transposed:
        gf0 = ops.convt_fwd_geom(n, din, dout, cin, cout, k, s, p)
        gd0 = ops.convt_dgrad_geom(n, din, dout, cin, cout, k, s, p)
    else:
        gf0 = ops.conv_fwd_geom(n, din, dout, cin, cout, k, s, p)
        gd0 = ops.conv_dgrad_geom(n, din, dout, cin, cout, k, s, p)
    gf, wf = ps.add(gf0, wd, L.PREC_BF16)
    gd, wdp = ps.add(gd0, wd, L.PREC_BF16)
    ps.pack()
    # the critic's k4 geometries go to the K-split kernel (format 3, conv_sk.hip), the rest to the halo kernel
    assert gf.w_packed in (2, 3) and gd.w_packed in (2, 3), "expected the halo / K-split kernels"
    yo = torch.empty(n, *dout, cout, device="cuda")
    stats = torch.empty(ops.stats_floats(gf), device="cuda")
    ops.conv(gf, _cl(x), wf, yo, ops.epilogue(act=L.ACT_RELU, residual=_cl(res), stats=stats))
    assert_close(_ncdhw(yo).numpy(), yref.numpy(), 2e-2, "halo fwd")
    # BN partials -> per-channel mean / biased variance of the kernel's output
    st = stats.double().cpu().view(-1, 2 * cout + 1)
    cnt = st[:, 2 * cout]
    tot = cnt.sum()
    mean = st[:, :cout].sum(0) / tot
    bm = st[:, :cout] / cnt.clamp(min=1)[:, None]
    m2 = st[:, cout:2 * cout].sum(0) + (cnt[:, None] * (bm - mean) ** 2).sum(0)
    yk = yo.double().cpu().view(-1, cout)
    assert int(tot) == yk.shape[0]
    assert_close(mean.numpy(), yk.mean(0).numpy(), 1e-4, "halo stats mean")
    assert_close((m2 / tot).numpy(), yk.var(0, unbiased=False).numpy(), 1e-4, "halo stats var")
    dxo = torch.empty(n, *din, cin, device="cuda")
    ops.conv(gd, _cl(gy), wdp, dxo)
    assert_close(_ncdhw(dxo).numpy(), dx.numpy(), 2e-2, "halo dgrad")
    if gf.w_packed == 2 and gd.w_packed == 2:
        # halo kernels staging from a bf16 shadow of the input: the same bf16
        # operands (round-to-nearest-even either way), so bit-identical outputs and statistics
        yo16, st16 = torch.empty_like(yo), torch.empty_like(stats)
        ops.conv(gf, _cl(x), wf, yo16, ops.epilogue(act=L.ACT_RELU, residual=_cl(res), stats=st16,
                                                    x_bf16=_cl(x).bfloat16()))
        assert torch.equal(yo16, yo), "bf16-shadow forward differs"
        assert torch.equal(st16, stats), "bf16-shadow statistics differ"
        dxo16 = torch.empty_like(dxo)
        ops.conv(gd, _cl(gy), wdp, dxo16, ops.epilogue(x_bf16=_cl(gy).bfloat16()))
        if (transposed, cin, cout, k, s, p) == (False, 64, 64, 3, 1, 1):
            # the ResNet-block shape with a shadow and no statistics takes conv_k3m (the same bf16
            # products summed in another fp32 order; its own test: test_conv_k3m_bf16)
            assert_close(dxo16.cpu().double().numpy(), dxo.cpu().double().numpy(), 1e-5, "k3m vs k3 input-grad")
        else:
            assert torch.equal(dxo16, dxo), "bf16-shadow input-grad differs"


@pytest.mark.parametrize("sp", [(12, 20, 36), (16, 16, 16), (20, 9, 72)])
def test_k7_bf16_mfma(sp):
    """bf16 MFMA variants of the generator's k7 convs (conv_k7_mfma.hip), all four roles plus the
    last conv's input-grad, against torch float64 within 2e-2 (bf16 operands, f32 accumulate); the
    first conv's BN partials against its own output within 1e-4."""
    from cgan3d_amd import ops, _lib as L
    BF = L.PREC_BF16
    g = torch.Generator().manual_seed(77)
    n, k, p = 2, 7, 3
    x1 = torch.randn(n, 1, *sp, generator=g, dtype=torch.float64)
    x16 = torch.randn(n, 16, *sp, generator=g, dtype=torch.float64)
    wf = (torch.randn(16, 1, k, k, k, generator=g, dtype=torch.float64) / np.sqrt(k**3)).requires_grad_()
    wl = (torch.randn(1, 16, k, k, k, generator=g, dtype=torch.float64) / np.sqrt(16 * k**3)).requires_grad_()
    bl = torch.randn(1, generator=g, dtype=torch.float64)
    x16r = x16.clone().requires_grad_()
    yf = _ref_conv(x1, wf, 1, p, True)
    zl = _ref_conv(x16r, wl, 1, p, True) + bl.view(1, 1, 1, 1, 1)
    yl = torch.tanh(zl)
    gf = torch.randn(yf.shape, generator=g, dtype=torch.float64)
    gl = torch.randn(zl.shape, generator=g, dtype=torch.float64)
    dwf, = torch.autograd.grad(yf, (wf,), gf)
    dx16, dwl = torch.autograd.grad(zl, (x16r, wl), gl)
    dims = tuple(sp)
    # first conv forward (+ BN partials)
    geo = ops.with_prec(ops.conv_fwd_geom(n, dims, dims, 1, 16, k, 1, p, True), BF)
    yo = torch.empty(n, *dims, 16, device="cuda")
    stats = torch.empty(ops.stats_floats(geo), device="cuda")
    ops.conv(geo, _cl(x1), wf.detach().float().cuda(), yo, ops.epilogue(stats=stats))
    assert_close(_ncdhw(yo).numpy(), yf.detach().numpy(), 2e-2, "k7 n2w fwd")
    st = stats.double().cpu().view(-1, 33)
    yk = yo.double().cpu().view(-1, 16)
    assert int(st[:, 32].sum()) == yk.shape[0]
    assert_close((st[:, :16].sum(0) / yk.shape[0]).numpy(), yk.mean(0).numpy(), 1e-4, "k7 stats mean")
    # per-block (sum, M2 about the block mean, count) merged (Chan) -> the population variance
    cnt, S, M2 = st[:, 32], st[:, :16], st[:, 16:32]
    live = cnt > 0
    bm = S[live] / cnt[live, None]
    mu = S.sum(0) / cnt.sum()
    m2 = M2[live].sum(0) + (cnt[live, None] * (bm - mu) ** 2).sum(0)
    assert_close((m2 / cnt.sum()).numpy(), yk.var(0, unbiased=False).numpy(), 1e-4, "k7 stats var")
    # the same statistics into fp64 accumulators (cgan3d_bn_fuse mode 3, the bf16 step's form)
    reps = 16
    acc = torch.zeros(reps * 2 * 16, device="cuda", dtype=torch.float64)
    ya = torch.empty_like(yo)
    ops.conv(geo, _cl(x1), wf.detach().float().cuda(), ya, ops.epilogue(fuse=ops.BnFuse(acc, 3, reps)))
    # the accumulator form runs the streamed-plane kernel (conv_k7p.hip, round 6): the same bf16
    # products summed in another fp32 order than the slab form's k7m_n2w kernel
    assert float((ya - yo).abs().max()) <= 1e-5 * float(yo.abs().max()), "k7p vs k7m forward"
    a2 = acc.cpu().view(reps, 2, 16).sum(0)
    N = yk.shape[0]
    assert_close((a2[0] / N).numpy(), yk.mean(0).numpy(), 1e-4, "k7 acc mean")
    assert_close((a2[1] / N - (a2[0] / N) ** 2).numpy(), yk.var(0, unbiased=False).numpy(), 1e-4, "k7 acc var")
    # last conv forward (bias, tanh, out2 = minuend - y)
    geo = ops.with_prec(ops.conv_fwd_geom(n, dims, dims, 16, 1, k, 1, p, True), BF)
    att = torch.empty(n, *dims, 1, device="cuda")
    o2 = torch.empty_like(att)
    mn = _cl(x1)
    ops.conv(geo, _cl(x16), wl.detach().float().cuda(), att,
             ops.epilogue(bias=bl.float().cuda(), act=L.ACT_TANH, minuend=mn, out2=o2))
    assert_close(_ncdhw(att).numpy(), yl.detach().numpy(), 2e-2, "k7 w2n fwd")
    assert_close(_ncdhw(o2).numpy(), (x1 - yl).detach().numpy(), 2e-2, "k7 w2n out2")
    # from a bf16 shadow of x the streamed-plane kernel runs (k7s_w2n_kernel: the same bf16
    # operands, another fp32 summation order): against float64 at the bf16 bar, and against the
    # fp32-staging kernel within fp32 reassociation noise (bf16 products summed exactly in fp32)
    att16, o216 = torch.empty_like(att), torch.empty_like(o2)
    ops.conv(geo, _cl(x16), wl.detach().float().cuda(), att16,
             ops.epilogue(bias=bl.float().cuda(), act=L.ACT_TANH, minuend=mn, out2=o216,
                          x_bf16=_cl(x16).bfloat16()))
    assert_close(_ncdhw(att16).numpy(), yl.detach().numpy(), 2e-2, "k7s w2n fwd")
    assert_close(_ncdhw(o216).numpy(), (x1 - yl).detach().numpy(), 2e-2, "k7s w2n out2")
    assert float((att16 - att).abs().max()) <= 1e-5, "k7s w2n vs k7m w2n (same bf16 operands)"
    # weight grads
    for name, gw, gath, alig, ref, w in (
            ("k7 wg n2w", ops.conv_wgrad_geom(n, dims, dims, 1, 16, k, 1, p, True), _cl(x1), _cl(gf), dwf, wf),
            ("k7 wg w2n", ops.conv_wgrad_geom(n, dims, dims, 16, 1, k, 1, p, True), _cl(x16), _cl(gl), dwl, wl)):
        gw = ops.with_prec(gw, BF)
        ws = torch.empty(ops.wgrad_ws_floats(gw), device="cuda")
        dwo = torch.empty(w.shape, device="cuda")
        ops.wgrad(gw, gath, alig, dwo, ws)
        assert_close(dwo.double().cpu().numpy(), ref.numpy(), 2e-2, name)
    # last conv input-grad: flipped n2w onto the zero-padded grid + reflect fold (as the engine)
    pd = tuple(d + 2 * p for d in dims)
    gd = ops.with_prec(ops.conv_dgrad_geom(n, pd, dims, 16, 1, k, 1, 0), BF)
    dpad = torch.empty(n, *pd, 16, device="cuda")
    ops.conv(gd, _cl(gl), wl.detach().float().cuda(), dpad)
    dxo = torch.empty(n, *dims, 16, device="cuda")
    ops.reflect_fold(dpad, dxo, n, dims, 16, p)
    assert_close(_ncdhw(dxo).numpy(), dx16.numpy(), 2e-2, "k7 n2w dgrad")


def _k7_fold_operands(n, dims, g, z16):
    """BatchNorm-backward operands of the layer under the last conv (its z, scale / shift, mean / invstd)
    for the folded mode-2 statistics of the k7 input-grad"""
    z = torch.randn(n, *dims, 16, generator=g).cuda()
    ss = torch.cat([torch.rand(16, generator=g) + 0.5, torch.randn(16, generator=g) * 0.1]).cuda()
    mi = torch.cat([torch.randn(16, generator=g) * 0.1, torch.rand(16, generator=g) + 0.5]).cuda()
    return (z.bfloat16() if z16 else z), ss, mi


@pytest.mark.parametrize("sp,tdc", [((12, 20, 36), 0), ((16, 16, 16), 5), ((20, 9, 72), 7), ((9, 33, 17), 64)])
def test_k7p_n2w_matches_k7m(sp, tdc):
    """The streamed-plane 1 -> 16 k7 kernel (conv_k7p.hip, round 6; cgan3d_set_tuning key 21 = output
    planes per block) against the per-tile k7m_n2w kernel (key 21 = -1) on the same bf16 operands, in
    every role the bf16 step gives it: the first conv's forward without statistics / with fp64
    accumulator statistics (mode 3), fp32 and bf16 output; the last conv's input-grad onto the padded grid
    with and without the reflect-folded mode-2 statistics (mode 4 accumulators), fp32 and bf16 z / output.
    Outputs agree to fp32 reassociation (1e-5 of the largest), statistics to 1e-5 relative, ragged tiles
    and chunks included; the forward also against torch float64 at the bf16 bar."""
    from cgan3d_amd import ops, _lib as L
    BF = L.PREC_BF16
    lib = L.load()
    g = torch.Generator().manual_seed(sum(sp) + tdc)
    n, k, p = 2, 7, 3
    x1 = torch.randn(n, 1, *sp, generator=g, dtype=torch.float64)
    wf = torch.randn(16, 1, k, k, k, generator=g, dtype=torch.float64) / np.sqrt(k**3)
    wl = torch.randn(1, 16, k, k, k, generator=g, dtype=torch.float64) / np.sqrt(16 * k**3)
    gl = torch.randn(n, 1, *sp, generator=g, dtype=torch.float64)
    gf = torch.randn(n, 16, *sp, generator=g, dtype=torch.float64)
    x16 = torch.randn(n, 16, *sp, generator=g, dtype=torch.float64)
    dims = tuple(sp)
    pd = tuple(d + 2 * p for d in dims)
    reps = 16

    def run(key):
        L.check(lib.cgan3d_set_tuning(21, key), "k7p tdc")
        out = {}
        geo = ops.with_prec(ops.conv_fwd_geom(n, dims, dims, 1, 16, k, 1, p, True), BF)
        for dt in (torch.float32, torch.bfloat16):
            y = torch.empty(n, *dims, 16, device="cuda", dtype=dt)
            ops.conv(geo, _cl(x1), wf.float().cuda(), y, ops.epilogue())
            out[f"fwd {dt}"] = y.float()
            acc = torch.zeros(reps * 2 * 16, device="cuda", dtype=torch.float64)
            y = torch.empty(n, *dims, 16, device="cuda", dtype=dt)
            ops.conv(geo, _cl(x1), wf.float().cuda(), y, ops.epilogue(fuse=ops.BnFuse(acc, 3, reps)))
            out[f"fwd3 {dt}"] = y.float()
            out[f"acc3 {dt}"] = acc.view(reps, 2, 16).sum(0)
        gd = ops.with_prec(ops.conv_dgrad_geom(n, pd, dims, 16, 1, k, 1, 0), BF)
        for z16 in (False, True):
            dt = torch.bfloat16 if z16 else torch.float32
            dpad = torch.empty(n, *pd, 16, device="cuda", dtype=dt)
            ops.conv(gd, _cl(gl), wl.float().cuda(), dpad, ops.epilogue())
            out[f"dgrad {dt}"] = dpad.float()
            gz = torch.Generator().manual_seed(5)
            z, ss, mi = _k7_fold_operands(n, dims, gz, z16)
            acc = torch.zeros(reps * 2 * 16, device="cuda", dtype=torch.float64)
            ep = ops.epilogue(bn_z=z, bn_ss=ss, bn_mi=mi, bn_act=L.ACT_RELU, fuse=ops.BnFuse(acc, 4, reps))
            ep.bn_fold = p
            dpad = torch.empty(n, *pd, 16, device="cuda", dtype=dt)
            ops.conv(gd, _cl(gl), wl.float().cuda(), dpad, ep)
            out[f"dgrad4 {dt}"] = dpad.float()
            out[f"acc4 {dt}"] = acc.view(reps, 2, 16).sum(0)
        # weight grads from the 16-channel operand's bf16 shadow (the step's form: k7p_wg_kernel, round 6)
        gw0 = ops.with_prec(ops.conv_wgrad_geom(n, dims, dims, 1, 16, k, 1, p, True), BF)
        ws = torch.empty(ops.wgrad_ws_floats(gw0), device="cuda")
        dw0 = torch.empty(16, 1, k, k, k, device="cuda")
        ops.wgrad(gw0, _cl(x1), _cl(gf), dw0, ws, aligned16=_cl(gf).bfloat16())
        out["wg first float32"] = dw0.clone()
        gw1 = ops.with_prec(ops.conv_wgrad_geom(n, dims, dims, 16, 1, k, 1, p, True), BF)
        ws = torch.empty(ops.wgrad_ws_floats(gw1), device="cuda")
        dw1 = torch.empty(1, 16, k, k, k, device="cuda")
        ops.wgrad(gw1, _cl(x16), _cl(gl), dw1, ws, gathered16=_cl(x16).bfloat16())
        out["wg last float32"] = dw1.clone()
        torch.cuda.synchronize()
        return out

    try:
        new, old = run(tdc), run(-1)
    finally:
        L.check(lib.cgan3d_set_tuning(21, 0), "k7p auto")
    for key in new:
        a, b = new[key].double().cpu(), old[key].double().cpu()
        scale = float(b.abs().max())
        bar = 1e-5 if "acc" in key or "float32" in key else 8e-3  # bf16 outputs: one rounding step apart at most
        assert float((a - b).abs().max()) <= bar * scale, (key, float((a - b).abs().max()), scale)
    yf = _ref_conv(x1, wf, 1, p, True)
    assert_close(_ncdhw(new["fwd3 torch.float32"]).numpy(), yf.numpy(), 2e-2, "k7p fwd vs float64")
    # the weight grads against float64 autograd (bf16 operands: the bf16 bar)
    wf_ = wf.clone().requires_grad_()
    dwf, = torch.autograd.grad(_ref_conv(x1, wf_, 1, p, True), (wf_,), gf)
    assert_close(new["wg first float32"].double().cpu().numpy(), dwf.numpy(), 2e-2, "k7p wg first vs float64")
    wl_ = wl.clone().requires_grad_()
    dwl, = torch.autograd.grad(_ref_conv(x16, wl_, 1, p, True), (wl_,), gl)
    assert_close(new["wg last float32"].double().cpu().numpy(), dwl.numpy(), 2e-2, "k7p wg last vs float64")


WGRAD_BF16_CASES = [
    # cin, cout, k, s, p, reflect, spatial (module input)
    (64, 64, 3, 1, 1, False, (8, 10, 12)),   # ResNet block (H % 4 != 0: generic kernel)
    (64, 64, 3, 1, 1, False, (16, 16, 16)),  # ResNet block at 64^3 patches: wgrad_k3_kernel
    (64, 64, 3, 1, 1, False, (5, 4, 8)),     # wgrad_k3_kernel, odd unit count, one unit per row
    (16, 32, 3, 2, 1, False, (12, 16, 20)),  # downsampling
    (16, 32, 3, 2, 1, False, (8, 16, 64)),   # downsampling 16 -> 32: wgrad_s2_kernel (4 x 8 x 32 outputs)
    (32, 64, 3, 2, 1, False, (8, 16, 32)),   # downsampling 32 -> 64: wgrad_s2_kernel<32, 64> (round 6)
    (32, 64, 3, 2, 1, False, (7, 16, 32)),   # ... odd input depth (a window plane past the volume)
    (8, 16, 4, 2, 1, False, (16, 16, 16)),   # critic middle
    (32, 64, 4, 2, 1, False, (8, 8, 8)),
    (12, 20, 3, 1, 1, True, (5, 6, 7)),      # odd channel counts, reflect
    (1, 8, 4, 2, 1, False, (16, 16, 16)),    # critic first layer (single-channel input)
]


@pytest.mark.parametrize("cin,cout,k,s,p,reflect,sp", WGRAD_BF16_CASES)
def test_wgrad_bf16(cin, cout, k, s, p, reflect, sp):
    """bf16-MFMA weight gradient (conv_wgrad.hip) against torch float64 within 2e-2, plus the
    ConvTranspose3d role (operands swapped) at the generator's upsampling shape."""
    from cgan3d_amd import ops, _lib as L
    g = torch.Generator().manual_seed(5 + cin + cout)
    n = 2
    x = torch.randn(n, cin, *sp, generator=g, dtype=torch.float64)
    w = (torch.randn(cout, cin, k, k, k, generator=g, dtype=torch.float64) / np.sqrt(cin * k**3)).requires_grad_()
    y = _ref_conv(x, w, s, p, reflect)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    dw, = torch.autograd.grad(y, (w,), gy)
    gw = ops.with_prec(ops.conv_wgrad_geom(n, tuple(sp), tuple(y.shape[2:]), cin, cout, k, s, p, reflect), L.PREC_BF16)
    ws = torch.empty(ops.wgrad_ws_floats(gw), device="cuda")
    dwo = torch.empty(w.shape, device="cuda")
    ops.wgrad(gw, _cl(x), _cl(gy), dwo, ws)
    assert_close(dwo.double().cpu().numpy(), dw.numpy(), 2e-2, "bf16 wgrad")
    if tuple(sp) in ((8, 16, 64), (8, 16, 32), (7, 16, 32)):
        # wgrad_s2_kernel (the generic kernel ignores shadows and sums with atomics, so no bitwise
        # comparison there; the ResNet shape takes wgrad_k3m_kernel from shadows: its own test below):
        # both operands from bf16 shadows, bit-identical
        dw16 = torch.empty_like(dwo)
        ops.wgrad(gw, _cl(x), _cl(gy), dw16, ws, gathered16=_cl(x).bfloat16(), aligned16=_cl(gy).bfloat16())
        assert torch.equal(dw16, dwo), "bf16-shadow weight grad differs"
    ops.wgrad(gw, _cl(x), _cl(gy), dwo, ws, accumulate=True)
    assert_close(dwo.double().cpu().numpy(), 2 * dw.numpy(), 2e-2, "bf16 wgrad accumulate")


@pytest.mark.parametrize("cin,cout,sp", [(16, 32, (8, 16, 64)), (32, 64, (8, 16, 32))])
@pytest.mark.parametrize("blocks", [2, 4, 8, 16])
def test_wgrad_s2_slab_unrolled_variants(cin, cout, sp, blocks):
    """Round 6: wgrad_s2_kernel's unrolled slab loops (2, 4 or 8 slabs per block, two slabs in flight
    for <16, 32>) — tuning key 10 sets the block count, so a 16-slab grid runs 8, 4, 2 or 1 slabs per
    block — against torch float64 (2e-2), and bit-identical between bf16 shadows and fp32 operands."""
    from cgan3d_amd import ops, _lib as L
    g = torch.Generator().manual_seed(17 + cin + blocks)
    n, k, s, p = 2, 3, 2, 1
    x = torch.randn(n, cin, *sp, generator=g, dtype=torch.float64)
    w = (torch.randn(cout, cin, k, k, k, generator=g, dtype=torch.float64) / np.sqrt(cin * k**3)).requires_grad_()
    y = _ref_conv(x, w, s, p, False)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    dw, = torch.autograd.grad(y, (w,), gy)
    lib = L.lib()
    key = blocks * (2 if cin == 32 else 1)  # the 32 <-> 64 level takes half of key 10's blocks
    try:
        assert lib.cgan3d_set_tuning(10, key) == 0
        gw = ops.with_prec(ops.conv_wgrad_geom(n, tuple(sp), tuple(y.shape[2:]), cin, cout, k, s, p, False), L.PREC_BF16)
        ws = torch.empty(ops.wgrad_ws_floats(gw), device="cuda")
        dwo, dw16 = torch.empty(w.shape, device="cuda"), torch.empty(w.shape, device="cuda")
        ops.wgrad(gw, _cl(x), _cl(gy), dwo, ws)
        ops.wgrad(gw, _cl(x), _cl(gy), dw16, ws, gathered16=_cl(x).bfloat16(), aligned16=_cl(gy).bfloat16())
    finally:
        lib.cgan3d_set_tuning(10, 128)
    assert_close(dwo.double().cpu().numpy(), dw.numpy(), 2e-2, "wgrad_s2 unrolled")
    assert torch.equal(dw16, dwo), "bf16-shadow vs fp32-operand stride-2 weight grad differ"


@pytest.mark.parametrize("cin,cout,sp", [(64, 32, (4, 6, 8)), (32, 16, (4, 8, 32)), (64, 32, (4, 8, 16))])
def test_wgrad_bf16_conv_transpose(cin, cout, sp):
    """ConvTranspose3d weight gradient (operands swapped); 32 -> 16 at (4, 8, 32) and 64 -> 32 at
    (4, 8, 16) take wgrad_s2_kernel (the up-sampling layers' shapes)."""
    from cgan3d_amd import ops, _lib as L
    g = torch.Generator().manual_seed(9 + cin)
    n, k, s, p = 2, 3, 2, 1
    x = torch.randn(n, cin, *sp, generator=g, dtype=torch.float64)
    w = (torch.randn(cin, cout, k, k, k, generator=g, dtype=torch.float64) / np.sqrt(cout * k**3)).requires_grad_()
    y = F.conv_transpose3d(x, w, stride=s, padding=p, output_padding=1)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    dw, = torch.autograd.grad(y, (w,), gy)
    gw = ops.with_prec(ops.convt_wgrad_geom(n, sp, tuple(y.shape[2:]), cin, cout, k, s, p), L.PREC_BF16)
    ws = torch.empty(ops.wgrad_ws_floats(gw), device="cuda")
    dwo = torch.empty(w.shape, device="cuda")
    ops.wgrad(gw, _cl(gy), _cl(x), dwo, ws)
    assert_close(dwo.double().cpu().numpy(), dw.numpy(), 2e-2, "bf16 convT wgrad")
    if tuple(sp) != (4, 6, 8):  # wgrad_s2_kernel from both operands' bf16 shadows: bit-identical
        dw16 = torch.empty_like(dwo)
        ops.wgrad(gw, _cl(gy), _cl(x), dw16, ws, gathered16=_cl(gy).bfloat16(), aligned16=_cl(x).bfloat16())
        assert torch.equal(dw16, dwo), "bf16-shadow convT weight grad differs"


S2_CASES = [
    # role, spatial of the 16-channel (fine) grid
    ("down_fwd", (10, 12, 36)),    # Conv3d 16 -> 32 k3 s2 p1 forward (S2F)
    ("down_fwd", (11, 9, 17)),     # odd fine grid: partial tiles on every axis
    ("up_dgrad", (10, 12, 36)),    # ConvTranspose3d 32 -> 16 input-grad = stride-2 conv (S2F)
    ("up_fwd", (10, 12, 36)),      # ConvTranspose3d 32 -> 16 forward, output_padding 1 (S2T)
    ("down_dgrad", (10, 12, 36)),  # Conv3d 16 -> 32 input-grad = transposed mapping (S2T)
    ("up_fwd", (6, 10, 34)),
]


@pytest.mark.parametrize("role,fine", S2_CASES)
def test_conv_s2_bf16(role, fine):
    """Stride-2 16 <-> 32-channel kernels (conv_s2.hip) in all four generator roles: output against
    torch float64 within 2e-2 (bf16 operands, fp32 accumulation), bias + ReLU epilogue, and both
    fused BatchNorm slab modes against the kernel's own output (1e-4)."""
    from cgan3d_amd import ops, _lib as L
    n, k, s, p = 2, 3, 2, 1
    fine = tuple(fine)
    coarse = tuple((d - 1) // 2 + 1 for d in fine)
    if role.startswith("up"):  # the ConvTranspose's coarse grid must map onto exactly 2x
        fine = tuple(2 * d for d in coarse)
    g = torch.Generator().manual_seed(3 + len(role) + fine[2])
    if role == "down_fwd":       # x16 (fine) -> y32 (coarse)
        w = torch.randn(32, 16, k, k, k, generator=g, dtype=torch.float64) / np.sqrt(16 * 27)
        x = torch.randn(n, 16, *fine, generator=g, dtype=torch.float64)
        ref = F.conv3d(x, w, stride=s, padding=p)
        geo0 = ops.conv_fwd_geom(n, fine, coarse, 16, 32, k, s, p)
    elif role == "down_dgrad":   # dz32 (coarse) -> dx16 (fine)
        w = torch.randn(32, 16, k, k, k, generator=g, dtype=torch.float64) / np.sqrt(32 * 27)
        x = torch.randn(n, 32, *coarse, generator=g, dtype=torch.float64)
        ref = torch.nn.grad.conv3d_input((n, 16, *fine), w, x, stride=s, padding=p)
        geo0 = ops.conv_dgrad_geom(n, fine, coarse, 16, 32, k, s, p)
    elif role == "up_fwd":       # ConvTranspose3d(32 -> 16): x32 (coarse) -> y16 (fine)
        w = torch.randn(32, 16, k, k, k, generator=g, dtype=torch.float64) / np.sqrt(32 * 27)
        x = torch.randn(n, 32, *coarse, generator=g, dtype=torch.float64)
        ref = F.conv_transpose3d(x, w, stride=s, padding=p, output_padding=1)
        geo0 = ops.convt_fwd_geom(n, coarse, fine, 32, 16, k, s, p)
    else:                        # up_dgrad: dy16 (fine) -> dx32 (coarse)
        w = torch.randn(32, 16, k, k, k, generator=g, dtype=torch.float64) / np.sqrt(16 * 27)
        x = torch.randn(n, 16, *fine, generator=g, dtype=torch.float64)
        ref = F.conv3d(x, w, stride=s, padding=p)
        geo0 = ops.convt_dgrad_geom(n, coarse, fine, 32, 16, k, s, p)
    cout = ref.shape[1]
    bias = torch.randn(cout, generator=g, dtype=torch.float64) * 0.1
    ps = ops.PackSet(torch.device("cuda"))
    geo, wp = ps.add(geo0, w.float().cuda(), L.PREC_BF16)
    ps.pack()
    assert geo.w_packed == 2, "expected the halo-format (conv_s2) kernel"
    dout = tuple(ref.shape[2:])
    y = torch.empty(n, *dout, cout, device="cuda")
    slots = ops.bn_slots(geo)
    part = torch.full(((2 * cout + 1) * slots,), float("nan"), device="cuda")
    ops.conv(geo, _cl(x), wp, y, ops.epilogue(bias=bias.float().cuda(), act=L.ACT_RELU, bn_part=part, bn_mode=1,
                                              bn_slots=slots))
    assert_close(_ncdhw(y).numpy(), torch.relu(ref + bias.view(1, -1, 1, 1, 1)).numpy(), 2e-2, f"{role} out")
    # staging from a bf16 shadow of the input (the same bf16 operands): bit-identical output and slab
    y16, part16 = torch.empty_like(y), torch.full_like(part, float("nan"))
    ops.conv(geo, _cl(x), wp, y16, ops.epilogue(bias=bias.float().cuda(), act=L.ACT_RELU, bn_part=part16, bn_mode=1,
                                                bn_slots=slots, x_bf16=_cl(x).bfloat16()))
    assert torch.equal(y16, y) and torch.equal(part16.nan_to_num(), part.nan_to_num()), \
        f"{role}: bf16-shadow result differs"
    sl = part.double().cpu().view(2 * cout + 1, slots)
    cnt = sl[2 * cout]
    tot = cnt.sum()
    yk = y.double().cpu().reshape(-1, cout)
    assert int(tot) == yk.shape[0]
    mean = sl[:cout].sum(1) / tot
    bm = sl[:cout] / cnt.clamp(min=1)
    m2 = sl[cout:2 * cout].sum(1) + (cnt * (bm - mean[:, None]) ** 2).sum(1)
    assert_close(mean.numpy(), yk.mean(0).numpy(), 1e-4, f"{role} slab mean")
    assert_close((m2 / tot).numpy(), yk.var(0, unbiased=False).numpy(), 1e-4, f"{role} slab var")
    # mode 2: (sum g, sum g*xhat) of a BatchNorm + ReLU layer whose input z has this output's shape
    z = torch.randn(n, *dout, cout, generator=g).cuda()
    ss = torch.cat([torch.rand(cout, generator=g) + 0.5, torch.randn(cout, generator=g) * 0.2]).cuda()
    mi = torch.cat([torch.randn(cout, generator=g) * 0.1, torch.rand(cout, generator=g) + 0.5]).cuda()
    part2 = torch.full((2 * cout * slots,), float("nan"), device="cuda")
    y2 = torch.empty_like(y)
    ops.conv(geo, _cl(x), wp, y2, ops.epilogue(bn_part=part2, bn_mode=2, bn_slots=slots, bn_z=z, bn_ss=ss, bn_mi=mi,
                                               bn_act=L.ACT_RELU))
    o = y2.double().cpu().reshape(-1, cout)
    zz = z.double().cpu().reshape(-1, cout)
    ssd, mid = ss.double().cpu(), mi.double().cpu()
    gg = o * ((zz * ssd[:cout] + ssd[cout:]) > 0).double()
    want = torch.cat([gg.sum(0), (gg * (zz - mid[:cout]) * mid[cout:]).sum(0)])
    got = part2.double().cpu().view(2 * cout, slots).sum(1)
    assert_close(got.numpy(), want.numpy(), 1e-4, f"{role} mode-2 slab")
    # mode 2 staged from the bf16 shadow (S2T: two resident blocks per CU instead of one): bit-identical
    y2b, part2b = torch.empty_like(y), torch.full_like(part2, float("nan"))
    ops.conv(geo, _cl(x), wp, y2b, ops.epilogue(bn_part=part2b, bn_mode=2, bn_slots=slots, bn_z=z, bn_ss=ss, bn_mi=mi,
                                                bn_act=L.ACT_RELU, x_bf16=_cl(x).bfloat16()))
    assert torch.equal(y2b, y2) and torch.equal(part2b.nan_to_num(), part2.nan_to_num()), \
        f"{role}: bf16-shadow mode-2 result differs"


SK_CASES = [
    # cin, cout, spatial (module input): the critic's middle layers, k4 s2 p1 (conv_sk.hip)
    (8, 16, (16, 16, 16)),
    (16, 32, (8, 8, 8)),
    (32, 64, (8, 8, 8)),
    (8, 16, (10, 12, 14)),  # partial 16-row tiles
    (8, 16, (32, 32, 48)),  # >= 1024 row tiles: one tile per wave (statistics rows per wave)
    (16, 32, (32, 32, 48)),  # one tile per wave with K = 32 steps: the runtime-trip-count K loop
]


@pytest.mark.parametrize("cin,cout,sp", SK_CASES)
def test_conv_sk_bf16(cin, cout, sp):
    """K-split small-grid bf16 kernel in the critic's three roles, against torch float64 within
    2e-2: forward with bias + LeakyReLU + BatchNorm statistics (weight-clip critic), the gradient
    penalty's forward-mode launch (mask = the output's previous contents, in place) and the
    input-grad with the layer below's LeakyReLU mask (discriminator.py:24-80)."""
    from cgan3d_amd import ops, _lib as L
    k, s, p, slope = 4, 2, 1, 0.2
    g = torch.Generator().manual_seed(21 + cin + cout + sp[0])
    n = 3
    x = torch.randn(n, cin, *sp, generator=g, dtype=torch.float64)
    w = torch.randn(cout, cin, k, k, k, generator=g, dtype=torch.float64) / np.sqrt(cin * k**3)
    b = torch.randn(cout, generator=g, dtype=torch.float64) * 0.1
    z = F.conv3d(x, w, b, stride=s, padding=p)
    yref = F.leaky_relu(z, slope)
    din, dout = tuple(sp), tuple(z.shape[2:])
    below = torch.randn(x.shape, generator=g, dtype=torch.float64)  # activations of the layer below
    gy = torch.randn(z.shape, generator=g, dtype=torch.float64)
    dx = torch.nn.grad.conv3d_input(x.shape, w, gy, stride=s, padding=p)
    dxref = torch.where(below > 0, dx, dx * slope)
    wd = w.float().cuda()
    ps = ops.PackSet(torch.device("cuda"))
    gf, wf = ps.add(ops.conv_fwd_geom(n, din, dout, cin, cout, k, s, p), wd, L.PREC_BF16)
    gd, wdp = ps.add(ops.conv_dgrad_geom(n, din, dout, cin, cout, k, s, p), wd, L.PREC_BF16)
    ps.pack()
    assert gf.w_packed == 3 and gd.w_packed == 3
    yo = torch.empty(n, *dout, cout, device="cuda")
    stats = torch.empty(ops.stats_floats(gf), device="cuda")
    ops.conv(gf, _cl(x), wf, yo, ops.epilogue(bias=b.float().cuda(), act=L.ACT_LRELU, slope=slope, stats=stats))
    assert_close(_ncdhw(yo).numpy(), yref.numpy(), 2e-2, "sk fwd")
    st = stats.double().cpu().view(-1, 2 * cout + 1)
    cnt = st[:, 2 * cout]
    tot = cnt.sum()
    mean = st[:, :cout].sum(0) / tot
    bm = st[:, :cout] / cnt.clamp(min=1)[:, None]
    m2 = st[:, cout:2 * cout].sum(0) + (cnt[:, None] * (bm - mean) ** 2).sum(0)
    yk = yo.double().cpu().view(-1, cout)
    assert int(tot) == yk.shape[0]
    assert_close(mean.numpy(), yk.mean(0).numpy(), 1e-4, "sk stats mean")
    assert_close((m2 / tot).numpy(), yk.var(0, unbiased=False).numpy(), 1e-4, "sk stats var")
    # gradient-penalty forward mode: nu = mask(y > 0) * conv(x) without bias, written over y
    nu = yo.clone()
    ops.conv(gf, _cl(x), wf, nu, ops.epilogue(mask_src=nu, slope=slope))
    zf = F.conv3d(x, w, stride=s, padding=p)
    nuref = torch.where(_ncdhw(yo) > 0, zf, zf * slope)
    assert_close(_ncdhw(nu).numpy(), nuref.numpy(), 2e-2, "sk forward-mode")
    dxo = torch.empty(n, *din, cin, device="cuda")
    ops.conv(gd, _cl(gy), wdp, dxo, ops.epilogue(mask_src=_cl(below), slope=slope))
    assert_close(_ncdhw(dxo).numpy(), dxref.numpy(), 2e-2, "sk dgrad")


@pytest.mark.parametrize("n,cin,cout,sp", [(12, 32, 64, (8, 8, 8)), (4, 32, 64, (8, 8, 8)), (2, 32, 64, (8, 8, 8)),
                                             (1, 32, 64, (8, 8, 8)), (3, 32, 64, (10, 8, 12))])
def test_conv_sk_n_split(n, cin, cout, sp):
    """N-split conv_sk (round 5): the critic's 32 -> 64 layer (K = 2048, few row tiles) with every
    block taking one 16-channel slice of its tile, in the forward (bias + LeakyReLU) and the gradient
    penalty's forward-mode (mask in place) roles.  Against torch float64 of the bf16-rounded operands
    at 1e-4 (fp32 accumulation of exact bf16 products) and of the unrounded ones within the bf16 bar."""
    from cgan3d_amd import ops, _lib as L
    k, s, p, slope = 4, 2, 1, 0.2
    g = torch.Generator().manual_seed(5 + n + cin + sp[0])
    x = torch.randn(n, cin, *sp, generator=g, dtype=torch.float64)
    w = torch.randn(cout, cin, k, k, k, generator=g, dtype=torch.float64) / np.sqrt(cin * k**3)
    b = torch.randn(cout, generator=g, dtype=torch.float64) * 0.1
    rb = lambda v: v.to(torch.bfloat16).double()  # noqa: E731
    z = F.conv3d(x, w, b, stride=s, padding=p)
    zb = F.conv3d(rb(x), rb(w), b.float().double(), stride=s, padding=p)
    din, dout = tuple(sp), tuple(z.shape[2:])
    ps = ops.PackSet(torch.device("cuda"))
    gf, wf = ps.add(ops.conv_fwd_geom(n, din, dout, cin, cout, k, s, p), w.float().cuda(), L.PREC_BF16)
    ps.pack()
    y = torch.full((n, *dout, cout), float("nan"), device="cuda")
    ops.conv(gf, _cl(x), wf, y, ops.epilogue(bias=b.float().cuda(), act=L.ACT_LRELU, slope=slope))
    nu = y.clone()
    ops.conv(gf, _cl(x), wf, nu, ops.epilogue(mask_src=nu, slope=slope))
    assert_close(_ncdhw(y).numpy(), F.leaky_relu(zb, slope).numpy(), 1e-4, "n-split fwd (bf16 operands)")
    assert_close(_ncdhw(y).numpy(), F.leaky_relu(z, slope).numpy(), 2e-2, "n-split fwd")
    # mask from the device's own forward output (a float64 z near 0 may differ in sign from the bf16 one)
    m = _ncdhw(y) > 0
    zf, zfb = F.conv3d(x, w, stride=s, padding=p), F.conv3d(rb(x), rb(w), stride=s, padding=p)
    assert_close(_ncdhw(nu).numpy(), torch.where(m, zfb, zfb * slope).numpy(), 1e-4, "n-split fwd-mode (bf16 operands)")
    assert_close(_ncdhw(nu).numpy(), torch.where(m, zf, zf * slope).numpy(), 2e-2, "n-split fwd-mode")


@pytest.mark.parametrize("n,cin,cout,sp", [(12, 8, 16, (32, 32, 32)), (12, 16, 32, (16, 16, 16)), (12, 32, 64, (8, 8, 8)),
                                             (3, 8, 16, (16, 32, 64)), (2, 32, 64, (16, 8, 8)), (12, 64, 1, (4, 4, 4)),
                                             (3, 64, 1, (3, 4, 2))])
def test_wgrad_sk_matches_float64(n, cin, cout, sp):
    """The staged-window critic weight gradient (round 5, cgan3d_conv3d_wgrad_sk): the three middle-layer
    variants (k4 s2, bf16 operands: against torch float64 of the bf16-rounded operands at 1e-4 relative
    L2 — fp32 accumulation of exact bf16 products — and the unrounded ones within the bf16 bar, 2e-2)
    and the last layer (64 -> 1 k4 s1, exact fp32: 1e-5 of float64); the result is ADDED into dW (a
    prefilled dW keeps its contents)."""
    from cgan3d_amd import ops, _lib as L
    k, p = 4, 1
    s = 1 if cout == 1 else 2
    g = torch.Generator().manual_seed(7 + n + cin + sp[1])
    x = torch.randn(n, cin, *sp, generator=g, dtype=torch.float64)
    dout = tuple(d // 2 for d in sp) if s == 2 else tuple(d - 1 for d in sp)
    dz = torch.randn(n, cout, *dout, generator=g, dtype=torch.float64)
    geo = ops.with_prec(ops.conv_wgrad_geom(n, tuple(sp), dout, cin, cout, k, s, p), L.PREC_BF16)
    assert ops.wgrad_sk_ok(geo)
    ws = torch.full((ops.wgrad_sk_ws_floats(geo),), float("nan"), device="cuda")  # any contents
    pre = torch.randn(cout, cin, k, k, k, generator=g).float().cuda()
    dw = pre.clone()
    ops.wgrad_sk([(geo, _cl(x), _cl(dz), ws, dw)])
    got = (dw - pre).double().cpu()
    want = torch.nn.grad.conv3d_weight(x, (cout, cin, k, k, k), dz, stride=s, padding=p)
    if cout == 1:  # exact fp32 last layer (fp32 operands)
        want32 = torch.nn.grad.conv3d_weight(x.float().double(), (cout, cin, k, k, k), dz.float().double(), stride=s,
                                             padding=p)
        assert float((got - want32).abs().max()) <= 1e-5 * float(want32.abs().max()) + 1e-6
        return
    rb = lambda t: t.float().bfloat16().double()  # noqa: E731
    want16 = torch.nn.grad.conv3d_weight(rb(x), (cout, cin, k, k, k), rb(dz), stride=s, padding=p)
    rel = float((got - want16).norm() / want16.norm())
    assert rel <= 1e-4, f"vs bf16-operand float64: rel L2 {rel:.2e}"
    assert_close(got.numpy(), want.numpy(), 2e-2, "wgrad_sk vs float64")


def test_adam_pack_matches_separate_launches():
    """cgan3d_adam_pack (step tick + Adam + repack of every packed format in one launch) leaves
    the same bits as cgan3d_adam_tick -> cgan3d_adam -> cgan3d_pack_weights_multi, over three
    steps through one ticket (which must stay zeroed)."""
    from torch import nn
    from cgan3d_amd import ops, _lib as L
    from cgan3d_amd.engine import Arena
    from cgan3d_amd.trainer.optim import FusedAdam
    torch.manual_seed(3)
    n = 2
    layers = [(16, 32, 3, 2, 1, (16, 16, 16), (8, 8, 8)),    # halo / stride-2 family (bf16 format 2)
              (64, 64, 3, 1, 1, (8, 8, 8), (8, 8, 8)),       # ResNet block (format 2)
              (8, 16, 4, 2, 1, (16, 16, 16), (8, 8, 8)),     # critic middle (format 3)
              (12, 20, 3, 1, 1, (5, 6, 7), (5, 6, 7))]       # generic (f32 format 1)
    mod = nn.Module()
    for i, (ci, co, k, s, p, di, do) in enumerate(layers):
        mod.register_parameter(f"w{i}", nn.Parameter(torch.randn(co, ci, k, k, k) * 0.1))
    mod.register_parameter("b", nn.Parameter(torch.randn(100)))
    runs = []
    for fused in (False, True):
        m2 = nn.Module()
        for k_, v in mod.named_parameters():
            m2.register_parameter(k_, nn.Parameter(v.detach().clone().cuda()))
        ar = Arena(m2, torch.device("cuda"))
        opt = FusedAdam(ar, 1e-3, (0.0, 0.9), 1e-8)
        ps = ops.PackSet(torch.device("cuda"))
        outs = []
        for i, (ci, co, k, s, p, di, do) in enumerate(layers):
            pc = L.PREC_BF16 if i < 3 else L.PREC_F32
            _, wp = ps.add(ops.conv_fwd_geom(n, di, do, ci, co, k, s, p), ar.views[f"w{i}"], pc)
            outs.append(wp)
        assert len(ps.descs) == 4
        g = torch.Generator(device="cuda").manual_seed(11)
        for _ in range(3):
            ar.grad.copy_(torch.randn(ar.numel, device="cuda", generator=g))
            if fused:
                opt.launch(packs=ps)
            else:
                ops.adam_tick(opt.hyper)
                ops.adam(ar.flat, ar.grad, ar.exp_avg, ar.exp_avg_sq, opt.hyper)
                ps.pack()
            assert torch.equal(opt.ticket.cpu(), torch.zeros(2, dtype=torch.int32))
        runs.append([ar.flat.clone(), ar.exp_avg.clone(), ar.exp_avg_sq.clone(), opt.hyper.clone()]
                    + [o.clone() for o in outs])
    assert float(runs[1][3][4]) == 3.0
    for j, (a, b) in enumerate(zip(*runs)):
        assert torch.equal(a, b), f"output {j}"


def test_copy_multi_and_batch_load():
    """cgan3d_copy_multi: vector body, byte tails, an unaligned small segment, a bool mask copied into
    uint8 bytes; and StepEngine.load_inputs' one-launch path fills the slots like torch copies."""
    from cgan3d_amd import ops
    g = torch.Generator(device="cpu").manual_seed(5)
    a = torch.randn(1000003, generator=g).cuda()
    b = torch.randint(0, 2, (777,), generator=g).bool().cuda()
    base = torch.randn(64, generator=g).cuda()
    c = base[1:6]  # 4-byte aligned only: bytewise segment
    da, db, dc = torch.empty_like(a), torch.empty(777, dtype=torch.uint8, device="cuda"), torch.empty(5, device="cuda")
    ops.copy_multi([(a, da), (b, db), (c, dc)])
    torch.cuda.synchronize()
    assert torch.equal(da, a) and torch.equal(db, b.to(torch.uint8)) and torch.equal(dc, c)
    with pytest.raises(ValueError):
        ops.copy_multi([(a, db)])
    # the engine's batch load: one launch for a bool mask, the torch copies for a float one
    from cgan3d_amd.data.synthetic import synth_patches
    from cgan3d_amd.engine import StepEngine
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.generator import ResnetGenerator
    from torch import nn
    S, n = 32, 2
    opt, _ = synth_patches(n, S, 3)
    sub, seg = synth_patches(n, S, 4)
    gm = ResnetGenerator(4, 2, 16).cuda()
    dm = PatchGANDiscriminator(1, 8, 3, negative_slope=0.2, norm_layer=nn.Identity).cuda()
    eng = StepEngine(gm, dm, gm.config, dm.config, n, n, (S, S, S))
    eps = torch.rand(n, device="cuda")
    for m in (torch.from_numpy(seg).cuda(), torch.from_numpy(seg).cuda().float()):
        eng.xc.zero_(), eng.subopt.zero_(), eng.mask.zero_(), eng.eps.zero_()
        eng.load_inputs(torch.from_numpy(opt).cuda(), torch.from_numpy(sub).cuda(), m, eps)
        torch.cuda.synchronize()
        assert torch.equal(eng.xc[:n].cpu().reshape(-1), torch.from_numpy(opt).reshape(-1))
        assert torch.equal(eng.subopt.cpu().reshape(-1), torch.from_numpy(sub).reshape(-1))
        assert torch.equal(eng.mask.cpu().reshape(-1), torch.from_numpy(seg).reshape(-1).to(torch.uint8))
        assert torch.equal(eng.eps.cpu(), eps.cpu())


K3M_CASES = [(2, (16, 16, 16)), (1, (6, 8, 10)), (2, (5, 7, 9)), (1, (9, 4, 17))]


@pytest.mark.parametrize("n,sp", K3M_CASES)
def test_conv_k3m_bf16(n, sp):
    """ResNet-block conv with every operand in LDS (conv_k3m.hip, 32x32x16 MFMA), as the bf16 step
    launches it: forward from the bf16 input shadow with a ReLU + residual epilogue and BatchNorm
    statistics into fp64 accumulators (cgan3d_bn_fuse mode 3), and the input-grad with the skip
    gradient and the BatchNorm-backward pairs (mode 4) — against float64 sums of the same bf16
    operands at 2e-5 (fp32 accumulation over 1728 terms), the statistics against the kernel's own
    outputs, and against conv_k3_kernel (tuning key 15 = 0: the same products, another fp32 order).
    Partial 4 x 4 x 8 tiles on every axis in the ragged cases."""
    from cgan3d_amd import ops, _lib as L
    cin = cout = 64
    g = torch.Generator().manual_seed(5 + sp[0])
    x = torch.randn(n, cin, *sp, generator=g, dtype=torch.float64).bfloat16().double()
    w = (torch.randn(cout, cin, 3, 3, 3, generator=g, dtype=torch.float64) / np.sqrt(cin * 27)).float()
    wq = w.bfloat16().double()
    res = torch.randn(n, cout, *sp, generator=g, dtype=torch.float64).float().double()
    gy = torch.randn(n, cout, *sp, generator=g, dtype=torch.float64).bfloat16().double()
    skip = torch.randn(n, cin, *sp, generator=g, dtype=torch.float64).float().double()
    yref = torch.relu(F.conv3d(x, wq, padding=1)) + res
    dxref = torch.nn.grad.conv3d_input(x.shape, wq, gy, padding=1) + skip
    ps = ops.PackSet(torch.device("cuda"))
    gf, wf = ps.add(ops.conv_fwd_geom(n, sp, sp, cin, cout, 3, 1, 1), w.cuda(), L.PREC_BF16)
    gd, wdp = ps.add(ops.conv_dgrad_geom(n, sp, sp, cin, cout, 3, 1, 1), w.cuda(), L.PREC_BF16)
    ps.pack()
    assert gf.w_packed == 2 and gd.w_packed == 2
    reps = 16
    # BatchNorm of the layer whose dL/dy the input-grad is (mode 4 pairs): its z, scale/shift, mean/invstd
    z = torch.randn(n, cin, *sp, generator=g, dtype=torch.float64).float()
    ss = torch.cat([torch.rand(cin, generator=g) + 0.5, torch.randn(cin, generator=g) * 0.1]).float()
    mi = torch.cat([torch.randn(cin, generator=g) * 0.1, torch.rand(cin, generator=g) + 0.5]).float()
    out = {}
    for key, flag in (("k3m", 1), ("k3", 0)):
        L.check(L.load().cgan3d_set_tuning(15, flag), "k3m switch")
        try:
            yo = torch.empty(n, *sp, cout, device="cuda")
            acc3 = torch.zeros(reps * 2 * cout, device="cuda", dtype=torch.float64)
            ops.conv(gf, _cl(x), wf, yo, ops.epilogue(act=L.ACT_RELU, residual=_cl(res), x_bf16=_cl(x).bfloat16(),
                                                      fuse=ops.BnFuse(acc3, 3, reps)))
            dxo = torch.empty(n, *sp, cin, device="cuda")
            acc4 = torch.zeros(reps * 2 * cin, device="cuda", dtype=torch.float64)
            ops.conv(gd, _cl(gy), wdp, dxo, ops.epilogue(residual=_cl(skip), x_bf16=_cl(gy).bfloat16(), bn_z=_cl(z),
                                                         bn_ss=ss.cuda(), bn_mi=mi.cuda(), bn_act=L.ACT_RELU,
                                                         fuse=ops.BnFuse(acc4, 4, reps)))
            torch.cuda.synchronize()
            out[key] = (yo.cpu(), acc3.cpu(), dxo.cpu(), acc4.cpu())
        finally:
            L.check(L.load().cgan3d_set_tuning(15, 1), "k3m on")
    yo, acc3, dxo, acc4 = out["k3m"]
    assert_close(_ncdhw(yo).numpy(), yref.numpy(), 2e-5, "k3m fwd")
    assert_close(_ncdhw(dxo).numpy(), dxref.numpy(), 2e-5, "k3m dgrad")
    for a, b_, nm in zip(out["k3m"], out["k3"], ("fwd", "acc3", "dgrad", "acc4")):
        if nm.startswith("acc"):  # the two grids spread their blocks over the replicas differently
            a, b_ = a.view(reps, -1).sum(0), b_.view(reps, -1).sum(0)
        assert_close(a.double().numpy(), b_.double().numpy(), 1e-5, f"k3m vs k3 {nm}")
    yk = yo.double().view(-1, cout)
    a3 = acc3.view(reps, 2, cout).sum(0)
    assert_close(a3[0].numpy(), yk.sum(0).numpy(), 1e-5, "mode-3 sum")
    assert_close(a3[1].numpy(), (yk * yk).sum(0).numpy(), 1e-5, "mode-3 sum of squares")
    zk = z.permute(0, 2, 3, 4, 1).reshape(-1, cin).double()
    gk = dxo.double().view(-1, cin)
    pre = zk * ss[:cin].double() + ss[cin:].double()
    gg = gk * (pre > 0).double()
    a4 = acc4.view(reps, 2, cin).sum(0)
    assert_close(a4[0].numpy(), gg.sum(0).numpy(), 1e-5, "mode-4 sum g")
    assert_close(a4[1].numpy(), (gg * (zk - mi[:cin].double()) * mi[cin:].double()).sum(0).numpy(), 1e-5,
                 "mode-4 sum g xhat")


@pytest.mark.parametrize("n,sp", K3M_CASES)
@pytest.mark.parametrize("act", ["relu", "none"])
def test_conv_k3m_bn_prologue(n, sp, act):
    """The ResNet chain's BatchNorm passes folded into the next conv (round 5, cgan3d_bn_pre): the
    forward (mode 1: staged z -> act(BN(z)), statistics finalized from the fp64 replicas in every
    block) and the input-grad (mode 2: staged dL/dy -> BatchNorm backward dL/dz) must give exactly the
    bits of the unfused pair (cgan3d_bn_apply_acc / cgan3d_bn_backward_acc, then conv_k3m): the conv
    output, its own accumulator statistics, the materialised operand (out_bf16, every voxel), the
    published scale / shift / mean / invstd / running buffers / dgamma / dbeta and the zeroed
    accumulator.  Ragged tiles on every axis in the K3M_CASES shapes."""
    from cgan3d_amd import ops, _lib as L
    c = 64
    A = L.ACT_RELU if act == "relu" else L.ACT_NONE
    g = torch.Generator().manual_seed(11 + sp[0] + n)
    dev = torch.device("cuda")
    nv = n * sp[0] * sp[1] * sp[2]
    w = (torch.randn(c, c, 3, 3, 3, generator=g, dtype=torch.float64) / np.sqrt(c * 27)).float()
    ps = ops.PackSet(dev)
    gf, wf = ps.add(ops.conv_fwd_geom(n, sp, sp, c, c, 3, 1, 1), w.cuda(), L.PREC_BF16)
    gd, wdp = ps.add(ops.conv_dgrad_geom(n, sp, sp, c, c, 3, 1, 1), w.cuda(), L.PREC_BF16)
    ps.pack()
    assert ops.bn_pre_ok(gf) and ops.bn_pre_ok(gd)
    reps = 16
    # z of the previous BatchNorm layer (bf16, as the chain keeps it), shifted so the mean matters
    z16 = (torch.randn(n, *sp, c, generator=g) * 1.7 + 0.4).to(dev).bfloat16()
    zk = z16.double().view(-1, c)
    acc3 = torch.zeros(reps, 2, c, dtype=torch.float64, device=dev)
    acc3[3, 0], acc3[3, 1] = zk.sum(0), (zk * zk).sum(0)  # one replica holds it all (any split sums alike)
    acc3 = acc3.view(-1)
    gamma = (torch.rand(c, generator=g) + 0.5).to(dev)
    beta = (torch.randn(c, generator=g) * 0.2).to(dev)

    def bufs():
        return (torch.zeros(c, device=dev) + 0.1, torch.ones(c, device=dev) * 0.9,
                torch.zeros((), dtype=torch.int64, device=dev))
    # --- forward: reference pair
    rm0, rv0, nb0 = bufs()
    ss0, mi0 = torch.empty(2 * c, device=dev), torch.empty(2 * c, device=dev)
    h16 = torch.empty(n, *sp, c, device=dev, dtype=torch.bfloat16)
    zero0 = torch.ones(300, dtype=torch.float64, device=dev)
    ops.bn_apply_acc(acc3, reps, c, nv, gamma, beta, rm0, rv0, nb0, ss0, mi0, z16, A, None, y16=h16, zero=zero0)
    y0 = torch.empty(n, *sp, c, device=dev, dtype=torch.bfloat16)
    accn0 = torch.zeros(reps * 2 * c, device=dev, dtype=torch.float64)
    ops.conv(gf, h16.float(), wf, y0, ops.epilogue(x_bf16=h16, fuse=ops.BnFuse(accn0, 3, reps)))
    # --- forward: folded
    rm1, rv1, nb1 = bufs()
    ss1, mi1 = torch.empty(2 * c, device=dev), torch.empty(2 * c, device=dev)
    h16f = torch.full_like(h16, float("nan"))
    zero1 = torch.ones(300, dtype=torch.float64, device=dev)
    y1 = torch.empty_like(y0)
    accn1 = torch.zeros_like(accn0)
    pre = ops.BnPre.forward(acc3, reps, c, nv, gamma, beta, rm1, rv1, nb1, ss1, mi1, A, h16f, zero=zero1)
    ops.conv(gf, z16.float(), wf, y1, ops.epilogue(x_bf16=z16, fuse=ops.BnFuse(accn1, 3, reps), pre=pre))
    torch.cuda.synchronize()
    assert torch.equal(h16f, h16), "folded forward: materialised operand"
    assert torch.equal(y1, y0), "folded forward: conv output"
    # fp64 atomics from many blocks: the sums agree up to their order of arrival
    torch.testing.assert_close(accn1.view(reps, -1).sum(0), accn0.view(reps, -1).sum(0), rtol=1e-12, atol=1e-9)
    for a_, b_, nm in ((ss1, ss0, "scale_shift"), (mi1, mi0, "mean_invstd"), (rm1, rm0, "running_mean"),
                       (rv1, rv0, "running_var"), (nb1, nb0, "num_batches_tracked"), (zero1, zero0, "zero")):
        assert torch.equal(a_, b_), f"folded forward: {nm}"
    assert int(nb1) == 1 and float(zero1.abs().max()) == 0.0
    # --- input-grad: dL/dy of this BatchNorm layer (bf16), its (sum g, sum g*xhat) replicas
    dy16 = torch.randn(n, *sp, c, generator=g).to(dev).bfloat16()
    sc, sh, mu, inv = ss0[:c].double(), ss0[c:].double(), mi0[:c].double(), mi0[c:].double()
    gk = dy16.double().view(-1, c) * ((zk * sc + sh > 0).double() if act == "relu" else 1.0)
    acc4 = torch.zeros(reps, 2, c, dtype=torch.float64, device=dev)
    acc4[7, 0], acc4[7, 1] = gk.sum(0), (gk * (zk - mu) * inv).sum(0)
    acc4 = acc4.view(-1)
    skip = torch.randn(n, *sp, c, generator=g).to(dev)
    dg0, db0 = torch.full((c,), 0.25, device=dev), torch.full((c,), -0.5, device=dev)
    dz16 = torch.empty_like(z16)
    zb0 = torch.ones(200, dtype=torch.float64, device=dev)
    ops.bn_backward_acc(dy16, z16, nv, c, acc4, reps, ss0, mi0, gamma, A, dg0, db0, None, accumulate=True, dz16=dz16,
                        zero=zb0)
    dx0 = torch.empty(n, *sp, c, device=dev)
    ops.conv(gd, dz16.float(), wdp, dx0, ops.epilogue(residual=skip, x_bf16=dz16))
    dg1, db1 = torch.full((c,), 0.25, device=dev), torch.full((c,), -0.5, device=dev)
    dz16f = torch.full_like(dz16, float("nan"))
    zb1 = torch.ones(200, dtype=torch.float64, device=dev)
    dx1 = torch.empty_like(dx0)
    pre = ops.BnPre.backward(z16, acc4, reps, c, nv, ss0, mi0, gamma, A, dg1, db1, dz16f, accumulate=True, zero=zb1)
    ops.conv(gd, dy16.float(), wdp, dx1, ops.epilogue(residual=skip, x_bf16=dy16, pre=pre))
    torch.cuda.synchronize()
    assert torch.equal(dz16f, dz16), "folded input-grad: materialised operand"
    assert torch.equal(dx1, dx0), "folded input-grad: conv output"
    for a_, b_, nm in ((dg1, dg0, "dgamma"), (db1, db0, "dbeta"), (zb1, zb0, "zero")):
        assert torch.equal(a_, b_), f"folded input-grad: {nm}"


@pytest.mark.parametrize("n,sp", [(2, (16, 16, 16)), (1, (5, 6, 9))])
def test_conv_k3m_bf16_storage(n, sp):
    """conv_k3m with bf16 storage (cgan3d_epilogue.out_bf16, the ResNet chain's engine.zs / dys): a
    bf16 output and mode-4 bn_z (bit 0) and a bf16 skip gradient (bit 1) against the fp32-storage
    launch on the same (bf16-representable) operands: the outputs are its fp32 values rounded to
    bf16 bit for bit, the fp64 statistics equal up to summation order (they come from the fp32
    registers either way)."""
    from cgan3d_amd import ops, _lib as L
    c = 64
    g = torch.Generator().manual_seed(11 + sp[1])
    x = torch.randn(n, c, *sp, generator=g, dtype=torch.float64).bfloat16().float()
    w = (torch.randn(c, c, 3, 3, 3, generator=g, dtype=torch.float64) / np.sqrt(c * 27)).float()
    skip = torch.randn(n, c, *sp, generator=g, dtype=torch.float64).bfloat16().float()
    z = torch.randn(n, c, *sp, generator=g, dtype=torch.float64).bfloat16().float()
    ss = torch.cat([torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.1]).float().cuda()
    mi = torch.cat([torch.randn(c, generator=g) * 0.1, torch.rand(c, generator=g) + 0.5]).float().cuda()
    ps = ops.PackSet(torch.device("cuda"))
    gf, wf = ps.add(ops.conv_fwd_geom(n, sp, sp, c, c, 3, 1, 1), w.cuda(), L.PREC_BF16)
    gd, wdp = ps.add(ops.conv_dgrad_geom(n, sp, sp, c, c, 3, 1, 1), w.cuda(), L.PREC_BF16)
    ps.pack()
    assert ops.out_bf16_ok(gf) and ops.out_bf16_ok(gd)
    reps = 16
    xs = _cl(x).bfloat16()
    runs = {}
    for key, yd, zd, rd in (("fp32", torch.float32, torch.float32, torch.float32),
                            ("bf16", torch.bfloat16, torch.bfloat16, torch.bfloat16),
                            ("res16", torch.float32, torch.float32, torch.bfloat16)):
        yo = torch.empty(n, *sp, c, device="cuda", dtype=yd)
        acc3 = torch.zeros(reps * 2 * c, device="cuda", dtype=torch.float64)
        ops.conv(gf, _cl(x), wf, yo, ops.epilogue(x_bf16=xs, fuse=ops.BnFuse(acc3, 3, reps)))
        dxo = torch.empty(n, *sp, c, device="cuda", dtype=yd)
        acc4 = torch.zeros(reps * 2 * c, device="cuda", dtype=torch.float64)
        ops.conv(gd, _cl(x), wdp, dxo, ops.epilogue(residual=_cl(skip).to(rd), x_bf16=xs, bn_z=_cl(z).to(zd),
                                                    bn_ss=ss, bn_mi=mi, bn_act=L.ACT_RELU,
                                                    fuse=ops.BnFuse(acc4, 4, reps)))
        torch.cuda.synchronize()
        runs[key] = (yo.cpu(), acc3.cpu(), dxo.cpu(), acc4.cpu())
    f, b, r = runs["fp32"], runs["bf16"], runs["res16"]
    assert torch.equal(b[0], f[0].bfloat16()), "bf16 forward output != rounded fp32 output"
    assert torch.equal(b[2], f[2].bfloat16()), "bf16 input-grad output != rounded fp32 output"
    # the fp64 atomics land in launch-dependent order: equal up to fp64 summation order
    for a_, b_, nm in ((b[1], f[1], "mode-3"), (b[3], f[3], "mode-4"), (r[3], f[3], "mode-4, bf16 residual")):
        assert_close(a_.view(reps, -1).sum(0).numpy(), b_.view(reps, -1).sum(0).numpy(), 1e-12, f"{nm} statistics")
    assert torch.equal(r[2], f[2]), "bf16 residual alone changed the input-grad"
    # a bf16 residual on a geometry other than the ResNet-block kernel is refused
    with pytest.raises(Exception):
        g2 = ops.conv_fwd_geom(n, sp, sp, c, c, 1, 1, 0)
        ops.conv(g2, _cl(x), w[:, :, :1, :1, :1].contiguous().cuda(), torch.empty(n, *sp, c, device="cuda"),
                 ops.epilogue(residual=_cl(skip).bfloat16()))


@pytest.mark.parametrize("n,sp", [(2, (16, 16, 16)), (1, (5, 4, 8)), (2, (3, 8, 24)), (1, (7, 12, 16))])
def test_wgrad_k3m_bf16(n, sp):
    """ResNet-block weight gradient from the bf16 shadows (wgrad_k3m_kernel: LDS-DMA stages, 32x32x16
    MFMA on transposed LDS reads, per-chunk partials + wgrad_reduce_lin_kernel) against float64 sums
    of the same bf16 operands at 2e-5, against wgrad_k3_kernel (tuning key 16 = 0: the same products,
    another fp32 order) at 1e-5, and the accumulate mode; chunks ending inside a stage and volume
    edges on every axis in the small cases."""
    from cgan3d_amd import ops, _lib as L
    cin = cout = 64
    g = torch.Generator().manual_seed(3 + sp[2])
    x = torch.randn(n, cin, *sp, generator=g, dtype=torch.float64).bfloat16().double()
    gy = torch.randn(n, cout, *sp, generator=g, dtype=torch.float64).bfloat16().double()
    w = torch.zeros(cout, cin, 3, 3, 3, dtype=torch.float64, requires_grad=True)
    y = F.conv3d(x, w, padding=1)
    dw, = torch.autograd.grad(y, (w,), gy)
    gw = ops.with_prec(ops.conv_wgrad_geom(n, sp, sp, cin, cout, 3, 1, 1), L.PREC_BF16)
    ws = torch.empty(ops.wgrad_ws_floats(gw), device="cuda")
    out = {}
    for key, flag in (("k3m", 1), ("k3", 0)):
        L.check(L.load().cgan3d_set_tuning(16, flag), "wk3m switch")
        try:
            dwo = torch.empty(w.shape, device="cuda")
            ops.wgrad(gw, _cl(x), _cl(gy), dwo, ws, gathered16=_cl(x).bfloat16(), aligned16=_cl(gy).bfloat16())
            torch.cuda.synchronize()
            out[key] = dwo.cpu()
        finally:
            L.check(L.load().cgan3d_set_tuning(16, 1), "wk3m on")
    assert_close(out["k3m"].double().numpy(), dw.numpy(), 2e-5, "wk3m vs fp64")
    assert_close(out["k3m"].double().numpy(), out["k3"].double().numpy(), 1e-5, "wk3m vs wgrad_k3_kernel")
    dwa = out["k3m"].cuda()
    ops.wgrad(gw, _cl(x), _cl(gy), dwa, ws, accumulate=True, gathered16=_cl(x).bfloat16(),
              aligned16=_cl(gy).bfloat16())
    assert_close(dwa.double().cpu().numpy(), 2 * dw.numpy(), 2e-5, "wk3m accumulate")


@pytest.mark.parametrize("n,din", [(2, (16, 16, 16)), (1, (5, 6, 7)), (3, (8, 4, 12))])
@pytest.mark.parametrize("role", ["convt_fwd", "conv_dgrad"])
def test_conv_t64_bf16(n, din, role):
    """The 32 <-> 64 level's stride-2 transposed conv with all eight parity classes per block (round 5,
    conv_t64.hip): ConvTranspose3d 64 -> 32 forward (output padding 1) and the input-grad of the
    Conv3d 32 -> 64 stride-2 (the same mapping).  Against torch float64 of the same bf16 operands at
    2e-5 (fp32 accumulation of exact products), a bf16 output equal to the fp32 one rounded, the mode-3
    statistics against the output's own sums and the mode-4 pairs against a float64 restatement.
    Ragged class tiles in the second and third shapes."""
    from cgan3d_amd import ops, _lib as L
    g = torch.Generator().manual_seed(3 + n + din[0])
    dout = tuple(2 * d for d in din)
    x = torch.randn(n, 64, *din, generator=g, dtype=torch.float64).bfloat16().double()
    if role == "convt_fwd":  # ConvTranspose3d weight [in 64, out 32, k, k, k]
        w = (torch.randn(64, 32, 3, 3, 3, generator=g, dtype=torch.float64) / np.sqrt(64 * 8)).float()
        yref = F.conv_transpose3d(x, w.bfloat16().double(), stride=2, padding=1, output_padding=1)
        geo0 = ops.convt_fwd_geom(n, din, dout, 64, 32, 3, 2, 1)
    else:  # Conv3d 32 -> 64 stride 2 (weight [64, 32, k, k, k]); its input-grad from dL/dz at din
        w = (torch.randn(64, 32, 3, 3, 3, generator=g, dtype=torch.float64) / np.sqrt(64 * 8)).float()
        yref = torch.nn.grad.conv3d_input((n, 32, *dout), w.bfloat16().double(), x, stride=2, padding=1)
        geo0 = ops.conv_dgrad_geom(n, dout, din, 32, 64, 3, 2, 1)
    ps = ops.PackSet(torch.device("cuda"))
    geo, wp = ps.add(geo0, w.cuda(), L.PREC_BF16)
    ps.pack()
    assert geo.w_packed == 2 and geo.transposed and geo.cin == 64 and geo.cout == 32
    xc, x16 = _cl(x), _cl(x).bfloat16()
    reps = 16
    y = torch.empty(n, *dout, 32, device="cuda")
    acc3 = torch.zeros(reps * 2 * 32, device="cuda", dtype=torch.float64)
    ops.conv(geo, xc, wp, y, ops.epilogue(x_bf16=x16, fuse=ops.BnFuse(acc3, 3, reps)))
    assert_close(_ncdhw(y).numpy(), yref.numpy(), 2e-5, "t64 output")
    yk = y.double().view(-1, 32).cpu()
    a3 = acc3.view(reps, 2, 32).sum(0).cpu()
    assert_close(a3[0].numpy(), yk.sum(0).numpy(), 1e-5, "t64 mode-3 sum")
    assert_close(a3[1].numpy(), (yk * yk).sum(0).numpy(), 1e-5, "t64 mode-3 sum of squares")
    y16 = torch.empty(n, *dout, 32, device="cuda", dtype=torch.bfloat16)
    ops.conv(geo, xc, wp, y16, ops.epilogue(x_bf16=x16, fuse=ops.BnFuse(torch.zeros_like(acc3), 3, reps)))
    assert torch.equal(y16, y.bfloat16()), "t64 bf16 output"
    # mode 4: the BatchNorm-backward pairs of the layer whose dL/dy this is
    z = torch.randn(n, *dout, 32, generator=g).cuda()
    ss = torch.cat([torch.rand(32, generator=g) + 0.5, torch.randn(32, generator=g) * 0.1]).cuda()
    mi = torch.cat([torch.randn(32, generator=g) * 0.1, torch.rand(32, generator=g) + 0.5]).cuda()
    acc4 = torch.zeros_like(acc3)
    y4 = torch.empty_like(y)
    ops.conv(geo, xc, wp, y4, ops.epilogue(x_bf16=x16, bn_z=z, bn_ss=ss, bn_mi=mi, bn_act=L.ACT_RELU,
                                           fuse=ops.BnFuse(acc4, 4, reps)))
    assert torch.equal(y4, y)
    zk, ssd, mid = z.double().view(-1, 32).cpu(), ss.double().cpu(), mi.double().cpu()
    gg = yk * ((zk * ssd[:32] + ssd[32:]) > 0).double()
    a4 = acc4.view(reps, 2, 32).sum(0).cpu()
    assert_close(a4[0].numpy(), gg.sum(0).numpy(), 1e-5, "t64 mode-4 sum g")
    assert_close(a4[1].numpy(), (gg * (zk - mid[:32]) * mid[32:]).sum(0).numpy(), 1e-5, "t64 mode-4 sum g xhat")
    # out_bf16 bit 0 with mode 4 (the step's bf16 dL/dy storage): bf16 output and bf16 z, the pairs from
    # the fp32 values and the stored z
    z16 = z.bfloat16()
    acc4b = torch.zeros_like(acc3)
    y4b = torch.empty(n, *dout, 32, device="cuda", dtype=torch.bfloat16)
    ops.conv(geo, xc, wp, y4b, ops.epilogue(x_bf16=x16, bn_z=z16, bn_ss=ss, bn_mi=mi, bn_act=L.ACT_RELU,
                                            fuse=ops.BnFuse(acc4b, 4, reps)))
    assert torch.equal(y4b, y.bfloat16()), "t64 bf16 output, mode 4"
    zb = z16.double().view(-1, 32).cpu()
    ggb = yk * ((zb * ssd[:32] + ssd[32:]) > 0).double()
    a4b = acc4b.view(reps, 2, 32).sum(0).cpu()
    assert_close(a4b[0].numpy(), ggb.sum(0).numpy(), 1e-5, "t64 bf16 mode-4 sum g")
    assert_close(a4b[1].numpy(), (ggb * (zb - mid[:32]) * mid[32:]).sum(0).numpy(), 1e-5, "t64 bf16 mode-4 sum g xhat")


@pytest.mark.parametrize("n,din", [(2, (32, 32, 32)), (1, (9, 12, 14)), (2, (17, 8, 24))])
@pytest.mark.parametrize("role", ["conv_fwd", "convt_dgrad"])
def test_conv_f64_bf16(n, din, role):
    """The 32 <-> 64 level's stride-2 conv 32 -> 64 with every operand in LDS (round 5, conv_f64.hip):
    the Conv3d forward (k3 s2 p1) and the input-grad of the ConvTranspose3d 64 -> 32 (the same
    mapping).  Against torch float64 of the same bf16 operands at 2e-5, a bf16 output equal to the
    fp32 one rounded, mode-3 statistics against the output's own sums and mode-4 pairs against a
    float64 restatement.  Ragged output tiles (and odd input extents) in the last two shapes."""
    from cgan3d_amd import ops, _lib as L
    g = torch.Generator().manual_seed(7 + n + din[0])
    dout = tuple((d - 1) // 2 + 1 for d in din)
    x = torch.randn(n, 32, *din, generator=g, dtype=torch.float64).bfloat16().double()
    if role == "conv_fwd":  # Conv3d weight [out 64, in 32, k, k, k]
        w = (torch.randn(64, 32, 3, 3, 3, generator=g, dtype=torch.float64) / np.sqrt(32 * 27)).float()
        yref = F.conv3d(x, w.bfloat16().double(), stride=2, padding=1)
        geo0 = ops.conv_fwd_geom(n, din, dout, 32, 64, 3, 2, 1)
    else:  # ConvTranspose3d 64 -> 32 (weight [in 64, out 32, k, k, k]) from dout to din; its input-grad
        w = (torch.randn(64, 32, 3, 3, 3, generator=g, dtype=torch.float64) / np.sqrt(32 * 27)).float()
        yref = F.conv3d(x, w.bfloat16().double(), stride=2, padding=1)  # the adjoint of conv_transpose3d
        geo0 = ops.convt_dgrad_geom(n, dout, din, 64, 32, 3, 2, 1)
    assert tuple(yref.shape[2:]) == dout
    ps = ops.PackSet(torch.device("cuda"))
    geo, wp = ps.add(geo0, w.cuda(), L.PREC_BF16)
    ps.pack()
    assert geo.w_packed == 2 and not geo.transposed and geo.cin == 32 and geo.cout == 64
    xc, x16 = _cl(x), _cl(x).bfloat16()
    reps = 16
    y = torch.empty(n, *dout, 64, device="cuda")
    acc3 = torch.zeros(reps * 2 * 64, device="cuda", dtype=torch.float64)
    ops.conv(geo, xc, wp, y, ops.epilogue(x_bf16=x16, fuse=ops.BnFuse(acc3, 3, reps)))
    assert_close(_ncdhw(y).numpy(), yref.numpy(), 2e-5, "f64 output")
    yk = y.double().view(-1, 64).cpu()
    a3 = acc3.view(reps, 2, 64).sum(0).cpu()
    assert_close(a3[0].numpy(), yk.sum(0).numpy(), 1e-5, "f64 mode-3 sum")
    assert_close(a3[1].numpy(), (yk * yk).sum(0).numpy(), 1e-5, "f64 mode-3 sum of squares")
    y16 = torch.empty(n, *dout, 64, device="cuda", dtype=torch.bfloat16)
    ops.conv(geo, xc, wp, y16, ops.epilogue(x_bf16=x16, fuse=ops.BnFuse(torch.zeros_like(acc3), 3, reps)))
    assert torch.equal(y16, y.bfloat16()), "f64 bf16 output"
    z = torch.randn(n, *dout, 64, generator=g).cuda()
    ss = torch.cat([torch.rand(64, generator=g) + 0.5, torch.randn(64, generator=g) * 0.1]).cuda()
    mi = torch.cat([torch.randn(64, generator=g) * 0.1, torch.rand(64, generator=g) + 0.5]).cuda()
    acc4 = torch.zeros_like(acc3)
    y4 = torch.empty_like(y)
    ops.conv(geo, xc, wp, y4, ops.epilogue(x_bf16=x16, bn_z=z, bn_ss=ss, bn_mi=mi, bn_act=L.ACT_RELU,
                                           fuse=ops.BnFuse(acc4, 4, reps)))
    assert torch.equal(y4, y)
    zk, ssd, mid = z.double().view(-1, 64).cpu(), ss.double().cpu(), mi.double().cpu()
    gg = yk * ((zk * ssd[:64] + ssd[64:]) > 0).double()
    a4 = acc4.view(reps, 2, 64).sum(0).cpu()
    assert_close(a4[0].numpy(), gg.sum(0).numpy(), 1e-5, "f64 mode-4 sum g")
    assert_close(a4[1].numpy(), (gg * (zk - mid[:64]) * mid[64:]).sum(0).numpy(), 1e-5, "f64 mode-4 sum g xhat")
    # out_bf16 bit 0 with mode 4 (the step's bf16 dL/dy storage): bf16 output and bf16 z, the pairs from
    # the fp32 values and the stored z
    z16 = z.bfloat16()
    acc4b = torch.zeros_like(acc3)
    y4b = torch.empty(n, *dout, 64, device="cuda", dtype=torch.bfloat16)
    ops.conv(geo, xc, wp, y4b, ops.epilogue(x_bf16=x16, bn_z=z16, bn_ss=ss, bn_mi=mi, bn_act=L.ACT_RELU,
                                            fuse=ops.BnFuse(acc4b, 4, reps)))
    assert torch.equal(y4b, y.bfloat16()), "f64 bf16 output, mode 4"
    zb = z16.double().view(-1, 64).cpu()
    ggb = yk * ((zb * ssd[:64] + ssd[64:]) > 0).double()
    a4b = acc4b.view(reps, 2, 64).sum(0).cpu()
    assert_close(a4b[0].numpy(), ggb.sum(0).numpy(), 1e-5, "f64 bf16 mode-4 sum g")
    assert_close(a4b[1].numpy(), (ggb * (zb - mid[:64]) * mid[64:]).sum(0).numpy(), 1e-5, "f64 bf16 mode-4 sum g xhat")


@pytest.mark.parametrize("n,sp,c", [(2, (12, 16, 16), 16), (1, (10, 9, 64), 16), (2, (9, 7, 8), 32),
                                    (2, (8, 12, 12), 16)])
@pytest.mark.parametrize("act", ["relu", "lrelu"])
def test_bn_backward_fold_rows(n, sp, c, act):
    """The generator's last BatchNorm backward with the reflect-pad fold (round 5c row kernel, bf16
    operands) gives exactly the bits of the grid-stride kernel run on the same values in fp32: dz16, dz,
    dgamma / dbeta (accumulated) and the zeroed accumulator.  (2, (8, 12, 12), 16) has 24 granules per
    row, not a power of two: the grid-stride fallback."""
    from cgan3d_amd import ops, _lib as L
    A, slope = (L.ACT_RELU, 0.0) if act == "relu" else (L.ACT_LRELU, 0.2)
    g = torch.Generator().manual_seed(5 + sp[2] + c)
    dev = torch.device("cuda")
    p, reps = 3, 16
    pad_sp = tuple(d + 2 * p for d in sp)
    padded16 = torch.randn(n, *pad_sp, c, generator=g).to(dev).bfloat16()
    z16 = (torch.randn(n, *sp, c, generator=g) * 1.3 + 0.2).to(dev).bfloat16()
    acc = torch.zeros(reps, 2, c, dtype=torch.float64, device=dev)
    acc[5, 0] = torch.randn(c, generator=g, dtype=torch.float64).to(dev) * 50
    acc[9, 1] = torch.randn(c, generator=g, dtype=torch.float64).to(dev) * 50
    acc = acc.view(-1)
    ss = torch.cat([torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.3]).to(dev)
    mi = torch.cat([torch.randn(c, generator=g) * 0.2, torch.rand(c, generator=g) + 0.7]).to(dev)
    gamma = (torch.rand(c, generator=g) + 0.5).to(dev)
    out = []
    for in16 in (True, False):
        pd, zz = (padded16, z16) if in16 else (padded16.float(), z16.float())
        dg, db = torch.full((c,), 0.25, device=dev), torch.full((c,), -0.5, device=dev)
        dz = torch.full((n, *sp, c), float("nan"), device=dev)
        dz16 = torch.full((n, *sp, c), float("nan"), device=dev, dtype=torch.bfloat16)
        zero = torch.ones(100, dtype=torch.float64, device=dev)
        ops.bn_backward_acc_fold(pd, zz, n, sp, c, p, acc, reps, ss, mi, gamma, A, dg, db, dz, slope=slope,
                                 accumulate=True, dz16=dz16, zero=zero)
        out.append((dz16, dz, dg, db, zero))
    torch.cuda.synchronize()
    for a_, b_, nm in zip(out[0], out[1], ("dz16", "dz", "dgamma", "dbeta", "zero")):
        assert torch.equal(a_, b_), nm
    assert float(out[0][4].abs().max()) == 0.0
    # dz16-only (the step's form) matches too
    dz16b = torch.empty_like(z16)
    ops.bn_backward_acc_fold(padded16, z16, n, sp, c, p, acc, reps, ss, mi, gamma, A, torch.zeros(c, device=dev),
                             torch.zeros(c, device=dev), None, slope=slope, dz16=dz16b)
    torch.cuda.synchronize()
    assert torch.equal(dz16b, out[0][0])
