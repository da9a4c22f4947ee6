"""Fused BatchNorm statistics (include/cgan3d.h cgan3d_epilogue bn_part / bn_mode,
cgan3d_bn_finalize_slab, cgan3d_bn_backward_slab, cgan3d_reflect_fold_ex).

The per-block partial pairs each producing kernel writes into its slab are summed and checked
against the same sums of that kernel's own output (float64, 1e-4: fp32 partials); the BatchNorm
forward / backward built on them against torch autograd (float64) within 1e-3, as the two-pass
path in test_gpu_ops.test_batchnorm_train_forward_backward (model/blocks.py:26-27,45-53).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import assert_close

pytestmark = pytest.mark.gpu


def _cl(t):
    return t.permute(0, 2, 3, 4, 1).contiguous().float().cuda()


def _ncdhw(t):
    return t.double().cpu().permute(0, 4, 1, 2, 3)


def _pairs(out, c, z=None, ss=None, mi=None, act=0):
    """(sum, sum of squares) of out, or (sum g, sum g*xhat) with g = out * act'(z*scale + shift)."""
    o = out.double().cpu().reshape(-1, c)
    if z is None:
        return torch.cat([o.sum(0), (o * o).sum(0)])
    zz = z.double().cpu().reshape(-1, c)
    ssd, mid = ss.double().cpu(), mi.double().cpu()
    pre = zz * ssd[:c] + ssd[c:]
    gg = o * ((pre > 0).double() if act == 1 else 1.0)
    xh = (zz - mid[:c]) * mid[c:]
    return torch.cat([gg.sum(0), (gg * xh).sum(0)])


# producer kinds: (name, precision, geometry builder, cin, cout, k, s, p, reflect, spatial)
PRODUCERS = [
    ("gemm_f32", 0, 8, 16, 3, 1, 1, False, (6, 8, 10)),
    ("gemm_bf16", 1, 16, 32, 3, 2, 1, False, (8, 12, 16)),
    ("halo_bf16", 1, 64, 64, 3, 1, 1, False, (6, 8, 10)),
    ("k7_f32", 0, 1, 16, 7, 1, 3, True, (8, 12, 16)),
    ("k7m_bf16", 1, 1, 16, 7, 1, 3, True, (12, 16, 20)),
]


@pytest.mark.parametrize("name,prec,cin,cout,k,s,p,reflect,sp", PRODUCERS)
def test_fused_forward_statistics(name, prec, cin, cout, k, s, p, reflect, sp, monkeypatch):
    from cgan3d_amd import ops
    monkeypatch.setattr(ops, "HALO", name.startswith("halo"))
    g = torch.Generator().manual_seed(5 + cin + cout)
    n = 2
    dout = tuple((d + 2 * p - k) // s + 1 for d in sp)
    geo = ops.with_prec(ops.conv_fwd_geom(n, sp, dout, cin, cout, k, s, p, reflect), prec)
    w = (torch.randn(cout, cin, k, k, k, generator=g) / np.sqrt(cin * k**3)).cuda()
    if k != 7:
        ps = ops.PackSet(torch.device("cuda"))
        geo, w = ps.add(geo, w, prec)
        ps.pack()
    if k != 7:
        assert (geo.w_packed == 2) == name.startswith("halo"), "unexpected kernel choice"
    x = _cl(torch.randn(n, cin, *sp, generator=g))
    y = torch.empty(n, *dout, cout, device="cuda")
    slots = ops.bn_slots(geo)
    part = torch.full(((2 * cout + 1) * slots,), float("nan"), device="cuda")  # every slot must be written
    ops.conv(geo, x, w, y, ops.epilogue(bn_part=part, bn_mode=1, bn_slots=slots))
    sl = part.double().cpu().view(2 * cout + 1, slots)
    cnt = sl[2 * cout]
    tot = cnt.sum()
    yk = y.double().cpu().reshape(-1, cout)
    assert int(tot) == yk.shape[0]
    mean = sl[:cout].sum(1) / tot
    bm = sl[:cout] / cnt.clamp(min=1)
    m2 = sl[cout:2 * cout].sum(1) + (cnt * (bm - mean[:, None]) ** 2).sum(1)
    assert_close(mean.numpy(), yk.mean(0).numpy(), 1e-4, f"{name} slab mean")
    assert_close((m2 / tot).numpy(), yk.var(0, unbiased=False).numpy(), 1e-4, f"{name} slab var")


@pytest.mark.parametrize("name,prec,cin,cout,k,s,p,sp", [
    ("gemm_f32", 0, 16, 8, 3, 1, 1, (6, 8, 10)),
    ("gemm_bf16_convt", 1, 32, 16, 3, 2, 1, (4, 6, 8)),
    ("halo_bf16", 1, 64, 64, 3, 1, 1, (6, 8, 10)),
])
def test_fused_backward_statistics(name, prec, cin, cout, k, s, p, sp, monkeypatch):
    """bn_gsum from input-grad launches (the dL/dy of the layer below), ReLU mask and residual."""
    from cgan3d_amd import ops, _lib as L
    monkeypatch.setattr(ops, "HALO", name.startswith("halo"))
    g = torch.Generator().manual_seed(17 + cin)
    n = 2
    # input-grad of a conv cout_l <- cin_l: its output has the layer input's shape (cout here)
    if "convt" in name:  # ConvTranspose3d(cout -> cin) input-grad = stride-2 forward conv
        din = tuple(2 * d for d in sp)
        geo0 = ops.convt_dgrad_geom(n, sp, din, cout, cin, k, s, p)
        wt = torch.randn(cout, cin, k, k, k, generator=g) / np.sqrt(cin * k**3)
        gin = torch.randn(n, cin, *din, generator=g)
        dout = sp
    else:
        geo0 = ops.conv_dgrad_geom(n, sp, sp, cout, cin, k, s, p)
        wt = torch.randn(cin, cout, k, k, k, generator=g) / np.sqrt(cout * k**3)
        gin = torch.randn(n, cin, *sp, generator=g)
        dout = sp
    geo = ops.with_prec(geo0, prec)
    ps = ops.PackSet(torch.device("cuda"))
    geo, wp = ps.add(geo, wt.cuda(), prec)
    ps.pack()
    assert (geo.w_packed == 2) == name.startswith("halo"), "unexpected kernel choice"
    out = torch.empty(n, *dout, cout, device="cuda")
    z = torch.randn(n, *dout, cout, generator=g).cuda()
    ss = torch.cat([torch.rand(cout, generator=g) + 0.5, torch.randn(cout, generator=g) * 0.2]).cuda()
    mi = torch.cat([torch.randn(cout, generator=g) * 0.1, torch.rand(cout, generator=g) + 0.5]).cuda()
    res = torch.randn(n, *dout, cout, generator=g).cuda()
    slots = ops.bn_slots(geo)
    part = torch.full((2 * cout * slots,), float("nan"), device="cuda")
    ep = ops.epilogue(residual=res, bn_part=part, bn_mode=2, bn_slots=slots, bn_z=z, bn_ss=ss, bn_mi=mi,
                      bn_act=L.ACT_RELU)
    ops.conv(geo, _cl(gin), wp, out, ep)
    got = part.double().cpu().view(2 * cout, slots).sum(1)
    assert_close(got.numpy(), _pairs(out, cout, z, ss, mi, L.ACT_RELU).numpy(), 1e-4, f"{name} backward slab")


@pytest.mark.parametrize("c,act", [(16, 1), (64, 0)])
def test_fused_batchnorm_vs_torch(c, act):
    """conv (bn_sum) -> bn_apply_acc -> reflect_fold_ex (bn_gsum) -> bn_backward_acc, against
    torch autograd of relu?(batch_norm(z)) with dL/dy = the reflect-pad adjoint of a random field."""
    from cgan3d_amd import ops, _lib as L
    g = torch.Generator().manual_seed(c + act)
    n, sp, P = 2, (8, 10, 12), 3
    x = torch.randn(n, 8, *sp, generator=g, dtype=torch.float64)
    w = torch.randn(c, 8, 3, 3, 3, generator=g, dtype=torch.float64) / 10
    gamma = torch.rand(c, generator=g, dtype=torch.float64) + 0.5
    beta = torch.randn(c, generator=g, dtype=torch.float64) * 0.1
    z = F.conv3d(x, w, padding=1).requires_grad_()
    gm, bt = gamma.clone().requires_grad_(), beta.clone().requires_grad_()
    rm, rv = torch.zeros(c, dtype=torch.float64), torch.ones(c, dtype=torch.float64)
    y = F.batch_norm(z, rm, rv, gm, bt, training=True, momentum=0.1, eps=1e-5)
    if act == L.ACT_RELU:
        y = F.relu(y)
    gpad = torch.randn(n, c, *(d + 2 * P for d in sp), generator=g, dtype=torch.float64)
    yp = F.pad(y, (P,) * 6, mode="reflect")
    dz, dgm, dbt = torch.autograd.grad(yp, (z, gm, bt), gpad)

    nvox = n * sp[0] * sp[1] * sp[2]
    geo = ops.conv_fwd_geom(n, sp, sp, 8, c, 3, 1, 1)
    zd = torch.empty(n, *sp, c, device="cuda")
    sf = ops.bn_slots(geo)
    pf = torch.empty((2 * c + 1) * sf, device="cuda")
    ops.conv(geo, _cl(x), w.float().cuda(), zd, ops.epilogue(bn_part=pf, bn_mode=1, bn_slots=sf))
    ss, mi = torch.empty(2 * c, device="cuda"), torch.empty(2 * c, device="cuda")
    rmd, rvd = torch.zeros(c, device="cuda"), torch.ones(c, device="cuda")
    nbt = torch.zeros((), dtype=torch.int64, device="cuda")
    gmd, btd = gamma.float().cuda(), beta.float().cuda()
    ops.bn_finalize_slab(pf, sf, c, nvox, gmd, btd, rmd, rvd, nbt, ss, mi)
    yd = torch.empty_like(zd)
    ops.bn_apply(zd, nvox, c, ss, act, yd)
    assert_close(_ncdhw(yd).numpy(), y.detach().numpy(), 1e-3, "fused bn fwd")
    assert_close(rmd.cpu().numpy(), rm.numpy(), 1e-3, "running_mean")
    assert_close(rvd.cpu().numpy(), rv.numpy(), 1e-3, "running_var")
    assert int(nbt.item()) == 1
    dyd = torch.empty_like(zd)
    sb = ops.reflect_fold_slots(n, sp, c)
    pb = torch.empty(2 * c * sb, device="cuda")
    ep = ops.epilogue(bn_part=pb, bn_mode=2, bn_slots=sb, bn_z=zd, bn_ss=ss, bn_mi=mi, bn_act=act)
    ops.reflect_fold(_cl(gpad), dyd, n, sp, c, P, ep=ep)
    dzd, dgd, dbd = torch.empty_like(zd), torch.empty(c, device="cuda"), torch.empty(c, device="cuda")
    ws = torch.empty(3 * c, device="cuda")
    dz16 = torch.empty(zd.shape, device="cuda", dtype=torch.bfloat16)
    ops.bn_backward_slab(dyd, zd, nvox, c, pb, sb, ss, mi, gmd, act, dgd, dbd, dzd, ws, dz16=dz16)
    assert_close(_ncdhw(dzd).numpy(), dz.numpy(), 1e-3, "fused bn dz")
    assert torch.equal(dz16, dzd.bfloat16()), "bf16 shadow of the BN input-grad"
    assert_close(dgd.double().cpu().numpy(), dgm.numpy(), 1e-3, "fused bn dgamma")
    assert_close(dbd.double().cpu().numpy(), dbt.numpy(), 1e-3, "fused bn dbeta")

