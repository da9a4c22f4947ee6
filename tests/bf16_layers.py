"""Teacher-forced layer-by-layer check of the bf16 step (test infrastructure: imports the oracle).

Why layer by layer.  The device's bf16 path rounds each convolution's operands to bf16
(round-to-nearest-even) and accumulates in fp32; the bf16-operand oracle (reference_torch with
BF16_OPERANDS) does the same with float64 accumulation.  Run end to end the two decorrelate: a
last-bit fp32/fp64 difference moves a few operands across a bf16 rounding boundary (probability
~1e-7 / 2^-8 per element), each move is a 2^-8 step, and every k3 / k7 layer multiplies the
relative discrepancy by ~sqrt(receptive field) ~ 40 — after three layers the two runs differ by
the full bf16 noise (tools/bf16_layers.py: per layer 1e-7, end to end 4e-3 on the generator's
output).  So the device's ARITHMETIC is pinned here with every layer fed the device's own inputs:
each convolution (forward, input-grad, weight-grad) and BatchNorm pass against the float64
restatement of the same bf16-rounded operands, and the end-to-end step is judged statistically in
test_gpu_configs.py (within twice the bf16-operand oracle's own deviation from the exact step).
"""
import numpy as np
import torch
import torch.nn.functional as F

from oracle import reference_torch as R


def rnd(t):
    """bf16 round-to-nearest-even, kept in float64."""
    return t.to(torch.bfloat16).to(t.dtype)


def rel_l2(a, e):
    a, e = np.asarray(a, np.float64).ravel(), np.asarray(e, np.float64).ravel()
    return float(np.linalg.norm(a - e) / max(np.linalg.norm(e), 1e-300))


def cf(t):
    """device NDHWC (or a view of it) -> float64 NCDHW on the CPU."""
    return t.detach().float().cpu().double().permute(0, 4, 1, 2, 3).contiguous()


def conv(x, w, b=None, stride=1, padding=0):
    return R._conv3d_cpu(x, w, b, **({} if (stride, padding) == (1, 0) else dict(stride=stride, padding=padding)))


class Recorder:
    def __init__(self):
        self.rows = {}

    def add(self, name, value, bar):
        self.rows[name] = (float(value), float(bar))

    def fails(self):
        return [f"{k}: {v:.3e} > {b:.1e}" for k, (v, b) in self.rows.items() if not v <= b]

    def report(self):
        return {k: v for k, (v, _) in self.rows.items()}


def generator_layers(eng, rec: Recorder, weights=None, tol=1e-4, tol16=2e-3):
    """The generator of a StepEngine after ``generator_forward`` + ``generator_update``;
    ``weights``: the generator's parameters before that update's Adam step (the forward and
    backward ran with them)."""
    G = eng.G
    W = {k: v.detach().cpu().double() for k, v in (weights or eng.gP).items()}
    grads = {k: v.detach().cpu().double() for k, v in eng.gG.items()}
    x = cf(eng.subopt)

    def dev_y(i):  # the device's layer-i output (its bf16 shadow where the fp32 tensor is not kept)
        return (cf(G.y16[i]), True) if G.y_dead[i] else (cf(G.y[i]), False)
    ins, outs = [], []
    # ---- forward, each layer from the device's own input
    res_in = None
    for i, ly in enumerate(G.layers):
        w = rnd(W[f"{ly.name}.conv.weight"])
        if i == 0:
            xin = rnd(F.pad(x, (3,) * 6, mode="reflect"))
        else:
            yp, _ = dev_y(i - 1)
            xin = rnd(yp)
        ins.append(xin)
        if ly.kind == "convt":
            z = F.conv_transpose3d(xin, w, stride=2, padding=1, output_padding=1)
        else:
            z = conv(xin, w, stride=ly.s, padding=0 if i == 0 else ly.p)
        # z kept in bf16 (the 64^3 16-channel layers, engine.zs): the restated z rounded the same way
        z16 = G.zs[i].dtype == torch.bfloat16
        rec.add(f"G fwd z {ly.name}" + (" (bf16)" if z16 else ""), rel_l2(cf(G.zs[i]), rnd(z) if z16 else z),
                tol16 if z16 else tol)
        zd = cf(G.zs[i])
        nb = f"{ly.name}.normalization"
        y = F.batch_norm(zd, None, None, W[f"{nb}.weight"], W[f"{nb}.bias"], True, 0.1, 1e-5)
        if ly.act == 1:
            y = F.relu(y)
        if ly.name.endswith("block0"):
            res_in = dev_y(i - 1)[0]
        if ly.residual:
            y = y + res_in
        yd, is16 = dev_y(i)
        rec.add(f"G fwd y {ly.name}" + (" (bf16 shadow)" if is16 else ""), rel_l2(yd, rnd(y) if is16 else y),
                tol16 if is16 else tol)
        outs.append(y)
    la = G.last
    ylast, _ = dev_y(len(G.layers) - 1)
    xl = rnd(F.pad(ylast, (3,) * 6, mode="reflect"))
    att = torch.tanh(conv(xl, rnd(W["model.last_conv.weight"]), W["model.last_conv.bias"]))
    rec.add("G fwd att", rel_l2(cf(G.att), att), tol)
    # ---- backward from the device's dL/d pre-tanh
    dzl = cf(G.dz_last)
    rec.add("G bias last_conv", rel_l2(grads["model.last_conv.bias"], dzl.sum().reshape(1)), tol)
    wl = W["model.last_conv.weight"].clone().requires_grad_(True)
    out = conv(xl, wl)
    (gw,) = torch.autograd.grad(out, wl, rnd(dzl))
    rec.add("G wgrad last_conv", rel_l2(grads["model.last_conv.weight"], gw), tol)
    # dL/dy of the last BatchNorm layer: the last conv's input-grad folded over the reflect pad
    yl = ylast.clone().requires_grad_(True)
    xp = F.pad(yl, (3,) * 6, mode="reflect")
    xpl = rnd(xp).detach().requires_grad_(True)  # the padded grid the device's input-grad lands on
    (dpad,) = torch.autograd.grad(conv(xpl, rnd(W["model.last_conv.weight"])), xpl, rnd(dzl))
    # the reflect fold; with the padded input-grad kept in bf16 (engine.dpads) the device's statistics
    # still come from its fp32 values (the producer's epilogue) and only the elementwise pass reads bf16
    (dy_next,) = torch.autograd.grad(xp, yl, dpad, retain_graph=True)
    dy_fold16 = torch.autograd.grad(xp, yl, rnd(dpad))[0] if G.dpads.dtype == torch.bfloat16 else None
    for i in range(len(G.layers) - 1, -1, -1):
        ly = G.layers[i]
        nb = f"{ly.name}.normalization"
        dy = dy_next
        if not (G.fold_bn and i == len(G.layers) - 1):
            d16 = G.dys[i].dtype == torch.bfloat16
            rec.add(f"G bwd dy {ly.name}" + (" (bf16)" if d16 else ""), rel_l2(cf(G.dys[i]), rnd(dy) if d16 else dy),
                    tol16 if d16 else tol)
        # BatchNorm (+ act) backward from the device's z and the restated / device dL/dy
        last = G.fold_bn and i == len(G.layers) - 1
        if G.z16[i]:
            # bf16-stored layer (engine.zs / dys / dpads): the statistics pair (sum g, sum g*xhat) from
            # the producer's fp32 dL/dy (restated: dy) and the bf16 z, the elementwise pass from the
            # stored bf16 dL/dy, with the device's forward mean / invstd and scale / shift
            C = ly.cout
            zz = cf(G.zs[i])
            mi, ssv = G.mi[i].detach().double().cpu(), G.ss[i].detach().double().cpu()
            bc = lambda v: v.view(1, C, 1, 1, 1)  # noqa: E731
            xh = (zz - bc(mi[:C])) * bc(mi[C:])
            mask = ((zz * bc(ssv[:C]) + bc(ssv[C:])) > 0).double() if ly.act == 1 else torch.ones_like(zz)
            gs = dy * mask
            ga = (dy_fold16 if last else cf(G.dys[i])) * mask
            nv = zz.numel() // C
            db, dg = gs.sum((0, 2, 3, 4)), (gs * xh).sum((0, 2, 3, 4))
            dz = bc(W[f"{nb}.weight"] * mi[C:]) * (ga - bc(db / nv) - xh * bc(dg / nv))
        else:
            zd = cf(G.zs[i]).requires_grad_(True)
            gmm = W[f"{nb}.weight"].clone().requires_grad_(True)
            bta = W[f"{nb}.bias"].clone().requires_grad_(True)
            y = F.batch_norm(zd, None, None, gmm, bta, True, 0.1, 1e-5)
            if ly.act == 1:
                y = F.relu(y)
            dy_in = dy if last else cf(G.dys[i])  # the device folds its padded input-grad on the fly
            dz, dg, db = torch.autograd.grad(y, (zd, gmm, bta), dy_in)
        rec.add(f"G bn dgamma {ly.name}", rel_l2(grads[f"{nb}.weight"], dg), tol)
        rec.add(f"G bn dbeta {ly.name}", rel_l2(grads[f"{nb}.bias"], db), tol)
        if G.dz_dead[i]:
            dz_dev, is16 = cf(G.dz16[i]), True
        else:
            dz_dev, is16 = cf(G.dz[i]), False
        rec.add(f"G bwd dz {ly.name}" + (" (bf16 shadow)" if is16 else ""), rel_l2(dz_dev, rnd(dz) if is16 else dz),
                tol16 if is16 else tol)
        dzr = rnd(dz_dev)
        # weight grad from the device's operands
        w_ = W[f"{ly.name}.conv.weight"].clone().requires_grad_(True)
        if ly.kind == "convt":
            out = F.conv_transpose3d(ins[i], w_, stride=2, padding=1, output_padding=1)
        else:
            out = conv(ins[i], w_, stride=ly.s, padding=0 if i == 0 else ly.p)
        (gw,) = torch.autograd.grad(out, w_, dzr)
        rec.add(f"G wgrad {ly.name}", rel_l2(grads[f"{ly.name}.conv.weight"], gw), tol)
        if i == 0:
            break
        # input-grad into the previous layer's output (+ the skip gradient at a block's input)
        xi = ins[i].clone().requires_grad_(True)
        wr = rnd(W[f"{ly.name}.conv.weight"])
        if ly.kind == "convt":
            out = F.conv_transpose3d(xi, wr, stride=2, padding=1, output_padding=1)
        else:
            out = conv(xi, wr, stride=ly.s, padding=ly.p)
        (dx,) = torch.autograd.grad(out, xi, dzr)
        if ly.name.endswith("block0"):
            dx = dx + cf(G.dys[i + 1])  # the skip gradient as stored (bf16 where the layer keeps it)
        dy_next = dx


def critic_weight_grads(eng, rec: Recorder, tol=1e-4):
    """The critic's weight / bias gradients of a StepEngine right after ``critic_update`` (GP conf):
    dW_l = sum over [real | fake | interpolation] of wgrad(a_{l-1}, dz_l), the interpolation rows of
    a holding the penalty's forward-mode tangent nu (engine.py), each from the device's own
    operands (bf16-rounded for the middle layers, exact for the first and last)."""
    D = eng.D
    nall = eng.b_opt + eng.b_sub + eng.b_gp
    nb = eng.b_opt + eng.b_sub
    grads = {k: v.detach().cpu().double() for k, v in eng.dG.items()}
    W = {k: v.detach().cpu().double() for k, v in eng.dP.items()}
    prev = cf(eng.xc[:nall])
    for i, ly in enumerate(D.layers):
        dz = cf(D.dz[i][:nall])
        exact = i == 0 or i == len(D.layers) - 1
        a_in, g_out = (prev, dz) if exact else (rnd(prev), rnd(dz))
        w_ = W[f"{ly.name}.weight"].clone().requires_grad_(True)
        (gw,) = torch.autograd.grad(conv(a_in, w_, stride=ly.s, padding=ly.p), w_, g_out)
        rec.add(f"D wgrad {ly.name}", rel_l2(grads[f"{ly.name}.weight"], gw), tol)
        if D.biased[i]:
            rec.add(f"D bias {ly.name}", rel_l2(grads[f"{ly.name}.bias"], dz[:nb].sum((0, 2, 3, 4))), tol)
        prev = cf(D.a[i][:nall])
