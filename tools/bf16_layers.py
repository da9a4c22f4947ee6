"""Diagnostic (GPU): the bf16 critic layer by layer against a float64 restatement with the same
bf16 operand roundings (forward activations and input-gradient chain).  Test infrastructure."""
import sys
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "contrast-gan-3d_amd"), str(REPO / "tests")]


def rnd(t):
    return t.to(torch.bfloat16).to(t.dtype)


def rel(a, e):
    a, e = np.asarray(a, np.float64).ravel(), np.asarray(e, np.float64).ravel()
    return float(np.linalg.norm(a - e) / max(np.linalg.norm(e), 1e-30))


def main(S=32, n=4):
    from cgan3d_amd import _lib as L
    from cgan3d_amd.engine import CriticPlan
    from oracle_step import models
    g, d = models(dict(n_resnet_blocks=1, n_updownsample_blocks=2, init_channels_out=8))
    P = d._tensors()
    plan = CriticPlan(d.config, n, (S, S, S), torch.device("cuda"), P, L.PREC_BF16)
    rng = np.random.default_rng(0)
    x = torch.from_numpy(rng.standard_normal((n, S, S, S, 1)).astype(np.float32)).cuda()
    plan.forward(P, x, 0, n)
    plan.dz[-1].fill_(1.0)
    dx = torch.empty_like(x)
    plan.input_grad(P, 0, n, dx, 0, n)
    torch.cuda.synchronize()
    # float64 restatement, NCDHW
    W = {k: v.detach().cpu().double() for k, v in P.items()}
    s = d.config.negative_slope
    h = x.cpu().double().permute(0, 4, 1, 2, 3)
    zs, hs = [], [h]
    names = [ly.name[:-len(".weight")] if ly.name.endswith(".weight") else ly.name for ly in plan.layers]
    for i, ly in enumerate(plan.layers):
        w, b = W[f"{ly.name}.weight"], W.get(f"{ly.name}.bias")
        last, first = i == len(plan.layers) - 1, i == 0
        hin = hs[-1] if (first or last) else rnd(hs[-1])
        wt = w if (first or last) else rnd(w)
        z = F.conv3d(hin, wt, b, stride=ly.s, padding=ly.p)
        zs.append(z)
        hs.append(z if last else F.leaky_relu(z, s))
    print("layer  fwd a rel-L2 (device vs bf16 float64)")
    for i in range(len(plan.layers)):
        a = plan.a[i][:n].cpu().numpy()
        e = hs[i + 1].permute(0, 2, 3, 4, 1).numpy()
        print(i, plan.layers[i].name, f"{rel(a, e):.3e}")
    # backward: dL/dz_last = 1
    gz = torch.ones_like(zs[-1])
    dzs = [None] * len(plan.layers)
    dzs[-1] = gz
    for i in range(len(plan.layers) - 1, 0, -1):
        ly = plan.layers[i]
        w = W[f"{ly.name}.weight"]
        last = i == len(plan.layers) - 1
        gin, wt = (dzs[i], w) if last else (rnd(dzs[i]), rnd(w))
        ga = torch.nn.grad.conv3d_input(hs[i].shape, wt, gin, stride=ly.s, padding=ly.p)
        dzs[i - 1] = ga * torch.where(zs[i - 1] > 0, 1.0, s).double()
    print("layer  dz rel-L2 (device vs bf16 float64)")
    for i in range(len(plan.layers) - 1, -1, -1):
        a = plan.dz[i][:n].cpu().numpy()
        e = dzs[i].permute(0, 2, 3, 4, 1).numpy()
        print(i, plan.layers[i].name, f"{rel(a, e):.3e}")
    ly = plan.layers[0]
    ex = torch.nn.grad.conv3d_input(hs[0].shape, W[f"{ly.name}.weight"], dzs[0], stride=ly.s, padding=ly.p)
    print("dx", f"{rel(dx.cpu().numpy(), ex.permute(0, 2, 3, 4, 1).numpy()):.3e}")


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def generator(S=32, n=2):
    """The bf16 generator forward (att) and backward (every parameter gradient from a fixed dL/d
    pre-tanh) against the float64 bf16-operand oracle."""
    from cgan3d_amd import _lib as L
    from cgan3d_amd.engine import GeneratorPlan
    from oracle import reference_torch as R
    from oracle_step import models
    g_args = dict(n_resnet_blocks=2, n_updownsample_blocks=2, init_channels_out=16)
    g, _ = models(g_args)
    P = g._tensors()
    plan = GeneratorPlan(g.config, n, (S, S, S), torch.device("cuda"), P, L.PREC_BF16)
    rng = np.random.default_rng(1)
    x = torch.from_numpy(rng.standard_normal((n, S, S, S, 1)).astype(np.float32)).cuda()
    plan.forward(P, x, training=True)
    att_dev = plan.att.cpu().numpy().copy()
    gz = torch.from_numpy(rng.standard_normal((n, S, S, S, 1)).astype(np.float32)).cuda()
    plan.dz_last.copy_(gz)
    G = {k: torch.zeros_like(v) for k, v in g.named_parameters()}
    plan.backward(P, G, x)
    torch.cuda.synchronize()
    p64 = {k: v.detach().cpu().double().clone() for k, v in g.state_dict().items()}
    keys = [k for k, _ in g.named_parameters()]
    for k in keys:
        p64[k].requires_grad_(True)
    R.BF16_OPERANDS = True
    try:
        xin = x.cpu().double().permute(0, 4, 1, 2, 3)
        att = R.generator_forward(p64, xin, R.GenConfig(**g_args), training=True)
        # dL/d pre-tanh = gz  ->  dL/d att = gz / (1 - att^2)
        ga = gz.cpu().double().permute(0, 4, 1, 2, 3) / (1 - att.detach() ** 2)
        grads = torch.autograd.grad(att, [p64[k] for k in keys], ga)
    finally:
        R.BF16_OPERANDS = False
    print("att rel-L2", f"{rel(att_dev, att.detach().permute(0, 2, 3, 4, 1).numpy()):.3e}")
    for k, gr in zip(keys, grads):
        print(f"{k:55s} {rel(G[k].cpu().numpy(), gr.numpy()):.3e}")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "gen":
    generator()


def generator_layers(S=32, n=2):
    """Per-layer pre-BatchNorm conv outputs z_i of the bf16 generator forward against a float64
    restatement with the same operand roundings (each layer fed the DEVICE's previous output, so a
    mismatch is attributed to the layer that makes it)."""
    from cgan3d_amd import _lib as L
    from cgan3d_amd.engine import GeneratorPlan
    from oracle_step import models
    g_args = dict(n_resnet_blocks=2, n_updownsample_blocks=2, init_channels_out=16)
    g, _ = models(g_args)
    P = g._tensors()
    plan = GeneratorPlan(g.config, n, (S, S, S), torch.device("cuda"), P, L.PREC_BF16)
    rng = np.random.default_rng(1)
    x = torch.from_numpy(rng.standard_normal((n, S, S, S, 1)).astype(np.float32)).cuda()
    plan.forward(P, x, training=True)
    torch.cuda.synchronize()
    W = {k: v.detach().cpu().double() for k, v in P.items()}
    cf = lambda t: t.cpu().double().permute(0, 4, 1, 2, 3)  # noqa: E731
    prev = cf(x)
    for i, ly in enumerate(plan.layers):
        w = rnd(W[f"{ly.name}.conv.weight"])
        if i == 0:
            hin = rnd(F.pad(prev, (3,) * 6, mode="reflect"))
            z = F.conv3d(hin, w)
        elif ly.kind == "conv":
            hin = rnd(prev)
            z = F.conv3d(hin, w, stride=ly.s, padding=ly.p)
        else:
            hin = rnd(prev)
            z = F.conv_transpose3d(hin, w, stride=2, padding=1, output_padding=1)
        dz = plan.zs[i].float().cpu().numpy()
        print(f"{i} {ly.name:40s} z rel-L2 {rel(dz, z.permute(0, 2, 3, 4, 1).numpy()):.3e}")
        # BatchNorm (+ act, + residual) applied to the device's own z: the apply pass alone
        zt = plan.zs[i].cpu().double().permute(0, 4, 1, 2, 3)
        nb = f"{ly.name}.normalization"
        yb = F.batch_norm(zt, None, None, W[f"{nb}.weight"], W[f"{nb}.bias"], True, 0.1, 1e-5)
        if ly.act == L.ACT_RELU:
            yb = F.relu(yb)
        if ly.name.endswith("block0"):
            res_in = prev
        if ly.residual:
            yb = yb + res_in
        yl = plan.y16[i] if plan.y_dead[i] else plan.y[i]
        print(f"   y rel-L2 {rel(yl.float().cpu().numpy(), yb.permute(0, 2, 3, 4, 1).numpy()):.3e} "
              f"(dead fp32: {plan.y_dead[i]}, shadow: {plan.y16[i] is not None})")
        # the device's own output of the layer feeds the next
        yl = plan.y16[i] if plan.y_dead[i] else plan.y[i]
        prev = cf(yl.float())
    la = plan.last
    hin = rnd(F.pad(prev, (3,) * 6, mode="reflect"))
    z = F.conv3d(hin, rnd(W["model.last_conv.weight"]), W["model.last_conv.bias"])
    print(f"last att rel-L2 {rel(plan.att.cpu().numpy(), torch.tanh(z).permute(0, 2, 3, 4, 1).numpy()):.3e}")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "genl":
    generator_layers()
