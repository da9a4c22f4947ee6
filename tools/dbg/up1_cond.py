"""Debug: conditioning of the last BatchNorm layer's bias gradient (sum over voxels of dL/d(BN out))
in the small-generator f32 GP step: |sum g| against sum |g| per channel, float64 oracle, and the
device's value."""
import copy
import sys
import numpy as np
import torch
import torch.nn.functional as F
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import test_gpu_step as T  # noqa: E402
from oracle import reference_torch as R  # noqa: E402
from cgan3d_amd.data.synthetic import synth_patches  # noqa: E402
from cgan3d_amd.engine import StepEngine  # noqa: E402

for init, b in [(8, 2), (8, 3)]:
    g_args = dict(n_resnet_blocks=1, n_updownsample_blocks=2, init_channels_out=init)
    S = 32
    g, d = T._models(g_args)
    dbl = lambda v: v.detach().cpu().clone().double() if v.is_floating_point() else v.detach().cpu().clone()  # noqa
    gpar = {k: dbl(v) for k, v in g.state_dict().items()}
    eng = StepEngine(g, d, g.config, d.config, b, b, (S, S, S), g_hyper=(1e-4, 0.0, 0.9, 1e-8),
                     d_hyper=(1e-4, 0.0, 0.9, 1e-8))
    cfg = R.StepConfig(gen=R.GenConfig(**g_args), critic=R.CriticConfig())
    opt, _ = synth_patches(b, S, 40)
    sub, seg = synth_patches(b, S, 50)
    eps = np.random.Generator(np.random.PCG64(60)).random((b, 1, 1, 1, 1)).astype(np.float32)
    eng.load_inputs(torch.from_numpy(opt).cuda(), torch.from_numpy(sub).cuda(), torch.from_numpy(seg).cuda(),
                    torch.from_numpy(eps).cuda())
    eng.generator_forward()
    eng.critic_update()
    d_after = {k: v.detach().cpu().clone().double() for k, v in d.state_dict().items()}
    eng.generator_update()
    torch.cuda.synchronize()
    dev_db = eng.g_arena.gviews["model.upsampling.1.normalization.bias"].cpu().double()
    # oracle forward with the up1 BatchNorm output kept
    p = copy.deepcopy(gpar)
    for k in p:
        if p[k].is_floating_point() and not k.endswith(("running_mean", "running_var")):
            p[k].requires_grad_(True)
    x = torch.from_numpy(sub).double()
    cg = cfg.gen
    h = F.pad(x, (3,) * 6, mode="reflect")
    h = F.relu(R.batch_norm(R._conv3d(h, p["model.first.conv.weight"]), p, "model.first.normalization", True))
    for i in range(cg.n_updownsample_blocks):
        pre = f"model.downsampling.{i}"
        h = F.relu(R.batch_norm(R._conv3d(h, p[f"{pre}.conv.weight"], stride=2, padding=1), p, f"{pre}.normalization", True))
    for r in range(cg.n_resnet_blocks):
        pre = f"model.resnet_backbone.{r}"
        t = R.batch_norm(R._conv3d(h, p[f"{pre}.block0.conv.weight"], padding=1), p, f"{pre}.block0.normalization", True)
        t = F.relu(R.batch_norm(R._conv3d(t, p[f"{pre}.block1.conv.weight"], padding=1), p, f"{pre}.block1.normalization", True))
        h = h + t
    bnout = None
    for j in range(cg.n_updownsample_blocks):
        pre = f"model.upsampling.{j}"
        h = R._conv_transpose3d(h, p[f"{pre}.conv.weight"], stride=2, padding=1, output_padding=1)
        h = R.batch_norm(h, p, f"{pre}.normalization", True)
        if j == cg.n_updownsample_blocks - 1:
            bnout = h
            bnout.retain_grad()
            pre = h.detach()
            for cc in range(pre.shape[1]):
                v = pre[:, cc].flatten()
                near = int((v.abs() < 1e-5).sum())
                vals, cnts = torch.unique(v, return_counts=True)
                print(f"   ch{cc}: |pre|<1e-5: {near}, most repeated value {float(vals[cnts.argmax()]):.3e} x{int(cnts.max())}")
        h = F.relu(h)
        if j == cg.n_updownsample_blocks - 1:
            rout = h
            rout.retain_grad()
    h = F.pad(h, (3,) * 6, mode="reflect")
    att = torch.tanh(R._conv3d(h, p["model.last_conv.weight"], p["model.last_conv.bias"]))
    oh = x - att
    lg = cfg.gan_w * -R.wasserstein(R.critic_forward(d_after, oh, cfg.critic))
    ls = cfg.sim_w * R.zncc_loss(oh, x) + cfg.hu_w * R.hu_loss(oh, torch.from_numpy(seg), cfg.hu_lo, cfg.hu_hi)
    (lg + ls).backward()
    gb = bnout.grad  # [n, c, D, H, W]
    s = gb.sum(dim=(0, 2, 3, 4))
    sa = gb.abs().sum(dim=(0, 2, 3, 4))
    ref_db = p["model.upsampling.1.normalization.bias"].grad
    # a ReLU mask flip at voxel v moves dbeta by dL/d(relu out)[v]: list the near-zero voxels' values
    pre_all, gr = bnout.detach(), rout.grad
    for cc in range(pre_all.shape[1]):
        v, gv = pre_all[:, cc].flatten(), gr[:, cc].flatten()
        idx = torch.nonzero(v.abs() < 1e-4).flatten()
        print(f"   ch{cc}: dbeta diff {float(dev_db[cc] - ref_db[cc]):+.3e}; |pre|<1e-4 voxels (pre, dL/drelu):",
              [(f"{float(v[i]):+.2e}", f"{float(gv[i]):+.3e}") for i in idx[:6]])
    print(init, b, "ref dbeta", s.numpy().round(8), "\n  sum|g|", sa.numpy().round(6), "\n  ratio", (s.abs() / sa).numpy(),
          "\n  dev dbeta", dev_db.numpy().round(8), "\n  rel err", ((dev_db - ref_db).abs() / ref_db.abs()).numpy(), flush=True)
