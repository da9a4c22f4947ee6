"""Debug: the generator's output gradient dL/d(pre-tanh) of one f32 GP step (G.dz_last) against the
float64 oracle, split into the adversarial (critic) and the ZNCC + HU parts."""
import copy
import sys
import numpy as np
import torch
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import test_gpu_step as T  # noqa: E402
from oracle import reference_torch as R  # noqa: E402
from cgan3d_amd.data.synthetic import synth_patches  # noqa: E402
from cgan3d_amd.engine import StepEngine  # noqa: E402

for init, bo, bs in [(8, 2, 2), (8, 3, 3), (16, 2, 2), (8, 4, 4)]:
    g_args = dict(n_resnet_blocks=1, n_updownsample_blocks=2, init_channels_out=init)
    S = 32
    g, d = T._models(g_args)
    dbl = lambda v: v.detach().cpu().clone().double() if v.is_floating_point() else v.detach().cpu().clone()  # noqa
    gpar = {k: dbl(v) for k, v in g.state_dict().items()}
    eng = StepEngine(g, d, g.config, d.config, bo, bs, (S, S, S), g_hyper=(1e-4, 0.0, 0.9, 1e-8),
                     d_hyper=(1e-4, 0.0, 0.9, 1e-8))
    m = min(bo, bs)
    cfg = R.StepConfig(gen=R.GenConfig(**g_args), critic=R.CriticConfig())
    opt, _ = synth_patches(bo, S, 40)
    sub, seg = synth_patches(bs, S, 50)
    eps = np.random.Generator(np.random.PCG64(60)).random((m, 1, 1, 1, 1)).astype(np.float32)
    eng.load_inputs(torch.from_numpy(opt).cuda(), torch.from_numpy(sub).cuda(), torch.from_numpy(seg).cuda(),
                    torch.from_numpy(eps).cuda())
    eng.generator_forward()
    eng.critic_update()
    d_after = {k: v.detach().cpu().clone().double() for k, v in d.state_dict().items()}
    eng.generator_update()
    torch.cuda.synchronize()
    dz = eng.G.dz_last.detach().cpu().double().numpy().reshape(bs, S, S, S)
    att_dev = eng.G.att.detach().cpu().double().numpy().reshape(bs, S, S, S)
    # oracle, float64
    gp2 = copy.deepcopy(gpar)
    subt = torch.from_numpy(sub).double()
    att = R.generator_forward(gp2, subt, cfg.gen, training=True).detach()
    al = att.clone().requires_grad_()
    oh = subt - al
    lg = cfg.gan_w * -R.wasserstein(R.critic_forward(d_after, oh, cfg.critic))
    ls = cfg.sim_w * R.zncc_loss(oh, subt) + cfg.hu_w * R.hu_loss(oh, torch.from_numpy(seg), cfg.hu_lo, cfg.hu_hi)
    ga, = torch.autograd.grad(lg, al, retain_graph=True)
    gs, = torch.autograd.grad(ls, al)
    dt = (1 - att ** 2)
    ref_a, ref_s = (ga * dt).numpy().reshape(bs, S, S, S), (gs * dt).numpy().reshape(bs, S, S, S)
    ref = ref_a + ref_s
    nr = lambda v: float(np.linalg.norm(v))  # noqa
    print(init, bo, bs, f"att rel {nr(att_dev - att.numpy().reshape(bs, S, S, S)) / nr(att.numpy()):.2e}",
          f"dz rel {nr(dz - ref) / nr(ref):.2e}", f"|adv| {nr(ref_a):.3e} |sim| {nr(ref_s):.3e}",
          f"dz-sim vs adv {nr(dz - ref_s - ref_a) / nr(ref_a):.2e}", flush=True)
