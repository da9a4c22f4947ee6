"""Debug: generator gradients of one f32 GP step (small generator, 32^3) against the float64 oracle for
several (|OPT|, |LOW|+|HIGH|) — relative L2 error of each G gradient tensor (worst 3 printed)."""
import sys
import numpy as np
import torch
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import test_gpu_step as T  # noqa: E402
from oracle import reference_torch as R  # noqa: E402
from cgan3d_amd.data.synthetic import synth_patches  # noqa: E402
from cgan3d_amd.engine import StepEngine  # noqa: E402

for g_args, S in [(dict(n_resnet_blocks=1, n_updownsample_blocks=2, init_channels_out=8), 32)]:
    for bo, bs in [(2, 2), (3, 3)]:
        g, d = T._models(g_args)
        dbl = lambda v: v.detach().cpu().clone().double() if v.is_floating_point() else v.detach().cpu().clone()  # noqa
        gpar = {k: dbl(v) for k, v in g.state_dict().items()}
        dpar = {k: dbl(v) for k, v in d.state_dict().items()}
        eng = StepEngine(g, d, g.config, d.config, bo, bs, (S, S, S), g_hyper=(1e-4, 0.0, 0.9, 1e-8),
                         d_hyper=(1e-4, 0.0, 0.9, 1e-8))
        m = min(bo, bs)
        cfg = R.StepConfig(gen=R.GenConfig(**g_args), critic=R.CriticConfig())
        opt, _ = synth_patches(bo, S, 40)
        sub, seg = synth_patches(bs, S, 50)
        eps = np.random.Generator(np.random.PCG64(60)).random((m, 1, 1, 1, 1)).astype(np.float32)
        gi = eng.draw_gp_indices(np.random.default_rng(5)) if eng.gp_idx is not None else None
        eng.load_inputs(torch.from_numpy(opt).cuda(), torch.from_numpy(sub).cuda(), torch.from_numpy(seg).cuda(),
                        torch.from_numpy(eps).cuda())
        eng.generator_forward()
        eng.critic_update()
        d_after = {k: v.detach().cpu().clone() for k, v in d.state_dict().items()}
        eng.generator_update()
        torch.cuda.synchronize()

        def use_device_critic(dp):
            for k in dp:
                dp[k].data.copy_(d_after[k])
        rec = {}
        R.train_step(gpar, dpar, R.AdamState(1e-4, 0.0, 0.9), R.AdamState(1e-4, 0.0, 0.9),
                     torch.from_numpy(opt).double(), torch.from_numpy(sub).double(), torch.from_numpy(seg),
                     torch.from_numpy(eps).double(), cfg, record=rec, after_critic=use_device_critic, gp_idx=gi)
        errs = []
        for k, gv in eng.g_arena.gviews.items():
            a, e = gv.cpu().double().numpy(), rec["G"][k].numpy()
            errs.append((float(np.linalg.norm(a - e) / max(np.linalg.norm(e), 1e-30)), k))
        for e, k in errs:
            print(f"   {e:.2e} {k}")
        errs.sort(reverse=True)
        derr = max(float(np.linalg.norm(gv.cpu().double().numpy() - rec["D"][k].numpy()) /
                         max(np.linalg.norm(rec["D"][k].numpy()), 1e-30)) for k, gv in eng.d_arena.gviews.items())
        print(g_args["init_channels_out"], bo, bs, "G worst", [(f"{e:.2e}", k) for e, k in errs[:3]], "D worst",
              f"{derr:.2e}", flush=True)
