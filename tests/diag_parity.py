"""Diagnostic (not collected by pytest): per-parameter gradient error of one 64^3 engine step against
the float64 oracle, beside the float32 oracle's own deviation and the engine's run-to-run spread.

    python tests/diag_parity.py [--size 64] [--batch 2] [--precision f32]
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "contrast-gan-3d_amd"))
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--precision", default="f32")
    ap.add_argument("--seed", type=int, default=0, help="batch seed offset (the 64^3 test uses 0 and 1)")
    a = ap.parse_args()
    from oracle import reference_torch as R
    from cgan3d_amd.data.synthetic import synth_patches
    from cgan3d_amd.engine import StepEngine
    from test_gpu_step import _models
    S, b = a.size, a.batch
    g_args = dict(n_resnet_blocks=4, n_updownsample_blocks=2, init_channels_out=16)
    opt, _ = synth_patches(b, S, 10 + a.seed)
    sub, seg = synth_patches(b, S, 20 + a.seed)
    eps = np.random.Generator(np.random.PCG64(30 + a.seed)).random((b, 1, 1, 1, 1)).astype(np.float32)
    grads = []
    for rep in range(2):
        g, d = _models(g_args)
        if rep == 0:
            gpar = {k: v.detach().cpu().clone().double() if v.is_floating_point() else v.detach().cpu().clone()
                    for k, v in g.state_dict().items()}
            dpar = {k: v.detach().cpu().clone().double() for k, v in d.state_dict().items()}
        eng = StepEngine(g, d, g.config, d.config, b, b, (S, S, S), g_hyper=(1e-4, 0.0, 0.9, 1e-8),
                         d_hyper=(1e-4, 0.0, 0.9, 1e-8), precision=a.precision)
        eng.load_inputs(torch.from_numpy(opt).cuda(), torch.from_numpy(sub).cuda(), torch.from_numpy(seg).cuda(),
                        torch.from_numpy(eps).cuda())
        eng.generator_forward()
        eng.critic_update()
        d_after = {k: v.detach().cpu().clone() for k, v in d.state_dict().items()}
        eng.generator_update()
        grads.append({net: {k: v.cpu().double().numpy().copy() for k, v in ar.gviews.items()}
                      for net, ar in (("G", eng.g_arena), ("D", eng.d_arena))})

    def use_device_critic(dp):
        for k in dp:
            dp[k].data.copy_(d_after[k])

    cfg = R.StepConfig(gen=R.GenConfig(**g_args), critic=R.CriticConfig())
    rec32, rec = {}, {}
    g32 = {k: v.float() if v.is_floating_point() else v.clone() for k, v in gpar.items()}
    d32 = {k: v.float() for k, v in dpar.items()}
    R.train_step(g32, d32, R.AdamState(1e-4, 0.0, 0.9), R.AdamState(1e-4, 0.0, 0.9), torch.from_numpy(opt),
                 torch.from_numpy(sub), torch.from_numpy(seg), torch.from_numpy(eps), cfg, record=rec32,
                 after_critic=use_device_critic)
    R.train_step(gpar, dpar, R.AdamState(1e-4, 0.0, 0.9), R.AdamState(1e-4, 0.0, 0.9),
                 torch.from_numpy(opt).double(), torch.from_numpy(sub).double(), torch.from_numpy(seg),
                 torch.from_numpy(eps).double(), cfg, record=rec, after_critic=use_device_critic)
    print(f"{'param':48s} {'ours':>9s} {'ref32':>9s} {'ours-r32':>9s} {'run2run':>9s}   (max abs err / max |ref64|)")
    for net in ("G", "D"):
        for k in grads[0][net]:
            e = rec[net][k].numpy()
            sc = max(np.abs(e).max(), 1e-30)
            ours = np.abs(grads[0][net][k] - e).max() / sc
            r32 = np.abs(rec32[net][k].numpy() - e).max() / sc
            rr = np.abs(grads[0][net][k] - grads[1][net][k]).max() / sc
            o32 = np.abs(grads[0][net][k] - rec32[net][k].numpy()).max() / sc
            flag = "  <--" if ours > max(1e-3, 2 * r32) else ""
            print(f"{net} {k:46s} {ours:9.2e} {r32:9.2e} {o32:9.2e} {rr:9.2e}{flag}")


if __name__ == "__main__":
    main()
