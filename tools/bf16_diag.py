"""Diagnostic (GPU): where does the device's bf16 step part from the bf16-operand oracle?

Runs one 64^3 (default) bf16 step on the device and the float64 bf16-operand oracle
(reference_torch.BF16_OPERANDS) from the same state, for variants that switch off parts of the
step (adversarial weight, gradient penalty), and prints the median / max per-tensor relative L2 of
the device's gradients against the oracle's.  Test infrastructure only (imports the oracle)."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "contrast-gan-3d_amd"), str(REPO / "tests")]

from oracle import reference_torch as R  # noqa: E402
from oracle_step import models, rel_errors, step_inputs  # noqa: E402


def run(S, b, gan_w, gp_w, sim_w, hu_w, nres=4):
    from cgan3d_amd.engine import StepEngine
    g_args = dict(n_resnet_blocks=nres, n_updownsample_blocks=2, init_channels_out=16)
    g, d = models(g_args)
    dbl = lambda v: v.detach().cpu().clone().double() if v.is_floating_point() else v.detach().cpu().clone()  # noqa
    gpar = {k: dbl(v) for k, v in g.state_dict().items()}
    dpar = {k: dbl(v) for k, v in d.state_dict().items()}
    eng = StepEngine(g, d, g.config, d.config, b, b, (S, S, S), g_hyper=(1e-4, 0.0, 0.9, 1e-8),
                     d_hyper=(1e-4, 0.0, 0.9, 1e-8), precision="bf16", gp_weight=gp_w, gan_w=gan_w, sim_w=sim_w,
                     hu_w=hu_w)
    opt, sub, seg, eps = step_inputs(b, S, 0)
    eng.load_inputs(torch.from_numpy(opt).cuda(), torch.from_numpy(sub).cuda(), torch.from_numpy(seg).cuda(),
                    torch.from_numpy(eps).cuda())
    eng.generator_forward()
    eng.critic_update()
    d_after = {k: v.detach().cpu().clone() for k, v in d.state_dict().items()}
    eng.generator_update()

    def use_dev(dp):
        for k in dp:
            dp[k].data.copy_(d_after[k])
    cfg = R.StepConfig(gen=R.GenConfig(**g_args), critic=R.CriticConfig(), gp_weight=gp_w, gan_w=gan_w, sim_w=sim_w,
                       hu_w=hu_w)
    rec = {}
    R.BF16_OPERANDS = True
    try:
        R.train_step(gpar, dpar, R.AdamState(1e-4, 0.0, 0.9), R.AdamState(1e-4, 0.0, 0.9),
                     torch.from_numpy(opt).double(), torch.from_numpy(sub).double(), torch.from_numpy(seg),
                     torch.from_numpy(eps).double(), cfg, record=rec, after_critic=use_dev)
    finally:
        R.BF16_OPERANDS = False
    out = {}
    for net, arena in (("G", eng.g_arena), ("D", eng.d_arena)):
        errs = {}
        for k, gv in arena.gviews.items():
            if k == "model.last.bias" or k not in rec[net]:
                continue
            e = rec[net][k].numpy()
            if not np.abs(e).max() > 0:
                continue
            errs[k] = rel_errors(gv.cpu().numpy(), e)[1]
        v = np.array(list(errs.values()))
        out[net] = {"median_l2": float(np.median(v)), "max_l2": float(v.max()),
                    "worst": max(errs, key=errs.get)}
    return out


if __name__ == "__main__":
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    b = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    res = {}
    for tag, kw in (("full", dict(gan_w=1.0, gp_w=10.0, sim_w=1.0, hu_w=1.0)),
                    ("no_gp", dict(gan_w=1.0, gp_w=0.0, sim_w=1.0, hu_w=1.0)),
                    ("no_adv", dict(gan_w=0.0, gp_w=10.0, sim_w=1.0, hu_w=1.0)),
                    ("adv_only", dict(gan_w=1.0, gp_w=10.0, sim_w=0.0, hu_w=0.0))):
        res[tag] = run(S, b, **kw)
        print(tag, json.dumps(res[tag]), flush=True)
    out = REPO / "gpurun_out"
    if out.is_dir():
        (out / "bf16_diag.json").write_text(json.dumps(res, indent=1))
