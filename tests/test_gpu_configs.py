"""Every single-GPU configuration of BASELINE.json on the HIP path, against the CPU oracle.

* configs[1] — 64^3, batch 4 (+4 subopt), bf16, the full 4-block generator + GP critic: the
  benchmarked step itself, one step against its own yardstick (below) and reported against the
  exact float64 step.
* configs[2] — 128^3, batch 1, fp32: one step against the float64 oracle at north_star's 1e-3
  (conftest.assert_parity, the reference's own float32 deviation as the yardstick, ceiling 5e-3).
* configs[4] — 128^3 bf16 with the gradient penalty (global batch 16 over 8 GPUs, 2 per GPU): one
  step of the per-GPU slice (2 OPT + 2 subopt patches) against its own yardstick.

The bf16 bars (stated here).  The device's bf16 path rounds both operands of every generator
convolution and of the critic's middle convolutions to bf16 (round-to-nearest-even) and
accumulates in fp32; everything else runs in fp32.  The float64 oracle with exactly those roundings
(``reference_torch.BF16_OPERANDS``) computes the same function, but end to end the two cannot agree
closer than the bf16 noise itself: a last-bit fp32/fp64 accumulation difference carries a few
operands across a bf16 rounding boundary and every layer multiplies the discrepancy by ~40
(tests/bf16_layers.py; measured: per layer 1e-7, the generator's output after 12 layers 4e-3).  So:

* the ARITHMETIC is pinned teacher forced (test_bf16_step_64_b4_layers_match_bf16_operand_arithmetic):
  every convolution / BatchNorm pass / weight gradient of the benchmark step against the float64
  restatement of the same bf16 operands from the device's own inputs, relative L2 <= 1e-4;
* the whole step is held statistically to the exact float64 step: per gradient tensor within
  max(3e-2, 2x the bf16-operand oracle's own deviation) in relative L2 and max(1e-1, 4x its largest
  element's deviation, 2x its L2 deviation) in max-abs; tensors exactly zero in real arithmetic
  (the critic's last bias) within 1e-3 of the network's largest gradient; losses within 2e-2;
  post-Adam parameters: every element whose exact gradient is above twice the bf16-operand
  oracle's gradient noise (and above 5e-2 of the tensor's largest) steps the same way as the exact
  step's (Adam's first steps are ~lr*sign(g)/sqrt(1-beta2)).  Reports (device and bf16-operand
  oracle, each against the exact step): gpurun_out/bf16_vs_oracle_*.json.
"""
import json
import os
from pathlib import Path

import numpy as np
import pytest

from conftest import assert_parity
from oracle_step import LOSS_SLOTS, rel_errors, run_vs_oracle

pytestmark = pytest.mark.gpu

EXACT_CEIL = 0.3
# end to end (see tests/bf16_layers.py for why the device and the bf16-operand oracle decorrelate
# after a few layers): per tensor within max(3e-2, 2x the bf16-operand oracle's own deviation from
# the exact step) in relative L2, max-abs within max(1e-1, 4x its largest-element deviation, 2x its
# L2 deviation); the generator's losses within 2e-2 of the exact step's
E2E_L2, E2E_MAX, E2E_LOSS = 3e-2, 1e-1, 2e-2
# exactly zero in real arithmetic: a conv bias feeding BatchNorm has zero gradient, and the critic's
# last bias gradient is d/db [mean D(fake) - mean D(real)] = 0 (+ the penalty's, also 0)
ZERO_GRADS = ("model.last.bias",)


def _dump(name, rec):
    out = Path(os.environ.get("GRAFT_REPO_ROOT", Path(__file__).resolve().parent.parent)) / "gpurun_out"
    if out.is_dir():
        (out / f"{name}.json").write_text(json.dumps(rec, indent=1))


def _bf16_check(S, b, tag):
    report = {"S": S, "b": b, "bars": {"l2": E2E_L2, "max": E2E_MAX, "loss": E2E_LOSS}, "tensors": {},
              "losses": {}, "adam": {}}
    fails = []
    for it, losses, refbf, ref64, grads, recbf, rec64, params in run_vs_oracle(S, b, 1, "bf16", yard="bf16"):
        for k, slot in LOSS_SLOTS:
            err = abs(float(losses[slot]) - ref64[k]) / max(abs(ref64[k]), 1e-3)
            report["losses"][k] = {"dev_exact": err, "yard_exact": abs(refbf[k] - ref64[k]) / max(abs(ref64[k]), 1e-3),
                                   "dev_yard": abs(float(losses[slot]) - refbf[k]) / max(abs(refbf[k]), 1e-3)}
            if err > E2E_LOSS:
                fails.append(f"loss {k}: rel err {err:.3e} from the exact step")
        for net in ("G", "D"):
            netmax = max(float(np.abs(g).max()) for g in grads[net].values())
            for k, gv in grads[net].items():
                e = rec64[net][k].numpy()
                if k in ZERO_GRADS or float(np.abs(e).max()) == 0.0:
                    err = float(np.abs(gv).max()) / netmax
                    report["tensors"][f"{net}/{k}"] = {"zero_grad_abs_over_net_max": err}
                    if err > 1e-3:
                        fails.append(f"{net}/{k}: zero gradient off by {err:.3e} of the net's max")
                    continue
                mx, l2 = rel_errors(gv, e)
                ymx, yl2 = rel_errors(recbf[net][k].numpy(), e)  # the bf16-operand oracle's own deviation
                tol_l2 = min(max(E2E_L2, 2.0 * yl2), EXACT_CEIL)
                tol_mx = min(max(E2E_MAX, 4.0 * ymx, 2.0 * yl2), 2 * EXACT_CEIL)
                report["tensors"][f"{net}/{k}"] = {"dev_exact_max": mx, "dev_exact_l2": l2, "yard_exact_max": ymx,
                                                   "yard_exact_l2": yl2,
                                                   "dev_yard_l2": rel_errors(gv, recbf[net][k].numpy())[1]}
                if l2 > tol_l2 or mx > tol_mx:
                    fails.append(f"grad {net}/{k}: rel max {mx:.3e} (tol {tol_mx:.2e}) L2 {l2:.3e} (tol {tol_l2:.2e})")
            before, dev_after, ora_after, g64, _ = params[net]
            for k, g in g64.items():
                g = g.numpy()
                noise = float(np.abs(recbf[net][k].numpy() - g).max())  # bf16-operand gradient noise
                big = np.abs(g) > max(2.0 * noise, 5e-2 * float(np.abs(g).max()))
                d_dev = dev_after[k].numpy().astype(np.float64) - before[k].numpy()
                d_ora = ora_after[k].numpy() - before[k].numpy().astype(np.float64)
                flips = int((np.sign(d_dev[big]) != np.sign(d_ora[big])).sum())
                report["adam"][f"{net}/{k}"] = [flips, int(big.sum()), int(g.size)]
                if flips:
                    fails.append(f"adam {net}/{k}: {flips} of {int(big.sum())} elements with gradients above the "
                                 f"bf16 noise stepped the wrong way")
    _dump(f"bf16_vs_oracle_{tag}", report)
    assert not fails, "; ".join(fails[:12])


def test_bf16_step_64_b4_layers_match_bf16_operand_arithmetic():
    """BASELINE.json configs[1], teacher forced (tests/bf16_layers.py): after one benchmark step
    every generator convolution (forward, input-grad, weight-grad), BatchNorm pass (forward,
    backward, affine gradients) and every critic weight / bias gradient of the penalty update
    against the float64 restatement of the same bf16-rounded operands, each from the device's own
    inputs: relative L2 <= 1e-4 (fp32 against float64 accumulation), <= 2e-3 where the device keeps
    only a bf16 copy of the tensor (compared after rounding: rounding-boundary flips)."""
    import torch
    from bf16_layers import Recorder, critic_weight_grads, generator_layers
    from cgan3d_amd.engine import StepEngine
    from oracle_step import models, step_inputs
    g, d = models(dict(n_resnet_blocks=4, n_updownsample_blocks=2, init_channels_out=16))
    eng = StepEngine(g, d, g.config, d.config, 4, 4, (64, 64, 64), g_hyper=(1e-4, 0.0, 0.9, 1e-8),
                     d_hyper=(1e-4, 0.0, 0.9, 1e-8), precision="bf16")
    opt, sub, seg, eps = step_inputs(4, 64, 0)
    eng.load_inputs(torch.from_numpy(opt).cuda(), torch.from_numpy(sub).cuda(), torch.from_numpy(seg).cuda(),
                    torch.from_numpy(eps).cuda())
    eng.generator_forward()
    eng.critic_update()
    rec = Recorder()
    critic_weight_grads(eng, rec)
    w_before = {k: v.detach().clone() for k, v in eng.gP.items()}  # the generator update's Adam moves them
    eng.generator_update()
    generator_layers(eng, rec, weights=w_before)
    _dump("bf16_layers_64_b4", rec.report())
    assert len(rec.rows) > 100
    fails = rec.fails()
    assert not fails, "; ".join(fails[:12])


def test_bf16_step_64_b4_matches_oracle():
    """BASELINE.json configs[1]: the benchmarked step (64^3, 4 + 4 patches, 4 ResNet blocks, bf16)."""
    _bf16_check(64, 4, "64_b4")


@pytest.mark.timeout(300)
def test_bf16_step_128_matches_oracle():
    """BASELINE.json configs[4]'s per-GPU slice: 128^3, bf16, gradient penalty, 2 OPT + 2 subopt
    patches (global batch 16 over 8 GPUs = 2 per GPU), same bars as above."""
    _bf16_check(128, 2, "128_b2")


@pytest.mark.timeout(240)
def test_f32_step_128_b1_matches_oracle():
    """BASELINE.json configs[2]: 128^3, 1 + 1 patch, fp32, at north_star's 1e-3: every tensor within
    1e-3 relative L2 of the float64 step (or twice the reference's own float32 deviation), single
    elements within 3e-3 of the tensor's largest.  The element bar is wider because at 128^3 the
    ResNet-level gradients are sums over 32^3 voxels with heavy cancellation (BatchNorm backward
    makes sum(dz) ~ 0): the device sums them in fp32 (fp64 across blocks), where torch's CPU
    BatchNorm backward accumulates in double, so the reference's own float32 deviation understates
    an fp32 device's by ~5x on those few elements (measured: relative L2 <= 5.2e-4 for every tensor,
    the largest element 2.1e-3 of its tensor's max, gpurun_out/f32_vs_oracle_128_b1.json)."""
    fails, report = [], {}
    for it, losses, ref32, ref64, grads, rec32, rec64, params in run_vs_oracle(128, 1, 1, "f32"):
        checks = [(f"it{it} {k}", losses[slot], ref32[k], ref64[k], 0.0) for k, slot in LOSS_SLOTS]
        checks += [(f"it{it} grad {net} {k}", gv, rec32[net][k].numpy(), rec64[net][k].numpy(),
                    1e-7 if k in ZERO_GRADS else 0.0)  # exactly 0 in real arithmetic
                   for net in ("G", "D") for k, gv in grads[net].items()]
        for name, a, r32, r64, atol in checks:
            report[name] = rel_errors(a, r64) if np.ndim(a) else abs(float(a) - float(r64))
            try:
                assert_parity(a, r32, r64, name, atol=atol, max_factor=3.0)
            except AssertionError as e:
                fails.append(str(e).split("\n")[0])
    _dump("f32_vs_oracle_128_b1", report)
    assert not fails, "; ".join(fails)
