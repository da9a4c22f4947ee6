"""Marginal cost of one more tiny launch inside the plan-mode step: the step recorded with an
extra 1-thread kernel after every launch vs the plain step (64^3 B=4 bf16), GPU-only timing
(host enqueue hidden behind a spin kernel)."""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "contrast-gan-3d_amd"))
import torch  # noqa: E402
from torch import nn  # noqa: E402


def gpu_ms(eng, n=20):
    for _ in range(3):
        eng.run_plan()
    torch.cuda.synchronize()
    e1, e2 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(150_000_000)
    e1.record()
    for _ in range(n):
        eng.run_plan()
    e2.record()
    torch.cuda.synchronize()
    return e1.elapsed_time(e2) / n


def main():
    from cgan3d_amd import ops, _lib as L
    from cgan3d_amd.data.synthetic import synth_patches
    from cgan3d_amd.engine import StepEngine
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.generator import ResnetGenerator
    from cgan3d_amd.model.init import pcg64_init_
    S, B = 64, 4
    g = pcg64_init_(ResnetGenerator(4, 2, 16), 0).cuda()
    d = pcg64_init_(PatchGANDiscriminator(1, 8, 3, negative_slope=0.2, norm_layer=nn.Identity), 1).cuda()
    eng = StepEngine(g, d, g.config, d.config, B, B, (S, S, S), precision="bf16")
    opt, _ = synth_patches(B, S, 1)
    sub, seg = synth_patches(B, S, 2)
    eng.load_inputs(torch.from_numpy(opt).cuda(), torch.from_numpy(sub).cuda(), torch.from_numpy(seg).cuda(),
                    torch.rand(B, device="cuda"))
    for _ in range(3):
        eng.step()
    eng.record()
    base = gpu_ms(eng)
    dummy = torch.zeros(8, device="cuda")
    orig = ops._launch
    count = [0]

    def with_tick(name, *args):
        rc = orig(name, *args)
        count[0] += 1
        L.lib().cgan3d_adam_tick(dummy.data_ptr(), L.stream())
        return rc
    ops._launch = with_tick
    eng.record()
    ops._launch = orig
    extra = gpu_ms(eng)
    print(f"step {base:.3f} ms; with {count[0]} extra 1-thread launches {extra:.3f} ms; "
          f"marginal {(extra - base) / count[0] * 1e3:.2f} us per launch")


if __name__ == "__main__":
    main()
