"""Wall time of the step's three phases (generator forward, critic update, generator update) with
HIP events, eager launches, 64^3 B=4 bf16 (the bench workload)."""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "contrast-gan-3d_amd"))

import torch  # noqa: E402
from torch import nn  # noqa: E402


def main():
    from cgan3d_amd.data.synthetic import synth_patches
    from cgan3d_amd.engine import StepEngine
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.generator import ResnetGenerator
    from cgan3d_amd.model.init import pcg64_init_
    S, B = 64, 4
    prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    g = pcg64_init_(ResnetGenerator(4, 2, 16), 0).cuda()
    d = pcg64_init_(PatchGANDiscriminator(1, 8, 3, negative_slope=0.2, norm_layer=nn.Identity), 1).cuda()
    eng = StepEngine(g, d, g.config, d.config, B, B, (S, S, S), precision=prec)
    opt, _ = synth_patches(B, S, 1)
    sub, seg = synth_patches(B, S, 2)
    eng.load_inputs(torch.from_numpy(opt).cuda(), torch.from_numpy(sub).cuda(), torch.from_numpy(seg).cuda(),
                    torch.rand(B, device="cuda"))
    phases = [("G forward", eng.generator_forward), ("critic update", eng.critic_update),
              ("generator update", eng.generator_update)]
    for _ in range(3):
        eng.step()
    torch.cuda.synchronize()
    tot = {n: 0.0 for n, _ in phases}
    reps = 10
    for _ in range(reps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(phases) + 1)]
        ev[0].record()
        for i, (_, fn) in enumerate(phases):
            fn()
            ev[i + 1].record()
        torch.cuda.synchronize()
        for i, (n, _) in enumerate(phases):
            tot[n] += ev[i].elapsed_time(ev[i + 1]) / reps
    for n, t in tot.items():
        print(f"{n:18s} {t * 1e3:8.1f} us")
    print(f"{'step':18s} {sum(tot.values()) * 1e3:8.1f} us")


if __name__ == "__main__":
    main()
