"""Host-side cost of the eager step: time to enqueue one step (no sync) vs GPU time per step,
eager and graph-replayed, 64^3 B=4 bf16 (the bench workload).

    python tools/host_time.py [bf16|f32]
"""
import sys
import time
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
    for _ in range(5):
        eng.step()
    torch.cuda.synchronize()
    # host enqueue time: the GPU is kept busy by a long queue, so this is pure host cost
    n = 30
    t0 = time.perf_counter()
    for _ in range(n):
        eng.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"eager: host enqueue {(t1 - t0) / n * 1e6:8.1f} us/step, wall {(t2 - t0) / n * 1e6:8.1f} us/step")
    eng.record()
    for _ in range(3):
        eng.run_plan()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        eng.run_plan()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"plan:  host enqueue {(t1 - t0) / n * 1e6:8.1f} us/step, wall {(t2 - t0) / n * 1e6:8.1f} us/step "
          f"({eng.plan.launches} ops)")
    eng.capture()
    torch.cuda.synchronize()
    for _ in range(3):
        eng.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        eng.replay()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"graph: wall {(t2 - t0) / n * 1e6:8.1f} us/step")


if __name__ == "__main__":
    main()
