"""Is the plan-mode step host-bound?  GPU time per step with the whole run enqueued behind a spin
kernel (host cost hidden) vs wall time per step with the host enqueuing as the GPU runs, 64^3 B=4.

    python tools/prequeue_step.py [bf16|f32]
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
    import os
    if os.environ.get("CGAN3D_FORCE_DP") == "1":  # the data-parallel path over a one-rank RCCL group
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29543")
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0), rank=0, world_size=1)
    S, B = 64, 4
    prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    g = pcg64_init_(ResnetGenerator(4, 2, 16), 0).cuda()
    d = pcg64_init_(PatchGANDiscriminator(1, 8, 3, negative_slope=0.2, norm_layer=nn.Identity), 1).cuda()
    eng = StepEngine(g, d, g.config, d.config, B, B, (S, S, S), precision=prec)
    opt, _ = synth_patches(B, S, 1)
    sub, seg = synth_patches(B, S, 2)
    eng.load_inputs(torch.from_numpy(opt).cuda(), torch.from_numpy(sub).cuda(), torch.from_numpy(seg).cuda(),
                    torch.rand(B, device="cuda"))
    for _ in range(3):
        eng.step()
    eng.record()
    for _ in range(3):
        eng.run_plan()
    torch.cuda.synchronize()
    n = 20
    t0 = time.perf_counter()
    for _ in range(n):
        eng.run_plan()
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    tw = time.perf_counter() - t0
    # calibrate the spin kernel, then hide the host enqueue behind it
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record()
    torch.cuda._sleep(50_000_000)
    e1.record()
    torch.cuda.synchronize()
    spin_ms = e0.elapsed_time(e1)
    cycles = int(50_000_000 * (th * 1e3 * 1.5 + 5) / spin_ms)
    torch.cuda._sleep(cycles)
    e1.record()
    t0 = time.perf_counter()
    for _ in range(n):
        eng.run_plan()
    th2 = time.perf_counter() - t0
    e2.record()
    torch.cuda.synchronize()
    gpu_ms = e1.elapsed_time(e2) / n
    print(f"host enqueue {th / n * 1e3:.3f} ms/step (while running) {th2 / n * 1e3:.3f} (behind spin); "
          f"wall {tw / n * 1e3:.3f} ms/step; GPU-only {gpu_ms:.3f} ms/step; spin {spin_ms:.1f} ms/50M cycles")


if __name__ == "__main__":
    main()
