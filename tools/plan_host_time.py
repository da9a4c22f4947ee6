"""Host cost of re-issuing the recorded step (cgan3d_plan_run, no sync) vs its GPU time, 64^3 B=4
bf16; CGAN3D_FORCE_DP=1 adds the one-rank RCCL data-parallel path (run under a process group).

    python tools/plan_host_time.py
"""
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "contrast-gan-3d_amd"))

import torch  # noqa: E402
from torch import nn  # noqa: E402


def main():
    if os.environ.get("CGAN3D_FORCE_DP") == "1":
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29601")
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0), rank=0, world_size=1)
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
    for _ in range(5):
        eng.run_plan()
    torch.cuda.synchronize()
    n = 40
    host = []
    t0 = time.perf_counter()
    for _ in range(n):
        a = time.perf_counter()
        eng.run_plan()
        host.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    host.sort()
    print(f"dp={eng.dp} launches/plan={eng.plan.launches} "
          f"host enqueue per step: median {host[n // 2] * 1e3:.3f} ms, p90 {host[int(n * 0.9)] * 1e3:.3f} ms; "
          f"wall per step {(t2 - t0) / n * 1e3:.3f} ms (host loop {(t1 - t0) / n * 1e3:.3f} ms)")


if __name__ == "__main__":
    main()
