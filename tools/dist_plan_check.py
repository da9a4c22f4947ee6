"""Two-rank check of the data-parallel step under a launch plan on ONE GPU (gloo over GPU tensors;
on an 8-GPU node the same code path runs RCCL):

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
        tools/dist_plan_check.py

Each rank feeds its own patches; after 3 plan-replayed steps both ranks must hold identical weights
(the all-reduced gradients drive identical Adam steps) and the plan must contain the two host
collectives between its C segments.
"""
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "contrast-gan-3d_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from torch import nn  # noqa: E402


def main():
    rank = int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    from cgan3d_amd.data.synthetic import synth_patches
    from cgan3d_amd.engine import StepEngine
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.generator import ResnetGenerator
    from cgan3d_amd.model.init import pcg64_init_
    S, B = 32, 2
    g = pcg64_init_(ResnetGenerator(2, 2, 16), 0).cuda()
    d = pcg64_init_(PatchGANDiscriminator(1, 8, 3, negative_slope=0.2, norm_layer=nn.Identity), 1).cuda()
    if rank == 1:  # different initial weights: the construction broadcast must overwrite them
        with torch.no_grad():
            for p in g.parameters():
                p.add_(0.01)
    eng = StepEngine(g, d, g.config, d.config, B, B, (S, S, S), precision="bf16")
    opt, _ = synth_patches(B, S, 100 + rank)
    sub, seg = synth_patches(B, S, 200 + rank)
    inputs = (torch.from_numpy(opt).cuda(), torch.from_numpy(sub).cuda(), torch.from_numpy(seg).cuda(),
              torch.full((B,), 0.3, device="cuda"))
    eng.load_inputs(*inputs)
    eng.step()  # eager warm-up (loads code objects)
    plan = eng.record()
    hosts = sum(1 for it in plan.items if not isinstance(it, int))
    assert hosts == 2, f"expected 2 host collectives in the plan, got {hosts}"
    for _ in range(3):
        eng.load_inputs(*inputs)
        eng.run_plan()
    torch.cuda.synchronize()
    losses = eng.losses.cpu()
    assert torch.isfinite(losses).all(), losses
    flat = torch.cat([eng.g_arena.flat, eng.d_arena.flat]).cpu()
    other = flat.clone()
    dist.broadcast(other, 0)
    diff = float((flat - other).abs().max())
    assert diff == 0.0, f"rank {rank}: weights differ from rank 0 by {diff}"
    print(f"rank {rank}: ok, {len(plan.items)} plan items ({hosts} host collectives), losses {losses[:7].tolist()}",
          flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
