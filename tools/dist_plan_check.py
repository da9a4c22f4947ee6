"""Two-rank check of the data-parallel step under a launch plan on ONE GPU (gloo over GPU tensors;
on an 8-GPU node the same code path runs RCCL):

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
        tools/dist_plan_check.py

1. Reference check (f32, eager): from identical state, one data-parallel step (bucketed generator
   all-reduces overlapped with the backward, critic all-reduce) equals a single-rank engine whose
   gradient averaging is a plain synchronous all-reduce of the whole arena: the averaged
   gradients of both networks and the weights after Adam.
2. Plan check (bf16): each rank feeds its own patches; after 3 plan-replayed steps both ranks must
   hold identical weights, and the plan must hold the host collectives between its C segments (one
   per generator bucket, the wait before the generator's Adam, the critic's all-reduce).
"""
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "contrast-gan-3d_amd"))
import cgan3d_amd  # noqa: E402

cgan3d_amd.configure_hw_queues()  # before torch touches the GPU

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from torch import nn  # noqa: E402


def reference_check(rank, S, B):
    from cgan3d_amd.data.synthetic import synth_patches
    from cgan3d_amd.engine import StepEngine
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.generator import ResnetGenerator
    from cgan3d_amd.model.init import pcg64_init_
    solo_pg = [dist.new_group([r]) for r in range(dist.get_world_size())][rank]
    engs = []
    for pg in (None, solo_pg):
        g = pcg64_init_(ResnetGenerator(2, 2, 16), 0).cuda()
        d = pcg64_init_(PatchGANDiscriminator(1, 8, 3, negative_slope=0.2, norm_layer=nn.Identity), 1).cuda()
        engs.append(StepEngine(g, d, g.config, d.config, B, B, (S, S, S), precision="f32", process_group=pg))
    dp, solo = engs
    assert dp.world == 2 and solo.world == 1 and len(dp.g_buckets) >= 2

    def plain_mean(flat_grad):  # the reference averaging: one synchronous all-reduce of the arena
        t = flat_grad.clone()
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        flat_grad.copy_(t / dist.get_world_size())
    solo._allreduce = plain_mean
    solo.g_split = 0  # whole-arena Adam after the wrapped backward (the split one starts inside it)
    orig_update = solo.generator_update

    def solo_generator_update():  # the single-rank engine skips _allreduce for G (world 1): add it
        D = solo.G.backward
        solo.G.backward = lambda *a, **k: (D(*a, **k), plain_mean(solo.g_arena.grad))
        try:
            orig_update()
        finally:
            solo.G.backward = D
    solo.generator_update = solo_generator_update
    opt, _ = synth_patches(B, S, 300 + rank)
    sub, seg = synth_patches(B, S, 400 + rank)
    inputs = (torch.from_numpy(opt).cuda(), torch.from_numpy(sub).cuda(), torch.from_numpy(seg).cuda(),
              torch.full((B,), 0.3 + 0.2 * rank, device="cuda"))
    for e in engs:
        e.load_inputs(*inputs)
        e.generator_forward()
        e.critic_update()
    dd = [e.d_arena.grad.clone() for e in engs]
    for e in engs:
        e.generator_update()
    torch.cuda.synchronize()
    for name, a, b in (("D grad", dd[0], dd[1]), ("G grad", dp.g_arena.grad, solo.g_arena.grad)):
        err = float((a - b).abs().max()) / max(float(b.abs().max()), 1e-30)
        assert err <= 1e-4, f"rank {rank}: data-parallel {name} differs from the averaged reference by {err:.2e}"
    # weights: Adam's step may flip sign on rounding-noise gradient elements (2 * lr / sqrt(1 - beta2))
    for a, b in ((dp.g_arena.flat, solo.g_arena.flat), (dp.d_arena.flat, solo.d_arena.flat)):
        d = (a - b).abs()
        assert float(d.max()) <= 2 * 1e-4 / 0.316 * 1.01 and float((d > 1e-6).float().mean()) <= 0.01
    print(f"rank {rank}: reference check ok ({len(dp.g_buckets)} generator buckets)", flush=True)
    del engs, dp, solo


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
    reference_check(rank, S, B)
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
    want = len(eng.g_buckets) + 2
    assert hosts == want, f"expected {want} host callables in the plan, got {hosts}"
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
