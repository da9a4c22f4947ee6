"""The RCCL data-parallel path on ONE GPU: a one-rank nccl process group with CGAN3D_FORCE_DP=1
runs the bucketed generator all-reduces (communication stream ordered after the main and side
streams, one RCCL all-reduce per bucket, wait before Adam) and the critic all-reduce — by default
as C-ABI launches on the process group's communicator (ops.NativeComm, cgan3d_allreduce_mean:
recorded into the launch plan, which stays one C segment), with CGAN3D_COMM=torch through torch.distributed as
host callables between the plan's C segments.  Over one rank the mean is the identity, so three plan-replayed steps must match
an engine without collectives (up to weight-gradient atomics order).  Each compared step starts
from the same state (the reference engine's weights, Adam moments and BatchNorm buffers copied in
place): with beta1 = 0 Adam turns a last-bit gradient difference into a whole step of the other
sign, so free-running replicas drift apart over a few steps whatever the collectives do.

    python tools/dist_nccl1_check.py
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


def sync_state(src, dst):
    """src's trained state into dst's resident buffers, in place (recorded plans keep addresses)."""
    with torch.no_grad():
        for a, b in ((src.g_arena, dst.g_arena), (src.d_arena, dst.d_arena)):
            for t1, t2 in ((a.flat, b.flat), (a.exp_avg, b.exp_avg), (a.exp_avg_sq, b.exp_avg_sq)):
                t2.copy_(t1)
        for P1, P2 in ((src.gP, dst.gP), (src.dP, dst.dP)):
            for k, v in P1.items():
                if k.endswith(("running_mean", "running_var", "num_batches_tracked")):
                    P2[k].copy_(v)
    dst.G.pack()
    dst.D.pack()


def main():
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29531"), RANK="0",
                      WORLD_SIZE="1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    from cgan3d_amd.data.synthetic import synth_patches
    from cgan3d_amd.engine import StepEngine
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.generator import ResnetGenerator
    from cgan3d_amd.model.init import pcg64_init_
    S, B = 32, 2
    engs = []
    for force in ("1", "0"):
        os.environ["CGAN3D_FORCE_DP"] = force
        g = pcg64_init_(ResnetGenerator(2, 2, 16), 0).cuda()
        d = pcg64_init_(PatchGANDiscriminator(1, 8, 3, negative_slope=0.2, norm_layer=nn.Identity), 1).cuda()
        engs.append(StepEngine(g, d, g.config, d.config, B, B, (S, S, S), precision="f32"))
    dp, ref = engs
    assert dp.dp and not ref.dp and len(dp.g_buckets) >= 2 and dp.comm is not None
    opt, _ = synth_patches(B, S, 7)
    sub, seg = synth_patches(B, S, 8)
    inputs = (torch.from_numpy(opt).cuda(), torch.from_numpy(sub).cuda(), torch.from_numpy(seg).cuda(),
              torch.full((B,), 0.4, device="cuda"))
    plans = []
    for e in engs:
        e.load_inputs(*inputs)
        e.step()  # eager (code objects load lazily)
        plans.append(e.record())
    hosts = sum(1 for it in plans[0].items if not isinstance(it, int))
    native = os.environ.get("CGAN3D_COMM", "native") != "torch"
    assert (dp.native is not None) == native
    assert hosts == (0 if native else len(dp.g_buckets) + 2), hosts
    for _ in range(3):
        sync_state(ref, dp)
        for e in engs:
            e.load_inputs(*inputs)
            e.run_plan()
    torch.cuda.synchronize()
    dl = float((dp.losses - ref.losses).abs().max())
    assert dl <= 1e-4 * float(ref.losses.abs().max()), f"losses differ by {dl}"
    for a, b in ((dp.g_arena, ref.g_arena), (dp.d_arena, ref.d_arena)):
        err = float((a.grad - b.grad).abs().max()) / float(b.grad.abs().max())
        assert err <= 1e-3, f"gradients differ by {err:.2e} of the largest"
    print(f"nccl one-rank data-parallel path ok ({'native RCCL' if native else 'torch.distributed'}): "
          f"{len(dp.g_buckets)} buckets, {hosts} host callables, {len(plans[0].items)} plan segments", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
