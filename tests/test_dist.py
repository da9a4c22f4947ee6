"""Multi-process data-parallel path on CPU (gloo, world size 2), kernels in dry-run mode.

The step shards patches over ranks and exchanges only gradients: StepEngine broadcasts rank 0's
state at construction (as DistributedDataParallel does) and averages each network's flat gradient
arena before its Adam update (engine._allreduce; RCCL all-reduce with the nccl backend on the GPU
box).  Here the HIP launches are no-ops (ops.DRY_RUN), so the test checks the collectives and the
operand plumbing of a full step, not arithmetic.
"""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from torch import nn

D_ARGS = dict(channels_in=1, init_channels_out=8, discriminator_depth=3, negative_slope=0.2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cgan3d_amd import ops
        from cgan3d_amd.engine import StepEngine
        from cgan3d_amd.model.discriminator import PatchGANDiscriminator
        from cgan3d_amd.model.generator import ResnetGenerator
        torch.manual_seed(100 + rank)  # different initial weights per rank: the engine must broadcast
        g = ResnetGenerator(2, 2, 8)
        d = PatchGANDiscriminator(**D_ARGS, norm_layer=nn.Identity)
        ops.DRY_RUN = True
        eng = StepEngine(g, d, g.config, d.config, 1, 1, (32, 32, 32), g_hyper=(1e-4, 0.0, 0.9, 1e-8),
                         d_hyper=(1e-4, 0.0, 0.9, 1e-8), device=torch.device("cpu"))
        assert eng.world == world
        # identical state after construction
        for ar in (eng.g_arena, eng.d_arena):
            ref = ar.flat.clone()
            dist.broadcast(ref, 0)
            assert torch.equal(ref, ar.flat), "parameters differ across ranks after construction"
        # gradient averaging
        for ar in (eng.g_arena, eng.d_arena):
            ar.grad.copy_(torch.arange(ar.grad.numel(), dtype=torch.float32) * (rank + 1))
            eng._allreduce(ar.grad)
            want = torch.arange(ar.grad.numel(), dtype=torch.float32) * (sum(range(1, world + 1)) / world)
            assert torch.allclose(ar.grad, want), "gradient arena is not the mean over ranks"
        # generator buckets: contiguous slices that tile the arena exactly once, closed in backward
        # order (stages descending), the first three layers in the small final bucket
        bk = eng.g_buckets
        assert len(bk) >= 2 and [st for st, _, _ in bk] == sorted((st for st, _, _ in bk), reverse=True)
        assert bk[0][2] == eng.g_arena.numel and bk[-1][1] == 0 and bk[-1][0] == 0
        assert all(bk[j][1] == bk[j + 1][2] for j in range(len(bk) - 1))
        # a full step with the collectives in place (kernels are no-ops here): the bucketed
        # all-reduces leave the mean over ranks in the generator arena, the critic's in its arena
        for ar in (eng.g_arena, eng.d_arena):
            ar.grad.copy_(torch.arange(ar.grad.numel(), dtype=torch.float32) * (rank + 1))
        eng.step()
        for ar in (eng.g_arena, eng.d_arena):
            want = torch.arange(ar.grad.numel(), dtype=torch.float32) * (sum(range(1, world + 1)) / world)
            assert torch.allclose(ar.grad, want), "step did not leave the mean gradient"
        # BatchNorm running buffers: rank 0's on every rank after sync_bn_buffers
        rm = eng.gP["model.first.normalization.running_mean"]
        rm.fill_(float(rank + 1))
        eng.sync_bn_buffers()
        assert torch.all(rm == 1.0), "running buffers not synchronised from rank 0"
        q.put((rank, "ok"))
    except Exception as e:  # surfaced by the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_data_parallel_step():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {0: "ok", 1: "ok"}, res
