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


def check_collective_order(log):
    """Every collective is ordered after every earlier one by stream dependencies (a communicator's
    collectives must run in issue order on every rank), and the main stream has joined
    every collective by the end of the sequence.  ``log``: StepEngine.comm_log events."""
    known = {}  # stream -> indices of collectives ordered before its current position
    colls = []
    for ev in log:
        if ev[0] == "wait":
            _, waiter, signaler = ev
            known[waiter] = known.get(waiter, set()) | known.get(signaler, set())
        else:
            s = ev[1]
            before = known.get(s, set())
            missing = [j for j in range(len(colls)) if j not in before]
            assert not missing, f"collective {len(colls)} on {s} not ordered after {missing}: {log}"
            colls.append(ev)
            known[s] = before | {len(colls) - 1}
    assert known.get("main", set()) == set(range(len(colls))), "main stream does not join every collective"
    return colls


def _worker_sequence(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cgan3d_amd import ops
        from cgan3d_amd.engine import StepEngine
        from cgan3d_amd.model.discriminator import PatchGANDiscriminator
        from cgan3d_amd.model.generator import ResnetGenerator
        torch.manual_seed(7)
        g = ResnetGenerator(4, 2, 16)  # the benchmark generator: several gradient buckets
        d = PatchGANDiscriminator(**D_ARGS, norm_layer=nn.Identity)
        ops.DRY_RUN = True
        eng = StepEngine(g, d, g.config, d.config, 1, 1, (32, 32, 32), device=torch.device("cpu"))
        # the native-RCCL code path: ops.NativeComm over this gloo group (on the GPU the same object drives
        # RCCL from the plan; here torch.distributed does the exchange)
        eng.native = ops.NativeComm(None, torch.device("cpu"))
        assert eng.native.handle is None and eng.native.world == world
        logs = []
        for it in range(2):
            eng.comm_log = []
            for ar in (eng.g_arena, eng.d_arena):
                ar.grad.copy_(torch.arange(ar.grad.numel(), dtype=torch.float32) * (rank + 1 + it))
            eng.step()
            for ar in (eng.g_arena, eng.d_arena):
                want = torch.arange(ar.grad.numel(), dtype=torch.float32) * (sum(range(1, world + 1)) / world + it)
                assert torch.allclose(ar.grad, want), "step did not leave the mean gradient"
            logs.append(list(eng.comm_log))
        eng.comm_log = []
        eng.step(do_critic=True, do_generator=False)  # the reference schedule's critic-only iteration
        logs.append(list(eng.comm_log))
        allv = [None] * world
        dist.all_gather_object(allv, logs)
        q.put((rank, ("ok", allv)))
    except Exception as e:  # surfaced by the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_two_rank_collective_sequence_native_path():
    """The data-parallel step's collective sequence on the native-RCCL path (collectives issued from
    the launch plan on the shared communicator): identical on both ranks (count, arena spans and so
    byte sizes, issuing stream, order), every collective ordered after the previous one by a stream
    dependency, the main stream joined to all of them before the step ends; one critic all-reduce on
    the main stream, then the generator buckets tiling its arena exactly once on the communication
    stream.  Two gloo ranks, kernels in dry-run mode."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_sequence, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert isinstance(res[r], tuple) and res[r][0] == "ok", res
    allv = res[0][1]
    assert allv[0] == allv[1], "ranks issue different collective sequences"
    full, full2, crit = allv[0]
    assert full == full2
    for log in (full, crit):
        colls = check_collective_order(log)
        assert colls[0][:3] == ("allreduce", "main", "D") and colls[0][3:] == (0, colls[0][4])
    colls = check_collective_order(full)
    g = [c for c in colls[1:]]
    assert len(g) >= 2 and all(c[1] == "comm" and c[2] == "G" for c in g)
    assert g[0][4] > g[-1][3] and all(g[j][3] == g[j + 1][4] for j in range(len(g) - 1)) and g[-1][3] == 0
    assert len(check_collective_order(crit)) == 1


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
