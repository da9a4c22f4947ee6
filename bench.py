"""Benchmark: 3D patches/s of the G+D train step (BASELINE.json metric), HIP step engine.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--size 64] [--batch 4]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Workload (BASELINE.json configs[1]): 64^3 patches, 4 OPT + 4 (LOW+HIGH) subopt patches per GPU per
step, full G+D step of the gradient-penalty configuration (generator forward, critic update with
WGAN-GP, generator update, Adam on both).  Synthetic HU patches, PCG64-initialised weights of the
reference architecture.  "patches" = subopt patches corrected per second;
value = all ranks' patches / max-over-ranks wall time of the K timed steps.  Inputs are resident in
HBM when the timed region starts (a device-to-device copy into the engine's slots is inside it).

Extra JSON fields: ``roofline`` for the dominant kernel (HIP events around each of its launches
in place inside eager steps run after the timed region, on the launch stream; algorithmic FLOPs
from the launch geometry, 2 * out-voxels * Cout * Cin * k^3; ``warm_cache`` the same launches
repeated back to back; ``step`` the whole step against the MFMA and HBM peaks),
``reference_schedule`` (patches/s when the generator trains every 5th iteration, as the
reference's basic_conf does), ``h2d`` (each batch copied from pinned host memory on a copy stream,
overlapped with the previous step — the PatchLoader's form; ``value`` stays HBM-resident), ``f32``
(the exact-fp32 parity path at the same workload), ``b128_f32`` (BASELINE.json configs[2]: 128^3
B=1 fp32) and ``cpu_baseline`` (the oracle — torch fp32 on the host cores — on a bounded sample,
rank 0 only, N=1 only).  ``loader`` (the drop-in Trainer fed by three PatchLoaders from int16 scans on disk, Trainer.fit's
loop).  ``--no-sub`` skips the extra lines, ``--sub a,b`` picks some.

Precision: ``--precision bf16`` (default; BASELINE.json's metric is quoted in bf16) runs every
convolution on bf16 MFMA operands with fp32 accumulation, BatchNorm / losses / Adam in fp32;
``--precision f32`` is the exact-fp32 parity path.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

# hardware queues per process, read when HIP initialises (before torch touches the GPU): the step
# uses a main and a side stream, and under data parallelism a communication stream plus RCCL's own;
# with HIP's default of 4 some of them share an in-order hardware queue, where one stream's
# cross-stream wait blocks the other's kernels (measured on one GPU, one-rank RCCL path: 2.56 ms/step
# at 4 queues, 2.21 at 8, 2.21 at 16; 2.06 without collectives at either setting)
# (cgan3d_amd.configure_hw_queues, called here before torch touches the GPU; the setting in force
# is reported in the JSON line as config.hw_queues)
HW_QUEUES_ENV = os.environ.get("GPU_MAX_HW_QUEUES")
REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "contrast-gan-3d_amd"))
sys.path.insert(0, str(REPO))
import cgan3d_amd  # noqa: E402

cgan3d_amd.configure_hw_queues()

import numpy as np  # noqa: E402
import torch  # noqa: E402

F32_PEAK_TFLOPS = 157.3   # MI355X f32 MFMA == f32 vector peak (MI355X_MICROARCH.md)
BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA
HBM_PEAK_GBS = 8000.0


def conv_flops(n, dout, cin, cout, k):
    """FlopCounterMode-style conv FLOPs: 2 * N * Cout * |out| * Cin * k^3."""
    return 2.0 * n * cout * dout[0] * dout[1] * dout[2] * cin * k**3


# roofline candidates: kernel description, launch role, geometry predicate, committed PMC summary
# (HBM bytes per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes, profiles/)
def progress(msg):
    """A progress line on stderr (a long default run then never looks silent to a watchdog)."""
    print(f"bench: {msg} ({time.strftime('%H:%M:%S')})", file=sys.stderr, flush=True)


ROOFLINES = {
    "halo_res": ("ResNet-block Conv3d 64->64 k3 s1 at (S/4)^3, forward + input-grad "
                 "(bf16: conv_k3m_kernel; f32: conv_gemm_kernel)",
                 "conv", lambda g: g.cin == 64 and g.cout == 64 and g.k == 3 and g.stride == 1,
                 "profiles/r06_pmc_conv_k3m.json", "conv_k3m_kernel"),
    "k7_w2n": ("k7s_w2n_kernel: generator last Conv3d 16->1 k7 (+bias, tanh, opt_hat) forward",
               "conv", lambda g: g.k == 7 and g.cin == 16 and g.cout == 1, None, "k7s_w2n_kernel"),
}
# (description, launch role, geometry match, committed PMC traffic summary, kernel-name filter of the
# bf16 plan's in-step timing: the launches of that kernel are the roofline kernel's launches)


def pmc_traffic(path, size, batch, precision):
    """HBM bytes per launch from a committed PMC summary measured on this workload (else None)."""
    f = REPO / path if path else None
    if f is None or not f.is_file() or (size, batch, precision) != (64, 4, "bf16"):
        return None
    return json.loads(f.read_text()).get("hbm_bytes_per_launch")


def bn_hbm(path="profiles/r05_b128_f32_pmc.json"):
    """The dominant BatchNorm kernel of the 128^3 B=1 f32 step (BASELINE.json configs[2], "HBM-bound,
    rocprof GB/s vs roofline"): FETCH_SIZE / WRITE_SIZE bytes per launch over its kernel-trace duration,
    from the committed rocprofv3 summary (tools/pmc_r5_summary.py hbm)."""
    f = REPO / path
    if not f.is_file():
        return None
    ks = [k for k in json.loads(f.read_text())["kernels"] if k["kernel"].startswith("cg::bn_") and k["trace_us"]]
    if not ks:
        return None
    k = max(ks, key=lambda r: r["trace_us"] * max(r["launches_in_trace"], 1))
    return {"kernel": k["kernel"], "bytes_per_launch": k["bytes_per_launch"], "avg_launch_us": k["trace_us"],
            "hbm_gbs": k["gbs"], "hbm_peak_gbs": HBM_PEAK_GBS, "hbm_frac": k["hbm_frac"], "source": path}


def cpu_baseline(size, seconds, g_args):
    """Oracle (torch fp32 CPU restatement of the reference step) on the host cores."""
    from cgan3d_amd.data.synthetic import synth_patches
    from cgan3d_amd.model.init import pcg64_state_dict
    from oracle import reference_torch as R

    # every core the process may use: the affinity mask, capped by the cgroup CPU quota
    # when one is set — on the GPU box the mask lists the whole host while the quota is this GPU's share
    # (16 CPUs); threads past the quota only time-slice (a 192-thread oracle step there ran > 3 minutes)
    affinity = max(1, len(os.sched_getaffinity(0)))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    threads = affinity if quota is None else max(1, min(affinity, int(quota + 0.5)))
    torch.set_num_threads(threads)
    gcfg = R.GenConfig(**g_args)
    cfg = R.StepConfig(gen=gcfg, critic=R.CriticConfig())
    gp = {k: torch.from_numpy(v.copy()) for k, v in pcg64_state_dict(list(R.gen_param_shapes(gcfg).items()), 0).items()}
    dp = {k: torch.from_numpy(v.copy()) for k, v in
          pcg64_state_dict(list(R.critic_param_shapes(R.CriticConfig()).items()), 1).items()}
    gopt, dopt = R.AdamState(1e-4, 0.0, 0.9), R.AdamState(1e-4, 0.0, 0.9)
    b = 1
    opt, _ = synth_patches(b, size, 1)
    sub, seg = synth_patches(b, size, 2)
    eps = torch.full((b, 1, 1, 1, 1), 0.5)
    args = (torch.from_numpy(opt), torch.from_numpy(sub), torch.from_numpy(seg), eps, cfg)
    R.train_step(gp, dp, gopt, dopt, *args)  # warm-up
    progress(f"cpu_baseline: warm-up step done on {threads} threads")
    n, t0 = 0, time.perf_counter()
    while True:
        R.train_step(gp, dp, gopt, dopt, *args)
        n += 1
        if n % 10 == 0:
            progress(f"cpu_baseline: {n} steps")
        el = time.perf_counter() - t0
        if el >= seconds or n >= 50:
            break
    cpu_model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(n * b / el, 4), "unit": "patches/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model, "torch_threads": torch.get_num_threads(), "cgroup_cpu_quota": quota,
            "affinity_cpus": affinity,
            "sample": f"oracle/reference_torch.py train_step, {size}^3, batch 1+1, GP conf, fp32, {n} steps in "
                      f"{el:.1f}s after 1 warm-up step; patches/s per subopt patch at batch 1 stands for the GPU "
                      f"line's batch (the CPU step's work and time grow linearly with the batch)"}


def sub_config(S, B, precision, dev, g_args, steps=20, warmup=3):
    """Another single-GPU configuration of the same step in this run (BASELINE.json configs[2]: 128^3
    B=1 fp32; the exact-f32 parity path at 64^3 B=4): plan mode, ``steps`` timed steps."""
    from torch import nn
    from cgan3d_amd.data.synthetic import synth_patches
    from cgan3d_amd.engine import StepEngine
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.generator import ResnetGenerator
    from cgan3d_amd.model.init import pcg64_init_
    g = pcg64_init_(ResnetGenerator(**g_args), 0).to(dev)
    d = pcg64_init_(PatchGANDiscriminator(1, 8, 3, negative_slope=0.2, norm_layer=nn.Identity), 1).to(dev)
    eng = StepEngine(g, d, g.config, d.config, B, B, (S, S, S), g_hyper=(1e-4, 0.0, 0.9, 1e-8),
                     d_hyper=(1e-4, 0.0, 0.9, 1e-8), device=dev, precision=precision)
    opt, _ = synth_patches(B, S, 71)
    sub, seg = synth_patches(B, S, 72)
    batch = (torch.from_numpy(opt).to(dev), torch.from_numpy(sub).to(dev), torch.from_numpy(seg).to(dev),
             torch.rand(B, device=dev))
    for _ in range(warmup):
        eng.load_inputs(*batch)
        eng.step()
    eng.record()
    eng.load_inputs(*batch)
    eng.run_plan()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.load_inputs(*batch)
        eng.run_plan()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    losses = eng.losses.cpu().numpy()
    assert np.isfinite(losses).all(), f"non-finite losses {losses}"
    ms = el / steps * 1e3
    scale = (S / 64.0) ** 3
    tflops = 46.48e9 * scale * B / (ms * 1e-3) / 1e12
    out = {"value": round(B * steps / el, 3), "unit": "patches/s", "ms_per_step": round(ms, 3), "steps": steps,
           "dtype": precision, "config": {"workload": f"{S}^3 patches, {B} OPT + {B} LOW/HIGH, full G+D step "
                                                     "(WGAN-GP conf)", "patch": S, "global_batch": B},
           "step_tflops": round(tflops, 3),
           "step_frac": round(tflops / (BF16_PEAK_TFLOPS if precision == "bf16" else F32_PEAK_TFLOPS), 4)}
    del eng, g, d
    torch.cuda.empty_cache()
    return out


def h2d_bench(eng, S, B, dev, steps):
    """The step with each batch coming from pinned host memory (the PatchLoader's form): batch i + 1's
    host-to-device copy on a copy stream while step i runs, the step waiting for its own batch's copy."""
    from cgan3d_amd.data.synthetic import synth_patches
    host, stage = [], []
    for j in range(2):
        opt, _ = synth_patches(B, S, 80 + j)
        sub, seg = synth_patches(B, S, 90 + j)
        h = (torch.from_numpy(opt), torch.from_numpy(sub), torch.from_numpy(seg), torch.rand(B))
        host.append(tuple(t.pin_memory() for t in h))
        stage.append(tuple(torch.empty_like(t, device=dev) for t in h))
    from cgan3d_amd import ops
    cs = ops.pooled_stream(dev, "copy")  # the PatchLoader's copy stream (created with the engine's streams)
    main = torch.cuda.current_stream(dev)
    ready = [torch.cuda.Event() for _ in range(2)]
    freed = [None, None]

    from concurrent.futures import ThreadPoolExecutor
    pool = ThreadPoolExecutor(max_workers=1)
    futs = {}

    def copy(i):  # on a worker thread, as the PatchLoader issues its copies (the call holds its thread)
        k = i % 2
        with torch.cuda.device(dev), torch.cuda.stream(cs):
            if freed[k] is not None:
                cs.wait_event(freed[k])
            for dst, src in zip(stage[k], host[i % 2]):
                dst.copy_(src, non_blocking=True)
            ready[k].record(cs)

    def step(i):
        k = i % 2
        futs[i + 1] = pool.submit(copy, i + 1)
        futs.pop(i).result()  # batch i's copy was queued during step i - 1
        main.wait_event(ready[k])
        eng.load_inputs(*stage[k])
        ev = torch.cuda.Event()
        ev.record(main)
        freed[k] = ev
        eng.run_plan()

    futs[0] = pool.submit(copy, 0)
    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(3, 3 + steps):
        step(i)
    host_s = time.perf_counter() - t0
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    futs.pop(3 + steps).result()
    pool.shutdown()
    mb = sum(t.numel() * t.element_size() for t in host[0]) / 1e6
    return {"value": round(B * steps / el, 3), "unit": "patches/s", "ms_per_step": round(el / steps * 1e3, 3),
            "steps": steps, "h2d_mb_per_step": round(mb, 2), "host_ms_per_step": round(host_s / steps * 1e3, 3),
            "timing": "pinned host batch -> HBM (SDMA) on the copy stream, queued by a worker thread during the "
                      "previous step (the PatchLoader's form)"}


class _NullLogger:
    """logger_interface stand-in: the reference's wandb logger is out of scope."""

    class logger:  # noqa: N801
        @staticmethod
        def log_loss(*a, **k):
            pass

    def __call__(self, *a, **k):
        pass

    def end_hook(self):
        pass


def _gp_trainer(iters, dev, precision):
    """The drop-in Trainer as train.py:154-176 builds it with the GP conf's partials."""
    from functools import partial
    from torch import nn
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.generator import ResnetGenerator
    from cgan3d_amd.model.loss import HULoss
    from cgan3d_amd.trainer.Trainer import Trainer
    return Trainer(iters, 1, None, 1, 1, 10**9, 10**9,
                   partial(ResnetGenerator, 4, 2, 16),
                   partial(PatchGANDiscriminator, channels_in=1, init_channels_out=8, discriminator_depth=3,
                           negative_slope=0.2, norm_layer=nn.Identity),
                   partial(torch.optim.Adam, lr=1e-4, betas=(0.0, 0.9)), partial(torch.optim.Adam, lr=1e-4, betas=(0.0, 0.9)),
                   HULoss(112.0 / 600.0, 212.0 / 600.0), _NullLogger(), dev, checkpoint_dir=None, checkpoint_every=None,
                   precision=precision)


def loader_bench(S, B, dev, steps, precision, warmup=5, workers=4, zero_copy=False):
    """Trainer.train_step fed by create_dataloaders' PatchLoaders, the loop Trainer.fit runs
    (Trainer.py:241-252): every iteration takes one batch per scan type (B OPT, B/2 LOW, B/2 HIGH)
    from int16 [W,H,D,2] scans memory-mapped from disk (synthetic HU volumes written to a temporary
    directory first), cropped by the host workers into pinned slots, copied to HBM on the copy stream
    and unpacked / scaled there, then the step's launch plan."""
    import shutil
    import tempfile
    from cgan3d_amd.data.synthetic import synth_patches
    from cgan3d_amd.trainer.Trainer import ScanTypes
    from cgan3d_amd.trainer.utils import create_dataloaders

    class FZC:  # FactorZeroCenterScaler(238, 600) (basic_conf.py)
        shift, factor = 238.0, 600.0

    tmp = tempfile.mkdtemp(prefix="cgan3d_scans_")
    loaders = ()
    try:
        fold = []
        for i, label in enumerate((0, 0, 0, 0, -1, -1, 1, 1)):
            vol, seg = synth_patches(1, S + 16, 500 + i)
            hu = np.round(vol[0, 0].astype(np.float64) * 600.0 + 238.0).astype(np.int16)
            p = f"{tmp}/scan{i}"
            np.save(p + ".npy", np.stack([hu, seg[0, 0].astype(np.int16)], -1))
            fold.append((p, label))
        sizes = {0: B, -1: B // 2, 1: B - B // 2}
        train, _ = create_dataloaders(fold, fold[:1], (S,) * 3, (S,) * 3, sizes, {0: 1}, np.random.default_rng(3),
                                      scaler=FZC(), num_workers=(workers, 1), device=dev)
        loaders = tuple(train.values())
        if zero_copy:  # A/B (tools/h2d_probe.py): mapped slots read by the unpack kernel over PCIe
            from cgan3d_amd.data.loader import PatchLoader
            for st, ld in list(train.items()):
                ld._finish()
                train[st] = PatchLoader(ld.paths, ld.patch, ld.batch_size, np.random.default_rng(3 + st), scaler=FZC(),
                                        device=dev, num_threads=workers, seed_for_shuffle=42, zero_copy=True)
            loaders = tuple(train.values())
        tr = _gp_trainer(warmup + steps, dev, precision)
        it = 0
        for _ in range(max(warmup, 3)):  # first: eager; second: the plan is recorded and run
            tr.train_step([next(train[st]) for st in ScanTypes], it)
            it += 1
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            tr.train_step([next(train[st]) for st in ScanTypes], it)
            it += 1
        host = time.perf_counter() - t0  # the host's share: ~el when the loop is host-bound
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        mb = sum(ld._host[0].numel() * ld._host[0].element_size() for ld in loaders) / 1e6
        return {"value": round(B * steps / el, 3), "unit": "patches/s", "ms_per_step": round(el / steps * 1e3, 3),
                "steps": steps, "h2d_mb_per_step": round(mb, 2), "host_ms_per_step": round(host / steps * 1e3, 3), "host_workers_per_loader": workers,
                "host_ms_per_step": round(host / steps * 1e3, 3), "zero_copy": zero_copy,
                "timing": "Trainer.train_step on next() of three PatchLoaders per iteration (Trainer.fit's loop): "
                          "int16 crops from mmap'd .npy scans into pinned slots by host workers, which also queue "
                          "the H2D copies on the copy stream; GPU unpack"}
    finally:
        for ld in loaders:
            ld._finish()
        shutil.rmtree(tmp, ignore_errors=True)


def bench_trainer(args, S, B, dev, world, rank, dist, batches):
    """Trainer.train_step (cgan3d_amd.trainer.Trainer, constructed as train.py:154-176 does with the
    GP conf's partials) on device-resident [OPT, LOW, HIGH] patch dicts; the generator trains every
    iteration, as in the engine bench."""
    tr = _gp_trainer(args.warmup + args.steps, dev, args.precision)
    h = B // 2
    pl = []
    for opt, sub, seg, _ in batches:
        pl.append([{"data": opt, "seg": torch.zeros_like(opt, dtype=torch.bool)},
                   {"data": sub[:h], "seg": seg[:h]}, {"data": sub[h:], "seg": seg[h:]}])
    it = 0
    for _ in range(max(args.warmup, 3)):  # first: eager; second: the plan is recorded and run
        tr.train_step(pl[it % len(pl)], it)
        it += 1
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.train_step(pl[it % len(pl)], it)
        it += 1
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist:
        t = torch.tensor([el], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    losses = tr.engine.losses.cpu().numpy()
    assert np.isfinite(losses).all(), f"non-finite losses {losses}"
    ms = el / args.steps * 1e3
    out = {
        "metric": "3D patches/sec (G+D train step), 64³ bf16, at 1/2/4/8 MI355X",
        "value": round(world * B * args.steps / el, 3), "unit": "patches/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.precision, "data": "synthetic",
        "config": {"workload": f"{S}^3 patches, {B} OPT + {B} LOW/HIGH per GPU, Trainer.train_step (WGAN-GP conf)",
                   "global_batch": world * B, "patch": S, "parallelism": f"dp{world}",
                   "launch_mode": "trainer (launch plans recorded by Trainer.train_step)",
                   "plans": sum(p is not None for p in tr._plans.values())},
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sub", action="store_true",
                    help="skip the extra lines (h2d: batches from pinned host memory; f32: the exact-fp32 path; "
                         "b128_f32: BASELINE configs[2], 128^3 B=1 fp32)")
    ap.add_argument("--sub", default="h2d,loader,f32,b128_f32,b128_bf16_b2",
                    help="comma list of the extra lines to run (default all; --no-sub: none)")
    ap.add_argument("--precision", choices=["f32", "bf16"], default="bf16",
                    help="MFMA operand precision of the convolutions (accumulation is f32)")
    ap.add_argument("--roofline", choices=sorted(ROOFLINES), default="halo_res")
    ap.add_argument("--via-trainer", action="store_true",
                    help="time the drop-in Trainer.train_step (the path train.py drives: plans recorded and "
                         "replayed by the Trainer itself) on device-resident patch batches, instead of the engine")
    ap.add_argument("--mode", choices=["plan", "eager", "graph"], default="plan",
                    help="plan (default): the step recorded once as a launch plan (cgan3d_plan_*) and re-issued "
                         "from C++ each step, two streams kept; eager: the Python wrappers launch every kernel; "
                         "graph: one captured HIP graph per step (1 GPU only)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    elif os.environ.get("CGAN3D_FORCE_DP") in ("1", "init", "native"):
        # "1": the data-parallel path over a one-rank RCCL group; "init" / "native" (diagnostics): the
        # group (and a native communicator) exist but the engine runs its single-GPU step
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29541")
        dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
        if os.environ["CGAN3D_FORCE_DP"] == "native":
            from cgan3d_amd import ops as _ops
            _probe_comm = _ops.NativeComm(None, dev, own=True)  # noqa: F841 (kept alive for the run)

    from torch import nn
    from cgan3d_amd.data.synthetic import synth_patches
    from cgan3d_amd.engine import StepEngine
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.generator import ResnetGenerator
    from cgan3d_amd.model.init import pcg64_init_
    from cgan3d_amd import _lib


    g_args = dict(n_resnet_blocks=4, n_updownsample_blocks=2, init_channels_out=16)  # basic_conf.py:49-53
    S, B = args.size, args.batch
    g = pcg64_init_(ResnetGenerator(**g_args), 0).to(dev)
    d = pcg64_init_(PatchGANDiscriminator(1, 8, 3, negative_slope=0.2, norm_layer=nn.Identity), 1).to(dev)
    eng = StepEngine(g, d, g.config, d.config, B, B, (S, S, S), g_hyper=(1e-4, 0.0, 0.9, 1e-8),
                     d_hyper=(1e-4, 0.0, 0.9, 1e-8), device=dev, precision=args.precision)
    mode = "eager" if (args.mode == "graph" and world > 1) else args.mode
    torch.cuda.manual_seed(1234 + rank)  # per-rank GP eps (seed + rank)
    batches = []
    for j in range(2):
        opt, _ = synth_patches(B, S, 1000 * rank + 10 * j)
        sub, seg = synth_patches(B, S, 1000 * rank + 10 * j + 1)
        batches.append((torch.from_numpy(opt).to(dev), torch.from_numpy(sub).to(dev),
                        torch.from_numpy(seg).to(dev), torch.rand(B, device=dev)))

    if args.via_trainer:
        return bench_trainer(args, S, B, dev, world, rank, dist, batches)

    from cgan3d_amd import ops
    roof_desc, roof_role, roof_match, roof_pmc, roof_kname = ROOFLINES[args.roofline]
    ev = []  # (start, end, algorithmic flops) per timed launch

    reps = 8
    timing = {"reps": reps}

    def hook(role, geo):
        if role != roof_role or not roof_match(geo):
            return None
        e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev.append((*e, conv_flops(geo.n, (geo.do_, geo.ho, geo.wo), geo.cin, geo.cout, geo.k)))
        if timing["reps"] == 0:
            # in-step: a spin kernel ahead of the bracket keeps the queue busy while the host
            # enqueues start event, launch and end event, so the bracket holds only the launch
            torch.cuda._sleep(200000)
        return (*e, timing["reps"])

    def one_step(i, timed):
        eng.load_inputs(*batches[i % len(batches)])
        ops.LAUNCH_HOOK = hook if timed else None
        eng.step()
        ops.LAUNCH_HOOK = None

    def graph_step(i):
        eng.load_inputs(*batches[i % len(batches)])
        eng.replay()

    def plan_step(i):
        eng.load_inputs(*batches[i % len(batches)])
        eng.run_plan()

    progress(f"warm-up ({args.warmup} steps)")
    for i in range(args.warmup):
        one_step(i, False)
    if mode == "graph":
        torch.cuda.synchronize()
        eng.capture()  # records one step; replays below run the whole step as one graph launch
    elif mode == "plan":
        eng.record()  # records one step's launches (nothing runs); run_plan() re-issues them
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    # per-step boundaries: an event on the main stream after each step (every step ends with the
    # main stream waiting for the side stream), read after the timed region -> median step time
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    progress(f"timed region ({args.steps} steps, {mode})")
    t0 = time.perf_counter()
    marks[0].record()
    for i in range(args.steps):
        if mode == "graph":
            graph_step(i)
        elif mode == "plan":
            plan_step(i)
        else:
            one_step(i, False)
        marks[i + 1].record()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    step_ms = np.array([marks[i].elapsed_time(marks[i + 1]) for i in range(args.steps)])
    # the roofline kernel's launch time: after the timed region, eager steps in which each of its
    # launches is followed by `reps` back-to-back repeats between two HIP events on its stream
    # (repeats keep the queue full, so host launch gaps stay out of the measurement)
    progress("roofline kernel timing")
    for i in range(min(args.steps, 10)):
        one_step(i, True)
    torch.cuda.synchronize()
    kern = [(a.elapsed_time(b) / reps, f) for a, b, f in ev]
    # the same launches timed in place inside the step (cold-ish caches, no repeats): the in-step
    # rate, which a plan-mode rocprofv3 kernel trace of the bench reproduces
    ev.clear()
    timing["reps"] = 0
    for i in range(min(args.steps, 10)):
        one_step(i, True)
    torch.cuda.synchronize()
    kern_in = [(a.elapsed_time(b), f) for a, b, f in ev]
    # the headline figure (round 6): the kernel's launches timed inside the plan-mode step itself —
    # a plan recorded with cgan3d_plan_time_filter issues each of them with its own start / stop
    # events (hipExtLaunchKernel's dispatch events; the rest of the step unchanged), run over the
    # bench batches after the timed region
    kern_plan = []
    if mode == "plan" and args.precision == "bf16" and roof_kname and not dist:  # (one process: a DP plan re-recorded
        # mid-run would re-issue its collectives outside the timed protocol)
        ops.plan_time_filter(roof_kname)
        try:
            tplan = eng.record()
        finally:
            ops.plan_time_filter(None)
        for i in range(min(args.steps, 10)):
            eng.load_inputs(*batches[i % len(batches)])
            tplan.run()
            torch.cuda.synchronize()
            kern_plan += tplan.kernel_times()
        kern_plan = [t for t in kern_plan if t > 0]
    # the reference's schedule (basic_conf.py:24, Trainer.py:174-184): the critic trains every
    # iteration, the generator every 5th; every iteration runs the generator forward on its batch
    ref_sched = None
    progress("reference schedule")
    if mode == "plan" and world == 1:
        crit_plan = eng.record(do_critic=True, do_generator=False)
        full_plan = eng.record()
        for i in range(5):
            (full_plan if i % 5 == 0 else crit_plan).run()
        torch.cuda.synchronize()
        n_it = 5 * max(1, args.steps // 5)
        t1 = time.perf_counter()
        for i in range(n_it):
            eng.load_inputs(*batches[i % len(batches)])
            (full_plan if i % 5 == 0 else crit_plan).run()
        torch.cuda.synchronize()
        el_ref = time.perf_counter() - t1
        ref_sched = {"value": round(B * n_it / el_ref, 3), "unit": "patches/s", "iterations": n_it,
                     "ms_per_iteration": round(el_ref / n_it * 1e3, 3),
                     "schedule": "critic every iteration, generator every 5th (basic_conf.py:24); "
                                 "generator forward every iteration"}
    if dist:
        t = torch.tensor([el], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    losses = eng.losses.cpu().numpy()
    assert np.isfinite(losses).all(), f"non-finite losses {losses}"
    # the kernel's launch duration: its launches inside the plan-mode step (kern_plan, above); the
    # warm-repeat figure beside it: 8 back-to-back repeats of each in-step launch between two HIP
    # events on its stream (the events' own dispatch cost amortised over the repeats; agrees with the
    # rocprofv3 kernel-trace average of the plan-mode step, profiles/r03_plan_kernel_stats.csv); the
    # single-launch bracket (spin kernel ahead, one launch between the events) is reported beside it
    rep_ms = float(np.mean([t for t, _ in kern]))
    single_ms = float(np.mean([t for t, _ in kern_in]))
    roof_flops = float(np.mean([f for _, f in kern]))
    kern_ms = rep_ms
    achieved = roof_flops / (kern_ms * 1e-3) / 1e12
    peak = BF16_PEAK_TFLOPS if args.precision == "bf16" else F32_PEAK_TFLOPS
    ms = el / args.steps * 1e3
    value = world * B * args.steps / el
    # whole-step roofline: the reference step's algorithmic work per subopt patch (BASELINE.md §2,
    # torch.utils.flop_counter on the reference, GP conf, useful work: 46.48 GFLOP at 64^3) and
    # its compulsory HBM bytes in bf16 (SURVEY.md §8d model: ~180 MB at 64^3), both scaling with
    # the voxel count, times this GPU's B patches, over the measured step time
    scale = (S / 64.0) ** 3
    step_flops, step_bytes = 46.48e9 * scale * B, 180e6 * scale * B
    step_tflops = step_flops / (ms * 1e-3) / 1e12
    step_gbs = step_bytes / (ms * 1e-3) / 1e9
    out = {
        "metric": "3D patches/sec (G+D train step), 64³ bf16, at 1/2/4/8 MI355X",
        "value": round(value, 3), "unit": "patches/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic",
        "config": {"workload": f"{S}^3 patches, {B} OPT + {B} LOW/HIGH per GPU, full G+D step (WGAN-GP conf)",
                   "global_batch": world * B, "patch": S, "parallelism": f"dp{world}",
                   "launch_mode": mode, "hw_queues": int(os.environ["GPU_MAX_HW_QUEUES"]),
                   "hw_queues_env": HW_QUEUES_ENV},
        "step_ms": {"median": round(float(np.median(step_ms)), 4), "p10": round(float(np.percentile(step_ms, 10)), 4),
                    "p90": round(float(np.percentile(step_ms, 90)), 4), "steps": int(args.steps),
                    "timing": "HIP events on the main stream between consecutive timed steps"},
        "roofline": {"kernel": roof_desc, "bound": "mfma", "achieved": round(achieved, 3), "peak": peak,
                     "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                     "traffic": pmc_traffic(roof_pmc, S, B, args.precision), "traffic_source": roof_pmc,
                     "avg_launch_ms": round(kern_ms, 4), "flops_per_launch": roof_flops, "launches_timed": len(kern),
                     "timing": f"HIP events around {reps} back-to-back repeats of each launch of the kernel inside eager "
                               f"steps, on its own operands and stream (per-launch dispatch cost amortised; agrees "
                               f"with the plan-mode rocprofv3 kernel trace, profiles/r06_plan_kernel_stats.csv)",
                     "in_plan": None if not kern_plan else {
                         "avg_launch_ms": round(float(np.mean(kern_plan)), 4), "launches_timed": len(kern_plan),
                         "achieved": round(roof_flops / (float(np.mean(kern_plan)) * 1e-3) / 1e12, 3),
                         "frac": round(roof_flops / (float(np.mean(kern_plan)) * 1e-3) / 1e12 / peak, 4),
                         "timing": "each launch inside plan-mode steps between its own start / stop events "
                                   "(hipExtLaunchKernel via cgan3d_plan_time_filter): includes the dispatch's "
                                   "queue latency, which the rocprofv3 kernel trace leaves out"},
                     "single_launch": {"avg_launch_ms": round(single_ms, 4),
                                       "achieved": round(roof_flops / (single_ms * 1e-3) / 1e12, 3),
                                       "timing": "one launch between two HIP events in place inside eager steps, a spin "
                                                 "kernel ahead (includes the launch's dispatch latency)"},
                     "step": {"bound": "mfma", "achieved": round(step_tflops, 3), "peak": peak, "unit": "TFLOP/s",
                              "frac": round(step_tflops / peak, 4), "flops_per_step": step_flops,
                              "hbm_achieved_gbs": round(step_gbs, 1), "hbm_peak_gbs": HBM_PEAK_GBS,
                              "hbm_frac": round(step_gbs / HBM_PEAK_GBS, 4), "bytes_per_step": step_bytes,
                              "source": "46.48 GFLOP and ~180 MB per 64^3 subopt patch (BASELINE.md §2, "
                                        "SURVEY.md §8d), x B, / ms_per_step"}},
    }
    if ref_sched is not None:
        out["reference_schedule"] = ref_sched
    subs = set() if args.no_sub else set(filter(None, args.sub.split(",")))
    if mode == "plan" and world == 1 and subs:
        # beside the resident number: the batch coming over PCIe from pinned host memory each step
        if "h2d" in subs:
            progress("sub-line h2d")
            out["h2d"] = h2d_bench(eng, S, B, dev, args.steps)
        del eng
        torch.cuda.empty_cache()
        # the drop-in Trainer fed by the PatchLoaders (the loop train.py's Trainer.fit runs)
        if "loader" in subs:
            progress("sub-line loader")
            out["loader"] = loader_bench(S, B, dev, args.steps, args.precision)
        torch.cuda.empty_cache()
        # the other single-GPU BASELINE configs in the same run: the exact-fp32 parity path at this
        # workload, and configs[2] (128^3 B=1 fp32)
        if "f32" in subs:
            progress("sub-line f32")
            out["f32"] = sub_config(S, B, "f32", dev, g_args) if args.precision != "f32" else None
        if "b128_f32" in subs:
            progress("sub-line b128_f32")
            out["b128_f32"] = sub_config(128, 1, "f32", dev, g_args, steps=10)
            bn = bn_hbm()
            if bn is not None:
                out["b128_f32"]["hbm_gbs"] = bn["hbm_gbs"]
                out["b128_f32"]["hbm_bn_kernel"] = bn
        # configs[4]'s per-GPU slice: 128^3 bf16 with the gradient penalty, 2 OPT + 2 subopt patches
        # (global batch 16 over 8 GPUs)
        if "b128_bf16_b2" in subs:
            progress("sub-line b128_bf16_b2")
            out["b128_bf16_b2"] = sub_config(128, 2, "bf16", dev, g_args, steps=10)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        progress("sub-line cpu_baseline")
        out["cpu_baseline"] = cpu_baseline(S, args.cpu_seconds, g_args)
    progress("bench line")
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
