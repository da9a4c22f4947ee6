"""Where the pinned-host batch copy goes: the resident plan step against the same
step with each batch copied from pinned host memory, in three forms, and the Trainer + PatchLoader loop.

    python tools/h2d_probe.py [--steps 50] [--only resident,pooled,after,fresh,loader]

resident: batches already in HBM (bench.py's value); pooled: bench.py's h2d line (copy of batch i+1 on
the pooled copy stream issued before step i); after: the same copy issued after step i's plan; fresh:
the round-4 form (a new torch stream for the copies); loader: bench.loader_bench.  Run it under
``rocprofv3 --kernel-trace --memory-copy-trace --stats`` with ``--only pooled`` to see whether the
copies are SDMA transfers or blit kernels."""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import bench  # noqa: E402  (sets the hardware-queue count before torch touches the GPU)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--only", default="resident,pooled,after,fresh,loader")
    a = ap.parse_args()
    which = a.only.split(",")
    from torch import nn
    from cgan3d_amd import ops
    from cgan3d_amd.data.synthetic import synth_patches
    from cgan3d_amd.engine import StepEngine
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.generator import ResnetGenerator
    from cgan3d_amd.model.init import pcg64_init_
    dev = torch.device("cuda", 0)
    S, B = 64, 4
    g = pcg64_init_(ResnetGenerator(4, 2, 16), 0).to(dev)
    d = pcg64_init_(PatchGANDiscriminator(1, 8, 3, negative_slope=0.2, norm_layer=nn.Identity), 1).to(dev)
    eng = StepEngine(g, d, g.config, d.config, B, B, (S, S, S), g_hyper=(1e-4, 0.0, 0.9, 1e-8),
                     d_hyper=(1e-4, 0.0, 0.9, 1e-8), device=dev, precision="bf16")
    host, stage, res = [], [], []
    for j in range(2):
        opt, _ = synth_patches(B, S, 80 + j)
        sub, seg = synth_patches(B, S, 90 + j)
        h = (torch.from_numpy(opt), torch.from_numpy(sub), torch.from_numpy(seg), torch.rand(B))
        host.append(tuple(t.pin_memory() for t in h))
        stage.append(tuple(torch.empty_like(t, device=dev) for t in h))
        res.append(tuple(t.to(dev) for t in h))
    for i in range(3):
        eng.load_inputs(*res[i % 2])
        eng.step()
    eng.record()
    main_s = torch.cuda.current_stream(dev)
    out = {}

    def timed(fn, n):
        for i in range(3):
            fn(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(3, 3 + n):
            fn(i)
        torch.cuda.synchronize()
        return round((time.perf_counter() - t0) / n * 1e3, 4)

    def resident(i):
        eng.load_inputs(*res[i % 2])
        eng.run_plan()

    def h2d(cs, after):
        ready = [torch.cuda.Event() for _ in range(2)]
        freed = [None, None]

        def copy(i):
            k = i % 2
            if freed[k] is not None:
                cs.wait_event(freed[k])
            with torch.cuda.stream(cs):
                for dst, src in zip(stage[k], host[k]):
                    dst.copy_(src, non_blocking=True)
                ready[k].record(cs)

        state = {"first": True}

        def step(i):
            k = i % 2
            if state["first"]:
                copy(i)
                state["first"] = False
            if not after:
                copy(i + 1)
            main_s.wait_event(ready[k])
            eng.load_inputs(*stage[k])
            ev = torch.cuda.Event()
            ev.record(main_s)
            freed[k] = ev
            eng.run_plan()
            if after:
                copy(i + 1)
        return step

    for name in which:
        if name == "resident":
            out[name] = timed(resident, a.steps)
        elif name == "pooled":
            out[name] = timed(h2d(ops.pooled_stream(dev, "copy"), False), a.steps)
        elif name == "after":
            out[name] = timed(h2d(ops.pooled_stream(dev, "copy"), True), a.steps)
        elif name == "fresh":
            out[name] = timed(h2d(torch.cuda.Stream(device=dev), False), a.steps)
        elif name == "copy_only":  # the copies alone, back to back on the copy stream
            cs = ops.pooled_stream(dev, "copy")
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with torch.cuda.stream(cs):
                for i in range(a.steps):
                    for dst, src in zip(stage[i % 2], host[i % 2]):
                        dst.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
            out[name] = round((time.perf_counter() - t0) / a.steps * 1e3, 4)
        elif name.startswith("zc"):  # zero-copy: mapped pinned buffers, one bounded copy kernel per step
            blocks = int(name[2:] or 32)
            mapped = []
            for j in range(2):
                mh = []
                for t in host[j]:
                    m = ops.MappedHost(t.shape, t.dtype)
                    m.tensor.copy_(t)
                    mh.append(m)
                mapped.append(mh)
            cs = ops.pooled_stream(dev, "copy")
            ready = [torch.cuda.Event() for _ in range(2)]
            freed = [None, None]

            def zcopy(i):
                k = i % 2
                if freed[k] is not None:
                    cs.wait_event(freed[k])
                with torch.cuda.stream(cs):
                    ops.copy_h2d(list(zip(mapped[k], stage[k])), blocks)
                    ready[k].record(cs)

            first = {"v": True}

            def zstep(i):
                k = i % 2
                if first["v"]:
                    zcopy(i)
                    first["v"] = False
                zcopy(i + 1)
                main_s.wait_event(ready[k])
                eng.load_inputs(*stage[k])
                ev2 = torch.cuda.Event()
                ev2.record(main_s)
                freed[k] = ev2
                eng.run_plan()
            out[name] = timed(zstep, a.steps)
            torch.cuda.synchronize()
            ok = all(torch.equal(stage[j][q].cpu(), host[j][q]) for j in range(2) for q in range(4))
            out[name + "_exact"] = ok
        elif name == "host":  # host cost per call (enqueue only, the queue kept busy by a spin kernel)
            def host_cost(fn, n=20):
                torch.cuda.synchronize()
                torch.cuda._sleep(int(2e9) // 1000)  # ~1 ms of queue work ahead per call batch
                t0 = time.perf_counter()
                for _ in range(n):
                    fn()
                t = (time.perf_counter() - t0) / n * 1e3
                torch.cuda.synchronize()
                return round(t, 4)
            cs = ops.pooled_stream(dev, "copy")
            ev = torch.cuda.Event()

            def tcopy():
                with torch.cuda.stream(cs):
                    stage[0][0].copy_(host[0][0], non_blocking=True)
            out[name] = {"run_plan_ms": host_cost(lambda: eng.run_plan(), 10),
                         "load_inputs_ms": host_cost(lambda: eng.load_inputs(*res[0])),
                         "torch_h2d_copy_ms": host_cost(tcopy),
                         "event_record_ms": host_cost(lambda: ev.record(main_s)),
                         "wait_event_ms": host_cost(lambda: main_s.wait_event(ev))}
        elif name == "loader":
            out[name] = bench.loader_bench(S, B, dev, a.steps, "bf16")
        elif name == "loader_zc":
            out[name] = bench.loader_bench(S, B, dev, a.steps, "bf16", zero_copy=True)
        elif name == "bench_h2d":  # bench.py's h2d sub-line (copies queued by a worker thread)
            out[name] = bench.h2d_bench(eng, S, B, dev, a.steps)
        print(name, out[name], flush=True)
    print(json.dumps({"ms_per_step": out}), flush=True)


if __name__ == "__main__":
    main()
