"""A kernel timeline of the plan-mode bench step without a profiler (round 6): the step recorded with
every library kernel timed by its own hipExtLaunchKernel start / stop events (cgan3d_plan_time_filter,
cgan3d_plan_timeline), run over the bench batches; prints the median-length step's launches per stream
with the idle gap before each, and the main stream's busy / idle totals (each timeline is the last of four
runs issued back to back, so the host is ahead of the GPU as in the bench).

    python tools/plan_timeline.py [--steps 20] [--out gpurun_out/plan_timeline.txt]

(rocprofv3's kernel trace of the same step is host-bound: its per-dispatch cost outruns the GPU, so its
gaps are the profiler's.  The event pairs here add each dispatch's own queue latency to its duration,
~2 us per launch, and nothing else.)
"""
import argparse
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "contrast-gan-3d_amd"))

import cgan3d_amd  # noqa: E402,F401  (GPU_MAX_HW_QUEUES as bench.py)
import torch  # noqa: E402
from torch import nn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--out", default=None)
    ap.add_argument("--filter", default="2cg", help="kernels to time ('|'-separated name substrings; every timed "
                    "launch adds its own event cost, so time few to see the untimed step's gaps)")
    a = ap.parse_args()
    from cgan3d_amd import ops
    from cgan3d_amd.data.synthetic import synth_patches
    from cgan3d_amd.engine import StepEngine
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.generator import ResnetGenerator
    from cgan3d_amd.model.init import pcg64_init_
    S, B = 64, 4
    g = pcg64_init_(ResnetGenerator(4, 2, 16), 0).cuda()
    d = pcg64_init_(PatchGANDiscriminator(1, 8, 3, negative_slope=0.2, norm_layer=nn.Identity), 1).cuda()
    eng = StepEngine(g, d, g.config, d.config, B, B, (S, S, S), g_hyper=(1e-4, 0.0, 0.9, 1e-8),
                     d_hyper=(1e-4, 0.0, 0.9, 1e-8), precision="bf16")
    batches = []
    for j in range(2):
        opt, _ = synth_patches(B, S, 10 * j)
        sub, seg = synth_patches(B, S, 10 * j + 1)
        batches.append((torch.from_numpy(opt).cuda(), torch.from_numpy(sub).cuda(), torch.from_numpy(seg).cuda(),
                        torch.rand(B, device="cuda")))
    for i in range(5):
        eng.load_inputs(*batches[i % 2])
        eng.step()
    ops.plan_time_filter(a.filter)  # default: every kernel of the library's namespace ("_ZN2cg...")
    try:
        plan = eng.record()
    finally:
        ops.plan_time_filter(None)
    runs = []
    for i in range(a.steps):
        # four runs back to back, the timeline read from the last: issued while the GPU is busy with the
        # previous ones (the host ahead of the GPU, as in the bench's timed region), not from a cold queue
        for k in range(4):
            eng.load_inputs(*batches[(i + k) % 2])
            plan.run()
        torch.cuda.synchronize()
        tl = plan.timeline()
        span = max(e for _, _, e, _ in tl) - min(s for _, s, _, _ in tl)
        runs.append((span, tl))
    runs.sort(key=lambda r: r[0])
    span, tl = runs[len(runs) // 2]
    lines = [f"median step: {len(tl)} launches, {span * 1e3:.1f} us from first start to last end "
             f"(spans {runs[0][0] * 1e3:.1f} .. {runs[-1][0] * 1e3:.1f} us over {len(runs)} runs)"]
    last_end = {}
    busy, idle = {}, {}
    for sid, s, e, nm in sorted(tl, key=lambda r: r[1]):
        gap = (s - last_end[sid]) * 1e3 if sid in last_end else 0.0
        last_end[sid] = e
        busy[sid] = busy.get(sid, 0.0) + (e - s) * 1e3
        idle[sid] = idle.get(sid, 0.0) + max(gap, 0.0)
        lines.append(f"{sid} {s * 1e3:8.1f} {(e - s) * 1e3:7.1f} gap {gap:6.1f}  {nm[:90]}")
    for sid in sorted(busy):
        lines.append(f"stream {sid}: busy {busy[sid]:.1f} us, idle between its launches {idle[sid]:.1f} us")
    text = "\n".join(lines)
    print(text)
    if a.out:
        Path(a.out).write_text(text + "\n")


if __name__ == "__main__":
    main()
