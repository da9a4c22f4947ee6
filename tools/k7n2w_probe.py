"""Time the generator's first conv (1 -> 16 k7 reflect, mode-1 BatchNorm statistics) and the last
conv's input-grad (1 -> 16 over the reflect-padded grid, with and without the folded mode-2
statistics) at 64^3 B=4 alone, under k7m debug switches (cgan3d_set_tuning key 11): 1 no unfold,
2 no MFMA, 4 no halo loads, 8 no output stores, 16 no weight staging, 32 exit after it."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "contrast-gan-3d_amd"))
import torch  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    from cgan3d_amd import ops, _lib as L
    n, S, C, P = 4, 64, 16, 3
    dims, pd = (S, S, S), (S + 2 * P,) * 3
    lib = L.load()
    fwd = ops.with_prec(ops.conv_fwd_geom(n, dims, dims, 1, C, 7, 1, P, True), L.PREC_BF16)
    x = torch.randn(n, *dims, 1, device="cuda")
    w = torch.randn(C, 1, 7, 7, 7, device="cuda") * 0.05
    y = torch.empty(n, *dims, C, device="cuda")
    sl = ops.bn_slots(fwd)
    part1 = torch.empty((2 * C + 1) * sl, device="cuda")
    ep1 = ops.epilogue(bn_part=part1, bn_mode=1, bn_slots=sl)
    dg = ops.with_prec(ops.conv_dgrad_geom(n, pd, dims, C, 1, 7, 1, 0), L.PREC_BF16)
    g = torch.randn(n, *dims, 1, device="cuda")
    wl = torch.randn(1, C, 7, 7, 7, device="cuda") * 0.05
    dpad = torch.empty(n, *pd, C, device="cuda")
    sl2 = ops.bn_slots(dg)
    part2 = torch.empty(2 * C * sl2, device="cuda")
    z = torch.randn(n, *dims, C, device="cuda")
    ss = torch.randn(2 * C, device="cuda")
    mi = torch.rand(2 * C, device="cuda") + 0.5
    ep2 = ops.epilogue(bn_part=part2, bn_mode=2, bn_slots=sl2, bn_z=z, bn_ss=ss, bn_mi=mi, bn_act=L.ACT_RELU,
                       bn_fold=P)
    for dbg in (0, 1, 2, 4, 8, 15, 16, 31, 32):
        L.check(lib.cgan3d_set_tuning(11, dbg), "dbg")
        t1 = timeit(lambda: ops.conv(fwd, x, w, y, ep1))
        t2 = timeit(lambda: ops.conv(dg, g, wl, dpad, ep2))
        t3 = timeit(lambda: ops.conv(dg, g, wl, dpad))
        print(f"dbg {dbg:2d}: first fwd+stats {t1:6.1f} us | last dgrad+fold {t2:6.1f} us | last dgrad {t3:6.1f} us",
              flush=True)
    L.check(lib.cgan3d_set_tuning(11, 0), "dbg")


if __name__ == "__main__":
    main()
