"""Time the generator's four stride-2 16 <-> 32 launches (conv_s2.hip) at 64^3 B=4 as the bf16 step
issues them: bf16 shadow input, BatchNorm statistics into fp64 accumulators (forwards: acc mode 3;
input-grads: acc mode 4 with z / scale-shift / mean-invstd of the layer they feed).

    python tools/s2_probe.py [--plain]
"""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "contrast-gan-3d_amd"))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--plain", action="store_true", help="also time each launch without BatchNorm statistics")
    args = ap.parse_args()
    from cgan3d_amd import ops, _lib as L
    BF = L.PREC_BF16
    dev = torch.device("cuda")
    B, S = 4, 64
    F3, H3 = (S,) * 3, (S // 2,) * 3
    keep = []

    def t(*s):
        return torch.randn(*s, device=dev)

    def packed(geo, w):
        ps = ops.PackSet(dev)
        geo, w = ps.add(geo, w, BF)
        ps.pack()
        keep.append(ps)
        return geo, w

    def acc(c):
        return torch.zeros(16 * 2 * c, dtype=torch.float64, device=dev)

    def bn4(c, dims):
        z = t(B, *dims, c)
        ss = torch.cat([torch.rand(c, device=dev) + 0.5, t(c) * 0.1])
        mi = torch.cat([t(c) * 0.1, torch.rand(c, device=dev) + 0.5])
        return dict(bn_z=z, bn_ss=ss, bn_mi=mi, bn_act=L.ACT_RELU, fuse=ops.BnFuse(acc(c), 4, 16))

    w_down = t(32, 16, 3, 3, 3) * 0.05  # Conv3d 16 -> 32 [cout][cin]
    w_up = t(32, 16, 3, 3, 3) * 0.05    # ConvTranspose3d 32 -> 16 [cin][cout]
    cases = []
    g, w = packed(ops.conv_fwd_geom(B, F3, H3, 16, 32, 3, 2, 1), w_down)
    x = t(B, *F3, 16)
    cases.append(("s2f fwd (down0)", g, x, w, torch.empty(B, *H3, 32, device=dev),
                  dict(x_bf16=x.bfloat16(), fuse=ops.BnFuse(acc(32), 3, 16))))
    g, w = packed(ops.convt_fwd_geom(B, H3, F3, 32, 16, 3, 2, 1), w_up)
    x = t(B, *H3, 32)
    cases.append(("s2t fwd (up1)", g, x, w, torch.empty(B, *F3, 16, device=dev),
                  dict(x_bf16=x.bfloat16(), fuse=ops.BnFuse(acc(16), 3, 16))))
    g, w = packed(ops.convt_dgrad_geom(B, H3, F3, 32, 16, 3, 2, 1), w_up)
    x = t(B, *F3, 16)
    cases.append(("s2f dgrad (up1)", g, x, w, torch.empty(B, *H3, 32, device=dev),
                  dict(x_bf16=x.bfloat16(), **bn4(32, H3))))
    g, w = packed(ops.conv_dgrad_geom(B, F3, H3, 16, 32, 3, 2, 1), w_down)
    x = t(B, *H3, 32)
    cases.append(("s2t dgrad (down0)", g, x, w, torch.empty(B, *F3, 16, device=dev),
                  dict(x_bf16=x.bfloat16(), **bn4(16, F3))))
    lib = L.load()
    for dbg in (0,):
        variants = [(n, g, x, w, y, kw) for n, g, x, w, y, kw in cases]
        if args.plain:
            variants += [(n + " plain", g, x, w, y, dict(x_bf16=kw["x_bf16"])) for n, g, x, w, y, kw in cases]
        for name, g, x, w, y, kw in variants:
            ep = ops.epilogue(**kw)
            for _ in range(3):
                ops.conv(g, x, w, y, ep)
            torch.cuda.synchronize()
            # repeats captured in a HIP graph: host launch overhead stays out of the timing
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                for _ in range(args.reps):
                    ops.conv(g, x, w, y, ep)
            graph.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            graph.replay()
            e1.record()
            torch.cuda.synchronize()
            print(f"{name}: {e0.elapsed_time(e1) / args.reps * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
