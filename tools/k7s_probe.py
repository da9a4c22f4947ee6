"""Time the generator's last conv (16 -> 1 k7 reflect, bf16 shadow input) at 64^3 B=4 alone: the
streamed-plane kernel at each output-plane chunk (cgan3d_set_tuning key 13), then the Toeplitz
k7m_w2n kernel (key 13 = -1)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "contrast-gan-3d_amd"))
import torch  # noqa: E402


def main():
    from cgan3d_amd import ops, _lib as L
    n, S = 4, 64
    dims = (S, S, S)
    geo = ops.with_prec(ops.conv_fwd_geom(n, dims, dims, 16, 1, 7, 1, 3, True), L.PREC_BF16)
    x = torch.randn(n, *dims, 16, device="cuda")
    x16 = x.bfloat16()
    w = torch.randn(1, 16, 7, 7, 7, device="cuda") * 0.01
    b = torch.zeros(1, device="cuda")
    y = torch.empty(n, *dims, 1, device="cuda")
    o2 = torch.empty_like(y)
    mn = torch.randn_like(y)
    lib = L.load()
    for knob in (13,):
        for tdc in (0, 8, 16):
            for dbg in (0,):
                L.check(lib.cgan3d_set_tuning(knob, tdc), "tdc")
                ep = ops.epilogue(bias=b, act=L.ACT_TANH, minuend=mn, out2=o2, x_bf16=x16)
                for _ in range(3):
                    ops.conv(geo, x, w, y, ep)
                torch.cuda.synchronize()
                # repeats captured in a HIP graph: host launch overhead stays out of the timing
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    for _ in range(20):
                        ops.conv(geo, x, w, y, ep)
                graph.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                graph.replay()
                e1.record()
                torch.cuda.synchronize()
                print(f"tdc {tdc} dbg {dbg}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us", flush=True)
    L.check(lib.cgan3d_set_tuning(13, -1), "off")
    for _ in range(3):
        ops.conv(geo, x, w, y, ops.epilogue(bias=b, act=L.ACT_TANH, minuend=mn, out2=o2, x_bf16=x16))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.conv(geo, x, w, y, ops.epilogue(bias=b, act=L.ACT_TANH, minuend=mn, out2=o2, x_bf16=x16))
    e1.record()
    torch.cuda.synchronize()
    print(f"old k7m_w2n: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us")


if __name__ == "__main__":
    main()
