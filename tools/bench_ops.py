"""Per-launch timing of single HIP kernels at the benchmark's shapes (kernel tuning aid).

    python tools/bench_ops.py [--case res_wgrad ...] [--tune KEY=V1,V2,...]

Each case builds its operands once, warms up, captures 20 back-to-back launches in a HIP graph
and times one replay between two HIP events; prints one line per (case, tuning value) with
µs/launch and TFLOP/s (algorithmic).

Phase probes (round 5; timing only, wrong results): build the probe library (make PROBES=1 in
contrast-gan-3d_amd/csrc) and run with CGAN3D_LIB_PATH=contrast-gan-3d_amd/cgan3d_amd/probe/libcgan3d.so
--tune 90=0,1,2,...: bit 1 skips the MFMA loop, 2 the operand loads / DMAs, 4 the unfold (k7m_n2w) or
the partial stores (wgrad_k3m), 8 the output stores, 16 the statistics (common.h CG_PROBE).
"""
import argparse
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "contrast-gan-3d_amd"))

import torch  # noqa: E402


def _cases(B=4, S=64):
    from cgan3d_amd import ops, _lib as L
    BF = L.PREC_BF16
    r = S // 4
    dev = torch.device("cuda")

    def t(*shape):
        return torch.randn(*shape, device=dev)

    def conv_case(geo, cin, cout, din, dout, packed=True, step_epi=False):
        """step_epi: the step's epilogue for the halo-level convs — bf16 input shadow, bf16 output and
        mode-3 accumulator statistics (what routes the 32 <-> 64 pair to conv_t64 / conv_f64)"""
        w = t(cout, cin, geo.k, geo.k, geo.k) * 0.05
        if packed:
            ps = ops.PackSet(dev)
            geo, w = ps.add(geo, w, BF)
            ps.pack()
        x, y = t(B, *din, geo.cin), torch.empty(B, *dout, geo.cout, device=dev)
        # transposed stride-2: each output voxel sums 27 / 8 taps on average (the input-voxel count
        # x 27 is the algorithmic figure)
        nv = B * din[0] * din[1] * din[2] if geo.transposed else B * dout[0] * dout[1] * dout[2]
        flops = 2.0 * nv * geo.cin * geo.cout * geo.k**3
        if step_epi:
            acc = torch.zeros(16 * 2 * geo.cout, device=dev, dtype=torch.float64)
            y16, x16 = y.bfloat16(), x.bfloat16()
            ep = ops.epilogue(x_bf16=x16, fuse=ops.BnFuse(acc, 3, 16))
            return (lambda: ops.conv(geo, x, w, y16, ep)), flops
        return (lambda: ops.conv(geo, x, w, y)), flops

    def wgrad_case(geo, din, dout, shadows=False):
        x, go = t(B, *din, geo.cin), t(B, *dout, geo.cout)
        dw = torch.empty(geo.cout, geo.cin, geo.k, geo.k, geo.k, device=dev)
        # room for any chunk count a --tune 9=... sweep asks for (wgrad_k3_kernel partials)
        ws = torch.empty(max(ops.wgrad_ws_floats(geo), 256 * 27 * 4096 if geo.cin == geo.cout == 64 else 0), device=dev)
        flops = 2.0 * B * dout[0] * dout[1] * dout[2] * geo.cin * geo.cout * geo.k**3
        kw = dict(gathered16=x.bfloat16(), aligned16=go.bfloat16()) if shadows else {}
        return (lambda: ops.wgrad(geo, x, go, dw, ws, **kw)), flops

    R3, H3, F3, P3 = (r,) * 3, (2 * r,) * 3, (S,) * 3, (S + 6,) * 3

    def crit(cin, cout, din, halo=True):
        """critic layer forward over the 3B critic batch (real | fake | interpolation)"""
        n3 = 3 * B
        dout = tuple(d // 2 for d in din)
        old, ops.HALO = ops.HALO, halo
        try:
            geo = ops.conv_fwd_geom(n3, din, dout, cin, cout, 4, 2, 1)
            w = t(cout, cin, 4, 4, 4) * 0.05
            ps = ops.PackSet(dev)
            geo, w = ps.add(geo, w, BF)
            ps.pack()
        finally:
            ops.HALO = old
        x, y = t(n3, *din, cin), torch.empty(n3, *dout, cout, device=dev)
        flops = 2.0 * n3 * dout[0] * dout[1] * dout[2] * cin * cout * 64
        return (lambda: ops.conv(geo, x, w, y)), flops

    def crit_dgrad(cin, cout, din):
        """critic layer input-grad over the 3B critic batch: the transposed k4 s2 map from dL/dz at the
        layer's output grid to dL/dx at din, with the LeakyReLU mask of the layer below"""
        n3 = 3 * B
        dout = tuple(d // 2 for d in din)
        geo = ops.conv_dgrad_geom(n3, din, dout, cin, cout, 4, 2, 1)
        w = t(cout, cin, 4, 4, 4) * 0.05
        ps = ops.PackSet(dev)
        geo, w = ps.add(geo, w, BF)
        ps.pack()
        dz, dx = t(n3, *dout, cout), torch.empty(n3, *din, cin, device=dev)
        m = t(n3, *din, cin)
        ep = ops.epilogue(mask_src=m, slope=0.2)
        flops = 2.0 * n3 * dout[0] * dout[1] * dout[2] * cin * cout * 64
        return (lambda: ops.conv(geo, dz, w, dx, ep)), flops

    def dgrad_m4(cin, cout, din, dout, bf16_out, transposed=False):
        """a stride-2 conv's input-grad as the step issues it at the 32 <-> 64 level (conv_t64 role 2):
        bf16 dL/dz shadow in, dL/dx out with the BatchNorm-backward statistics of the layer below
        (mode 4: its z, scale / shift, mean / invstd) — fp32 or bf16 output and z"""
        geo = (ops.convt_dgrad_geom if transposed else ops.conv_dgrad_geom)(B, din, dout, cin, cout, 3, 2, 1)
        w = t(cin, cout, 3, 3, 3) * 0.05 if transposed else t(cout, cin, 3, 3, 3) * 0.05
        ps = ops.PackSet(dev)
        geo, w = ps.add(geo, w, BF)
        ps.pack()
        dz = t(B, *dout, cout)
        dz16 = dz.bfloat16()
        dx = torch.empty(B, *din, cin, device=dev, dtype=torch.bfloat16 if bf16_out else torch.float32)
        z = t(B, *din, cin)
        z = z.bfloat16() if bf16_out else z
        acc = torch.zeros(16 * 2 * cin, device=dev, dtype=torch.float64)
        ss, mi = torch.ones(2 * cin, device=dev), torch.ones(2 * cin, device=dev)
        ep = ops.epilogue(x_bf16=dz16, bn_z=z, bn_ss=ss, bn_mi=mi, bn_act=L.ACT_RELU, fuse=ops.BnFuse(acc, 4, 16))
        flops = 2.0 * B * dout[0] * dout[1] * dout[2] * cin * cout * 27
        return (lambda: ops.conv(geo, dz, w, dx, ep)), flops

    def ref_add3(shape):
        """calibration: torch's bf16 add (two reads, one write) over a tensor of `shape`; figure = HBM bytes"""
        a, b = t(*shape).bfloat16(), t(*shape).bfloat16()
        o = torch.empty_like(a)
        return (lambda: torch.add(a, b, out=o)), 3 * a.numel() * 2

    def bn_bwd(c, sp, reps=16):
        """a BatchNorm backward pass from the fp64 replicas (bn_bwd_apply_acc_kernel<true>: dy, z bf16 in,
        dz16 out); figure = HBM bytes"""
        dy, z = t(B, *sp, c).bfloat16(), t(B, *sp, c).bfloat16()
        acc = torch.zeros(reps * 2 * c, device=dev, dtype=torch.float64)
        ss, mi = torch.ones(2 * c, device=dev), torch.ones(2 * c, device=dev)
        gamma, dg, db = torch.ones(c, device=dev), torch.zeros(c, device=dev), torch.zeros(c, device=dev)
        dz16 = torch.empty_like(z)
        nv = B * sp[0] * sp[1] * sp[2]
        return (lambda: ops.bn_backward_acc(dy, z, nv, c, acc, reps, ss, mi, gamma, 1, dg, db, None,
                                            dz16=dz16)), 3 * z.numel() * 2

    def bn_fold(fp32_dz=False, reps=16):
        """the generator's last BatchNorm backward with the reflect-pad fold (bn_bwd_apply_fold_kernel,
        bf16 step operands: padded dL/dy and z in, dz16 out); the figure is HBM bytes (column = TB/s)"""
        c, p = 16, 3
        padded = t(B, *(d + 2 * p for d in F3), c).bfloat16()
        z = t(B, *F3, c).bfloat16()
        acc = torch.zeros(reps * 2 * c, device=dev, dtype=torch.float64)
        acc[c:2 * c] = 1.0
        ss, mi = torch.ones(2 * c, device=dev), torch.ones(2 * c, device=dev)
        gamma, dg, db = torch.ones(c, device=dev), torch.zeros(c, device=dev), torch.zeros(c, device=dev)
        dz16 = torch.empty(B, *F3, c, device=dev, dtype=torch.bfloat16)
        dz = torch.empty(B, *F3, c, device=dev) if fp32_dz else None
        nbytes = B * S**3 * c * (2 + 2 + 2 + (4 if fp32_dz else 0))
        return (lambda: ops.bn_backward_acc_fold(padded, z, B, F3, c, p, acc, reps, ss, mi, gamma, 1, dg, db, dz,
                                                 dz16=dz16)), nbytes

    def res_wgrad_k3m():
        """ResNet-block weight grad as the bf16 step issues it (both operands' bf16 shadows:
        wgrad_k3m_kernel + wgrad_reduce_lin_kernel)"""
        geo = ops.with_prec(ops.conv_wgrad_geom(B, R3, R3, 64, 64, 3, 1, 1), BF)
        x, go = t(B, *R3, 64), t(B, *R3, 64)
        x16, go16 = x.bfloat16(), go.bfloat16()
        dw = torch.empty(64, 64, 3, 3, 3, device=dev)
        ws = torch.empty(ops.wgrad_ws_floats(geo), device=dev)
        flops = 2.0 * B * r**3 * 64 * 64 * 27
        return (lambda: ops.wgrad(geo, x, go, dw, ws, gathered16=x16, aligned16=go16)), flops

    def crit_wgrad():
        """the critic's first layer weight-grad over the 3B critic batch (conv_c1.hip)"""
        n3 = 3 * B
        geo = ops.conv_wgrad_geom(n3, F3, H3, 1, 8, 4, 2, 1)
        x, go = t(n3, *F3, 1), t(n3, *H3, 8)
        dw = torch.empty(8, 1, 4, 4, 4, device=dev)
        ws = torch.empty(max(ops.wgrad_ws_floats(geo), 1), device=dev)
        return (lambda: ops.wgrad(geo, x, go, dw, ws)), 2.0 * n3 * H3[0] ** 3 * 8 * 64

    def res_k3m(dgrad, reps=16, stats=True, res=True):
        """ResNet-block conv as the bf16 step issues it: bf16 shadow input, fp64 accumulator statistics
        (mode 3 forward with the residual + ReLU epilogue; mode 4 input-grad), conv_k3m_kernel"""
        geo0 = (ops.conv_dgrad_geom if dgrad else ops.conv_fwd_geom)(B, R3, R3, 64, 64, 3, 1, 1)
        w = t(64, 64, 3, 3, 3) * 0.05
        ps = ops.PackSet(dev)
        geo, w = ps.add(geo0, w, BF)
        ps.pack()
        x, y = t(B, *R3, 64), torch.empty(B, *R3, 64, device=dev)
        x16 = x.bfloat16()
        acc = torch.zeros(reps * 2 * 64, device=dev, dtype=torch.float64)
        rt = t(B, *R3, 64) if res else None
        if dgrad:
            z, ss, mi = t(B, *R3, 64), torch.rand(128, device=dev) + 0.5, torch.rand(128, device=dev) + 0.5
            ep = ops.epilogue(x_bf16=x16, residual=rt, bn_z=z if stats else None, bn_ss=ss, bn_mi=mi,
                              bn_act=L.ACT_NONE, fuse=ops.BnFuse(acc, 4, reps) if stats else None)
        else:
            ep = ops.epilogue(x_bf16=x16, act=L.ACT_RELU, residual=rt, fuse=ops.BnFuse(acc, 3, reps) if stats else None)
        flops = 2.0 * B * r**3 * 64 * 64 * 27
        return (lambda: ops.conv(geo, x, w, y, ep)), flops

    def k7_first_step():
        """generator first conv (1 -> 16 k7 reflect) as the bf16 step issues it: bf16 z out, fp64
        accumulator statistics (k7m_n2w_kernel<true>)"""
        geo = ops.with_prec(ops.conv_fwd_geom(B, F3, F3, 1, 16, 7, 1, 3, True), BF)
        w = t(16, 1, 7, 7, 7) * 0.05
        x, y = t(B, *F3, 1), torch.empty(B, *F3, 16, device=dev, dtype=torch.bfloat16)
        acc = torch.zeros(16 * 2 * 16, device=dev, dtype=torch.float64)
        ep = ops.epilogue(fuse=ops.BnFuse(acc, 3, 16))
        return (lambda: ops.conv(geo, x, w, y, ep)), 2.0 * B * S**3 * 16 * 343

    def k7_last_dgrad_step():
        """the generator last conv's input-grad as the bf16 step issues it: onto the reflect-padded grid,
        bf16 output, the folded mode-2 statistics of the BatchNorm below from its bf16 z (fp64 accumulators)"""
        P3_ = (S + 6,) * 3
        geo = ops.with_prec(ops.conv_dgrad_geom(B, P3_, F3, 16, 1, 7, 1, 0), BF)
        w = t(1, 16, 7, 7, 7) * 0.05
        dz = t(B, *F3, 1)
        y = torch.empty(B, *P3_, 16, device=dev, dtype=torch.bfloat16)
        z = t(B, *F3, 16).bfloat16()
        ss, mi = torch.ones(32, device=dev), torch.ones(32, device=dev)
        acc = torch.zeros(16 * 2 * 16, device=dev, dtype=torch.float64)
        ep = ops.epilogue(bn_z=z, bn_ss=ss, bn_mi=mi, bn_act=L.ACT_RELU, fuse=ops.BnFuse(acc, 4, 16))
        ep.bn_fold = 3
        return (lambda: ops.conv(geo, dz, w, y, ep)), 2.0 * B * S**3 * 16 * 343

    def k7_wgrad_step(last):
        """a k7 weight grad as the bf16 step issues it: the 16-channel operand from its bf16 shadow
        (dL/dz of the first conv / the last conv's input)"""
        cin, cout = (16, 1) if last else (1, 16)
        geo = ops.with_prec(ops.conv_wgrad_geom(B, F3, F3, cin, cout, 7, 1, 3, True), BF)
        x, go = t(B, *F3, cin), t(B, *F3, cout)
        dw = torch.empty(cout, cin, 7, 7, 7, device=dev)
        ws = torch.empty(ops.wgrad_ws_floats(geo), device=dev)
        kw = dict(gathered16=x.bfloat16()) if last else dict(aligned16=go.bfloat16())
        return (lambda: ops.wgrad(geo, x, go, dw, ws, **kw)), 2.0 * B * S**3 * 16 * 343

    return {
        "k7_first_wgrad_step": lambda: k7_wgrad_step(False),
        "k7_last_wgrad_step": lambda: k7_wgrad_step(True),
        "k7_first_step": lambda: k7_first_step(),
        "k7_last_dgrad_step": lambda: k7_last_dgrad_step(),
        "res_fwd_k3m": lambda: res_k3m(False),
        "res_dgrad_k3m": lambda: res_k3m(True),
        "res_fwd_k3m_r64": lambda: res_k3m(False, reps=64),
        "res_dgrad_k3m_r64": lambda: res_k3m(True, reps=64),
        "res_fwd_k3m_nostat": lambda: res_k3m(False, stats=False),
        "res_fwd_k3m_plain": lambda: res_k3m(False, stats=False, res=False),
        "crit_first": lambda: crit(1, 8, F3),
        "crit_first_wgrad": lambda: crit_wgrad(),
        "res_wgrad_k3m": lambda: res_wgrad_k3m(),
        "crit_m0": lambda: crit(8, 16, H3),
        "crit_m1": lambda: crit(16, 32, R3),
        "crit_m2": lambda: crit(32, 64, (r // 2,) * 3),
        "crit_m2_gemm": lambda: crit(32, 64, (r // 2,) * 3, halo=False),
        "down1_dgrad_m4": lambda: dgrad_m4(32, 64, H3, R3, False),
        "down1_dgrad_m4_bf16": lambda: dgrad_m4(32, 64, H3, R3, True),
        "up0_dgrad_m4": lambda: dgrad_m4(64, 32, R3, H3, False, True),
        "bn_fold64": lambda: bn_fold(),
        "bn_fold64_dz": lambda: bn_fold(True),
        "bn_fold64_r1": lambda: bn_fold(reps=1),
        "ref_add3_64": lambda: ref_add3((B, S, S, S, 16)),
        "ref_add3_16": lambda: ref_add3((B, r, r, r, 64)),
        "bn_bwd16": lambda: bn_bwd(64, R3),
        "bn_bwd16_r1": lambda: bn_bwd(64, R3, reps=1),
        "bn_bwd32": lambda: bn_bwd(32, H3),
        "crit_m0_dgrad": lambda: crit_dgrad(8, 16, H3),
        "crit_m1_dgrad": lambda: crit_dgrad(16, 32, R3),
        "crit_m2_dgrad": lambda: crit_dgrad(32, 64, (r // 2,) * 3),
        "res_fwd": lambda: conv_case(ops.conv_fwd_geom(B, R3, R3, 64, 64, 3, 1, 1), 64, 64, R3, R3),
        "res_wgrad": lambda: wgrad_case(ops.with_prec(ops.conv_wgrad_geom(B, R3, R3, 64, 64, 3, 1, 1), BF), R3, R3),
        "down0_wgrad": lambda: wgrad_case(ops.with_prec(ops.conv_wgrad_geom(B, F3, H3, 16, 32, 3, 2, 1), BF), F3, H3),
        "down0_wgrad_step": lambda: wgrad_case(ops.with_prec(ops.conv_wgrad_geom(B, F3, H3, 16, 32, 3, 2, 1), BF), F3, H3,
                                               shadows=True),
        "down1_wgrad_step": lambda: wgrad_case(ops.with_prec(ops.conv_wgrad_geom(B, H3, R3, 32, 64, 3, 2, 1), BF), H3, R3,
                                               shadows=True),
        "down0_fwd": lambda: conv_case(ops.conv_fwd_geom(B, F3, H3, 16, 32, 3, 2, 1), 16, 32, F3, H3),
        "up0_fwd": lambda: conv_case(ops.convt_fwd_geom(B, R3, H3, 64, 32, 3, 2, 1), 64, 32, R3, H3),
        "down1_fwd": lambda: conv_case(ops.conv_fwd_geom(B, H3, R3, 32, 64, 3, 2, 1), 32, 64, H3, R3),
        "up0_fwd_step": lambda: conv_case(ops.convt_fwd_geom(B, R3, H3, 64, 32, 3, 2, 1), 64, 32, R3, H3, step_epi=True),
        "down1_fwd_step": lambda: conv_case(ops.conv_fwd_geom(B, H3, R3, 32, 64, 3, 2, 1), 32, 64, H3, R3, step_epi=True),
        "up1_fwd": lambda: conv_case(ops.convt_fwd_geom(B, H3, F3, 32, 16, 3, 2, 1), 32, 16, H3, F3),
        "k7_last_fwd": lambda: conv_case(ops.with_prec(ops.conv_fwd_geom(B, F3, F3, 16, 1, 7, 1, 3, True), BF), 16, 1,
                                         F3, F3, packed=False),
        "k7_first_fwd": lambda: conv_case(ops.with_prec(ops.conv_fwd_geom(B, F3, F3, 1, 16, 7, 1, 3, True), BF), 1, 16,
                                          F3, F3, packed=False),
        "k7_last_dgrad": lambda: conv_case(ops.with_prec(ops.conv_dgrad_geom(B, P3, F3, 16, 1, 7, 1, 0), BF), 1, 16,
                                           F3, P3, packed=False),
        "k7_first_wgrad": lambda: wgrad_case(ops.with_prec(ops.conv_wgrad_geom(B, F3, F3, 1, 16, 7, 1, 3, True), BF),
                                             F3, F3),
        "k7_last_wgrad": lambda: wgrad_case(ops.with_prec(ops.conv_wgrad_geom(B, F3, F3, 16, 1, 7, 1, 3, True), BF),
                                            F3, F3),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", nargs="*", default=None)
    ap.add_argument("--tune", default=None, help="KEY=v1,v2,... (cgan3d_set_tuning)")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    from cgan3d_amd import _lib as L
    lib = L.load()
    cases = _cases()
    names = args.case or list(cases)
    tunes = [(None, None)]
    if args.tune:
        k, vs = args.tune.split("=")
        tunes = [(int(k), int(v)) for v in vs.split(",")]
    for key, val in tunes:
        if key is not None:
            L.check(lib.cgan3d_set_tuning(key, val), "set_tuning")
        for nm in names:
            fn, flops = cases[nm]()
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            # the repeats are captured in a HIP graph: host launch overhead stays out of the timing
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                for _ in range(args.reps):
                    fn()
            graph.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            graph.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.reps
            tag = f" tune{key}={val}" if key is not None else ""
            print(f"{nm:14s}{tag:16s} {us:9.2f} us  {flops / us / 1e6:8.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
