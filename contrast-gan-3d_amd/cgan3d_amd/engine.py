"""The G+D training step as an explicit, hand-scheduled sequence of HIP launches.

This is the hot path (BASELINE.json north_star): ``Trainer.train_step``
(contrast_gan_3D/trainer/Trainer.py:163-203) = generator forward, critic update with the WGAN
gradient penalty (Trainer.py:108-142, model/utils.py:12-41), generator update
(Trainer.py:144-161), Adam on both (basic_conf.py:55,67).

Instead of recording an autograd graph (and a double-backward graph for the GP), the backward
passes are derived by hand and scheduled explicitly:

* Generator backward: BN / ReLU / residual / ConvTranspose / reflect-pad chain rule.
* Critic update: one batched forward over ``[real | fake | interpolation]`` (exact: the GP-conf
  critic has no batch coupling), one batched input-grad chain (the interpolation rows seeded
  with ones give g = dD/dx), the GP reduction producing gamma = dGP/dg, then the *forward-mode*
  chain nu_l = mask_l * conv_l(nu_{l-1}) from gamma, which turns the double backward into plain
  weight-gradients: dW_l += wgrad(nu_{l-1}, dz_l[interp]).  Biases get no GP gradient and
  LeakyReLU masks are piecewise constant, so this equals torch's double backward exactly in
  real arithmetic.  The reference's zero-valued generator backward through the GP
   is not executed.
* The critic weight-gradients the reference computes during the generator update are discarded
  by its next ``zero_grad`` (Trainer.py:111) and are not computed here.

All buffers are allocated once per (batch, patch) shape; every launch goes to the current
stream with device-resident scalars (Adam step/lr), so ``step`` can be captured in a HIP graph.
Activations are channels-last fp32 (see include/cgan3d.h).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib as L
from . import ops

Dims = Tuple[int, int, int]

# Environment switches (the whole list):
#   CGAN3D_DEBUG=flag[,flag]   comparator paths the tests run against the default (read at plan
#                              construction): no_shadow (fp32 conv inputs, no bf16 shadows), keep_fp32
#                              (write fp32 tensors only shadow readers consume), no_bn_fuse (BatchNorm
#                              slabs + finalize launches instead of fp64 accumulators), no_bn_fold
#                              (reflect-fold pass before the last BatchNorm backward), serial (no side
#                              streams: a kernel trace then shows unshared durations), system_fence
#                              (cross-stream event records with the system-scope fence, csrc/plan.hip),
#                              fp32_store (the 64^3 16-channel z / dy in fp32 instead of bf16),
#                              event_record (a marker event per cross-stream wait instead of the
#                              waited-on launch's own completion event, csrc/plan.hip), own_streams (a new
#                              side / communication stream per plan instead of ops.pooled_stream),
#                              no_wgrad_sk (the critic's middle-layer weight grads on the generic kernel),
#                              no_defer_reduce (one partial-reduce launch per ResNet weight grad),
#                              bn_pre (opt-in: the ResNet chain's BatchNorm passes folded into the next
#                              conv's staging, cgan3d_bn_pre — measured slower)
#   CGAN3D_FORCE_DP=1          the data-parallel path over a one-rank group (tools / tests)
#   CGAN3D_COMM=native|torch|own   data-parallel collectives: RCCL from the launch plan on the process
#                              group's communicator (default), torch.distributed host callables (the
#                              fallback), or a communicator of the library's own (ops.NativeComm)
#   CGAN3D_G_BUCKET_BYTES      generator gradient bucket size under data parallelism
#   CGAN3D_TUNE, CGAN3D_LIB_PATH   launch-shape knobs, another build of the library (_lib.py)
#   CGAN3D_TRAINER_PLANS=0     the drop-in Trainer issues every step eagerly (no recorded plans)
DEBUG_FLAGS = ("no_shadow", "keep_fp32", "no_bn_fuse", "no_bn_fold", "serial", "system_fence", "fp32_store",
               "event_record", "own_streams", "no_wgrad_sk", "no_defer_reduce", "bn_pre")


def debug(flag: str) -> bool:
    """True if comparator ``flag`` is set in CGAN3D_DEBUG (read when a plan is built)."""
    assert flag in DEBUG_FLAGS, flag
    flags = set(filter(None, os.environ.get("CGAN3D_DEBUG", "").replace(" ", "").split(",")))
    unknown = flags - set(DEBUG_FLAGS)
    if unknown:
        raise ValueError(f"CGAN3D_DEBUG: unknown flags {sorted(unknown)} (known: {', '.join(DEBUG_FLAGS)})")
    return flag in flags


# generator BatchNorm backward: statistics fused into the kernel that produces dL/dy
BN_FUSED_BWD = True
# weight grads of consecutive ResNet-block layers per cross-stream wait (GeneratorPlan.backward;
# groups of 1 or 4 measured 1.92 / 1.96 against 1.88 ms/step at 2)
WGRAD_GROUP = 2
# the generator's first WGRAD_TAIL_MAIN layers (the end of its backward) compute their weight grads
# on the main stream: nothing is left there to overlap them with, and on the side stream they cost
# two cross-stream hand-offs and share the chip with the stride-2 input-grad (1 and 3
# measured 1.895 / 1.931 against 1.880 ms/step at 2 in round 2; re-swept on the round-6 kernels, where
# the first stride-2 layer's weight grad beside its input-grad pays: 1 measured 1.264 against 1.277
# ms/step at 2, 0 1.29, profiles/r06_ab_knobs.txt)
WGRAD_TAIL_MAIN = 1
# data parallelism: generator gradient bucket size (all-reduce started per bucket during the backward)
# (measured on one GPU over a one-rank RCCL group: each extra bucket ~15 us of step time, so the
# default makes ~2-3 buckets of the 4.1 MB arena: 2.21 ms/step at 1 MB, 2.16 with 2 buckets)
G_BUCKET_BYTES = int(os.environ.get("CGAN3D_G_BUCKET_BYTES", str(2 << 20)))
# BatchNorm statistics through fp64 accumulators (include/cgan3d.h cgan3d_bn_fuse; bf16): the
# producing conv adds its statistics into FUSE_REPS replicas, the layer's one elementwise launch
# finalizes and applies them
FUSE_REPS = 16


def _half(d: Dims) -> Dims:
    return tuple((x + 2 * 1 - 3) // 2 + 1 for x in d)


def _conv_out(d: Dims, k, s, p, planar: bool = False) -> Dims:
    """Output dims of a conv; ``planar`` (the 2-D variants on dims (1, H, W)): depth passes through."""
    if planar:
        return (1,) + tuple((x + 2 * p - k) // s + 1 for x in d[1:])
    return tuple((x + 2 * p - k) // s + 1 for x in d)


def _planar_dims(dims, planar: bool) -> Dims:
    """(H, W) or (1, H, W) -> (1, H, W) for the 2-D variants; 3-D dims unchanged."""
    dims = tuple(int(x) for x in dims)
    if planar and len(dims) == 2:
        return (1,) + dims
    if planar and dims[0] != 1:
        raise ValueError(f"2-D variant: dims must be (H, W) or (1, H, W), got {dims}")
    if len(dims) != 3:
        raise ValueError(f"dims must have three entries, got {dims}")
    return dims


class Arena:
    """One flat fp32 buffer for a module's parameters (+ grads + Adam moments).

    ``p.data`` and ``p.grad`` become views into the arena, so one launch updates every tensor
    (fused multi-tensor Adam) and the module's ``state_dict`` stays the reference's.
    """

    def __init__(self, module: torch.nn.Module, device):
        self.names, self.params = [], []
        for n, p in module.named_parameters():
            self.names.append(n)
            self.params.append(p)
        total = sum(p.numel() for p in self.params)
        self.flat = torch.empty(total, device=device, dtype=torch.float32)
        # grad storage padded to whole 64-byte lines: the per-update memset of the arena
        # (ops.zero(grad_padded)) is then one fill with no unaligned tail
        self.grad_padded = torch.zeros((total + 15) // 16 * 16, device=device, dtype=torch.float32)
        self.grad = self.grad_padded[:total]
        self.exp_avg = torch.zeros(total, device=device, dtype=torch.float32)
        self.exp_avg_sq = torch.zeros(total, device=device, dtype=torch.float32)
        self.views, self.gviews = {}, {}
        off = 0
        with torch.no_grad():
            for n, p in zip(self.names, self.params):
                k = p.numel()
                v = self.flat[off:off + k].view_as(p)
                v.copy_(p.data)
                p.data = v
                p.grad = self.grad[off:off + k].view_as(p)
                self.views[n] = v
                self.gviews[n] = p.grad
                off += k
        self.numel = total

    def rebind_grads(self):
        """Re-attach ``p.grad`` views (a user ``zero_grad(set_to_none=True)`` drops them)."""
        for p, g in zip(self.params, self.gviews.values()):
            p.grad = g


# ----------------------------------------------------------------------------------------------
@dataclass
class _GLayer:
    kind: str            # conv | convt | last
    name: str            # state_dict prefix
    k: int
    s: int
    p: int
    reflect: bool
    cin: int
    cout: int
    din: Dims
    dout: Dims
    act: int = L.ACT_RELU
    residual: bool = False


class GeneratorPlan:
    """Buffers + launch geometry of ResnetGenerator (model/generator.py:9-90) for a batch shape."""

    def __init__(self, cfg, n: int, dims: Dims, device, P: Dict[str, torch.Tensor], prec: int = L.PREC_F32,
                 allow_resize: bool = False):
        """``allow_resize`` (forward-only plans): input dims that are not multiples of 4 give an
        output of other dims, as the reference's convolution arithmetic does (the whole-scan
        corrector then resizes it, eval/CCTAContrastCorrector.py:42-52)."""
        c0 = cfg.init_channels_out
        # host-schedule knobs (CGAN3D_TUNE keys 100 / 101, sweeps): weight-grad hand-off group size,
        # layers at the end of the backward whose weight grads stay on the main stream
        self.wgrad_group = L.py_tune(100, WGRAD_GROUP)
        self.wgrad_tail_main = L.py_tune(101, WGRAD_TAIL_MAIN)
        # the 2-D variants (experiments/conf_2D.py, is_2D): planar geometries on dims (1, H, W), f32
        self.planar = pl = bool(getattr(cfg, "is_2D", False))
        if pl and prec != L.PREC_F32:
            raise NotImplementedError("the 2-D variants run the exact-f32 path (precision='f32')")
        dims = _planar_dims(dims, pl)
        self.n, self.dims, self.device = n, tuple(dims), device
        self.packs = ops.PackSet(device)  # packed [tap][cin][cout] weight copies, refreshed per update
        # ... of the layers whose weight grads end the backward on the main stream (pack_tail)
        self.packs_tail = ops.PackSet(device)
        layers: List[_GLayer] = [_GLayer("conv", "model.first", 7, 1, 3, True, 1, c0, dims, dims)]
        d = tuple(dims)
        for i in range(cfg.n_updownsample_blocks):
            ci = c0 * 2**i
            dn = _conv_out(d, 3, 2, 1, pl)
            layers.append(_GLayer("conv", f"model.downsampling.{i}", 3, 2, 1, False, ci, 2 * ci, d, dn))
            d = dn
        cr = c0 * 2**cfg.n_updownsample_blocks
        for r in range(cfg.n_resnet_blocks):
            layers.append(_GLayer("conv", f"model.resnet_backbone.{r}.block0", 3, 1, 1, False, cr, cr, d, d,
                                  act=L.ACT_NONE))
            layers.append(_GLayer("conv", f"model.resnet_backbone.{r}.block1", 3, 1, 1, False, cr, cr, d, d,
                                  residual=True))
        for j, i in enumerate(range(cfg.n_updownsample_blocks, 0, -1)):
            ci = c0 * 2**i
            up = tuple(x if (pl and a == 0) else 2 * x for a, x in enumerate(d))  # k3 s2 p1 output_padding 1
            layers.append(_GLayer("convt", f"model.upsampling.{j}", 3, 2, 1, False, ci, ci // 2, d, up))
            d = up
        if not allow_resize:
            assert d == tuple(dims), f"generator output dims {d} != input dims {dims} (need dims % 4 == 0)"
        self.out_dims = d
        self.last = _GLayer("last", "model.last_conv", 7, 1, 3, True, c0, 1, d, d, act=L.ACT_TANH)
        self.layers = layers

        def buf(dd, c):
            return torch.empty((n, *dd, c), device=device, dtype=torch.float32)

        self.geo_fwd, self.geo_dgrad, self.geo_wgrad, self.wf, self.wd = [], [], [], [], []
        self.z, self.y, self.dy, self.dz, self.ss, self.mi = [], [], [], [], [], []
        # fused BatchNorm statistics: per-block partial slabs written by the producing kernels
        self.slots_f, self.part_f = [], []
        ws = 0
        for li, ly in enumerate(layers):
            if ly.kind == "conv":
                gf = ops.conv_fwd_geom(n, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p, ly.reflect, planar=pl)
                gd = ops.conv_dgrad_geom(n, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p, planar=pl)
                gw = ops.conv_wgrad_geom(n, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p, ly.reflect, planar=pl)
            else:
                gf = ops.convt_fwd_geom(n, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p, planar=pl)
                gd = ops.convt_dgrad_geom(n, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p, planar=pl)
                gw = ops.convt_wgrad_geom(n, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p, planar=pl)
            gw = ops.with_prec(gw, prec)
            wt = P[f"{ly.name}.conv.weight"]
            ps = self.packs_tail if li < self.wgrad_tail_main else self.packs
            gf, wf = ps.add(gf, wt, prec)
            gd, wd = ps.add(gd, wt, prec)
            self.wf.append(wf)
            self.wd.append(wd)
            self.geo_fwd.append(gf)
            self.geo_dgrad.append(gd)
            self.geo_wgrad.append(gw)
            self.z.append(buf(ly.dout, ly.cout))
            self.y.append(buf(ly.dout, ly.cout))
            self.dy.append(buf(ly.dout, ly.cout))
            self.dz.append(buf(ly.dout, ly.cout))
            self.slots_f.append(ops.bn_slots(gf))
            self.part_f.append(torch.empty((2 * ly.cout + 1) * self.slots_f[-1], device=device))
            self.ss.append(torch.empty(2 * ly.cout, device=device))
            self.mi.append(torch.empty(2 * ly.cout, device=device))
            nvox = n * ly.dout[0] * ly.dout[1] * ly.dout[2]
            ws = max(ws, ops.wgrad_ws_floats(gw), ops.bn_backward_ws_floats(nvox, ly.cout))
        la = self.last
        pd = tuple(x if (pl and a == 0) else x + 2 * la.p for a, x in enumerate(la.din))
        self.geo_last_fwd = ops.with_prec(ops.conv_fwd_geom(n, la.din, la.dout, la.cin, 1, la.k, 1, la.p, True,
                                                            planar=pl), prec)
        self.geo_last_wgrad = ops.with_prec(ops.conv_wgrad_geom(n, la.din, la.dout, la.cin, 1, la.k, 1, la.p, True,
                                                                planar=pl), prec)
        self.geo_last_dgrad = ops.with_prec(ops.conv_dgrad_geom(n, pd, la.dout, la.cin, 1, la.k, 1, 0, planar=pl),
                                            prec)  # padded grid
        # backward slabs: layer i's dL/dy comes from layer i+1's input-grad launch, the last one's
        # from the reflect fold of the last conv's input-grad
        self.slots_b = [ops.bn_slots(self.geo_dgrad[i + 1]) for i in range(len(layers) - 1)]
        self.slots_b.append(ops.reflect_fold_slots(n, la.din, la.cin))
        self.part_b = [torch.empty(2 * ly.cout * sl, device=device) for ly, sl in zip(layers, self.slots_b)]
        # bf16: the last BatchNorm layer's backward statistics come from the last conv's input-grad
        # launch itself (folded over the reflect pad) and its elementwise pass folds the padded grid
        # on the fly — no reflect-fold pass and no fp32 dL/dy of that layer (cgan3d_epilogue.bn_fold)
        self.fold_bn = (BN_FUSED_BWD and not debug("no_bn_fold")
                        and ops.bn_fold_ok(self.geo_last_dgrad))
        if self.fold_bn:
            self.slots_b[-1] = ops.bn_slots(self.geo_last_dgrad)
            self.part_b[-1] = torch.empty(2 * layers[-1].cout * self.slots_b[-1], device=device)
        self.att = buf(la.dout, 1)
        self.dz_last = buf(la.dout, 1)
        self.dpad = buf(pd, la.cin)
        ws = max(ws, ops.wgrad_ws_floats(self.geo_last_wgrad), ops.channel_sum_ws_floats(n * la.dout[0] * la.dout[1] * la.dout[2], 1))
        self.ws = torch.empty(ws, device=device)
        # bf16 shadows of conv inputs (forward: the previous BatchNorm's output; input-grad: the
        # layer's own BatchNorm input-grad), written by the BatchNorm pass that produces the fp32
        # tensor: the halo-staging kernels (ResNet-block conv_k3, the stride-2 S2F / S2T and
        # 32 <-> 64 halo kernels, the last k7 conv) copy their halo from half the bytes with no conversion, and the
        # ResNet / stride-2 weight grads read both operands from them.  bf16 mode only (those
        # kernels round to bf16 anyway): results are bit-identical with or without.
        shadow_kinds = {("conv", 3, 1, 64, 64), ("conv", 3, 2, 16, 32), ("convt", 3, 2, 32, 16),
                        ("conv", 3, 2, 32, 64), ("convt", 3, 2, 64, 32)}
        self.y16, self.dz16 = [None] * len(layers), [None] * len(layers)

        def bf(dd, c):
            return torch.empty((n, *dd, c), device=device, dtype=torch.bfloat16)

        if prec == L.PREC_BF16 and not debug("no_shadow"):
            for i, ly in enumerate(layers):
                if (ly.kind, ly.k, ly.s, ly.cin, ly.cout) not in shadow_kinds or ly.reflect:
                    continue
                if i > 0 and self.geo_fwd[i].w_packed == 2:
                    self.y16[i - 1] = bf(layers[i - 1].dout, ly.cin)
                if self.geo_dgrad[i].w_packed == 2:
                    self.dz16[i] = bf(ly.dout, ly.cout)
            # ... and of the last conv's input (its 16 -> 1 k7 kernel stages a halo of it per tile)
            self.y16[-1] = bf(layers[-1].dout, layers[-1].cout)
            # ... and of the first layer's input-grad (its k7 weight grad's 16-channel operand)
            if BN_FUSED_BWD and ops.shadow_only(self.geo_wgrad[0], 1):
                self.dz16[0] = bf(layers[0].dout, layers[0].cout)
        # fp32 tensors that only shadow-reading kernels consume are not written at all (bf16 mode):
        # at 64^3 the 16-channel outputs / input-grads of the first and last BatchNorm layers, 67 MB
        # each; the tensors stay allocated (same plan addresses), their contents undefined
        self.y_dead, self.dz_dead = [False] * len(layers), [False] * len(layers)
        if not debug("keep_fp32"):
            for i, ly in enumerate(layers):
                if self.y16[i] is not None:
                    if i == len(layers) - 1:
                        self.y_dead[i] = ops.shadow_only(self.geo_last_fwd, 0) and ops.shadow_only(
                            self.geo_last_wgrad, 1)
                    elif not layers[i + 1].name.endswith("block0") and self.dz16[i + 1] is not None:
                        self.y_dead[i] = (ops.shadow_only(self.geo_fwd[i + 1], 0)
                                          and ops.shadow_only(self.geo_wgrad[i + 1], 1))
                if self.dz16[i] is not None and BN_FUSED_BWD:
                    reads_ok = i == 0 or (self.y16[i - 1] is not None and ops.shadow_only(self.geo_dgrad[i], 0))
                    self.dz_dead[i] = reads_ok and ops.shadow_only(self.geo_wgrad[i], 1)
        # BatchNorm statistics through fp64 accumulators (cgan3d_bn_fuse acc_mode 3 / 4) wherever the
        # producing conv can write them (halo-tiled, stride-2 and 1 -> 16 k7 kernels; bf16): the
        # finalize is folded into the elementwise pass, one launch per layer and direction (ac_f[j]:
        # cgan3d_bn_apply_acc; ac_b[j]: cgan3d_bn_backward_acc / _acc_fold); CGAN3D_DEBUG=no_bn_fuse keeps
        # the slab + finalize path (A/B).  Each elementwise launch zeroes the accumulator its
        # predecessor in the same direction read, the first the last one's, so none needs a memset.
        nl = len(layers)
        self.ac_f, self.ac_b = [False] * nl, [False] * nl
        if not debug("no_bn_fuse") and prec == L.PREC_BF16 and not pl and BN_FUSED_BWD:
            self.ac_f = [ops.bn_fuse_ok(self.geo_fwd[j]) for j in range(nl)]
            self.ac_b = [j + 1 < nl and ops.bn_fuse_ok(self.geo_dgrad[j + 1]) for j in range(nl)]
            self.ac_b[-1] = bool(self.fold_bn and ops.bn_fuse_ok(self.geo_last_dgrad))
            if sum(self.ac_f) < 2:
                self.ac_f = [False] * nl
            if sum(self.ac_b) < 2:
                self.ac_b = [False] * nl

        def accs(flags):
            return [torch.zeros(FUSE_REPS * 2 * ly.cout, device=device, dtype=torch.float64) if f else None
                    for ly, f in zip(layers, flags)]
        self.acc_f, self.acc_b = accs(self.ac_f), accs(self.ac_b)
        fo = [j for j in range(nl) if self.ac_f[j]]              # their elementwise passes run in this order
        bo = [j for j in range(nl - 1, -1, -1) if self.ac_b[j]]  # (backward)
        self.acc_zero_f = {j: self.acc_f[fo[k - 1]] for k, j in enumerate(fo)}
        self.acc_zero_b = {j: self.acc_b[bo[k - 1]] for k, j in enumerate(bo)}
        # bf16 storage of BatchNorm inputs and their gradients (round 4): a layer whose conv output z,
        # and the dL/dy the next layer's input-grad writes, are only read by kernels that take bf16
        # (cgan3d_conv3d_out_bf16_ok for both producers; the accumulator BatchNorm passes) keeps them in
        # bf16 in training mode: at 64^3 the first and the last 16-channel layers (z, dy / the last
        # conv's padded input-grad: 67-88 MB fp32 tensors read 2-3 times each).  The statistics still
        # come from the producers' fp32 values.  zs / dys / dpads name the training-mode storage; z / dy
        # / dpad stay fp32 (eval forward, slab paths).  CGAN3D_DEBUG=fp32_store keeps fp32 (A/B).
        self.z16 = [False] * nl
        if any(self.ac_f) and any(self.ac_b) and not debug("fp32_store"):
            for j in range(nl):
                prod = self.geo_last_dgrad if j == nl - 1 else self.geo_dgrad[j + 1]
                # the stride-2 producers write bf16 only when they stage from their input's shadow
                shadows = (j == 0 or self.y16[j - 1] is not None) and (j == nl - 1 or self.dz16[j + 1] is not None)
                self.z16[j] = bool(self.ac_f[j] and self.ac_b[j] and ops.out_bf16_ok(self.geo_fwd[j])
                                   and ops.out_bf16_ok(prod) and (j < nl - 1 or self.fold_bn) and shadows)
        self.zs = [bf(ly.dout, ly.cout) if f else z for ly, f, z in zip(layers, self.z16, self.z)]
        self.dys = [bf(ly.dout, ly.cout) if f and j < nl - 1 else d
                    for j, (ly, f, d) in enumerate(zip(layers, self.z16, self.dy))]
        self.dpads = bf(pd, la.cin) if self.z16[-1] else self.dpad
        # The ResNet chain's BatchNorm passes folded into the next conv (round 5, cgan3d_bn_pre): layer
        # j's forward pass (no residual) into layer j + 1's ResNet-block forward, which stages z_j and
        # writes the activation's bf16 shadow; layer j's backward pass into its own input-grad conv,
        # which stages dL/dy_j and writes dL/dz_j's shadow for the weight grad.  Needs bf16 z / dy
        # storage, shadow-only consumers of the fp32 tensors and the ResNet-block kernel.  Off by
        # default: the folded convs measured 17-22 us against 10.4-12.7 us plus a 5-6 us pass, 1.423 vs
        # 1.381 ms/step (CGAN3D_DEBUG=bn_pre turns it on).
        self.pre_f, self.pre_b = [False] * nl, [False] * nl
        if debug("bn_pre"):
            for j in range(nl):
                self.pre_f[j] = bool(j + 1 < nl and self.ac_f[j] and self.z16[j] and not layers[j].residual
                                     and self.y16[j] is not None and self.y_dead[j]
                                     and ops.bn_pre_ok(self.geo_fwd[j + 1]))
                self.pre_b[j] = bool(j > 0 and self.ac_b[j] and self.z16[j] and j < nl - 1
                                     and self.dz16[j] is not None and self.dz_dead[j]
                                     and ops.bn_pre_ok(self.geo_dgrad[j]))
        # weight gradients run on a side stream, beside the input-gradient chain (each wgrad only
        # needs its layer's dz and input, both final when it is enqueued); own workspace
        wsw = max([ops.wgrad_ws_floats(gw) for gw in self.geo_wgrad] + [ops.wgrad_ws_floats(self.geo_last_wgrad)])
        self.ws_side = torch.empty(wsw, device=device)
        # all-zero workspace of the weight grads that sum into theirs by atomics (ops.wgrad ws_clean:
        # each leaves it zeroed, so no memset per layer); they all run on the side stream, in turn
        self.ws_clean = torch.zeros(wsw, device=device)
        self._csum = {}  # bias-sum launch sets (ops.ChannelSumSet) per gradient dict
        # ResNet weight grads whose partial reduce is deferred to one launch per backward (round 5)
        self.ws_defer, self._deferred_red = {}, []
        # (CGAN3D_DEBUG=serial serialises them, so a kernel trace shows unshared durations)
        on_gpu = torch.device(device).type == "cuda" and not debug("serial")
        self.side = ops.pooled_stream(device, "g_side") if on_gpu else None
        self.pack()

    def _on_side(self, fn):
        """Enqueue ``fn``'s launches on the side stream after everything enqueued so far."""
        if self.side is None:
            return fn()
        ops.stream_wait(self.side, torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.side):
            fn()

    def pack(self):
        """Refresh the packed weight copies; call after every weight update."""
        self.packs.pack()
        self.packs_tail.pack()

    def pack_early(self):
        """The packed copies of the layers updated ahead of the tail (StepEngine._g_early)."""
        self.packs.pack()

    def pack_tail(self):
        self.packs_tail.pack()

    # -- forward: x [n,D,H,W,1] -> att (tanh output); opt_hat_out = x - att (Trainer.py:170-171)
    # Training-mode BatchNorm statistics are fused into the producing conv: fp64 accumulators (ac_f)
    # or per-block partials into a slab (bn_mode 1), finalized by the elementwise launch.
    def forward(self, P: Dict[str, torch.Tensor], x: torch.Tensor, opt_hat_out: Optional[torch.Tensor] = None,
                training: bool = True):
        h = x
        h_res = None
        for i, ly in enumerate(self.layers):
            if ly.name.endswith("block0"):
                h_res = h
            nb = f"{ly.name}.normalization"
            nvox = self.n * ly.dout[0] * ly.dout[1] * ly.dout[2]
            res = h_res if ly.residual else None
            h16 = self.y16[i - 1] if i > 0 else None
            if training:
                if self.ac_f[i]:  # statistics into fp64 accumulators, one finalize + apply launch
                    ep = ops.epilogue(x_bf16=h16, fuse=ops.BnFuse(self.acc_f[i], 3, FUSE_REPS))
                else:
                    ep = ops.epilogue(bn_part=self.part_f[i], bn_mode=1, bn_slots=self.slots_f[i], x_bf16=h16)
                if i > 0 and self.pre_f[i - 1]:  # the previous layer's BatchNorm applied while staging
                    ep.x_bf16, ep.pre = self.zs[i - 1], self._pre_fwd(P, i - 1)
                ops.conv(self.geo_fwd[i], h, self.wf[i], self.zs[i], ep)
                if self.pre_f[i]:
                    pass  # applied by layer i + 1's conv
                elif self.ac_f[i]:
                    ops.bn_apply_acc(self.acc_f[i], FUSE_REPS, ly.cout, nvox, P[f"{nb}.weight"], P[f"{nb}.bias"],
                                     P[f"{nb}.running_mean"], P[f"{nb}.running_var"], P[f"{nb}.num_batches_tracked"],
                                     self.ss[i], self.mi[i], self.zs[i], ly.act, None if self.y_dead[i] else self.y[i],
                                     residual=res, y16=self.y16[i], zero=self.acc_zero_f[i])
                else:
                    ops.bn_apply_slab(self.part_f[i], self.slots_f[i], ly.cout, nvox, P[f"{nb}.weight"],
                                      P[f"{nb}.bias"], P[f"{nb}.running_mean"], P[f"{nb}.running_var"],
                                      P[f"{nb}.num_batches_tracked"], self.ss[i], self.mi[i], self.z[i], ly.act,
                                      None if self.y_dead[i] else self.y[i], residual=res, y16=self.y16[i])
            else:
                ops.conv(self.geo_fwd[i], h, self.wf[i], self.z[i], ops.epilogue(x_bf16=h16))
                self._eval_scale_shift(P, nb, i)
                ops.bn_apply(self.z[i], nvox, ly.cout, self.ss[i], ly.act, self.y[i], residual=res, y16=self.y16[i])
            h = self.y[i]
        la = self.last
        ep = ops.epilogue(bias=P["model.last_conv.bias"], act=L.ACT_TANH,
                          minuend=x if opt_hat_out is not None else None, out2=opt_hat_out, x_bf16=self.y16[-1])
        ops.conv(self.geo_last_fwd, h, P["model.last_conv.weight"], self.att, ep)
        return self.att

    def _pre_fwd(self, P, j):
        """Layer j's BatchNorm (+ act) in the next conv's staging (cgan3d_bn_pre mode 1)."""
        ly, nb = self.layers[j], f"{self.layers[j].name}.normalization"
        return ops.BnPre.forward(self.acc_f[j], FUSE_REPS, ly.cout, self.n * ly.dout[0] * ly.dout[1] * ly.dout[2],
                                 P[f"{nb}.weight"], P[f"{nb}.bias"], P[f"{nb}.running_mean"], P[f"{nb}.running_var"],
                                 P[f"{nb}.num_batches_tracked"], self.ss[j], self.mi[j], ly.act, self.y16[j],
                                 zero=self.acc_zero_f[j])

    def _pre_bwd(self, P, G, j):
        """Layer j's BatchNorm backward in its input-grad conv's staging (cgan3d_bn_pre mode 2)."""
        ly, nb = self.layers[j], f"{self.layers[j].name}.normalization"
        return ops.BnPre.backward(self.zs[j], self.acc_b[j], FUSE_REPS, ly.cout,
                                  self.n * ly.dout[0] * ly.dout[1] * ly.dout[2], self.ss[j], self.mi[j],
                                  P[f"{nb}.weight"], ly.act, G[f"{nb}.weight"], G[f"{nb}.bias"], self.dz16[j],
                                  zero=self.acc_zero_b[j])

    def _bn_grad_epi(self, i, fused: bool = False):
        """Epilogue that accumulates BatchNorm layer i's backward statistics from its dL/dy (into
        the fp64 accumulator of the fused backward when ``fused``)."""
        if not BN_FUSED_BWD:
            return ops.epilogue()
        if fused:
            return ops.epilogue(bn_z=self.zs[i], bn_ss=self.ss[i], bn_mi=self.mi[i], bn_act=self.layers[i].act,
                                fuse=ops.BnFuse(self.acc_b[i], 4, FUSE_REPS))
        return ops.epilogue(bn_part=self.part_b[i], bn_mode=2, bn_slots=self.slots_b[i], bn_z=self.z[i],
                            bn_ss=self.ss[i], bn_mi=self.mi[i], bn_act=self.layers[i].act)

    def _eval_scale_shift(self, P, nb, i):
        # eval-mode BN (Trainer.validate, Trainer.py:248-249): running statistics
        with torch.no_grad():
            inv = torch.rsqrt(P[f"{nb}.running_var"] + 1e-5)
            sc = P[f"{nb}.weight"] * inv
            c = sc.numel()
            self.ss[i][:c].copy_(sc)
            self.ss[i][c:].copy_(P[f"{nb}.bias"] - P[f"{nb}.running_mean"] * sc)

    # -- backward from dz_last = dL/d(pre-tanh) ; writes parameter grads into G (grad views)
    def _wgrad(self, g, a, b, dw, zeroed: bool, main: bool = False, defer_layer: Optional[int] = None, **kw):
        """Weight gradient on the side stream's workspaces: into a pre-zeroed gradient arena
        (``zeroed``) every layer accumulates, and the atomic-workspace geometries take the clean one.
        ``main``: launched on the main stream instead, with the main stream's workspace.
        ``defer_layer``: a partials geometry (the ResNet k3 kernel) leaves its partials in the layer's
        own workspace; ``_reduce_deferred`` sums every such layer in one launch (round 5)."""
        if main:
            return ops.wgrad(g, a, b, dw, self.ws, accumulate=zeroed, **kw)
        if defer_layer is not None:
            wl = self.ws_defer.get(defer_layer)
            if wl is None:
                wl = self.ws_defer[defer_layer] = torch.empty(ops.wgrad_ws_floats(g), device=self.ws.device)
            self._deferred_red.append((g, wl, dw, zeroed))
            return ops.wgrad(g, a, b, dw, wl, accumulate=zeroed, defer_reduce=True, **kw)
        if zeroed and ops.wgrad_ws_atomic(g):
            return ops.wgrad(g, a, b, dw, self.ws_clean, accumulate=True, ws_clean=True, **kw)
        return ops.wgrad(g, a, b, dw, self.ws_side, accumulate=zeroed, **kw)

    def backward(self, P: Dict[str, torch.Tensor], G: Dict[str, torch.Tensor], x: torch.Tensor,
                 grads_enqueued: Optional[Callable[[int], None]] = None, zeroed: bool = False,
                 side_first: Optional[Callable[[], None]] = None, side_after: Optional[Callable[[], None]] = None):
        """``grads_enqueued(i)`` (optional) is called once every launch producing layer i's
        parameter gradients is enqueued (i = len(layers) for the last conv, which goes first; then
        len(layers) - 1 down to 0): the data-parallel engine starts bucket all-reduces there.
        ``zeroed``: the gradient views in G were zeroed (one memset of the arena) after the last
        reader, so weight gradients are added into them without a memset per layer."""
        la = self.last
        n = self.n
        u = self.y[-1]

        nvl = n * la.dout[0] * la.dout[1] * la.dout[2]
        key = (id(G), "last_bias")
        if key not in self._csum:
            self._csum[key] = ops.ChannelSumSet(self.device, [(self.dz_last, nvl, 1, G["model.last_conv.bias"], False)])

        # the last conv's weight and bias grads, beside its input-grad when there is a side stream
        # (measured: after the input-grad instead, 1.78 vs 1.76 ms/step)
        # ``side_first``: the caller's own launch for that side segment (the generator loss)
        self._on_side(lambda: (side_first() if side_first is not None else None,
                               self._wgrad(self.geo_last_wgrad, u, self.dz_last, G["model.last_conv.weight"],
                                           zeroed, gathered16=self.y16[-1] if self.y_dead[-1] else None),
                               self._csum[key].run()))
        pending = []  # (layer, weight-grad launcher) not yet handed to the side stream
        # single GPU: the ResNet weight grads leave their partials in per-layer workspaces and the
        # lowest ResNet layer's hand-off sums all of them in one launch (8 reduce launches -> 1;
        # under data parallelism every bucket needs its layers' final gradients: per-layer reduce)
        # only the side-stream layers defer (layers below wgrad_tail_main run their weight grad on the
        # main stream, reduced in place): the combined reduce rides on the lowest DEFERRED layer's flush
        k3 = [i for i in range(len(self.layers)) if ops.wgrad_partials(self.geo_wgrad[i]) > 0
              and not (i < self.wgrad_tail_main and self.side is not None)]
        defer_red = (grads_enqueued is None and self.side is not None and len(k3) > 1
                     and not debug("no_defer_reduce"))
        k3_last = min(k3) if defer_red else None
        self._deferred_red = []

        def flush():
            fns = [f for _, f in pending]
            red = k3_last is not None and any(j == k3_last for j, _ in pending)
            self._on_side(lambda: ([f() for f in fns], self._reduce_deferred() if red else None))
            if grads_enqueued is not None:
                for j, _ in pending:
                    grads_enqueued(j)
            pending.clear()
        if grads_enqueued is not None:
            grads_enqueued(len(self.layers))
        if self.fold_bn:
            ep = self._bn_grad_epi(len(self.layers) - 1, fused=self.ac_b[-1])
            ep.bn_fold = la.p
            ops.conv(self.geo_last_dgrad, self.dz_last, P["model.last_conv.weight"], self.dpads, ep)
        else:
            ops.conv(self.geo_last_dgrad, self.dz_last, P["model.last_conv.weight"], self.dpad)
            ops.reflect_fold(self.dpad, self.dy[-1], n, la.din, la.cin, la.p,
                             ep=self._bn_grad_epi(len(self.layers) - 1), planar=self.planar)

        def resnet_pair(j):  # layers j and j - 1 both in the ResNet chain
            return "resnet_backbone" in self.layers[j].name and "resnet_backbone" in self.layers[j - 1].name
        for i in range(len(self.layers) - 1, -1, -1):
            ly = self.layers[i]
            nb = f"{ly.name}.normalization"
            nvox = n * ly.dout[0] * ly.dout[1] * ly.dout[2]
            if self.pre_b[i]:  # BatchNorm backward in this layer's input-grad (its wgrad reads dz16 after it)
                self._input_grad(P, G, i)
            elif self.ac_b[i] and self.fold_bn and i == len(self.layers) - 1:
                ops.bn_backward_acc_fold(self.dpads, self.zs[i], n, ly.dout, ly.cout, la.p, self.acc_b[i], FUSE_REPS,
                                         self.ss[i], self.mi[i], P[f"{nb}.weight"], ly.act, G[f"{nb}.weight"],
                                         G[f"{nb}.bias"], None if self.dz_dead[i] else self.dz[i], dz16=self.dz16[i],
                                         zero=self.acc_zero_b[i])
            elif self.ac_b[i]:
                ops.bn_backward_acc(self.dys[i], self.zs[i], nvox, ly.cout, self.acc_b[i], FUSE_REPS, self.ss[i], self.mi[i],
                                    P[f"{nb}.weight"], ly.act, G[f"{nb}.weight"], G[f"{nb}.bias"],
                                    None if self.dz_dead[i] else self.dz[i], dz16=self.dz16[i], zero=self.acc_zero_b[i])
            elif BN_FUSED_BWD and self.fold_bn and i == len(self.layers) - 1:
                ops.bn_backward_slab_fold(self.dpad, self.z[i], n, ly.dout, ly.cout, la.p, self.part_b[i],
                                          self.slots_b[i], self.ss[i], self.mi[i], P[f"{nb}.weight"], ly.act,
                                          G[f"{nb}.weight"], G[f"{nb}.bias"], None if self.dz_dead[i] else self.dz[i],
                                          self.ws, dz16=self.dz16[i])
            elif BN_FUSED_BWD:
                ops.bn_backward_slab(self.dy[i], self.z[i], nvox, ly.cout, self.part_b[i], self.slots_b[i],
                                     self.ss[i], self.mi[i], P[f"{nb}.weight"], ly.act, G[f"{nb}.weight"],
                                     G[f"{nb}.bias"], None if self.dz_dead[i] else self.dz[i], self.ws,
                                     dz16=self.dz16[i])
            else:
                ops.bn_backward(self.dy[i], self.z[i], nvox, ly.cout, self.ss[i], self.mi[i], P[f"{nb}.weight"],
                                ly.act, G[f"{nb}.weight"], G[f"{nb}.bias"], self.dz[i], self.ws)
            xin = self.y[i - 1] if i > 0 else x
            wname = f"{ly.name}.conv.weight"
            # both operands' bf16 shadows, when the layer has them, feed the weight grad
            x16 = self.y16[i - 1] if i > 0 else None
            d16 = self.dz16[i] if BN_FUSED_BWD else None
            if i == 0 and self.dz_dead[0]:  # k7 first conv: only its 16-channel operand has a shadow
                x16 = None
            elif x16 is None or d16 is None:
                x16 = d16 = None
            main = i < self.wgrad_tail_main and self.side is not None
            dl = i if (defer_red and i in k3 and not main) else None
            if ly.kind == "convt":  # ConvTranspose3d: the output-grad is the gathered operand
                fn = (lambda g=self.geo_wgrad[i], a=self.dz[i], b=xin, w=G[wname], a16=d16, b16=x16, m=main, dl=dl:
                      self._wgrad(g, a, b, w, zeroed, main=m, gathered16=a16, aligned16=b16, defer_layer=dl))
            else:
                fn = (lambda g=self.geo_wgrad[i], a=xin, b=self.dz[i], w=G[wname], a16=x16, b16=d16, m=main, dl=dl:
                      self._wgrad(g, a, b, w, zeroed, main=m, gathered16=a16, aligned16=b16, defer_layer=dl))
            if main:
                if pending:
                    flush()
                fn()
                if grads_enqueued is not None:
                    grads_enqueued(i)
                if i == 0:
                    break
                pending_done = True
            else:
                pending.append((i, fn))
                pending_done = False
            # consecutive ResNet-block layers hand their weight grads to the side stream in groups
            # of WGRAD_GROUP: one cross-stream wait per group (an event record costs the main stream
            # ~4 us, tools/launch_micro.hip) at the price of starting a wgrad one layer later
            if not pending_done and (i == 0 or len(pending) >= self.wgrad_group or not resnet_pair(i)):
                flush()
            if i == 0:
                break
            if not self.pre_b[i]:
                self._input_grad(P, G, i)
            if i == self.wgrad_tail_main and side_after is not None and self.side is not None:
                # every gradient of layers >= i must be enqueued (side: weight grads; main: BatchNorm
                # grads) and their weights' last reader, this input-grad, too: the caller's launches
                # for those layers (their update) on the side stream, beside the main stream's tail.
                # A ResNet-chain boundary layer may still hold its weight grad back for grouping:
                # hand it over first, or the update would read a partial gradient.
                if pending:
                    flush()
                self._on_side(side_after)
        if self._deferred_red:  # a deferred weight grad whose partials no reduce was issued for
            raise RuntimeError(f"{len(self._deferred_red)} deferred ResNet weight-grad reduces were never issued")
        if self.side is not None:  # the weight gradients are complete before anything reads them
            ops.stream_wait(torch.cuda.current_stream(self.device), self.side)

    def _reduce_deferred(self):
        """Sum the partials of every deferred ResNet weight grad into dW (one launch, side stream)."""
        items, self._deferred_red = self._deferred_red, []
        for k in range(0, len(items), 16):
            ops.reduce_multi(items[k:k + 16])

    def _input_grad(self, P, G, i: int):
        """dL/dy of layer i - 1 from dz_i (a ResNet block0 also receives the skip gradient
        dL/dh_{r+1}), with layer i - 1's BatchNorm backward statistics."""
        ly = self.layers[i]
        ep = self._bn_grad_epi(i - 1, fused=self.ac_b[i - 1])
        ep.residual = self.dys[i + 1] if ly.name.endswith("block0") else None  # bf16 when layer i + 1 keeps it
        ep.x_bf16 = self.dz16[i] if BN_FUSED_BWD else None  # only the slab backward writes it
        if self.pre_b[i]:  # stages dL/dy_i, maps it to dL/dz_i (and writes dz16[i]) on the way
            ep.x_bf16, ep.pre = self.dys[i], self._pre_bwd(P, G, i)
        ops.conv(self.geo_dgrad[i], self.dz[i], self.wd[i], self.dys[i - 1], ep)


def _running_scale_shift(P, nb, ss):
    """Eval-mode BatchNorm (Trainer.validate, Trainer.py:248-249): scale/shift from the running
    statistics, written into ``ss`` = [scale | shift]."""
    with torch.no_grad():
        inv = torch.rsqrt(P[f"{nb}.running_var"] + 1e-5)
        sc = P[f"{nb}.weight"] * inv
        c = sc.numel()
        ss[:c].copy_(sc)
        ss[c:].copy_(P[f"{nb}.bias"] - P[f"{nb}.running_mean"] * sc)


# ----------------------------------------------------------------------------------------------
@dataclass
class _DLayer:
    name: str
    k: int
    s: int
    p: int
    cin: int
    cout: int
    din: Dims
    dout: Dims


class CriticPlan:
    """Buffers + geometry of PatchGANDiscriminator (model/discriminator.py:9-84) for up to ``nmax``
    samples: the GP conf (Identity norm, gradient_penalty_conf.py:14; conv bias + LeakyReLU in
    the conv epilogue) and the BatchNorm critic of the weight-clip conf (basic_conf.py:60-66;
    middle convs without bias, BatchNorm3d + LeakyReLU).  With BatchNorm every ``forward`` call
    normalises its own batch (the reference calls the critic on the real and on the fake batch
    separately, Trainer.py:119-120); ``bn_pass`` selects the slot that keeps that call's
    statistics for its backward."""

    def __init__(self, cfg, nmax: int, dims: Dims, device, P: Dict[str, torch.Tensor], prec: int = L.PREC_F32):
        self.pl = pl = bool(getattr(cfg, "is_2D", False))  # the 2-D variants: planar geometries, f32
        if pl and prec != L.PREC_F32:
            raise NotImplementedError("the 2-D variants run the exact-f32 path (precision='f32')")
        dims = _planar_dims(dims, pl)
        self.cfg, self.nmax, self.dims, self.device = cfg, nmax, tuple(dims), device
        self.prec = prec
        c0, s = cfg.init_channels_out, cfg.negative_slope
        self.slope = s
        d = tuple(dims)
        ls = []
        dn = _conv_out(d, 4, 2, 1, pl)
        ls.append(_DLayer("model.first.conv", 4, 2, 1, cfg.channels_in, c0, d, dn))
        d = dn
        out_ = c0
        for m in range(cfg.discriminator_depth):
            in_, out_ = min(2**m, 8) * c0, min(2 ** (m + 1), 8) * c0
            dn = _conv_out(d, 4, 2, 1, pl)
            ls.append(_DLayer(f"model.middle.{m}.conv", 4, 2, 1, in_, out_, d, dn))
            d = dn
        dn = _conv_out(d, 4, 1, 1, pl)
        assert min(dn) > 0, f"patch {dims} too small for the critic"
        ls.append(_DLayer("model.last", 4, 1, 1, out_, 1, d, dn))
        self.layers = ls
        self.bn = cfg.norm == "batch"
        # BatchNorm layers: the middle convs of the BN critic (no conv bias, blocks.py:34)
        self.is_bn = [self.bn and ly.name.startswith("model.middle.") for ly in ls]
        # LayerNorm layers: the middle convs of the gp_layernorm conf's critic (no conv bias; per-sample
        # normalisation over (C, D, H, W), no affine parameters: gp_layernorm.py:9-11)
        self.ln = cfg.norm == "layer"
        self.is_ln = [self.ln and ly.name.startswith("model.middle.") for ly in ls]
        self.biased = [not (self.is_bn[i] or self.is_ln[i]) for i in range(len(ls))]
        self.logit_ps = dn[0] * dn[1] * dn[2]
        self.a = [torch.empty((nmax, *ly.dout, ly.cout), device=device) for ly in ls]   # activations (last = logits)
        self.dz = [torch.empty((nmax, *ly.dout, ly.cout), device=device) for ly in ls]  # dL/dz (last = dlogits)
        ws = 0
        for ly in ls:
            g = ops.conv_wgrad_geom(nmax, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p, planar=self.pl)
            nv = nmax * ly.dout[0] * ly.dout[1] * ly.dout[2]
            # (the bf16 weight grads' partial slabs: the geometry at the plan's precision sizes them)
            ws = max(ws, ops.wgrad_ws_floats(g), ops.wgrad_ws_floats(ops.with_prec(g, prec)),
                     ops.channel_sum_ws_floats(nv, ly.cout), ops.bn_backward_ws_floats(nv, ly.cout))
        self.ws = torch.empty(ws, device=device)
        self.ws_clean = torch.zeros(ws, device=device)  # see GeneratorPlan.ws_clean
        # per-layer all-zero workspaces of the weight grads whose unpack is deferred: every layer's
        # result waits in its own workspace and one launch moves them all into dW (_flush_unpack)
        self.defer = True
        self.ws_layer, self._deferred, self._unpack = {}, [], {}
        # All GP-configuration weight / bias gradients on a side stream beside the penalty's
        # forward-mode chain measured 2.7 % slower per step at 64^3 B=4 (the chain's kernels are
        # short and lose CUs to the gradient launches): no such stream (``side`` stays None)
        self.side = None
        self.ws_side = self.ws
        # only the penalty update's bias sums and first-layer weight grad (c1_wgrad, ~36 us at 64^3
        # B=4, needs nothing the forward-mode chain produces) go to a side stream — one hand-off each
        # way, beside the small-grid forward-mode chain
        self.side0 = None
        if torch.device(device).type == "cuda" and not debug("serial"):
            self.side0 = ops.pooled_stream(device, "d_side")
        # (round 6, measured and not kept: the real / fake rows' staged-window weight grads on the
        # generator's idle side stream beside the forward-mode chain, the interpolation rows' after it:
        # 1.281-1.286 vs 1.276-1.277 ms/step — the chain's small-grid kernels lose CUs to it)
        if self.bn:  # conv outputs, pre-activation grads, statistics and per-pass scale/shift
            self.z = [torch.empty_like(self.a[i]) if b else None for i, b in enumerate(self.is_bn)]
            self.dy = [torch.empty_like(self.a[i]) if b else None for i, b in enumerate(self.is_bn)]
            self.stats = [None] * len(ls)  # sized below from the launch geometry (packed / bf16 choice)
            self.ss = [[torch.empty(2 * ly.cout, device=device) for ly in ls] for _ in range(2)]
            self.mi = [[torch.empty(2 * ly.cout, device=device) for ly in ls] for _ in range(2)]
            self.bn_scratch = [torch.empty(2 * ly.cout, device=device) for ly in ls]  # discarded dgamma/dbeta
        if self.ln:
            # conv outputs z, dL/da, and per-sample partial sums (ops.ln_*) of every LayerNorm layer;
            # the penalty's tangent (zdot, adot) and primal-adjoint (abar, zbar) chains over the
            # interpolation rows (at most nmax), and the penalty direction gamma
            vol = [ly.dout[0] * ly.dout[1] * ly.dout[2] * ly.cout for ly in ls]
            self.L = vol
            self.z = [torch.empty_like(self.a[i]) if b else None for i, b in enumerate(self.is_ln)]
            self.dy = [torch.empty_like(self.a[i]) if b else None for i, b in enumerate(self.is_ln)]
            npart = [ops.ln_partial_doubles(nmax, v) for v in vol]
            self.lnp = {k: [torch.empty(npart[i], device=device, dtype=torch.float64) if b else None
                            for i, b in enumerate(self.is_ln)] for k in ("stats", "bwd", "jvp", "sig", "adj")}
            self.zdot = [torch.empty_like(self.a[i]) if b else None for i, b in enumerate(self.is_ln)]
            self.adot = [torch.empty_like(self.a[i]) for i in range(len(ls) - 1)]
            self.abar = [torch.empty_like(self.a[i]) for i in range(len(ls) - 1)]
            self.zbar = [torch.empty_like(self.a[i]) for i in range(len(ls) - 1)]
            self.gam = torch.empty((nmax, *dims, cfg.channels_in), device=device)
        # packed weight copies per (layer, role); the packed layout does not depend on batch/dims
        self.packs = ops.PackSet(device)
        self.wf, self.wd = [], []
        # the last layer (64 -> 1) stays exact fp32 in every role, as the first does: its forward and
        # weight grad are the fp32 VALU cout == 1 kernels, and its input-grad (1 -> 64, the start of
        # every critic backward) takes the fp32 implicit GEMM — rounding the dlogits and its weights
        # to bf16 there would perturb the whole input-gradient chain feeding the generator
        self.prec_d = [L.PREC_F32 if i == len(ls) - 1 else prec for i in range(len(ls))]
        for i, ly in enumerate(ls):
            w = P[f"{ly.name}.weight"]
            gf, wf = self.packs.add(ops.conv_fwd_geom(nmax, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p, planar=self.pl), w, prec)
            gd, wd = self.packs.add(ops.conv_dgrad_geom(nmax, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p, planar=self.pl), w,
                                    self.prec_d[i])
            self.wf.append(wf if gf.w_packed else None)
            self.wd.append(wd if gd.w_packed else None)
        for i, ly in enumerate(ls):
            if self.is_bn[i]:
                gs = self._geo(ops.conv_fwd_geom(nmax, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p, planar=self.pl), self.wf[i])
                self.stats[i] = torch.empty(ops.stats_floats(gs), device=device)
        self.pack()

    def pack(self):
        """Refresh the packed weight copies (one launch); call after every weight update."""
        self.packs.pack()

    def _geo(self, g, packed, prec=None):
        return ops.with_packing(g, self.prec if prec is None else prec) if packed is not None else g

    def _sl(self, t, off, n):
        return t[off:off + n]

    def forward(self, P, x, off: int, n: int, bn_pass: int = 0, training: bool = True):
        """a_l[off:off+n] = critic activations of x (n samples); logits in a[-1].  BatchNorm
        layers normalise over these n samples (training: batch statistics, running buffers
        updated; eval: running statistics) and keep scale/shift in slot ``bn_pass``."""
        h = x
        for i, ly in enumerate(self.layers):
            g = self._geo(ops.conv_fwd_geom(n, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p, planar=self.pl), self.wf[i])
            w = self.wf[i] if self.wf[i] is not None else P[f"{ly.name}.weight"]
            out = self._sl(self.a[i], off, n)
            if self.is_bn[i]:
                nb = ly.name[:-len(".conv")] + ".normalization"
                z = self._sl(self.z[i], off, n)
                ss, mi = self.ss[bn_pass][i], self.mi[bn_pass][i]
                if training:
                    ops.conv(g, h, w, z, ops.epilogue(stats=self.stats[i]))
                    ops.bn_finalize(self.stats[i], ops.stats_floats(g) // (2 * ly.cout + 1), ly.cout, P[f"{nb}.weight"],
                                    P[f"{nb}.bias"], P[f"{nb}.running_mean"], P[f"{nb}.running_var"],
                                    P[f"{nb}.num_batches_tracked"], ss, mi)
                else:
                    ops.conv(g, h, w, z)
                    _running_scale_shift(P, nb, ss)
                nvox = n * ly.dout[0] * ly.dout[1] * ly.dout[2]
                ops.bn_apply(z, nvox, ly.cout, ss, L.ACT_LRELU, out, slope=self.slope)
            elif self.is_ln[i]:
                z = self._sl(self.z[i], off, n)
                ops.conv(g, h, w, z)
                ps = self._lp("stats", i, off)
                ops.ln_reduce(L.LN_STATS, n, self.L[i], self.slope, ps, z=z, p_stats=ps)
                ops.ln_apply(L.LN_STATS, n, self.L[i], self.slope, out, z=z, p_stats=ps)
            else:
                last = i == len(self.layers) - 1
                ep = ops.epilogue(bias=P[f"{ly.name}.bias"], act=L.ACT_NONE if last else L.ACT_LRELU,
                                  slope=self.slope)
                ops.conv(g, h, w, out, ep)
            h = out
        return self._sl(self.a[-1], off, n)

    def _lp(self, kind: str, i: int, off: int):
        """LayerNorm layer i's partial sums of ``kind`` from sample ``off`` on."""
        t = self.lnp[kind][i]
        k = t.numel() // self.nmax
        return t[off * k:]

    def input_grad(self, P, off: int, n: int, dx_out: torch.Tensor, dx_off: int, dx_n: int, bn_pass: int = 0,
                   G=None, bn_accumulate: bool = False, ep0=None):
        """dz chain from dz[-1][off:off+n] (dlogits) down to dz[0]; then dD/dx for samples
        [dx_off, dx_off+dx_n) (absolute indices inside the batch) into dx_out.  BatchNorm layers
        back-propagate with the statistics of ``bn_pass``; their gamma/beta gradients go to ``G``
        (added when ``bn_accumulate``) or are discarded when ``G`` is None."""
        for i in range(len(self.layers) - 1, 0, -1):
            ly = self.layers[i]
            g = self._geo(ops.conv_dgrad_geom(n, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p, planar=self.pl), self.wd[i],
                          self.prec_d[i])
            w = self.wd[i] if self.wd[i] is not None else P[f"{ly.name}.weight"]
            if self.is_bn[i - 1]:  # dL/da -> BatchNorm + LeakyReLU backward -> dL/dz
                lp = self.layers[i - 1]
                nb = lp.name[:-len(".conv")] + ".normalization"
                dy = self._sl(self.dy[i - 1], off, n)
                ops.conv(g, self._sl(self.dz[i], off, n), w, dy)
                nvox = n * lp.dout[0] * lp.dout[1] * lp.dout[2]
                dg, db = ((G[f"{nb}.weight"], G[f"{nb}.bias"]) if G is not None else
                          (self.bn_scratch[i - 1][:lp.cout], self.bn_scratch[i - 1][lp.cout:]))
                ops.bn_backward(dy, self._sl(self.z[i - 1], off, n), nvox, lp.cout, self.ss[bn_pass][i - 1],
                                self.mi[bn_pass][i - 1], P[f"{nb}.weight"], L.ACT_LRELU, dg, db,
                                self._sl(self.dz[i - 1], off, n), self.ws, slope=self.slope,
                                accumulate=bn_accumulate and G is not None)
            elif self.is_ln[i - 1]:  # dL/da -> LayerNorm + LeakyReLU backward -> dL/dz
                da, z = self._sl(self.dy[i - 1], off, n), self._sl(self.z[i - 1], off, n)
                ops.conv(g, self._sl(self.dz[i], off, n), w, da)
                ps, pb = self._lp("stats", i - 1, off), self._lp("bwd", i - 1, off)
                Li = self.L[i - 1]
                ops.ln_reduce(L.LN_BWD, n, Li, self.slope, pb, z=z, da=da, p_stats=ps)
                ops.ln_apply(L.LN_BWD, n, Li, self.slope, self._sl(self.dz[i - 1], off, n), z=z, da=da, p_stats=ps,
                             p_bwd=pb)
            else:
                ops.conv(g, self._sl(self.dz[i], off, n), w, self._sl(self.dz[i - 1], off, n),
                         ops.epilogue(mask_src=self._sl(self.a[i - 1], off, n), slope=self.slope))
        ly = self.layers[0]
        if dx_n > 0:
            g = self._geo(ops.conv_dgrad_geom(dx_n, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p, planar=self.pl), self.wd[0])
            w = self.wd[0] if self.wd[0] is not None else P[f"{ly.name}.weight"]
            ops.conv(g, self._sl(self.dz[0], dx_off, dx_n), w, dx_out, ep0)

    def gp_forward_mode(self, P, gamma: torch.Tensor, off: int, n: int):
        """nu_l = mask_l * conv_l(nu_{l-1}) (no bias), nu_0 = gamma, written in place over
        a_l[off:off+n] (after the masks there have been consumed)."""
        h = gamma
        for i, ly in enumerate(self.layers[:-1]):
            g = self._geo(ops.conv_fwd_geom(n, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p, planar=self.pl), self.wf[i])
            out = self._sl(self.a[i], off, n)
            w = self.wf[i] if self.wf[i] is not None else P[f"{ly.name}.weight"]
            ops.conv(g, h, w, out, ops.epilogue(mask_src=out, slope=self.slope))
            h = out

    def _on_side(self, fn):
        """Enqueue ``fn``'s launches on the side stream after everything enqueued so far."""
        if self.side is None:
            return fn()
        ops.stream_wait(self.side, torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.side):
            fn()

    def join_side(self):
        if self.side is not None:
            ops.stream_wait(torch.cuda.current_stream(self.device), self.side)
        if self.side0 is not None:
            ops.stream_wait(torch.cuda.current_stream(self.device), self.side0)

    def _wgrad(self, g, a, b, dw, ws, zeroed: bool, layer: Optional[int] = None):
        """``layer``: defer the unpack of an atomic-workspace weight grad into the layer's own clean
        workspace (moved into dW by ``_flush_unpack``, on the same stream, before anything reads it)."""
        if zeroed and ops.wgrad_ws_atomic(g):
            if layer is not None and self.defer:
                wl = self.ws_layer.get(layer)
                if wl is None:
                    wl = self.ws_layer[layer] = torch.zeros(ops.wgrad_ws_floats(g), device=self.ws.device)
                ops.wgrad(g, a, b, dw, wl, accumulate=True, ws_clean=True, defer_unpack=True)
                self._deferred.append((layer, g, wl, dw))
                return None
            return ops.wgrad(g, a, b, dw, self.ws_clean, accumulate=True, ws_clean=True)
        return ops.wgrad(g, a, b, dw, ws, accumulate=zeroed)

    def _wgrad_geo(self, j: int, n_all: int):
        ly = self.layers[j]
        return ops.with_prec(ops.conv_wgrad_geom(n_all, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p,
                                                 planar=self.pl), self.prec)

    def _groupable(self, j: int, n_all: int, zeroed: bool) -> bool:
        """Layer j's weight grad can join one grouped launch (ops.wgrad_group): the deferred-unpack
        path into its own clean workspace, a geometry the generic bf16 kernel takes."""
        if not (zeroed and self.defer):
            return False
        g = self._wgrad_geo(j, n_all)
        return ops.wgrad_ws_atomic(g) and ops.wgrad_group_ok(g)

    def _wgrad_group(self, G, layers, n_all: int):
        """The weight grads of ``layers`` (operands a_{j-1}, dz_j over n_all samples) in one launch:
        independent small grids run side by side instead of one after another; each result waits in
        its layer's clean workspace for the unpack launch (_flush_unpack)."""
        items = []
        for j in layers:
            g = self._wgrad_geo(j, n_all)
            wl = self.ws_layer.get(j)
            if wl is None:
                wl = self.ws_layer[j] = torch.zeros(ops.wgrad_ws_floats(g), device=self.ws.device)
            items.append((g, self.a[j - 1][:n_all], self.dz[j][:n_all], wl))
            self._deferred.append((j, g, wl, G[f"{self.layers[j].name}.weight"]))
        ops.wgrad_group(items)

    def _wgrad_sk(self, G, layers, n_all: int, r0: int = 0):
        """The weight grads of ``layers`` (a_{j-1}, dz_j over samples r0 .. r0 + n_all) on the staged-window
        kernel, added into the zeroed gradient arena (two launches: partial tiles, then their sums)."""
        items = []
        for j in layers:
            g = self._wgrad_geo(j, n_all)
            key = ("sk_ws", j, n_all, r0)
            wsj = self.__dict__.setdefault("_sk_ws", {}).get(key)
            if wsj is None:
                wsj = self._sk_ws[key] = torch.empty(ops.wgrad_sk_ws_floats(g), device=self.ws.device)
            items.append((g, self.a[j - 1][r0:r0 + n_all], self.dz[j][r0:r0 + n_all], wsj,
                          G[f"{self.layers[j].name}.weight"]))
        ops.wgrad_sk(items)

    def _flush_unpack(self):
        """One launch moving every deferred weight grad into dW (workspaces left zeroed)."""
        if not self._deferred:
            return
        key = tuple((layer, dw.data_ptr()) for layer, _, _, dw in self._deferred)
        us = self._unpack.get(key)
        if us is None:
            us = self._unpack[key] = ops.UnpackSet(self.ws.device, [(g, wl, dw, True) for _, g, wl, dw in self._deferred])
        self._deferred = []
        us.run()

    def gp_grads_overlapped(self, P, G, x_all: torch.Tensor, gamma: torch.Tensor, off: int, n: int, n_all: int,
                            n_bias: int, zeroed: bool = False):
        """``gp_forward_mode`` + ``weight_grads`` with the gradient launches on the side stream:
        the bias sums as soon as the input-grad chain is done, dW_l as soon as nu_{l-1} (the
        forward-mode output it gathers) is written; the forward-mode chain stays on the main
        stream.  Call ``join_side`` before anything reads the gradients or reuses a / dz."""
        ws = self.ws_side

        def wgrad(i, prev):
            ly = self.layers[i]
            g = ops.with_prec(ops.conv_wgrad_geom(n_all, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p, planar=self.pl), self.prec)
            self._wgrad(g, prev, self.dz[i][:n_all], G[f"{ly.name}.weight"], ws, zeroed, layer=i)
        if self.side0 is not None:  # bias sums + the first layer's weight grad beside the chain below
            ops.stream_wait(self.side0, torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.side0):
                self._bias_sums(G, n_bias, side=True).run()
                # x_all's interpolation rows hold gamma = nu_0; its own all-zero workspace, unpacked
                # on this stream (nothing of it is deferred to the main stream's unpack launch)
                ly = self.layers[0]
                g = ops.with_prec(ops.conv_wgrad_geom(n_all, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p,
                                                      planar=self.pl), self.prec)
                if getattr(self, "ws_side0", None) is None:
                    self.ws_side0 = torch.zeros(ops.wgrad_ws_floats(g), device=self.ws.device)
                atomic = zeroed and ops.wgrad_ws_atomic(g)
                ops.wgrad(g, x_all, self.dz[0][:n_all], G[f"{ly.name}.weight"], self.ws_side0, accumulate=zeroed,
                          ws_clean=atomic)
        else:
            self._on_side(lambda: self._bias_sums(G, n_bias, side=True).run())
            self._on_side(lambda: wgrad(0, x_all))
        h = gamma
        group = []  # layers whose weight grads run together in one launch after the chain (_wgrad_group)
        skl = []    # ... on the staged-window critic kernel (ops.wgrad_sk, round 5)
        for i, ly in enumerate(self.layers[:-1]):
            g = self._geo(ops.conv_fwd_geom(n, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p, planar=self.pl), self.wf[i])
            out = self._sl(self.a[i], off, n)
            w = self.wf[i] if self.wf[i] is not None else P[f"{ly.name}.weight"]
            ops.conv(g, h, w, out, ops.epilogue(mask_src=out, slope=self.slope))
            h = out
            if self.side is None and zeroed and ops.wgrad_sk_ok(self._wgrad_geo(i + 1, n_all)) and not debug("no_wgrad_sk"):
                skl.append(i + 1)
            elif self.side is None and self._groupable(i + 1, n_all, zeroed):
                group.append(i + 1)
            else:
                self._on_side(lambda i=i: wgrad(i + 1, self.a[i][:n_all]))  # a_i now holds nu_i in its interp rows
        for k in range(0, len(skl), 4):
            self._wgrad_sk(G, skl[k:k + 4], n_all)
        for k in range(0, len(group), 4):  # a grouped launch takes at most 4 (discriminator_depth >= 5)
            self._wgrad_group(G, group[k:k + 4], n_all)
        self._on_side(self._flush_unpack)

    def _bias_sums(self, G, n_bias: int, side: bool = False) -> "ops.ChannelSumSet":
        """db_l = sum of dz_l over the first n_bias samples, every biased layer in two launches
        (built once per (n_bias, stream role); the gradient views and dz buffers keep their addresses)."""
        key = (n_bias, side, id(G))
        cache = self.__dict__.setdefault("_csum", {})
        if key not in cache:
            items = [(self.dz[i], n_bias * ly.dout[0] * ly.dout[1] * ly.dout[2], ly.cout, G[f"{ly.name}.bias"], False)
                     for i, ly in enumerate(self.layers) if self.biased[i]]
            cache[key] = ops.ChannelSumSet(self.device, items)
        return cache[key]

    def weight_grads(self, P, G, x_all: torch.Tensor, n_all: int, n_bias: int, zeroed: bool = False):
        """dW_l = wgrad(a_{l-1}, dz_l) over n_all samples; db_l = sum dz_l over the first n_bias."""
        prev = x_all
        for i, ly in enumerate(self.layers):
            g = ops.with_prec(ops.conv_wgrad_geom(n_all, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p, planar=self.pl), self.prec)
            self._wgrad(g, prev, self.dz[i][:n_all], G[f"{ly.name}.weight"], self.ws, zeroed, layer=i)
            prev = self.a[i][:n_all]
        self._flush_unpack()
        self._bias_sums(G, n_bias).run()

    def gp_grads_ln(self, P, G, x_all: torch.Tensor, gamma: torch.Tensor, off: int, n: int):
        """Critic gradients of the LayerNorm critic with the gradient penalty (gp_layernorm conf),
        into a zeroed arena G.  Rows [0, off) are the real / fake samples of the Wasserstein loss,
        rows [off, off + n) the interpolation, whose dz chain (input_grad) carries dSum(D)/dx;
        ``gamma`` = dGP/dg.  The penalty's parameter gradient is d/dtheta of the directional
        derivative s = <dD/dx, gamma> (model/utils.py:34-41 differentiated): a tangent forward
        along gamma (LayerNorm linearised at the interpolation's statistics), whose adjoint is the
        existing dz chain, plus the primal adjoint the LayerNorm tangent injects at every middle
        layer (ln.hip header), propagated down through the primal convs.  Weight gradients:
        wgrad(a_{l-1}, dz_l) over real/fake + wgrad(adot_{l-1}, dz_l) + wgrad(a_{l-1}, zbar_l) over
        the interpolation; the first bias also receives sum zbar_0."""
        nl = len(self.layers)
        sl = self.slope
        sl_ = lambda t: t[off:off + n]  # noqa: E731
        geo = lambda i, m, role: self._geo(getattr(ops, role)(m, self.layers[i].din, self.layers[i].dout,  # noqa: E731
                                                               self.layers[i].cin, self.layers[i].cout, 4,
                                                               self.layers[i].s, 1),
                                           self.wf[i] if role == "conv_fwd_geom" else self.wd[i])
        wt = lambda i, role: ((self.wf[i] if role == "fwd" else self.wd[i]) if (  # noqa: E731
            self.wf[i] if role == "fwd" else self.wd[i]) is not None else P[f"{self.layers[i].name}.weight"])
        # 1. tangent forward along gamma
        for i in range(nl - 1):
            src = gamma if i == 0 else self.adot[i - 1][:n]
            if self.is_ln[i]:
                zd, z, da = self.zdot[i][:n], sl_(self.z[i]), sl_(self.dy[i])
                ops.conv(geo(i, n, "conv_fwd_geom"), src, wt(i, "fwd"), zd)
                ps, pj, pg = self._lp("stats", i, off), self._lp("jvp", i, 0), self._lp("sig", i, 0)
                ops.ln_reduce(L.LN_JVP, n, self.L[i], sl, pj, z=z, zdot=zd, p_stats=ps)
                ops.ln_apply(L.LN_JVP, n, self.L[i], sl, self.adot[i][:n], z=z, zdot=zd, p_stats=ps, p_jvp=pj)
                ops.ln_reduce(L.LN_SIG, n, self.L[i], sl, pg, z=z, da=da, adot=self.adot[i][:n], p_stats=ps)
            else:
                ops.conv(geo(i, n, "conv_fwd_geom"), src, wt(i, "fwd"), self.adot[i][:n],
                         ops.epilogue(mask_src=sl_(self.a[i]), slope=sl))
        # 2. primal adjoint, top LayerNorm layer down (nothing reaches the top one from above)
        for i in range(nl - 2, -1, -1):
            if i < nl - 2:
                ab = self.abar[i][:n] if self.is_ln[i] else self.zbar[i][:n]
                ep = None if self.is_ln[i] else ops.epilogue(mask_src=sl_(self.a[i]), slope=sl)
                ops.conv(geo(i + 1, n, "conv_dgrad_geom"), self.zbar[i + 1][:n], wt(i + 1, "dgrad"), ab, ep)
            else:
                ab = None
            if self.is_ln[i]:
                z, da, zd = sl_(self.z[i]), sl_(self.dy[i]), self.zdot[i][:n]
                ps, pb = self._lp("stats", i, off), self._lp("bwd", i, off)
                pj, pg, pa = self._lp("jvp", i, 0), self._lp("sig", i, 0), self._lp("adj", i, 0)
                kw = dict(z=z, da=da, zdot=zd, abar=ab, p_stats=ps, p_bwd=pb, p_jvp=pj)
                ops.ln_reduce(L.LN_ADJ, n, self.L[i], sl, pa, **kw)
                ops.ln_apply(L.LN_ADJ, n, self.L[i], sl, self.zbar[i][:n], p_sig=pg, p_adj=pa, **kw)
            elif ab is None:
                raise NotImplementedError("LayerNorm critic: the layer below the last conv must be a LayerNorm block")
        # 3. weight gradients (accumulated) and biases
        for i, ly in enumerate(self.layers):
            wg = lambda m: ops.with_prec(ops.conv_wgrad_geom(m, ly.din, ly.dout, ly.cin, ly.cout, ly.k, ly.s, ly.p, planar=self.pl),  # noqa
                                         self.prec)
            dw = G[f"{ly.name}.weight"]
            prev = x_all if i == 0 else self.a[i - 1]
            self._wgrad(wg(off), prev[:off], self.dz[i][:off], dw, self.ws, True)
            self._wgrad(wg(n), gamma if i == 0 else self.adot[i - 1][:n], sl_(self.dz[i]), dw, self.ws, True)
            if i < nl - 1:
                self._wgrad(wg(n), sl_(prev), self.zbar[i][:n], dw, self.ws, True)
        self._bias_sums(G, off).run()
        key = ("zbar0", n, id(G))
        cache = self.__dict__.setdefault("_csum", {})
        if key not in cache:
            ly = self.layers[0]
            cache[key] = ops.ChannelSumSet(self.device, [(self.zbar[0], n * ly.dout[0] * ly.dout[1] * ly.dout[2],
                                                          ly.cout, G[f"{ly.name}.bias"], True)])
        cache[key].run()


# ----------------------------------------------------------------------------------------------
class StepEngine:
    """One fused G+D train step for fixed (b_opt, b_sub, patch dims) on one GPU."""

    def __init__(self, generator, critic, g_cfg, d_cfg, b_opt: int, b_sub: int, dims: Dims, *,
                 g_hyper: Sequence[float] = (1e-4, 0.0, 0.9, 1e-8), d_hyper: Sequence[float] = (1e-4, 0.0, 0.9, 1e-8),
                 gp_weight: float = 10.0, hu_bounds=(112.0 / 600.0, 212.0 / 600.0), gan_w=1.0, sim_w=1.0, hu_w=1.0,
                 device=None, g_optim=None, d_optim=None, process_group=None, precision: str = "f32",
                 weight_clip: Optional[float] = None):
        if d_cfg.norm not in ("identity", "batch", "layer"):
            raise NotImplementedError(f"StepEngine: critic norm {d_cfg.norm!r}")
        # gradient penalty unless weight clipping (Trainer.py:122-131): the GP conf (Identity-norm
        # critic), the gp_layernorm conf (LayerNorm critic, gp_layernorm.py:9-11) or the weight-clip
        # conf (BatchNorm critic, basic_conf.py:37,60-66)
        self.use_gp = weight_clip is None
        if self.use_gp and d_cfg.norm == "batch":
            raise NotImplementedError("gradient penalty through a BatchNorm critic needs BatchNorm double backward "
                                      "(no reference configuration uses it: SURVEY.md §8f row 4)")
        device = device or torch.device("cuda", torch.cuda.current_device())
        self.device = device
        # the 2-D variants (experiments/conf_2D.py): patches [N, 1, H, W] as planar (1, H, W) grids
        self.planar = bool(getattr(g_cfg, "is_2D", False))
        if self.planar != bool(getattr(d_cfg, "is_2D", False)):
            raise ValueError("StepEngine: generator and critic must both be 2-D or both 3-D")
        dims = _planar_dims(dims, self.planar)
        self.dims = tuple(dims)
        self.b_opt, self.b_sub, self.b_gp = b_opt, b_sub, min(b_opt, b_sub)
        self.vox = dims[0] * dims[1] * dims[2]
        self.gp_weight, self.gan_w, self.sim_w, self.hu_w = gp_weight, gan_w, sim_w, hu_w
        self.lo, self.hi = hu_bounds
        nmax = b_opt + b_sub + self.b_gp
        if precision not in ("f32", "bf16"):
            raise ValueError(f"precision must be 'f32' or 'bf16', got {precision!r}")
        self.precision = precision
        prec = L.PREC_BF16 if precision == "bf16" else L.PREC_F32
        from .trainer.optim import FusedAdam
        if g_optim is None:
            lr, b1, b2, eps = g_hyper
            g_optim = FusedAdam(Arena(generator, device), lr, (b1, b2), eps)
        if d_optim is None:
            lr, b1, b2, eps = d_hyper
            d_optim = FusedAdam(Arena(critic, device), lr, (b1, b2), eps, weight_clip=weight_clip)
        self.g_optim, self.d_optim = g_optim, d_optim
        # patch-level data parallelism: one gradient all-reduce per update
        self.pg = process_group
        self.world = 1
        if process_group is not None or (torch.distributed.is_available() and torch.distributed.is_initialized()):
            self.world = torch.distributed.get_world_size(process_group)
        # data-parallel collectives on; CGAN3D_FORCE_DP=1 also at world size 1 (exercises the RCCL
        # path, buckets and streams on a single GPU: tools/dist_nccl1_check.py)
        self.dp = self.world > 1 or (os.environ.get("CGAN3D_FORCE_DP") == "1" and torch.distributed.is_initialized())
        self.g_arena, self.d_arena = g_optim.arena, d_optim.arena
        self.gP = dict(self.g_arena.views)
        self.gP.update({k: v for k, v in generator.state_dict(keep_vars=True).items() if k not in self.gP})
        self.dP = dict(self.d_arena.views)
        self.dP.update({k: v for k, v in critic.state_dict(keep_vars=True).items() if k not in self.dP})
        self.gG, self.dG = self.g_arena.gviews, self.d_arena.gviews
        # plans after the arenas: their packed-weight descriptors point at the arena storage
        self.G = GeneratorPlan(g_cfg, b_sub, dims, device, self.gP, prec)
        # critic rows [0, nmax): the critic update's batch; [nmax, nmax + b_sub): the generator
        # update's pass over opt_hat (own rows, so both dlogits can be constant buffers, below)
        self.D = CriticPlan(d_cfg, nmax + b_sub, dims, device, self.dP, prec)
        # critic input slots [real | fake(opt_hat) | interpolation -> gamma]
        self.xc = torch.empty((nmax, *dims, 1), device=device)
        self.subopt = torch.empty((b_sub, *dims, 1), device=device)
        self.mask = torch.empty((b_sub, *dims, 1), device=device, dtype=torch.uint8)
        self.eps = torch.empty(self.b_gp, device=device)
        # |real| != |fake| (model/utils.py:21-25): the penalty interpolates min(|real|, |fake|) rows drawn
        # with replacement from each batch (set_gp_indices / draw_gp_indices, before each step; the
        # interpolation kernel reads them from this device buffer, so recorded plans follow them)
        self.gp_idx = None
        if b_opt != b_sub and weight_clip is None:
            self.gp_idx = torch.cat([torch.arange(self.b_gp), torch.arange(self.b_gp)]).to(torch.int32).to(device)
        self.gbuf = torch.empty((self.b_gp, *dims, 1), device=device)    # g = dD/dx at the interpolation
        self.dcrit = torch.empty((b_sub, *dims, 1), device=device)       # dL_G/d opt_hat via the critic
        self.losses = torch.zeros(8, device=device)
        self.loss_ws = torch.empty(ops.loss_ws_floats(), device=device)
        # The generator's similarity / HU losses and their gradient depend only on its forward, so
        # they run on the generator's side stream beside the critic update (with the zeroing of the
        # generator's gradient arena); the critic's first-layer input-grad of the generator update
        # then folds its adversarial gradient through the output tanh into G.dz_last in place
        # (L.ACT_NEG_DTANH; measured 1.646 against 1.664 ms/step with everything after that input-grad).
        g0 = self.D.layers[0]
        self.gloss_side = (self.G.side is not None and
                           ops.neg_dtanh_ok(self.D._geo(ops.conv_dgrad_geom(b_sub, g0.din, g0.dout, g0.cin, g0.cout, g0.k,
                                                                             g0.s, g0.p, planar=self.D.pl),
                                                        self.D.wd[0])))
        self.loss_ws_g = torch.empty(ops.loss_ws_floats(), device=device) if self.gloss_side else self.loss_ws
        # the gradient penalty's per-sample sums of squares straight from the critic's first-layer
        # input-grad (one float per block; a separate reduction pass measured 1.630 against 1.622 ms/step)
        nsq = ops.sumsq_blocks(self.D._geo(ops.conv_dgrad_geom(self.b_gp, g0.din, g0.dout, g0.cin, g0.cout, g0.k, g0.s,
                                                               g0.p, planar=self.D.pl), self.D.wd[0]))
        # The generator's Adam in two parts: every layer whose gradients are complete when the
        # backward's side stream finishes its last weight grad (all but the first WGRAD_TAIL_MAIN
        # layers) is updated and repacked on the side stream beside the main stream's tail; the
        # tail layers' parameters (a prefix of the arena) after it, with the step tick.  Single
        # GPU only (data parallelism all-reduces the whole gradient first).
        self.g_split = 0
        if self.G.side is not None and not self.dp:
            pre = tuple(self.G.layers[li].name + "." for li in range(min(self.G.wgrad_tail_main, len(self.G.layers))))
            ar, off, lo, ok = self.g_arena, 0, None, True
            for nm, pp in zip(ar.names, ar.params):
                tail = nm.startswith(pre) if pre else False
                if tail and lo is not None:
                    ok = False  # a tail parameter after an early one: not a prefix
                if not tail and lo is None:
                    lo = off
                off += pp.numel()
            if ok and lo and lo < ar.numel:
                self.g_split = lo
        self.gp_part = (torch.empty(nsq, device=device) if nsq and self.b_gp and self.use_gp and not self.D.ln
                        else None)
        # dL/dlogits of both critic passes are constants (Trainer.py:117-131, 150-152): written once here
        # into their rows of D.dz[-1]; the losses come from the GP pass (critic) and from a launch
        # beside the generator's backward (generator), so no logits launch sits on the step's path
        self.fold_logits = self.gp_part is not None and self.gloss_side
        self.g_off = nmax if self.fold_logits else 0  # critic rows of the generator update
        if self.fold_logits:
            self._write_dlogits()
        self._pending = []  # in-flight bucket all-reduces of the generator gradients
        self.comm_log = None  # a list: the collective sequence is logged there (_log_comm)
        self.g_buckets = self._make_g_buckets(G_BUCKET_BYTES) if (self.dp and G_BUCKET_BYTES > 0) else []
        on_gpu = torch.device(device).type == "cuda"
        self.comm = ops.pooled_stream(device, "comm") if (self.dp and on_gpu) else None
        if self.comm is not None and int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
            import warnings
            warnings.warn("StepEngine: data parallelism with fewer than 8 hardware queues (GPU_MAX_HW_QUEUES): the "
                          "communication stream shares an in-order queue (measured +16 % step time at 4); call "
                          "cgan3d_amd.configure_hw_queues() before the first GPU use", RuntimeWarning, stacklevel=2)
        # RCCL from C++ (ops.NativeComm): with the nccl backend the all-reduces are C-ABI launches,
        # recorded into the step's launch plan like kernels — one plan per step, no host callables
        # (CGAN3D_COMM=torch: torch.distributed's collectives as host callables, the fallback)
        self.native = None
        if (self.dp and on_gpu and torch.distributed.get_backend(process_group) == "nccl"
                and ops.COMM_MODE != "torch"):
            self.native = ops.NativeComm(process_group, device)
        if self.world > 1:
            self.broadcast_state()

    def _make_g_buckets(self, bucket_bytes: int):
        """Generator gradient buckets for data parallelism: the backward produces parameter
        gradients from the last layer to the first, i.e. from the end of the flat arena (forward
        order) toward its start, so a bucket is a contiguous arena slice closed at a layer boundary
        once it holds >= ``bucket_bytes``; the first three layers (the last gradients produced, on
        the critical path to Adam) form their own small final bucket.  Returns
        [(layer stage that closes the bucket, lo, hi)] in backward order."""
        ar = self.g_arena
        span, off = {}, 0
        for n, p in zip(ar.names, ar.params):
            span[n] = (off, off + p.numel())
            off += p.numel()
        nl = len(self.G.layers)
        stages = [(nl, [k for k in span if k.startswith("model.last_conv.")])]
        for i in range(nl - 1, -1, -1):
            stages.append((i, [k for k in span if k.startswith(self.G.layers[i].name + ".")]))
        buckets, hi, acc = [], ar.numel, 0
        for stage, names in stages:
            lo = min(span[k][0] for k in names)
            assert max(span[k][1] for k in names) == hi - acc, "generator arena is not in layer order"
            acc = hi - lo
            if stage == 3 or (acc * 4 >= bucket_bytes and stage > 3) or stage == 0:
                buckets.append((stage, lo, hi))
                hi, acc = lo, 0
        assert hi == 0 and acc == 0
        return buckets

    def _cur_stream(self):
        """The current torch stream (None on a CPU dry run)."""
        return torch.cuda.current_stream(self.device) if torch.device(self.device).type == "cuda" else None

    def _arena_span(self, grad: torch.Tensor):
        """(network, first, last + 1) of ``grad``'s elements inside its gradient arena."""
        for net, ar in (("G", self.g_arena), ("D", self.d_arena)):
            lo = (grad.data_ptr() - ar.grad.data_ptr()) // 4
            if 0 <= lo and lo + grad.numel() <= ar.numel:
                return net, lo, lo + grad.numel()
        return "?", 0, grad.numel()

    def _log_comm(self, *event):
        """Collective-sequence log (tests/test_dist.py): ("allreduce", stream, net, lo, hi) and
        ("wait", waiter, signaler) in issue order, when ``comm_log`` is a list.  Every rank must issue
        the same collectives in the same order on the shared communicator, and each collective must
        be ordered after the previous one by a stream dependency."""
        if self.comm_log is not None:
            self.comm_log.append(event)

    def _bucket_ready(self, stage: int):
        """GeneratorPlan.backward callback: start the all-reduce of a bucket whose gradients are all
        enqueued (a host callable inside a recorded plan: ops.plan_host)."""
        for st, lo, hi in self.g_buckets:
            if st == stage:
                if self.native is not None:  # recorded into the plan as it is
                    self._start_allreduce(self.g_arena.grad[lo:hi])
                else:
                    ops.plan_host(lambda lo=lo, hi=hi: self._start_allreduce(self.g_arena.grad[lo:hi]))

    def _start_allreduce(self, grad: torch.Tensor):
        """Mean over ranks of ``grad``, started now and overlapped with whatever is enqueued next:
        RCCL on a communication stream ordered after the main and side streams' work so far (both
        produce gradients); ``_finish_allreduce`` makes the main stream wait before Adam.  gloo
        (CPU tensors): synchronous."""
        dist = torch.distributed
        if self.native is not None:
            ops.stream_wait(self.comm, self._cur_stream())
            self._log_comm("wait", "comm", "main")
            if self.G.side is not None:
                ops.stream_wait(self.comm, self.G.side)
                self._log_comm("wait", "comm", "side")
            with torch.cuda.stream(self.comm):  # (None on a CPU dry run: no-op context)
                self._log_comm("allreduce", "comm", *self._arena_span(grad))
                self.native.allreduce_mean(grad)
            self._pending.append(None)
            return
        self._log_comm("allreduce", "sync", *self._arena_span(grad))
        if dist.get_backend(self.pg) != "nccl":
            if self.G.side is not None:  # gloo over GPU tensors orders only after the current stream
                torch.cuda.current_stream(self.device).wait_stream(self.G.side)
            dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=self.pg)
            grad.mul_(1.0 / self.world)
            return
        cur = torch.cuda.current_stream(self.device)
        self.comm.wait_stream(cur)
        if self.G.side is not None:
            self.comm.wait_stream(self.G.side)
        with torch.cuda.stream(self.comm):
            self._pending.append(dist.all_reduce(grad, op=dist.ReduceOp.AVG, group=self.pg, async_op=True))

    def _finish_allreduce(self):
        if self.native is not None:  # the main stream waits for the communication stream
            ops.stream_wait(self._cur_stream(), self.comm)
            self._log_comm("wait", "main", "comm")
            self._pending.clear()
            return

        def wait():
            for w in self._pending:
                w.wait()  # the current stream waits for the collective
            self._pending.clear()
        ops.plan_host(wait)

    def broadcast_state(self, src: int = 0):
        """Start every rank from rank ``src``'s weights, BatchNorm buffers and Adam moments (what
        DistributedDataParallel does at construction); the packed weight copies are refreshed."""
        dist = torch.distributed
        for ar in (self.g_arena, self.d_arena):
            for t in (ar.flat, ar.exp_avg, ar.exp_avg_sq):
                dist.broadcast(t, src, group=self.pg)
        for P in (self.gP, self.dP):
            for k, v in P.items():
                if k.endswith(("running_mean", "running_var", "num_batches_tracked")):
                    dist.broadcast(v.data, src, group=self.pg)
        self.G.pack()
        self.D.pack()

    def sync_bn_buffers(self, src: int = 0):
        """BatchNorm running statistics of rank ``src`` on every rank (one coalesced broadcast).

        Policy under data parallelism: every rank normalises with its own batch statistics and
        updates its own running buffers (as DistributedDataParallel does between its per-forward
        buffer broadcasts); rank ``src``'s buffers evolve exactly as DDP's rank 0 buffers do, since
        they only ever see that rank's batches.  The running buffers are read only by eval-mode
        forwards (Trainer.validate) and checkpoints (written by rank 0), so the Trainer calls this
        before both instead of broadcasting every step."""
        if self.world == 1:
            return
        bufs = [v for P in (self.gP, self.dP) for k, v in P.items() if k.endswith(("running_mean", "running_var"))]
        if not bufs:
            return
        flat = torch.cat([b.detach().reshape(-1) for b in bufs])
        torch.distributed.broadcast(flat, src, group=self.pg)
        off = 0
        with torch.no_grad():
            for b in bufs:
                b.copy_(flat[off:off + b.numel()].view_as(b))
                off += b.numel()

    @property
    def opt_hat(self):
        return self.xc[self.b_opt:self.b_opt + self.b_sub]

    def load_inputs(self, opt: torch.Tensor, subopt: torch.Tensor, mask: torch.Tensor, eps: torch.Tensor):
        """Copy a batch (NCDHW with C=1 == NDHWC) into the engine's resident input slots: one
        launch when the operands allow a plain byte copy (fp32 patches and weights, a bool / uint8
        mask, 16-byte aligned), else one torch copy each."""
        ins = (opt, subopt, mask, eps)
        slots = (self.xc[:self.b_opt], self.subopt, self.mask, self.eps)
        if (all(t.is_cuda and t.is_contiguous() and t.data_ptr() % 16 == 0 and t.numel() == s.numel()
                for t, s in zip(ins, slots)) and opt.dtype == subopt.dtype == eps.dtype == torch.float32
                and mask.dtype in (torch.bool, torch.uint8) and not ops.DRY_RUN and not ops.recording()):
            ops.copy_multi(list(zip(ins, slots)))  # a bool mask's bytes are its 0 / 1 uint8 values
            return
        self.xc[:self.b_opt].view(-1).copy_(opt.reshape(-1), non_blocking=True)
        self.subopt.view(-1).copy_(subopt.reshape(-1), non_blocking=True)
        self.mask.view(-1).copy_(mask.reshape(-1), non_blocking=True)
        self.eps.copy_(eps.reshape(-1), non_blocking=True)

    def set_gp_indices(self, real_rows, fake_rows):
        """Rows of the real (OPT) and fake (opt_hat) batches the gradient penalty interpolates when
        their sizes differ (model/utils.py:21-25: ``real_batch[rng.integers(len(real), size=m)]``)."""
        if self.gp_idx is None:
            raise ValueError("set_gp_indices: |real| == |fake|, the penalty interpolates rows 1:1")
        r = np.asarray(real_rows, dtype=np.int64).reshape(-1)
        f = np.asarray(fake_rows, dtype=np.int64).reshape(-1)
        if r.size != self.b_gp or f.size != self.b_gp:
            raise ValueError(f"set_gp_indices: {self.b_gp} rows each")
        if r.min() < 0 or r.max() >= self.b_opt or f.min() < 0 or f.max() >= self.b_sub:
            raise ValueError("set_gp_indices: row out of range")
        # staged in a ring of pinned buffers and copied without blocking the host (a pageable copy
        # would wait for the previous step to finish); a slot's event guards its reuse
        if not self.gp_idx.is_cuda:
            self.gp_idx.copy_(torch.from_numpy(np.concatenate([r, f]).astype(np.int32)))
            return
        if not hasattr(self, "_gp_ring"):
            self._gp_ring = [(torch.empty(2 * self.b_gp, dtype=torch.int32, pin_memory=True), torch.cuda.Event())
                             for _ in range(4)]
            self._gp_slot = 0
        buf, ev = self._gp_ring[self._gp_slot]
        self._gp_slot = (self._gp_slot + 1) % len(self._gp_ring)
        ev.synchronize()  # the copy that last read this slot (four calls ago) is done
        buf.copy_(torch.from_numpy(np.concatenate([r, f]).astype(np.int32)))
        self.gp_idx.copy_(buf, non_blocking=True)
        ev.record(torch.cuda.current_stream(self.gp_idx.device))

    def draw_gp_indices(self, rng: np.random.Generator):
        """The reference's draw (model/utils.py:24-25): real rows first, then fake rows."""
        r = rng.integers(self.b_opt, size=self.b_gp)
        f = rng.integers(self.b_sub, size=self.b_gp)
        self.set_gp_indices(r, f)
        return r, f

    # -------------------------------------------------------------------------------------------
    def _write_dlogits(self):
        """The constant dlogits (float32 arithmetic, as critic_logits_kernel / gen_logits_kernel)."""
        ps, bo, bs, bg = self.D.logit_ps, self.b_opt, self.b_sub, self.b_gp
        w = torch.tensor(self.gan_w, dtype=torch.float32)
        er, ef, eg = bo * ps, bs * ps, bg * ps
        dl = torch.empty((self.g_off + bs) * ps, dtype=torch.float32)
        dl[:er] = -w / torch.tensor(float(er), dtype=torch.float32)
        dl[er:er + ef] = w / torch.tensor(float(ef), dtype=torch.float32)
        dl[er + ef:er + ef + eg] = 1.0
        dl[er + ef + eg:self.g_off * ps] = 0.0
        dl[self.g_off * ps:] = -w / torch.tensor(float(ef), dtype=torch.float32)
        self.D.dz[-1].view(-1)[:dl.numel()].copy_(dl.to(self.device))

    def generator_forward(self):
        self.G.forward(self.gP, self.subopt, opt_hat_out=self.opt_hat, training=True)
        self.opt_hat_foreign = False  # opt_hat is this forward's output again (Trainer.train_critic)
        if self.gloss_side:
            self.G._on_side(self._generator_loss_grad)

    def _generator_loss_grad(self):
        """ZNCC + HU losses (Trainer.py:148-157) and their gradient through the output tanh into
        G.dz_last; optimizer_G.zero_grad (Trainer.py:146) of the gradient arena."""
        bs, V = self.b_sub, self.vox
        ops.generator_output_grad(self.opt_hat, self.subopt, self.G.att, self.mask, None, bs * V, self.lo, self.hi,
                                  self.sim_w, self.hu_w, self.G.dz_last, self.losses, self.loss_ws_g)
        ops.zero(self.g_arena.grad_padded)

    def critic_update(self):
        if not self.use_gp:
            return self._critic_update_clip()
        D, bo, bs, bg, V = self.D, self.b_opt, self.b_sub, self.b_gp, self.vox
        nall = bo + bs + bg
        if self.gp_idx is None:
            ops.gp_interpolate(self.xc[:bg], self.xc[bo:bo + bg], self.eps, self.xc[bo + bs:], bg, V)
        else:  # |real| != |fake|: resampled rows (model/utils.py:21-25)
            ops.gp_interpolate(self.xc[:bo], self.xc[bo:bo + bs], self.eps, self.xc[bo + bs:], bg, V, idx=self.gp_idx)
        D.forward(self.dP, self.xc, 0, nall)
        if not self.fold_logits:
            ops.critic_logits_grad(D.a[-1], bo, bs, bg, D.logit_ps, self.gan_w, D.dz[-1], self.losses)
        D.input_grad(self.dP, 0, nall, self.gbuf, bo + bs, bg,
                     ep0=ops.epilogue(stats=self.gp_part) if self.gp_part is not None else None)
        if D.ln:  # LayerNorm critic: the interpolation stays in xc (its primal adjoint needs it)
            gamma = D.gam[:bg]
            ops.gradient_penalty(self.gbuf, bg, V, self.gp_weight, gamma, self.losses, self.loss_ws)
            ops.zero(self.d_arena.grad_padded)  # optimizer_D.zero_grad (Trainer.py:109)
            D.gp_grads_ln(self.dP, self.dG, self.xc, gamma, bo + bs, bg)
            self._allreduce(self.d_arena.grad)
            self._optim_step(self.d_optim, self.D)
            return
        gamma = self.xc[bo + bs:]
        if self.gp_part is not None:  # the input-grad wrote the per-sample sums of squares
            ops.gradient_penalty_part(self.gbuf, self.gp_part, bg, self.gp_part.numel() // bg, V, self.gp_weight,
                                      gamma, self.losses, logits=D.a[-1] if self.fold_logits else None, n_real=bo,
                                      n_fake=bs, logit_ps=D.logit_ps, gan_w=self.gan_w,
                                      zero=self.d_arena.grad_padded)  # optimizer_D.zero_grad (Trainer.py:109)
        else:
            ops.gradient_penalty(self.gbuf, bg, V, self.gp_weight, gamma, self.losses, self.loss_ws)
            ops.zero(self.d_arena.grad_padded)  # optimizer_D.zero_grad (Trainer.py:109): every layer then accumulates
        D.gp_grads_overlapped(self.dP, self.dG, self.xc, gamma, bo + bs, bg, nall, bo + bs, zeroed=True)
        D.join_side()
        self._allreduce(self.d_arena.grad)  # on the critical path: the G update uses the new critic
        self._optim_step(self.d_optim, self.D)  # (Adam writing the packed copies itself: +13 us, round 3)

    def _critic_update_clip(self):
        """Weight-clip conf (basic_conf.py:37,60-66): BatchNorm critic run on the real and on the
        fake batch separately (each with its own batch statistics, Trainer.py:119-120), W-loss
        without GP, Adam, then clamp to +-weight_clip (Trainer.py:136-138, inside the Adam kernel)."""
        D, bo, bs = self.D, self.b_opt, self.b_sub
        D.forward(self.dP, self.xc[:bo], 0, bo, bn_pass=0)
        D.forward(self.dP, self.opt_hat, bo, bs, bn_pass=1)
        ops.critic_logits_grad(D.a[-1], bo, bs, 0, D.logit_ps, self.gan_w, D.dz[-1], self.losses)
        ops.zero(self.d_arena.grad_padded)  # optimizer_D.zero_grad (Trainer.py:109)
        D.input_grad(self.dP, 0, bo, self.gbuf, 0, 0, bn_pass=0, G=self.dG)
        D.input_grad(self.dP, bo, bs, self.gbuf, 0, 0, bn_pass=1, G=self.dG, bn_accumulate=True)
        D.weight_grads(self.dP, self.dG, self.xc[:bo + bs], bo + bs, bo + bs, zeroed=True)
        self._allreduce(self.d_arena.grad)
        self._optim_step(self.d_optim, self.D)

    def generator_update(self):
        D, bs, V = self.D, self.b_sub, self.vox
        if self.gloss_side:  # the loss gradient and the zeroed arena (generator_forward) are in
            ops.stream_wait(torch.cuda.current_stream(self.device), self.G.side)
        go = self.g_off
        D.forward(self.dP, self.opt_hat, go, bs)
        if not self.fold_logits:
            ops.generator_logits_grad(D.a[-1][:bs], bs * D.logit_ps, self.gan_w, D.dz[-1], self.losses)
        if self.gloss_side:
            D.input_grad(self.dP, go, bs, self.G.dz_last, go, bs,
                         ep0=ops.epilogue(residual=self.G.dz_last, mask_src=self.G.att, act=L.ACT_NEG_DTANH))
        else:
            D.input_grad(self.dP, 0, bs, self.dcrit, 0, bs)
            ops.generator_output_grad(self.opt_hat, self.subopt, self.G.att, self.mask, self.dcrit, bs * V, self.lo,
                                      self.hi, self.sim_w, self.hu_w, self.G.dz_last, self.losses, self.loss_ws)
            ops.zero(self.g_arena.grad_padded)  # optimizer_G.zero_grad (Trainer.py:146): every layer then accumulates
        if self.dp and self.g_buckets:  # bucketed, overlapped with the rest of the backward
            self.G.backward(self.gP, self.gG, self.subopt, grads_enqueued=self._bucket_ready, zeroed=True,
                            side_first=self._gen_logit_loss)
            self._finish_allreduce()
        else:
            self.G.backward(self.gP, self.gG, self.subopt, zeroed=True, side_first=self._gen_logit_loss,
                            side_after=self._g_early if self.g_split else None)
            if self.dp:  # CGAN3D_G_BUCKET_BYTES=0: one all-reduce of the whole gradient (main stream)
                self._allreduce(self.g_arena.grad)
        if self.g_split:
            self._g_tail()
        else:
            self._optim_step(self.g_optim, self.G)

    def _g_early(self):
        """Adam (step + 1, no tick) and repack of the generator layers updated ahead of the tail."""
        a, lo = self.g_arena, self.g_split
        ops.adam_range(a.flat[lo:], a.grad[lo:], a.exp_avg[lo:], a.exp_avg_sq[lo:], self.g_optim.hyper)
        self.G.pack_early()

    def _g_tail(self):
        """Adam of the tail layers (the arena prefix) with the step tick, then their repack."""
        a, lo, opt = self.g_arena, self.g_split, self.g_optim
        ops.adam_pack(a.flat[:lo], a.grad[:lo], a.exp_avg[:lo], a.exp_avg_sq[:lo], opt.hyper, opt.ticket)
        opt._opt_called = True  # what torch's LR schedulers check optimizer.step() for
        if not ops.recording():  # a recorded plan counts its steps when it runs (note_step)
            opt._host_step += 1
        self.G.pack_tail()

    def _gen_logit_loss(self):
        """The generator's adversarial loss (and the full generator loss) from its critic logits, beside
        its backward (fold_logits: the dlogits are constant)."""
        if self.fold_logits:
            bs, go = self.b_sub, self.g_off
            ops.generator_logits_grad(self.D.a[-1][go:go + bs], bs * self.D.logit_ps, self.gan_w, None, self.losses)

    @staticmethod
    def _optim_step(optim, plan):
        """optimizer.step() (Trainer.py:135,158): Adam with the step tick in one launch, then the
        plan's packed weight copies (one coalesced repack launch)."""
        optim.launch()
        plan.pack()

    def _allreduce(self, flat_grad: torch.Tensor):
        """Mean of the per-rank gradients (RCCL over xGMI with the nccl backend; gloo on CPU)."""
        if not self.dp:
            return
        if self.native is not None:  # on the main stream: the generator update needs the new critic
            self._log_comm("allreduce", "main", *self._arena_span(flat_grad))
            self.native.allreduce_mean(flat_grad)
            return
        self._log_comm("allreduce", "sync", *self._arena_span(flat_grad))
        dist = torch.distributed

        def reduce():
            if dist.get_backend(self.pg) == "nccl":
                dist.all_reduce(flat_grad, op=dist.ReduceOp.AVG, group=self.pg)
            else:
                dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM, group=self.pg)
                flat_grad.mul_(1.0 / self.world)
        ops.plan_host(reduce)  # inside a recorded plan: runs between its C segments

    def capture(self, do_critic: bool = True, do_generator: bool = True):
        """Record one whole step (~200 launches) as a HIP graph; ``replay()`` then costs one launch.

        Valid because every launch reads its scalars from device memory (Adam step/lr) and every
        buffer is resident; inputs are loaded into the same slots before each replay.  Run one
        eager ``step()`` first (kernel code objects load lazily, which capture cannot record)."""
        if self.world > 1:
            raise NotImplementedError("graph capture with collectives: launch eagerly under DDP")
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(graph, stream=s):
                self.step(do_critic, do_generator)
        torch.cuda.current_stream(self.device).wait_stream(s)
        self.graph = graph
        return graph

    def replay(self):
        self.graph.replay()
        return self.losses

    def record(self, do_critic: bool = True, do_generator: bool = True) -> "ops.Plan":
        """Record one step as a launch plan (cgan3d_plan_*): ``run_plan()`` then re-issues its
        ~200 launches from C++ on the same two streams, without the Python wrappers' per-launch
        cost.  Nothing is executed while recording.  Collectives (world > 1) stay host callables
        between the plan's C segments.  Same validity rules as ``capture``; the plan runs on the
        streams current at recording time."""
        ops.plan_begin()
        try:
            self.step(do_critic, do_generator)
        except BaseException:
            ops.plan_abort()
            raise
        self.plan = ops.plan_end()
        return self.plan

    def run_plan(self):
        self.plan.run()
        return self.losses

    def step(self, do_critic: bool = True, do_generator: bool = True):
        """Trainer.train_step body (Trainer.py:169-184) on the resident inputs."""
        self.generator_forward()
        if do_critic:
            self.critic_update()
        if do_generator:
            self.generator_update()
        return self.losses
