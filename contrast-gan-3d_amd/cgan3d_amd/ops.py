"""Thin launch wrappers over the C-ABI (include/cgan3d.h), operating on device tensors.

Activations are fp32 NDHWC tensors ``[N, D, H, W, C]``; weights stay in torch layout.  Every
wrapper launches on the current torch stream and never synchronises, so a whole step can be
captured in a HIP graph.  Geometry helpers build the gather descriptors for each role a conv
plays in the step (forward, input-grad, weight-grad; Conv3d and ConvTranspose3d).

Every wrapper first checks on the host that each operand's extent matches what the kernel and
its grid will touch (a kernel fault on the GPU box can reset the node).  With ``DRY_RUN = True``
only these checks run — the whole step can be shape-checked on CPU tensors without a GPU.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional, Sequence

import torch

from . import _lib as L
from ._lib import ConvGeom, Epilogue, PackDesc, check, ptr

DRY_RUN = False


def _geom(n, di, do, cin, cout, k, s, p, transposed, reflect, sa, sb, planar=False) -> ConvGeom:
    g = ConvGeom()
    g.n = n
    g.di, g.hi, g.wi = di
    g.do_, g.ho, g.wo = do
    g.cin, g.cout, g.k, g.stride, g.pad = cin, cout, k, s, p
    g.transposed, g.reflect = int(transposed), int(reflect)
    g.w_sa, g.w_sb = sa, sb
    g.w_packed, g.prec = 0, L.PREC_F32
    g.planar = int(planar)
    return g


def taps(g) -> int:
    """Kernel taps of a geometry: k^3, or k^2 for the 2-D variants (``planar``)."""
    return g.k ** 2 if g.planar else g.k ** 3


def uses_gemm(g: ConvGeom) -> bool:
    """True when cgan3d_conv3d_fwd routes this geometry to the implicit-GEMM kernel (which can read
    packed weights and run in bf16); k7 single-channel and cout == 1 launches use direct kernels."""
    if g.cout < 2:
        return False
    if g.planar:  # 2-D variants: every cout >= 2 role on the implicit GEMM
        return True
    if g.cin == 1 and g.cout == 8 and g.k == 4 and g.stride == 2 and g.pad == 1 and not g.transposed:
        return False  # critic first layer: conv_c1.hip reads torch-layout weights
    if g.cin == 1 and g.transposed and L.load().cgan3d_conv3d_cin1t(ctypes.byref(g)):
        return False  # the critic's last-layer input-grad: direct fp32 kernel on torch-layout weights
    return not (g.k == 7 and g.stride == 1 and g.cin == 1 and g.cout in (8, 16))


# bf16 launches whose geometry the halo-tiled kernel takes use it (conv_halo.hip)
HALO = True


def halo_eligible(g: ConvGeom) -> bool:
    return bool(L.load().cgan3d_halo_eligible(ctypes.byref(g)))


# conv_sk.hip takes the critic's k4 convs in bf16 (format 3)
SK = True

# data-parallel collectives (engine.StepEngine): "native" (default) RCCL from the launch plan on the
# process group's communicator, "torch" torch.distributed host callables (the fallback), "own" a
# communicator of this library's (NativeComm own=True)
COMM_MODE = os.environ.get("CGAN3D_COMM", "native")
if COMM_MODE not in ("native", "torch", "own"):
    raise ValueError(f"CGAN3D_COMM={COMM_MODE!r}: native, torch or own")


def with_packing(g: ConvGeom, prec: int = L.PREC_F32) -> ConvGeom:
    """Copy of ``g`` that reads packed weights (cgan3d_pack_weights) and runs in ``prec``: in bf16
    format 3 (K-split small-grid kernel, bf16 [b][tap][a]) or 2 (halo kernel, bf16 [tap][b][a])
    where eligible (cgan3d_packed_format), else format 1 ([tap][a][b] f32)."""
    h = ConvGeom()
    ctypes.pointer(h)[0] = g
    h.w_packed, h.prec = 1, prec
    if prec == L.PREC_BF16 and HALO:
        f = int(L.load().cgan3d_packed_format(ctypes.byref(h)))
        if f == 3 and not SK:
            f = 2 if halo_eligible(h) else 1
        h.w_packed = f
    return h


def with_prec(g: ConvGeom, prec: int) -> ConvGeom:
    """Copy of ``g`` computing in ``prec`` (unpacked weights): the k7 single-channel kernels and
    the weight-gradient launches read it."""
    h = ConvGeom()
    ctypes.pointer(h)[0] = g
    h.prec = prec
    return h


def packed_elements(g: ConvGeom) -> int:
    """Elements (f32 or bf16) the pack kernel writes for ``g``."""
    if g.w_packed in (2, 3):
        return taps(g) * g.cin * g.cout
    return taps(g) * g.cin * ((g.cout + 3) // 4 * 4)


def packed_weight_floats(g: ConvGeom) -> int:
    return int(L.load().cgan3d_packed_weight_floats(ctypes.byref(g)))


def pack_desc(g: ConvGeom, w: torch.Tensor, wp: torch.Tensor) -> PackDesc:
    _need(w, _w_extent(g), "pack w", exact=False)
    _need(wp, packed_weight_floats(g), "pack wp")
    d = PackDesc()
    d.w, d.wp, d.sa, d.sb = ptr(w), ptr(wp), g.w_sa, g.w_sb
    d.taps, d.cin, d.cout, d.ldb = taps(g), g.cin, g.cout, (g.cout + 3) // 4 * 4
    d.format = g.w_packed
    return d


def pack_weights(g: ConvGeom, w: torch.Tensor, wp: torch.Tensor):
    pack_desc(g, w, wp)
    check(_launch("cgan3d_pack_weights", ctypes.byref(g), ptr(w), ptr(wp)), "pack_weights")


def pack_weights_multi(descs_dev: torch.Tensor, n: int, max_total: int):
    """descs_dev: device uint8 tensor holding n PackDesc structs (built by PackSet)."""
    if descs_dev.numel() != n * ctypes.sizeof(PackDesc):
        raise ValueError("pack_weights_multi: descriptor buffer size mismatch")
    check(_launch("cgan3d_pack_weights_multi", ptr(descs_dev), n, max_total), "pack_weights_multi")


class PackSet:
    """All packed weight copies of one network, refreshed by ONE launch after each optimiser step."""

    def __init__(self, device):
        self.device, self.descs, self.max_total = device, [], 0
        self.dev = None

    def add(self, g: ConvGeom, w: torch.Tensor, prec: int):
        """Returns (geometry, weight) to launch with: packed when the GEMM path applies."""
        if not uses_gemm(g):
            return with_prec(g, prec), w
        gp = with_packing(g, prec)
        wp = torch.zeros(packed_weight_floats(gp), device=self.device)
        self.descs.append((pack_desc(gp, w, wp), wp, w))  # keeps the source alive: the descriptor holds its pointer
        self.max_total = max(self.max_total, packed_elements(gp))
        self.dev = None
        return gp, wp

    def device_descs(self) -> torch.Tensor:
        if self.dev is None:
            raw = b"".join(bytes(d[0]) for d in self.descs)
            self.dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device)
        return self.dev

    def pack(self):
        if not self.descs:
            return
        pack_weights_multi(self.device_descs(), len(self.descs), self.max_total)


# --- geometry per role ------------------------------------------------------------------------
# Conv3d(cin -> cout), weight [cout, cin, k,k,k]; din = input dims, dout = output dims.
# planar=True: the 2-D variants (Conv2d / ConvTranspose2d, weights [., ., k, k]) on dims (1, H, W)
def conv_fwd_geom(n, din, dout, cin, cout, k, s, p, reflect=False, planar=False):
    t = k**2 if planar else k**3
    return _geom(n, din, dout, cin, cout, k, s, p, 0, reflect, t, cin * t, planar)


def conv_dgrad_geom(n, din, dout, cin, cout, k, s, p, planar=False):
    t = k**2 if planar else k**3
    return _geom(n, dout, din, cout, cin, k, s, p, 1, 0, cin * t, t, planar)


def conv_wgrad_geom(n, din, dout, cin, cout, k, s, p, reflect=False, planar=False):
    t = k**2 if planar else k**3
    return _geom(n, din, dout, cin, cout, k, s, p, 0, reflect, t, cin * t, planar)


# ConvTranspose3d(cin -> cout), weight [cin, cout, k,k,k]; din = input dims, dout = output dims
def convt_fwd_geom(n, din, dout, cin, cout, k, s, p, planar=False):
    t = k**2 if planar else k**3
    return _geom(n, din, dout, cin, cout, k, s, p, 1, 0, cout * t, t, planar)


def convt_dgrad_geom(n, din, dout, cin, cout, k, s, p, planar=False):
    t = k**2 if planar else k**3
    return _geom(n, dout, din, cout, cin, k, s, p, 0, 0, t, cout * t, planar)


def convt_wgrad_geom(n, din, dout, cin, cout, k, s, p, planar=False):
    """gathered operand = the ConvTranspose output-grad; aligned operand = its input."""
    t = k**2 if planar else k**3
    return _geom(n, dout, din, cout, cin, k, s, p, 0, 0, t, cout * t, planar)


class BnFuse:
    """BatchNorm statistics into fp64 accumulators (include/cgan3d.h cgan3d_bn_fuse): the producing
    conv adds its statistic pairs into ``acc_out`` (float64 [reps][2][cout]) — ``acc_mode`` 3 forward
    (sum, sum of squares), 4 input-grad (sum g, sum g*xhat, with the epilogue's bn_z / bn_ss / bn_mi)."""

    def __init__(self, acc_out=None, acc_mode=0, reps=1):
        self.acc_out, self.acc_mode, self.reps = acc_out, int(acc_mode), int(reps)

    def check(self, g, what):
        if self.acc_mode:
            _need(self.acc_out, self.reps * 2 * g.cout, f"{what} acc_out", dtype=torch.float64)

    def c(self) -> "L.BnFuse":
        f = L.BnFuse()
        f.acc_out, f.acc_mode, f.reps = ptr(self.acc_out), self.acc_mode, self.reps
        return f


def out_bf16_ok(g) -> bool:
    """cgan3d_conv3d_out_bf16_ok: the launch of ``g`` can write a bf16 output (and read a bf16 bn_z)."""
    return bool(L.load().cgan3d_conv3d_out_bf16_ok(ctypes.byref(g)))


def neg_dtanh_ok(g) -> bool:
    """cgan3d_conv3d_neg_dtanh_ok: the input-grad geometry takes the L.ACT_NEG_DTANH epilogue."""
    return bool(L.load().cgan3d_conv3d_neg_dtanh_ok(ctypes.byref(g)))


def bn_pre_ok(g: ConvGeom) -> bool:
    """The launch of ``g`` can apply its input's BatchNorm while staging (cgan3d_conv3d_bn_pre_ok)."""
    return bool(L.load().cgan3d_conv3d_bn_pre_ok(ctypes.byref(g)))


def bn_fuse_ok(g) -> bool:
    """True if the launch of ``g`` can produce BnFuse accumulators."""
    return bool(L.load().cgan3d_bn_fuse_ok(ctypes.byref(g)))


class BnPre:
    """The conv input's BatchNorm applied while the ResNet-block kernel stages its halo
    (include/cgan3d.h cgan3d_bn_pre, round 5): ``forward`` (mode 1: the launch's x_bf16 is the previous
    layer's bf16 z) or ``backward`` (mode 2: x_bf16 is the layer's bf16 dL/dy).  Tensors are kept for
    the checks and for the struct's lifetime."""

    def __init__(self, mode, c, nvox, acc, reps, gamma, scale_shift, mean_invstd, act, out16, slope=0.0, zero=None,
                 z=None, beta=None, rmean=None, rvar=None, nbt=None, momentum=0.1, eps=1e-5, dgamma=None, dbeta=None,
                 accumulate=False):
        self.mode, self.c, self.nvox, self.reps = int(mode), int(c), int(nvox), int(reps)
        self.acc, self.gamma, self.ss, self.mi, self.act, self.out16 = acc, gamma, scale_shift, mean_invstd, act, out16
        self.slope, self.zero, self.z, self.beta = float(slope), zero, z, beta
        self.rmean, self.rvar, self.nbt, self.momentum, self.eps = rmean, rvar, nbt, float(momentum), float(eps)
        self.dgamma, self.dbeta, self.accumulate = dgamma, dbeta, bool(accumulate)

    @classmethod
    def forward(cls, acc, reps, c, nvox, gamma, beta, rmean, rvar, nbt, scale_shift, mean_invstd, act, out16,
                slope=0.0, zero=None, momentum=0.1, eps=1e-5):
        return cls(1, c, nvox, acc, reps, gamma, scale_shift, mean_invstd, act, out16, slope, zero, beta=beta,
                   rmean=rmean, rvar=rvar, nbt=nbt, momentum=momentum, eps=eps)

    @classmethod
    def backward(cls, z, acc, reps, c, nvox, scale_shift, mean_invstd, gamma, act, dgamma, dbeta, out16, slope=0.0,
                 accumulate=False, zero=None):
        return cls(2, c, nvox, acc, reps, gamma, scale_shift, mean_invstd, act, out16, slope, zero, z=z,
                   dgamma=dgamma, dbeta=dbeta, accumulate=accumulate)

    def check(self, g, x16):
        if not int(L.load().cgan3d_conv3d_bn_pre_ok(ctypes.byref(g))):
            raise ValueError("conv: BatchNorm prologue (pre) only on the ResNet-block kernel")
        n = self.nvox * self.c
        _need(x16, n, "conv pre x_bf16", dtype=torch.bfloat16)
        _need(self.out16, n, "conv pre out16", dtype=torch.bfloat16)
        _need(self.acc, self.reps * 2 * self.c, "conv pre acc", dtype=torch.float64, exact=False)
        for t, nm in ((self.gamma, "gamma"),) + (((self.beta, "beta"),) if self.mode == 1 else
                                                 ((self.dgamma, "dgamma"), (self.dbeta, "dbeta"))):
            _need(t, self.c, f"conv pre {nm}")
        for t, nm in ((self.ss, "scale_shift"), (self.mi, "mean_invstd")):
            _need(t, 2 * self.c, f"conv pre {nm}")
        if self.mode == 2:
            _need(self.z, n, "conv pre z", dtype=torch.bfloat16)
        if self.zero is not None:
            _need(self.zero, self.zero.numel(), "conv pre zero", dtype=torch.float64)

    def c_struct(self) -> "L.BnPre":
        p = L.BnPre()
        p.mode, p.z, p.acc, p.reps, p.nvox = self.mode, ptr(self.z), ptr(self.acc), self.reps, self.nvox
        p.gamma, p.beta, p.running_mean, p.running_var = ptr(self.gamma), ptr(self.beta), ptr(self.rmean), ptr(self.rvar)
        p.num_batches_tracked, p.momentum, p.eps = ptr(self.nbt), self.momentum, self.eps
        p.scale_shift, p.mean_invstd, p.dgamma, p.dbeta = ptr(self.ss), ptr(self.mi), ptr(self.dgamma), ptr(self.dbeta)
        p.accumulate, p.act, p.slope, p.out_bf16 = int(self.accumulate), int(self.act), self.slope, ptr(self.out16)
        p.zero, p.zero_n = ptr(self.zero), self.zero.numel() if self.zero is not None else 0
        return p


class Epi:
    """Fused-epilogue operands (include/cgan3d.h cgan3d_epilogue), kept as tensors for checks."""

    def __init__(self, bias=None, residual=None, mask_src=None, minuend=None, out2=None, stats=None,
                 act=L.ACT_NONE, slope=0.0, bn_part=None, bn_mode=0, bn_slots=0, bn_z=None, bn_ss=None,
                 bn_mi=None, bn_act=L.ACT_NONE, bn_slope=0.0, x_bf16=None, bn_fold=0, fuse=None, pre=None):
        self.fuse = fuse  # BnFuse or None
        self.pre = pre  # BnPre or None: the input's BatchNorm applied while staging (conv_k3m)
        self.bias, self.residual, self.mask_src = bias, residual, mask_src
        self.x_bf16 = x_bf16  # bf16 copy of the conv input (ResNet-block kernel halo source)
        self.minuend, self.out2, self.stats = minuend, out2, stats
        self.act, self.slope = act, float(slope)
        # fused BatchNorm statistics slab (per-block partial pairs): see include/cgan3d.h
        self.bn_part, self.bn_mode, self.bn_slots = bn_part, int(bn_mode), int(bn_slots)
        self.bn_z, self.bn_ss, self.bn_mi = bn_z, bn_ss, bn_mi
        self.bn_act, self.bn_slope = bn_act, float(bn_slope)
        self.bn_fold = int(bn_fold)  # mode 2 over a reflect-padded k7 input-grad grid (include/cgan3d.h)
        self.out_bf16 = 0  # set by conv() from the output's dtype (include/cgan3d.h out_bf16)

    def check_bn(self, nout, c, what, nz=None):
        if not self.bn_mode:
            return
        _need(self.bn_part, (2 * c + (self.bn_mode == 1)) * self.bn_slots, f"{what} bn_part", exact=False)
        if self.bn_mode == 2:
            _need(self.bn_z, nout if nz is None else nz, f"{what} bn_z")
            _need(self.bn_ss, 2 * c, f"{what} bn_ss")
            _need(self.bn_mi, 2 * c, f"{what} bn_mi")

    def c(self) -> Epilogue:
        e = Epilogue()
        e.bias, e.residual, e.mask_src = ptr(self.bias), ptr(self.residual), ptr(self.mask_src)
        e.minuend, e.out2, e.stats = ptr(self.minuend), ptr(self.out2), ptr(self.stats)
        e.act, e.slope = self.act, self.slope
        e.bn_part, e.bn_mode, e.bn_slots, e.bn_z = ptr(self.bn_part), self.bn_mode, self.bn_slots, ptr(self.bn_z)
        e.bn_ss, e.bn_mi, e.bn_act, e.bn_slope = ptr(self.bn_ss), ptr(self.bn_mi), self.bn_act, self.bn_slope
        e.x_bf16 = ptr(self.x_bf16)
        e.bn_fold = self.bn_fold
        e.out_bf16 = self.out_bf16
        if self.fuse is not None:
            e.fuse = ctypes.pointer(self.fuse.c())  # the pointer object keeps the struct alive
        if self.pre is not None:
            e.pre = ctypes.pointer(self.pre.c_struct())
        return e


def epilogue(**kw) -> Epi:
    return Epi(**kw)


# --- host-side operand checks -------------------------------------------------------------------
def _need(t, n, what, dtype=torch.float32, exact=True):
    if t is None:
        raise ValueError(f"{what}: missing operand")
    if t.dtype != dtype:
        raise TypeError(f"{what}: dtype {t.dtype} != {dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{what}: operand must be contiguous")
    if (t.numel() != n) if exact else (t.numel() < n):
        raise ValueError(f"{what}: has {t.numel()} elements, kernel touches {n}")


def _vox_in(g):
    return g.n * g.di * g.hi * g.wi


def _vox_out(g):
    return g.n * g.do_ * g.ho * g.wo


def _w_extent(g):
    return (g.cin - 1) * g.w_sa + (g.cout - 1) * g.w_sb + taps(g)


def _launch(name, *args):
    if DRY_RUN:
        return 0
    return getattr(L.lib(), name)(*args, L.stream())


def stream_wait(waiter, signaler):
    """``waiter`` (torch stream) waits for the work enqueued so far on ``signaler`` — recorded
    when inside a plan, unlike torch's ``Stream.wait_stream``."""
    if DRY_RUN or waiter is None or signaler is None:
        return
    check(L.lib().cgan3d_stream_wait(waiter.cuda_stream, signaler.cuda_stream), "stream_wait")


_STREAM_POOL: Dict[int, Dict[str, "torch.cuda.Stream"]] = {}
POOL_ROLES = ("g_side", "d_side", "comm", "copy")  # copy: host-to-device batches (PatchLoader)


def pooled_stream(device, role: str) -> "torch.cuda.Stream":
    """One stream per (device, role), shared by every engine and plan of the process.

    HIP hands a new stream the next hardware queue round-robin (GPU_MAX_HW_QUEUES), so engines that
    each created their own side streams ran on different queue mappings — the same exact-f32 step
    measured 5.2 ms/step as the first engine of a process, 8.5 as the second and 5.1 as the fourth
    (profiles/r04_f32_sub_probe.txt).  All roles are created together on first use, so every engine
    gets the mapping of the first; plans run in turn on one host thread, so sharing keeps their order."""
    if role not in POOL_ROLES:
        raise ValueError(f"pooled_stream: role {role!r} not in {POOL_ROLES}")
    if "own_streams" in os.environ.get("CGAN3D_DEBUG", ""):  # A/B: a new stream per plan (rounds 1-4)
        return torch.cuda.Stream(device=device)
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    pool = _STREAM_POOL.get(idx)
    if pool is None:
        pool = _STREAM_POOL[idx] = {r: torch.cuda.Stream(device=idx) for r in POOL_ROLES}
    return pool[role]


class NativeComm:
    """RCCL all-reduces as C-ABI launches over a torch.distributed process group's ranks
    (include/cgan3d.h cgan3d_comm_*), recorded into launch plans like a kernel.

    Default: the process group's own communicator (ProcessGroupNCCL._comm_ptr), driven through the
    RCCL library torch loaded — one communicator per process.  ``own=True`` (or
    CGAN3D_COMM=own): a communicator of this library, rank 0's unique id broadcast through
    ``group`` once (measured: a second communicator in the process slows every kernel of a one-GPU
    step ~2.4x, profiles/r03_dp1_probe.json).  When the group's communicator cannot be reached (a
    torch without ``_comm_ptr``, or another RCCL library than the one this build drives) the own
    communicator is used, with a warning.

    A group on another backend (gloo, CPU dry runs — tests/test_dist.py): the same object and call
    sequence, the collective itself done by torch.distributed on ``group`` (``self.handle`` None)."""

    def __init__(self, group=None, device=None, own=None):
        import torch.distributed as dist
        self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)
        self.owned = False
        self.group = group
        self.handle = None
        if dist.get_backend(group) != "nccl":
            return
        lib = L.lib()
        if own is None:
            own = COMM_MODE == "own"
        if not own:
            ptr = self._torch_comm(group, device)
            shared = int(lib.cgan3d_comm_shared_library()) == 1
            if ptr and shared:
                self.handle = ctypes.c_void_p(ptr)
                return
            import warnings
            why = ("ProcessGroupNCCL._comm_ptr is unavailable in this torch" if not ptr else
                   "torch's RCCL library is not the one libcgan3d drives")
            warnings.warn(f"NativeComm: {why}; using a communicator of this library instead (CGAN3D_COMM=own: "
                          "one more communicator in the process, measured ~2.4x slower kernels on one GPU)",
                          RuntimeWarning, stacklevel=2)
        self.owned = True
        nb = int(lib.cgan3d_comm_id_bytes())
        uid = torch.zeros(nb, dtype=torch.uint8, device=device)
        if self.rank == 0:
            host = (ctypes.c_char * nb)()
            check(lib.cgan3d_comm_unique_id(host), "comm_unique_id")
            uid.copy_(torch.frombuffer(bytearray(host.raw), dtype=torch.uint8))
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast(uid, src, group=group)
        raw = bytes(uid.cpu().numpy().tobytes())
        h = ctypes.c_void_p()
        check(lib.cgan3d_comm_init(raw, self.world, self.rank, ctypes.byref(h)), "comm_init")
        self.handle = h

    @staticmethod
    def _torch_comm(group, device):
        """The ncclComm_t of ``group``'s nccl backend (0 if unavailable); a first collective
        creates it when the group was not initialised eagerly (init_process_group(device_id=))."""
        import torch.distributed as dist
        pg = group if group is not None else dist.distributed_c10d._get_default_group()
        try:
            be = pg._get_backend(torch.device(device))
            ptr = int(be._comm_ptr())
            if not ptr:
                dist.all_reduce(torch.zeros(1, device=device), group=group)
                torch.cuda.synchronize(device)
                ptr = int(be._comm_ptr())
            return ptr
        except (AttributeError, RuntimeError):
            return 0

    def allreduce_mean(self, t: torch.Tensor):
        """t = mean over the ranks of t (fp32, contiguous), on the current stream."""
        if self.handle is None:  # non-RCCL group (gloo): torch.distributed does the exchange
            import torch.distributed as dist
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            t.mul_(1.0 / self.world)
            return
        _need(t, t.numel(), "allreduce_mean")
        check(_launch("cgan3d_allreduce_mean", self.handle, ptr(t), t.numel()), "allreduce_mean")

    def __del__(self):
        if getattr(self, "owned", False) and getattr(self, "handle", None) is not None and L._lib is not None:
            L._lib.cgan3d_comm_destroy(self.handle)
            self.handle = None


class Plan:
    """A recorded step: C-side launch plans (cgan3d_plan_*, include/cgan3d.h) interleaved with host
    callables that cannot be recorded (RCCL collectives).  ``run()`` re-issues it."""

    def __init__(self):
        self.items = []
        self.launches = 0

    def run(self):
        lib = L.lib()
        for it in self.items:
            if isinstance(it, int):
                check(lib.cgan3d_plan_run(it), "plan_run")
            else:
                it()

    def kernel_times(self):
        """Durations (ms) of the launches timed in the last ``run()`` (``plan_time_filter`` at record
        time), in record order; call after synchronising."""
        lib, out = L.lib(), []
        for it in self.items:
            if isinstance(it, int):
                n = int(lib.cgan3d_plan_times(it, None, 0))
                buf = (ctypes.c_float * max(n, 1))()
                lib.cgan3d_plan_times(it, buf, n)
                out += [float(v) for v in buf[:n]]
        return out

    def timeline(self):
        """The timed launches of the last ``run()`` as (stream index, start ms, end ms, kernel name), times from
        each C segment's first timed launch (one segment without collectives); call after synchronising."""
        lib, out = L.lib(), []
        for it in self.items:
            if isinstance(it, int):
                n = int(lib.cgan3d_plan_timeline(it, None, None, None, 0))
                a, b, sid = (ctypes.c_float * max(n, 1))(), (ctypes.c_float * max(n, 1))(), (ctypes.c_int32 * max(n, 1))()
                lib.cgan3d_plan_timeline(it, a, b, sid, n)
                for i in range(n):
                    nm = lib.cgan3d_plan_timed_name(it, i)
                    out.append((int(sid[i]), float(a[i]), float(b[i]), nm.decode() if nm else "?"))
        return out

    def __del__(self):
        if L._lib is not None:
            for it in self.items:
                if isinstance(it, int):
                    L._lib.cgan3d_plan_destroy(it)
        self.items = []


_RECORDING: Optional[Plan] = None


def plan_time_filter(substring: Optional[str]):
    """Plans recorded while set time each launch of a kernel whose name contains ``substring`` with its
    own HIP events (cgan3d_plan_time_filter; ``Plan.kernel_times``); None clears it."""
    check(L.lib().cgan3d_plan_time_filter(substring.encode() if substring else None), "plan_time_filter")


def recording() -> bool:
    return _RECORDING is not None


def plan_begin() -> Plan:
    global _RECORDING
    if _RECORDING is not None:
        raise RuntimeError("plan_begin: already recording")
    check(L.lib().cgan3d_plan_begin(), "plan_begin")
    _RECORDING = Plan()
    return _RECORDING


def _plan_close():
    h = ctypes.c_void_p()
    check(L.lib().cgan3d_plan_end(ctypes.byref(h)), "plan_end")
    _RECORDING.launches += int(L.lib().cgan3d_plan_size(h))
    _RECORDING.items.append(h.value)


def plan_host(fn):
    """While recording: close the current C plan, append host callable ``fn``, open a new plan.
    Otherwise: call ``fn`` now."""
    if _RECORDING is None:
        return fn()
    _plan_close()
    _RECORDING.items.append(fn)
    check(L.lib().cgan3d_plan_begin(), "plan_begin")


def plan_end() -> Plan:
    global _RECORDING
    if _RECORDING is None:
        raise RuntimeError("plan_end: not recording")
    _plan_close()
    p, _RECORDING = _RECORDING, None
    return p


def plan_abort():
    """Drop a recording (after an exception while recording)."""
    global _RECORDING
    if _RECORDING is None:
        return
    try:
        _plan_close()
    finally:
        _RECORDING = None


# bench.py's roofline timer: LAUNCH_HOOK(role, geometry) returns (start, end, reps) — two
# torch.cuda.Event recorded on the launch stream around ``reps`` back-to-back repeats of that
# launch (idempotent: same operands, same outputs), or around the step's own launch when reps is
# 0 — or None.
LAUNCH_HOOK = None


def _timed(role, g, name, *args):
    ev = LAUNCH_HOOK(role, g) if LAUNCH_HOOK is not None else None
    if ev is None:
        return _launch(name, *args)
    if ev[2] == 0:  # the step's own launch, in place (in-step timing)
        ev[0].record()
        rc = _launch(name, *args)
        ev[1].record()
        return rc
    rc = _launch(name, *args)  # the step's own launch; then the timed repeats
    ev[0].record()
    for _ in range(ev[2]):
        rc = rc or _launch(name, *args)
    ev[1].record()
    return rc


# --- launches -----------------------------------------------------------------------------------
def stats_floats(g: ConvGeom) -> int:
    return int(L.load().cgan3d_conv3d_stats_floats(ctypes.byref(g)))


def conv(g: ConvGeom, x: torch.Tensor, w: torch.Tensor, y: torch.Tensor, ep: Optional[Epi] = None):
    _need(x, _vox_in(g) * g.cin, "conv x")
    if g.w_packed:
        if not uses_gemm(g):
            raise ValueError("conv: packed weights only on the implicit-GEMM path")
        _need(w, packed_weight_floats(g), "conv packed w")
    else:
        _need(w, _w_extent(g), "conv w", exact=False)
    ny = _vox_out(g) * g.cout
    out16 = y is not None and y.dtype == torch.bfloat16
    res16 = ep is not None and ep.residual is not None and ep.residual.dtype == torch.bfloat16
    if out16 or res16:  # bf16 storage of BatchNorm inputs / gradients (include/cgan3d.h out_bf16)
        if ep is None or not out_bf16_ok(g):
            raise ValueError("conv: a bf16 output / residual only where cgan3d_conv3d_out_bf16_ok (with an epilogue)")
        ep.out_bf16 = (1 if out16 else 0) | (2 if res16 else 0)
    elif ep is not None:
        ep.out_bf16 = 0
    _need(y, ny, "conv y", dtype=y.dtype if out16 else torch.float32)
    if ep is not None:
        if ep.bias is not None:
            _need(ep.bias, g.cout, "conv bias")
        for nm in ("residual", "mask_src", "minuend", "out2"):
            if getattr(ep, nm) is not None:
                _need(getattr(ep, nm), ny, f"conv {nm}", dtype=torch.bfloat16 if nm == "residual" and res16 else torch.float32)
        if ep.stats is not None:  # the critic first-layer input-grad: per-block sums of squares
            _need(ep.stats, sumsq_blocks(g) or stats_floats(g), "conv stats", exact=False)
        if ep.x_bf16 is not None:
            _need(ep.x_bf16, _vox_in(g) * g.cin, "conv x_bf16", dtype=torch.bfloat16)
        f = ep.bn_fold
        nz = None if not f else g.n * (g.do_ - 2 * f) * (g.ho - 2 * f) * (g.wo - 2 * f) * g.cout
        ep.check_bn(ny, g.cout, "conv", nz)
        if ep.fuse is not None:
            ep.fuse.check(g, "conv")
            if ep.fuse.acc_mode == 4:  # the statistics read z at every output (folded: the unpadded grid)
                _need(ep.bn_z, ny if nz is None else nz, "conv bn_z", dtype=y.dtype)
        elif out16 and ep.bn_z is not None:
            raise ValueError("conv: a bf16 output takes accumulator statistics only")
        if ep.pre is not None:
            ep.pre.check(g, ep.x_bf16)
    check(_timed("conv", g, "cgan3d_conv3d_fwd", ctypes.byref(g), ptr(x), ptr(w), ptr(y),
                 ctypes.byref(ep.c()) if ep is not None else None), "conv3d_fwd")


def wgrad_ws_floats(g: ConvGeom) -> int:
    return int(L.load().cgan3d_conv3d_wgrad_ws_floats(ctypes.byref(g)))


def wgrad_ws_atomic(g: ConvGeom) -> bool:
    """True if the weight gradient of ``g`` sums into its workspace by atomics (it may then take a
    clean workspace: ``wgrad(..., ws_clean=True)``)."""
    r = int(L.load().cgan3d_conv3d_wgrad_ws_mode(ctypes.byref(g)))
    if r < 0:
        raise ValueError("wgrad_ws_atomic: invalid geometry")
    return bool(r)


def zero(t: torch.Tensor):
    """Zero a contiguous device tensor (a memset recorded in launch plans)."""
    if not t.is_contiguous():
        raise ValueError("zero: tensor must be contiguous")
    check(_launch("cgan3d_zero", ptr(t), t.numel() * t.element_size()), "zero")


def copy_multi(pairs):
    """``dst.copy_(src)`` for each (src, dst) pair of contiguous device tensors with the same byte
    size, in one launch (include/cgan3d.h cgan3d_copy_multi; at most 8 pairs, no dtype conversion:
    the bytes are copied)."""
    if not 0 < len(pairs) <= 8:
        raise ValueError("copy_multi: 1..8 pairs")
    for s, d in pairs:
        if not (s.is_contiguous() and d.is_contiguous()):
            raise ValueError("copy_multi: operands must be contiguous")
        if s.numel() * s.element_size() != d.numel() * d.element_size():
            raise ValueError("copy_multi: byte sizes differ")
    n = len(pairs)
    src = (ctypes.c_void_p * n)(*[s.data_ptr() for s, _ in pairs])
    dst = (ctypes.c_void_p * n)(*[d.data_ptr() for _, d in pairs])
    nb = (ctypes.c_int64 * n)(*[s.numel() * s.element_size() for s, _ in pairs])
    check(_launch("cgan3d_copy_multi", src, dst, nb, n), "copy_multi")


def shadow_only(g: ConvGeom, role: int) -> bool:
    """True if, given bf16 shadows, the kernel ``g`` dispatches to reads only them (role 0: conv
    input via ``epilogue(x_bf16=...)``; role 1: weight-gradient operands) — cgan3d_conv3d_shadow_only."""
    return bool(L.load().cgan3d_conv3d_shadow_only(ctypes.byref(g), int(role)))


def bn_fold_ok(g: ConvGeom) -> bool:
    """True if ``g``'s launch takes ``epilogue(bn_fold=...)`` (cgan3d_conv3d_bn_fold_ok)."""
    return bool(L.load().cgan3d_conv3d_bn_fold_ok(ctypes.byref(g)))


def wgrad(g: ConvGeom, gathered, aligned, dw, ws, accumulate=False, gathered16=None, aligned16=None,
          ws_clean=False, defer_unpack=False, defer_reduce=False):
    """Weight gradient; ``gathered16`` / ``aligned16``: optional bf16 shadows of the operands.
    ``ws_clean``: ``ws`` is all-zero and is left all-zero (geometries with ``wgrad_ws_atomic``).
    ``defer_unpack`` (with ``ws_clean``): the result stays in ``ws`` until an ``UnpackSet`` run.
    ``defer_reduce`` (geometries with ``wgrad_partials``): the partials stay in ``ws`` until a
    ``reduce_multi`` launch sums them into ``dw``."""
    if defer_unpack and not ws_clean:
        raise ValueError("wgrad: defer_unpack needs ws_clean")
    if defer_reduce and wgrad_partials(g) <= 0:
        raise ValueError("wgrad: defer_reduce on a geometry without partials")
    _need(gathered, _vox_in(g) * g.cin, "wgrad gathered")
    _need(aligned, _vox_out(g) * g.cout, "wgrad aligned")
    _need(dw, g.cin * g.cout * taps(g), "wgrad dw")
    if _w_extent(g) > dw.numel():
        raise ValueError("wgrad: weight strides exceed dw")
    _need(ws, wgrad_ws_floats(g), "wgrad ws", exact=False)
    flags = ((L.WGRAD_ACCUMULATE if accumulate else 0) | (L.WGRAD_WS_CLEAN if ws_clean else 0)
             | (L.WGRAD_DEFER_UNPACK if defer_unpack else 0) | (L.WGRAD_DEFER_REDUCE if defer_reduce else 0))
    check(_timed("wgrad", g, "cgan3d_conv3d_wgrad_ex", ctypes.byref(g), ptr(gathered), ptr(aligned), ptr(dw),
                 flags, ptr(ws), _need16(gathered16, _vox_in(g) * g.cin, "wgrad gathered16"),
                 _need16(aligned16, _vox_out(g) * g.cout, "wgrad aligned16")), "conv3d_wgrad")


def wgrad_partials(g: ConvGeom) -> int:
    """Per-block partial sums the weight gradient of ``g`` reduces (0: it sums another way)."""
    return int(L.load().cgan3d_conv3d_wgrad_partials(ctypes.byref(g)))


def reduce_multi(items):
    """Deferred weight-gradient reduces in one launch (cgan3d_wgrad_reduce_multi): ``items`` =
    [(g, ws, dw, accumulate)] as left by ``wgrad(..., defer_reduce=True)``."""
    if not 0 < len(items) <= 16:
        raise ValueError("reduce_multi: 1..16 items")
    descs = (L.ReduceDesc * len(items))()
    for d, (g, ws, dw, acc) in zip(descs, items):
        P = wgrad_partials(g)
        if P <= 0:
            raise ValueError("reduce_multi: geometry without partials")
        _need(ws, P * 27 * g.cin * g.cout, "reduce_multi ws", exact=False)
        _need(dw, g.cin * g.cout * taps(g), "reduce_multi dw")
        d.ws, d.dw, d.sa, d.sb = ptr(ws), ptr(dw), g.w_sa, g.w_sb
        d.P, d.cin, d.cout, d.accumulate = P, g.cin, g.cout, int(acc)
    check(_launch("cgan3d_wgrad_reduce_multi", ctypes.cast(descs, ctypes.c_void_p), len(items)), "wgrad_reduce_multi")


def wgrad_group_ok(g: ConvGeom) -> bool:
    """True if ``g``'s weight gradient can join a ``wgrad_group`` launch."""
    return bool(L.load().cgan3d_conv3d_wgrad_group_ok(ctypes.byref(g)))


def wgrad_group(items):
    """Several weight gradients in one launch (cgan3d_conv3d_wgrad_group): ``items`` = [(g, gathered,
    aligned, ws)], each ``ws`` an all-zero workspace the result is added into, as ``wgrad(...,
    accumulate=True, ws_clean=True, defer_unpack=True)`` — moved into dW by an ``UnpackSet`` run."""
    if not 0 < len(items) <= 4:
        raise ValueError("wgrad_group: 1..4 items")
    for g, a, b, ws in items:
        if not wgrad_group_ok(g):
            raise ValueError("wgrad_group: geometry not eligible (cgan3d_conv3d_wgrad_group_ok)")
        _need(a, _vox_in(g) * g.cin, "wgrad_group gathered")
        _need(b, _vox_out(g) * g.cout, "wgrad_group aligned")
        _need(ws, wgrad_ws_floats(g), "wgrad_group ws", exact=False)
    n = len(items)
    geoms = (ConvGeom * n)(*[g for g, _, _, _ in items])
    ga = (ctypes.c_void_p * n)(*[a.data_ptr() for _, a, _, _ in items])
    al = (ctypes.c_void_p * n)(*[b.data_ptr() for _, _, b, _ in items])
    wss = (ctypes.c_void_p * n)(*[w.data_ptr() for _, _, _, w in items])
    check(_launch("cgan3d_conv3d_wgrad_group", geoms, ga, al, wss, n), "wgrad_group")


def wgrad_sk_ok(g: ConvGeom) -> bool:
    """True if ``g``'s weight gradient can run on the staged-window critic kernel (``wgrad_sk``)."""
    return bool(L.load().cgan3d_conv3d_wgrad_sk_ok(ctypes.byref(g)))


def wgrad_sk_ws_floats(g: ConvGeom) -> int:
    return int(L.load().cgan3d_conv3d_wgrad_sk_ws_floats(ctypes.byref(g)))


def wgrad_sk(items):
    """The critic's k4 s2 middle-layer weight gradients (cgan3d_conv3d_wgrad_sk): ``items`` = [(g,
    gathered, aligned, ws, dw)]; per-block partials into ``ws`` (any contents), then their sums ADDED
    into ``dw`` (torch layout).  Two launches for up to four layers."""
    if not 0 < len(items) <= 4:
        raise ValueError("wgrad_sk: 1..4 items")
    for g, a, b, ws, dw in items:
        if not wgrad_sk_ok(g):
            raise ValueError("wgrad_sk: geometry not eligible (cgan3d_conv3d_wgrad_sk_ok)")
        _need(a, _vox_in(g) * g.cin, "wgrad_sk gathered")
        _need(b, _vox_out(g) * g.cout, "wgrad_sk aligned")
        _need(ws, wgrad_sk_ws_floats(g), "wgrad_sk ws", exact=False)
        _need(dw, g.cin * g.cout * taps(g), "wgrad_sk dw")
        for t, nm in ((a, "gathered"), (b, "aligned"), (ws, "ws")):
            if t.data_ptr() % 16:
                raise ValueError(f"wgrad_sk: {nm} must be 16-byte aligned")
    n = len(items)
    geoms = (ConvGeom * n)(*[it[0] for it in items])
    arr = [(ctypes.c_void_p * n)(*[it[k].data_ptr() for it in items]) for k in (1, 2, 3, 4)]
    check(_launch("cgan3d_conv3d_wgrad_sk", geoms, *arr, n), "wgrad_sk")


def bn_finalize(stats, nblk, c, gamma, beta, rmean, rvar, nbt, scale_shift, mean_invstd, momentum=0.1, eps=1e-5):
    _need(stats, nblk * (2 * c + 1), "bn_finalize stats", exact=False)
    for t, nm in ((gamma, "gamma"), (beta, "beta"), (rmean, "running_mean"), (rvar, "running_var")):
        _need(t, c, f"bn_finalize {nm}")
    _need(nbt, 1, "bn_finalize num_batches_tracked", dtype=torch.int64)
    _need(scale_shift, 2 * c, "bn_finalize scale_shift")
    _need(mean_invstd, 2 * c, "bn_finalize mean_invstd")
    check(_launch("cgan3d_bn_finalize", ptr(stats), nblk, c, ptr(gamma), ptr(beta), ptr(rmean), ptr(rvar), ptr(nbt),
                  momentum, eps, ptr(scale_shift), ptr(mean_invstd)), "bn_finalize")


def _need16(t, n, what):
    if t is not None:
        _need(t, n, what, dtype=torch.bfloat16)
    return ptr(t)


def bn_apply(z, nvox, c, scale_shift, act, y, residual=None, slope=0.0, y16=None):
    _need(z, nvox * c, "bn_apply z")
    _need(y, nvox * c, "bn_apply y")
    _need(scale_shift, 2 * c, "bn_apply scale_shift")
    if residual is not None:
        _need(residual, nvox * c, "bn_apply residual")
    check(_launch("cgan3d_bn_apply", ptr(z), nvox, c, ptr(scale_shift), act, slope, ptr(residual), ptr(y),
                  _need16(y16, nvox * c, "bn_apply y16")), "bn_apply")


def bn_slots(g: ConvGeom) -> int:
    """Slots of the fused BatchNorm slab of a conv launch (0: the kernel has no fused statistics)."""
    return int(L.load().cgan3d_conv3d_bn_slots(ctypes.byref(g)))


def reflect_fold_slots(n, dims: Sequence[int], c) -> int:
    return int(L.load().cgan3d_reflect_fold_slots(n, *dims, c))


def bn_finalize_slab(part, nslots, c, nvox, gamma, beta, rmean, rvar, nbt, scale_shift, mean_invstd, momentum=0.1,
                     eps=1e-5, _checks_only=False):
    """BatchNorm forward statistics from a mode-1 slab (the producing conv's per-block partials)."""
    _need(part, (2 * c + 1) * nslots, "bn_finalize_slab part", exact=False)
    for t, nm in ((gamma, "gamma"), (beta, "beta")):
        _need(t, c, f"bn_finalize_slab {nm}")
    for t, nm in ((rmean, "running_mean"), (rvar, "running_var")):
        if t is not None:
            _need(t, c, f"bn_finalize_slab {nm}")
    if nbt is not None:
        _need(nbt, 1, "bn_finalize_slab num_batches_tracked", dtype=torch.int64)
    _need(scale_shift, 2 * c, "bn_finalize_slab scale_shift")
    _need(mean_invstd, 2 * c, "bn_finalize_slab mean_invstd")
    if _checks_only:
        return
    check(_launch("cgan3d_bn_finalize_slab", ptr(part), nslots, c, nvox, ptr(gamma), ptr(beta), ptr(rmean), ptr(rvar),
                  ptr(nbt), momentum, eps, ptr(scale_shift), ptr(mean_invstd)), "bn_finalize_slab")


def _need_ticket(t, what):
    if t.dtype != torch.int32 or t.numel() < 2 or not t.is_contiguous():
        raise ValueError(f"{what}: ticket must be >= 2 contiguous int32 words (zeroed once)")
    if t.device.type != "cuda" and not DRY_RUN:
        raise ValueError(f"{what}: ticket must be a device tensor")


def tickets(n: int, device) -> torch.Tensor:
    """``n`` launch tickets (2 zeroed int32 words each, left zeroed by every launch); ``tickets(n)[i]``."""
    return torch.zeros((n, 2), dtype=torch.int32, device=device)


def bn_apply_slab(part, nslots, c, nvox, gamma, beta, rmean, rvar, nbt, scale_shift, mean_invstd, z, act, y,
                  residual=None, slope=0.0, momentum=0.1, eps=1e-5, y16=None):
    """``bn_finalize_slab`` + ``bn_apply`` (one launch when the slab is small)."""
    bn_finalize_slab(part, nslots, c, nvox, gamma, beta, rmean, rvar, nbt, scale_shift, mean_invstd, momentum, eps,
                     _checks_only=True)
    _need(z, nvox * c, "bn_apply_slab z")
    if y is None and y16 is None:
        raise ValueError("bn_apply_slab: y may be None only when y16 is given")
    if y is not None:
        _need(y, nvox * c, "bn_apply_slab y")
    if residual is not None:
        _need(residual, nvox * c, "bn_apply_slab residual")
    check(_launch("cgan3d_bn_apply_slab", ptr(part), nslots, c, nvox, ptr(gamma), ptr(beta), ptr(rmean), ptr(rvar),
                  ptr(nbt), momentum, eps, ptr(scale_shift), ptr(mean_invstd), ptr(z), act, float(slope),
                  ptr(residual), ptr(y), _need16(y16, nvox * c, "bn_apply_slab y16")), "bn_apply_slab")


def bn_backward_slab(dy, z, nvox, c, part, nslots, scale_shift, mean_invstd, gamma, act, dgamma, dbeta, dz, ws,
                     slope=0.0, accumulate=False, dz16=None):
    """BatchNorm backward from a mode-2 slab (written by the kernel that produced dy)."""
    if dz is None and dz16 is None:
        raise ValueError("bn_backward_slab: dz may be None only when dz16 is given")
    for t, nm in ((dy, "dy"), (z, "z"), (dz, "dz")):
        if t is not None:
            _need(t, nvox * c, f"bn_backward_slab {nm}")
    _need(part, 2 * c * nslots, "bn_backward_slab part", exact=False)
    for t, nm in ((scale_shift, "scale_shift"), (mean_invstd, "mean_invstd")):
        _need(t, 2 * c, f"bn_backward_slab {nm}")
    for t, nm in ((gamma, "gamma"), (dgamma, "dgamma"), (dbeta, "dbeta")):
        _need(t, c, f"bn_backward_slab {nm}")
    _need(ws, 3 * c, "bn_backward_slab ws", exact=False)
    check(_launch("cgan3d_bn_backward_slab", ptr(dy), ptr(z), nvox, c, ptr(part), nslots, ptr(scale_shift),
                  ptr(mean_invstd), ptr(gamma), act, slope, ptr(dgamma), ptr(dbeta), ptr(dz), int(accumulate),
                  ptr(ws), _need16(dz16, nvox * c, "bn_backward_slab dz16")), "bn_backward_slab")


def bn_apply_acc(acc, reps, c, nvox, gamma, beta, rmean, rvar, nbt, scale_shift, mean_invstd, z, act, y,
                 residual=None, slope=0.0, momentum=0.1, eps=1e-5, y16=None, zero=None):
    """BatchNorm train forward + act (+ residual) from the producing conv's fp64 accumulators
    (cgan3d_bn_apply_acc: finalize and elementwise pass in one launch; ``zero``: a float64 tensor
    block 0 zeroes first)."""
    _need(acc, reps * 2 * c, "bn_apply_acc acc", dtype=torch.float64, exact=False)
    for t, nm in ((gamma, "gamma"), (beta, "beta")):
        _need(t, c, f"bn_apply_acc {nm}")
    for t, nm in ((scale_shift, "scale_shift"), (mean_invstd, "mean_invstd")):
        _need(t, 2 * c, f"bn_apply_acc {nm}")
    z16 = z.dtype == torch.bfloat16  # z kept in bf16 by its producer (include/cgan3d.h in_bf16)
    _need(z, nvox * c, "bn_apply_acc z", dtype=z.dtype if z16 else torch.float32)
    if y is None and y16 is None:
        raise ValueError("bn_apply_acc: y may be None only when y16 is given")
    for t, nm in ((y, "y"), (residual, "residual")):
        if t is not None:
            _need(t, nvox * c, f"bn_apply_acc {nm}")
    if zero is not None:
        _need(zero, zero.numel(), "bn_apply_acc zero", dtype=torch.float64)
    check(_launch("cgan3d_bn_apply_acc", ptr(acc), reps, c, nvox, ptr(gamma), ptr(beta), ptr(rmean), ptr(rvar),
                  ptr(nbt), momentum, eps, ptr(scale_shift), ptr(mean_invstd), ptr(z), act, float(slope),
                  ptr(residual), ptr(y), _need16(y16, nvox * c, "bn_apply_acc y16"), ptr(zero),
                  zero.numel() if zero is not None else 0, int(z16)), "bn_apply_acc")


def bn_backward_acc(dy, z, nvox, c, acc, reps, scale_shift, mean_invstd, gamma, act, dgamma, dbeta, dz, slope=0.0,
                    accumulate=False, dz16=None, zero=None):
    """BatchNorm backward from the fp64 accumulators the kernel that produced dy filled
    (cgan3d_bn_backward_acc: one launch)."""
    if dz is None and dz16 is None:
        raise ValueError("bn_backward_acc: dz may be None only when dz16 is given")
    in16 = dy.dtype == torch.bfloat16  # dy and z kept in bf16 by their producers (include/cgan3d.h in_bf16)
    for t, nm in ((dy, "dy"), (z, "z")):
        _need(t, nvox * c, f"bn_backward_acc {nm}", dtype=torch.bfloat16 if in16 else torch.float32)
    if dz is not None:
        _need(dz, nvox * c, "bn_backward_acc dz")
    _need(acc, reps * 2 * c, "bn_backward_acc acc", dtype=torch.float64, exact=False)
    for t, nm in ((scale_shift, "scale_shift"), (mean_invstd, "mean_invstd")):
        _need(t, 2 * c, f"bn_backward_acc {nm}")
    for t, nm in ((gamma, "gamma"), (dgamma, "dgamma"), (dbeta, "dbeta")):
        _need(t, c, f"bn_backward_acc {nm}")
    if zero is not None:
        _need(zero, zero.numel(), "bn_backward_acc zero", dtype=torch.float64)
    check(_launch("cgan3d_bn_backward_acc", ptr(dy), ptr(z), nvox, c, ptr(acc), reps, ptr(scale_shift),
                  ptr(mean_invstd), ptr(gamma), act, slope, ptr(dgamma), ptr(dbeta), ptr(dz), int(accumulate),
                  _need16(dz16, nvox * c, "bn_backward_acc dz16"), ptr(zero), zero.numel() if zero is not None else 0,
                  int(in16)), "bn_backward_acc")


def bn_backward_acc_fold(padded, z, n, dims: Sequence[int], c, pad, acc, reps, scale_shift, mean_invstd, gamma,
                         act, dgamma, dbeta, dz, slope=0.0, accumulate=False, dz16=None, zero=None):
    """``bn_backward_slab_fold`` with the statistics from the fp64 accumulators of the last conv's
    input-grad launch (cgan3d_bn_backward_acc_fold: one launch)."""
    d, h, w = dims
    nvox = n * d * h * w
    in16 = padded.dtype == torch.bfloat16  # padded and z kept in bf16 (include/cgan3d.h in_bf16)
    dt = torch.bfloat16 if in16 else torch.float32
    _need(padded, n * (d + 2 * pad) * (h + 2 * pad) * (w + 2 * pad) * c, "bn_backward_acc_fold padded", dtype=dt)
    if dz is None and dz16 is None:
        raise ValueError("bn_backward_acc_fold: dz may be None only when dz16 is given")
    _need(z, nvox * c, "bn_backward_acc_fold z", dtype=dt)
    if dz is not None:
        _need(dz, nvox * c, "bn_backward_acc_fold dz")
    _need(acc, reps * 2 * c, "bn_backward_acc_fold acc", dtype=torch.float64, exact=False)
    for t, nm in ((scale_shift, "scale_shift"), (mean_invstd, "mean_invstd")):
        _need(t, 2 * c, f"bn_backward_acc_fold {nm}")
    for t, nm in ((gamma, "gamma"), (dgamma, "dgamma"), (dbeta, "dbeta")):
        _need(t, c, f"bn_backward_acc_fold {nm}")
    if zero is not None:
        _need(zero, zero.numel(), "bn_backward_acc_fold zero", dtype=torch.float64)
    check(_launch("cgan3d_bn_backward_acc_fold", ptr(padded), ptr(z), n, d, h, w, c, pad, ptr(acc), reps,
                  ptr(scale_shift), ptr(mean_invstd), ptr(gamma), act, slope, ptr(dgamma), ptr(dbeta), ptr(dz),
                  int(accumulate), _need16(dz16, nvox * c, "bn_backward_acc_fold dz16"), ptr(zero),
                  zero.numel() if zero is not None else 0, int(in16)), "bn_backward_acc_fold")


def bn_backward_slab_fold(padded, z, n, dims: Sequence[int], c, pad, part, nslots, scale_shift, mean_invstd, gamma,
                          act, dgamma, dbeta, dz, ws, slope=0.0, accumulate=False, dz16=None):
    """``bn_backward_slab`` with dy = reflect_fold(padded) folded on the fly (cgan3d_bn_backward_slab_fold)."""
    d, h, w = dims
    nvox = n * d * h * w
    _need(padded, n * (d + 2 * pad) * (h + 2 * pad) * (w + 2 * pad) * c, "bn_backward_slab_fold padded")
    if dz is None and dz16 is None:
        raise ValueError("bn_backward_slab_fold: dz may be None only when dz16 is given")
    for t, nm in ((z, "z"), (dz, "dz")):
        if t is not None:
            _need(t, nvox * c, f"bn_backward_slab_fold {nm}")
    _need(part, 2 * c * nslots, "bn_backward_slab_fold part", exact=False)
    for t, nm in ((scale_shift, "scale_shift"), (mean_invstd, "mean_invstd")):
        _need(t, 2 * c, f"bn_backward_slab_fold {nm}")
    for t, nm in ((gamma, "gamma"), (dgamma, "dgamma"), (dbeta, "dbeta")):
        _need(t, c, f"bn_backward_slab_fold {nm}")
    _need(ws, 3 * c, "bn_backward_slab_fold ws", exact=False)
    check(_launch("cgan3d_bn_backward_slab_fold", ptr(padded), ptr(z), n, d, h, w, c, pad, ptr(part), nslots,
                  ptr(scale_shift), ptr(mean_invstd), ptr(gamma), act, float(slope), ptr(dgamma), ptr(dbeta), ptr(dz),
                  int(accumulate), ptr(ws), _need16(dz16, nvox * c, "bn_backward_slab_fold dz16")),
          "bn_backward_slab_fold")


def bn_backward_ws_floats(nvox, c) -> int:
    return int(L.load().cgan3d_bn_backward_ws_floats(nvox, c))


def bn_backward(dy, z, nvox, c, scale_shift, mean_invstd, gamma, act, dgamma, dbeta, dz, ws, slope=0.0,
                accumulate=False):
    for t, nm in ((dy, "dy"), (z, "z"), (dz, "dz")):
        _need(t, nvox * c, f"bn_backward {nm}")
    for t, nm in ((scale_shift, "scale_shift"), (mean_invstd, "mean_invstd")):
        _need(t, 2 * c, f"bn_backward {nm}")
    for t, nm in ((gamma, "gamma"), (dgamma, "dgamma"), (dbeta, "dbeta")):
        _need(t, c, f"bn_backward {nm}")
    _need(ws, bn_backward_ws_floats(nvox, c), "bn_backward ws", exact=False)
    check(_launch("cgan3d_bn_backward", ptr(dy), ptr(z), nvox, c, ptr(scale_shift), ptr(mean_invstd), ptr(gamma),
                  act, slope, ptr(dgamma), ptr(dbeta), ptr(dz), int(accumulate), ptr(ws)), "bn_backward")


def channel_sum_ws_floats(nvox, c) -> int:
    return int(L.load().cgan3d_channel_sum_ws_floats(nvox, c))


def channel_sum(x, nvox, c, out, ws):
    _need(x, nvox * c, "channel_sum x")
    _need(out, c, "channel_sum out")
    _need(ws, channel_sum_ws_floats(nvox, c), "channel_sum ws", exact=False)
    check(_launch("cgan3d_channel_sum", ptr(x), nvox, c, ptr(out), ptr(ws)), "channel_sum")


class UnpackSet:
    """Several deferred weight gradients (``wgrad(..., defer_unpack=True)``) moved from their packed
    workspaces into dW in one launch (cgan3d_wgrad_unpack_multi), the workspaces re-zeroed.  Built
    once per (workspaces, gradient views); the descriptors live on the device."""

    def __init__(self, device, items):
        """items: [(geometry, ws, dw, accumulate)]; every ws / dw keeps its address."""
        descs, self.keep = [], []
        for g, ws, dw, acc in items:
            t = taps(g)
            _need(ws, t * g.cin * g.cout, "UnpackSet ws", exact=False)
            _need(dw, g.cin * g.cout * t, "UnpackSet dw")
            d = L.UnpackDesc()
            d.ws, d.dw, d.sa, d.sb = ptr(ws), ptr(dw), g.w_sa, g.w_sb
            d.taps, d.cin, d.cout, d.accumulate = t, g.cin, g.cout, int(acc)
            descs.append(d)
            self.keep += [ws, dw]
        self.n = len(descs)
        self.max_total = max(taps(g) * g.cin * g.cout for g, _, _, _ in items)
        self.dev = torch.frombuffer(bytearray(b"".join(bytes(d) for d in descs)), dtype=torch.uint8).to(device)

    def run(self):
        check(_launch("cgan3d_wgrad_unpack_multi", ptr(self.dev), self.n, self.max_total), "wgrad_unpack_multi")


class ChannelSumSet:
    """Per-channel sums of several tensors in two launches (cgan3d_channel_sum_multi): the critic's
    bias gradients.  Built once per (tensors, sizes); the descriptors live on the device."""

    def __init__(self, device, items, nblk: int = 0):
        """items: [(x, nvox, c, out, accumulate)]; every x / out keeps its address.  ``nblk``
        (partial sums per tensor): by default ~16 float4-rows of work per thread of the largest."""
        if nblk <= 0:
            big = max(nvox * c for _, nvox, c, _, _ in items)
            nblk = max(1, min(1024, -(-big // (256 * 16))))
        self.nblk, self.keep = nblk, []
        descs = []
        for x, nvox, c, out, acc in items:
            if c <= 0 or 256 % c:
                raise ValueError(f"ChannelSumSet: channels {c} must divide 256")
            _need(x, nvox * c, "channel_sum_multi x", exact=False)
            _need(out, c, "channel_sum_multi out")
            ws = torch.empty(nblk * c, device=device, dtype=torch.float64)
            d = L.CsumDesc()
            d.x, d.out, d.ws, d.nvox, d.c, d.accumulate = ptr(x), ptr(out), ptr(ws), nvox, c, int(acc)
            descs.append(d)
            self.keep += [x, out, ws]
        self.n = len(descs)
        self.cmax = max(c for _, _, c, _, _ in items)
        raw = b"".join(bytes(d) for d in descs)
        self.dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(device)

    def run(self):
        check(_launch("cgan3d_channel_sum_multi", ptr(self.dev), self.n, self.nblk, self.cmax), "channel_sum_multi")


def ln_partial_doubles(n: int, L_: int) -> int:
    return int(L.load().cgan3d_ln_partial_doubles(n, L_))


def _ln_args(mode, n, L_, slope, z, p_stats, da=None, zdot=None, adot=None, abar=None, p_bwd=None, p_jvp=None,
             p_sig=None, p_adj=None):
    for t, nm in ((z, "z"), (da, "da"), (zdot, "zdot"), (adot, "adot"), (abar, "abar")):
        if t is not None:
            _need(t, n * L_, f"ln {nm}", exact=False)
    npart = ln_partial_doubles(n, L_)
    for t, nm in ((p_stats, "p_stats"), (p_bwd, "p_bwd"), (p_jvp, "p_jvp"), (p_sig, "p_sig"), (p_adj, "p_adj")):
        if t is not None:
            _need(t, npart, f"ln {nm}", dtype=torch.float64, exact=False)
    a = L.LnArgs()
    a.n, a.mode, a.L, a.slope, a.eps = n, mode, L_, slope, 1e-5
    a.z, a.da, a.zdot, a.adot, a.abar = ptr(z), ptr(da), ptr(zdot), ptr(adot), ptr(abar)
    a.p_stats, a.p_bwd, a.p_jvp, a.p_sig, a.p_adj = ptr(p_stats), ptr(p_bwd), ptr(p_jvp), ptr(p_sig), ptr(p_adj)
    return a


def ln_reduce(mode, n, L_, slope, part, **kw):
    """Per-sample partial sums of a LayerNorm mode (cgan3d_ln_reduce; modes L.LN_*)."""
    a = _ln_args(mode, n, L_, slope, **kw)
    _need(part, ln_partial_doubles(n, L_), "ln_reduce part", dtype=torch.float64, exact=False)
    check(_launch("cgan3d_ln_reduce", ctypes.byref(a), ptr(part)), "ln_reduce")


def ln_apply(mode, n, L_, slope, out, **kw):
    """Elementwise LayerNorm pass of a mode from its partials (cgan3d_ln_apply)."""
    a = _ln_args(mode, n, L_, slope, **kw)
    _need(out, n * L_, "ln_apply out", exact=False)
    check(_launch("cgan3d_ln_apply", ctypes.byref(a), ptr(out)), "ln_apply")


def reflect_fold(padded, out, n, dims: Sequence[int], c, pad, ep: Optional[Epi] = None, planar: bool = False):
    """Adjoint of reflection padding; ``ep.bn_gsum`` adds the fused BatchNorm backward statistics.
    ``planar``: dims (1, H, W) of the 2-D variants, padded in H and W only."""
    d, h, w = dims
    if planar:
        if d != 1:
            raise ValueError("reflect_fold: planar dims must be (1, H, W)")
        _need(padded, n * (h + 2 * pad) * (w + 2 * pad) * c, "reflect_fold2d padded")
        _need(out, n * h * w * c, "reflect_fold2d out")
        if ep is not None and ep.bn_mode:
            if ep.bn_slots != reflect_fold_slots(n, dims, c):
                raise ValueError("reflect_fold: bn_slots != reflect_fold_slots()")
            ep.check_bn(n * h * w * c, c, "reflect_fold2d")
        check(_launch("cgan3d_reflect_fold2d", ptr(padded), ptr(out), n, h, w, c, pad,
                      ctypes.byref(ep.c()) if ep is not None else None), "reflect_fold2d")
        return
    _need(padded, n * (d + 2 * pad) * (h + 2 * pad) * (w + 2 * pad) * c, "reflect_fold padded")
    _need(out, n * d * h * w * c, "reflect_fold out")
    if ep is None:
        check(_launch("cgan3d_reflect_fold", ptr(padded), ptr(out), n, d, h, w, c, pad), "reflect_fold")
        return
    if ep.bn_mode and ep.bn_slots != reflect_fold_slots(n, dims, c):
        raise ValueError("reflect_fold: bn_slots != reflect_fold_slots()")
    ep.check_bn(n * d * h * w * c, c, "reflect_fold")
    check(_launch("cgan3d_reflect_fold_ex", ptr(padded), ptr(out), n, d, h, w, c, pad, ctypes.byref(ep.c())),
          "reflect_fold_ex")


def gp_interpolate(real, fake, eps, out, b, per_sample, idx=None):
    """out = eps * real + (1 - eps) * fake per sample; ``idx`` (device int32 [2 b]): rows of ``real`` /
    ``fake`` resampled by the host when their batch sizes differ (model/utils.py:21-25)."""
    _need(out, b * per_sample, "gp_interpolate out")
    _need(eps, b, "gp_interpolate eps")
    if idx is None:
        for t, nm in ((real, "real"), (fake, "fake")):
            _need(t, b * per_sample, f"gp_interpolate {nm}")
        check(_launch("cgan3d_gp_interpolate", ptr(real), ptr(fake), ptr(eps), ptr(out), b, per_sample),
              "gp_interpolate")
        return
    if idx.dtype != torch.int32 or idx.numel() != 2 * b or not idx.is_contiguous():
        raise ValueError("gp_interpolate: idx must be contiguous int32 [2 b]")
    if real.numel() % per_sample or fake.numel() % per_sample:
        raise ValueError("gp_interpolate: real / fake must hold whole samples")
    # the rows in idx are range-checked by whoever writes them (StepEngine.set_gp_indices), on the host,
    # and clamped to the two batches' row counts in the kernel
    check(_launch("cgan3d_gp_interpolate_idx", ptr(real), ptr(fake), ptr(idx), ptr(eps), ptr(out), b, per_sample,
                  real.numel() // per_sample, fake.numel() // per_sample), "gp_interpolate_idx")


def tanh_backward(y, dy, dz):
    _need(dy, y.numel(), "tanh_backward dy")
    _need(dz, y.numel(), "tanh_backward dz")
    check(_launch("cgan3d_tanh_backward", ptr(y), ptr(dy), ptr(dz), y.numel()), "tanh_backward")


def loss_ws_floats() -> int:
    return int(L.load().cgan3d_loss_ws_floats(0))


def critic_logits_grad(logits, n_real, n_fake, n_gp, per_sample, gan_w, dlogits, losses):
    n = (n_real + n_fake + n_gp) * per_sample
    _need(logits, n, "critic_logits_grad logits", exact=False)
    _need(dlogits, n, "critic_logits_grad dlogits", exact=False)
    _need(losses, 8, "losses")
    check(_launch("cgan3d_critic_logits_grad", ptr(logits), n_real, n_fake, n_gp, per_sample, gan_w, ptr(dlogits),
                  ptr(losses)), "critic_logits_grad")


def gradient_penalty(grad, b, per_sample, lambda_, gamma_out, losses, ws):
    _need(grad, b * per_sample, "gradient_penalty grad")
    _need(gamma_out, b * per_sample, "gradient_penalty gamma")
    _need(losses, 8, "losses")
    _need(ws, loss_ws_floats(), "gradient_penalty ws", exact=False)
    check(_launch("cgan3d_gradient_penalty", ptr(grad), b, per_sample, lambda_, ptr(gamma_out), ptr(losses),
                  ptr(ws)), "gradient_penalty")


def gradient_penalty_part(grad, part, b, chunks, per_sample, lambda_, gamma_out, losses, logits=None, n_real=0,
                          n_fake=0, logit_ps=0, gan_w=0.0, zero=None):
    """cgan3d_gradient_penalty_part: the GP from per-sample partial sums of squares part[b][chunks]
    (and, given the critic's logits, the Wasserstein term and critic loss in the same launch;
    given `zero`, fp32 zeros written over it by the same launch)."""
    _need(grad, b * per_sample, "gradient_penalty_part grad")
    _need(part, b * chunks, "gradient_penalty_part part", exact=False)
    _need(gamma_out, b * per_sample, "gradient_penalty_part gamma")
    _need(losses, 8, "losses")
    if logits is not None:
        _need(logits, (n_real + n_fake) * logit_ps, "gradient_penalty_part logits", exact=False)
    if zero is not None:
        _need(zero, zero.numel(), "gradient_penalty_part zero")
    check(_launch("cgan3d_gradient_penalty_part", ptr(grad), ptr(part), b, chunks, per_sample, lambda_,
                  ptr(gamma_out), ptr(losses), ptr(logits), n_real, n_fake, logit_ps, gan_w, ptr(zero),
                  0 if zero is None else zero.numel()), "gradient_penalty_part")


def sumsq_blocks(g) -> int:
    """cgan3d_conv3d_sumsq_blocks: per-block sum-of-squares slots of an input-grad launch (0: none)."""
    return int(L.load().cgan3d_conv3d_sumsq_blocks(ctypes.byref(g)))


def generator_logits_grad(logits, n, gan_w, dlogits, losses):
    """dlogits None: the generator's adversarial loss only (constant dlogits kept by the caller)."""
    _need(logits, n, "generator_logits_grad logits", exact=False)
    if dlogits is not None:
        _need(dlogits, n, "generator_logits_grad dlogits", exact=False)
    _need(losses, 8, "losses")
    check(_launch("cgan3d_generator_logits_grad", ptr(logits), n, gan_w, ptr(dlogits), ptr(losses)),
          "generator_logits_grad")


def generator_output_grad(opt_hat, subopt, att, mask_u8, d_critic, n, lo, hi, sim_w, hu_w, dz_last, losses, ws):
    for t, nm in ((opt_hat, "opt_hat"), (subopt, "subopt"), (att, "att"), (dz_last, "dz_last")):
        _need(t, n, f"generator_output_grad {nm}")
    _need(mask_u8, n, "generator_output_grad mask", dtype=torch.uint8)
    if d_critic is not None:
        _need(d_critic, n, "generator_output_grad d_critic")
    _need(losses, 8, "losses")
    _need(ws, loss_ws_floats(), "generator_output_grad ws", exact=False)
    check(_launch("cgan3d_generator_output_grad", ptr(opt_hat), ptr(subopt), ptr(att), ptr(mask_u8), ptr(d_critic),
                  n, lo, hi, sim_w, hu_w, ptr(dz_last), ptr(losses), ptr(ws)), "generator_output_grad")


def adam_tick(hyper):
    _need(hyper, 6, "adam hyper")
    check(_launch("cgan3d_adam_tick", ptr(hyper)), "adam_tick")


def adam(param, grad, exp_avg, exp_avg_sq, hyper):
    for t, nm in ((grad, "grad"), (exp_avg, "exp_avg"), (exp_avg_sq, "exp_avg_sq")):
        _need(t, param.numel(), f"adam {nm}")
    _need(hyper, 6, "adam hyper")
    check(_launch("cgan3d_adam", ptr(param), ptr(grad), ptr(exp_avg), ptr(exp_avg_sq), param.numel(), ptr(hyper)),
          "adam")


def adam_range(param, grad, exp_avg, exp_avg_sq, hyper):
    """cgan3d_adam_range: Adam over part of an arena with step + 1, the step counter left as it is."""
    for t, nm in ((grad, "grad"), (exp_avg, "exp_avg"), (exp_avg_sq, "exp_avg_sq")):
        _need(t, param.numel(), f"adam_range {nm}")
    _need(hyper, 6, "adam_range hyper")
    check(_launch("cgan3d_adam_range", ptr(param), ptr(grad), ptr(exp_avg), ptr(exp_avg_sq), param.numel(), ptr(hyper)),
          "adam_range")


def adam_pack(param, grad, exp_avg, exp_avg_sq, hyper, ticket, packs: Optional["PackSet"] = None):
    """``adam_tick`` + ``adam`` + ``packs.pack()`` as one launch (cgan3d_adam_pack); every packed
    copy's source weight must be a contiguous view into ``param``."""
    for t, nm in ((grad, "grad"), (exp_avg, "exp_avg"), (exp_avg_sq, "exp_avg_sq")):
        _need(t, param.numel(), f"adam_pack {nm}")
    _need(hyper, 6, "adam_pack hyper")
    _need_ticket(ticket, "adam_pack")
    nd = 0
    if packs is not None and packs.descs:
        lo, hi = param.data_ptr(), param.data_ptr() + 4 * param.numel()
        for _, _, w in packs.descs:
            if not (w.is_contiguous() and lo <= w.data_ptr() and w.data_ptr() + 4 * w.numel() <= hi):
                raise ValueError("adam_pack: a packed weight is not a contiguous view into the parameter arena")
        nd = len(packs.descs)
    check(_launch("cgan3d_adam_pack", ptr(param), ptr(grad), ptr(exp_avg), ptr(exp_avg_sq), param.numel(), ptr(hyper),
                  ptr(packs.device_descs()) if nd else None, nd, ptr(ticket)), "adam_pack")


def unpack_patches(src: torch.Tensor, data: torch.Tensor, seg: torch.Tensor, shift: float, factor: float):
    """src: device [..., 2] (HU, label) int16 or float32 -> data (float32) and seg (bool/uint8)."""
    if src.dtype not in (torch.int16, torch.float32):
        raise TypeError(f"unpack_patches: src dtype {src.dtype} (int16 or float32)")
    if not src.is_contiguous() or src.shape[-1] != 2:
        raise ValueError("unpack_patches: src must be contiguous [..., 2]")
    nvox = src.numel() // 2
    _need(data, nvox, "unpack_patches data")
    _need(seg, nvox, "unpack_patches seg", dtype=seg.dtype)
    if seg.dtype not in (torch.bool, torch.uint8):
        raise TypeError("unpack_patches: seg must be bool or uint8")
    check(_launch("cgan3d_unpack_patches", ptr(src), 0 if src.dtype == torch.int16 else 1, nvox, float(shift),
                  float(factor), ptr(data), ptr(seg)), "unpack_patches")


class MappedHost:
    """Pinned host memory mapped into the device's address space (include/cgan3d.h cgan3d_host_alloc):
    ``tensor`` is a CPU view the host fills, ``dev`` the address kernels read it at over PCIe
    (copy_multi_ex / unpack_patches_ex on a copy stream): a batch reaches HBM in one small launch
    instead of a host-blocking SDMA copy (tools/h2d_probe.py)."""

    def __init__(self, shape, dtype: torch.dtype):
        numel = 1
        for s in shape:
            numel *= int(s)
        item = torch.empty((), dtype=dtype).element_size()
        self.nbytes = max(16, (numel * item + 15) // 16 * 16)
        h, d = ctypes.c_void_p(), ctypes.c_void_p()
        check(L.lib().cgan3d_host_alloc(self.nbytes, ctypes.byref(h), ctypes.byref(d)), "host_alloc")
        self.host, self.dev = h.value, d.value
        self._buf = (ctypes.c_uint8 * self.nbytes).from_address(self.host)
        self.tensor = torch.frombuffer(self._buf, dtype=dtype, count=numel).view(tuple(int(s) for s in shape))
        self._lib = L.lib()

    def __del__(self):
        host, self.host = getattr(self, "host", None), None
        if host:
            self.tensor = self._buf = None
            self._lib.cgan3d_host_free(ctypes.c_void_p(host))


def copy_h2d(pairs, max_blocks: int = 32):
    """Copy each (MappedHost, contiguous device tensor of its byte size) pair on the current stream in one
    launch of at most ``max_blocks`` workgroups reading the host memory over PCIe (cgan3d_copy_multi_ex)."""
    if not 0 < len(pairs) <= 8:
        raise ValueError("copy_h2d: 1..8 pairs")
    for mh, d in pairs:
        nb = d.numel() * d.element_size()
        if not (d.is_cuda and d.is_contiguous()) or nb > mh.nbytes:
            raise ValueError("copy_h2d: destination must be a contiguous device tensor within the host buffer")
    n = len(pairs)
    src = (ctypes.c_void_p * n)(*[mh.dev for mh, _ in pairs])
    dst = (ctypes.c_void_p * n)(*[d.data_ptr() for _, d in pairs])
    nb = (ctypes.c_int64 * n)(*[d.numel() * d.element_size() for _, d in pairs])
    check(_launch("cgan3d_copy_multi_ex", src, dst, nb, n, int(max_blocks)), "copy_h2d")


def unpack_patches_mapped(src: MappedHost, data: torch.Tensor, seg: torch.Tensor, shift: float, factor: float,
                          max_blocks: int = 64):
    """unpack_patches from a mapped host buffer (int16 or float32 [..., 2]) straight into the device
    tensors: the loader's host-to-HBM step in one launch (cgan3d_unpack_patches_ex)."""
    t = src.tensor
    if t.dtype not in (torch.int16, torch.float32) or t.shape[-1] != 2:
        raise TypeError("unpack_patches_mapped: src must be int16 / float32 [..., 2]")
    nvox = t.numel() // 2
    if not (data.is_cuda and seg.is_cuda):
        raise ValueError("unpack_patches_mapped: data and seg must be device tensors")
    _need(data, nvox, "unpack_patches_mapped data")
    _need(seg, nvox, "unpack_patches_mapped seg", dtype=seg.dtype)
    if seg.dtype not in (torch.bool, torch.uint8):
        raise TypeError("unpack_patches_mapped: seg must be bool or uint8")
    check(_launch("cgan3d_unpack_patches_ex", src.dev, 0 if t.dtype == torch.int16 else 1, nvox, float(shift),
                  float(factor), ptr(data), ptr(seg), int(max_blocks)), "unpack_patches_mapped")


def augment_ws_floats(n: int, dims, n_elastic: int) -> int:
    return int(L.lib().cgan3d_augment_ws_floats(n, *dims, n_elastic))


def spatial_augment(data: torch.Tensor, seg: torch.Tensor, params: torch.Tensor, noise: Optional[torch.Tensor],
                    gauss: Optional[torch.Tensor], n_elastic: int, data_out: torch.Tensor, seg_out: torch.Tensor,
                    ws: torch.Tensor, dims=None):
    """SpatialTransform_2 on a patch batch (cgan3d_spatial_augment): data [n, 1?, a0, a1, a2] float32,
    seg of the same shape (bool / uint8), per-sample params [n, 16]; out of place.  ``dims``: (a0, a1,
    a2) when the trailing three dims are not the patch (a 2-D patch (W, H) runs as (1, W, H))."""
    n = data.shape[0]
    dims = tuple(data.shape[-3:]) if dims is None else tuple(int(d) for d in dims)
    vox = dims[0] * dims[1] * dims[2]
    _need(data, n * vox, "spatial_augment data")
    _need(data_out, n * vox, "spatial_augment data_out")
    for t, nm in ((seg, "seg"), (seg_out, "seg_out")):
        if t.dtype not in (torch.bool, torch.uint8):
            raise TypeError(f"spatial_augment: {nm} must be bool or uint8")
        _need(t, n * vox, f"spatial_augment {nm}", dtype=t.dtype)
    _need(params, n * 16, "spatial_augment params")
    if n_elastic:
        _need(noise, n_elastic * 3 * vox, "spatial_augment noise", exact=False)
        _need(gauss, n_elastic * 3 * max(dims), "spatial_augment gauss", exact=False)
    _need(ws, augment_ws_floats(n, dims, n_elastic), "spatial_augment ws", exact=False)
    check(_launch("cgan3d_spatial_augment", ptr(data), ptr(seg), n, *dims, ptr(params),
                  ptr(noise) if n_elastic else None, n_elastic, ptr(gauss) if n_elastic else None, ptr(data_out),
                  ptr(seg_out), ptr(ws)), "spatial_augment")


def mirror(data: torch.Tensor, seg: torch.Tensor, flags: torch.Tensor, data_out: torch.Tensor,
           seg_out: torch.Tensor, dims):
    """MirrorTransform on a device batch (cgan3d_mirror): data / seg [n, 1?, *patch] with ``dims`` =
    (a0, a1, a2) (a 2-D patch (W, H) as (1, W, H)), sample s flipped along a_d for every set bit d
    of flags[s] (device int32 [n]); out of place."""
    n = data.shape[0]
    dims = tuple(int(d) for d in dims)
    vox = dims[0] * dims[1] * dims[2]
    _need(data, n * vox, "mirror data")
    _need(data_out, n * vox, "mirror data_out")
    for t, nm in ((seg, "seg"), (seg_out, "seg_out")):
        if t.dtype not in (torch.bool, torch.uint8):
            raise TypeError(f"mirror: {nm} must be bool or uint8")
        _need(t, n * vox, f"mirror {nm}", dtype=t.dtype)
    _need(flags, n, "mirror flags", dtype=torch.int32)
    check(_launch("cgan3d_mirror", ptr(data), ptr(seg), n, *dims, ptr(flags), ptr(data_out), ptr(seg_out)), "mirror")


def patch_accumulate(patches: torch.Tensor, origins: torch.Tensor, out: torch.Tensor, weight: torch.Tensor):
    """out[origin + patch] += patch, weight[...] += 1 for a batch [b, 1?, p0, p1, p2] (origins [b, 3] int32)."""
    b, pd = patches.shape[0], tuple(patches.shape[-3:])
    sd = tuple(out.shape[-3:])
    _need(patches, b * pd[0] * pd[1] * pd[2], "patch_accumulate patches")
    _need(origins, 3 * b, "patch_accumulate origins", dtype=torch.int32)
    _need(out, sd[0] * sd[1] * sd[2], "patch_accumulate out")
    _need(weight, sd[0] * sd[1] * sd[2], "patch_accumulate weight")
    check(_launch("cgan3d_patch_accumulate", ptr(patches), b, *pd, ptr(origins), ptr(out), ptr(weight), *sd),
          "patch_accumulate")


def patch_normalize(out: torch.Tensor, weight: torch.Tensor):
    _need(weight, out.numel(), "patch_normalize weight")
    _need(out, out.numel(), "patch_normalize out")
    check(_launch("cgan3d_patch_normalize", ptr(out), ptr(weight), out.numel()), "patch_normalize")
