"""ctypes binding of libcgan3d.so — the C-ABI declared in include/cgan3d.h.

The library is built in-tree (``contrast-gan-3d_amd/csrc/Makefile`` → ``cgan3d_amd/libcgan3d.so``).
It is loaded *after* torch so that its ``libamdhip64.so.7`` dependency binds to the HIP runtime
torch already mapped (one runtime per process: torch's streams and device pointers are valid in
our kernels).  There is no fallback: if the library or a GPU is missing, calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import torch  # noqa: F401  (must be imported first: see module docstring)

# CGAN3D_LIB_PATH: another build of the same library (back-to-back A/B of two builds, tools/gpu_ab_lib.sh)
LIB_PATH = Path(os.environ.get("CGAN3D_LIB_PATH") or Path(__file__).resolve().parent / "libcgan3d.so")

ACT_NONE, ACT_RELU, ACT_LRELU, ACT_TANH, ACT_NEG_DTANH = 0, 1, 2, 3, 4
WGRAD_ACCUMULATE, WGRAD_WS_CLEAN, WGRAD_DEFER_UNPACK, WGRAD_DEFER_REDUCE = 1, 2, 4, 8  # cgan3d_conv3d_wgrad_ex flags
# device loss slots written by the loss kernels (include/cgan3d.h)
L_D, L_WD, L_GP, L_G, L_SIM, L_HU, L_GFULL = range(7)


class ConvGeom(C.Structure):
    _fields_ = [("n", C.c_int32), ("di", C.c_int32), ("hi", C.c_int32), ("wi", C.c_int32),
                ("do_", C.c_int32), ("ho", C.c_int32), ("wo", C.c_int32),
                ("cin", C.c_int32), ("cout", C.c_int32), ("k", C.c_int32), ("stride", C.c_int32),
                ("pad", C.c_int32), ("transposed", C.c_int32), ("reflect", C.c_int32),
                ("w_sa", C.c_int64), ("w_sb", C.c_int64), ("w_packed", C.c_int32), ("prec", C.c_int32),
                ("planar", C.c_int32)]


class UnpackDesc(C.Structure):
    _fields_ = [("ws", C.c_void_p), ("dw", C.c_void_p), ("sa", C.c_int64), ("sb", C.c_int64),
                ("taps", C.c_int32), ("cin", C.c_int32), ("cout", C.c_int32), ("accumulate", C.c_int32)]


class PackDesc(C.Structure):
    _fields_ = [("w", C.c_void_p), ("wp", C.c_void_p), ("sa", C.c_int64), ("sb", C.c_int64),
                ("taps", C.c_int32), ("cin", C.c_int32), ("cout", C.c_int32), ("ldb", C.c_int32),
                ("format", C.c_int32), ("reserved", C.c_int32)]


class CsumDesc(C.Structure):
    _fields_ = [("x", C.c_void_p), ("out", C.c_void_p), ("ws", C.c_void_p), ("nvox", C.c_int64), ("c", C.c_int32),
                ("accumulate", C.c_int32)]


class LnArgs(C.Structure):
    _fields_ = [("n", C.c_int32), ("mode", C.c_int32), ("L", C.c_int64), ("slope", C.c_float), ("eps", C.c_float),
                ("z", C.c_void_p), ("da", C.c_void_p), ("zdot", C.c_void_p), ("adot", C.c_void_p),
                ("abar", C.c_void_p), ("p_stats", C.c_void_p), ("p_bwd", C.c_void_p), ("p_jvp", C.c_void_p),
                ("p_sig", C.c_void_p), ("p_adj", C.c_void_p)]


LN_STATS, LN_BWD, LN_JVP, LN_SIG, LN_ADJ = range(5)

PREC_F32, PREC_BF16 = 0, 1


class BnFuse(C.Structure):
    """include/cgan3d.h cgan3d_bn_fuse: BatchNorm statistics into fp64 accumulators."""
    _fields_ = [("acc_out", C.c_void_p), ("acc_mode", C.c_int32), ("reps", C.c_int32)]


class ReduceDesc(C.Structure):
    """include/cgan3d.h cgan3d_reduce_desc: one deferred ResNet weight-gradient reduce."""
    _fields_ = [("ws", C.c_void_p), ("dw", C.c_void_p), ("sa", C.c_int64), ("sb", C.c_int64),
                ("P", C.c_int32), ("cin", C.c_int32), ("cout", C.c_int32), ("accumulate", C.c_int32)]


class BnPre(C.Structure):
    """include/cgan3d.h cgan3d_bn_pre: the conv input's BatchNorm applied while the ResNet-block kernel
    stages its halo (mode 1 forward, 2 input-grad)."""
    _fields_ = [("mode", C.c_int32), ("z", C.c_void_p), ("acc", C.c_void_p), ("reps", C.c_int32),
                ("nvox", C.c_int64), ("gamma", C.c_void_p), ("beta", C.c_void_p), ("running_mean", C.c_void_p),
                ("running_var", C.c_void_p), ("num_batches_tracked", C.c_void_p), ("momentum", C.c_float),
                ("eps", C.c_float), ("scale_shift", C.c_void_p), ("mean_invstd", C.c_void_p), ("dgamma", C.c_void_p),
                ("dbeta", C.c_void_p), ("accumulate", C.c_int32), ("act", C.c_int32), ("slope", C.c_float),
                ("out_bf16", C.c_void_p), ("zero", C.c_void_p), ("zero_n", C.c_int32)]


class Epilogue(C.Structure):
    _fields_ = [("bias", C.c_void_p), ("residual", C.c_void_p), ("mask_src", C.c_void_p),
                ("minuend", C.c_void_p), ("out2", C.c_void_p), ("stats", C.c_void_p),
                ("act", C.c_int32), ("slope", C.c_float),
                ("bn_part", C.c_void_p), ("bn_mode", C.c_int32), ("bn_slots", C.c_int32), ("bn_z", C.c_void_p),
                ("bn_ss", C.c_void_p), ("bn_mi", C.c_void_p), ("bn_act", C.c_int32), ("bn_slope", C.c_float),
                ("x_bf16", C.c_void_p), ("bn_fold", C.c_int32), ("fuse", C.POINTER(BnFuse)),
                ("out_bf16", C.c_int32), ("pre", C.POINTER(BnPre))]


_P, _I32, _I64, _F = C.c_void_p, C.c_int32, C.c_int64, C.c_float
_SIGS = {
    "cgan3d_version": ([], C.c_char_p),
    "cgan3d_get_last_error": ([], C.c_char_p),
    "cgan3d_set_tuning": ([_I32, _I32], _I32),
    "cgan3d_conv3d_stats_floats": ([_P], _I64),
    "cgan3d_conv3d_fwd": ([_P, _P, _P, _P, _P, _P], _I32),
    "cgan3d_packed_weight_floats": ([_P], _I64),
    "cgan3d_halo_eligible": ([_P], _I32),
    "cgan3d_packed_format": ([_P], _I32),
    "cgan3d_pack_weights": ([_P, _P, _P, _P], _I32),
    "cgan3d_pack_weights_multi": ([_P, _I32, _I64, _P], _I32),
    "cgan3d_conv3d_wgrad_ws_floats": ([_P], _I64),
    "cgan3d_conv3d_wgrad": ([_P, _P, _P, _P, _I32, _P, _P], _I32),
    "cgan3d_conv3d_shadow_only": ([_P, _I32], _I32),
    "cgan3d_conv3d_bn_fold_ok": ([_P], _I32),
    "cgan3d_bn_fuse_ok": ([_P], _I32),
    "cgan3d_conv3d_bn_pre_ok": ([_P], _I32),
    "cgan3d_conv3d_neg_dtanh_ok": ([_P], _I32),
    "cgan3d_conv3d_cin1t": ([_P], _I32),
    "cgan3d_conv3d_sumsq_blocks": ([_P], _I64),
    "cgan3d_conv3d_wgrad_group_ok": ([_P], _I32),
    "cgan3d_conv3d_wgrad_group": ([_P, _P, _P, _P, _I32, _P], _I32),
    "cgan3d_conv3d_wgrad_ex": ([_P, _P, _P, _P, _I32, _P, _P, _P, _P], _I32),
    "cgan3d_bn_finalize": ([_P, _I64, _I32, _P, _P, _P, _P, _P, _F, _F, _P, _P, _P], _I32),
    "cgan3d_bn_apply": ([_P, _I64, _I32, _P, _I32, _F, _P, _P, _P, _P], _I32),
    "cgan3d_conv3d_bn_slots": ([_P], _I64),
    "cgan3d_bn_finalize_slab": ([_P, _I32, _I32, _I64, _P, _P, _P, _P, _P, _F, _F, _P, _P, _P], _I32),
    "cgan3d_bn_apply_slab": ([_P, _I32, _I32, _I64, _P, _P, _P, _P, _P, _F, _F, _P, _P, _P, _I32, _F, _P, _P, _P,
                              _P], _I32),
    "cgan3d_bn_backward_slab": ([_P, _P, _I64, _I32, _P, _I32, _P, _P, _P, _I32, _F, _P, _P, _P, _I32, _P, _P, _P],
                                _I32),
    "cgan3d_bn_backward_ws_floats": ([_I64, _I32], _I64),
    "cgan3d_bn_apply_acc": ([_P, _I32, _I32, _I64, _P, _P, _P, _P, _P, _F, _F, _P, _P, _P, _I32, _F, _P, _P, _P, _P,
                             _I32, _I32, _P], _I32),
    "cgan3d_bn_backward_acc_fold": ([_P, _P, _I32, _I32, _I32, _I32, _I32, _I32, _P, _I32, _P, _P, _P, _I32, _F, _P,
                                     _P, _P, _I32, _P, _P, _I32, _I32, _P], _I32),
    "cgan3d_bn_backward_acc": ([_P, _P, _I64, _I32, _P, _I32, _P, _P, _P, _I32, _F, _P, _P, _P, _I32, _P, _P, _I32,
                                _I32, _P], _I32),
    "cgan3d_conv3d_out_bf16_ok": ([_P], _I32),
    "cgan3d_bn_backward_slab_fold": ([_P, _P, _I32, _I32, _I32, _I32, _I32, _I32, _P, _I32, _P, _P, _P, _I32, _F, _P,
                                      _P, _P, _I32, _P, _P, _P], _I32),
    "cgan3d_bn_backward": ([_P, _P, _I64, _I32, _P, _P, _P, _I32, _F, _P, _P, _P, _I32, _P, _P], _I32),
    "cgan3d_channel_sum_ws_floats": ([_I64, _I32], _I64),
    "cgan3d_channel_sum": ([_P, _I64, _I32, _P, _P, _P], _I32),
    "cgan3d_channel_sum_multi": ([_P, _I32, _I32, _I32, _P], _I32),
    "cgan3d_reflect_fold": ([_P, _P, _I32, _I32, _I32, _I32, _I32, _I32, _P], _I32),
    "cgan3d_reflect_fold_slots": ([_I32, _I32, _I32, _I32, _I32], _I32),
    "cgan3d_reflect_fold_ex": ([_P, _P, _I32, _I32, _I32, _I32, _I32, _I32, _P, _P], _I32),
    "cgan3d_reflect_fold2d": ([_P, _P, _I32, _I32, _I32, _I32, _I32, _P, _P], _I32),
    "cgan3d_gp_interpolate": ([_P, _P, _P, _P, _I32, _I64, _P], _I32),
    "cgan3d_gp_interpolate_idx": ([_P, _P, _P, _P, _P, _I32, _I64, _I32, _I32, _P], _I32),
    "cgan3d_conv3d_wgrad_sk_ok": ([_P], _I32),
    "cgan3d_conv3d_wgrad_partials": ([_P], _I32),
    "cgan3d_wgrad_reduce_multi": ([_P, _I32, _P], _I32),
    "cgan3d_conv3d_wgrad_sk_ws_floats": ([_P], _I64),
    "cgan3d_conv3d_wgrad_sk": ([_P, _P, _P, _P, _P, _I32, _P], _I32),
    "cgan3d_tanh_backward": ([_P, _P, _P, _I64, _P], _I32),
    "cgan3d_unpack_patches": ([_P, _I32, _I64, _F, _F, _P, _P, _P], _I32),
    "cgan3d_unpack_patches_ex": ([_P, _I32, _I64, _F, _F, _P, _P, _I32, _P], _I32),
    "cgan3d_augment_ws_floats": ([_I32, _I32, _I32, _I32, _I32], _I64),
    "cgan3d_patch_accumulate": ([_P, _I32, _I32, _I32, _I32, _P, _P, _P, _I32, _I32, _I32, _P], _I32),
    "cgan3d_patch_normalize": ([_P, _P, _I64, _P], _I32),
    "cgan3d_spatial_augment": ([_P, _P, _I32, _I32, _I32, _I32, _P, _P, _I32, _P, _P, _P, _P, _P], _I32),
    "cgan3d_mirror": ([_P, _P, _I32, _I32, _I32, _I32, _P, _P, _P, _P], _I32),
    "cgan3d_loss_ws_floats": ([_I64], _I64),
    "cgan3d_critic_logits_grad": ([_P, _I32, _I32, _I32, _I32, _F, _P, _P, _P], _I32),
    "cgan3d_gradient_penalty": ([_P, _I32, _I64, _F, _P, _P, _P, _P], _I32),
    "cgan3d_gradient_penalty_part": ([_P, _P, _I32, _I32, _I64, _F, _P, _P, _P, _I32, _I32, _I32, _F, _P, _I64, _P],
                                     _I32),
    "cgan3d_generator_logits_grad": ([_P, _I32, _F, _P, _P, _P], _I32),
    "cgan3d_generator_output_grad": ([_P, _P, _P, _P, _P, _I64, _F, _F, _F, _F, _P, _P, _P, _P], _I32),
    "cgan3d_adam_tick": ([_P, _P], _I32),
    "cgan3d_adam": ([_P, _P, _P, _P, _I64, _P, _P], _I32),
    "cgan3d_adam_range": ([_P, _P, _P, _P, _I64, _P, _P], _I32),
    "cgan3d_adam_pack": ([_P, _P, _P, _P, _I64, _P, _P, _I32, _P, _P], _I32),
    "cgan3d_zero": ([_P, _I64, _P], _I32),
    "cgan3d_copy_multi": ([_P, _P, _P, _I32, _P], _I32),
    "cgan3d_copy_multi_ex": ([_P, _P, _P, _I32, _I32, _P], _I32),
    "cgan3d_host_alloc": ([_I64, _P, _P], _I32),
    "cgan3d_host_free": ([_P], _I32),
    "cgan3d_wgrad_unpack_multi": ([_P, _I32, _I64, _P], _I32),
    "cgan3d_ln_partial_doubles": ([_I32, _I64], _I64),
    "cgan3d_ln_reduce": ([_P, _P, _P], _I32),
    "cgan3d_ln_apply": ([_P, _P, _P], _I32),
    "cgan3d_conv3d_wgrad_ws_mode": ([_P], _I32),
    "cgan3d_plan_begin": ([], _I32),
    "cgan3d_plan_end": ([C.POINTER(C.c_void_p)], _I32),
    "cgan3d_plan_size": ([_P], _I64),
    "cgan3d_plan_run": ([_P], _I32),
    "cgan3d_plan_destroy": ([_P], _I32),
    "cgan3d_plan_time_filter": ([C.c_char_p], _I32),
    "cgan3d_plan_times": ([_P, _P, _I64], _I64),
    "cgan3d_plan_timeline": ([_P, _P, _P, _P, _I64], _I64),
    "cgan3d_plan_timed_name": ([_P, _I64], C.c_char_p),
    "cgan3d_stream_wait": ([_P, _P], _I32),
    "cgan3d_comm_shared_library": ([], _I32),
    "cgan3d_comm_id_bytes": ([], _I32),
    "cgan3d_comm_unique_id": ([_P], _I32),
    "cgan3d_comm_init": ([_P, _I32, _I32, C.POINTER(C.c_void_p)], _I32),
    "cgan3d_comm_destroy": ([_P], _I32),
    "cgan3d_allreduce_mean": ([_P, _P, _I64, _P], _I32),
}

_lib = None


def exported_symbols():
    return list(_SIGS)


def load(path: os.PathLike | str | None = None) -> C.CDLL:
    """Load and type the library (no GPU needed to load; kernels need one to run)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path is not None else LIB_PATH
    if not p.is_file():
        raise RuntimeError(f"cgan3d: HIP library not built: {p} (run __graft_entry__.build() or make -C csrc)")
    lib = C.CDLL(str(p))
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    if path is None:
        _lib = lib
        # CGAN3D_TUNE="key=value,key=value": cgan3d_set_tuning before anything is built (sweeps);
        # keys >= 100 are the host schedule's own knobs (py_tune)
        for k, v in tune_pairs():
            if k < 100:
                check(lib.cgan3d_set_tuning(k, v), f"set_tuning {k}={v}")
    return lib


def tune_pairs():
    """(key, value) pairs of CGAN3D_TUNE."""
    out = []
    for kv in filter(None, os.environ.get("CGAN3D_TUNE", "").replace(" ", "").split(",")):
        k, v = kv.split("=")
        out.append((int(k), int(v)))
    return out


def py_tune(key: int, default: int) -> int:
    """A host-schedule knob from CGAN3D_TUNE (keys >= 100; read when an engine is built)."""
    for k, v in tune_pairs():
        if k == key:
            return v
    return default


def lib() -> C.CDLL:
    if _lib is None:
        if not torch.cuda.is_available():
            raise RuntimeError("cgan3d: the HIP path needs a GPU (torch.cuda.is_available() is False)")
        load()
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = _lib.cgan3d_get_last_error().decode() if _lib is not None else ""
        raise RuntimeError(f"cgan3d {what} failed (status {rc}): {msg}")


def ptr(t: "torch.Tensor | None") -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream
