"""Spatial augmentation on the GPU: drop-in for batchgenerators' ``SpatialTransform_2`` as the
reference's training transform uses it (``experiments/basic_conf.py:87-113``: elastic deformation
p = 0.1 with deformation_scale (0, 0.25), scaling p = 0.2 in (0.7, 1.4), rotation p = 0.2 by up to
+-30 degrees about each axis, ``random_crop=False``).

batchgenerators is a dependency of the reference, not part of its tree, and is not installed
here: the algorithm below restates ``augment_spatial_2`` from the package's published source
(batchgenerators 0.25, unpinned in the reference's ``env.yml``): per sample, on the zero-centred
voxel grid of the patch,

* elastic (``elastic_deform_coordinates_2``), with probability p_el: def_scale ~ U(deformation_scale);
  per axis sigma = def_scale * patch, magnitude ~ U(sigma / 8, sigma / 2); per axis a field of
  U[-1, 1) noise smoothed by a Gaussian of those sigmas in Fourier space (scipy
  ``fourier_gaussian``), scaled to max |field| = magnitude, added to the coordinates;
* rotation (``rotate_coords_3d``), with probability p_rot: angles ~ U(angle_x/y/z);
  coords <- (coords^T . Rx Ry Rz)^T;
* scaling (``scale_coords``), with probability p_scale: sc ~ U(scale[0], 1) with probability 1/2
  when scale[0] < 1, else U(max(scale[0], 1), scale[1]);
* if any was drawn: coordinates re-centred (mean subtracted) and moved to the patch centre
  (shape / 2 - 0.5); data sampled with order-3 splines, mode 'nearest'; seg with order 0, constant
  0 outside; otherwise the patch is returned unchanged.

The host draws these per-sample parameters (numpy ``Generator``: the loader's); the GPU does the
per-voxel work (``cgan3d_spatial_augment``, ``csrc/augment.hip``).  Parity: against a numpy/scipy
restatement of the same algorithm (``oracle/augment_ref.py``, ``tests/test_gpu_augment.py``) —
unpinned by the reference itself, whose augmenter cannot run here.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from .. import ops

N_PARAMS = 16


def _uniform(rng: np.random.Generator, lo: float, hi: float) -> float:
    """np.random.uniform's formula lo + (hi - lo) * U[0, 1), which batchgenerators relies on also
    when hi < lo (e.g. scale (0.8, 0.9): U(max(0.8, 1), 0.9)); Generator.uniform rejects that."""
    return lo + (hi - lo) * rng.random()


def gaussian_kernel(n: int, sigma: float) -> np.ndarray:
    """Circular convolution kernel of scipy.ndimage.fourier_gaussian along an axis of length n:
    the inverse DFT of exp(-2 pi^2 sigma^2 (k / n)^2), k folded to [-n/2, n/2)."""
    k = np.arange(n)
    k = np.where(k < (n + 1) // 2, k, k - n).astype(np.float64)
    h = np.exp(-2.0 * np.pi ** 2 * sigma ** 2 * (k / n) ** 2)
    return np.real(np.fft.ifft(h))


def rotation_matrix(ax: float, ay: float, az: float) -> np.ndarray:
    """batchgenerators rotate_coords_3d: coords' = (coords^T . Rx . Ry . Rz)^T = M coords, M = (Rx Ry Rz)^T."""
    cx, sx, cy, sy, cz, sz = np.cos(ax), np.sin(ax), np.cos(ay), np.sin(ay), np.cos(az), np.sin(az)
    rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return (np.eye(3) @ rx @ ry @ rz).T


class SpatialTransform_2:  # noqa: N801 (batchgenerators' name)
    """Constructor of batchgenerators' SpatialTransform_2 (same argument names and defaults);
    the reference configuration's subset is supported: order_data 3 / 'nearest', order_seg 0 /
    'constant' 0, random_crop False, one scale for all axes."""

    def __init__(self, patch_size, patch_center_dist_from_border=30, do_elastic_deform=True,
                 deformation_scale=(0, 0.25), do_rotation=True, angle_x=(0, 2 * np.pi), angle_y=(0, 2 * np.pi),
                 angle_z=(0, 2 * np.pi), do_scale=True, scale=(0.75, 1.25), border_mode_data="nearest",
                 border_cval_data=0, order_data=3, border_mode_seg="constant", border_cval_seg=0, order_seg=0,
                 random_crop=True, data_key="data", label_key="seg", p_el_per_sample=1, p_scale_per_sample=1,
                 p_rot_per_sample=1, independent_scale_for_each_axis=False, p_rot_per_axis: float = 1,
                 p_independent_scale_per_axis: float = 1):
        if (order_data, border_mode_data, order_seg, border_mode_seg, border_cval_seg) != (3, "nearest", 0,
                                                                                           "constant", 0):
            raise NotImplementedError("SpatialTransform_2: order_data 3 / 'nearest' and order_seg 0 / 'constant' 0 "
                                      "(the reference configuration) are supported")
        if random_crop:
            raise NotImplementedError("SpatialTransform_2: random_crop=False (basic_conf.py:91) is supported")
        if independent_scale_for_each_axis:
            raise NotImplementedError("SpatialTransform_2: one scale for all axes is supported")
        self.patch_size = tuple(int(p) for p in patch_size)
        if len(self.patch_size) not in (2, 3):
            raise ValueError(f"SpatialTransform_2: 2-D or 3-D patches, got {self.patch_size}")
        if len(self.patch_size) == 2 and do_elastic_deform:
            raise NotImplementedError("SpatialTransform_2: 2-D patches without elastic deformation "
                                      "(experiments/conf_2D.py switches it off)")
        self.do_elastic_deform, self.deformation_scale = do_elastic_deform, tuple(deformation_scale)
        self.do_rotation = do_rotation
        self.angle_x, self.angle_y, self.angle_z = tuple(angle_x), tuple(angle_y), tuple(angle_z)
        self.do_scale, self.scale = do_scale, tuple(scale)
        self.p_el_per_sample, self.p_scale_per_sample = p_el_per_sample, p_scale_per_sample
        self.p_rot_per_sample, self.p_rot_per_axis = p_rot_per_sample, p_rot_per_axis
        self.data_key, self.label_key = data_key, label_key

    @classmethod
    def from_transform(cls, t) -> "SpatialTransform_2":
        """From a batchgenerators SpatialTransform_2 instance (its attributes), e.g. the first
        transform of the reference's ``train_transform()`` Compose."""
        names = ("patch_size", "patch_center_dist_from_border", "do_elastic_deform", "deformation_scale",
                 "do_rotation", "angle_x", "angle_y", "angle_z", "do_scale", "scale", "border_mode_data",
                 "border_cval_data", "order_data", "border_mode_seg", "border_cval_seg", "order_seg", "random_crop",
                 "data_key", "label_key", "p_el_per_sample", "p_scale_per_sample", "p_rot_per_sample",
                 "independent_scale_for_each_axis", "p_rot_per_axis", "p_independent_scale_per_axis")
        return cls(**{k: getattr(t, k) for k in names if hasattr(t, k)})

    # -- host: per-sample parameters ------------------------------------------------------------
    @property
    def kernel_dims(self):
        """(a0, a1, a2) the kernels run on: the patch, a 2-D patch (W, H) as (1, W, H)."""
        return self.patch_size if len(self.patch_size) == 3 else (1,) + self.patch_size

    def draw(self, rng: np.random.Generator, n: int):
        """Per-sample parameters [n, 16], the elastic samples' noise [n_el, 3, *patch] and Gaussian
        kernel rows [n_el, 3, max(patch)], in augment_spatial_2's order of random draws."""
        if len(self.patch_size) == 2:
            return self._draw_2d(rng, n)
        ps = self.patch_size
        kst = max(ps)
        prm = np.zeros((n, N_PARAMS), np.float32)
        noise, gauss, decisions = [], [], []
        for s in range(n):
            m = np.eye(3)
            slot, mags, modified = -1, np.zeros(3), False
            dec = {}
            decisions.append(dec)
            # augment_spatial_2 evaluates `uniform() < p_el_per_sample and do_elastic_deform`: the
            # draw happens even with elastic deformation off, which keeps the later draws in place
            if rng.uniform() < self.p_el_per_sample and self.do_elastic_deform:
                def_scale = _uniform(rng, *self.deformation_scale)
                sig = [def_scale * p for p in ps]
                mags = np.array([_uniform(rng, sg / 8.0, sg / 2.0) for sg in sig])
                noise.append(np.stack([rng.random(ps) * 2 - 1 for _ in range(3)]).astype(np.float32))
                g = np.zeros((3, kst), np.float32)
                for ax in range(3):
                    g[ax, :ps[ax]] = gaussian_kernel(ps[ax], sig[ax])
                gauss.append(g)
                slot, modified = len(noise) - 1, True
                dec.update(sigmas=sig, mags=mags.tolist(), noise=noise[-1])
            if self.do_rotation and rng.uniform() < self.p_rot_per_sample:
                a = [_uniform(rng, *r) if rng.uniform() <= self.p_rot_per_axis else 0.0
                     for r in (self.angle_x, self.angle_y, self.angle_z)]
                m = rotation_matrix(*a) @ m
                dec["angles"] = a
                modified = True
            if self.do_scale and rng.uniform() < self.p_scale_per_sample:
                if rng.random() < 0.5 and self.scale[0] < 1:
                    sc = _uniform(rng, self.scale[0], 1)
                else:
                    sc = _uniform(rng, max(self.scale[0], 1), self.scale[1])
                m = sc * m
                dec["scale"] = sc
                modified = True
            prm[s, :9] = m.reshape(-1)
            prm[s, 9:12] = [p / 2.0 - 0.5 for p in ps]
            prm[s, 12] = slot if modified else -2
            prm[s, 13:16] = mags + 1e-8
        noise = np.stack(noise) if noise else None
        gauss = np.stack(gauss) if gauss else None
        self.last_decisions = decisions  # per sample {sigmas, mags, noise, angles, scale} (tests)
        return prm, noise, gauss

    def _draw_2d(self, rng: np.random.Generator, n: int):
        """2-D patches (experiments/conf_2D.py): augment_spatial_2's draws for dim == 2 — the elastic
        draw (its decision only: conf_2D switches the deformation off), one angle (a_x) turned by
        rotate_coords_2d (coords' = coords^T . R, R = [[cos, -sin], [sin, cos]]), the scale — as the
        kernels' (1, W, H) parameters: the first axis passes through."""
        W, H = self.patch_size
        prm = np.zeros((n, N_PARAMS), np.float32)
        decisions = []
        for s in range(n):
            m = np.eye(2)
            modified, dec = False, {}
            decisions.append(dec)
            rng.uniform()  # `uniform() < p_el_per_sample and do_elastic_deform`: drawn, never taken
            if self.do_rotation and rng.uniform() < self.p_rot_per_sample:
                a = _uniform(rng, *self.angle_x) if rng.uniform() <= self.p_rot_per_axis else 0.0
                c, sn = np.cos(a), np.sin(a)
                m = np.array([[c, -sn], [sn, c]]).T @ m
                dec["angles"] = [a]
                modified = True
            if self.do_scale and rng.uniform() < self.p_scale_per_sample:
                if rng.random() < 0.5 and self.scale[0] < 1:
                    sc = _uniform(rng, self.scale[0], 1)
                else:
                    sc = _uniform(rng, max(self.scale[0], 1), self.scale[1])
                m = sc * m
                dec["scale"] = sc
                modified = True
            m3 = np.eye(3)
            m3[1:, 1:] = m
            prm[s, :9] = m3.reshape(-1)
            prm[s, 9:12] = [0.0, W / 2.0 - 0.5, H / 2.0 - 0.5]
            prm[s, 12] = -1 if modified else -2
            prm[s, 13:16] = 1e-8
        self.last_decisions = decisions
        return prm, None, None

    # -- device ---------------------------------------------------------------------------------
    def apply(self, data: torch.Tensor, seg: torch.Tensor, prm, noise, gauss, data_out: torch.Tensor,
              seg_out: torch.Tensor, ws: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """Run the drawn transform on a device batch (out of place)."""
        dev = data.device
        n, dims = data.shape[0], tuple(data.shape[-len(self.patch_size):])
        if dims != self.patch_size:
            raise ValueError(f"SpatialTransform_2: patch {dims} != patch_size {self.patch_size}")
        n_el = 0 if noise is None else int(noise.shape[0])
        t = lambda a: a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa
        if ws is None:
            ws = torch.empty(ops.augment_ws_floats(n, self.kernel_dims, n_el), device=dev)
        ops.spatial_augment(data, seg, t(prm), t(noise) if n_el else None, t(gauss) if n_el else None, n_el,
                            data_out, seg_out, ws, dims=self.kernel_dims)
        return data_out, seg_out

    def run(self, params, data, seg, data_out, seg_out, ws=None):
        """Loader interface: ``params`` = what ``draw`` returned, on the device."""
        return self.apply(data, seg, *params, data_out, seg_out, ws=ws)

    def __call__(self, rng: np.random.Generator, data: torch.Tensor, seg: torch.Tensor):
        prm, noise, gauss = self.draw(rng, data.shape[0])
        return self.apply(data, seg, prm, noise, gauss, torch.empty_like(data), torch.empty_like(seg))


class MirrorTransform:
    """batchgenerators' MirrorTransform (same constructor), as experiments/conf_2D.py:36-43 uses it
    after SpatialTransform_2: ``MirrorTransform(axes=(0, 1), p_per_sample=0.5)``.  Restated from the
    package's published source (0.25; batchgenerators is not installed here): per sample, with
    probability p_per_sample, ``augment_mirroring`` flips the sample along each spatial axis in
    ``axes`` with probability 1/2 — one uniform draw per axis in order, axis 2 only for 3-D samples.
    The host draws the per-sample flags from the loader's generator; ``cgan3d_mirror`` flips on
    the GPU.  Parity: against a numpy restatement (tests/test_gpu_augment.py) — unpinned by the
    reference, whose augmenter cannot run here."""

    def __init__(self, axes=(0, 1, 2), data_key="data", label_key="seg", p_per_sample=1):
        self.axes = tuple(int(a) for a in axes)
        if self.axes and max(self.axes) > 2:
            raise ValueError("MirrorTransform takes the spatial axes (0, 1, 2)")
        self.data_key, self.label_key, self.p_per_sample = data_key, label_key, p_per_sample
        self.patch_size = None  # set by the loader: the patch it runs on

    @classmethod
    def from_transform(cls, t) -> "MirrorTransform":
        return cls(**{k: getattr(t, k) for k in ("axes", "data_key", "label_key", "p_per_sample") if hasattr(t, k)})

    def draw(self, rng: np.random.Generator, n: int, ndim: Optional[int] = None):
        """Per-sample flags [n] int32: bit d = flip spatial axis d (augment_mirroring's draws)."""
        ndim = ndim if ndim is not None else len(self.patch_size)
        flags = np.zeros(n, np.int32)
        for s in range(n):
            if rng.uniform() < self.p_per_sample:
                f = 0
                if 0 in self.axes and rng.uniform() < 0.5:
                    f |= 1
                if 1 in self.axes and rng.uniform() < 0.5:
                    f |= 2
                if 2 in self.axes and ndim == 3 and rng.uniform() < 0.5:
                    f |= 4
                flags[s] = f
        return (flags,)

    def run(self, params, data, seg, data_out, seg_out, ws=None):
        """Loader interface: flip the device batch out of place by the drawn flags (device int32)."""
        (flags,) = params
        ps = tuple(self.patch_size)
        dims = ps if len(ps) == 3 else (1,) + ps
        if len(ps) == 2:  # spatial axis d of a (W, H) patch is kernel axis d + 1
            flags = flags * 2
        ops.mirror(data, seg, flags, data_out, seg_out, dims)
        return data_out, seg_out
