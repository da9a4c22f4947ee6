"""Synthetic CCTA-like HU patches (SURVEY.md §8d "Synthetic inputs").

The reference trains on random crops of clipped HU volumes scaled by
``FactorZeroCenterScaler(-1024, 1500, 600)`` (``contrast_gan_3D/data/Scaler.py:37-45``,
``experiments/basic_conf.py:43``): ``(HU - 238) / 600`` with HU clipped to [-1024, 1500]
(``utils/io_utils.py:92-95``).  There is no dataset in this container, so patches are
generated: Gaussian soft tissue N(40, 350) HU plus 2-4 tubular "vessels" at U(250, 600) HU;
the centre-line mask (the reference's ``seg`` channel, ``data/CCTADataLoader.py:97-108``)
marks voxels within half a voxel of each vessel axis.

Pure numpy, deterministic given ``seed`` (PCG64).
"""
from __future__ import annotations

import numpy as np

MIN_HU, MAX_HU = -1024, 1500  # contrast_gan_3D/constants.py:6
HU_SHIFT = (MAX_HU - abs(MIN_HU)) // 2  # ZeroCenterScaler.__post_init__, data/Scaler.py:18
HU_FACTOR = 600  # basic_conf.py:38 max_HU_delta
DESIRED_HU_BOUNDS = (350, 450)  # basic_conf.py:39


def scale_hu(hu):
    """FactorZeroCenterScaler.__call__ (data/Scaler.py:43-44)."""
    return (np.asarray(hu, dtype=np.float64) - HU_SHIFT) / HU_FACTOR


def scaled_hu_bounds():
    """``scaler(np.array(desired_HU_bounds))`` as computed at ``train.py:146``."""
    lo, hi = scale_hu(np.array(DESIRED_HU_BOUNDS))
    return float(lo), float(hi)


def _segment_distance(shape, p0, p1):
    zz, yy, xx = np.meshgrid(*[np.arange(s, dtype=np.float32) for s in shape], indexing="ij")
    pts = np.stack([zz, yy, xx], axis=-1)
    d = (p1 - p0).astype(np.float32)
    dd = float(np.dot(d, d)) + 1e-12
    t = np.clip(((pts - p0) @ d) / dd, 0.0, 1.0)
    proj = p0 + t[..., None] * d
    return np.linalg.norm(pts - proj, axis=-1)


def synth_patches(n: int, size, seed: int, with_vessels: bool = True):
    """Return ``(data float32 [n,1,D,H,W], seg bool [n,1,D,H,W])`` scaled like the reference."""
    if isinstance(size, int):
        size = (size, size, size)
    rng = np.random.Generator(np.random.PCG64(seed))
    data = np.empty((n, 1, *size), np.float32)
    seg = np.zeros((n, 1, *size), bool)
    for i in range(n):
        hu = rng.normal(40.0, 350.0, size)
        if with_vessels:
            for _ in range(int(rng.integers(2, 5))):
                p0 = rng.uniform(0, np.array(size) - 1)
                p1 = rng.uniform(0, np.array(size) - 1)
                radius = rng.uniform(1.5, 3.0)
                dist = _segment_distance(size, p0, p1)
                hu = np.where(dist <= radius, rng.uniform(250.0, 600.0), hu)
                seg[i, 0] |= dist <= 0.5
        hu = np.clip(np.round(hu), MIN_HU, MAX_HU).astype(np.int16)
        data[i, 0] = scale_hu(hu).astype(np.float32)
    return data, seg
