"""Loader factory with the signature of the reference's ``create_dataloaders``
(``contrast_gan_3D/trainer/utils.py:44-107``), building one :class:`PatchLoader` per scan label
instead of a batchgenerators augmenter around a ``CCTADataLoader``."""
from __future__ import annotations

import warnings
from collections import defaultdict
from pathlib import Path
from typing import Dict, List, Optional, Tuple, Union

import numpy as np

from ..data.augment import MirrorTransform, SpatialTransform_2
from ..data.loader import PatchLoader

DEFAULT_SEED = 42  # contrast_gan_3D/constants.py


def divide_scans_in_fold(fold) -> Dict[int, List[Union[str, Path]]]:
    """[(path, label), ...] -> {label: [path, ...]} (trainer/utils.py:36-40)."""
    ret = defaultdict(list)
    for path, label in fold:
        ret[label].append(path)
    return ret


def create_dataloaders(train_fold, val_fold, train_patch_size, val_patch_size, train_batch_sizes: Dict[int, int],
                       val_batch_sizes: Dict[int, int], rng: np.random.Generator, scaler=None,
                       num_workers: Tuple[int, int] = (1, 1), train_transform: Optional[callable] = None,
                       seed: int = DEFAULT_SEED, augmenter_class=None, device=None):
    """Returns ({label: PatchLoader} for training, {label: PatchLoader} for validation).

    ``augmenter_class`` is accepted for signature compatibility and ignored (the loader is its
    own prefetching pipeline).  ``train_transform`` (the reference conf's factory of a
    batchgenerators ``Compose([SpatialTransform_2(...), NumpyToTensor, ...])``, or a
    :class:`cgan3d_amd.data.augment.SpatialTransform_2`) becomes the training loaders' GPU spatial
    augmentation, followed by its MirrorTransform where it has one (conf_2D.py:36-43); the tensor
    conversions are what the loader does anyway."""
    spatial = transforms_from(train_transform) or None

    def build(fold, patch, sizes, workers, tf):
        return {label: PatchLoader(paths, patch, sizes[label], rng, scaler=scaler, shuffle=True, device=device,
                                   num_threads=max(1, workers), seed_for_shuffle=seed, transform=tf)
                for label, paths in divide_scans_in_fold(fold).items()}

    return (build(train_fold, train_patch_size, train_batch_sizes, num_workers[0], spatial),
            build(val_fold, val_patch_size, val_batch_sizes, num_workers[1], None))


def spatial_transform_from(train_transform) -> Optional[SpatialTransform_2]:
    """The SpatialTransform_2 inside the reference conf's ``train_transform`` (basic_conf.py:107-113):
    a factory returning a batchgenerators Compose, a Compose, a transform, or None."""
    if train_transform is None:
        return None
    t = train_transform
    if callable(t) and not hasattr(t, "transforms") and type(t).__name__ != "SpatialTransform_2":
        t = t()
    for c in getattr(t, "transforms", [t]):
        if isinstance(c, SpatialTransform_2):
            return c
        if type(c).__name__ == "SpatialTransform_2":  # batchgenerators' own instance: its attributes
            return SpatialTransform_2.from_transform(c)
    warnings.warn("create_dataloaders: train_transform holds no SpatialTransform_2; no augmentation applied")
    return None


def transforms_from(train_transform) -> list:
    """The device-supported transforms of the reference conf's ``train_transform``, in order:
    SpatialTransform_2 (basic_conf.py:87-113, conf_2D.py:21-41) and MirrorTransform (conf_2D.py:36-43),
    from a factory returning a batchgenerators Compose, a Compose, a transform, or None; tensor
    conversions (NumpyToTensor) are the loader's own, anything else is reported and skipped."""
    if train_transform is None:
        return []
    t = train_transform
    if callable(t) and not hasattr(t, "transforms") and type(t).__name__ not in ("SpatialTransform_2", "MirrorTransform"):
        t = t()
    out = []
    for c in getattr(t, "transforms", [t]):
        name = type(c).__name__
        if isinstance(c, (SpatialTransform_2, MirrorTransform)):
            out.append(c)
        elif name == "SpatialTransform_2":  # batchgenerators' own instances: their attributes
            out.append(SpatialTransform_2.from_transform(c))
        elif name == "MirrorTransform":
            out.append(MirrorTransform.from_transform(c))
        elif name != "NumpyToTensor":
            warnings.warn(f"create_dataloaders: {name} in train_transform has no device implementation; skipped")
    if not out:
        warnings.warn("create_dataloaders: train_transform holds no SpatialTransform_2; no augmentation applied")
    return out
