"""ORACLE — numpy restatement of the reference's patch sampling (CCTADataLoader), for the loader tests.
TEST INFRASTRUCTURE ONLY (tests/ may import it; the product path never does).

Follows ``contrast_gan_3D/data/CCTADataLoader.py:50-104`` line by line (get_samplable_2D,
generate_one) with ``utils/geometry.py:21-26`` (world_to_image_coords) and ``:114-138``
(ensure_valid_bounds, get_patch_bounds), and batchgenerators' ``pad_nd_image`` + random ``crop``
(restated from the package's 0.25 source; batchgenerators is not installed here).  The one
deliberate difference, shared with the product loader: every random draw, the crop offsets
included, comes from the loader's ``numpy.random.Generator`` instead of batchgenerators' global
``np.random``.  The reference module itself cannot be imported on Python 3.10
(CCTADataLoader.py:69 is 3.11 syntax), so this restatement is pinned by the reference's source text,
not by a run of it.
"""
import numpy as np


def world_to_image_coords(world_coords, offset, spacing):
    """utils/geometry.py:21-26 (numpy arrays)."""
    assert np.shape(world_coords) == np.shape(offset) == np.shape(spacing) == (3,)
    ret = ((np.asarray(world_coords) - offset) / spacing).round()
    return ret.astype(int)


def ensure_valid_bounds(s, e, target_size, size):
    """utils/geometry.py:114-120."""
    assert not (s < 0 and e > size), f"{target_size} < {size}"
    if s < 0:
        s, e = 0, target_size
    if e > size:
        s, e = size - target_size, size
    return s, e


def get_patch_bounds(target_shape, source_shape, coords):
    """utils/geometry.py:131-138 with utils/__init__.py:53-58 (parse_patch_size)."""
    half = np.array(target_shape)
    for i, dim in enumerate(half):
        if dim == -1:
            half[i] = source_shape[i]
    half = half // 2
    target_shape = np.array(target_shape)
    bbox = np.dstack([coords - half, coords + half + target_shape % 2]).squeeze()
    for (i, (s, e)), target_size, size in zip(enumerate(bbox), target_shape, source_shape):
        bbox[i] = ensure_valid_bounds(s, e, target_size, size)
    return bbox


def pad_nd_image(image, new_shape):
    """batchgenerators pad_nd_image (constant 0): the trailing dims padded to at least new_shape,
    below = diff // 2, above = the rest."""
    old = np.array(image.shape[-len(new_shape):])
    new = np.maximum(np.array(new_shape), old)
    diff = new - old
    below = diff // 2
    pads = [(0, 0)] * (image.ndim - len(new_shape)) + list(zip(below, diff - below))
    return np.pad(image, pads)


def random_crop(data, seg, crop_size, rng):
    """batchgenerators crop(crop_type="random") of [B, C, *spatial] with get_lbs_for_random_crop's
    offsets (randint(0, s - p) where s - p > 0, else (s - p) // 2), drawn from ``rng``."""
    lbs = []
    for i, p in enumerate(crop_size):
        s = data.shape[i + 2]
        lbs.append(int(rng.integers(0, s - p)) if s - p > 0 else (s - p) // 2)
    sl = (slice(None), slice(None)) + tuple(slice(lb, lb + p) for lb, p in zip(lbs, crop_size))
    return data[sl], seg[sl]


def get_samplable_2d(data_and_seg, meta, patch_shape, rng):
    """CCTADataLoader.get_samplable_2D (CCTADataLoader.py:50-70): (slice patch [W', H', 2], do_crop)."""
    patch_shape = np.array(patch_shape)
    sample_along_centerlines = rng.random() < 0.5
    if sample_along_centerlines:
        centerlines = meta["centerlines_world"]
        centerline_idx = rng.integers(0, len(centerlines))
        x, y, z = world_to_image_coords(centerlines[centerline_idx, :3], meta["offset"], meta["spacing"])
        bbox = get_patch_bounds(patch_shape, data_and_seg[..., z, 0].shape, np.array([y, x]))
        indexer = [slice(*bbox[0]), slice(*bbox[1]), z]
    else:
        indexer = [..., rng.choice(data_and_seg.shape[2])]
    return data_and_seg[(*indexer, slice(None))], not sample_along_centerlines


def generate_one_2d(data_and_seg, meta, patch_shape, rng, shift, factor):
    """CCTADataLoader.generate_one (CCTADataLoader.py:88-104) for 2-D patches, with the
    FactorZeroCenterScaler (data/Scaler.py:37-45) applied: (data [W, H] float32, mask [W, H])."""
    ccta_and_seg, do_crop = get_samplable_2d(data_and_seg, meta, patch_shape, rng)
    ccta_and_seg = ccta_and_seg[None, None]
    patch, mask = ccta_and_seg[..., 0], ccta_and_seg[..., 1]
    if do_crop:
        ccta_and_seg = pad_nd_image(ccta_and_seg, (*patch_shape, 2))
        ccta_and_seg = ccta_and_seg.astype(np.float32)
        patch, mask = random_crop(ccta_and_seg[..., 0], ccta_and_seg[..., 1], patch_shape, rng)
    # generate_train_batch's `data[i] = patch` (CCTADataLoader.py:105) fails on any other shape
    assert patch.shape[-2:] == tuple(patch_shape), f"patch {patch.shape[-2:]} != {tuple(patch_shape)}"
    patch = (patch.astype(np.float32) - np.float32(shift)) / np.float32(factor)
    return patch[0, 0], mask[0, 0]
