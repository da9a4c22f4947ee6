"""ORACLE — numpy/scipy restatement of batchgenerators' augment_spatial_2 for one sample.
TEST INFRASTRUCTURE ONLY (tests/ may import it; the product path never does).

batchgenerators (the reference's augmentation dependency, ``experiments/basic_conf.py:8,87-113``;
unpinned in ``env.yml``, restated from its 0.25 source) is not installed here.  This follows its
published algorithm step by step with the same scipy calls it makes (``fftn`` +
``ndimage.fourier_gaussian`` + ``ifftn`` for the elastic field, ``np.dot`` with the rotation
matrices, ``ndimage.map_coordinates`` for the resampling), given one sample's random decisions,
so the GPU kernel can be checked against it.  Parity is unpinned by the reference itself.
"""
import numpy as np
from scipy import ndimage as ndi


def zero_centered_mesh(shape):
    tmp = tuple(np.arange(i) for i in shape)
    coords = np.array(np.meshgrid(*tmp, indexing="ij")).astype(float)
    for d in range(len(shape)):
        coords[d] -= ((np.array(shape).astype(float) - 1) / 2.0)[d]
    return coords


def elastic_deform_coordinates_2(coords, sigmas, magnitudes, noise):
    offsets = []
    for d in range(len(coords)):
        f = np.fft.ifftn(ndi.fourier_gaussian(np.fft.fftn(noise[d].astype(np.float64)), sigmas)).real
        mx = np.max(np.abs(f))
        offsets.append(f / (mx / (magnitudes[d] + 1e-8)))
    return np.array(offsets) + coords


def rotate_coords_3d(coords, ax, ay, az):
    rot = np.identity(len(coords))
    c, s = np.cos(ax), np.sin(ax)
    rot = np.dot(rot, np.array([[1, 0, 0], [0, c, -s], [0, s, c]]))
    c, s = np.cos(ay), np.sin(ay)
    rot = np.dot(rot, np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]]))
    c, s = np.cos(az), np.sin(az)
    rot = np.dot(rot, np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]]))
    return np.dot(coords.reshape(len(coords), -1).transpose(), rot).transpose().reshape(coords.shape)


def augment_sample(data, seg, dec):
    """One sample of augment_spatial_2 (random_crop=False, patch = data shape) with the decisions
    ``dec`` = {sigmas, mags, noise} (elastic), {angles} (rotation), {scale}; empty: unchanged."""
    if not dec:
        return data.copy(), seg.copy()
    shape = data.shape
    coords = zero_centered_mesh(shape)
    if "noise" in dec:
        coords = elastic_deform_coordinates_2(coords, dec["sigmas"], dec["mags"], dec["noise"])
    if "angles" in dec:
        coords = rotate_coords_3d(coords, *dec["angles"])
    if "scale" in dec:
        coords = coords * dec["scale"]
    coords -= coords.mean(axis=tuple(range(1, coords.ndim)), keepdims=True)
    for d in range(3):
        coords[d] += shape[d] / 2.0 - 0.5
    out = ndi.map_coordinates(data.astype(np.float64), coords, order=3, mode="nearest").astype(np.float32)
    so = np.zeros(seg.shape, np.float64)
    for lab in np.unique(seg):  # interpolate_img(is_seg=True)
        r = ndi.map_coordinates((seg == lab).astype(float), coords, order=0, mode="constant", cval=0)
        so[r >= 0.5] = lab
    return out, so.astype(seg.dtype)
