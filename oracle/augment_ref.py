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


def rotate_coords_2d(coords, angle):
    rot = np.array([[np.cos(angle), -np.sin(angle)], [np.sin(angle), np.cos(angle)]])
    return np.dot(coords.reshape(len(coords), -1).transpose(), rot).transpose().reshape(coords.shape)


def augment_mirroring(sample_data, sample_seg, axes, draw):
    """batchgenerators augment_mirroring on one sample [C, x, y(, z)] (numpy, in place), with
    ``draw()`` the uniform source: axis 0, 1, then 2 (3-D samples only), each flipped when its draw
    is below 0.5."""
    if 0 in axes and draw() < 0.5:
        sample_data[:, :] = sample_data[:, ::-1]
        sample_seg[:, :] = sample_seg[:, ::-1]
    if 1 in axes and draw() < 0.5:
        sample_data[:, :, :] = sample_data[:, :, ::-1]
        sample_seg[:, :, :] = sample_seg[:, :, ::-1]
    if 2 in axes and len(sample_data.shape) == 4:
        if draw() < 0.5:
            sample_data[:, :, :, :] = sample_data[:, :, :, ::-1]
            sample_seg[:, :, :, :] = sample_seg[:, :, :, ::-1]
    return sample_data, sample_seg


def mirror_transform(data, seg, axes, p_per_sample, draw):
    """batchgenerators MirrorTransform.__call__ on a batch [B, C, ...] (numpy, in place)."""
    for b in range(len(data)):
        if draw() < p_per_sample:
            augment_mirroring(data[b], seg[b], axes, draw)
    return data, seg


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
        coords = (rotate_coords_3d(coords, *dec["angles"]) if len(shape) == 3 else
                  rotate_coords_2d(coords, dec["angles"][0]))
    if "scale" in dec:
        coords = coords * dec["scale"]
    coords -= coords.mean(axis=tuple(range(1, coords.ndim)), keepdims=True)
    for d in range(len(shape)):
        coords[d] += shape[d] / 2.0 - 0.5
    out = ndi.map_coordinates(data.astype(np.float64), coords, order=3, mode="nearest").astype(np.float32)
    so = np.zeros(seg.shape, np.float64)
    for lab in np.unique(seg):  # interpolate_img(is_seg=True)
        r = ndi.map_coordinates((seg == lab).astype(float), coords, order=0, mode="constant", cval=0)
        so[r >= 0.5] = lab
    return out, so.astype(seg.dtype)


def spatial_2_decisions(u, n, ndim, do_elastic_deform=False, p_el_per_sample=1, do_rotation=True,
                        p_rot_per_sample=1, p_rot_per_axis=1, angle_x=(0, 2 * np.pi), angle_y=(0, 2 * np.pi),
                        angle_z=(0, 2 * np.pi), do_scale=True, p_scale_per_sample=1, scale=(0.75, 1.25)):
    """augment_spatial_2's per-sample random decisions in its draw order (batchgenerators 0.25), for
    transforms without elastic deformation (its decision is still drawn), with ``u()`` the U[0, 1)
    source (np.random.uniform(lo, hi) = lo + (hi - lo) u()): [{angles, scale} per sample]."""
    assert not do_elastic_deform
    out = []
    for _ in range(n):
        dec = {}
        u()  # `np.random.uniform() < p_el_per_sample and do_elastic_deform`
        if do_rotation and u() < p_rot_per_sample:
            a_x = angle_x[0] + (angle_x[1] - angle_x[0]) * u() if u() <= p_rot_per_axis else 0
            if ndim == 3:
                a_y = angle_y[0] + (angle_y[1] - angle_y[0]) * u() if u() <= p_rot_per_axis else 0
                a_z = angle_z[0] + (angle_z[1] - angle_z[0]) * u() if u() <= p_rot_per_axis else 0
                dec["angles"] = [a_x, a_y, a_z]
            else:
                dec["angles"] = [a_x]
        if do_scale and u() < p_scale_per_sample:
            if u() < 0.5 and scale[0] < 1:
                sc = scale[0] + (1 - scale[0]) * u()
            else:
                lo = max(scale[0], 1)
                sc = lo + (scale[1] - lo) * u()
            dec["scale"] = sc
        out.append(dec)
    return out
