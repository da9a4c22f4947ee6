"""GPU spatial augmentation (csrc/augment.hip, data/augment.py) against the numpy/scipy
restatement of batchgenerators' augment_spatial_2 (oracle/augment_ref.py) on identical drawn
decisions.  Parity is against that restatement, unpinned by the reference (batchgenerators is a
dependency outside the reference tree and is not installed here).

Tolerances: data within 2e-4 of the patch's value range (fp32 coordinates and spline prefilter vs
scipy's float64); seg exact except where a sample coordinate lies within 1e-3 voxel of a
rounding boundary (x.5) or of the patch edge, where fp32 and fp64 coordinates may round apart."""
import numpy as np
import pytest
import torch

from oracle import augment_ref as A

pytestmark = pytest.mark.gpu


def _smooth(rng, shape):
    return np.asarray(np.cumsum(np.cumsum(rng.standard_normal(shape), 0), 1) / 8.0, np.float32)


def _coords_near_boundary(shape, dec):
    """Voxels whose sample coordinate is within 1e-3 of a rounding or domain boundary."""
    c = A.zero_centered_mesh(shape)
    if "noise" in dec:
        c = A.elastic_deform_coordinates_2(c, dec["sigmas"], dec["mags"], dec["noise"])
    if "angles" in dec:
        c = A.rotate_coords_3d(c, *dec["angles"])
    if "scale" in dec:
        c = c * dec["scale"]
    c -= c.mean(axis=(1, 2, 3), keepdims=True)
    near = np.zeros(shape, bool)
    for d in range(3):
        c[d] += shape[d] / 2.0 - 0.5
        near |= np.abs(c[d] - np.floor(c[d]) - 0.5) < 1e-3
        near |= (np.abs(c[d]) < 1e-3) | (np.abs(c[d] - (shape[d] - 1)) < 1e-3)
    return near


@pytest.mark.parametrize("case", ["rot_scale", "elastic", "all", "reference_conf"])
def test_spatial_augment_matches_restatement(case):
    from cgan3d_amd.data.augment import SpatialTransform_2
    shape, n = (24, 20, 28), 6
    kw = dict(patch_size=shape, random_crop=False, angle_x=(-np.pi / 6, np.pi / 6), angle_y=(-np.pi / 6, np.pi / 6),
              angle_z=(-np.pi / 6, np.pi / 6), scale=(0.7, 1.4), deformation_scale=(0, 0.25))
    p = {"rot_scale": dict(p_el_per_sample=0, p_rot_per_sample=1, p_scale_per_sample=1),
         "elastic": dict(p_el_per_sample=1, p_rot_per_sample=0, p_scale_per_sample=0),
         "all": dict(p_el_per_sample=1, p_rot_per_sample=1, p_scale_per_sample=1),
         "reference_conf": dict(p_el_per_sample=0.1, p_rot_per_sample=0.2, p_scale_per_sample=0.2)}[case]
    t = SpatialTransform_2(**kw, **p)
    rng = np.random.default_rng({"rot_scale": 1, "elastic": 2, "all": 3, "reference_conf": 4}[case])
    x = np.stack([_smooth(rng, shape) for _ in range(n)])[:, None]
    s = (rng.random((n, 1, *shape)) < 0.3)
    prm, noise, gauss = t.draw(np.random.default_rng(10), n)
    xd, sd = torch.from_numpy(x).cuda(), torch.from_numpy(s).cuda()
    out, so = t.apply(xd, sd, prm, noise, gauss, torch.empty_like(xd), torch.empty_like(sd))
    out, so = out.cpu().numpy(), so.cpu().numpy()
    for j, dec in enumerate(t.last_decisions):
        ref, sref = A.augment_sample(x[j, 0], s[j, 0].astype(np.float32), dec)
        rng_ = float(x[j].max() - x[j].min())
        err = float(np.abs(out[j, 0] - ref).max())
        assert err <= 2e-4 * rng_, (case, j, sorted(dec), err, rng_)
        bad = so[j, 0] != (sref > 0.5)
        if not dec:
            assert np.array_equal(out[j, 0], x[j, 0]) and not bad.any()
        near = _coords_near_boundary(shape, dec)
        assert not (bad & ~near).any(), (case, j, int(bad.sum()), int((bad & ~near).sum()))


def test_loader_applies_transform(tmp_path):
    """PatchLoader(transform=...) returns augmented batches: with every augmentation drawn, the
    batch differs from the unaugmented crop, the mask stays boolean, the values stay finite."""
    from cgan3d_amd.data.augment import SpatialTransform_2
    from cgan3d_amd.data.loader import PatchLoader
    rng = np.random.default_rng(0)
    paths = []
    for i in range(2):
        hu = (rng.standard_normal((20, 20, 20)) * 100).astype(np.int16)
        lab = (rng.random((20, 20, 20)) < 0.2).astype(np.int16)
        p = str(tmp_path / f"p{i}")
        np.save(p + ".npy", np.stack([hu, lab], -1))
        paths.append(p)
    t = SpatialTransform_2((16, 16, 16), random_crop=False, p_el_per_sample=1, p_rot_per_sample=1,
                           p_scale_per_sample=1, angle_x=(0.3, 0.5), scale=(0.8, 0.9))
    plain = PatchLoader(paths, (16, 16, 16), 2, np.random.default_rng(7), depth=2, num_threads=1, seed_for_shuffle=1)
    aug = PatchLoader(paths, (16, 16, 16), 2, np.random.default_rng(7), depth=2, num_threads=1, seed_for_shuffle=1,
                      transform=t)
    for _ in range(3):
        a, b = next(plain), next(aug)
        assert b["data"].shape == a["data"].shape and b["seg"].dtype == torch.bool
        assert torch.isfinite(b["data"]).all()
        assert not torch.equal(a["data"], b["data"])
