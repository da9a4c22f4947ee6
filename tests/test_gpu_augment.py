"""GPU spatial augmentation (csrc/augment.hip, data/augment.py) against the numpy/scipy
restatement of batchgenerators' augment_spatial_2 (oracle/augment_ref.py) on identical drawn
decisions.  Parity is against that restatement, unpinned by the reference (batchgenerators is a
dependency outside the reference tree and is not installed here).

Tolerances: data within 2e-4 of the patch's value range (fp32 coordinates and spline prefilter vs
scipy's float64); seg exact except where a sample coordinate lies within 1e-3 voxel of a
rounding boundary (x.5) or of the patch edge, where fp32 and fp64 coordinates may round apart."""
import sys
from pathlib import Path

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


def _near_boundary_2d(shape, dec):
    c = A.zero_centered_mesh(shape)
    if "angles" in dec:
        c = A.rotate_coords_2d(c, dec["angles"][0])
    if "scale" in dec:
        c = c * dec["scale"]
    c -= c.mean(axis=(1, 2), keepdims=True)
    near = np.zeros(shape, bool)
    for d in range(2):
        c[d] += shape[d] / 2.0 - 0.5
        near |= np.abs(c[d] - np.floor(c[d]) - 0.5) < 1e-3
        near |= (np.abs(c[d]) < 1e-3) | (np.abs(c[d] - (shape[d] - 1)) < 1e-3)
    return near


def test_spatial_augment_2d_matches_restatement():
    """SpatialTransform_2 on 2-D patches (experiments/conf_2D.py:21-41: rotation by up to a full turn,
    no elastic deformation) against the restatement of augment_spatial_2's 2-D branch
    (rotate_coords_2d, order-3 / order-0 map_coordinates), scaling included."""
    from cgan3d_amd.data.augment import SpatialTransform_2
    shape, n = (24, 20), 12
    t = SpatialTransform_2(shape, random_crop=False, do_elastic_deform=False, angle_x=(-2 * np.pi, 2 * np.pi),
                           p_rot_per_sample=0.6, p_scale_per_sample=0.3, scale=(0.8, 1.2))
    rng = np.random.default_rng(21)
    x = np.stack([_smooth(rng, shape) for _ in range(n)])[:, None]
    s = (rng.random((n, 1, *shape)) < 0.3)
    prm, noise, gauss = t.draw(np.random.default_rng(24), n)
    want_dec = A.spatial_2_decisions(np.random.default_rng(24).random, n, 2, do_elastic_deform=False,
                                     angle_x=(-2 * np.pi, 2 * np.pi), p_rot_per_sample=0.6, p_scale_per_sample=0.3,
                                     scale=(0.8, 1.2))
    assert [sorted(d) for d in t.last_decisions] == [sorted(d) for d in want_dec]
    xd, sd = torch.from_numpy(x).cuda(), torch.from_numpy(s).cuda()
    out, so = t.apply(xd, sd, prm, noise, gauss, torch.empty_like(xd), torch.empty_like(sd))
    out, so = out.cpu().numpy(), so.cpu().numpy()
    assert any(want_dec) and not all(want_dec)
    for j, dec in enumerate(want_dec):
        ref, sref = A.augment_sample(x[j, 0], s[j, 0].astype(np.float32), dec)
        if not dec:
            assert np.array_equal(out[j, 0], x[j, 0]) and np.array_equal(so[j, 0], s[j, 0])
            continue
        err = float(np.abs(out[j, 0] - ref).max())
        assert err <= 2e-4 * float(x[j].max() - x[j].min()), (j, dec, err)
        bad = so[j, 0] != (sref > 0.5)
        assert not (bad & ~_near_boundary_2d(shape, dec)).any(), (j, int(bad.sum()))


@pytest.mark.parametrize("dims,axes", [((8, 6, 5), (0, 1, 2)), ((12, 10), (0, 1)), ((7, 9, 4), (1,))])
def test_mirror_matches_restatement(dims, axes):
    """MirrorTransform (cgan3d_mirror) against batchgenerators' MirrorTransform / augment_mirroring
    restated in numpy (oracle/augment_ref.py), same draws: bit-exact."""
    from cgan3d_amd.data.augment import MirrorTransform
    n = 16
    rng = np.random.default_rng(3)
    x = rng.standard_normal((n, 1, *dims)).astype(np.float32)
    s = rng.random((n, 1, *dims)) < 0.4
    t = MirrorTransform(axes=axes, p_per_sample=0.5)
    t.patch_size = dims
    (flags,) = t.draw(np.random.default_rng(9), n)
    xd, sd = torch.from_numpy(x).cuda(), torch.from_numpy(s).cuda()
    out, so = t.run((torch.from_numpy(flags).cuda(),), xd, sd, torch.empty_like(xd), torch.empty_like(sd))
    want, wseg = x.copy(), s.copy()
    A.mirror_transform(want, wseg, axes, 0.5, np.random.default_rng(9).random)
    np.testing.assert_array_equal(out.cpu().numpy(), want)
    np.testing.assert_array_equal(so.cpu().numpy(), wseg)
    assert 0 < int((flags != 0).sum()) < n


def test_loader_2d_conf2d_batches(tmp_path):
    """conf_2D's training data path end to end (experiments/conf_2D.py:4-43): PatchLoader over 2-D
    patches of [W, H, D, 2] int16 scans with their meta records — get_samplable_2D's slices
    (centre-line patches and random slices padded and cropped), FactorZeroCenterScaler, then
    SpatialTransform_2 (rotation by up to a full turn, p 0.5, no elastic / scale) and MirrorTransform
    (axes (0, 1), p 0.5) — against the numpy restatements fed by a twin generator, batch by batch:
    unrotated samples bit-exact (crops and mirrors), rotated ones at the interpolation tolerance."""
    from cgan3d_amd.data.augment import MirrorTransform, SpatialTransform_2
    from cgan3d_amd.data.loader import PatchLoader
    from oracle import loader_ref as R
    sys.path.insert(0, str(Path(__file__).parent))
    from test_loader import _scan_2d
    rng = np.random.default_rng(0)
    paths, scans = [], {}
    for i, shp in enumerate([(40, 36, 6), (20, 44, 5), (12, 14, 4)]):
        vol, meta = _scan_2d(rng, shp)
        if shp[0] < 16 or shp[1] < 16:
            meta["centerlines_world"] = meta["centerlines_world"][:0]  # (the loader then draws only random slices)
        p = str(tmp_path / f"scan{i}")
        np.save(p + ".npy", vol)
        np.savez(p + "_meta.npz", name=f"scan{i}", **meta)
        paths.append(p)
        scans[p] = (vol, meta)
    paths = paths[:2]  # the third scan has no centre line: get_samplable_2D would fail on it half the time

    class FZC:
        shift, factor = 238, 600

    patch, B = (16, 16), 6
    rot = dict(do_elastic_deform=False, do_scale=False, do_rotation=True, angle_x=(-2 * np.pi, 2 * np.pi),
               angle_y=(-2 * np.pi, 2 * np.pi), angle_z=(-2 * np.pi, 2 * np.pi), p_rot_per_sample=0.5)
    tfs = [SpatialTransform_2(patch, random_crop=False, **rot), MirrorTransform(axes=(0, 1), p_per_sample=0.5)]
    loader = PatchLoader(paths, patch, B, np.random.default_rng(17), scaler=FZC(), depth=3, num_threads=2,
                         seed_for_shuffle=4, transform=tfs)
    twin = np.random.default_rng(17)
    counts = {"rotated": 0, "mirrored": 0, "plain": 0}
    for _ in range(5):
        b = next(loader)
        data, seg = b["data"].cpu().numpy(), b["seg"].cpu().numpy()
        assert data.shape == (B, 1, *patch) and seg.dtype == np.bool_
        want = np.zeros((B, 1, *patch), np.float32)
        wseg = np.zeros((B, 1, *patch), np.float32)
        for j, p in enumerate(b["path"]):
            vol, meta = scans[p]
            want[j, 0], wseg[j, 0] = R.generate_one_2d(vol, meta, patch, twin, 238, 600)
        decs = A.spatial_2_decisions(twin.random, B, 2, do_elastic_deform=False, angle_x=rot["angle_x"],
                                     p_rot_per_sample=0.5, do_scale=False)
        rot_out = np.zeros_like(want)
        rot_seg = np.zeros_like(wseg)
        for j, dec in enumerate(decs):
            rot_out[j, 0], rot_seg[j, 0] = A.augment_sample(want[j, 0], wseg[j, 0], dec) if dec else (want[j, 0],
                                                                                                      wseg[j, 0])
        before = rot_out.copy()
        A.mirror_transform(rot_out, rot_seg, (0, 1), 0.5, twin.random)
        for j, dec in enumerate(decs):
            mirrored = not np.array_equal(before[j], rot_out[j])
            counts["rotated" if dec else ("mirrored" if mirrored else "plain")] += 1
            if not dec:
                np.testing.assert_array_equal(data[j], rot_out[j])
                np.testing.assert_array_equal(seg[j], rot_seg[j] != 0)
            else:
                err = float(np.abs(data[j] - rot_out[j]).max())
                assert err <= 2e-4 * float(want[j].max() - want[j].min() + 1e-6), (j, dec, err)
    assert counts["rotated"] and counts["mirrored"] and counts["plain"], counts
    loader._finish()
