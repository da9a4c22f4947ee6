"""Patch loader (cgan3d_amd/data/loader.py) against a numpy restatement of the reference's
CCTADataLoader.generate_one (contrast_gan_3D/data/CCTADataLoader.py:88-104): pad_nd_image
(zero padding, below = diff // 2) then a random crop, FactorZeroCenterScaler
((HU - shift) / factor in float32, data/Scaler.py:37-45) and the bool mask (trainer/utils.py:100).

CPU: the crop geometry and the host copy.  GPU: whole batches through the pinned ring, the H2D
copy and the unpack kernel, bit-exact against numpy.
"""
import copy

import numpy as np
import pytest

from cgan3d_amd.data.loader import _scaler_params, crop_box, read_crop


def _oracle_patch(vol, patch, box):
    """pad_nd_image + crop at the box's offsets, numpy."""
    pads = [(max(p - s, 0) // 2, max(p - s, 0) - max(p - s, 0) // 2) for s, p in zip(vol.shape[:3], patch)]
    padded = np.pad(vol, pads + [(0, 0)])
    lo = [b[0] if s >= p else 0 for b, s, p in zip(box, vol.shape[:3], patch)]
    return padded[lo[0]:lo[0] + patch[0], lo[1]:lo[1] + patch[1], lo[2]:lo[2] + patch[2]]


SHAPES = [(24, 24, 24), (16, 16, 16), (12, 20, 31), (5, 16, 40), (40, 9, 3)]


@pytest.mark.parametrize("shape", SHAPES)
def test_crop_matches_pad_then_crop(shape):
    rng = np.random.default_rng(0)
    patch = (16, 16, 16)
    vol = rng.integers(-1024, 3000, size=(*shape, 2)).astype(np.int16)
    out = np.full((*patch, 2), 77, dtype=np.int16)
    for _ in range(20):
        box = crop_box(shape, patch, rng)
        read_crop(vol, patch, box, out)
        np.testing.assert_array_equal(out, _oracle_patch(vol, patch, box))


def test_crop_offsets_cover_range():
    rng = np.random.default_rng(1)
    seen = {crop_box((20, 16, 8), (16, 16, 16), rng)[0][0] for _ in range(400)}
    assert seen == set(range(4))  # get_lbs_for_random_crop: randint(0, S - P), the upper end excluded
    assert crop_box((20, 16, 8), (16, 16, 16), rng)[1:] == [(0, 0, 16), (0, 4, 8)]


def test_scaler_params():
    class FZC:  # FactorZeroCenterScaler(low=-260, high=736, factor=600): shift = 238
        shift, factor = 238, 600

    class ZC:
        shift = 10

    assert _scaler_params(FZC()) == (238.0, 600.0)
    assert _scaler_params(ZC()) == (10.0, 1.0)
    assert _scaler_params(None) == (0.0, 1.0)
    assert _scaler_params(lambda x: x) == (0.0, 1.0)
    with pytest.raises(TypeError):
        _scaler_params(lambda x: 2 * x)


def _coord_volume(shape):
    """HU encodes the voxel's coordinates (so a patch reveals where it was cut); label 1 on a
    lattice of voxels."""
    x, y, z = np.meshgrid(*[np.arange(s) for s in shape], indexing="ij")
    hu = (x * shape[1] * shape[2] + y * shape[2] + z - 2000).astype(np.int16)
    lab = ((x + 2 * y + z) % 3 == 0).astype(np.int16)
    return np.stack([hu, lab], -1)


@pytest.mark.gpu
def test_mapped_host_copy_and_unpack():
    """Zero-copy upload (cgan3d_host_alloc + cgan3d_copy_multi_ex / cgan3d_unpack_patches_ex): a kernel
    reading mapped pinned memory over PCIe gives the bytes of the SDMA copy, and the four-voxel unpack
    the values of the one-voxel kernel, tails included."""
    import torch
    from cgan3d_amd import ops
    g = torch.Generator().manual_seed(0)
    for nvox in (4 * 2500 + 3, 5, 64 ** 3):
        for dt in (torch.int16, torch.float32):
            mh = ops.MappedHost((nvox, 2), dt)
            src = torch.randint(-1024, 3000, (nvox, 2), generator=g).to(dt)
            src[:, 1] = (torch.rand(nvox, generator=g) < 0.3).to(dt)
            mh.tensor.copy_(src)
            data, seg = torch.empty(nvox, device="cuda"), torch.empty(nvox, dtype=torch.bool, device="cuda")
            ops.unpack_patches_mapped(mh, data, seg, 238.0, 600.0, max_blocks=8)
            d2, s2 = torch.empty_like(data), torch.empty_like(seg)
            ops.unpack_patches(src.cuda(), d2, s2, 238.0, 600.0)
            torch.cuda.synchronize()
            assert torch.equal(data, d2) and torch.equal(seg, s2), (nvox, dt)
    for n in (1001, 4096, 3):
        mh = ops.MappedHost((n,), torch.float32)
        mh.tensor.copy_(torch.randn(n, generator=g))
        mb = ops.MappedHost((n + 5,), torch.bool)
        mb.tensor.copy_(torch.rand(n + 5, generator=g) < 0.5)
        d, db = torch.empty(n, device="cuda"), torch.empty(n + 5, dtype=torch.bool, device="cuda")
        ops.copy_h2d([(mh, d), (mb, db)], max_blocks=4)
        torch.cuda.synchronize()
        assert torch.equal(d.cpu(), mh.tensor) and torch.equal(db.cpu(), mb.tensor)


@pytest.mark.gpu
@pytest.mark.parametrize("zero_copy", [True, False])
@pytest.mark.parametrize("src_dtype", [np.int16, np.float32])
def test_loader_batches_bit_exact(tmp_path, src_dtype, zero_copy):
    import torch
    from cgan3d_amd.data.loader import PatchLoader

    patch = (16, 16, 16)
    shapes = [(24, 20, 18), (12, 16, 30), (16, 16, 16)]
    paths, vols = [], {}
    for i, s in enumerate(shapes):
        v = _coord_volume(s).astype(src_dtype)
        p = str(tmp_path / f"patient{i}")
        np.save(p + ".npy", v)
        paths.append(p)
        vols[p] = v

    class FZC:
        shift, factor = 238, 600

    loader = PatchLoader(paths, patch, batch_size=2, rng=np.random.default_rng(3), scaler=FZC(), depth=3,
                         num_threads=2, seed_for_shuffle=5, zero_copy=zero_copy)
    seen = set()
    for _ in range(7):
        b = next(loader)
        data, seg = b["data"], b["seg"]
        assert data.shape == (2, 1, *patch) and data.dtype == torch.float32 and data.is_cuda
        assert seg.shape == (2, 1, *patch) and seg.dtype == torch.bool
        data, seg = data.cpu().numpy(), seg.cpu().numpy()
        for j, p in enumerate(b["path"]):
            seen.add(p)
            assert b["name"][j] == p.rsplit("/", 1)[-1]
            vol = vols[p]
            # recover the crop origin from the coordinate encoding of the first unpadded voxel
            box = [(0, (P - s) // 2, s) if s < P else None for s, P in zip(vol.shape[:3], patch)]
            first = tuple(bx[1] if bx else 0 for bx in box)
            hu0 = int(round(float(data[j, 0][first]) * 600 + 238)) + 2000
            org = np.unravel_index(hu0, vol.shape[:3])
            box = [bx if bx else (int(o), 0, P) for bx, o, P in zip(box, org, patch)]
            ref = _oracle_patch(vol, patch, box).astype(np.float32)
            want = (ref[..., 0] - np.float32(238)) / np.float32(600)
            np.testing.assert_array_equal(data[j, 0], want)
            np.testing.assert_array_equal(seg[j, 0], ref[..., 1] != 0)
    assert seen == set(paths)
    loader._finish()


def _scan_2d(rng, shape, n_cl=12):
    """A [W, H, D, 2] int16 scan whose HU encodes the voxel coordinates, and its meta record with
    centre-line points in world coordinates (offset, anisotropic spacing) on the label channel."""
    W, H, D = shape
    x, y, z = np.meshgrid(np.arange(W), np.arange(H), np.arange(D), indexing="ij")
    hu = (x * H * D + y * D + z - 2000).astype(np.int16)
    offset, spacing = np.array([-30.0, 12.5, 4.0]), np.array([0.4, 0.45, 0.6])
    img = np.stack([rng.integers(0, W, n_cl), rng.integers(0, H, n_cl), rng.integers(0, D, n_cl)], -1)
    lab = np.zeros((W, H, D), np.int16)
    lab[img[:, 0], img[:, 1], img[:, 2]] = 1
    world = img * spacing + offset + rng.uniform(-0.15, 0.15, img.shape) * spacing
    meta = {"offset": offset, "spacing": spacing, "centerlines_world": np.concatenate([world, np.ones((n_cl, 1))], 1)}
    return np.stack([hu, lab], -1), meta


@pytest.mark.parametrize("shape,patch", [((40, 36, 7), (16, 16)), ((12, 40, 5), (16, 16)), ((16, 16, 3), (16, 16))])
def test_sample_2d_matches_get_samplable_2d(shape, patch):
    """conf_2D's slice sampler (CCTADataLoader.get_samplable_2D + generate_one, CCTADataLoader.py:50-104)
    against the numpy restatement (oracle/loader_ref.py) on twin generators: the same slices, centre-line
    patches (the reference's (y, x) bounds order kept) and pad-then-random-crop patches, draw for draw."""
    from cgan3d_amd.data.loader import sample_2d
    from oracle import loader_ref as R
    rng = np.random.default_rng(5)
    vol, meta = _scan_2d(rng, shape)
    ours, ref = np.random.default_rng(11), np.random.default_rng(11)
    out = np.zeros((*patch, 2), np.int16)
    kinds = {"centre": 0, "slice": 0, "refused": 0}
    for _ in range(60):
        along = copy.deepcopy(ref).random() < 0.5  # the branch get_samplable_2D is about to take
        try:
            want, mask = R.generate_one_2d(vol, meta, patch, ref, 0.0, 1.0)
        except (AssertionError, IndexError):  # a centre-line patch wider than the slice: the reference asserts
            with pytest.raises(ValueError):
                sample_2d(vol.shape, meta, patch, ours)
            kinds["refused"] += 1
            continue
        z, box = sample_2d(vol.shape, meta, patch, ours)
        read_crop(vol, patch, (z, box), out)
        np.testing.assert_array_equal(out[..., 0].astype(np.float32), want)
        np.testing.assert_array_equal(out[..., 1].astype(np.float32), np.asarray(mask, np.float32))
        kinds["centre" if along else "slice"] += 1
    assert ours.random() == ref.random()  # the generators advanced in step
    assert kinds["slice"] > 10 and (kinds["centre"] > 10 or kinds["refused"] > 10), kinds


def test_patch_bounds_edges():
    from cgan3d_amd.data.loader import patch_bounds
    from oracle import loader_ref as R
    for coords in ([0, 0], [3, 30], [39, 35], [20, 17], [7, 8]):
        for patch in ((16, 16), (15, 9), (40, 36)):
            want = R.get_patch_bounds(np.array(patch), (40, 36), np.array(coords))
            np.testing.assert_array_equal(patch_bounds(patch, (40, 36), np.array(coords)), want)
    with pytest.raises(ValueError):
        patch_bounds((50, 16), (40, 36), np.array([20, 10]))


def test_meta_pkl_restricted_unpickler(tmp_path):
    """The reference's ``_meta.pkl`` (data/utils.py:48-54: dict of numpy arrays) loads; a pickle that
    names any other global (code) is refused."""
    import os
    import pickle

    import pytest
    from cgan3d_amd.data.loader import load_meta
    meta = {"offset": np.array([1.5, -2.0, 3.0]), "spacing": np.array([0.4, 0.4, 0.5], np.float32),
            "centerlines_world": np.arange(12.0).reshape(3, 4), "name": "scan_0", "n": 3, "f": np.float64(2.5)}
    with open(tmp_path / "a_meta.pkl", "wb") as f:
        pickle.dump(meta, f)
    got = load_meta(str(tmp_path / "a"))
    assert set(got) == set(meta) and got["name"] == "scan_0" and got["n"] == 3 and got["f"] == 2.5
    for k in ("offset", "spacing", "centerlines_world"):
        assert got[k].dtype == meta[k].dtype and np.array_equal(got[k], meta[k])

    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))
    with open(tmp_path / "b_meta.pkl", "wb") as f:
        pickle.dump({"offset": Evil()}, f)
    with pytest.raises(pickle.UnpicklingError):
        load_meta(str(tmp_path / "b"))
