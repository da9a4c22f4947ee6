"""Spatial augmentation, host side and oracle (CPU): the GPU kernel's inputs drawn like
batchgenerators' augment_spatial_2 (experiments/basic_conf.py:87-113), and the numpy/scipy
restatement (oracle/augment_ref.py) pinned on cases with known answers.  batchgenerators itself is
absent (a dependency of the reference, not in its tree): parity against it is unpinned."""
import numpy as np
import pytest
from scipy import ndimage as ndi

from oracle import augment_ref as A

REF_ARGS = dict(patch_size=(16, 16, 16), random_crop=False, do_elastic_deform=True, deformation_scale=(0, 0.25),
                p_el_per_sample=0.1, do_scale=True, scale=(0.7, 1.4), p_scale_per_sample=0.2, do_rotation=True,
                angle_x=(-np.pi / 6, np.pi / 6), angle_y=(-np.pi / 6, np.pi / 6), angle_z=(-np.pi / 6, np.pi / 6),
                p_rot_per_sample=0.2)


def test_gaussian_kernel_is_fourier_gaussian():
    from cgan3d_amd.data.augment import gaussian_kernel
    for n, sig in ((16, 0.0), (20, 3.3), (64, 16.0), (33, 5.5)):
        delta = np.zeros(n)
        delta[0] = 1
        ref = np.fft.ifft(ndi.fourier_gaussian(np.fft.fft(delta), sig)).real
        assert np.abs(ref - gaussian_kernel(n, sig)).max() < 1e-12


def test_rotation_matrix_matches_rotate_coords_3d():
    from cgan3d_amd.data.augment import rotation_matrix
    rng = np.random.default_rng(0)
    c = rng.standard_normal((3, 5, 6, 7))
    a = rng.uniform(-1, 1, 3)
    got = np.einsum("ij,j...->i...", rotation_matrix(*a), c)
    assert np.abs(got - A.rotate_coords_3d(c, *a)).max() < 1e-12


def test_draw_probabilities_and_ranges():
    from cgan3d_amd.data.augment import SpatialTransform_2
    t = SpatialTransform_2(**REF_ARGS)
    prm, noise, gauss = t.draw(np.random.default_rng(1), 4000)
    dec = t.last_decisions
    el = np.array(["noise" in d for d in dec])
    rot = np.array(["angles" in d for d in dec])
    sc = np.array(["scale" in d for d in dec])
    for frac, p in ((el.mean(), 0.1), (rot.mean(), 0.2), (sc.mean(), 0.2)):
        assert abs(frac - p) < 4 * np.sqrt(p * (1 - p) / 4000)
    assert noise.shape == (el.sum(), 3, 16, 16, 16) and gauss.shape == (el.sum(), 3, 16)
    assert (prm[:, 12] == -2).sum() == sum(not d for d in dec)  # untouched samples are copied
    scales = np.array([d["scale"] for d in dec if "scale" in d])
    assert scales.min() >= 0.7 and scales.max() <= 1.4
    angles = np.array([d["angles"] for d in dec if "angles" in d])
    assert np.abs(angles).max() <= np.pi / 6
    for d in dec:
        if "noise" in d:
            assert all(s / 8 <= m <= s / 2 for s, m in zip(d["sigmas"], d["mags"]))
            assert d["noise"].min() >= -1 and d["noise"].max() < 1


def test_oracle_quarter_turn_is_rot90():
    """A 90-degree rotation samples integer coordinates: the cubic spline interpolates them exactly,
    so the restatement must reproduce np.rot90 of the patch (checks its axis conventions)."""
    rng = np.random.default_rng(2)
    x = rng.standard_normal((8, 8, 8)).astype(np.float32)
    s = (rng.random((8, 8, 8)) < 0.3).astype(np.float32)
    out, so = A.augment_sample(x, s, {"angles": [np.pi / 2, 0.0, 0.0]})
    # coords' = Rx^T g: axis-1 / axis-2 plane rotated
    ref = np.rot90(x, k=1, axes=(1, 2))
    if np.abs(out - ref).max() > 1e-4:
        ref = np.rot90(x, k=-1, axes=(1, 2))
    assert np.abs(out - ref).max() < 1e-4
    assert np.array_equal(so, np.rot90(s, k=1, axes=(1, 2))) or np.array_equal(so, np.rot90(s, k=-1, axes=(1, 2)))


def test_oracle_identity_and_unit_scale():
    rng = np.random.default_rng(3)
    x = rng.standard_normal((8, 9, 10)).astype(np.float32)
    s = (rng.random((8, 9, 10)) < 0.3).astype(np.float32)
    out, so = A.augment_sample(x, s, {})
    assert np.array_equal(out, x) and np.array_equal(so, s)
    out, so = A.augment_sample(x, s, {"scale": 1.0})
    assert np.abs(out - x).max() < 1e-5 and np.array_equal(so, s)


def test_spatial_transform_from_batchgenerators_like_compose():
    """create_dataloaders picks the SpatialTransform_2 out of the conf's Compose factory."""
    from cgan3d_amd.data.augment import SpatialTransform_2
    from cgan3d_amd.trainer.utils import spatial_transform_from

    class SpatialTransform_2_bg:  # attribute layout of batchgenerators' transform
        pass
    bg = SpatialTransform_2_bg()
    for k, v in REF_ARGS.items():
        setattr(bg, k, v)
    bg.order_data, bg.border_mode_data, bg.order_seg, bg.border_mode_seg, bg.border_cval_seg = 3, "nearest", 0, \
        "constant", 0
    SpatialTransform_2_bg.__name__ = "SpatialTransform_2"

    class Compose:
        def __init__(self, ts):
            self.transforms = ts
    t = spatial_transform_from(lambda: Compose([bg, object()]))
    assert isinstance(t, SpatialTransform_2) and t.p_el_per_sample == 0.1 and t.scale == (0.7, 1.4)
    assert spatial_transform_from(None) is None
    with pytest.raises(NotImplementedError):
        SpatialTransform_2((8, 8, 8), random_crop=True)


def test_overrides_module_swaps_the_loader_factory():
    """integration/cgan3d_gp_overrides.py rebinds train.py's ``train_u`` (train.py:18,131) to a shim
    whose create_dataloaders is the PatchLoader factory."""
    import importlib.util
    from pathlib import Path
    from cgan3d_amd.trainer import utils as ours
    p = Path(__file__).resolve().parents[1] / "integration" / "cgan3d_gp_overrides.py"
    spec = importlib.util.spec_from_file_location("cgan3d_gp_overrides_t", p)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    assert m.train_u.create_dataloaders is ours.create_dataloaders


def test_transforms_from_conf_2d_like_compose():
    """create_dataloaders takes conf_2D's train_transform (conf_2D.py:36-43): SpatialTransform_2 then
    MirrorTransform(axes=(0, 1), p_per_sample=0.5), NumpyToTensor dropped — in order, from
    batchgenerators-shaped instances; the 2-D draws keep augment_spatial_2's order (one angle)."""
    from cgan3d_amd.data.augment import MirrorTransform, SpatialTransform_2
    from cgan3d_amd.trainer.utils import transforms_from
    from oracle import augment_ref as A

    def bg(name, **attrs):
        cls = type(name, (), {})
        o = cls()
        for k, v in attrs.items():
            setattr(o, k, v)
        return o
    rot = dict(angle_x=(-2 * np.pi, 2 * np.pi), angle_y=(-2 * np.pi, 2 * np.pi), angle_z=(-2 * np.pi, 2 * np.pi))
    sp = bg("SpatialTransform_2", patch_size=(32, 32), random_crop=False, do_elastic_deform=False, do_scale=False,
            do_rotation=True, p_rot_per_sample=0.5, order_data=3, border_mode_data="nearest", order_seg=0,
            border_mode_seg="constant", border_cval_seg=0, **rot)
    mi = bg("MirrorTransform", axes=(0, 1), data_key="data", label_key="seg", p_per_sample=0.5)

    class Compose:
        def __init__(self, ts):
            self.transforms = ts
    ts = transforms_from(Compose([sp, mi, bg("NumpyToTensor"), bg("NumpyToTensor")]))
    assert [type(t) for t in ts] == [SpatialTransform_2, MirrorTransform]
    assert ts[0].patch_size == (32, 32) and ts[1].axes == (0, 1) and ts[1].p_per_sample == 0.5
    prm, noise, gauss = ts[0].draw(np.random.default_rng(4), 12)
    want = A.spatial_2_decisions(np.random.default_rng(4).random, 12, 2, p_rot_per_sample=0.5, do_scale=False, **rot)
    assert [d.get("angles") for d in ts[0].last_decisions] == [d.get("angles") for d in want]
    assert noise is None and gauss is None and set(prm[:, 12]) <= {-1.0, -2.0}
    rotated = prm[:, 12] == -1
    assert rotated.any() and not rotated.all()
    assert np.allclose(prm[rotated, 0], 1) and np.allclose(prm[rotated][:, [1, 2, 3, 6]], 0)
    with pytest.raises(NotImplementedError):
        SpatialTransform_2((16, 16), random_crop=False)  # 2-D elastic deformation (on by default)
