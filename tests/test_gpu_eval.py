"""Whole-scan inference (eval/CCTAContrastCorrector.py, reference eval/CCTAContrastCorrector.py:
60-81): the HIP corrector against the oracle generator (float64) tiled and averaged by a numpy
restatement of patchly's squeeze-mode GridSampler + averaging Aggregator (patchly is not
installed: grid order and averaging unpinned by the reference itself).

Default: the reference's semantics — the generator stays in train mode (the reference never calls
``.eval()``, :33-38), so each DataLoader batch of tiles (C-order grid, ``batch_size`` per batch) is
normalised with its own BatchNorm statistics and updates the running buffers.  The build-only
``eval_mode=True`` option runs eval-mode BatchNorm (running statistics)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

G_ARGS = dict(n_resnet_blocks=1, n_updownsample_blocks=2, init_channels_out=8)


def _generator():
    from cgan3d_amd.model.generator import ResnetGenerator
    from cgan3d_amd.model.init import pcg64_init_
    gen = pcg64_init_(ResnetGenerator(**G_ARGS), 5)
    with torch.no_grad():  # non-trivial running statistics
        for k, v in gen.state_dict().items():
            if k.endswith("running_mean"):
                v.uniform_(-0.2, 0.2)
            elif k.endswith("running_var"):
                v.uniform_(0.5, 1.5)
    return gen


def _oracle(scan, sd, batch_size, training, ps=(32, 32, 32)):
    """patch - G(patch) per C-order batch of grid tiles through the float64 oracle, averaged."""
    from oracle import reference_torch as R
    from cgan3d_amd.eval.CCTAContrastCorrector import grid_origins
    p64 = {k: v.double() if v.is_floating_point() else v.clone() for k, v in sd.items()}
    acc = np.zeros(scan.shape)
    cnt = np.zeros(scan.shape)
    orgs = grid_origins(scan.shape, ps)
    for b0 in range(0, len(orgs), batch_size):
        chunk = orgs[b0:b0 + batch_size]
        sls = [tuple(slice(a, a + p) for a, p in zip(o, ps)) for o in chunk]
        x = torch.from_numpy(np.stack([((scan[sl] - 238) / 600).astype(np.float64) for sl in sls]))[:, None]
        y = (x - R.generator_forward(p64, x, R.GenConfig(**G_ARGS), training=training))[:, 0].numpy()
        for sl, yi in zip(sls, y):
            acc[sl] += yi
            cnt[sl] += 1
    return acc / cnt * 600 + 238, p64


@pytest.mark.parametrize("eval_mode", [False, True])
def test_corrector_matches_oracle(eval_mode):
    from cgan3d_amd.eval.CCTAContrastCorrector import CCTAContrastCorrector, _FactorZeroCenterScaler
    gen = _generator()
    sd = {k: v.detach().clone() for k, v in gen.state_dict().items()}
    corr = CCTAContrastCorrector(lambda: gen, _FactorZeroCenterScaler(238, 600), torch.device("cuda"),
                                 inference_patch_size=(32, 32, 32), eval_mode=eval_mode)
    assert corr.model.training == (not eval_mode)
    rng = np.random.default_rng(0)
    scan = (rng.standard_normal((40, 36, 48)) * 200 + 200).astype(np.float32)
    got = corr(scan, batch_size=3).numpy()  # 8 tiles: batches of 3, 3, 2
    want, p64 = _oracle(scan, sd, 3, training=not eval_mode)
    assert got.shape == scan.shape
    err = np.abs(got - want).max() / np.abs(want).max()
    assert err <= 1e-4, err
    # train mode: the running buffers advanced once per batch, as in the reference
    for k, v in gen.state_dict().items():
        if k.endswith(("running_mean", "running_var")):
            a, e = v.cpu().numpy(), p64[k].numpy()
            assert np.abs(a - e).max() <= 1e-4 * max(np.abs(e).max(), 1.0), k
        elif k.endswith("num_batches_tracked"):
            assert int(v) == int(sd[k]) + (0 if eval_mode else 3), k


def test_corrector_2d_slices_match_oracle():
    """correct_scan_2D (reference :83-99): the scan's last-axis slices through the 2-D generator
    (conf_2D, train-mode BatchNorm per batch of slices) against the float64 oracle."""
    from oracle import reference_torch as R
    from cgan3d_amd.eval.CCTAContrastCorrector import CCTAContrastCorrector, _FactorZeroCenterScaler
    from cgan3d_amd.model.generator import ResnetGenerator
    from cgan3d_amd.model.init import pcg64_init_
    g2 = dict(n_resnet_blocks=2, n_updownsample_blocks=2, init_channels_out=8, is_2D=True)
    gen = pcg64_init_(ResnetGenerator(**g2), 6)
    sd = {k: v.detach().double().clone() if v.is_floating_point() else v.clone() for k, v in gen.state_dict().items()}
    corr = CCTAContrastCorrector(lambda: gen, _FactorZeroCenterScaler(238, 600), torch.device("cuda"))
    assert corr.correct_scan == corr.correct_scan_2D and corr.inference_patch_size == (512, 512)
    rng = np.random.default_rng(2)
    scan = (rng.standard_normal((40, 36, 5)) * 200 + 200).astype(np.float32)
    got = corr(scan, batch_size=2).numpy()
    want = np.empty(scan.shape)
    for i in range(0, 5, 2):
        x = torch.from_numpy(np.stack([(scan[..., j] - 238) / 600 for j in range(i, min(5, i + 2))]).astype(np.float64))
        x = x[:, None]
        y = (x - R.generator_forward(sd, x, R.GenConfig(2, 2, 8, is_2D=True), training=True))[:, 0].numpy()
        for j in range(len(y)):
            want[..., i + j] = y[j] * 600 + 238
    assert got.shape == scan.shape
    err = np.abs(got - want).max() / np.abs(want).max()
    assert err <= 1e-4, err


def test_corrector_upsamples_odd_patches():
    """Inference patch dims that are not multiples of 4 (reference :42-52): the generator's output
    (convolution arithmetic: 30 -> 15 -> 8 -> 16 -> 32) is resized to the patch by nn.Upsample's
    nearest rule before patch - G(patch); checked against the float64 oracle resized by torch's own
    F.interpolate(mode="nearest")."""
    from oracle import reference_torch as R
    from cgan3d_amd.eval.CCTAContrastCorrector import (CCTAContrastCorrector, _FactorZeroCenterScaler, grid_origins,
                                                        model_output_shape)
    gen = _generator()
    sd = {k: v.detach().clone() for k, v in gen.state_dict().items()}
    ps = (30, 32, 28)
    assert model_output_shape(gen, ps) == (32, 32, 28)
    corr = CCTAContrastCorrector(lambda: gen, _FactorZeroCenterScaler(238, 600), torch.device("cuda"),
                                 inference_patch_size=ps, eval_mode=True)
    rng = np.random.default_rng(4)
    scan = (rng.standard_normal((44, 32, 40)) * 200 + 200).astype(np.float32)
    got = corr(scan, batch_size=4).numpy()
    p64 = {k: v.double() if v.is_floating_point() else v.clone() for k, v in sd.items()}
    acc, cnt = np.zeros(scan.shape), np.zeros(scan.shape)
    for o in grid_origins(scan.shape, ps):
        sl = tuple(slice(a, a + p) for a, p in zip(o, ps))
        x = torch.from_numpy(((scan[sl] - 238) / 600).astype(np.float64))[None, None]
        att = R.generator_forward(p64, x, R.GenConfig(**G_ARGS), training=False)
        att = torch.nn.functional.interpolate(att, size=ps, mode="nearest")
        acc[sl] += (x - att)[0, 0].numpy()
        cnt[sl] += 1
    want = acc / cnt * 600 + 238
    err = np.abs(got - want).max() / np.abs(want).max()
    assert err <= 1e-4, err
