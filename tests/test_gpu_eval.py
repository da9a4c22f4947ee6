"""Whole-scan inference (eval/CCTAContrastCorrector.py, reference eval/CCTAContrastCorrector.py:
60-81): the HIP corrector against the oracle generator (eval mode, float64) tiled and averaged by
a numpy restatement of patchly's squeeze-mode GridSampler + averaging Aggregator (patchly is not
installed: grid and averaging unpinned by the reference itself)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_corrector_matches_oracle():
    from functools import partial
    from oracle import reference_torch as R
    from cgan3d_amd.eval.CCTAContrastCorrector import CCTAContrastCorrector, _FactorZeroCenterScaler, grid_origins
    from cgan3d_amd.model.generator import ResnetGenerator
    from cgan3d_amd.model.init import pcg64_init_
    g_args = dict(n_resnet_blocks=1, n_updownsample_blocks=2, init_channels_out=8)
    gen = pcg64_init_(ResnetGenerator(**g_args), 5)
    with torch.no_grad():  # non-trivial running statistics for eval mode
        for k, v in gen.state_dict().items():
            if k.endswith("running_mean"):
                v.uniform_(-0.2, 0.2)
            elif k.endswith("running_var"):
                v.uniform_(0.5, 1.5)
    sd = {k: v.detach().clone() for k, v in gen.state_dict().items()}
    sc = _FactorZeroCenterScaler(238, 600)
    corr = CCTAContrastCorrector(lambda: gen, sc, torch.device("cuda"), inference_patch_size=(32, 32, 32))
    rng = np.random.default_rng(0)
    scan = (rng.standard_normal((40, 36, 48)) * 200 + 200).astype(np.float32)
    got = corr(scan, batch_size=3).numpy()
    # restatement: every grid patch through the float64 oracle, averaged where patches overlap
    p64 = {k: v.double() if v.is_floating_point() else v for k, v in sd.items()}
    acc = np.zeros(scan.shape)
    cnt = np.zeros(scan.shape)
    for o in grid_origins(scan.shape, (32, 32, 32)):
        sl = tuple(slice(a, a + 32) for a in o)
        x = torch.from_numpy(((scan[sl] - 238) / 600).astype(np.float64))[None, None]
        y = (x - R.generator_forward(p64, x, R.GenConfig(**g_args), training=False))[0, 0].numpy()
        acc[sl] += y
        cnt[sl] += 1
    want = acc / cnt * 600 + 238
    assert got.shape == scan.shape
    err = np.abs(got - want).max() / np.abs(want).max()
    assert err <= 1e-5, err
