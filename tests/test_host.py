"""Host-side tests (no GPU): C-ABI symbol table, module layout, dry-run shape checks of the step."""
import re
from pathlib import Path

import pytest
import torch
from torch import nn

from conftest import REPO

D_ARGS = dict(channels_in=1, init_channels_out=8, discriminator_depth=3, negative_slope=0.2)


def test_library_exports_every_header_symbol():
    from cgan3d_amd import _lib
    header = (REPO / "include" / "cgan3d.h").read_text()
    declared = set(re.findall(r"\b(cgan3d_[a-z0-9_]+)\s*\(", header))
    assert declared, "no declarations parsed"
    lib = _lib.load()  # loading needs no GPU
    for name in declared:
        assert hasattr(lib, name), f"libcgan3d.so lacks {name}"
    assert declared == set(_lib.exported_symbols()), declared ^ set(_lib.exported_symbols())
    assert lib.cgan3d_version().decode().startswith("cgan3d")


def test_state_dict_layout_matches_reference():
    """Same keys, order and shapes as the reference modules (pinned via the oracle's layout, which
    tests/test_oracle.py checks against the reference's own state_dict order)."""
    from oracle import reference_torch as R
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.generator import ResnetGenerator
    g = ResnetGenerator(4, 2, 16)
    assert [(k, tuple(v.shape)) for k, v in g.state_dict().items()] == list(R.gen_param_shapes(R.GenConfig()).items())
    d = PatchGANDiscriminator(**D_ARGS, norm_layer=nn.Identity)
    assert [(k, tuple(v.shape)) for k, v in d.state_dict().items()] == \
        list(R.critic_param_shapes(R.CriticConfig()).items())
    assert sum(p.numel() for p in g.parameters()) == 1_035_297
    assert sum(p.numel() for p in d.parameters()) == 176_761


@pytest.mark.parametrize("g_args,S,b,clip", [
    (dict(n_resnet_blocks=1, n_updownsample_blocks=2, init_channels_out=8), 32, 1, False),
    (dict(n_resnet_blocks=4, n_updownsample_blocks=2, init_channels_out=16), 64, 4, False),
    (dict(n_resnet_blocks=4, n_updownsample_blocks=2, init_channels_out=16), 32, 2, False),
    (dict(n_resnet_blocks=4, n_updownsample_blocks=2, init_channels_out=16), 64, 4, True),  # BN critic, clip
    (dict(n_resnet_blocks=1, n_updownsample_blocks=2, init_channels_out=8), (32, 40, 48), 2, False),  # anisotropic
    # experiments/conf_2D.py: 2-D generator (6 blocks) and 2-D BatchNorm critic (16 -> 128 channels), clip
    (dict(n_resnet_blocks=6, n_updownsample_blocks=2, init_channels_out=16, is_2D=True), (128, 128), 8, True),
])
def test_engine_step_dry_run_shapes(g_args, S, b, clip):
    """Every launch of a full step gets operands whose extents match the kernel's footprint."""
    from cgan3d_amd import ops
    from cgan3d_amd.engine import StepEngine
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.generator import ResnetGenerator
    g = ResnetGenerator(**g_args)
    is2d = g_args.get("is_2D", False)
    d_args = dict(D_ARGS, init_channels_out=16, is_2D=True) if is2d else D_ARGS
    d = PatchGANDiscriminator(**d_args, **({} if clip else dict(norm_layer=nn.Identity)))
    dims = tuple(S) if isinstance(S, tuple) else (S, S, S)
    ops.DRY_RUN = True
    try:
        eng = StepEngine(g, d, g.config, d.config, b, b, dims, g_hyper=(1e-4, 0.0, 0.9, 1e-8),
                         d_hyper=(1e-4, 0.0, 0.9, 1e-8), device=torch.device("cpu"),
                         weight_clip=0.01 if clip else None)
        eng.step()
    finally:
        ops.DRY_RUN = False
    if is2d:
        assert eng.dims == (1, *S) and eng.G.planar and eng.D.pl
        assert eng.D.layers[-2].cout == 128


@pytest.mark.parametrize("S,b", [(64, 4), ((64, 48, 32), 2)])
def test_bf16_engine_batchnorm_accumulators(S, b):
    """bf16 engine (dry run): every generator BatchNorm layer takes its statistics from fp64
    accumulators its producing conv fills (include/cgan3d.h cgan3d_bn_fuse: halo-tiled, stride-2 and
    k7 kernels) and runs one finalize + elementwise launch per direction; every launch passes the
    host checks, and each elementwise launch zeroes its predecessor's accumulator (the first the
    last one's)."""
    from cgan3d_amd import ops
    from cgan3d_amd.engine import StepEngine
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.generator import ResnetGenerator
    g = ResnetGenerator(4, 2, 16)
    d = PatchGANDiscriminator(**D_ARGS, norm_layer=nn.Identity)
    dims = tuple(S) if isinstance(S, tuple) else (S, S, S)
    ops.DRY_RUN = True
    try:
        eng = StepEngine(g, d, g.config, d.config, b, b, dims, device=torch.device("cpu"), precision="bf16")
        eng.step()
    finally:
        ops.DRY_RUN = False
    G = eng.G
    nl = len(G.layers)
    assert all(G.ac_f) and all(G.ac_b) and G.fold_bn
    fo, bo = list(range(nl)), list(range(nl - 1, -1, -1))
    assert G.acc_zero_f[fo[0]] is G.acc_f[fo[-1]] and all(G.acc_zero_f[fo[k]] is G.acc_f[fo[k - 1]] for k in range(1, nl))
    assert G.acc_zero_b[bo[0]] is G.acc_b[bo[-1]] and all(G.acc_zero_b[bo[k]] is G.acc_b[bo[k - 1]] for k in range(1, nl))


def test_2d_models_match_reference_layout():
    """conf_2D's modules (is_2D): Conv2d / ConvTranspose2d / BatchNorm2d with the reference's keys."""
    from oracle import reference_torch as R
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    from cgan3d_amd.model.generator import ResnetGenerator
    gc = R.GenConfig(6, 2, 16, is_2D=True)
    g = ResnetGenerator(6, 2, 16, is_2D=True)
    assert [(k, tuple(v.shape)) for k, v in g.state_dict().items()] == list(R.gen_param_shapes(gc).items())
    d = PatchGANDiscriminator(1, 16, 3, is_2D=True, negative_slope=0.2)
    dc = R.CriticConfig(init_channels_out=16, norm="batch", is_2D=True)
    assert [(k, tuple(v.shape)) for k, v in d.state_dict().items()] == list(R.critic_param_shapes(dc).items())


def test_conv_wrapper_rejects_mismatched_operand():
    from cgan3d_amd import ops
    g = ops.conv_fwd_geom(1, (8, 8, 8), (8, 8, 8), 16, 16, 3, 1, 1)
    x = torch.empty(1, 8, 8, 8, 16)
    w = torch.empty(16, 16, 3, 3, 3)
    ops.DRY_RUN = True
    try:
        ops.conv(g, x, w, torch.empty(1, 8, 8, 8, 16))
        with pytest.raises(ValueError):
            ops.conv(g, x, w, torch.empty(1, 4, 4, 4, 16))
    finally:
        ops.DRY_RUN = False


def test_conf_overwrites_module_builds_trainer_like_train_py(tmp_path):
    """integration/cgan3d_gp_overrides.py replaces train.py's globals (train.py:106-107); the
    Trainer it exports accepts train.py's positional call (train.py:154-176) and builds the
    reference-shaped models and Adam optimisers (on the CPU here: no kernel runs until a step)."""
    import importlib.util
    from functools import partial
    from pathlib import Path
    spec = importlib.util.spec_from_file_location(
        "cgan3d_gp_overrides", Path(__file__).resolve().parents[1] / "integration" / "cgan3d_gp_overrides.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)

    class _LI:
        logger = None

        def end_hook(self):
            pass

    opt = partial(torch.optim.Adam, lr=1e-4, betas=(0.0, 0.9))
    tr = m.Trainer(10, 2, 400, 5, 1, 100, 500, m.generator_class, m.critic_class, opt, opt,
                   m.HULoss(0.18667, 0.35333, (6, 1, 128, 128, 128)), _LI(), torch.device("cpu"), False,
                   checkpoint_dir=tmp_path, weight_clip=m.weight_clip, generator_lr_scheduler_class=None,
                   critic_lr_scheduler_class=None, checkpoint_every=1000, rng=None)
    from cgan3d_amd.model.utils import count_parameters
    assert count_parameters(tr.generator) == 1035297 and count_parameters(tr.critic) == 176761
    assert set(tr.optimizer_G.state_dict()["param_groups"][0]) >= {"lr", "betas", "eps"}


def test_wgrad_sk_eligibility_follows_the_variant_tiles():
    """cgan3d_conv3d_wgrad_sk_ok (host code, no GPU): the 8 -> 16 variant's tile is 4 x 8 x 16 (d, h, w),
    so an output width that is a multiple of 8 but not of 16 is not eligible (include/cgan3d.h states it,
    ADVICE r05); 16 -> 32 takes 4 x 4 x 8, 32 -> 64 takes 4 x 4 x 4."""
    from cgan3d_amd import ops, _lib as L
    BF = L.PREC_BF16

    def ok(cin, cout, dout):
        din = tuple(2 * d for d in dout)
        return ops.wgrad_sk_ok(ops.with_prec(ops.conv_wgrad_geom(12, din, dout, cin, cout, 4, 2, 1), BF))
    assert ok(8, 16, (16, 16, 16)) and ok(8, 16, (4, 8, 16))
    assert not ok(8, 16, (16, 16, 8)) and not ok(8, 16, (8, 8, 24))
    assert ok(16, 32, (8, 8, 8)) and not ok(16, 32, (8, 8, 4))
    assert ok(32, 64, (4, 4, 4)) and not ok(32, 64, (4, 4, 2))
