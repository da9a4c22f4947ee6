"""LayerNorm critic (experiments/gp_layernorm.py:9-11) host-side checks, CPU only: the module's
configuration gate and LayerNorm shape check, and a dry-run StepEngine step with the LayerNorm
critic and the gradient penalty (ops.DRY_RUN: every launch's operand sizes, dtypes and contiguity
are checked on the host; the kernels are no-ops) — the arithmetic is checked on the GPU
(tests/test_gpu_step.py, fixture step_gp_layernorm)."""
import pytest
import torch
from torch import nn

D_ARGS = dict(channels_in=1, init_channels_out=8, discriminator_depth=3, negative_slope=0.2)


def _ln_critic(S=32, **kw):
    from cgan3d_amd.model.discriminator import PatchGANDiscriminator
    args = dict(norm_layer=nn.LayerNorm, patch_size=(1, S, S, S), elementwise_affine=False)
    args.update(kw)
    return PatchGANDiscriminator(**D_ARGS, **args)


def test_layernorm_critic_state_dict_matches_reference_layout():
    d = _ln_critic()
    assert d.config.norm == "layer" and d._unsupported is None
    # no conv bias in the middle blocks, no LayerNorm parameters (elementwise_affine=False)
    assert [k for k in d.state_dict()] == ["model.first.conv.weight", "model.first.conv.bias",
                                           "model.middle.0.conv.weight", "model.middle.1.conv.weight",
                                           "model.middle.2.conv.weight", "model.last.weight", "model.last.bias"]
    assert tuple(d.model.middle[0].normalization.normalized_shape) == (16, 8, 8, 8)


def test_layernorm_critic_gates():
    assert _ln_critic(elementwise_affine=True)._unsupported  # affine LayerNorm: not the conf's
    d = _ln_critic(S=32)
    with pytest.raises(RuntimeError, match="normalized_shape"):
        d._check_layernorm_shape([64, 64, 64])  # a LayerNorm built for 32^3 patches, fed 64^3
    d._check_layernorm_shape([32, 32, 32])


def test_layernorm_gp_step_dry_run():
    from cgan3d_amd import ops
    from cgan3d_amd.engine import StepEngine
    from cgan3d_amd.model.generator import ResnetGenerator
    g = ResnetGenerator(1, 2, 8)
    d = _ln_critic()
    old = ops.DRY_RUN
    ops.DRY_RUN = True
    try:
        eng = StepEngine(g, d, g.config, d.config, 2, 2, (32, 32, 32), device=torch.device("cpu"))
        assert eng.D.ln and eng.use_gp
        eng.step()
        eng.record()  # the plan path records the same launches
    finally:
        ops.DRY_RUN = old
