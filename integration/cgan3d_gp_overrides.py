"""``--conf-overwrites`` module for the reference's ``train.py`` (contrast_gan_3D/train.py:97-107,
218-223): routes the gradient-penalty experiment onto the MI355X HIP step.

    python contrast_gan_3D/train.py --conf-overwrites /path/to/repo/integration/cgan3d_gp_overrides.py

``train.py`` does ``globals().update(vars(<this module>))`` before it builds the Trainer
(train.py:106-107, 154-176), so every name defined here replaces the experiment's: the model
factories, the HU loss class, the ``Trainer`` class itself and ``train_u`` (whose
``create_dataloaders`` then builds the pinned-host -> HBM PatchLoaders with the GPU spatial
augmentation of the experiment's ``train_transform``).  The optimizer partials, LR schedulers,
batch sizes, transform parameters and logger of the experiment are left untouched.
"""
import sys
from functools import partial
from pathlib import Path

from torch import nn

_PKG = Path(__file__).resolve().parents[1] / "contrast-gan-3d_amd"
if str(_PKG) not in sys.path:
    sys.path.insert(0, str(_PKG))

import cgan3d_amd  # noqa: E402

# the step's streams each get a hardware queue (cgan3d_amd/__init__.py); train.py imports this module
# before it touches the GPU (train.py:97-107 run before the Trainer is built)
cgan3d_amd.configure_hw_queues()

from cgan3d_amd.model.discriminator import PatchGANDiscriminator  # noqa: E402
from cgan3d_amd.model.generator import ResnetGenerator  # noqa: E402
from cgan3d_amd.model.loss import HULoss  # noqa: E402,F401  (train.py:166 instantiates it)
from cgan3d_amd.trainer.Trainer import Trainer as _HipTrainer  # noqa: E402

# experiments/basic_conf.py:49-54 and :60-66, gradient_penalty_conf.py:7-15
generator_args = dict(n_resnet_blocks=4, n_updownsample_blocks=2, init_channels_out=16)
critic_args = dict(channels_in=1, init_channels_out=8, discriminator_depth=3, negative_slope=0.2,
                   norm_layer=nn.Identity)
generator_class = partial(ResnetGenerator, **generator_args)
critic_class = partial(PatchGANDiscriminator, **critic_args)
weight_clip = None
gp_weight = 10

# "f32" reproduces the reference's arithmetic; "bf16" runs the convolutions on bf16 MFMA
Trainer = partial(_HipTrainer, precision="f32")


class _TrainUtilsShim:
    """Stand-in for train.py's module global ``train_u`` (``from contrast_gan_3D.trainer import
    utils as train_u``, train.py:18): ``create_dataloaders`` (train.py:131) builds the pinned-host ->
    HBM PatchLoaders with the GPU spatial augmentation; every other attribute (config_from_globals,
    global_overrides, ...) is the reference module's own."""

    def __init__(self):
        from cgan3d_amd.trainer import utils as _ours
        self.create_dataloaders = _ours.create_dataloaders

    def __getattr__(self, name):
        from contrast_gan_3D.trainer import utils as _ref
        return getattr(_ref, name)


train_u = _TrainUtilsShim()
