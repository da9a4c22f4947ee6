"""CCTAContrastCorrector — drop-in for ``contrast_gan_3D/eval/CCTAContrastCorrector.py:24-139``
(whole-scan inference with the trained generator), 3-D path, on the HIP generator.

``correct_scan_3D`` (reference :60-81) tiles the scan with patchly's ``GridSampler`` (step = patch,
squeeze mode: the last patch of a dim is moved back to end at the border, overlapping its
neighbour), runs ``patch - G(patch)`` on scaled patches, and averages overlapping outputs with
patchly's ``Aggregator``.

BatchNorm mode.  The reference never calls ``model.eval()`` (reference :33-38): its generator stays in
train mode, so every batch of tiles is normalised with ITS OWN batch statistics and every batch
updates the running buffers (momentum 0.1) — the output of a tile depends on the other tiles of its
batch.  This is the default here too (same C-order batching of the grid, same ``batch_size``).
``eval_mode=True`` is a build-only option (not in the reference): running statistics, batch
independent, buffers untouched.  patchly is a dependency of the reference outside its tree
(not installed here); its grid and averaging are restated here: ``grid_origins`` on the host, the
patch accumulation and the average in HIP (``cgan3d_patch_accumulate`` / ``cgan3d_patch_normalize``),
the generator on the HIP kernels.  The 2-D path (``correct_scan_2D``) belongs to the 2-D variants
 and raises.
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass, field
from pathlib import Path
from typing import Callable, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch
from torch import Tensor, nn

from .. import ops


def grid_origins(shape: Sequence[int], patch: Sequence[int], step: Optional[Sequence[int]] = None) -> List[Tuple]:
    """patchly GridSampler (squeeze mode) patch origins, C order: per dim 0, step, 2 step, ... while
    the patch fits, plus one patch ending at the border when the last one stops short."""
    step = tuple(step or patch)
    per_dim = []
    for s, p, t in zip(shape, patch, step):
        if p > s:
            raise ValueError(f"grid_origins: patch {tuple(patch)} larger than the scan {tuple(shape)}")
        o = list(range(0, s - p + 1, t))
        if o[-1] + p < s:
            o.append(s - p)
        per_dim.append(o)
    return list(itertools.product(*per_dim))


@dataclass
class CCTAContrastCorrector:
    model: Callable[[], nn.Module]
    scaler: object
    device: torch.device
    inference_patch_size: Optional[Sequence[int]] = None
    checkpoint_path: Optional[Path] = None
    upsampler: Callable[[Tensor], Tensor] = field(init=False, default=None)
    eval_mode: bool = False  # build-only option: eval-mode BatchNorm (see the module docstring)

    def __post_init__(self):
        self.model: nn.Module = self.model()
        if self.checkpoint_path is not None:
            self.load_model(self.checkpoint_path)
        self.device = torch.device(self.device)
        # the reference leaves the module in its default train mode (reference :33-38)
        self.model = self.model.to(self.device)
        if self.eval_mode:
            self.model.eval()
        if self.inference_patch_size is None or len(self.inference_patch_size) < 3:
            raise NotImplementedError("CCTAContrastCorrector: the 2-D path is SURVEY.md §8f row 4")
        self.inference_patch_size = tuple(int(p) for p in self.inference_patch_size)
        self.correct_scan = self.correct_scan_3D

    def load_model(self, checkpoint_path: Union[str, Path]):
        ckpt = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
        self.model.load_state_dict(ckpt["generator"])
        self.checkpoint_path = Path(checkpoint_path)

    def _scale(self, x: np.ndarray) -> np.ndarray:
        return np.asarray(self.scaler(x), dtype=np.float32) if self.scaler is not None else x.astype(np.float32)

    @torch.no_grad()
    def correct_scan_3D(self, ccta: np.ndarray, batch_size: int, desc: Optional[str] = None) -> Tensor:
        shape, ps = tuple(ccta.shape), self.inference_patch_size
        orgs = grid_origins(shape, ps)
        out = torch.zeros((1, *shape), device=self.device)
        weight = torch.zeros((1, *shape), device=self.device)
        stream = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None
        for b0 in range(0, len(orgs), batch_size):
            chunk = orgs[b0:b0 + batch_size]
            host = np.stack([self._scale(ccta[o[0]:o[0] + ps[0], o[1]:o[1] + ps[1], o[2]:o[2] + ps[2]])
                             for o in chunk])[:, None]
            patch = torch.from_numpy(host).pin_memory().to(self.device, non_blocking=True) if stream else \
                torch.from_numpy(host).to(self.device)
            corrected = patch - self.model(patch)  # CCTAEvalDataset3D item -> patch - G(patch) (:77-79)
            ops.patch_accumulate(corrected.contiguous(), torch.tensor(chunk, dtype=torch.int32, device=self.device),
                                 out, weight)
        ops.patch_normalize(out, weight)
        return out

    @torch.no_grad()
    def __call__(self, ccta: np.ndarray, batch_size: int = 16, **kwargs) -> Tensor:
        corrected = self.correct_scan(ccta, batch_size, **kwargs)
        unscale = getattr(self.scaler, "unscale", None)
        if unscale is not None:
            corrected = unscale(corrected)
        return corrected.squeeze().detach().cpu()

    @classmethod
    def from_checkpoint(cls, inference_patch_size, device, checkpoint_path, generator_class=None, scaler=None):
        """As the reference's (:124-139): the basic conf's generator (4 ResNet blocks, 2 up/down,
        16 channels) and FactorZeroCenterScaler(238, 600) unless given."""
        from functools import partial
        from ..model.generator import ResnetGenerator
        if generator_class is None:
            generator_class = partial(ResnetGenerator, n_resnet_blocks=4, n_updownsample_blocks=2,
                                      init_channels_out=16)
        if scaler is None:
            scaler = _FactorZeroCenterScaler(238, 600)
        return cls(generator_class, scaler, device, inference_patch_size=inference_patch_size,
                   checkpoint_path=checkpoint_path)


class _FactorZeroCenterScaler:
    """contrast_gan_3D/data/Scaler.py:37-48: (x - shift) / factor and its inverse."""

    def __init__(self, shift, factor):
        self.shift, self.factor = shift, factor

    def __call__(self, x):
        return (x - self.shift) / self.factor

    def unscale(self, x):
        return x * self.factor + self.shift
