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
the generator on the HIP kernels.

``correct_scan_2D`` (reference :83-99): the 2-D generator (experiments/conf_2D.py) over the scan's
axial slices (the last axis, CCTAEvalDataset2D), ``batch_size`` slices per batch, stacked back to
the scan's shape.  When no patch size (or a 2-D one) is given the reference sets the inference
patch size to (512, 512), as here.

Upsampler (reference :42-52): when the generator's output shape for the inference patch differs
from the patch (patch dims that are not multiples of 4: the stride-2 convs round up, the
transposed convs double), the output is resized to the patch with nn.Upsample's default
nearest-neighbour rule (source index floor(i * in / out)) before ``patch - G(patch)``.
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


def model_output_shape(model: nn.Module, patch: Sequence[int]) -> Tuple[int, ...]:
    """Spatial output shape of the generator for ``patch`` (compute_convolution_filters_shape,
    reference model/utils.py:70-95, through convolution_output_shape's arithmetic)."""
    shape = tuple(int(p) for p in patch)
    for m in model.modules():
        if isinstance(m, (nn.ConvTranspose3d, nn.ConvTranspose2d)):
            k, p, s, op = m.kernel_size[0], m.padding[0], m.stride[0], m.output_padding[0]
            shape = tuple((x - 1) * s - 2 * p + k + op for x in shape)
        elif isinstance(m, (nn.Conv3d, nn.Conv2d)):
            k, p, s = m.kernel_size[0], m.padding[0], m.stride[0]
            shape = tuple((x + 2 * p - k) // s + 1 for x in shape)
    return shape


def nearest_resize(t: Tensor, size: Sequence[int]) -> Tensor:
    """nn.Upsample(size=size) (mode "nearest") on [N, C, *spatial]: source index floor(i * in / out)
    per axis — an index gather."""
    out = t
    for a, n_out in enumerate(size):
        ax = 2 + a
        n_in = out.shape[ax]
        if n_in == n_out:
            continue
        # float32 scale and product, as aten's nearest_neighbor_compute_source_index
        src = np.floor(np.arange(n_out, dtype=np.float32) * np.float32(n_in / n_out)).astype(np.int64)
        idx = torch.from_numpy(np.minimum(src, n_in - 1))
        out = out.index_select(ax, idx.to(out.device))
    return out


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
        self.correct_scan = self.correct_scan_3D
        if self.inference_patch_size is None or len(self.inference_patch_size) < 3:
            self.correct_scan = self.correct_scan_2D
            self.inference_patch_size = (512, 512)
        self.inference_patch_size = tuple(int(p) for p in self.inference_patch_size)
        out = model_output_shape(self.model, self.inference_patch_size)
        self.upsampler = (lambda t: t) if out == self.inference_patch_size else \
            (lambda t, size=self.inference_patch_size: nearest_resize(t, size))

    def load_model(self, checkpoint_path: Union[str, Path]):
        ckpt = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
        self.model.load_state_dict(ckpt["generator"])
        self.checkpoint_path = Path(checkpoint_path)

    def _scale(self, x: np.ndarray) -> np.ndarray:
        # float32 first, as CCTAEvalDataset2D/3D do (ccta.astype(np.float32)): an int16 scan would
        # otherwise wrap in the scaler's shift (x - 238 below -32530) and round differently
        x = np.asarray(x, dtype=np.float32)
        return np.asarray(self.scaler(x), dtype=np.float32) if self.scaler is not None else x

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
            corrected = patch - self.upsampler(self.model(patch))  # CCTAEvalDataset3D item -> patch - G(patch) (:77-79)
            ops.patch_accumulate(corrected.contiguous(), torch.tensor(chunk, dtype=torch.int32, device=self.device),
                                 out, weight)
        ops.patch_normalize(out, weight)
        return out

    @torch.no_grad()
    def correct_scan_2D(self, ccta: np.ndarray, batch_size: int, desc: Optional[str] = None) -> Tensor:
        """The scan's slices along its last axis through the 2-D generator (reference :83-99):
        output [1, *ccta.shape]."""
        nsl = ccta.shape[-1]
        out = torch.empty((nsl, 1, *ccta.shape[:-1]), device=self.device)
        for i in range(0, nsl, batch_size):
            host = np.stack([self._scale(np.ascontiguousarray(ccta[..., j])) for j in range(i, min(nsl, i + batch_size))])
            batch = torch.from_numpy(host[:, None])
            batch = batch.pin_memory().to(self.device, non_blocking=True) if self.device.type == "cuda" else batch
            out[i:i + len(host)] = batch - self.upsampler(self.model(batch))
        return out.permute(1, 2, 3, 0)

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
        16 channels) for a 3-D patch size, conf_2D's (is_2D, 6 ResNet blocks) otherwise, and
        FactorZeroCenterScaler(238, 600) unless given."""
        from functools import partial
        from ..model.generator import ResnetGenerator
        if generator_class is None:
            if inference_patch_size is None or len(inference_patch_size) < 3:
                generator_class = partial(ResnetGenerator, n_resnet_blocks=6, n_updownsample_blocks=2,
                                          init_channels_out=16, is_2D=True)
            else:
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
