"""Deterministic, framework-independent parameter initialisation (PCG64 recipe).

Used by the parity fixtures (``tests/golden/make_golden.py``) and the benchmark so that the
reference modules and this package's modules — which share ``state_dict`` keys — start from
bit-identical weights without storing them.  Bounds follow torch's default conv init scale
(``1/sqrt(fan_in)``, fan_in = ``weight[0].numel()``, which is also what torch uses for
``ConvTranspose3d``'s ``[Cin, Cout, k, k, k]`` weights); BatchNorm affine parameters are
randomised away from (1, 0) so the tests exercise them; running buffers keep torch's
defaults (mean 0, var 1, 0 batches tracked).
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch


def pcg64_state_dict(named_shapes, seed: int) -> "OrderedDict[str, np.ndarray]":
    """``named_shapes``: iterable of (state_dict key, shape).  Returns numpy arrays."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = OrderedDict()
    last_fan_in = 1
    for name, shape in named_shapes:
        shape = tuple(shape)
        if name.endswith("running_mean"):
            out[name] = np.zeros(shape, np.float32)
        elif name.endswith("running_var"):
            out[name] = np.ones(shape, np.float32)
        elif name.endswith("num_batches_tracked"):
            out[name] = np.zeros(shape, np.int64)
        elif ".normalization." in name and name.endswith("weight"):
            out[name] = rng.uniform(0.5, 1.5, shape).astype(np.float32)
        elif ".normalization." in name and name.endswith("bias"):
            out[name] = rng.uniform(-0.2, 0.2, shape).astype(np.float32)
        elif len(shape) >= 3:
            last_fan_in = int(np.prod(shape[1:]))
            b = 1.0 / np.sqrt(last_fan_in)
            out[name] = rng.uniform(-b, b, shape).astype(np.float32)
        else:  # conv bias
            b = 1.0 / np.sqrt(last_fan_in)
            out[name] = rng.uniform(-b, b, shape).astype(np.float32)
    return out


def pcg64_init_(module: torch.nn.Module, seed: int) -> torch.nn.Module:
    """Load the PCG64 recipe into ``module`` (any module with the reference's keys)."""
    sd = module.state_dict()
    vals = pcg64_state_dict([(k, v.shape) for k, v in sd.items()], seed)
    with torch.no_grad():
        for k, v in sd.items():
            v.copy_(torch.from_numpy(vals[k]).to(v.dtype))
    return module
