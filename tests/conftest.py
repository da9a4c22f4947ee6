"""Test configuration: markers, import paths, shared helpers.

``-m "not gpu"`` runs here (no GPU): the oracle against the reference's golden fixtures, the
host-side logic, the multi-rank (gloo) paths and the C-ABI library's symbol table.
``-m gpu`` runs on an MI355X: the HIP path against the oracle through the C-ABI.
"""
import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "contrast-gan-3d_amd"))
GOLDEN = REPO / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = dict(np.load(GOLDEN / f"{name}.npz", allow_pickle=False))
        return cache[name]
    return load


def assert_close(actual, expected, rtol=1e-3, name="", atol=0.0):
    """Parity bar (north_star: 'within 1e-3 relative fp32 tolerance'), scale-aware:
    max|a-e| <= rtol * max|e| + atol and ||a-e||_2 <= rtol * ||e||_2 + atol * sqrt(n).
    ``atol`` is only for quantities that are exactly zero in real arithmetic (e.g. the critic's
    last bias gradient, d/db [mean(D(fake)) - mean(D(real))] = 1 - 1)."""
    import numpy as np
    a = np.asarray(actual, dtype=np.float64)
    e = np.asarray(expected, dtype=np.float64)
    assert a.shape == e.shape, f"{name}: shape {a.shape} != {e.shape}"
    scale = max(float(np.abs(e).max()) if e.size else 0.0, 1e-30)
    err = float(np.abs(a - e).max()) if e.size else 0.0
    nrm = float(np.linalg.norm(e))
    dif = float(np.linalg.norm(a - e))
    ok = err <= rtol * scale + atol and dif <= rtol * nrm + atol * np.sqrt(max(e.size, 1))
    assert ok, (f"{name}: max abs err {err:.3e} (scale {scale:.3e}), rel L2 {dif / (nrm or 1e-30):.3e} "
                f"> {rtol} (atol {atol})")
