"""MI355X-native G+D training step of contrast-gan-3D (HIP kernels behind include/cgan3d.h).

Hardware queues: the step runs a main and a side stream, and under data parallelism a
communication stream plus RCCL's own.  With HIP's default of 4 hardware queues per process some of
them share an in-order queue, where one stream's cross-stream wait blocks another's kernels (one
GPU, one-rank RCCL path: 2.56 ms/step at 4 queues, 2.21 at 8; the single-GPU step without
collectives is the same at either setting).  HIP reads GPU_MAX_HW_QUEUES once, when it initialises,
so the setting belongs to the program's entry point: ``configure_hw_queues()`` raises it before the
first GPU call (bench.py and integration/cgan3d_gp_overrides.py call it).  Importing the package
changes nothing in the process environment; a data-parallel StepEngine warns when fewer than 8
queues are in force.
"""
import os as _os
import warnings as _warnings

HW_QUEUES = 8


def configure_hw_queues(n: int = HW_QUEUES) -> int:
    """Raise GPU_MAX_HW_QUEUES to ``n`` (a larger user value is kept) if HIP has not initialised in
    this process yet; otherwise warn that the setting cannot apply.  Returns the value in force."""
    cur = int(_os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    if cur >= n:
        return cur
    try:
        import torch
        initialised = torch.cuda.is_initialized()
    except Exception:  # pragma: no cover - torch always present in this package's environment
        initialised = False
    if initialised:
        _warnings.warn(f"cgan3d_amd.configure_hw_queues: HIP is already initialised with GPU_MAX_HW_QUEUES={cur}; "
                       f"call it before the first GPU use for {n} queues", RuntimeWarning, stacklevel=2)
        return cur
    _os.environ["GPU_MAX_HW_QUEUES"] = str(n)
    return n
