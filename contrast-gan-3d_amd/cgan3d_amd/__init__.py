"""MI355X-native G+D training step of contrast-gan-3D (HIP kernels behind include/cgan3d.h).

Hardware queues: the step runs a main and a side stream, and under data parallelism a
communication stream plus RCCL's own.  With HIP's default of 4 hardware queues per process some of
them share an in-order queue, where one stream's cross-stream wait blocks another's kernels (one
GPU, one-rank RCCL path: 2.56 ms/step at 4 queues, 2.21 at 8).  HIP reads GPU_MAX_HW_QUEUES when it
initialises, so importing this package before the first GPU call raises it to 8 (a user's larger
value is kept); bench.py reports the value in force.
"""
import os as _os

if int(_os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
    _os.environ["GPU_MAX_HW_QUEUES"] = "8"
