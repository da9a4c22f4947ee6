"""Is the bench line's ``f32`` sub-object (8.3 ms/step) slower than the standalone ``--precision f32``
line (5.2 ms/step) because of how it is timed or because it runs after the bf16 engine in the same
process?  Times bench.sub_config(64, 4, "f32") in a fresh process, then again after a bf16 engine of
the default workload has been built and stepped.

    python tools/f32_sub_probe.py
"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "contrast-gan-3d_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda")
    g_args = dict(n_resnet_blocks=4, n_updownsample_blocks=2, init_channels_out=16)
    print("fresh process:", bench.sub_config(64, 4, "f32", dev, g_args)["ms_per_step"], "ms/step", flush=True)
    print("again:", bench.sub_config(64, 4, "f32", dev, g_args)["ms_per_step"], "ms/step", flush=True)
    print("bf16 sub_config:", bench.sub_config(64, 4, "bf16", dev, g_args)["ms_per_step"], "ms/step", flush=True)
    print("f32 after bf16:", bench.sub_config(64, 4, "f32", dev, g_args)["ms_per_step"], "ms/step", flush=True)


if __name__ == "__main__":
    main()
