"""Debug: the GP-resample step test at (3, 2) under each CGAN3D_DEBUG comparator (pass / first lines)."""
import os
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import test_gpu_step as T  # noqa: E402

for flag in ["", "serial", "no_bn_fuse", "keep_fp32", "no_shadow", "fp32_store", "no_bn_fold", "no_defer_reduce",
             "no_wgrad_sk", "serial,no_bn_fuse,no_bn_fold"]:
    os.environ["CGAN3D_DEBUG"] = flag
    try:
        T.test_step_gp_resampled_batches_match_oracle(3, 2)
        print(repr(flag), "PASS", flush=True)
    except AssertionError as ex:
        lines = str(ex).split("\n")
        print(repr(flag), "FAIL", len(lines), lines[0][:160], flush=True)
