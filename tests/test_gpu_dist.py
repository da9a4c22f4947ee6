"""Data-parallel step under a launch plan, two ranks sharing one GPU (gloo over GPU tensors; the
8-GPU bench runs the same plan with RCCL): tools/dist_plan_check.py asserts identical weights on
both ranks after three plan-replayed steps and the two host collectives between the plan's C
segments (engine.StepEngine._allreduce / ops.plan_host)."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]


def test_two_rank_plan_step():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", "29517", str(REPO / "tools" / "dist_plan_check.py")]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=110)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "rank 0: ok" in out and "rank 1: ok" in out, out[-4000:]


@pytest.mark.parametrize("torch_comm", ["0", "1"])
def test_rccl_bucketed_path_one_rank(torch_comm):
    """The RCCL path itself (bucketed async all-reduces on a communication stream, inside a launch
    plan) on a one-rank nccl group: tools/dist_nccl1_check.py (the mean over one rank is exact) —
    through RCCL calls recorded in the plan on the process group's own communicator (default:
    ops.NativeComm over ProcessGroupNCCL's ncclComm_t), and through torch.distributed host callables
    (CGAN3D_COMM=torch, the documented fallback)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="2953" + torch_comm,
               CGAN3D_COMM="torch" if torch_comm == "1" else "native")
    r = subprocess.run([sys.executable, str(REPO / "tools" / "dist_nccl1_check.py")], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=110)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "path ok" in out, out[-4000:]
