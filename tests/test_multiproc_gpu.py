"""Multi-process GPU rehearsal (pytest -m gpu): 2 torch.distributed ranks on ONE MI355X, each with
2 co-located peers on the fused MLP engine, cross-rank FedAvg through the weights plane
(parallel/weights_plane.py) over gloo (RCCL refuses two ranks per device). The worker processes are
started before this process touches the GPU, and never by exec from a GPU-initialised process."""
import json
import os
import subprocess
import sys

import pytest

from _ports import free_port

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_two_ranks_fused_engine_cross_rank_fedavg(precision):
    env = dict(os.environ, MYFYP_DIST_BACKEND="gloo", MP_PRECISION=precision, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.join(ROOT, "tests", "_mp_fused_worker.py")]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert res.returncode == 0, res.stderr[-4000:]
    out = json.loads([l for l in res.stdout.splitlines() if l.startswith("{")][-1])
    assert out["world"] == 2 and out["peers"] == 4 and out["fused"], out
    assert out["max_diff"] < 1e-6, out  # every peer holds the same FedAvg model after the last round
    assert out["moved"] > 1e-3, out  # and it trained
    # the last round's aggregate is the host float64 sample-weighted mean of the 4 trained rows
    assert out["n_pre"] == 4 and out["wsum"] > 0, out
    assert out["fedavg_err"] <= 1e-6 * max(1.0, out["fedavg_scale"]), out
