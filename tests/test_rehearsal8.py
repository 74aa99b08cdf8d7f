"""The headline's multi-GPU process layout rehearsed on the CPU: 8 ranks, one
small-MLP peer each, the collective workflow over gloo + the shared-memory control plane
(SURVEY §7.3's 8-peer slice; reference convergence case: /root/reference/test/node_test.py:79-132).
The 8-GPU run itself is the driver's; this pins the protocol at its rank count."""
import json
import os
import subprocess
import sys

import pytest

from _ports import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch(tmp_path, **env_extra):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OUT_DIR=str(tmp_path), OMP_NUM_THREADS="1", **env_extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.join(ROOT, "tests", "workers", "rehearsal8_worker.py")]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    hung = [f for f in sorted(tmp_path.glob("hang_*.txt")) if f.stat().st_size]

    def learning_stack(text: str) -> str:  # control-plane state + the learning thread's innermost frames
        head = "".join(l + "\n" for l in text.splitlines() if l.startswith("shm gen"))
        for block in text.split("\n\n"):
            if "_start_learning" in block:
                return head + "\n".join(block.splitlines()[:6])
        return head + text[:600]

    hangs = "".join(f"--- {f.name}\n{learning_stack(f.read_text())}\n" for f in hung)
    assert res.returncode == 0, hangs + res.stdout[-2000:] + res.stderr[-2000:]
    return {json.loads(f.read_text())["rank"]: json.loads(f.read_text()) for f in tmp_path.glob("rank*.json")}


@pytest.mark.slow
def test_eight_ranks_finish_with_equal_models(tmp_path):
    outs = _launch(tmp_path, ROUNDS="4")
    assert set(outs) == set(range(8))
    for o in outs.values():
        assert o["finished_rounds"] == 4 and o["members"] == list(range(8)) and o["recoveries"] == 0, o
    sums = [o["checksum"] for o in outs.values()]
    assert max(sums) - min(sums) < 1e-3 * max(1.0, abs(sums[0])), sums
    cp = outs[0]["control_plane"]
    assert cp["cp_gather"]["n"] >= 4 and cp["cp_sync_members"]["n"] >= 4, cp


@pytest.mark.slow
def test_eight_ranks_rank5_dies_inside_the_all_reduce(tmp_path):
    """Rank 5's process exits right before it issues round 2's FedAvg all-reduce, when the other
    seven are already inside it: the survivors notice, agree, rebuild their groups over the seven
    and re-run the aggregation, and finish every round within 60 s (no timeout waited out)."""
    outs = _launch(tmp_path, ROUNDS="4", KILL_RANK="5", KILL_ROUND="2")
    survivors = [r for r in range(8) if r != 5]
    assert set(outs) == set(survivors)
    for o in outs.values():
        assert o["finished_rounds"] == 4 and o["members"] == survivors, o
        assert o["recoveries"] >= 1 and o["elapsed"] < 60, o
    sums = [o["checksum"] for o in outs.values()]
    assert max(sums) - min(sums) < 1e-3 * max(1.0, abs(sums[0])), sums
