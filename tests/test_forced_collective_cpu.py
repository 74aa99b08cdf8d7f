"""CPU rehearsal of the forced-collective mode (``MYFYP_FORCE_COLLECTIVE=1``): a single process
takes every multi-rank weights-plane path through a world-size-1 gloo group (the GPU version,
``test_rccl_forced_gpu.py``, runs it through RCCL); results equal the solo fast paths."""

import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, forced: bool):
    out = str(tmp_path / f"out_{int(forced)}.pt")
    env = dict(os.environ, MYFYP_FORCE_COLLECTIVE="1" if forced else "0", OUT=out, AGG_DEVICE="cpu", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    env.pop("MASTER_PORT", None)
    res = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "workers", "forced_collective_worker.py")], capture_output=True, text=True,
                         timeout=240, cwd=ROOT, env=env)
    assert res.returncode == 0, res.stdout[-3000:] + res.stderr[-5000:]
    with open(out + ".json") as f:
        return torch.load(out, weights_only=True), json.load(f)


def test_forced_world1_gloo_matches_solo(tmp_path):
    solo, _ = _run(tmp_path, False)
    forced, info = _run(tmp_path, True)
    assert info["forced"] and info["backend"] == "gloo"
    for case, c in info["cases"].items():
        assert not c["solo"], case
    assert set(solo) == set(forced)
    for case in solo:
        torch.testing.assert_close(forced[case], solo[case], rtol=0, atol=1e-6, msg=case)
