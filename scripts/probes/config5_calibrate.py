"""Calibration runs for tests/test_config5_gpu.py: engine and torch-oracle accuracy curves of the
small config 5 (Dirichlet(0.5), FedProx, one peer killed in round 1) at a few data sizes / seeds."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

from test_config5_gpu import _run  # noqa: E402

from myfyp_amd.utils.utils import set_test_settings  # noqa: E402

set_test_settings()
n, sim, rounds = int(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3])
for fused, seed in ((True, 1), (True, 2), (False, 1), (False, 2), (False, 3)):
    loss, curve = _run(fused, seed, rounds=rounds, n_per_peer=n, similarity=sim)
    print(f"n={n} sim={sim} fused={fused} seed={seed} acc {np.round(curve, 3).tolist()} loss {np.round(loss, 3).tolist()}", flush=True)
