"""Calibration of tests/test_config5_gpu.py's FIXED bounds: per-round training
loss and accuracy curves of the small config 5 for the HIP engine and the torch fp32 oracle over
several seeds. ``MYFYP_DEBUG_LR_SCALE=1.05`` in the environment gives the mutated engine.

    python scripts/probes/config5_calibrate2.py e1 e2 t1 t2   # e = engine, t = torch; digit = seed
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

from test_config5_gpu import _run  # noqa: E402

from myfyp_amd.utils.utils import set_test_settings  # noqa: E402

set_test_settings()
scale = os.environ.get("MYFYP_DEBUG_LR_SCALE", "1")
for spec in sys.argv[1:]:
    fused, seed = spec[0] == "e", int(spec[1:])
    loss, curve = _run(fused, seed)
    print(f"scale={scale} fused={fused} seed={seed} acc {np.round(curve, 4).tolist()} loss {np.round(loss, 4).tolist()}", flush=True)
