"""Run the same fp32-engine fit twice from identical weights / batches: results must be bitwise
identical (no atomics in the numerics path). Differences point at a hand-off race."""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import test_mlp_f32_gpu as T  # noqa: E402

from myfyp_amd.parallel.mlp_engine import MLPGroup  # noqa: E402
from myfyp_amd.settings import Settings  # noqa: E402

dev = torch.device("cuda")
Settings.MLP_PRECISION, Settings.GANG_WINDOW = "fp32", 5.0
for B in (32, 64):
    res = []
    for rep in range(3):
        MLPGroup.reset_all()
        spec = {"name": "adam", "lr": 1e-3}
        learners, refs, g, n = T._setup(dev, 2, B, 1400, 3, spec)
        T._pin_perms(dev, g, learners, n)
        T._fit_all(learners)
        res.append([[p.detach().clone() for p in l.model.get_model().parameters()] for l in learners])
    for rep in (1, 2):
        for i in range(2):
            diffs = [(a != b).sum().item() for a, b in zip(res[0][i], res[rep][i])]
            print(f"B{B} run0-vs-run{rep} peer{i} differing elements per tensor: {diffs}", flush=True)
