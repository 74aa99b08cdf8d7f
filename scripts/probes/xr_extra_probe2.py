"""Probe: where (which W1 column range / which b1 entries) the fp32 epoch's update differs from
torch at a given owner K split, EXTRA path with a zero term (FedProx mu = 0)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_mlp_f32_gpu as T  # noqa: E402
from myfyp_amd.parallel.mlp_engine import MLPGroup  # noqa: E402

dev = torch.device("cuda", 0)
for ks in [int(k) for k in sys.argv[1].split(",")]:
    for extra_on in (False, True):
        MLPGroup.reset_all()
        spec = {"name": "sgd", "lr": 1e-3, "momentum": 0.9}
        learners, refs, g, n = T._setup(dev, 2, 64, 900, 5, spec, scale=0.5)
        g.force_f32_ks = ks
        g.force_f32_variant = 1
        perms = T._pin_perms(dev, g, learners, n)
        p0 = [[p.detach().clone() for p in l.model.get_model().parameters()] for l in learners]
        extras = [{"anchor": l.flat_params().detach().clone().contiguous(), "mu": 0.0} for l in learners] if extra_on else None
        T._fit_all(learners, extras)
        l = learners[0]
        x, y = l.device_data(True)
        T._torch_reference(refs[0], x, y, [perms[(0, 0)]], 64, spec, 1, extra=None)
        pe = [p.detach() for p in l.model.get_model().parameters()]
        pr = [p.detach() for p in refs[0].parameters()]
        dW = ((pe[0] - p0[0][0]) - (pr[0] - p0[0][0])).abs().cpu().numpy()  # [256, 784]
        rW = (pr[0] - p0[0][0]).abs().cpu().numpy()
        db = ((pe[1] - p0[0][1]) - (pr[1] - p0[0][1])).abs().cpu().numpy()
        rb = (pr[1] - p0[0][1]).abs().cpu().numpy()
        # per K step (32 columns) and per column group (16 rows)
        kerr = [float(dW[:, 32 * s : 32 * s + 32].sum() / max(1e-30, rW[:, 32 * s : 32 * s + 32].sum())) for s in range(25)]
        cerr = [float(dW[16 * c : 16 * c + 16].sum() / max(1e-30, rW[16 * c : 16 * c + 16].sum())) for c in range(16)]
        berr = [float(db[16 * c : 16 * c + 16].sum() / max(1e-30, rb[16 * c : 16 * c + 16].sum())) for c in range(16)]
        print(f"ks={ks} extra={extra_on} W1 err by K step {np.round(kerr, 4).tolist()}", flush=True)
        print(f"ks={ks} extra={extra_on} W1 err by col group {np.round(cerr, 4).tolist()}", flush=True)
        print(f"ks={ks} extra={extra_on} b1 err by col group {np.round(berr, 4).tolist()}", flush=True)
