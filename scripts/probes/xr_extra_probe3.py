"""Probe: the fp32 epoch's update error against torch for EVERY parameter, owner K split from argv,
the FedProx extra path with a zero term (mu = 0) vs without extras; MYFYP_F32_XR_EXTRA=1 lets the
extra-term epoch run at K split 4 / 8. Errors: |Δ_engine - Δ_torch|_1 / |Δ_torch|_1 per tensor."""
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
peers = int(os.environ.get("PEERS", "2"))
mom = float(os.environ.get("MOM", "0.9"))
for ks in [int(k) for k in sys.argv[1].split(",")]:
    for extra_on in (False, True):
        MLPGroup.reset_all()
        spec = {"name": "sgd", "lr": 1e-3, "momentum": mom}
        learners, refs, g, n = T._setup(dev, peers, 64, 900, 5, spec, scale=0.5)
        g.force_f32_ks = ks
        g.force_f32_variant = 1
        perms = T._pin_perms(dev, g, learners, n)
        p0 = [[p.detach().clone() for p in l.model.get_model().parameters()] for l in learners]
        extras = [{"anchor": l.flat_params().detach().clone().contiguous(), "mu": 0.0} for l in learners] if extra_on else None
        T._fit_all(learners, extras)
        used = g.f32_ks()
        for i, l in enumerate(learners[:1]):
            x, y = l.device_data(True)
            T._torch_reference(refs[i], x, y, [perms[(0, i)]], 64, spec, 1, extra=None)
            errs = []
            for (name, pe), pr, pz in zip(l.model.get_model().named_parameters(), refs[i].parameters(), p0[i]):
                de, dr = (pe.detach() - pz), (pr.detach() - pz)
                errs.append(f"{name} {float((de - dr).abs().sum() / dr.abs().sum().clamp_min(1e-30)):.2e}")
            print(f"ks={ks} used={used} extra={extra_on} peers={peers} mom={mom} plain={os.environ.get('MYFYP_F32_PLAIN_PUB', '1')}: " + ", ".join(errs), flush=True)
