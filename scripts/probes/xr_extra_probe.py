"""Probe: relative update errors of the fp32 epoch with FedProx / SCAFFOLD terms at every owner K
split (layout 1), against torch — the test_f32_fedprox_scaffold_terms_match_torch setup, printing
every parameter's error instead of asserting."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import test_mlp_f32_gpu as T  # noqa: E402
from myfyp_amd.parallel.mlp_engine import MLPGroup  # noqa: E402

dev = torch.device("cuda", 0)
for kind in sys.argv[1].split(","):
    for ks in [int(k) for k in sys.argv[2].split(",")]:
        MLPGroup.reset_all()
        spec = {"fedprox": {"name": "sgd", "lr": 1e-3, "momentum": 0.9}, "fedprox0": {"name": "sgd", "lr": 1e-3, "momentum": 0.9},
                "scaffold": {"name": "sgd", "lr": 1e-4}, "scaffold0": {"name": "sgd", "lr": 1e-4},
                "sgdm": {"name": "sgd", "lr": 1e-3, "momentum": 0.9}, "adam": {"name": "adam", "lr": 1e-3}}[kind]
        learners, refs, g, n = T._setup(dev, int(os.environ.get("PEERS", "2")), 64, 900, 5, spec, scale=0.5)
        g.force_f32_ks = ks
        g.force_f32_variant = 1
        assert g.f32_ks() == ks, (g.f32_ks(), ks)
        perms = T._pin_perms(dev, g, learners, n)
        p0 = [[p.detach().clone() for p in l.model.get_model().parameters()] for l in learners]
        gen = torch.Generator(device="cpu").manual_seed(9)
        extras = []
        for l in learners:
            flat = l.flat_params().detach()
            if kind == "fedprox":
                extras.append({"anchor": (flat + 0.01 * torch.randn(flat.shape, generator=gen).to(dev)).contiguous(), "mu": 0.5})
            elif kind == "fedprox0":  # the EXTRA path with a zero term: mu = 0
                extras.append({"anchor": (flat + 0.01 * torch.randn(flat.shape, generator=gen).to(dev)).contiguous(), "mu": 0.0})
            elif kind == "scaffold0":  # c_global == c_local: zero correction
                c = 0.1 * torch.randn(flat.shape, generator=gen).to(dev)
                extras.append({"c_global": c, "c_local": c.clone()})
            elif kind == "scaffold":
                extras.append({"c_global": 0.1 * torch.randn(flat.shape, generator=gen).to(dev), "c_local": 0.1 * torch.randn(flat.shape, generator=gen).to(dev)})
            else:
                extras.append(None)
        T._fit_all(learners, extras if extras[0] is not None else None)
        errs = []
        for i, l in enumerate(learners):
            x, y = l.device_data(True)
            T._torch_reference(refs[i], x, y, [perms[(0, i)]], 64, spec, 1, extra=extras[i])
            errs.append([round(T._rel_update(pe, pr, pz), 6) for (name, pe), pr, pz in zip(l.model.get_model().named_parameters(), refs[i].parameters(), p0[i])])
        print(f"{kind} ks={ks} persistent={g.uses_persistent()} var={g.f32_variant()} ks_used={g.f32_ks()} plain_pub={os.environ.get('MYFYP_F32_PLAIN_PUB', '1')} errs={errs}", flush=True)
