"""FedProx (Adam, mu 0.5) through the fp32 persistent epoch at owner K splits 1 and 2 vs torch fp32:
per-parameter relative update error, count of coordinates off by > lr/2, and where the W1 ones sit
(column -> K step of 32 -> K part). Separates a split-specific bug (a whole K step / part wrong)
from Adam amplifying fp32 rounding differences at coordinates whose gradient nearly cancels; also
compares engine and torch fp32 against an fp64 run, and torch fp32 against itself restarted from
weights one ulp away (the chaos check behind the SGD choice in test_f32_fedprox_scaffold_terms_*)."""
import importlib.util
import os
import sys
from collections import Counter

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
spec_ = importlib.util.spec_from_file_location("t32", os.path.join(ROOT, "tests", "test_mlp_f32_gpu.py"))
t = importlib.util.module_from_spec(spec_)
spec_.loader.exec_module(t)

from myfyp_amd.ops import _native  # noqa: E402
from myfyp_amd.parallel.mlp_engine import MLPGroup  # noqa: E402
from myfyp_amd.settings import Settings  # noqa: E402

_native.load(required=True)
dev = torch.device("cuda")
Settings.MLP_PRECISION, Settings.GANG_WINDOW, Settings.USE_FUSED_KERNELS = "fp32", 5.0, True
for kind in sys.argv[1:] or ["fedprox"]:
    for ks in (1, 2):
        MLPGroup.reset_all()
        spec = {"fedprox": {"name": "adam", "lr": 1e-3}, "fedprox_sgd": {"name": "sgd", "lr": 1e-3}, "scaffold_adam": {"name": "adam", "lr": 1e-3}}.get(
            kind, {"name": "adam", "lr": 1e-3, "weight_decay": 1e-2})
        learners, refs, g, n = t._setup(dev, 2, 64, 900, 5, spec, scale=0.5)
        g.force_f32_ks = ks
        assert g.f32_ks() == ks
        perms = t._pin_perms(dev, g, learners, n)
        p0 = [[p.detach().clone() for p in l.model.get_model().parameters()] for l in learners]
        gen = torch.Generator(device="cpu").manual_seed(9)
        extras = []
        for l in learners:
            flat = l.flat_params().detach()
            if kind.startswith("fedprox"):
                extras.append({"anchor": (flat + 0.01 * torch.randn(flat.shape, generator=gen).to(dev)).contiguous(), "mu": 0.5})
            elif kind == "scaffold_adam":
                extras.append({"c_global": 0.1 * torch.randn(flat.shape, generator=gen).to(dev), "c_local": 0.1 * torch.randn(flat.shape, generator=gen).to(dev)})
            else:
                extras.append(None)
        has_extra = extras[0] is not None
        t._fit_all(learners, extras if has_extra else None)
        import copy as _copy
        refs64 = [_copy.deepcopy(r).double() for r in refs]
        for m64 in refs64:
            def _fwd(x, m64=m64):
                h = x.reshape(x.shape[0], -1).double()
                for layer in m64.layers:
                    h = layer(h)
                return torch.log_softmax(h, dim=1)
            m64.forward = _fwd
        for i, l in enumerate(learners):
            x, y = l.device_data(True)
            ex64 = None if extras[i] is None else {k: (v.double() if torch.is_tensor(v) else v) for k, v in extras[i].items()}
            t._torch_reference(refs64[i], x.double(), y, [perms[(0, i)]], 64, spec, 1, extra=ex64)
            # chaos check: the same fp32 torch run from weights nudged by one ulp
            nudged = _copy.deepcopy(refs[i])
            with torch.no_grad():
                for q in nudged.parameters():
                    q.copy_(torch.nextafter(q, torch.full_like(q, float("inf"))))
            t._torch_reference(refs[i], x, y, [perms[(0, i)]], 64, spec, 1, extra=extras[i])
            t._torch_reference(nudged, x, y, [perms[(0, i)]], 64, spec, 1, extra=extras[i])
            for (name, pr), pn, pz in zip(refs[i].named_parameters(), nudged.parameters(), p0[i]):
                print(f"  ulp-nudged torch vs torch {kind} peer {i} {name:18s} {t._rel_update(pn, pr, pz):.2e}", flush=True)
            for (name, pe), pr, p64, pz in zip(l.model.get_model().named_parameters(), refs[i].parameters(), refs64[i].parameters(), p0[i]):
                print(f"  vs fp64 {kind} ks={ks} peer {i} {name:18s} engine {t._rel_update(pe, p64, pz):.2e} torch-fp32 {t._rel_update(pr, p64, pz):.2e}", flush=True)
            for (name, pe), pr, pz in zip(l.model.get_model().named_parameters(), refs[i].parameters(), p0[i]):
                rel = t._rel_update(pe, pr, pz)
                d = ((pe.detach() - pz) - (pr.detach() - pz)).abs()
                bad = (d > 0.5 * spec["lr"]).nonzero()
                where = ""
                if name == "layers.0.weight" and len(bad):
                    cols = bad[:, 1].tolist()
                    where = f" K steps {sorted(Counter(c // 32 for c in cols).items())[:12]} rows {sorted(Counter(r // 16 for r in bad[:, 0].tolist()).items())[:8]}"
                print(f"{kind} ks={ks} peer {i} {name:18s} rel {rel:.2e} off>lr/2: {len(bad)} / {d.numel()} max {d.max().item():.2e}{where}", flush=True)
MLPGroup.reset_all()
