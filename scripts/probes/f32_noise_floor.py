"""fp32 engine vs torch fp32 vs torch fp64: relative update errors per tensor (one/two epochs, Adam).
Separates the engine's error from fp32's own noise floor (Adam sign-normalises tiny gradients)."""
import copy
import sys
import threading

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import test_mlp_f32_gpu as T  # noqa: E402

from myfyp_amd.parallel.mlp_engine import MLPGroup  # noqa: E402
from myfyp_amd.settings import Settings  # noqa: E402

dev = torch.device("cuda")
Settings.MLP_PRECISION, Settings.GANG_WINDOW = "fp32", 5.0
for B, epochs, lr in [(64, 1, 1e-3), (64, 2, 1e-3), (32, 1, 1e-3), (64, 1, 1e-4)]:
    MLPGroup.reset_all()
    spec = {"name": "adam", "lr": lr}
    learners, refs, g, n = T._setup(dev, 2, B, 1400, 3, spec)
    perms = T._pin_perms(dev, g, learners, n)
    p0 = [[p.detach().clone() for p in l.model.get_model().parameters()] for l in learners]
    for l in learners:
        l.set_epochs(epochs)
    T._fit_all(learners)
    for i, l in enumerate(learners):
        x, y = l.device_data(True)
        r32 = refs[i]
        r64 = copy.deepcopy(r32).double()
        r64.forward = (lambda m: (lambda xx: torch.log_softmax(torch.nn.Sequential(*m.layers)(xx.reshape(xx.shape[0], -1).double()), dim=1)))(r64)
        T._torch_reference(r32, x, y, [perms[(ep, i)] for ep in range(epochs)], B, spec, epochs)
        # fp64 reference (inputs cast to double)
        T._torch_reference(r64, x, y, [perms[(ep, i)] for ep in range(epochs)], B, spec, epochs)
        for (name, pe), pr, pd, pz in zip(l.model.get_model().named_parameters(), r32.parameters(), r64.parameters(), p0[i]):
            print(f"B{B} ep{epochs} lr{lr} peer{i} {name:18s} eng-vs-t32 {T._rel_update(pe, pr, pz):.2e}  "
                  f"eng-vs-t64 {T._rel_update(pe, pd, pz):.2e}  t32-vs-t64 {T._rel_update(pr, pd, pz):.2e}", flush=True)
