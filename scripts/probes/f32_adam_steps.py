"""Adam fp32 engine vs torch fp32 by number of steps; largest-deviation coordinates."""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import test_mlp_f32_gpu as T  # noqa: E402

from myfyp_amd.parallel.mlp_engine import MLPGroup  # noqa: E402
from myfyp_amd.settings import Settings  # noqa: E402

dev = torch.device("cuda")
Settings.MLP_PRECISION, Settings.GANG_WINDOW = "fp32", 5.0
B = 32
for steps in (1, 2, 3, 5, 8, 22):
    MLPGroup.reset_all()
    spec = {"name": "adam", "lr": 1e-3}
    learners, refs, g, n = T._setup(dev, 2, B, 2 * B * steps, 3, spec)
    perms = T._pin_perms(dev, g, learners, n)
    p0 = [[p.detach().clone() for p in l.model.get_model().parameters()] for l in learners]
    T._fit_all(learners)
    for i, l in enumerate(learners):
        x, y = l.device_data(True)
        T._torch_reference(refs[i], x, y, [perms[(0, i)]], B, spec, 1)
        out = []
        for k, (pe, pr, pz) in enumerate(zip(l.model.get_model().parameters(), refs[i].parameters(), p0[i])):
            de, dr = pe.detach() - pz, pr.detach() - pz
            rel = T._rel_update(pe, pr, pz)
            diff = (de - dr).abs().flatten()
            j = int(diff.argmax())
            nbig = int((diff > 1e-4).sum())
            out.append(f"t{k} rel {rel:.1e} n>1e-4 {nbig} max@{j} eng {de.flatten()[j].item():+.3e} ref {dr.flatten()[j].item():+.3e}")
        print(f"steps {steps} peer{i}: " + " | ".join(out), flush=True)
