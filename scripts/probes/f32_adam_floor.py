"""Adam trajectory sensitivity to fp32 summation order: torch fp32 (GPU) vs the same run with each
batch's rows permuted (identical math, different rounding), vs torch on CPU, vs the fp32 engine."""
import copy
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import test_mlp_f32_gpu as T  # noqa: E402

from myfyp_amd.parallel.mlp_engine import MLPGroup  # noqa: E402
from myfyp_amd.settings import Settings  # noqa: E402

dev = torch.device("cuda")
Settings.MLP_PRECISION, Settings.GANG_WINDOW = "fp32", 5.0


def shuffled_perms(perms, B, seed):
    out = []
    g = torch.Generator().manual_seed(seed)
    for p in perms:
        q = p.clone()
        for s in range(0, q.numel(), B):
            blk = q[s : s + B]
            q[s : s + B] = blk[torch.randperm(blk.numel(), generator=g)]
        out.append(q)
    return out


for B, epochs, n_train, seed, scale, wd in [(64, 1, 1400, 3, 1.0, 0.0), (64, 2, 1400, 3, 1.0, 0.0), (32, 1, 1400, 3, 1.0, 0.0), (64, 1, 900, 4, 0.5, 1e-2)]:
    MLPGroup.reset_all()
    spec = {"name": "adam", "lr": 1e-3, "weight_decay": wd}
    learners, refs, g, n = T._setup(dev, 2, B, n_train, seed, spec, scale=scale)
    perms = T._pin_perms(dev, g, learners, n)
    p0 = [[p.detach().clone() for p in l.model.get_model().parameters()] for l in learners]
    for l in learners:
        l.set_epochs(epochs)
    T._fit_all(learners)
    for i, l in enumerate(learners):
        x, y = l.device_data(True)
        pl = [perms[(ep, i)] for ep in range(epochs)]
        r_a = refs[i]
        r_b = copy.deepcopy(r_a)
        r_c = copy.deepcopy(r_a).cpu()
        T._torch_reference(r_a, x, y, pl, B, spec, epochs)
        T._torch_reference(r_b, x, y, shuffled_perms(pl, B, 7), B, spec, epochs)
        T._torch_reference(r_c, x.cpu(), y.cpu(), pl, B, spec, epochs)
        for (name, pe), pa, pb, pc, pz in zip(l.model.get_model().named_parameters(), r_a.parameters(), r_b.parameters(), r_c.parameters(), p0[i]):
            print(f"B{B} ep{epochs} wd{wd} peer{i} {name:16s} eng-t32 {T._rel_update(pe, pa, pz):.2e}  t32-t32perm {T._rel_update(pb, pa, pz):.2e}  "
                  f"t32gpu-t32cpu {T._rel_update(pc.to(dev), pa, pz):.2e}", flush=True)
