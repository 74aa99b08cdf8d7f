"""Per-parameter (and per W1 column block) relative update error of the fp32 engine vs torch fp32
Adam after one epoch: localises a numerics regression to a layer / K step."""
import os
import sys

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch  # noqa: E402

import test_mlp_f32_gpu as T  # noqa: E402
from myfyp_amd.parallel.mlp_engine import MLPGroup  # noqa: E402
from myfyp_amd.settings import Settings  # noqa: E402

Settings.MLP_PRECISION, Settings.GANG_WINDOW, Settings.USE_FUSED_KERNELS = "fp32", 5.0, True
MLPGroup.reset_all()
dev = torch.device("cuda")
spec = {"name": os.environ.get("OPT", "sgd"), "lr": 1e-3}
steps = int(os.environ.get("STEPS", "1"))
peers = int(os.environ.get("PEERS", "1"))
ntr = int(os.environ.get("NTRAIN", str(64 * steps * peers)))
learners, refs, g, n = T._setup(dev, peers, 64, ntr, 3, spec)
perms = T._pin_perms(dev, g, learners, n)
p0 = [[p.detach().clone() for p in l.model.get_model().parameters()] for l in learners]
T._fit_all(learners)
_ = [l.evaluate() for l in learners]
print("recoveries", g.recoveries())
for i in range(peers):
    x, y = learners[i].device_data(True)
    T._torch_reference(refs[i], x, y, [perms[(0, i)]], 64, spec, 1)
    print("peer", i, "n", n[i])
    for (name, pe), pr, pz in zip(learners[i].model.get_model().named_parameters(), refs[i].parameters(), p0[i]):
        print(f"  {name:18s} rel {T._rel_update(pe, pr, pz):.3e}")
for (name, pe), pr, pz in zip(learners[0].model.get_model().named_parameters(), refs[0].parameters(), p0[0]):
    print(f"{name:18s} rel {T._rel_update(pe, pr, pz):.3e}")
    if name == "layers.0.weight":
        de, dr = (pe - pz).double(), (pr - pz).double()
        for s0 in range(0, 784, 32):
            blk = slice(s0, min(784, s0 + 32))
            e = (de[:, blk] - dr[:, blk]).norm() / (dr[:, blk].norm() + 1e-30)
            print(f"   K step {s0 // 32:2d} cols {s0:3d}..{min(784, s0 + 32) - 1:3d}: rel {e.item():.3e}")
        for o in range(0, 256, 16):
            e = (de[o:o + 16] - dr[o:o + 16]).norm() / (dr[o:o + 16].norm() + 1e-30)
            print(f"   owner rows {o:3d}..{o + 15:3d}: rel {e.item():.3e}")
if os.environ.get("DETAIL"):
    for (name, pe), pr, pz in zip(learners[0].model.get_model().named_parameters(), refs[0].parameters(), p0[0]):
        if name in ("layers.0.weight", "layers.0.bias"):
            de, dr = (pe - pz).detach().flatten(), (pr - pz).detach().flatten()
            idx = torch.arange(0, de.numel(), max(1, de.numel() // 12))[:12]
            print(name, "engine", [f"{v:.2e}" for v in de[idx].tolist()])
            print(name, "torch ", [f"{v:.2e}" for v in dr[idx].tolist()])
            ratio = (de / dr.where(dr.abs() > 0, torch.ones_like(dr)))
            print(name, "ratio median", float(ratio.median()), "frac zero engine", float((de == 0).float().mean()), "frac zero torch", float((dr == 0).float().mean()))
