"""Single step, B=32, peer 1 (the case where Adam flips update signs): gradients at the worst
coordinates from the engine (SGD lr=1 => grad = -delta), torch fp32 and fp64; plus the largest
absolute gradient errors of each tensor and the ReLU margins of the units involved."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import test_mlp_f32_gpu as T  # noqa: E402

from myfyp_amd.parallel.mlp_engine import MLPGroup  # noqa: E402
from myfyp_amd.settings import Settings  # noqa: E402

dev = torch.device("cuda")
Settings.MLP_PRECISION, Settings.GANG_WINDOW = "fp32", 5.0
B = 32
MLPGroup.reset_all()
spec = {"name": "sgd", "lr": 1.0}
learners, refs, g, n = T._setup(dev, 2, B, 2 * B, 3, spec)
perms = T._pin_perms(dev, g, learners, n)
p0 = [[p.detach().clone() for p in l.model.get_model().parameters()] for l in learners]
T._fit_all(learners)


def grads(params, x, y, dtype):
    ps = [p.detach().to(dtype).requires_grad_(True) for p in params]
    h = x.reshape(x.shape[0], -1).to(dtype)
    pre = []
    for k in range(0, len(ps), 2):
        h = h @ ps[k].t() + ps[k + 1]
        pre.append(h.detach())
        if k < len(ps) - 2:
            h = torch.relu(h)
    F.cross_entropy(torch.log_softmax(h, 1), y).backward()
    return [p.grad for p in ps], pre


for i in (0, 1):
    l = learners[i]
    x, y = l.device_data(True)
    idx = perms[(0, i)].to(dev)
    xb, yb = x[idx], y[idx]
    g32, pre32 = grads(p0[i], xb, yb, torch.float32)
    g64, pre64 = grads(p0[i], xb, yb, torch.float64)
    ge = [(pz - pe.detach()) for pe, pz in zip(l.model.get_model().parameters(), p0[i])]
    for k in range(6):
        e_eng = (ge[k].double() - g64[k]).abs()
        e_t32 = (g32[k].double() - g64[k]).abs()
        print(f"peer{i} t{k}: max|err| eng {e_eng.max().item():.2e} t32 {e_t32.max().item():.2e}  mean eng {e_eng.mean().item():.2e} t32 {e_t32.mean().item():.2e}")
        top = torch.topk(e_eng.flatten(), 3).indices.tolist()
        for j in top:
            print(f"    @{j}: eng {ge[k].flatten()[j].item():+.6e} t32 {g32[k].flatten()[j].item():+.6e} t64 {g64[k].flatten()[j].item():+.6e}")
    # pre-activation margins
    for L in range(2):
        m = pre64[L].abs().min().item()
        d = (pre32[L].double() - pre64[L]).abs().max().item()
        print(f"peer{i} layer{L} min|preact| {m:.3e}  t32 preact max err {d:.2e}")

# the coordinates whose single-step Adam update flipped sign (f32_adam_steps.py, steps 1 peer1)
i = 1
l = learners[i]
x, y = l.device_data(True)
idx = perms[(0, i)].to(dev)
xb, yb = x[idx].reshape(B, -1).double(), y[idx]
g32, pre32 = grads(p0[i], x[idx], yb, torch.float32)
g64, pre64 = grads(p0[i], x[idx], yb, torch.float64)
ge = [(pz - pe.detach()) for pe, pz in zip(l.model.get_model().parameters(), p0[i])]
for k, j in ((0, 26776), (2, 27080)):
    print(f"t{k}@{j}: eng {ge[k].flatten()[j].item():+.6e} t32 {g32[k].flatten()[j].item():+.6e} t64 {g64[k].flatten()[j].item():+.6e}")
o1, kk = divmod(26776, 784)
print("X column nonzeros:", xb[:, kk].nonzero().flatten().tolist(), xb[:, kk][xb[:, kk] != 0].tolist())
print("preact layer0 unit", o1, pre64[0][:, o1].tolist())
o2, o1b = divmod(27080, 256)
print("W2 coord rows", o2, o1b, "H1 col:", torch.relu(pre64[0][:, o1b]).tolist())
print("preact layer1 unit", o2, pre64[1][:, o2].tolist())
