"""One fp32-engine SGD step vs fp64 autograd gradient, per tensor (no Adam amplification)."""
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
for B, nsamp in [(64, 64), (64, 50), (32, 32), (64, 128)]:
    MLPGroup.reset_all()
    lr = 1.0
    spec = {"name": "sgd", "lr": lr}
    learners, refs, g, n = T._setup(dev, 2, B, 2 * nsamp, 3, spec, scale=0.5)
    perms = T._pin_perms(dev, g, learners, n)
    p0 = [[p.detach().clone() for p in l.model.get_model().parameters()] for l in learners]
    T._fit_all(learners)
    for i, l in enumerate(learners):
        x, y = l.device_data(True)
        m64 = [p.detach().double().requires_grad_(True) for p in p0[i]]
        idx = perms[(0, i)][:B].to(dev)
        h = x[idx].reshape(len(idx), -1).double()
        for k in range(0, len(m64), 2):
            h = h @ m64[k].t() + m64[k + 1]
            if k < len(m64) - 2:
                h = torch.relu(h)
        loss = F.cross_entropy(torch.log_softmax(h, 1), y[idx])
        loss.backward()
        for k, (pe, pz, pg) in enumerate(zip(l.model.get_model().parameters(), p0[i], m64)):
            ge = (pz.double() - pe.detach().double()) / lr
            gr = pg.grad
            rel = ((ge - gr).norm() / gr.norm()).item()
            err = (ge - gr).abs()
            j = int(err.argmax())
            print(f"B{B} n{nsamp} peer{i} t{k} shape{tuple(pz.shape)} rel {rel:.2e} maxerr {err.max().item():.2e} at {j} ge {ge.flatten()[j].item():.4e} gr {gr.flatten()[j].item():.4e}", flush=True)
