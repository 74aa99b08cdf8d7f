"""Per-parameter comparison of one ResNet-18 engine step against torch fp32 autograd."""
import os
import sys
import threading

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch
import torch.nn.functional as F

from test_cnn_engine_gpu import _make_learners, _torch_step
from myfyp_amd.models import ResNet18

batch = int(sys.argv[1]) if len(sys.argv) > 1 else 16
mom = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
learners, refs, parts = _make_learners(lambda i: ResNet18(seed=20 + i), 1, batch, 64, batch, 0.05, mom, 0.0)
g = learners[0]._engine.group
g.perm_fn = lambda ep: torch.arange(g.nmax, dtype=torch.int32, device="cuda").unsqueeze(0).repeat(g.capacity, 1)
ref = refs[0]
before = [p.detach().clone() for p in ref.parameters()]
lr_ = learners[0]
x, y = lr_.device_data(True)
# torch forward with bf16-rounded autocast for a second opinion
loss_eng_steps = lr_.fit()
loss_t = _torch_step(ref, x[:batch], y[:batch], 0.05, mom, 0.0)
print("engine stats loss/sample", float(g.stat.view(g.capacity, 4)[0, 0]) / batch, "torch loss", loss_t)
eng = dict(lr_.model.get_model().named_parameters())
for (name, p_ref), p0 in zip(ref.named_parameters(), before):
    d_ref = (p_ref.detach() - p0).flatten()
    d_eng = (eng[name].detach() - p0).flatten()
    if d_ref.norm() < 1e-10:
        print(f"{name:40s} zero ref update; eng norm {float(d_eng.norm()):.3e}")
        continue
    cos = float(F.cosine_similarity(d_ref, d_eng, dim=0))
    rel = float((d_ref - d_eng).norm() / d_ref.norm())
    print(f"{name:40s} cos {cos:.4f} rel {rel:.4f} |ref| {float(d_ref.norm()):.3e} |eng| {float(d_eng.norm()):.3e}")
