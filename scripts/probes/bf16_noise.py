"""How far is a bf16-autocast torch ResNet-18 step from the fp32 one? (noise floor for the engine test)"""
import os, sys
sys.path.insert(0, os.getcwd())
import torch, torch.nn.functional as F
from myfyp_amd.models import ResNet18
from myfyp_amd.learning.dataset.synthetic import synthetic_cifar10
batch = int(sys.argv[1]) if len(sys.argv) > 1 else 16
d = synthetic_cifar10(batch, 16, seed=3)
x = torch.from_numpy(d.column("image")).cuda()[:batch]; y = torch.from_numpy(d.column("label")).cuda()[:batch]
def grads(dtype):
    m = ResNet18(seed=20).cuda().train()
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype == "bf16"):
        loss = F.cross_entropy(m(x).float(), y)
    loss.backward()
    return {n: p.grad.detach().clone() for n, p in m.named_parameters()}
g32, g16 = grads("fp32"), grads("bf16")
for n in list(g32)[:12] + list(g32)[-6:]:
    a, b = g32[n].flatten(), g16[n].flatten()
    print(f"{n:36s} cos {float(F.cosine_similarity(a, b, dim=0)):.4f} rel {float((a-b).norm()/a.norm()):.4f}")
