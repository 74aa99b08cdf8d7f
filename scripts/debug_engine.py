"""Diagnose the fused MLP engine: per-parameter gradient error after ONE SGD step vs autograd."""
import copy, sys, threading
import torch, torch.nn.functional as F
sys.path.insert(0, ".")
from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
from myfyp_amd.learning.frameworks.torch import TorchLearner, TorchModel
from myfyp_amd.models import MLP
from myfyp_amd.parallel.mlp_engine import MLPGroup
from myfyp_amd.settings import Settings

dev = torch.device("cuda")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
P = int(sys.argv[2]) if len(sys.argv) > 2 else 1
Settings.GANG_WINDOW = 2.0
data = synthetic_mnist(B * P, 64, seed=7)
parts = data.generate_partitions(P, RandomIIDPartitionStrategy)
lr = 1e-3
learners, refs = [], []
for i in range(P):
    m = MLP(seed=3 + i)
    m.optimizer_spec = lambda: {"name": "sgd", "lr": lr}
    refs.append(copy.deepcopy(m).to(dev))
    learners.append(TorchLearner(TorchModel(m), parts[i], f"p{i}", batch_size=B))
g = learners[0]._engine.group
n = [parts[i].get_num_samples() for i in range(P)]
perms = [torch.arange(n[i]) for i in range(P)]
def perm_fn(ep):
    out = torch.zeros(g.capacity, g.nmax, dtype=torch.int32)
    for i, l in enumerate(learners):
        out[l._engine.slot, : n[i]] = perms[i].to(torch.int32)
    return out.to(dev)
g.perm_fn = perm_fn
p0s = [[p.detach().clone() for p in l.model.get_model().parameters()] for l in learners]
ts = [threading.Thread(target=l.fit) for l in learners]
[t.start() for t in ts]; [t.join() for t in ts]
torch.cuda.synchronize()
for i in range(P):
    x, y = learners[i].device_data(True)
    idx = perms[i][:B].to(dev)
    refs[i].zero_grad()
    out = refs[i](x[idx])
    loss = F.cross_entropy(out, y[idx])
    loss.backward()
    print(f"peer {i} ref loss {loss.item():.4f} rows {min(B, n[i])}")
    for (name, pe), pr, pz in zip(learners[i].model.get_model().named_parameters(), refs[i].parameters(), p0s[i]):
        ge = (pz - pe.detach()) / lr
        gr = pr.grad
        rel = (ge - gr).norm() / (gr.norm() + 1e-12)
        cos = torch.nn.functional.cosine_similarity(ge.flatten(), gr.flatten(), dim=0)
        ratio = ge.norm() / (gr.norm() + 1e-12)
        print(f"  {name:18s} rel_err {rel:.4f} cos {cos:.4f} norm_ratio {ratio:.4f}")
    # forward check on train batch: compare engine eval loss path later
MLPGroup.reset_all()
