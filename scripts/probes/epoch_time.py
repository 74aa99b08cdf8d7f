"""GPU time of one fused epoch (hipGraph replay) for 8 grouped peers: events around run_epoch."""
import os, sys, threading
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
from myfyp_amd.learning.frameworks.torch import TorchModel
from myfyp_amd.learning.frameworks.torch.torch_learner import TorchLearner
from myfyp_amd.models import MLP
from myfyp_amd.ops import _native
from myfyp_amd.settings import Settings
Settings.USE_FUSED_KERNELS = True
P, B = int(os.environ.get("PEERS", 8)), 64
parts = synthetic_mnist(60000, 10000, seed=1).generate_partitions(P, RandomIIDPartitionStrategy)
ls = [TorchLearner(TorchModel(MLP(seed=i)), parts[i], f"p{i}", batch_size=B, device="cuda") for i in range(P)]
g = ls[0]._engine.group
for it in range(3):
    ths = [threading.Thread(target=l.fit) for l in ls]
    [t.start() for t in ths]; [t.join() for t in ths]
torch.cuda.synchronize()
lib = _native.load(required=True)
stream = torch.cuda.current_stream().cuda_stream
t0 = np.zeros(g.capacity, dtype=np.int32)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
times = []
for rep in range(10):
    e0.record()
    lib.mlp_engine_run_epoch(g._engine, t0.ctypes.data, stream)
    e1.record()
    torch.cuda.synchronize()
    times.append(e0.elapsed_time(e1))
steps = g.max_steps
print(f"peers={P} steps/epoch={steps} epoch ms median={np.median(times):.3f} -> us/step={1000*np.median(times)/steps:.2f}")
