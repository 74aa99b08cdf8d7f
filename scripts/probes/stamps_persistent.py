"""Phase timing of the persistent MLP epoch kernel (needs MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so).
8 grouped peers, B = 64, two fits; prints per-step phase durations of peer 0's owner 0 and head."""
import os
import sys
import threading

sys.path.insert(0, os.getcwd())
import numpy as np
import torch

from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
from myfyp_amd.learning.frameworks.torch import TorchModel
from myfyp_amd.learning.frameworks.torch.torch_learner import TorchLearner
from myfyp_amd.models import MLP
from myfyp_amd.ops import _native
from myfyp_amd.settings import Settings

Settings.USE_FUSED_KERNELS = True
lib = _native.load(required=True)
assert hasattr(lib, "mlp_debug_persistent_stamps"), "not the stamped library"
import ctypes

lib.mlp_debug_persistent_stamps.argtypes = [ctypes.c_void_p]
lib.mlp_debug_persistent_stamps.restype = ctypes.c_int
P, B = int(os.environ.get("PEERS", "8")), 64
parts = synthetic_mnist(60000, 10000, seed=1).generate_partitions(8, RandomIIDPartitionStrategy)
ls = []
for i in range(P):
    m = MLP(seed=i)
    if os.environ.get("OPT") == "sgd":
        m.optimizer_spec = lambda: {"name": "sgd", "lr": 1e-3}
    ls.append(TorchLearner(TorchModel(m), parts[i], f"p{i}", batch_size=B, device="cuda"))
g = ls[0]._engine.group
assert g.uses_persistent()
for it in range(2):
    ths = [threading.Thread(target=l.fit) for l in ls]
    [t.start() for t in ths]
    [t.join() for t in ths]
torch.cuda.synchronize()
st = np.zeros((2, 32, 8), dtype=np.uint64)
assert lib.mlp_debug_persistent_stamps(st.ctypes.data) == 0
st = st.astype(np.int64)
t0 = st[0, 0, 0]
us = lambda v: (v - t0) / 100.0
print("owner: A(fwd+publish) | wait dH2 | dH2 load+C1 | C2+C3 (dW1,dW2+Adam) | W2 publish+X stage | step")
print("head : wait W2 | wait H1+loads | H2 | logits+softmax | dH2+publish | dW3/bias | step")
for t in range(2, 12):
    o, h = st[0, t], st[1, t]
    do = np.diff(o[:6]) / 100.0
    dh = np.diff(h[:7]) / 100.0
    step_o = (st[0, t + 1, 0] - o[0]) / 100.0
    step_h = (st[1, t + 1, 0] - h[0]) / 100.0
    print(f"t={t:2d} owner {' '.join(f'{x:6.2f}' for x in do)} | {step_o:6.2f}   head {' '.join(f'{x:6.2f}' for x in dh)} | {step_h:6.2f}")
print("owner A start -> head H1 ready (us):", [round((st[1, t, 2] - st[0, t, 0]) / 100.0, 2) for t in range(2, 8)])
print("head dH2 published -> owner dH2 seen (us):", [round((st[0, t, 2] - st[1, t, 5]) / 100.0, 2) for t in range(2, 8)])
print("owner W2 published -> head W2 seen (us):", [round((st[1, t + 1, 1] - st[0, t, 5]) / 100.0, 2) for t in range(2, 8)])
