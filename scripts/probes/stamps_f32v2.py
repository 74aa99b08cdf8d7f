"""Phase timing of the fp32 persistent MLP epoch, gang layout 2 (mlp_persistent_f32v2.hip; run with
MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so MYFYP_F32_VARIANT=2). PEERS grouped peers (default 8),
B = 64, two fits; per-step phase durations (us) of peer 0's owner 0."""
import ctypes
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
Settings.MLP_PRECISION = "fp32"
lib = _native.load(required=True)
assert hasattr(lib, "mlp_debug_persistent_f32v2_stamps"), "not the stamped library"
lib.mlp_debug_persistent_f32v2_stamps.argtypes = [ctypes.c_void_p]
lib.mlp_debug_persistent_f32v2_stamps.restype = ctypes.c_int
P, B = int(os.environ.get("PEERS", "8")), 64
parts = synthetic_mnist(60000, 10000, seed=1).generate_partitions(8, RandomIIDPartitionStrategy)
ls = [TorchLearner(TorchModel(MLP(seed=i)), parts[i], f"p{i}", batch_size=B, device="cuda") for i in range(P)]
g = ls[0]._engine.group
assert g.uses_persistent() and g.f32_variant() == 2, g.f32_variant()
for it in range(2):
    ths = [threading.Thread(target=l.fit) for l in ls]
    [t.start() for t in ths]
    [t.join() for t in ths]
torch.cuda.synchronize()
st = np.zeros((32, 16), dtype=np.uint64)
assert lib.mlp_debug_persistent_f32v2_stamps(st.ctypes.data) == 0
st = st.astype(np.int64)
names = ["A fwd+reduce", "B H2p+publish", "wait F1", "R reduce+softmax+dH2+publish", "wait F2", "C: dH2/dW3 load+W3 upd", "C: frags+dW2 MFMA",
         "C: C1 MFMA+partials", "C: split+W2 upd", "C2 dW1+Adam+X"]
print("owner 0 of peer 0:", " | ".join(names), "| step")
rows = []
for t in range(2, 30):
    o = st[t]
    d = np.diff(o[:11]) / 100.0
    step = (st[t + 1, 0] - o[0]) / 100.0
    rows.append(np.concatenate([d, [step]]))
    print(f"t={t:2d} {' '.join(f'{x:5.2f}' for x in d)} | {step:5.2f}")
m = np.median(np.array(rows), axis=0)
print("median", " ".join(f"{x:5.2f}" for x in m))
sub = np.array([[(st[t, 11] - st[t, 3]) / 100.0, (st[t, 12] - st[t, 11]) / 100.0, (st[t, 13] - st[t, 12]) / 100.0, (st[t, 4] - st[t, 13]) / 100.0]
                for t in range(2, 30)])
print("R split: loads+partials | H2 rows | softmax | dH2+dW3p+publish :", " ".join(f"{x:5.2f}" for x in np.median(sub, axis=0)))
