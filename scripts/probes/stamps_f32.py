"""Phase timing of the fp32 persistent MLP epoch kernel (MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so).
PEERS grouped peers (default 8), B = 64, two fits; per-step phase durations (us) of peer 0's owner 0
and head 0, and the hand-off latencies between them. The owner K split follows the engine's choice
(MYFYP_F32_KS forces one; at K split > 1 owner 0 is column group 0's K part 0, whose stamp 2 comes
after the in-XCD reduction of the K parts and the reduced slice's publish)."""
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
assert hasattr(lib, "mlp_debug_persistent_f32_stamps"), "not the stamped library"
lib.mlp_debug_persistent_f32_stamps.argtypes = [ctypes.c_void_p]
lib.mlp_debug_persistent_f32_stamps.restype = ctypes.c_int
P, B = int(os.environ.get("PEERS", "8")), 64
parts = synthetic_mnist(60000, 10000, seed=1).generate_partitions(8, RandomIIDPartitionStrategy)
ls = [TorchLearner(TorchModel(MLP(seed=i)), parts[i], f"p{i}", batch_size=B, device="cuda") for i in range(P)]
g = ls[0]._engine.group
assert g.uses_persistent()
print(f"peers {P}, owner K split {g.f32_ks()}, variant {g.f32_variant()}")
for it in range(2):
    ths = [threading.Thread(target=l.fit) for l in ls]
    [t.start() for t in ths]
    [t.join() for t in ths]
torch.cuda.synchronize()
st = np.zeros((2, 128, 10), dtype=np.uint64)  # g_p32_stamps[2][128][10]
assert lib.mlp_debug_persistent_f32_stamps(st.ctypes.data) == 0
st = st.astype(np.int64)
print("owner: fwd+reduce | H1 publish | W2 replica | wait dH2 | dH2 load+C1+split | C2 (dW1+Adam+X) | step")
print("head : wait H1 | H1 load | H2+PL | PL publish | wait PL | softmax | dH2+publish | off-path | step")
rows = []
for t in range(2, 14):
    o, h = st[0, t], st[1, t]
    do = np.diff(o[:7]) / 100.0
    dh = np.diff(h[:9]) / 100.0
    step_o = (st[0, t + 1, 0] - o[0]) / 100.0
    step_h = (st[1, t + 1, 0] - h[0]) / 100.0
    rows.append(np.concatenate([do, [step_o], dh, [step_h]]))
    print(f"t={t:2d} owner {' '.join(f'{x:5.2f}' for x in do)} | {step_o:5.2f}   head {' '.join(f'{x:5.2f}' for x in dh)} | {step_h:5.2f}")
m = np.median(np.array(rows), axis=0)
print("median owner", " ".join(f"{x:5.2f}" for x in m[:7]), " head", " ".join(f"{x:5.2f}" for x in m[7:]))
print("owner H1 published -> head H1 seen (us):", [round((st[1, t, 1] - st[0, t, 2]) / 100.0, 2) for t in range(2, 10)])
print("head dH2 published -> owner dH2 seen (us):", [round((st[0, t, 4] - st[1, t, 7]) / 100.0, 2) for t in range(2, 10)])
print("head PL published -> head PL all seen (us):", [round((st[1, t, 5] - st[1, t, 4]) / 100.0, 2) for t in range(2, 10)])
