"""Where an fp32 persistent epoch's time goes beyond its steps (stamped library:
MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so): peer 0 owner 0's kernel entry -> first step,
every step's duration, last step -> gang commit -> write-back done. 8 peers, B = 64, two fits."""
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
for fn in ("mlp_debug_persistent_f32_stamps", "mlp_debug_persistent_f32_epoch_stamps"):
    getattr(lib, fn).argtypes = [ctypes.c_void_p]
    getattr(lib, fn).restype = ctypes.c_int
P, B = int(os.environ.get("PEERS", "8")), 64
parts = synthetic_mnist(60000, 10000, seed=1).generate_partitions(8, RandomIIDPartitionStrategy)
ls = [TorchLearner(TorchModel(MLP(seed=i)), parts[i], f"p{i}", batch_size=B, device="cuda") for i in range(P)]
g = ls[0]._engine.group
print("variant", g.f32_variant(), "ks", g.f32_ks(), "steps", (parts[0].get_num_samples(True) + B - 1) // B)
for it in range(3):
    ths = [threading.Thread(target=l.fit) for l in ls]
    [t.start() for t in ths]
    [t.join() for t in ths]
torch.cuda.synchronize()
st = np.zeros((2, 128, 10), dtype=np.uint64)
ep = np.zeros(4, dtype=np.uint64)
assert lib.mlp_debug_persistent_f32_stamps(st.ctypes.data) == 0
assert lib.mlp_debug_persistent_f32_epoch_stamps(ep.ctypes.data) == 0
st, ep = st.astype(np.int64), ep.astype(np.int64)
n = int((parts[0].get_num_samples(True) + B - 1) // B)
starts = st[0, :n, 0]
ends = st[0, :n, 6]
steps = (ends - starts) / 100.0
print(f"entry -> step 0 start: {(starts[0] - ep[0]) / 100.0:.2f} us")
print(f"step 0 .. {n - 1}: {(ends[n - 1] - starts[0]) / 100.0:.1f} us; per step median {np.median(steps):.2f}, "
      f"first 5 {np.round(steps[:5], 2).tolist()}, last 5 {np.round(steps[-5:], 2).tolist()}")
gaps = (starts[1:] - ends[:-1]) / 100.0
print(f"between steps (owner 0: step end -> next start) median {np.median(gaps):.2f} us, total {gaps.sum():.1f}")
print(f"last step end -> gang commit passed: {(ep[2] - ends[n - 1]) / 100.0:.2f} us; -> write-back done: {(ep[3] - ep[2]) / 100.0:.2f} us")
print(f"entry -> write-back done: {(ep[3] - ep[0]) / 100.0:.1f} us")
q = np.percentile(steps, [10, 50, 90, 99])
print("step percentiles p10/p50/p90/p99:", np.round(q, 2).tolist())
