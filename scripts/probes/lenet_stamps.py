"""Phase timestamps of the fused LeNet step (diagnostics build, -DMLP_STAMPS).

Run with MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so: trains 8 grouped LeNet-5 peers for one
epoch and prints workgroup (0, 0)'s phase boundaries of the last step in microseconds."""

import ctypes
import os
import sys
import threading

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy  # noqa: E402
from myfyp_amd.learning.dataset.synthetic import synthetic_cifar10  # noqa: E402
from myfyp_amd.learning.frameworks.torch import TorchModel  # noqa: E402
from myfyp_amd.learning.frameworks.torch.torch_learner import TorchLearner  # noqa: E402
from myfyp_amd.models import LeNet5  # noqa: E402
from myfyp_amd.ops import _native  # noqa: E402

NAMES = ["start", "idx/labels", "gather", "conv1", "conv2", "fc1", "fc2", "fc3", "xent", "fc3 dgrad", "fc2 dgrad", "fc1 dgrad",
         "pool2 bwd + act", "conv2 wgrad + dgrad", "conv1 wgrad"]

peers, n = 8, 8 * 4096
parts = synthetic_cifar10(n, 1024, seed=1).generate_partitions(peers, RandomIIDPartitionStrategy)
learners = [TorchLearner(TorchModel(LeNet5(seed=i)), parts[i], f"st-{i}", batch_size=64, device="cuda") for i in range(peers)]
for rep in range(3):
    ths = [threading.Thread(target=lr.fit) for lr in learners]
    [t.start() for t in ths]
    [t.join() for t in ths]
torch.cuda.synchronize()
lib = _native.load(required=True)
fn = lib.lenet_debug_stamps
fn.argtypes, fn.restype = [ctypes.c_void_p], ctypes.c_int
buf = np.zeros(24, dtype=np.uint64)
assert fn(buf.ctypes.data) == 0
t = buf.astype(np.float64) / 100.0  # 100 MHz -> us
print("fused lenet step, workgroup (0,0), last step (us since start):")
for i in range(1, 15):
    print(f"  {NAMES[i]:22s} {t[i] - t[0]:8.2f}  (+{t[i] - t[i - 1]:6.2f})")
print(f"  wave 0: conv2 wgrad done {t[15] - t[0]:8.2f}, W2 dgrad fragments {t[16] - t[0]:8.2f}, dgrad done {t[17] - t[0]:8.2f}")
