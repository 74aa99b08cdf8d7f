"""Per-block phase timing of the fused MLP step (needs MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so).
Runs 8 grouped peers for one eager epoch; the stamps of the LAST step are analysed."""
import ctypes, os, sys, threading
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from myfyp_amd.ops import _native
from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
from myfyp_amd.learning.frameworks.torch import TorchModel
from myfyp_amd.learning.frameworks.torch.torch_learner import TorchLearner
from myfyp_amd.models import MLP
from myfyp_amd.settings import Settings
Settings.USE_FUSED_KERNELS = True
lib = _native.load(required=True)
assert hasattr(lib, "mlp_debug_stamps"), "not the stamped library"
P, B = 8, 64
parts = synthetic_mnist(60000, 10000, seed=1).generate_partitions(P, RandomIIDPartitionStrategy)
ls = [TorchLearner(TorchModel(MLP(seed=i)), parts[i], f"p{i}", batch_size=B, device="cuda") for i in range(P)]
g = ls[0]._engine.group
g.eager = bool(int(os.environ.get("EAGER", "1")))
for it in range(2):
    ths = [threading.Thread(target=l.fit) for l in ls]
    [t.start() for t in ths]; [t.join() for t in ths]
torch.cuda.synchronize()
st = np.zeros((3, 4096, 4), dtype=np.uint64)
assert lib.mlp_debug_stamps(st.ctypes.data) == 0
names = ["fc1", "head", "wgrad(W1 blocks)"]
t0 = min(int(st[k][:, 0][st[k][:, 0] > 0].min()) for k in range(3))
for k in range(3):
    s = st[k].astype(np.int64)
    live = s[:, 0] > 0
    s = s[live]
    ok = (s[:, 3] > 0)
    s = s[ok] if ok.any() else s
    rel = (s - t0) / 100.0  # 100 MHz -> us
    print(f"{names[k]:18s} blocks={len(s):5d} start[min,p50,max]=({rel[:,0].min():.2f},{np.median(rel[:,0]):.2f},{rel[:,0].max():.2f}) "
          f"end max={rel[:,3].max():.2f} | per-block phases p50 us: "
          f"{np.median(rel[:,1]-rel[:,0]):.2f} / {np.median(rel[:,2]-rel[:,1]):.2f} / {np.median(rel[:,3]-rel[:,2]):.2f}  total p50 {np.median(rel[:,3]-rel[:,0]):.2f} max {np.max(rel[:,3]-rel[:,0]):.2f}")
