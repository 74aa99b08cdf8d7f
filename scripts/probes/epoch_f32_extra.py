"""Wall time of one grouped fp32 MLP fit (8 peers, B = 64, one local epoch) with the FedProx or
SCAFFOLD extra term (AGG=fedprox|scaffold|fedavg), for the gang-layout choice of the Adam + extra
instantiations (MYFYP_F32_VARIANT=1|2 forces a layout; unset = the engine's choice). Prints the
median over FITS fits and the layout that ran."""
import os
import sys
import threading
import time

sys.path.insert(0, os.getcwd())
import numpy as np
import torch

from myfyp_amd.learning.aggregators import FedAvg, FedProx, Scaffold
from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
from myfyp_amd.learning.frameworks.torch import TorchModel
from myfyp_amd.learning.frameworks.torch.torch_learner import TorchLearner
from myfyp_amd.models import MLP
from myfyp_amd.settings import Settings

Settings.USE_FUSED_KERNELS = True
Settings.MLP_PRECISION = "fp32"
agg_name = os.environ.get("AGG", "fedprox")
P, B, fits = 8, 64, int(os.environ.get("FITS", "12"))
parts = synthetic_mnist(60000, 10000, seed=1).generate_partitions(P, RandomIIDPartitionStrategy)


def make_agg():
    return {"fedprox": lambda: FedProx(proximal_mu=0.01), "scaffold": lambda: Scaffold(), "fedavg": lambda: FedAvg()}[agg_name]()


ls = [TorchLearner(TorchModel(MLP(seed=i)), parts[i], f"p{i}", aggregator=make_agg(), batch_size=B, device="cuda") for i in range(P)]
g = ls[0]._engine.group
assert g.uses_persistent()
times = []
for it in range(fits + 2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ths = [threading.Thread(target=l.fit) for l in ls]
    [t.start() for t in ths]
    [t.join() for t in ths]
    torch.cuda.synchronize()
    if it >= 2:
        times.append(time.perf_counter() - t0)
print(f"[epoch_f32_extra] agg={agg_name} layout={g.f32_variant()} ks={g.f32_ks()} median fit ms {1e3 * float(np.median(times)):.3f} "
      f"min {1e3 * min(times):.3f}", flush=True)
