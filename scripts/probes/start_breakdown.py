"""Where Node.start() time goes for the headline setup (8 peers, fused MLP engine, prewarm on):
per-node start time and cumulative time in the engine's setup phases. Prints one JSON line."""

import json
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))

import torch  # noqa: E402

from myfyp_amd.communication.protocols.collective.collective_protocol import CollectiveCommunicationProtocol  # noqa: E402
from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy  # noqa: E402
from myfyp_amd.learning.dataset.synthetic import synthetic_mnist  # noqa: E402
from myfyp_amd.learning.frameworks.torch import TorchModel  # noqa: E402
from myfyp_amd.models import MLP  # noqa: E402
from myfyp_amd.node import Node  # noqa: E402
from myfyp_amd.ops import _native  # noqa: E402
from myfyp_amd.parallel import mlp_engine  # noqa: E402
from myfyp_amd.parallel.federation import Federation  # noqa: E402
from myfyp_amd.settings import Settings  # noqa: E402

acc: dict = {}


def timed(owner, name, sync=True):
    fn = getattr(owner, name)

    def w(*a, **k):
        if sync and torch.cuda.is_available():
            torch.cuda.synchronize()
        t = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            if sync and torch.cuda.is_available():
                torch.cuda.synchronize()
            s = acc.setdefault(name, [0, 0.0])
            s[0] += 1
            s[1] += time.perf_counter() - t

    setattr(owner, name, w)


for n in ("_ensure_engine", "_bind_data", "prewarm", "attach"):
    if hasattr(mlp_engine.MLPGroup, n):
        timed(mlp_engine.MLPGroup, n)

t0 = time.perf_counter()
lib = _native.load(required=True)
t_load = time.perf_counter() - t0
Settings.BATCH_SIZE = 64
t0 = time.perf_counter()
fed = Federation.init()
t_fed = time.perf_counter() - t0
data = synthetic_mnist(60000, 10000, seed=2024, similarity=0.75, noise=1.0)
parts = data.generate_partitions(8, RandomIIDPartitionStrategy)
nodes = [Node(TorchModel(MLP(seed=100 + g)), parts[g], address=f"peer-{g}", protocol=CollectiveCommunicationProtocol, learner_kwargs={"batch_size": 64})
         for g in range(8)]
per = []
t_all = time.perf_counter()
for nd in nodes:
    t = time.perf_counter()
    nd.start()
    per.append(round(1e3 * (time.perf_counter() - t), 2))
total = time.perf_counter() - t_all
out = {"lib_load_ms": round(1e3 * t_load, 2), "fed_init_ms": round(1e3 * t_fed, 2), "node_start_ms": per, "total_ms": round(1e3 * total, 2),
       "phases_ms": {k: [v[0], round(1e3 * v[1], 2)] for k, v in acc.items()}}
print(json.dumps(out), flush=True)
for nd in nodes:
    nd.stop()
Federation.reset()
