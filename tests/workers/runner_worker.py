"""torchrun worker: a YAML-style collective experiment split over ranks (tests/test_runtime_features.py)."""

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from myfyp_amd.parallel.federation import Federation  # noqa: E402
from myfyp_amd.runner import run_experiment  # noqa: E402

cfg = {
    "experiment": {
        "name": "ranks", "rounds": 2, "epochs": 1, "trainset_size": 4, "seed": 5,
        "dataset": {"source": "synthetic", "name": "mnist", "n_train": 800, "n_test": 200, "batch_size": 32,
                    "partitioning": {"strategy": "RandomIIDPartitionStrategy"}},
        "model": {"name": "MLP"}, "aggregator": {"name": "FedAvg"},
        "attack": {"node": 3, "kind": "sign_flip"},
    },
    "network": {"protocol": "collective", "nodes": 4},
    "settings": {"general": {"LOG_LEVEL": "WARNING"}, "device": {"USE_FUSED_KERNELS": False}},
}
res = run_experiment(cfg, verbose=False)
fed = Federation.get()
assert res["world"] == 2 and len(res["nodes"]) == 2, res["nodes"]
# every rank sees every peer's evaluation metrics after the gather
assert sorted(res["global_logs"]) == sorted(f"ranks-node-{i}" for i in range(4)), list(res["global_logs"])
for node, metrics in res["global_logs"].items():
    assert [r for r, _ in metrics["test_metric"]][:2] == [0, 1], (node, metrics["test_metric"])
print(f"rank {fed.rank} OK {sorted(res['global_logs'])}", flush=True)
fed.shutdown()
