"""FYP harness: normal vs Byzantine (sign-flip / Gaussian-noise) experiment, side-by-side metric table."""

# Parity: exp_SAVE3.txt:60-332 (seeded runs, STAR topology, RandomIID n*50 partitions,
# attack on node attack_node_idx's initial weights, table of test_loss/metric/F1/precision/recall).

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from myfyp_amd.runner import run_experiment  # noqa: E402
from myfyp_amd.utils.utils import set_test_settings  # noqa: E402

KEYS = ["test_loss", "test_metric", "test_f1", "test_precision", "test_recall"]


def config(name: str, seed: int, n: int, r: int, attack=None, protocol: str = "memory", reduced: bool = True, batch_size: int = 16) -> dict:
    exp = {
        "name": name,
        "rounds": r,
        "epochs": 1,
        "seed": seed,
        "same_init": True,
        "wait_timeout": 240,
        "dataset": {"source": "synthetic", "name": "mnist", "n_train": 30000, "n_test": 5000, "batch_size": batch_size,
                    "partitioning": {"strategy": "RandomIIDPartitionStrategy", "reduced_dataset": reduced, "reduction_factor": 50}},
        "model": {"name": "MLP"},
        "aggregator": {"name": "FedAvg"},
    }
    if attack:
        exp["attack"] = attack
    return {"experiment": exp, "network": {"protocol": protocol, "nodes": n, "topology": "star"}}


def final(logs: dict, key: str):
    if not logs:
        return "N/A"
    node = sorted(logs)[0]
    vals = logs[node].get(key)
    return vals[-1][1] if vals else "N/A"


def main(seed: int = 666, n: int = 3, r: int = 1, attack: str = "sign_flip", node: int = 0, sigma: float = 0.1, protocol: str = "memory") -> dict:
    set_test_settings()
    normal = run_experiment(config(f"fyp-normal-{seed}", seed, n, r, protocol=protocol), verbose=False)
    att = {"node": node, "kind": attack, "sigma": sigma}
    attacked = run_experiment(config(f"fyp-{attack}-{seed}", seed, n, r, attack=att, protocol=protocol), verbose=False)
    print(f"{'Metric':<14} | {'Normal Experiment':<32} | {'Attack Experiment (' + attack + ')':<32}")
    print("-" * 84)
    for k in KEYS:
        print(f"{k:<14} | {str(final(normal['global_logs'], k)):<32} | {str(final(attacked['global_logs'], k)):<32}")
    return {"normal": normal, "attack": attacked}


if __name__ == "__main__":
    ap = argparse.ArgumentParser(description="Byzantine-attack comparison (FYP harness).")
    ap.add_argument("--seed", type=int, default=666)
    ap.add_argument("--nodes", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--attack", choices=["sign_flip", "gaussian_noise"], default="sign_flip")
    ap.add_argument("--attack_node", type=int, default=0)
    ap.add_argument("--sigma", type=float, default=0.1)
    ap.add_argument("--protocol", default="memory", choices=["memory", "grpc", "collective"])
    a = ap.parse_args()
    main(a.seed, a.nodes, a.rounds, a.attack, a.attack_node, a.sigma, a.protocol)
