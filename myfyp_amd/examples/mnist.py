"""MNIST MLP federated experiment: n nodes, r rounds, e epochs over memory/grpc/unix/collective protocols."""

# Parity: p2pfl/examples/mnist.py:73-255 (same flags; adds --aggregator fedmedian/fedprox/krum/
# trimmedmean, --batch_size, --dataset synthetic|huggingface, collective protocol). matplotlib
# plots are written to --plot_dir instead of plt.show(); --profiling uses cProfile (yappi is not
# available) and writes one pstat per run under profile/mnist/<uuid>/.

import argparse
import os
import sys
import time
import uuid

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from myfyp_amd.management.logger import logger  # noqa: E402
from myfyp_amd.runner import run_experiment  # noqa: E402
from myfyp_amd.settings import Settings  # noqa: E402
from myfyp_amd.utils.topologies import TopologyType  # noqa: E402
from myfyp_amd.utils.utils import set_standalone_settings  # noqa: E402


def _parse_args() -> argparse.Namespace:
    p = argparse.ArgumentParser(description="P2PFL-style MNIST experiment on the MI355X engine.")
    p.add_argument("--nodes", type=int, default=2, help="The number of nodes.")
    p.add_argument("--rounds", type=int, default=2, help="The number of rounds.")
    p.add_argument("--epochs", type=int, default=1, help="The number of epochs.")
    p.add_argument("--show_metrics", action="store_true", default=True, help="Show metrics.")
    p.add_argument("--measure_time", action="store_true", default=False, help="Measure time.")
    p.add_argument("--token", type=str, default="", help="The API token for the Web Logger.")
    p.add_argument("--protocol", type=str, default="memory", choices=["grpc", "unix", "memory", "collective"])
    p.add_argument("--framework", type=str, default="pytorch", choices=["pytorch", "rocm"])
    p.add_argument("--aggregator", type=str, default="fedavg", choices=["fedavg", "scaffold", "fedmedian", "fedprox", "krum", "trimmedmean"])
    p.add_argument("--profiling", action="store_true", default=False, help="Enable profiling (cProfile).")
    p.add_argument("--reduced_dataset", action="store_true", default=False, help="Use a reduced dataset (nodes*50 partitions).")
    p.add_argument("--use_scaffold", action="store_true", default=False, help="Use the Scaffold aggregator.")
    p.add_argument("--disable_ray", action="store_true", default=False, help="Accepted for compatibility (no Ray).")
    p.add_argument("--topology", type=str, choices=[t.value for t in TopologyType], default="line")
    p.add_argument("--batch_size", type=int, default=64)
    p.add_argument("--dataset", type=str, default="synthetic", choices=["synthetic", "huggingface"])
    p.add_argument("--seed", type=int, default=666)
    p.add_argument("--plot_dir", type=str, default="", help="Write metric plots here (png).")
    return p.parse_args()


def mnist(n: int, r: int, e: int, show_metrics: bool = True, measure_time: bool = False, protocol: str = "memory", aggregator: str = "fedavg",
          reduced_dataset: bool = False, topology: TopologyType = TopologyType.LINE, batch_size: int = 64, dataset: str = "synthetic", seed: int = 666,
          plot_dir: str = "") -> dict:
    if n > Settings.TTL:
        raise ValueError("For in-line topology TTL must be greater than the number of nodes.")
    if r < 1:
        raise ValueError("Skipping training, amount of round is less than 1")
    cfg = {
        "experiment": {
            "name": f"mnist-{uuid.uuid4().hex[:8]}",
            "rounds": r,
            "epochs": e,
            "seed": seed,
            "wait_timeout": 3600,
            "dataset": {
                "source": dataset,
                "name": "p2pfl/MNIST" if dataset == "huggingface" else "mnist",
                "batch_size": batch_size,
                "partitioning": {"strategy": "RandomIIDPartitionStrategy", "reduced_dataset": reduced_dataset, "reduction_factor": 50},
            },
            "model": {"name": "MLP"},
            "aggregator": {"name": aggregator},
        },
        "network": {"protocol": protocol, "nodes": n, "topology": topology.value if isinstance(topology, TopologyType) else topology},
    }
    t0 = time.time()
    res = run_experiment(cfg, verbose=show_metrics)
    if plot_dir:
        _plot(res, plot_dir)
    if measure_time:
        print("--- %s seconds ---" % (time.time() - t0))
    return res


def _plot(res: dict, plot_dir: str) -> None:
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:  # pragma: no cover
        print("matplotlib not available; skipping plots")
        return
    os.makedirs(plot_dir, exist_ok=True)
    for node, metrics in res["global_logs"].items():
        for metric, values in metrics.items():
            x, y = zip(*values)
            plt.figure()
            plt.plot(x, y, label=metric)
            plt.scatter(x[-1], y[-1], color="red")
            plt.title(f"{node} - {metric}")
            plt.xlabel("Round")
            plt.ylabel(metric)
            plt.legend()
            plt.savefig(os.path.join(plot_dir, f"{node.replace('/', '_')}-{metric}.png"))
            plt.close()


if __name__ == "__main__":
    args = _parse_args()
    set_standalone_settings()
    Settings.WAIT_HEARTBEATS_CONVERGENCE = 1.0
    if args.token:
        logger.connect_web("http://localhost:3000/api/v1", args.token)
    agg = "scaffold" if args.use_scaffold else args.aggregator
    prof = None
    if args.profiling:
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
    try:
        mnist(args.nodes, args.rounds, args.epochs, args.show_metrics, args.measure_time, args.protocol, agg, args.reduced_dataset,
              TopologyType(args.topology), args.batch_size, args.dataset, args.seed, args.plot_dir)
    finally:
        if prof is not None:
            prof.disable()
            d = os.path.join("profile", "mnist", str(uuid.uuid4()))
            os.makedirs(d, exist_ok=True)
            prof.dump_stats(os.path.join(d, "main.pstat"))
