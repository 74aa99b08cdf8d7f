"""YAML/dict experiment runner (``p2pfl run cfg.yaml``; reference examples ``mnist.py``).

One description drives every experiment the examples, the CLI and the FYP harness run::

    experiment:
      name: mnist-fedavg
      rounds: 3
      epochs: 1
      trainset_size: 4          # Settings.TRAIN_SET_SIZE
      seed: 666
      wait_timeout: 3600        # seconds (wait_to_finish)
      dataset:
        source: synthetic       # synthetic | huggingface | csv | json | parquet | npz
        name: mnist             # synthetic: mnist | cifar10 ; huggingface: hub id / local path
        n_train: 60000
        n_test: 10000
        batch_size: 64
        partitioning:
          strategy: RandomIIDPartitionStrategy   # or DirichletPartitionStrategy, ...
          reduced_dataset: false
          reduction_factor: 50                   # partitions = nodes * factor when reduced
          params: {alpha: 0.5}
      model:
        name: MLP               # MLP | LeNet5 | ResNet18, or package + model_build_fn
        params: {}              # + compression: {ptq: {dtype: float16}, topk: {k: 0.1}, zlib: {level: 6}}
      aggregator:
        name: FedAvg            # FedAvg | FedMedian | Scaffold | FedProx | Krum | TrimmedMean
        params: {}
      attack: {node: 1, kind: sign_flip, sigma: 0.1, persistent: false}
      faults: [{node: 2, kill_at: TrainStage, round: 1}]
      checkpoint: {dir: ckpt, every: 1, resume: false}
    network:
      protocol: memory          # memory | grpc | unix | collective (class names also accepted)
      nodes: 4
      topology: full            # star | full | line | ring | grid | random
    settings:                   # flat or nested Settings overrides
      general: {LOG_LEVEL: INFO}

``package``/class names written for p2pfl (``p2pfl.learning.aggregators.fedavg`` + ``FedAvg``) are
mapped onto this package, so reference-style configs run unmodified.
"""

from __future__ import annotations

import importlib
import os
import time
from typing import Any, Dict, List, Optional

from myfyp_amd.settings import Settings

# -------------------------------------------------------------------------------------------- registries
_PROTOCOLS = {
    "memory": ("myfyp_amd.communication.protocols.memory.memory_communication_protocol", "InMemoryCommunicationProtocol"),
    "inmemorycommunicationprotocol": ("myfyp_amd.communication.protocols.memory.memory_communication_protocol", "InMemoryCommunicationProtocol"),
    "memorycommunicationprotocol": ("myfyp_amd.communication.protocols.memory.memory_communication_protocol", "InMemoryCommunicationProtocol"),
    "grpc": ("myfyp_amd.communication.protocols.grpc.grpc_communication_protocol", "GrpcCommunicationProtocol"),
    "unix": ("myfyp_amd.communication.protocols.grpc.grpc_communication_protocol", "GrpcCommunicationProtocol"),
    "grpccommunicationprotocol": ("myfyp_amd.communication.protocols.grpc.grpc_communication_protocol", "GrpcCommunicationProtocol"),
    "collective": ("myfyp_amd.communication.protocols.collective.collective_protocol", "CollectiveCommunicationProtocol"),
    "collectivecommunicationprotocol": ("myfyp_amd.communication.protocols.collective.collective_protocol", "CollectiveCommunicationProtocol"),
}
_AGGREGATORS = {
    "fedavg": ("myfyp_amd.learning.aggregators.fedavg", "FedAvg"),
    "fedmedian": ("myfyp_amd.learning.aggregators.fedmedian", "FedMedian"),
    "scaffold": ("myfyp_amd.learning.aggregators.scaffold", "Scaffold"),
    "fedprox": ("myfyp_amd.learning.aggregators.fedprox", "FedProx"),
    "krum": ("myfyp_amd.learning.aggregators.krum", "Krum"),
    "trimmedmean": ("myfyp_amd.learning.aggregators.trimmed_mean", "TrimmedMean"),
    "neighboravg": ("myfyp_amd.learning.aggregators.neighbor_avg", "NeighborAvg"),
}
_MODELS = {"mlp": "MLP", "lenet5": "LeNet5", "lenet": "LeNet5", "resnet18": "ResNet18", "resnet": "ResNet18"}


def _import(module: str, name: str):
    if module.startswith("p2pfl."):
        module = "myfyp_amd." + module[len("p2pfl.") :]
    return getattr(importlib.import_module(module), name)


def resolve_protocol(spec: Any):
    if isinstance(spec, type):
        return spec
    if isinstance(spec, dict):
        if spec.get("package") and not spec["package"].startswith("p2pfl."):
            return _import(spec["package"], spec["protocol"])
        spec = spec.get("protocol", "memory")
    key = str(spec).lower()
    if key not in _PROTOCOLS:
        raise ValueError(f"unknown protocol {spec!r}; choose from memory, grpc, unix, collective")
    return _import(*_PROTOCOLS[key])


def build_aggregator(spec: Optional[Dict[str, Any]]):
    spec = dict(spec or {})
    name = spec.get("name") or spec.get("aggregator") or "FedAvg"
    params = dict(spec.get("params") or {})
    pkg = spec.get("package")
    if pkg and not pkg.startswith("p2pfl."):
        return _import(pkg, name)(**params)
    key = name.lower()
    if key not in _AGGREGATORS:
        raise ValueError(f"unknown aggregator {name!r}; choose from {sorted(_AGGREGATORS)}")
    return _import(*_AGGREGATORS[key])(**params)


def build_model(spec: Optional[Dict[str, Any]], seed: Optional[int] = None, index: int = 0):
    """Return a fresh ``P2PFLModel``. ``seed`` (if any) makes every node's init identical to the
    reference's per-node ``set_seed`` behaviour; ``index`` offsets it otherwise."""
    from myfyp_amd.learning.frameworks.torch import TorchModel

    spec = dict(spec or {})
    params = dict(spec.get("params") or {})
    if spec.get("model_build_fn") and spec.get("package") and not spec["package"].startswith("p2pfl."):
        return _import(spec["package"], spec["model_build_fn"])(**params)
    name = spec.get("name", "MLP")
    cls_name = _MODELS.get(str(name).lower())
    if cls_name is None:
        raise ValueError(f"unknown model {name!r}; choose from MLP, LeNet5, ResNet18")
    import myfyp_amd.models as zoo

    compression = params.pop("compression", spec.get("compression"))
    if "seed" not in params and seed is not None:
        params["seed"] = seed + index
    return TorchModel(getattr(zoo, cls_name)(**params), compression=compression)


def build_dataset(spec: Optional[Dict[str, Any]]):
    from myfyp_amd.learning.dataset.p2pfl_dataset import P2PFLDataset
    from myfyp_amd.learning.dataset.synthetic import synthetic_cifar10, synthetic_mnist

    spec = dict(spec or {})
    src = str(spec.get("source", "synthetic")).lower()
    name = str(spec.get("name", "mnist"))
    if src == "synthetic":
        kw = {k: spec[k] for k in ("n_train", "n_test", "seed", "noise", "similarity") if k in spec}
        if name.lower() in ("mnist", "p2pfl/mnist"):
            return synthetic_mnist(**kw)
        if name.lower() in ("cifar10", "cifar-10", "p2pfl/cifar10"):
            return synthetic_cifar10(**kw)
        raise ValueError(f"unknown synthetic dataset {name!r}")
    if src == "huggingface":
        return P2PFLDataset.from_huggingface(name)
    if src in ("csv", "json", "parquet"):
        return getattr(P2PFLDataset, f"from_{src}")(spec["data_files"])
    if src == "npz":
        import numpy as np

        with np.load(spec["path"], allow_pickle=False) as z:
            return P2PFLDataset.from_arrays({"image": z["x_train"], "label": z["y_train"]}, {"image": z["x_test"], "label": z["y_test"]})
    raise ValueError(f"unknown dataset source {src!r}")


def _partitions(data, n_nodes: int, spec: Dict[str, Any], seed: int):
    import myfyp_amd.learning.dataset.partition_strategies as ps

    part = dict(spec.get("partitioning") or {})
    strategy = getattr(ps, part.get("strategy", "RandomIIDPartitionStrategy"))
    n_parts = n_nodes * int(part.get("reduction_factor", 50)) if part.get("reduced_dataset") else n_nodes
    return data.generate_partitions(n_parts, strategy, seed=seed, **dict(part.get("params") or {}))


def _address(protocol_key: str, i: int, exp: str) -> str:
    if protocol_key == "unix":
        return f"unix:///tmp/myfyp-{exp}-{os.getpid()}-{i}.sock"
    if protocol_key == "grpc":
        return "127.0.0.1"
    return f"{exp}-node-{i}"


# -------------------------------------------------------------------------------------------- runner
def load_config(cfg: Any) -> Dict[str, Any]:
    """Path or dict → dict (applies the ``settings`` section)."""
    if isinstance(cfg, (str, os.PathLike)):
        return Settings.from_yaml(str(cfg))
    cfg = dict(cfg)
    if "settings" in cfg:
        Settings.update(cfg["settings"])
    return cfg


def run_experiment(cfg: Any, verbose: bool = True) -> Dict[str, Any]:
    """Build nodes from the description, run learning to completion, return a results dict:
    ``{"exp_name", "elapsed_s", "global_logs", "local_logs", "histories", "nodes"}``."""
    from myfyp_amd import fault_injection
    from myfyp_amd.management import checkpoint as ckpt
    from myfyp_amd.management.logger import logger
    from myfyp_amd.node import Node
    from myfyp_amd.utils.seed import set_seed
    from myfyp_amd.utils.topologies import TopologyFactory, TopologyType
    from myfyp_amd.utils.utils import wait_convergence, wait_to_finish

    cfg = load_config(cfg)
    exp = dict(cfg.get("experiment") or {})
    net = dict(cfg.get("network") or {})
    name = exp.get("name", "experiment")
    rounds, epochs = int(exp.get("rounds", 1)), int(exp.get("epochs", 1))
    seed = exp.get("seed", Settings.SEED)
    if seed is not None:
        set_seed(int(seed))
    if "trainset_size" in exp:
        Settings.TRAIN_SET_SIZE = int(exp["trainset_size"])
    ds_spec = dict(exp.get("dataset") or {})
    if "batch_size" in ds_spec:
        Settings.BATCH_SIZE = int(ds_spec["batch_size"])
    ck = dict(exp.get("checkpoint") or {})
    if ck.get("dir"):
        Settings.CHECKPOINT_DIR = ck["dir"]
        Settings.CHECKPOINT_EVERY = int(ck.get("every", 1))

    n = int(net.get("nodes", 2))
    proto_spec = net.get("protocol", "memory")
    proto_key = str(proto_spec.get("protocol", "memory") if isinstance(proto_spec, dict) else proto_spec).lower()
    protocol = resolve_protocol(proto_spec)
    collective = getattr(protocol, "workflow", "gossip") == "collective"

    data = build_dataset(ds_spec)
    parts = _partitions(data, n, ds_spec, int(seed) if seed is not None else 666)
    fed = None
    if collective:
        from myfyp_amd.parallel.federation import Federation

        # `devices: N` (or network.devices): one process drives N GPUs (device mesh)
        ndev = exp.get("devices", net.get("devices"))
        fed = Federation.init(devices=int(ndev) if ndev else None)
    nodes: List[Any] = []
    by_index: Dict[int, Any] = {}
    start_round = 0
    t_start = time.time()
    # one process per GPU (torchrun): rank r builds the contiguous block of peers it owns
    world, rank = (fed.world, fed.rank) if fed is not None else (1, 0)
    local = [i for i in range(n) if (i * world) // n == rank]
    try:
        for i in local:
            model = build_model(exp.get("model"), seed=None if seed is None else int(seed), index=i if not exp.get("same_init") else 0)
            node = Node(model, parts[i], address=_address(proto_key, i, name), protocol=protocol, aggregator=build_aggregator(exp.get("aggregator")), exp_name=name)
            node.start()
            nodes.append(node)
            by_index[i] = node
        if ck.get("resume") and ck.get("dir"):
            metas = [ckpt.restore_node(nd, directory=ck["dir"], exp_name=name) for nd in nodes]
            start_round = min(int(m.get("round", 0)) for m in metas)
        att = exp.get("attack")
        if att and int(att.get("node", 0)) in by_index:
            victim = by_index[int(att.get("node", 0))]
            if att.get("persistent"):
                fault_injection.ModelPoisoning(victim, att.get("kind", "sign_flip"), float(att.get("sigma", 0.1)), float(att.get("factor", -1.0)), int(att.get("seed", 0)))
            else:
                fault_injection.apply_attack(victim, att.get("kind", "sign_flip"), float(att.get("sigma", 0.1)), float(att.get("factor", -1.0)), int(att.get("seed", 0)))
        for f in exp.get("faults") or []:
            if int(f["node"]) not in by_index:
                continue
            victim = by_index[int(f["node"])]
            if "kill_at" in f:
                fault_injection.kill_at(victim, f["kill_at"], f.get("round"))
            if "delay_at" in f:
                fault_injection.delay_at(victim, f["delay_at"], float(f.get("seconds", 1.0)), f.get("round"))
        if collective:
            fed.finalize()
        else:
            topo = TopologyType(str(net.get("topology", "full")).lower())
            TopologyFactory.connect_nodes(TopologyFactory.generate_matrix(topo, n), nodes)
            wait_convergence(nodes, n - 1, only_direct=False, wait=float(net.get("convergence_timeout", 60)))
        t_start = time.time()
        if rank == 0:  # the start message reaches the other ranks' peers over the control bus
            nodes[0].set_start_learning(rounds=rounds, epochs=epochs, start_round=start_round)
        wait_to_finish(nodes, timeout=float(exp.get("wait_timeout", 3600)))
        elapsed = time.time() - t_start
        if fed is not None:
            fed.gather_logs()
        res = {
            "exp_name": name,
            "elapsed_s": elapsed,
            "global_logs": logger.get_global_logs().get(name, {}),
            "local_logs": logger.get_local_logs().get(name, {}),
            "histories": {nd.addr: list(nd.learning_workflow.history) for nd in nodes},
            "nodes": [nd.addr for nd in nodes],
            "start_round": start_round,
            "rank": rank,
            "world": world,
        }
        if verbose and rank == 0:
            print(format_results(res))
        return res
    finally:
        for nd in nodes:
            nd.stop()
        if fed is not None:
            from myfyp_amd.parallel.federation import Federation

            if fed.world == 1:
                Federation.reset()


def format_results(res: Dict[str, Any]) -> str:
    """Final-round metric table (the FYP harness prints test_loss/metric/F1/precision/recall)."""
    keys = ["test_loss", "test_metric", "test_f1", "test_precision", "test_recall"]
    lines = [f"experiment {res['exp_name']}: {res['elapsed_s']:.2f} s", f"{'node':<28}" + "".join(f"{k:>16}" for k in keys)]
    for addr in sorted(res["global_logs"]):
        m = res["global_logs"][addr]
        vals = [m[k][-1][1] if m.get(k) else float("nan") for k in keys]
        lines.append(f"{addr:<28}" + "".join(f"{v:>16.4f}" for v in vals))
    return "\n".join(lines)
