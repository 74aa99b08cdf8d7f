"""Worker of tests/test_rccl_forced_gpu.py: the weights plane on ONE GPU, either solo (single-rank
fast paths) or FORCED through a world-size-1 RCCL process group (``MYFYP_FORCE_COLLECTIVE=1``:
every multi-rank code path — side-stream bucketed FedAvg with RCCL all-reduces, delayed
averaging, the init-model broadcast, SCAFFOLD's all-reduce, FedMedian's all-gather, the group
rebuild over the survivors). Each case starts from the same seeds; the final parameters of every
case go to ``$OUT`` (torch.save of CPU tensors) for the test to compare solo vs forced.
"""

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from myfyp_amd.communication.protocols.collective.collective_protocol import CollectiveCommunicationProtocol  # noqa: E402
from myfyp_amd.learning.aggregators import FedAvg, FedMedian, Scaffold  # noqa: E402
from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy  # noqa: E402
from myfyp_amd.learning.dataset.synthetic import synthetic_cifar10, synthetic_mnist  # noqa: E402
from myfyp_amd.learning.frameworks.torch import TorchModel  # noqa: E402
from myfyp_amd.management.logger import logger  # noqa: E402
from myfyp_amd.models import MLP, ResNet18  # noqa: E402
from myfyp_amd.node import Node  # noqa: E402
from myfyp_amd.parallel import weights_plane  # noqa: E402
from myfyp_amd.parallel.federation import Federation  # noqa: E402
from myfyp_amd.parallel.mlp_engine import MLPGroup  # noqa: E402
from myfyp_amd.settings import Settings  # noqa: E402
from myfyp_amd.utils.seed import set_seed  # noqa: E402
from myfyp_amd.utils.utils import wait_to_finish  # noqa: E402

FORCED = os.environ.get("MYFYP_FORCE_COLLECTIVE", "0") == "1"
CPU = os.environ.get("AGG_DEVICE", "cuda") == "cpu"  # CPU rehearsal: gloo world-1 group, small MLP
HIDDEN = [16, 8] if CPU else [256, 128]


def _sync() -> None:
    if not CPU:
        torch.cuda.synchronize()


INFO: dict = {"forced": FORCED, "cases": {}}


def _fresh() -> Federation:
    Federation.reset()
    MLPGroup.reset_all()
    fed = Federation.init()
    INFO["backend"] = None
    if fed.collective:
        import torch.distributed as dist

        INFO["backend"] = dist.get_backend(fed.group)
    return fed


def _record(fed: Federation, case: str) -> None:
    snap = fed.comm.snapshot()
    INFO["cases"][case] = {"solo": fed.solo, "comm_calls": {k: v["calls"] for k, v in snap.items()}, "recoveries": fed.recoveries}


def _flats(nodes):
    return torch.stack([weights_plane._pack(nd.learner).detach().float().cpu() for nd in nodes])


def _experiment(fed, case, make_model, data, n, rounds, batch, aggregator=FedAvg, rebuild=False):
    set_seed(21)
    parts = data.generate_partitions(n, RandomIIDPartitionStrategy)
    nodes = [Node(TorchModel(make_model(i)), parts[i], address=f"{case}-{i}", aggregator=aggregator(), protocol=CollectiveCommunicationProtocol,
                  learner_kwargs={"batch_size": batch}) for i in range(n)]
    try:
        for nd in nodes:
            nd.start()
        assert CPU or all(nd.learner._engine is not None for nd in nodes), "fused engine not attached"
        fed.finalize()
        if rebuild and fed.forced:  # group rebuild over the (same) survivors: new_group + abort of the old RCCL group
            fed._apply_members(list(fed.members), force=True)
        nodes[0].set_start_learning(rounds=rounds, epochs=1)
        wait_to_finish(nodes, timeout=300)
        _sync()
        _record(fed, case)
        return _flats(nodes)
    finally:
        for nd in nodes:
            nd.stop()


def case_mlp_fedavg(fed):
    Settings.TRAIN_SET_SIZE = 4
    return _experiment(fed, "mlp_fedavg", lambda i: MLP(hidden_sizes=HIDDEN, seed=i), synthetic_mnist(4000, 400, seed=5), 4, 3, 64, rebuild=True)


def case_mlp_delayed(fed):
    Settings.TRAIN_SET_SIZE = 4
    Settings.DELAYED_AVERAGING = True
    try:
        return _experiment(fed, "mlp_delayed", lambda i: MLP(hidden_sizes=HIDDEN, seed=i), synthetic_mnist(4000, 400, seed=5), 4, 3, 64)
    finally:
        Settings.DELAYED_AVERAGING = False


def case_resnet_train(fed):
    """Two rounds of ResNet-18 training + FedAvg through the pipeline (training itself is not
    bit-reproducible run to run: BN-backward sums use atomics, so only the peers' agreement is
    compared)."""
    Settings.TRAIN_SET_SIZE = 2
    return _experiment(fed, "resnet_train", lambda i: ResNet18(seed=40 + i), synthetic_cifar10(256, 64, seed=3), 2, 2, 32)


def case_resnet_fedavg(fed):
    """FedAvg of ResNet-18 engine rows (parameters + BN running statistics) set to seeded values:
    bucketed side-stream pipeline (forced) vs the one-launch local mean (solo)."""
    data = synthetic_cifar10(64, 16, seed=3)
    nodes = [Node(TorchModel(ResNet18(seed=50 + i)), data, address=f"rf-{i}", aggregator=FedAvg(), protocol=CollectiveCommunicationProtocol,
                  learner_kwargs={"batch_size": 32}) for i in range(3)]
    try:
        for nd in nodes:
            nd.start()
        fed.finalize()
        g = torch.Generator().manual_seed(17)
        with torch.no_grad():
            for nd in nodes:
                for t in weights_plane.state_tensors(nd.learner):
                    t.copy_(torch.randn(t.shape, generator=g).to(t.dtype))
        weights_plane.aggregate_mean(fed, {nd.addr: (w, None) for nd, w in zip(nodes, [3.0, 0.0, 5.0])}, final=True)
        fed.confirm_collectives()
        _sync()
        _record(fed, "resnet_fedavg")
        return _flats(nodes)
    finally:
        for nd in nodes:
            nd.stop()


def _direct_nodes(make_agg, k, tag):
    data = synthetic_mnist(200, 50)
    return [Node(TorchModel(MLP(hidden_sizes=HIDDEN, seed=i)), data, address=f"{tag}-{i}", aggregator=make_agg(), protocol=CollectiveCommunicationProtocol) for i in range(k)]


def case_init_broadcast(fed):
    nodes = _direct_nodes(FedAvg, 3, "bc")
    try:
        for nd in nodes:
            nd.start()
        fed.finalize()
        with torch.no_grad():
            for i, nd in enumerate(nodes):
                nd.learner.flat_params().copy_(torch.randn(nd.learner.flat_params().numel(), generator=torch.Generator().manual_seed(i)))
        weights_plane.sync_initial_model(fed, {nd.addr: None for nd in nodes}, nodes[1].addr)
        _sync()
        _record(fed, "init_broadcast")
        return _flats(nodes)
    finally:
        for nd in nodes:
            nd.stop()


def case_scaffold(fed):
    weights = [10.0, 0.0, 30.0, 20.0]
    nodes = _direct_nodes(lambda: Scaffold(global_lr=0.7), len(weights), "sc")
    try:
        for nd in nodes:
            nd.start()
        fed.finalize()
        g = torch.Generator().manual_seed(5)
        n = nodes[0].learner.flat_params().numel()
        x0 = torch.randn(n, generator=g)
        for nd in nodes:
            lr = nd.learner
            cb = weights_plane._scaffold_cb(lr)
            dev = lr.flat_params().device
            with torch.no_grad():
                lr.flat_params().copy_(x0)
            cb.x0 = x0.to(dev)
            cb.delta_y, cb.delta_c = (torch.randn(n, generator=g) * 0.1).to(dev), torch.randn(n, generator=g).to(dev)
        weights_plane.aggregate_scaffold(fed, {nd.addr: (w, None) for nd, w in zip(nodes, weights)}, nodes[0].aggregator)
        _sync()
        _record(fed, "scaffold")
        gc = torch.cat([t.detach().float().cpu().reshape(-1) for t in nodes[0].learner.get_model().get_info("scaffold")["global_c"]])
        return torch.cat([_flats(nodes), gc[None]])
    finally:
        for nd in nodes:
            nd.stop()


def case_median(fed):
    weights = [1.0, 0.0, 2.0, 3.0, 4.0]
    nodes = _direct_nodes(FedMedian, len(weights), "md")
    try:
        for nd in nodes:
            nd.start()
        fed.finalize()
        g = torch.Generator().manual_seed(9)
        with torch.no_grad():
            for nd in nodes:
                f = nd.learner.flat_params()
                f.copy_(torch.randn(f.numel(), generator=g))
        weights_plane.aggregate_median(fed, {nd.addr: (w, None) for nd, w in zip(nodes, weights)})
        _sync()
        _record(fed, "median")
        return _flats(nodes)
    finally:
        for nd in nodes:
            nd.stop()


CASES = {
    "init_broadcast": case_init_broadcast,
    "mlp_fedavg": case_mlp_fedavg,
    "mlp_delayed": case_mlp_delayed,
    "scaffold": case_scaffold,
    "median": case_median,
    "resnet_fedavg": case_resnet_fedavg,
    "resnet_train": case_resnet_train,
}


def main() -> None:
    assert CPU or torch.cuda.is_available()
    if CPU:
        Settings.DEVICE = "cpu"
        del CASES["resnet_fedavg"], CASES["resnet_train"]
    logger.set_level("WARNING")
    Settings.LOG_LEVEL = "WARNING"
    Settings.GANG_WINDOW = 5.0
    Settings.HEARTBEAT_TIMEOUT = 600
    Settings.VOTE_TIMEOUT = Settings.AGGREGATION_TIMEOUT = 600
    Settings.BUCKET_BYTES = 256 << 10  # several buckets even for the MLP: the pipeline really interleaves
    names = os.environ.get("CASES", ",".join(CASES)).split(",")
    out = {}
    for name in names:
        t0 = time.time()
        fed = _fresh()
        out[name] = CASES[name](fed)
        print(f"[forced={FORCED}] {name}: {time.time() - t0:.1f}s {INFO['cases'].get(name)}", flush=True)
    torch.save(out, os.environ["OUT"])
    with open(os.environ["OUT"] + ".json", "w") as f:
        json.dump(INFO, f)
    fed = Federation._instance
    if fed is not None:
        fed.shutdown()


if __name__ == "__main__":
    main()
