"""torchrun worker: 2 peers per rank; one device SCAFFOLD step and one device FedMedian step across
the ranks, checked against the closed forms every rank can compute from the shared seeds."""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from myfyp_amd.communication.protocols.collective.collective_protocol import CollectiveCommunicationProtocol  # noqa: E402
from myfyp_amd.learning.aggregators import FedMedian, Scaffold  # noqa: E402
from myfyp_amd.learning.dataset.synthetic import synthetic_mnist  # noqa: E402
from myfyp_amd.learning.frameworks.torch import TorchModel  # noqa: E402
from myfyp_amd.models import MLP  # noqa: E402
from myfyp_amd.node import Node  # noqa: E402
from myfyp_amd.parallel import weights_plane  # noqa: E402
from myfyp_amd.parallel.federation import Federation  # noqa: E402
from myfyp_amd.settings import Settings  # noqa: E402

PPR = 2


def _vec(seed, n):
    return torch.randn(n, generator=torch.Generator().manual_seed(seed))


def main() -> None:
    Settings.DEVICE = os.environ.get("AGG_DEVICE", "cpu")
    fed = Federation.init()
    world = fed.world
    gids = [fed.rank * PPR + j for j in range(PPR)]
    data = synthetic_mnist(200, 50)
    weights = {g: float(g % 3) for g in range(world * PPR)}  # peers 0 and 3 are non-trainers
    hidden = [8, 8] if Settings.DEVICE == "cpu" else [256, 128]  # fused MLP engine rows on the GPU
    sc = [Node(TorchModel(MLP(hidden_sizes=hidden)), data, address=f"s{g}", aggregator=Scaffold(global_lr=0.5), protocol=CollectiveCommunicationProtocol) for g in gids]
    md = [Node(TorchModel(MLP(hidden_sizes=hidden)), data, address=f"m{g}", aggregator=FedMedian(), protocol=CollectiveCommunicationProtocol) for g in gids]
    for nd in sc + md:
        nd.start()
    fed.finalize()
    n = sc[0].learner.flat_params().numel()
    x0 = _vec(1, n)
    for g, nd in zip(gids, sc):
        cb = weights_plane._scaffold_cb(nd.learner)
        with torch.no_grad():
            nd.learner.flat_params().copy_(x0.to(nd.learner.flat_params().device))
        dev = nd.learner.flat_params().device
        cb.x0, cb.delta_y, cb.delta_c = x0.to(dev), (_vec(100 + g, n) * 0.1).to(dev), _vec(200 + g, n).to(dev)
    weights_plane.aggregate_scaffold(fed, {nd.addr: (weights[g], None) for g, nd in zip(gids, sc)}, sc[0].aggregator)
    tr = [g for g in range(world * PPR) if weights[g] > 0]
    tot = sum(weights[g] for g in tr)
    x_exp = x0.double().numpy() + 0.5 * sum(weights[g] * (_vec(100 + g, n) * 0.1).double().numpy() for g in tr) / tot
    c_exp = sum(_vec(200 + g, n).double().numpy() for g in tr) / len(tr)
    for nd in sc:
        assert np.abs(nd.learner.flat_params().double().cpu().numpy() - x_exp).max() < 1e-6
        gc = np.concatenate([t.double().cpu().numpy().ravel() for t in nd.learner.get_model().get_info("scaffold")["global_c"]])
        assert np.abs(gc - c_exp).max() < 1e-6
    for g, nd in zip(gids, md):
        with torch.no_grad():
            nd.learner.flat_params().copy_(_vec(300 + g, n).to(nd.learner.flat_params().device))
    weights_plane.aggregate_median(fed, {nd.addr: (weights[g], None) for g, nd in zip(gids, md)})
    med = np.median(np.stack([_vec(300 + g, n).double().numpy() for g in tr]), axis=0)
    for nd in md:
        assert np.abs(nd.learner.flat_params().double().cpu().numpy() - med).max() < 1e-6
    print(f"rank {fed.rank} OK", flush=True)
    for nd in sc + md:
        nd.stop()
    fed.shutdown()


if __name__ == "__main__":
    main()
