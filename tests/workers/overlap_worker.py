"""torchrun worker: FedAvg on the weights plane across ranks with 2 peers per rank.

Checks, on every rank:
* side-stream bucketed FedAvg (OVERLAP_COLLECTIVES, tiny buckets so there are many) is bit-equal
  to the synchronous path and matches the closed form;
* delayed averaging: round r keeps the local weights, round r+1 lands x += avg_r - x_r, the final
  round aggregates exactly.
AGG_DEVICE=cuda puts the peers on the fused engine (stacked rows, HIP kernels); default cpu.
"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from myfyp_amd.communication.protocols.collective.collective_protocol import CollectiveCommunicationProtocol  # noqa: E402
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
    hidden = [8, 8] if Settings.DEVICE == "cpu" else [256, 128]
    nodes = [Node(TorchModel(MLP(hidden_sizes=hidden)), synthetic_mnist(200, 50), address=f"o{g}", protocol=CollectiveCommunicationProtocol) for g in gids]
    for nd in nodes:
        nd.start()
    fed.finalize()
    flat = {g: nd.learner.flat_params() for g, nd in zip(gids, nodes)}
    n = flat[gids[0]].numel()
    dev = flat[gids[0]].device
    weights = {g: float(1 + g % 3) for g in range(world * PPR)}
    weights[1] = 0.0  # a non-trainer joins with weight 0
    arrived = {nd.addr: (weights[g], None) for g, nd in zip(gids, nodes)}
    tot = sum(weights.values())

    def set_rows(seed):
        with torch.no_grad():
            for g in gids:
                flat[g].copy_(_vec(seed + g, n).to(dev))

    def mean_of(seed):
        return sum(weights[g] * _vec(seed + g, n).double().numpy() for g in range(world * PPR)) / tot

    # ---- exact: overlapped (many buckets) vs synchronous, bitwise
    results = {}
    for overlap in (True, False):
        Settings.OVERLAP_COLLECTIVES = overlap
        Settings.BUCKET_BYTES = 64 << 10  # 16k floats per bucket
        set_rows(100)
        weights_plane.aggregate_mean(fed, arrived, final=True)
        results[overlap] = {g: flat[g].detach().cpu().clone() for g in gids}
    exp = mean_of(100)
    for g in gids:
        assert torch.equal(results[True][g], results[False][g]), f"overlapped != synchronous on peer {g}"
        assert np.abs(results[True][g].double().numpy() - exp).max() < 1e-5
    # ---- delayed averaging over three rounds
    Settings.DELAYED_AVERAGING = True
    set_rows(200)
    x0 = {g: _vec(200 + g, n).double().numpy() for g in range(world * PPR)}
    weights_plane.aggregate_mean(fed, arrived, final=False)
    for g in gids:  # round 0: local weights kept
        assert np.abs(flat[g].detach().cpu().double().numpy() - x0[g]).max() == 0.0
    with torch.no_grad():  # "training" of round 1
        for g in gids:
            flat[g].add_(_vec(300 + g, n).to(dev) * 0.01)
    x1 = {g: x0[g] + (_vec(300 + g, n) * 0.01).double().numpy() for g in range(world * PPR)}
    avg0 = sum(weights[g] * x0[g] for g in x0) / tot
    weights_plane.aggregate_mean(fed, arrived, final=False)
    for g in gids:  # round 1: the round-0 average landed as a correction, round-1 reduce started
        land = x1[g] + avg0 - x0[g]
        assert np.abs(flat[g].detach().cpu().double().numpy() - land).max() < 1e-5
    y1 = {g: x1[g] + avg0 - x0[g] for g in x1}
    weights_plane.aggregate_mean(fed, arrived, final=True)
    avg1 = sum(weights[g] * y1[g] for g in y1) / tot
    for g in gids:  # final round: landed, then exact average -> every peer equal
        # y1 + avg1 - y1 = avg1 for everyone, then the exact mean of equal rows = avg1
        assert np.abs(flat[g].detach().cpu().double().numpy() - avg1).max() < 1e-5
    Settings.DELAYED_AVERAGING = False
    print(f"rank {fed.rank} OK", flush=True)
    for nd in nodes:
        nd.stop()
    fed.shutdown()


if __name__ == "__main__":
    main()
