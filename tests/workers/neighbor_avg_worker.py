"""torchrun worker: 2 peers per rank on a ring; checks one NeighborAvg mixing step exactly."""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from myfyp_amd.communication.protocols.collective.collective_protocol import CollectiveCommunicationProtocol  # noqa: E402
from myfyp_amd.learning.aggregators.neighbor_avg import NeighborAvg  # noqa: E402
from myfyp_amd.learning.dataset.synthetic import synthetic_mnist  # noqa: E402
from myfyp_amd.learning.frameworks.torch import TorchModel  # noqa: E402
from myfyp_amd.models import MLP  # noqa: E402
from myfyp_amd.node import Node  # noqa: E402
from myfyp_amd.parallel import weights_plane  # noqa: E402
from myfyp_amd.parallel.federation import Federation  # noqa: E402


def main() -> None:
    fed = Federation.init()
    ppr = 2
    data = synthetic_mnist(200, 50)
    gids = [fed.rank * ppr + j for j in range(ppr)]
    agg = NeighborAvg(topology="ring")
    nodes = [Node(TorchModel(MLP(hidden_sizes=[8, 8])), data, address=f"p{g}", aggregator=agg, protocol=CollectiveCommunicationProtocol) for g in gids]
    for nd in nodes:
        nd.start()
    fed.finalize()
    for g, nd in zip(gids, nodes):
        with torch.no_grad():
            nd.learner.flat_params().fill_(float(g + 1))
    weights_plane.aggregate_neighbors(fed, {nd.addr: None for nd in nodes}, agg)
    peers = fed.all_peers()
    w = agg.mixing_matrix(len(peers))
    vals = np.array([float(peers.index(f"p{g}") + 1) for g in range(len(peers))])
    for g, nd in zip(gids, nodes):
        expect = float(w[peers.index(nd.addr)] @ np.array([float(int(p[1:]) + 1) for p in peers]))
        got = nd.learner.flat_params()
        assert torch.allclose(got, torch.full_like(got, expect), atol=1e-5), (nd.addr, float(got[0]), expect)
    print(f"rank {fed.rank} OK", flush=True)
    for nd in nodes:
        nd.stop()
    fed.shutdown()


if __name__ == "__main__":
    main()
