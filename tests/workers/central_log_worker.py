"""torchrun worker: a 3-round collective experiment over 2 ranks x 2 peers; rank 0 must see the
other rank's peers' metrics LIVE (relayed over the control bus), before any end-of-run merge."""

import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from myfyp_amd.communication.protocols.collective.collective_protocol import CollectiveCommunicationProtocol  # noqa: E402
from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy  # noqa: E402
from myfyp_amd.learning.dataset.synthetic import synthetic_mnist  # noqa: E402
from myfyp_amd.learning.frameworks.torch import TorchModel  # noqa: E402
from myfyp_amd.management.logger import logger  # noqa: E402
from myfyp_amd.models import MLP  # noqa: E402
from myfyp_amd.node import Node  # noqa: E402
from myfyp_amd.parallel.federation import Federation  # noqa: E402
from myfyp_amd.settings import Settings  # noqa: E402
from myfyp_amd.utils.utils import wait_to_finish  # noqa: E402

PPR = 2


def main() -> None:
    Settings.DEVICE = "cpu"
    Settings.BATCH_SIZE = 32
    Settings.TRAIN_SET_SIZE = 4
    Settings.CENTRAL_LOG_PERIOD = 0.2
    fed = Federation.init()
    parts = synthetic_mnist(2000, 400, seed=3).generate_partitions(fed.world * PPR, RandomIIDPartitionStrategy)
    gids = [fed.rank * PPR + j for j in range(PPR)]
    nodes = [Node(TorchModel(MLP(hidden_sizes=[16, 16], seed=g)), parts[g], address=f"cl{g}", protocol=CollectiveCommunicationProtocol, exp_name="central")
             for g in gids]
    for nd in nodes:
        nd.start()
    fed.finalize()
    if fed.rank == 0:
        nodes[0].set_start_learning(rounds=3, epochs=1)
    wait_to_finish(nodes, timeout=120)
    if fed.rank == 0:
        remote = [f"cl{g}" for g in range(PPR, fed.world * PPR)]
        deadline = time.time() + 10
        while time.time() < deadline:
            logs = logger.get_global_logs().get("central", {})
            if all(len(logs.get(a, {}).get("test_metric", [])) >= 3 for a in remote):
                break
            time.sleep(0.1)
        logs = logger.get_global_logs().get("central", {})
        for a in remote:
            assert len(logs.get(a, {}).get("test_metric", [])) >= 3, (a, logs.get(a))
        local = logger.get_local_logs().get("central", {})
        assert any(a in nodes_ for nodes_ in local.values() for a in remote), "no relayed local (per-step) metrics"
        assert fed.central is not None and fed.central.received > 0
    else:
        assert fed.central is not None
        fed.central.flush()
        assert fed.central.sent > 0
    print(f"rank {fed.rank} OK", flush=True)
    for nd in nodes:
        nd.stop()
    fed.shutdown()


if __name__ == "__main__":
    main()
