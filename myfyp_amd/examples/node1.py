"""gRPC node 1 of the two-process quickstart: listens on --port until stopped (or --wait seconds)."""

# Parity: p2pfl/examples/node1.py:42-55. Data: synthetic MNIST-shaped (no network).

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from myfyp_amd.communication.protocols.grpc.grpc_communication_protocol import GrpcCommunicationProtocol  # noqa: E402
from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy  # noqa: E402
from myfyp_amd.learning.dataset.synthetic import synthetic_mnist  # noqa: E402
from myfyp_amd.learning.frameworks.torch import TorchModel  # noqa: E402
from myfyp_amd.models import MLP  # noqa: E402
from myfyp_amd.node import Node  # noqa: E402
from myfyp_amd.utils.utils import set_test_settings  # noqa: E402


def node1(port: int, wait: float = 0.0, n_train: int = 6000) -> None:
    set_test_settings()
    data = synthetic_mnist(n_train, n_train // 6, seed=1).generate_partitions(2, RandomIIDPartitionStrategy)[0]
    node = Node(TorchModel(MLP()), data, address=f"127.0.0.1:{port}", protocol=GrpcCommunicationProtocol)
    node.start()
    try:
        if wait > 0:
            deadline = time.time() + wait
            while time.time() < deadline:
                time.sleep(0.2)
        else:
            input("Press any key to stop\n")
    finally:
        node.stop()


if __name__ == "__main__":
    ap = argparse.ArgumentParser(description="gRPC MNIST node (listener).")
    ap.add_argument("--port", type=int, required=True, help="The port.")
    ap.add_argument("--wait", type=float, default=0.0, help="Run for this many seconds instead of waiting for a key.")
    a = ap.parse_args()
    node1(a.port, a.wait)
