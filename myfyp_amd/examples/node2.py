"""gRPC node 2 of the two-process quickstart: connects to node 1 on --port and runs 2 rounds."""

# Parity: p2pfl/examples/node2.py:43-67. Data: synthetic MNIST-shaped (no network).

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


def node2(port: int, rounds: int = 2, epochs: int = 1, n_train: int = 6000) -> None:
    set_test_settings()
    data = synthetic_mnist(n_train, n_train // 6, seed=1).generate_partitions(2, RandomIIDPartitionStrategy)[1]
    node = Node(TorchModel(MLP()), data, address="127.0.0.1", protocol=GrpcCommunicationProtocol)
    node.start()
    try:
        node.connect(f"127.0.0.1:{port}")
        time.sleep(1)
        print("Start learning", flush=True)
        node.set_start_learning(rounds=rounds, epochs=epochs)
        while node.state.round is not None or not node.learning_workflow.finished:
            time.sleep(0.2)
        print("Learning finished", flush=True)
    finally:
        node.stop()


if __name__ == "__main__":
    ap = argparse.ArgumentParser(description="gRPC MNIST node (initiator).")
    ap.add_argument("--port", type=int, required=True, help="The port to connect.")
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    node2(a.port, a.rounds)
