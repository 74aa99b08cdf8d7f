"""gRPC transport over TCP and Unix sockets (+ mTLS when openssl is available)."""

import os
import shutil
import subprocess
import time

import pytest

from myfyp_amd.communication.commands.command import Command
from myfyp_amd.communication.protocols.grpc.grpc_communication_protocol import GrpcCommunicationProtocol, from_proto, to_proto
from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
from myfyp_amd.learning.frameworks.torch import TorchModel
from myfyp_amd.models import MLP
from myfyp_amd.node import Node
from myfyp_amd.settings import Settings
from myfyp_amd.utils.utils import check_equal_models, wait_convergence, wait_to_finish


class Rec(Command):
    def __init__(self):
        self.got = []

    @staticmethod
    def get_name():
        return "rec"

    def execute(self, source, round, *args, **kwargs):
        self.got.append((source, round, args, kwargs.get("weights")))


def test_proto_roundtrip():
    msg = {"source": "a", "round": 2, "cmd": "x", "ttl": 3, "hash": 99, "args": ["1", "2"]}
    assert from_proto(to_proto(msg)) == msg
    w = {"source": "a", "round": 1, "cmd": "w", "weights": b"abc", "contributors": ["a"], "weight": 7}
    assert from_proto(to_proto(w)) == w


@pytest.mark.parametrize("unix", [False, True])
def test_grpc_messages_and_weights(unix, tmp_path):
    addrs = [f"unix://{tmp_path}/n{i}.sock" for i in range(2)] if unix else ["127.0.0.1", "127.0.0.1"]
    a, b = GrpcCommunicationProtocol(addrs[0]), GrpcCommunicationProtocol(addrs[1])
    rec = Rec()
    b.add_command(rec)
    a.start()
    b.start()
    try:
        assert a.connect(b.get_address())
        wait_convergence([a, b], 1, wait=5)
        a.send(b.get_address(), a.build_msg("rec", ["hello"], round=4))
        a.send(b.get_address(), a.build_weights("rec", 5, b"\x00\x01payload", ["a"], 3))
        deadline = time.time() + 5
        while len(rec.got) < 2 and time.time() < deadline:
            time.sleep(0.05)
        assert rec.got[0][:3] == (a.get_address(), 4, ("hello",))
        assert rec.got[1][3] == b"\x00\x01payload"
    finally:
        a.stop()
        b.stop()


def test_grpc_two_node_learning():
    Settings.BATCH_SIZE = 16
    parts = synthetic_mnist(2000, 200, seed=9, similarity=0.3).generate_partitions(2, RandomIIDPartitionStrategy)
    from myfyp_amd.communication.protocols.grpc.grpc_communication_protocol import GrpcCommunicationProtocol as G

    nodes = [Node(TorchModel(MLP(seed=i)), parts[i], address="127.0.0.1", protocol=G) for i in range(2)]
    for n in nodes:
        n.start()
    try:
        nodes[0].connect(nodes[1].addr)
        wait_convergence(nodes, 1, wait=10)
        nodes[0].set_start_learning(rounds=1, epochs=1)
        wait_to_finish(nodes, timeout=120)
        check_equal_models(nodes)
    finally:
        for n in nodes:
            n.stop()


@pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl not available")
def test_grpc_mtls(tmp_path):
    src = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "myfyp_amd", "certificates", "gen-certs.sh")
    shutil.copy(src, tmp_path)
    subprocess.run(["bash", str(tmp_path / "gen-certs.sh")], check=True, capture_output=True)
    Settings.USE_SSL = True
    Settings.CA_CRT, Settings.SERVER_CRT, Settings.SERVER_KEY = str(tmp_path / "ca.crt"), str(tmp_path / "server.crt"), str(tmp_path / "server.key")
    Settings.CLIENT_CRT, Settings.CLIENT_KEY = str(tmp_path / "client.crt"), str(tmp_path / "client.key")
    a, b = GrpcCommunicationProtocol("127.0.0.1"), GrpcCommunicationProtocol("127.0.0.1")
    rec = Rec()
    b.add_command(rec)
    a.start()
    b.start()
    try:
        assert a.connect(b.get_address())
        a.send(b.get_address(), a.build_msg("rec", ["secure"]))
        deadline = time.time() + 5
        while not rec.got and time.time() < deadline:
            time.sleep(0.05)
        assert rec.got and rec.got[0][2] == ("secure",)
    finally:
        a.stop()
        b.stop()
