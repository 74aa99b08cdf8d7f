"""gRPC transport (parity: ``protocols/grpc/grpc_communication_protocol.py:49-263``).

Unary RPCs ``handshake``/``disconnect``/``send`` on ``node.NodeServices`` with the reference's
protobuf schema (``proto/``); TCP (IPv4/IPv6) or Unix-domain sockets; optional mutual TLS when
``Settings.USE_SSL`` and the certificate files exist (``certificates/gen-certs.sh``). Weights travel
as the pickle wire format in ``Weights.weights``. The pieces live in the reference's module layout:
``grpc_client`` (stub + client), ``grpc_neighbors``, ``grpc_server`` (servicer + server lifecycle).
"""

from __future__ import annotations

from myfyp_amd.communication.protocols.base_protocol import BaseCommunicationProtocol
from myfyp_amd.communication.protocols.client import Client
from myfyp_amd.communication.protocols.grpc.address import AddressParser
from myfyp_amd.communication.protocols.grpc.grpc_client import GrpcClient, GrpcStub, from_proto, to_proto  # noqa: F401 (re-exports)
from myfyp_amd.communication.protocols.grpc.grpc_neighbors import GrpcNeighbors
from myfyp_amd.communication.protocols.grpc.grpc_server import GrpcServer
from myfyp_amd.communication.protocols.neighbors import Neighbors


class GrpcCommunicationProtocol(BaseCommunicationProtocol):
    """Reference-compatible gRPC transport."""

    def __init__(self, addr: str = "127.0.0.1", commands=None) -> None:
        self._server = GrpcServer(self)
        super().__init__(addr, commands)

    def parse_address(self, addr: str) -> str:
        return AddressParser(addr or "127.0.0.1").get_parsed_address()

    def build_neighbors(self, addr: str) -> Neighbors:
        return GrpcNeighbors(addr)

    def build_client(self, addr: str, neighbors: Neighbors) -> Client:
        return GrpcClient(addr, neighbors)

    def start_transport(self) -> None:
        self._server.start()

    def stop_transport(self) -> None:
        self._server.stop()

    def wait_for_termination(self) -> None:
        self._server.wait_for_termination()
