"""gRPC client side (parity: ``protocols/grpc/grpc_client.py:54-206``).

:class:`GrpcStub` is one peer's channel + ``NodeServicesStub`` exposing the generic stub interface
(``handle_message``/``handle_weights``/``handshake``/``remote_disconnect``) that
:class:`~myfyp_amd.communication.protocols.client.StubClient` drives, so the gRPC and in-memory
transports share one send/broadcast/remove-on-error implementation. :class:`GrpcClient` is that
client for gRPC neighbours. Channels are secure (mTLS) when ``Settings.USE_SSL`` and every
certificate file exists.
"""

from __future__ import annotations

import os

import grpc

from myfyp_amd.communication.protocols.client import StubClient
from myfyp_amd.communication.protocols.exceptions import NeighborNotConnectedError
from myfyp_amd.communication.protocols.grpc import proto
from myfyp_amd.communication.protocols.grpc.proto.node_pb2_grpc import NodeServicesStub
from myfyp_amd.settings import Settings

MAX_MESSAGE_BYTES = 1024 * 1024 * 1024
CHANNEL_OPTIONS = [("grpc.max_send_message_length", MAX_MESSAGE_BYTES), ("grpc.max_receive_message_length", MAX_MESSAGE_BYTES)]


def ssl_enabled() -> bool:
    return bool(Settings.USE_SSL) and all(os.path.exists(p) for p in (Settings.CA_CRT, Settings.SERVER_CRT, Settings.SERVER_KEY, Settings.CLIENT_CRT, Settings.CLIENT_KEY))


def read_file(p: str) -> bytes:
    with open(p, "rb") as f:
        return f.read()


def to_proto(msg: dict):
    """Transport-neutral message dict → ``RootMessage``."""
    if "weights" in msg:
        return proto.RootMessage(
            source=msg["source"],
            round=msg["round"],
            cmd=msg["cmd"],
            weights=proto.Weights(weights=msg["weights"], contributors=list(msg["contributors"]), num_samples=int(msg["weight"])),
        )
    return proto.RootMessage(
        source=msg["source"], round=msg["round"], cmd=msg["cmd"], message=proto.Message(ttl=msg["ttl"], hash=msg["hash"], args=list(msg["args"]))
    )


def from_proto(req) -> dict:
    """``RootMessage`` → transport-neutral message dict (round -1 when unset)."""
    rnd = req.round if req.HasField("round") else -1
    if req.WhichOneof("payload_type") == "weights":
        w = req.weights
        return {"source": req.source, "round": rnd, "cmd": req.cmd, "weights": w.weights, "contributors": list(w.contributors), "weight": w.num_samples}
    m = req.message
    return {"source": req.source, "round": rnd, "cmd": req.cmd, "ttl": m.ttl, "hash": m.hash, "args": list(m.args)}


class GrpcStub:
    """Client-side stub for one peer."""

    def __init__(self, self_addr: str, addr: str) -> None:
        self.self_addr = self_addr
        self.addr = addr
        if ssl_enabled():
            creds = grpc.ssl_channel_credentials(
                root_certificates=read_file(Settings.CA_CRT), private_key=read_file(Settings.CLIENT_KEY), certificate_chain=read_file(Settings.CLIENT_CRT)
            )
            self.channel = grpc.secure_channel(addr, creds, options=CHANNEL_OPTIONS)
        else:
            self.channel = grpc.insecure_channel(addr, options=CHANNEL_OPTIONS)
        self.stub = NodeServicesStub(self.channel)

    def is_running(self) -> bool:
        return True

    def _call(self, msg: dict) -> dict:
        res = self.stub.send(to_proto(msg), timeout=Settings.GRPC_TIMEOUT)
        return {"error": res.error} if res.HasField("error") else {}

    handle_message = _call
    handle_weights = _call

    def handshake(self, addr: str) -> bool:
        res = self.stub.handshake(proto.HandShakeRequest(addr=addr), timeout=Settings.GRPC_TIMEOUT)
        if res.HasField("error"):
            raise NeighborNotConnectedError(res.error)
        return True

    def remote_disconnect(self, addr: str) -> None:
        try:
            self.stub.disconnect(proto.HandShakeRequest(addr=addr), timeout=Settings.GRPC_TIMEOUT)
        finally:
            self.channel.close()

    def close(self) -> None:
        self.channel.close()


class GrpcClient(StubClient):
    """``build_message``/``build_weights``/``send``/``broadcast`` over gRPC neighbour stubs."""
