"""gRPC transport (parity: ``protocols/grpc/*``: server, client, neighbours, mTLS).

Unary RPCs ``handshake``/``disconnect``/``send`` on ``node.NodeServices`` with the reference's
protobuf schema (``proto.py``); TCP (IPv4/IPv6) or Unix-domain sockets; optional mutual TLS when
``Settings.USE_SSL`` and the certificate files exist (``certificates/gen-certs.sh``). Weights travel
as the pickle wire format in ``Weights.weights``.

Differences from the reference: the server thread pool scales with the host (reference: 2
workers, ``grpc_server.py:67``) and message-size limits are raised to 1 GiB on both ends.
"""

from __future__ import annotations

import os
from concurrent import futures
from typing import Any, Dict, Optional

import grpc

from myfyp_amd.communication.protocols.base_protocol import BaseCommunicationProtocol
from myfyp_amd.communication.protocols.client import Client, StubClient
from myfyp_amd.communication.protocols.exceptions import NeighborNotConnectedError
from myfyp_amd.communication.protocols.grpc import proto
from myfyp_amd.communication.protocols.grpc.address import AddressParser
from myfyp_amd.communication.protocols.neighbors import Neighbors
from myfyp_amd.management.logger import logger
from myfyp_amd.settings import Settings

_MAX_MSG = 1024 * 1024 * 1024
_OPTIONS = [("grpc.max_send_message_length", _MAX_MSG), ("grpc.max_receive_message_length", _MAX_MSG)]


def _ssl_enabled() -> bool:
    return bool(Settings.USE_SSL) and all(os.path.exists(p) for p in (Settings.CA_CRT, Settings.SERVER_CRT, Settings.SERVER_KEY, Settings.CLIENT_CRT, Settings.CLIENT_KEY))


def _read(p: str) -> bytes:
    with open(p, "rb") as f:
        return f.read()


def to_proto(msg: dict):
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
    rnd = req.round if req.HasField("round") else -1
    if req.WhichOneof("payload_type") == "weights":
        w = req.weights
        return {"source": req.source, "round": rnd, "cmd": req.cmd, "weights": w.weights, "contributors": list(w.contributors), "weight": w.num_samples}
    m = req.message
    return {"source": req.source, "round": rnd, "cmd": req.cmd, "ttl": m.ttl, "hash": m.hash, "args": list(m.args)}


class GrpcStub:
    """Client-side stub for one peer, exposing the generic stub interface."""

    def __init__(self, self_addr: str, addr: str) -> None:
        self.self_addr = self_addr
        self.addr = addr
        if _ssl_enabled():
            creds = grpc.ssl_channel_credentials(root_certificates=_read(Settings.CA_CRT), private_key=_read(Settings.CLIENT_KEY), certificate_chain=_read(Settings.CLIENT_CRT))
            self.channel = grpc.secure_channel(addr, creds, options=_OPTIONS)
        else:
            self.channel = grpc.insecure_channel(addr, options=_OPTIONS)
        self._send = self.channel.unary_unary(f"/{proto.SERVICE}/send", request_serializer=lambda m: m.SerializeToString(), response_deserializer=proto.ResponseMessage.FromString)
        self._handshake = self.channel.unary_unary(
            f"/{proto.SERVICE}/handshake", request_serializer=lambda m: m.SerializeToString(), response_deserializer=proto.ResponseMessage.FromString
        )
        self._disconnect = self.channel.unary_unary(f"/{proto.SERVICE}/disconnect", request_serializer=lambda m: m.SerializeToString(), response_deserializer=proto.Empty.FromString)

    def is_running(self) -> bool:
        return True

    def _call(self, msg: dict) -> dict:
        res = self._send(to_proto(msg), timeout=Settings.GRPC_TIMEOUT)
        return {"error": res.error} if res.HasField("error") else {}

    handle_message = _call
    handle_weights = _call

    def handshake(self, addr: str) -> bool:
        res = self._handshake(proto.HandShakeRequest(addr=addr), timeout=Settings.GRPC_TIMEOUT)
        if res.HasField("error"):
            raise NeighborNotConnectedError(res.error)
        return True

    def remote_disconnect(self, addr: str) -> None:
        try:
            self._disconnect(proto.HandShakeRequest(addr=addr), timeout=Settings.GRPC_TIMEOUT)
        finally:
            self.channel.close()

    def close(self) -> None:
        self.channel.close()


class GrpcNeighbors(Neighbors):
    """Direct neighbour = channel + stub (+ handshake RPC)."""

    def connect(self, addr: str, non_direct: bool = False, handshake_msg: bool = True) -> Any:
        if non_direct:
            return (None, None, self.now())
        stub = GrpcStub(self.self_addr, addr)
        if handshake_msg:
            try:
                stub.handshake(self.self_addr)
            except Exception:
                stub.close()
                raise
        return (stub.channel, stub, self.now())

    def disconnect(self, addr: str, disconnect_msg: bool = True) -> None:
        entry = self.neis.get(addr)
        if entry is None or entry[1] is None:
            return
        try:
            if disconnect_msg:
                entry[1].remote_disconnect(self.self_addr)
            else:
                entry[1].close()
        except Exception:
            pass

    def temporary_stub(self, addr: str):
        return GrpcStub(self.self_addr, addr)


class GrpcCommunicationProtocol(BaseCommunicationProtocol):
    """Reference-compatible gRPC transport."""

    def __init__(self, addr: str = "127.0.0.1", commands=None) -> None:
        self._server: Optional[grpc.Server] = None
        super().__init__(addr, commands)

    def parse_address(self, addr: str) -> str:
        return AddressParser(addr or "127.0.0.1").get_parsed_address()

    def build_neighbors(self, addr: str) -> Neighbors:
        return GrpcNeighbors(addr)

    def build_client(self, addr: str, neighbors: Neighbors) -> Client:
        return StubClient(addr, neighbors)

    # ------------------------------------------------------------------ server
    def _rpc_handshake(self, req, ctx):
        if self.handshake(req.addr):
            return proto.ResponseMessage()
        return proto.ResponseMessage(error="Cannot add the node (duplicated or wrong direction)")

    def _rpc_disconnect(self, req, ctx):
        self.remote_disconnect(req.addr)
        return proto.Empty()

    def _rpc_send(self, req, ctx):
        msg = from_proto(req)
        res = self.handle_weights(msg) if "weights" in msg else self.handle_message(msg)
        return proto.ResponseMessage(error=res["error"]) if "error" in res else proto.ResponseMessage()

    def start_transport(self) -> None:
        workers = max(4, min(32, (os.cpu_count() or 4)))
        server = grpc.server(futures.ThreadPoolExecutor(max_workers=workers), options=_OPTIONS)
        handlers = {
            "handshake": grpc.unary_unary_rpc_method_handler(self._rpc_handshake, request_deserializer=proto.HandShakeRequest.FromString, response_serializer=lambda m: m.SerializeToString()),
            "disconnect": grpc.unary_unary_rpc_method_handler(self._rpc_disconnect, request_deserializer=proto.HandShakeRequest.FromString, response_serializer=lambda m: m.SerializeToString()),
            "send": grpc.unary_unary_rpc_method_handler(self._rpc_send, request_deserializer=proto.RootMessage.FromString, response_serializer=lambda m: m.SerializeToString()),
        }
        server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(proto.SERVICE, handlers),))
        if _ssl_enabled():
            creds = grpc.ssl_server_credentials([(_read(Settings.SERVER_KEY), _read(Settings.SERVER_CRT))], root_certificates=_read(Settings.CA_CRT), require_client_auth=True)
            server.add_secure_port(self.addr, creds)
        else:
            server.add_insecure_port(self.addr)
        server.start()
        self._server = server
        logger.info(self.addr, f"gRPC server started at {self.addr}")

    def stop_transport(self) -> None:
        if self._server is not None:
            self._server.stop(0.5)
            self._server = None

    def wait_for_termination(self) -> None:
        if self._server is not None:
            self._server.wait_for_termination()
