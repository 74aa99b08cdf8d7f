"""gRPC server side (parity: ``protocols/grpc/grpc_server.py:48-237``).

:class:`GrpcServer` is the ``NodeServices`` servicer of one protocol: it decodes ``RootMessage``s
and hands them to the protocol's transport-independent dispatch (dedup → TTL relay → command,
``base_protocol.BaseCommunicationProtocol.handle_message``), and owns the ``grpc.Server``
lifecycle (TCP or ``unix://`` address, mTLS with client authentication when enabled).

Difference from the reference: the RPC thread pool scales with the host (reference: 2 workers,
``grpc_server.py:67``), so a burst of partial models cannot queue behind two slow handlers.
"""

from __future__ import annotations

import os
from concurrent import futures
from typing import Optional

import grpc

from myfyp_amd.communication.protocols.grpc import proto
from myfyp_amd.communication.protocols.grpc.grpc_client import CHANNEL_OPTIONS, from_proto, read_file, ssl_enabled
from myfyp_amd.communication.protocols.grpc.proto.node_pb2_grpc import NodeServicesServicer, add_NodeServicesServicer_to_server
from myfyp_amd.management.logger import logger
from myfyp_amd.settings import Settings


class GrpcServer(NodeServicesServicer):
    def __init__(self, protocol) -> None:
        self.protocol = protocol
        self._server: Optional[grpc.Server] = None

    # ------------------------------------------------------------------ RPCs
    def handshake(self, request, context):
        if self.protocol.handshake(request.addr):
            return proto.ResponseMessage()
        return proto.ResponseMessage(error="Cannot add the node (duplicated or wrong direction)")

    def disconnect(self, request, context):
        self.protocol.remote_disconnect(request.addr)
        return proto.Empty()

    def send(self, request, context):
        msg = from_proto(request)
        res = self.protocol.handle_weights(msg) if "weights" in msg else self.protocol.handle_message(msg)
        return proto.ResponseMessage(error=res["error"]) if "error" in res else proto.ResponseMessage()

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> None:
        addr = self.protocol.addr
        workers = max(4, min(32, (os.cpu_count() or 4)))
        server = grpc.server(futures.ThreadPoolExecutor(max_workers=workers), options=CHANNEL_OPTIONS)
        add_NodeServicesServicer_to_server(self, server)
        if ssl_enabled():
            creds = grpc.ssl_server_credentials(
                [(read_file(Settings.SERVER_KEY), read_file(Settings.SERVER_CRT))], root_certificates=read_file(Settings.CA_CRT), require_client_auth=True
            )
            server.add_secure_port(addr, creds)
        else:
            server.add_insecure_port(addr)
        server.start()
        self._server = server
        logger.info(addr, f"gRPC server started at {addr}")

    def stop(self, grace: float = 0.5) -> None:
        if self._server is not None:
            self._server.stop(grace)
            self._server = None

    def wait_for_termination(self) -> None:
        if self._server is not None:
            self._server.wait_for_termination()
