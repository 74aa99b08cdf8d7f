"""gRPC neighbours (parity: ``protocols/grpc/grpc_neighbors.py:35-144``): a direct neighbour is a
channel + stub opened with a ``handshake`` RPC; a non-direct one (learned from relayed heartbeats)
is ``(None, None, last_beat)``."""

from __future__ import annotations

from typing import Any

from myfyp_amd.communication.protocols.grpc.grpc_client import GrpcStub
from myfyp_amd.communication.protocols.neighbors import Neighbors


class GrpcNeighbors(Neighbors):
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
