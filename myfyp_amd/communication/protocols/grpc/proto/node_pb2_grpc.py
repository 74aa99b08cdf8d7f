"""``node.NodeServices`` service bindings (parity: ``grpc/proto/node_pb2_grpc.py``): the client
stub, the servicer base class and ``add_NodeServicesServicer_to_server``.

Method paths are ``/node.NodeServices/{handshake,disconnect,send}`` with the reference request and
response types, so reference p2pfl peers and these peers call each other unchanged.
"""

from __future__ import annotations

import grpc

from myfyp_amd.communication.protocols.grpc.proto import SERVICE, Empty, HandShakeRequest, ResponseMessage, RootMessage

_SER = lambda m: m.SerializeToString()  # noqa: E731
# name → (request type, response type)
METHODS = {
    "handshake": (HandShakeRequest, ResponseMessage),
    "disconnect": (HandShakeRequest, Empty),
    "send": (RootMessage, ResponseMessage),
}


class NodeServicesStub:
    """Client-side callables ``handshake``, ``disconnect``, ``send`` bound to one channel."""

    def __init__(self, channel: grpc.Channel) -> None:
        for name, (_, resp) in METHODS.items():
            setattr(self, name, channel.unary_unary(f"/{SERVICE}/{name}", request_serializer=_SER, response_deserializer=resp.FromString))


class NodeServicesServicer:
    """Server-side interface; subclasses implement the three RPCs."""

    def handshake(self, request, context):
        context.set_code(grpc.StatusCode.UNIMPLEMENTED)
        raise NotImplementedError("handshake")

    def disconnect(self, request, context):
        context.set_code(grpc.StatusCode.UNIMPLEMENTED)
        raise NotImplementedError("disconnect")

    def send(self, request, context):
        context.set_code(grpc.StatusCode.UNIMPLEMENTED)
        raise NotImplementedError("send")


def add_NodeServicesServicer_to_server(servicer: NodeServicesServicer, server: grpc.Server) -> None:
    handlers = {
        name: grpc.unary_unary_rpc_method_handler(getattr(servicer, name), request_deserializer=req.FromString, response_serializer=_SER)
        for name, (req, _) in METHODS.items()
    }
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(SERVICE, handlers),))
