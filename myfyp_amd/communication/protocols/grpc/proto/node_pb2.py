"""Message classes of ``node.proto`` under the module name protoc would generate
(parity: ``p2pfl/communication/protocols/grpc/proto/node_pb2.py``).

The classes come from the descriptor assembled in :mod:`..proto` at import time; no generated
code is checked in, so there is no protoc/grpcio-tools step and no version skew between the stubs
and the installed protobuf runtime.
"""

from myfyp_amd.communication.protocols.grpc.proto import Empty, HandShakeRequest, Message, ResponseMessage, RootMessage, Weights

__all__ = ["Message", "Weights", "RootMessage", "HandShakeRequest", "ResponseMessage", "Empty"]
