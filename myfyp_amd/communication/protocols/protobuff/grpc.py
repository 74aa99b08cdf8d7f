"""``p2pfl.communication.protocols.protobuff.grpc`` (newer upstream path)."""

from myfyp_amd.communication.protocols.grpc.grpc_communication_protocol import GrpcCommunicationProtocol

__all__ = ["GrpcCommunicationProtocol"]
