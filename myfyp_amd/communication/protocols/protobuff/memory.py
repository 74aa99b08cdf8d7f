"""``p2pfl.communication.protocols.protobuff.memory`` (newer upstream path, ``exp_SAVE3.txt:9``)."""

from myfyp_amd.communication.protocols.memory.memory_communication_protocol import InMemoryCommunicationProtocol

MemoryCommunicationProtocol = InMemoryCommunicationProtocol

__all__ = ["InMemoryCommunicationProtocol", "MemoryCommunicationProtocol"]
