"""Newer upstream p2pfl's ``communication.protocols.protobuff`` import paths, as the FYP scripts use
them (``/root/reference/exp_SAVE3.txt:9`` imports ``...protobuff.memory.MemoryCommunicationProtocol``).
Both submodules name the protocols of this package; there is no separate protobuf layer: the
in-process memory protocol passes messages as objects, the gRPC one serialises with the
``grpc/proto`` messages."""
