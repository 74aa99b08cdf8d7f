"""Emit ``node.proto`` (parity: ``grpc/proto/generate_proto.py``).

The reference runs grpcio-tools to turn ``node.proto`` into Python stubs. Here the schema lives in
one descriptor built at import time (:mod:`..proto`), so the direction is reversed: this tool prints
the IDL of that descriptor, for peers written in other languages or for diffing against the
reference schema (``p2pfl/communication/protocols/grpc/proto/node.proto:26-60``).

    python -m myfyp_amd.communication.protocols.grpc.proto.generate_proto > node.proto
"""

from __future__ import annotations

from google.protobuf import descriptor

from myfyp_amd.communication.protocols.grpc import proto

_TYPES = {
    descriptor.FieldDescriptor.TYPE_INT32: "int32",
    descriptor.FieldDescriptor.TYPE_INT64: "int64",
    descriptor.FieldDescriptor.TYPE_STRING: "string",
    descriptor.FieldDescriptor.TYPE_BYTES: "bytes",
}


def _field(f) -> str:
    t = f.message_type.name if f.type == descriptor.FieldDescriptor.TYPE_MESSAGE else _TYPES[f.type]
    repeated = f.is_repeated if hasattr(f, "is_repeated") else f.label == descriptor.FieldDescriptor.LABEL_REPEATED
    label = "repeated " if repeated else ""
    opt = "optional " if f.containing_oneof is not None and f.containing_oneof.name.startswith("_") else ""
    return f"{label}{opt}{t} {f.name} = {f.number};"


def render() -> str:
    out = ['syntax = "proto3";', "", "package node;", ""]
    for cls in (proto.Message, proto.Weights, proto.RootMessage, proto.HandShakeRequest, proto.ResponseMessage, proto.Empty):
        d = cls.DESCRIPTOR
        out.append(f"message {d.name} {{")
        real_oneofs = [o for o in d.oneofs if not o.name.startswith("_")]
        for f in d.fields:
            if f.containing_oneof is None or f.containing_oneof.name.startswith("_"):
                out.append(f"  {_field(f)}")
        for o in real_oneofs:
            out.append(f"  oneof {o.name} {{")
            out.extend(f"    {_field(f)}" for f in o.fields)
            out.append("  }")
        out.append("}")
        out.append("")
    out.append("service NodeServices {")
    out.append("  rpc handshake(HandShakeRequest) returns (ResponseMessage);")
    out.append("  rpc disconnect(HandShakeRequest) returns (Empty);")
    out.append("  rpc send(RootMessage) returns (ResponseMessage);")
    out.append("}")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    print(render(), end="")
