"""``node.proto`` message classes, built at import time from a descriptor (no protoc step).

Field numbers, names, package (``node``) and the service/method paths
(``/node.NodeServices/{handshake,disconnect,send}``) match the reference
(``p2pfl/communication/protocols/grpc/proto/node.proto:26-60``), so this transport is wire-compatible
with reference p2pfl peers.
"""

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

SERVICE = "node.NodeServices"

_F = descriptor_pb2.FieldDescriptorProto


def _build():
    fd = descriptor_pb2.FileDescriptorProto(name="myfyp_node.proto", package="node", syntax="proto3")

    def msg(name, fields, oneofs=()):
        m = fd.message_type.add(name=name)
        for o in oneofs:
            m.oneof_decl.add(name=o)
        for num, fname, ftype, label, tname, oneof in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = tname
            if oneof is not None:
                f.oneof_index = oneof
        return m

    opt, rep = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED
    msg("Message", [(1, "ttl", _F.TYPE_INT32, opt, None, None), (2, "hash", _F.TYPE_INT64, opt, None, None), (3, "args", _F.TYPE_STRING, rep, None, None)])
    msg(
        "Weights",
        [(1, "weights", _F.TYPE_BYTES, opt, None, None), (2, "contributors", _F.TYPE_STRING, rep, None, None), (3, "num_samples", _F.TYPE_INT32, opt, None, None)],
    )
    # proto3 ``optional int32 round`` = synthetic oneof "_round"
    m = msg(
        "RootMessage",
        [
            (1, "source", _F.TYPE_STRING, opt, None, None),
            (2, "round", _F.TYPE_INT32, opt, None, 1),
            (3, "cmd", _F.TYPE_STRING, opt, None, None),
            (4, "message", _F.TYPE_MESSAGE, opt, ".node.Message", 0),
            (5, "weights", _F.TYPE_MESSAGE, opt, ".node.Weights", 0),
        ],
        oneofs=("payload_type", "_round"),
    )
    m.field[1].proto3_optional = True
    msg("HandShakeRequest", [(1, "addr", _F.TYPE_STRING, opt, None, None)])
    r = msg("ResponseMessage", [(1, "error", _F.TYPE_STRING, opt, None, 0)], oneofs=("_error",))
    r.field[0].proto3_optional = True
    msg("Empty", [])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = lambda n: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"node.{n}"))  # noqa: E731
    return get("Message"), get("Weights"), get("RootMessage"), get("HandShakeRequest"), get("ResponseMessage"), get("Empty")


Message, Weights, RootMessage, HandShakeRequest, ResponseMessage, Empty = _build()
