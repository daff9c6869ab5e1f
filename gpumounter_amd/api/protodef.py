"""Tiny DSL that turns message/enum/service declarations into runtime protobuf classes.

There is no ``protoc`` / ``grpc_tools`` in this environment, so wire-compatible
message classes are built from ``descriptor_pb2.FileDescriptorProto`` at import time. The
resulting classes are ordinary generated-style protobuf messages (same wire format as protoc
output, JSON via ``json_format``).
"""
from __future__ import annotations

import base64
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

F = descriptor_pb2.FieldDescriptorProto

_TYPES = {
    "string": F.TYPE_STRING, "int32": F.TYPE_INT32, "int64": F.TYPE_INT64,
    "uint32": F.TYPE_UINT32, "uint64": F.TYPE_UINT64, "bool": F.TYPE_BOOL,
    "double": F.TYPE_DOUBLE, "float": F.TYPE_FLOAT, "bytes": F.TYPE_BYTES,
}

# field spec: (name, number, type, label) where type is a scalar name, "msg:.pkg.Name",
# "enum:.pkg.Name.Enum" or "map:<scalar key>,<scalar value>"; label "opt" | "rep"
FieldSpec = Tuple[str, int, str, str]


class ProtoFile:
    def __init__(self, name: str, package: str, pool: Optional[descriptor_pool.DescriptorPool] = None):
        self.fdp = descriptor_pb2.FileDescriptorProto(name=name, package=package, syntax="proto3")
        self.package = package
        self.pool = pool or descriptor_pool.Default()
        self._built = False

    def message(self, name: str, fields: Sequence[FieldSpec] = (),
                enums: Dict[str, Iterable[Tuple[str, int]]] = None) -> "ProtoFile":
        m = self.fdp.message_type.add(name=name)
        for ename, values in (enums or {}).items():
            e = m.enum_type.add(name=ename)
            for vname, num in values:
                e.value.add(name=vname, number=num)
        for fname, num, ftype, label in fields:
            f = m.field.add(name=fname, number=num, json_name=_json_name(fname))
            f.label = F.LABEL_REPEATED if label == "rep" else F.LABEL_OPTIONAL
            if ftype.startswith("map:"):
                # proto3 map<K, V> = repeated nested <Field>Entry{key=1, value=2} (map_entry)
                kt, vt = ftype[4:].split(",")
                entry = "".join(p[:1].upper() + p[1:] for p in fname.split("_")) + "Entry"
                e = m.nested_type.add(name=entry)
                e.options.map_entry = True
                for en, ev, et in (("key", 1, kt), ("value", 2, vt)):
                    ef = e.field.add(name=en, number=ev, json_name=en, type=_TYPES[et.strip()])
                    ef.label = F.LABEL_OPTIONAL
                f.label = F.LABEL_REPEATED
                f.type = F.TYPE_MESSAGE
                f.type_name = f".{self.package}.{name}.{entry}"
            elif ftype.startswith("msg:"):
                f.type = F.TYPE_MESSAGE
                f.type_name = ftype[4:]
            elif ftype.startswith("enum:"):
                f.type = F.TYPE_ENUM
                f.type_name = ftype[5:]
            else:
                f.type = _TYPES[ftype]
        return self

    def service(self, name: str, methods: Sequence[Tuple[str, str, str]]) -> "ProtoFile":
        s = self.fdp.service.add(name=name)
        for mname, req, resp in methods:
            s.method.add(name=mname, input_type=f".{self.package}.{req}",
                         output_type=f".{self.package}.{resp}")
        return self

    def build(self) -> Dict[str, type]:
        try:
            fd = self.pool.FindFileByName(self.fdp.name)
        except KeyError:
            fd = self.pool.Add(self.fdp) if hasattr(self.pool, "Add") else None
            fd = self.pool.FindFileByName(self.fdp.name)
        classes = {}
        for mname in fd.message_types_by_name:
            classes[mname] = message_factory.GetMessageClass(fd.message_types_by_name[mname])
        self._built = True
        return classes


def _json_name(name: str) -> str:
    parts = name.split("_")
    return parts[0] + "".join(p[:1].upper() + p[1:] for p in parts[1:])


def method_path(package: str, service: str, method: str) -> str:
    return f"/{package}.{service}/{method}"


def fields_of(cls) -> List[Tuple[str, int]]:
    return [(f.name, f.number) for f in cls.DESCRIPTOR.fields]


# ------------------------------------------------------------------------------ fast to_dict
_FD = None
_CONV: Dict[object, list] = {}


def _converters(desc) -> list:
    """Per message type: (name, getter-kind, extra) for every field, computed once."""
    global _FD
    if _FD is None:
        from google.protobuf.descriptor import FieldDescriptor as _F
        _FD = _F
    conv = _CONV.get(desc)
    if conv is not None:
        return conv
    conv = []
    for f in desc.fields:
        rep = f.is_repeated if hasattr(f, "is_repeated") else f.label == _FD.LABEL_REPEATED
        if f.type == _FD.TYPE_MESSAGE:
            if f.message_type.GetOptions().map_entry:
                kind = "map"
            else:
                kind = "msg"
            extra = f.message_type
        elif f.type == _FD.TYPE_ENUM:
            kind, extra = "enum", {v.number: v.name for v in f.enum_type.values}
        elif f.type in (_FD.TYPE_INT64, _FD.TYPE_UINT64, _FD.TYPE_SINT64, _FD.TYPE_FIXED64,
                        _FD.TYPE_SFIXED64):
            kind, extra = "int64", None          # proto3 JSON: 64-bit integers as strings
        elif f.type == _FD.TYPE_BYTES:
            kind, extra = "bytes", None
        else:
            kind, extra = "plain", None
        conv.append((f.name, kind, extra, rep))
    _CONV[desc] = conv
    return conv


def to_dict(msg) -> dict:
    """``json_format.MessageToDict(msg, preserving_proto_field_name=True,
    always_print_fields_with_no_presence=True)`` for the proto3 messages of this package, without
    the generic reflection walk (several times faster on the master's reply path)."""
    out = {}
    for name, kind, extra, rep in _converters(msg.DESCRIPTOR):
        v = getattr(msg, name)
        if kind == "msg":
            out[name] = [to_dict(x) for x in v] if rep else to_dict(v)
        elif kind == "map":
            out[name] = {str(k): (to_dict(x) if hasattr(x, "DESCRIPTOR") else x)
                         for k, x in v.items()}
        elif kind == "enum":
            out[name] = [extra.get(x, x) for x in v] if rep else extra.get(v, v)
        elif kind == "int64":
            out[name] = [str(x) for x in v] if rep else str(v)
        elif kind == "bytes":
            out[name] = [base64.b64encode(x).decode() for x in v] if rep else \
                base64.b64encode(v).decode()
        else:
            out[name] = list(v) if rep else v
    return out
