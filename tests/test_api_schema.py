"""gpu_mount.proto (the canonical text) == the runtime descriptors (gpumounter_amd/api/gpu_mount.py),
and fields 1-4 / result enums stay wire-identical to the reference's pkg/api/gpu-mount/api.proto.

There is no protoc here, so both .proto files are read with a small parser of the
proto3 subset they use: messages, nested enums, scalar/message/enum fields, ``repeated``,
services with unary rpcs.
"""
import os
import re

import pytest

from gpumounter_amd.api import gpu_mount as api
from gpumounter_amd.api.protodef import F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OURS = os.path.join(ROOT, "gpumounter_amd", "api", "gpu_mount.proto")
REF = "/root/reference/pkg/api/gpu-mount/api.proto"

_SCALAR = {F.TYPE_STRING: "string", F.TYPE_INT32: "int32", F.TYPE_INT64: "int64",
           F.TYPE_UINT32: "uint32", F.TYPE_UINT64: "uint64", F.TYPE_BOOL: "bool",
           F.TYPE_DOUBLE: "double", F.TYPE_FLOAT: "float", F.TYPE_BYTES: "bytes"}


def parse_proto(text: str):
    """→ (package, {msg: {"fields": {name: (num, type, repeated)}, "enums": {E: {V: n}}}},
    {service: {rpc: (req, resp)}})"""
    text = re.sub(r"//[^\n]*", "", text)
    pkg = re.search(r"\bpackage\s+([\w.]+)\s*;", text).group(1)
    tokens = re.findall(r"[A-Za-z_][\w.]*|\d+|[{}();=]", text)
    msgs, svcs = {}, {}
    i = 0

    def block(i):
        """index just past the matching '}' of the '{' at tokens[i]."""
        depth = 0
        while True:
            if tokens[i] == "{":
                depth += 1
            elif tokens[i] == "}":
                depth -= 1
                if depth == 0:
                    return i + 1
            i += 1

    while i < len(tokens):
        t = tokens[i]
        if t == "message":
            name, start = tokens[i + 1], i + 2
            end = block(start)
            body = tokens[start + 1:end - 1]
            m = {"fields": {}, "enums": {}}
            j = 0
            while j < len(body):
                if body[j] == "enum":
                    ename = body[j + 1]
                    k = j + 3
                    vals = {}
                    while body[k] != "}":
                        vals[body[k]] = int(body[k + 2])
                        k += 4
                    m["enums"][ename] = vals
                    j = k + 1
                    continue
                rep = body[j] == "repeated"
                if rep:
                    j += 1
                ftype, fname, num = body[j], body[j + 1], int(body[j + 3])
                m["fields"][fname] = (num, ftype, rep)
                j += 5
            msgs[name] = m
            i = end
        elif t == "service":
            name, start = tokens[i + 1], i + 2
            end = block(start)
            body = tokens[start + 1:end - 1]
            rpcs = {}
            for k, tok in enumerate(body):
                if tok == "rpc":
                    rpcs[body[k + 1]] = (body[k + 3], body[k + 7])
            svcs[name] = rpcs
            i = end
        else:
            i += 1
    return pkg, msgs, svcs


def runtime_schema():
    fdp = api._pf.fdp
    msgs, svcs = {}, {}
    for m in fdp.message_type:
        fields = {}
        for f in m.field:
            if f.type in _SCALAR:
                t = _SCALAR[f.type]
            else:
                t = f.type_name.rsplit(".", 1)[-1]
            fields[f.name] = (f.number, t, f.label == F.LABEL_REPEATED)
        msgs[m.name] = {"fields": fields,
                        "enums": {e.name: {v.name: v.number for v in e.value}
                                  for e in m.enum_type}}
    for s in fdp.service:
        svcs[s.name] = {m.name: (m.input_type.rsplit(".", 1)[-1],
                                 m.output_type.rsplit(".", 1)[-1]) for m in s.method}
    return fdp.package, msgs, svcs


def test_proto_text_equals_runtime_descriptors():
    with open(OURS) as fh:
        text_schema = parse_proto(fh.read())
    assert text_schema == runtime_schema()


def test_wire_compatible_with_the_reference_proto():
    if not os.path.exists(REF):
        pytest.skip("reference checkout not present (parity pinned where it is)")
    with open(REF) as fh:
        rpkg, rmsgs, rsvcs = parse_proto(fh.read())
    pkg, msgs, svcs = runtime_schema()
    assert pkg == rpkg
    for name, m in rmsgs.items():
        for fname, spec in m["fields"].items():
            assert msgs[name]["fields"][fname] == spec, (name, fname)
        assert msgs[name]["enums"] == m["enums"], name
    for name, rpcs in rsvcs.items():
        assert svcs[name] == rpcs
