"""Runtime-built protobuf classes for ``video_streaming.proto`` (no protoc in the image).

A small proto3 parser turns the vendored ``.proto`` into a ``FileDescriptorProto``; message
classes come from the protobuf runtime's message factory, so encoding is the real protobuf wire
format. The reference used protoc-generated stubs (python/proto/video_streaming_pb2.py,
server/proto/video_streaming.pb.go).

    from video_edge_ai_proxy_amd.proto import pb, SERVICE
    vf = pb.VideoFrame(width=640)
"""
from __future__ import annotations

import re
import types
from dataclasses import dataclass
from pathlib import Path

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PROTO_PATH = Path(__file__).with_name("video_streaming.proto")

_SCALARS = {
    "double": descriptor_pb2.FieldDescriptorProto.TYPE_DOUBLE,
    "float": descriptor_pb2.FieldDescriptorProto.TYPE_FLOAT,
    "int64": descriptor_pb2.FieldDescriptorProto.TYPE_INT64,
    "uint64": descriptor_pb2.FieldDescriptorProto.TYPE_UINT64,
    "int32": descriptor_pb2.FieldDescriptorProto.TYPE_INT32,
    "fixed64": descriptor_pb2.FieldDescriptorProto.TYPE_FIXED64,
    "fixed32": descriptor_pb2.FieldDescriptorProto.TYPE_FIXED32,
    "bool": descriptor_pb2.FieldDescriptorProto.TYPE_BOOL,
    "string": descriptor_pb2.FieldDescriptorProto.TYPE_STRING,
    "bytes": descriptor_pb2.FieldDescriptorProto.TYPE_BYTES,
    "uint32": descriptor_pb2.FieldDescriptorProto.TYPE_UINT32,
    "sfixed32": descriptor_pb2.FieldDescriptorProto.TYPE_SFIXED32,
    "sfixed64": descriptor_pb2.FieldDescriptorProto.TYPE_SFIXED64,
    "sint32": descriptor_pb2.FieldDescriptorProto.TYPE_SINT32,
    "sint64": descriptor_pb2.FieldDescriptorProto.TYPE_SINT64,
}

_TOKEN = re.compile(r'"[^"]*"|[A-Za-z_][\w.]*|\d+|[{}()=;<>,\[\]]')


def _tokens(text: str) -> list[str]:
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    return _TOKEN.findall(text)


@dataclass
class Method:
    name: str
    input_type: str
    output_type: str
    client_streaming: bool
    server_streaming: bool


@dataclass
class Service:
    full_name: str
    methods: list

    def path(self, method: str) -> str:
        return f"/{self.full_name}/{method}"


def parse_proto(text: str, name: str = "video_streaming.proto"):
    """Parse a proto3 file (messages, nested messages, repeated scalars/messages, services)."""
    toks = _tokens(text)
    fd = descriptor_pb2.FileDescriptorProto(name=name, syntax="proto3")
    services: list[Service] = []
    pos = 0

    def expect(t):
        nonlocal pos
        if toks[pos] != t:
            raise SyntaxError(f"expected {t!r}, got {toks[pos]!r} (token {pos})")
        pos += 1

    def parse_message(msg: descriptor_pb2.DescriptorProto):
        nonlocal pos
        expect("{")
        while toks[pos] != "}":
            t = toks[pos]
            if t == "message":
                pos += 1
                sub = msg.nested_type.add(name=toks[pos])
                pos += 1
                parse_message(sub)
                continue
            if t in ("enum", "oneof", "map"):
                raise NotImplementedError(f"proto feature {t!r} not supported by the mini parser")
            label = descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL
            if t == "repeated":
                label = descriptor_pb2.FieldDescriptorProto.LABEL_REPEATED
                pos += 1
            ftype, fname = toks[pos], toks[pos + 1]
            pos += 2
            expect("=")
            num = int(toks[pos])
            pos += 1
            expect(";")
            f = msg.field.add(name=fname, number=num, label=label)
            f.json_name = re.sub(r"_([a-z0-9])", lambda m: m.group(1).upper(), fname)
            if ftype in _SCALARS:
                f.type = _SCALARS[ftype]
            else:
                f.type = descriptor_pb2.FieldDescriptorProto.TYPE_MESSAGE
                f.type_name = ftype  # resolved below
        pos += 1

    while pos < len(toks):
        t = toks[pos]
        if t == "syntax":
            pos += 1
            expect("=")
            pos += 1
            expect(";")
        elif t == "package":
            fd.package = toks[pos + 1]
            pos += 2
            expect(";")
        elif t == "message":
            m = fd.message_type.add(name=toks[pos + 1])
            pos += 2
            parse_message(m)
        elif t == "service":
            sname = toks[pos + 1]
            pos += 2
            expect("{")
            sd = fd.service.add(name=sname)
            methods = []
            while toks[pos] != "}":
                expect("rpc")
                mname = toks[pos]
                pos += 1
                expect("(")
                cs = toks[pos] == "stream"
                pos += cs
                itype = toks[pos]
                pos += 1
                expect(")")
                expect("returns")
                expect("(")
                ss = toks[pos] == "stream"
                pos += ss
                otype = toks[pos]
                pos += 1
                expect(")")
                if toks[pos] == "{":
                    expect("{")
                    expect("}")
                if toks[pos] == ";":
                    pos += 1
                sd.method.add(name=mname, input_type=f".{fd.package}.{itype}",
                              output_type=f".{fd.package}.{otype}", client_streaming=cs,
                              server_streaming=ss)
                methods.append(Method(mname, itype, otype, cs, ss))
            pos += 1
            services.append(Service(f"{fd.package}.{sname}", methods))
        else:
            raise SyntaxError(f"unexpected token {t!r}")

    # resolve message type names (innermost scope first, then package scope)
    def resolve(msg, scope):
        for f in msg.field:
            if f.type == descriptor_pb2.FieldDescriptorProto.TYPE_MESSAGE and not f.type_name.startswith("."):
                cands = [f"{scope}.{msg.name}.{f.type_name}", f"{scope}.{f.type_name}",
                         f"{fd.package}.{f.type_name}"]
                f.type_name = "." + next(c for c in cands if c in known)
        for sub in msg.nested_type:
            resolve(sub, f"{scope}.{msg.name}")

    known = set()

    def collect(msg, scope):
        known.add(f"{scope}.{msg.name}")
        for sub in msg.nested_type:
            collect(sub, f"{scope}.{msg.name}")

    for m in fd.message_type:
        collect(m, fd.package)
    for m in fd.message_type:
        resolve(m, fd.package)
    return fd, services


def _build():
    fd, services = parse_proto(PROTO_PATH.read_text())
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    ns = types.SimpleNamespace()

    def add(msg_desc, prefix=""):
        cls = message_factory.GetMessageClass(msg_desc)
        setattr(ns, prefix + msg_desc.name, cls)
        for sub in msg_desc.nested_types:
            add(sub, prefix + msg_desc.name + "_")
        return cls

    for m in fd.message_type:
        add(pool.FindMessageTypeByName(f"{fd.package}.{m.name}"))
    return fd, pool, ns, services


FILE_DESCRIPTOR, POOL, pb, SERVICES = _build()
SERVICE = SERVICES[0]
PACKAGE = FILE_DESCRIPTOR.package

__all__ = ["pb", "SERVICE", "PACKAGE", "parse_proto", "FILE_DESCRIPTOR", "POOL"]
