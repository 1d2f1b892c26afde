"""Build protobuf message classes at runtime from a compact schema (no protoc in this image).

Schema: {MessageName: [(field_name, number, type, label, type_name_or_None), ...]}
  type:  "string" | "bool" | "int64" | "int32" | "uint32" | "bytes" | "double" | "message"
  label: "opt" | "rep" | "map" | "oneof:<group>"   (for "map", type is the VALUE type, key is
         string; fields sharing a oneof group get field presence, so a 0 is still sent)
Produces wire-compatible classes for the given proto package (field numbers are what matter).
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_T = descriptor_pb2.FieldDescriptorProto
TYPES = {"string": _T.TYPE_STRING, "bool": _T.TYPE_BOOL, "int64": _T.TYPE_INT64, "int32": _T.TYPE_INT32,
         "uint32": _T.TYPE_UINT32, "uint64": _T.TYPE_UINT64, "bytes": _T.TYPE_BYTES, "double": _T.TYPE_DOUBLE,
         "sint64": _T.TYPE_SINT64, "message": _T.TYPE_MESSAGE}


def _camel(s):
    return "".join(p[:1].upper() + p[1:] for p in s.split("_"))


def build(package: str, filename: str, schema: dict, syntax="proto3", pool=None):
    fdp = descriptor_pb2.FileDescriptorProto(name=filename, package=package, syntax=syntax)
    for mname, fields in schema.items():
        mp = fdp.message_type.add(name=mname)
        oneofs: dict = {}
        for fname, num, ftype, label, tname in fields:
            f = mp.field.add(name=fname, number=num, json_name=fname)
            if label == "map":
                entry = mp.nested_type.add(name=_camel(fname) + "Entry")
                entry.options.map_entry = True
                k = entry.field.add(name="key", number=1, type=_T.TYPE_STRING, label=_T.LABEL_OPTIONAL, json_name="key")
                v = entry.field.add(name="value", number=2, type=TYPES[ftype], label=_T.LABEL_OPTIONAL, json_name="value")
                if ftype == "message":
                    v.type_name = f".{package}.{tname}"
                del k
                f.type = _T.TYPE_MESSAGE
                f.type_name = f".{package}.{mname}.{entry.name}"
                f.label = _T.LABEL_REPEATED
            else:
                f.type = TYPES[ftype]
                f.label = _T.LABEL_REPEATED if label == "rep" else _T.LABEL_OPTIONAL
                if ftype == "message":
                    f.type_name = f".{package}.{tname}"
                if label.startswith("oneof:"):
                    group = label.split(":", 1)[1]
                    if group not in oneofs:
                        oneofs[group] = len(mp.oneof_decl)
                        mp.oneof_decl.add(name=group)
                    f.oneof_index = oneofs[group]
    pool = pool or descriptor_pool.DescriptorPool()
    fd = pool.Add(fdp)
    fdesc = pool.FindFileByName(filename)
    del fd
    return {name: message_factory.GetMessageClass(fdesc.message_types_by_name[name]) for name in schema}
