#!/usr/bin/env python3
"""Generate the protobuf storage schema table from the reference's generated.proto files.

    python hack/gen_proto_schema.py [--reference /root/reference] [--out kubernetes_amd/api/generated/k8s_proto_schema.json]

The reference's etcd object format is `k8s\\0` + runtime.Unknown{TypeMeta, raw = the v1 protobuf
of the object} (`staging/src/k8s.io/apimachinery/pkg/runtime/serializer/protobuf/protobuf.go:42`),
with the field numbers of `staging/src/k8s.io/api/<group>/<version>/generated.proto` (plus
apimachinery, apiextensions, kube-aggregator and metrics). This script parses those .proto
files and the Go struct tags beside them (`types.go`: `json:"name"` and `json:",inline"` — the
JSON name of a field and whether an embedded struct's fields appear inline in JSON) and emits one
compact JSON table that both the Python codec and the native codec (`native/pbcodec`) load:

    {"messages": {"<fq message>": [[json name, number, label, type, key type, inline], ...]},
     "kinds": {"<group>/<version>/<Kind>": "<fq message>"}}

label: "opt" | "rep" | "map"; type: a scalar ("string", "bytes", "bool", "int32", "int64",
"double") or a fully-qualified message name; key type: the scalar map key type or "".
Comments and everything else of the .proto files are dropped: the table holds field numbers
and names only.
"""
from __future__ import annotations

import argparse
import json
import os
import re

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_OUT = os.path.join(HERE, "kubernetes_amd", "api", "generated", "k8s_proto_schema.json")

SCALARS = {"string", "bytes", "bool", "int32", "int64", "double", "float", "uint32", "uint64", "sint32", "sint64"}

# proto package directory -> API group served for it
GROUPS = {
    "core": "", "apps": "apps", "batch": "batch", "extensions": "extensions", "policy": "policy",
    "autoscaling": "autoscaling", "rbac": "rbac.authorization.k8s.io", "storage": "storage.k8s.io",
    "networking": "networking.k8s.io", "certificates": "certificates.k8s.io", "scheduling": "scheduling.k8s.io",
    "settings": "settings.k8s.io", "admissionregistration": "admissionregistration.k8s.io",
    "authentication": "authentication.k8s.io", "authorization": "authorization.k8s.io",
    "events": "events.k8s.io", "imagepolicy": "imagepolicy.k8s.io", "admission": "admission.k8s.io",
    "apiextensions": "apiextensions.k8s.io", "apiregistration": "apiregistration.k8s.io",
    "metrics": "metrics.k8s.io", "custom_metrics": "custom.metrics.k8s.io",
}

SKIP = ("testapigroup", "/example", "/audit/")

FIELD = re.compile(r"^\s*(optional|repeated|required)?\s*(map<\s*(\w+)\s*,\s*([\w.]+)\s*>|[\w.]+)\s+(\w+)\s*=\s*(\d+)")
MESSAGE = re.compile(r"^\s*message\s+(\w+)\s*\{")
TAG_JSON = re.compile(r'json:"([^"]*)"')
TAG_PB = re.compile(r'protobuf:"[^"]*name=(\w+)')
STRUCT = re.compile(r"^type\s+(\w+)\s+struct\s*\{")


def strip_comments(text):
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return "\n".join(line.split("//", 1)[0] for line in text.splitlines())


def parse_proto(path):
    """-> (package, {message: [(label, type, keytype, name, number)]}) ; nested messages are not
    used by the k8s protos."""
    text = strip_comments(open(path).read())
    pkg = re.search(r"^\s*package\s+([\w.]+)\s*;", text, re.M).group(1)
    msgs, cur, depth = {}, None, 0
    for line in text.splitlines():
        m = MESSAGE.match(line)
        if m and depth == 0:
            cur = m.group(1)
            msgs[cur] = []
            depth = line.count("{") - line.count("}")
            continue
        if cur is not None:
            f = FIELD.match(line)
            if f and depth == 1:
                label = f.group(1) or "optional"
                if f.group(3):
                    msgs[cur].append(("map", f.group(4), f.group(3), f.group(5), int(f.group(6))))
                else:
                    msgs[cur].append(("rep" if label == "repeated" else "opt", f.group(2), "", f.group(5), int(f.group(6))))
            depth += line.count("{") - line.count("}")
            if depth <= 0:
                cur, depth = None, 0
    return pkg, msgs


def parse_go_tags(dirpath):
    """{struct: {proto field name: (json name, inline)}} from the Go types in dirpath."""
    out = {}
    for fn in sorted(os.listdir(dirpath)):
        if not fn.endswith(".go") or fn.endswith("_test.go") or fn.startswith("zz_generated") or fn.endswith(".pb.go"):
            continue
        cur = None
        for line in open(os.path.join(dirpath, fn)):
            m = STRUCT.match(line)
            if m:
                cur = m.group(1)
                out.setdefault(cur, {})
                continue
            if cur is None:
                continue
            if line.startswith("}"):
                cur = None
                continue
            pb = TAG_PB.search(line)
            js = TAG_JSON.search(line)
            if pb and js:
                jname = js.group(1).split(",")[0]
                out[cur][pb.group(1)] = (jname, ",inline" in js.group(1) and not jname)
    return out


def resolve(t, pkg, known):
    if t in SCALARS:
        return t
    if "." in t:
        return t if t.startswith("k8s.io") else f"{pkg}.{t}"
    return f"{pkg}.{t}"


def generate(reference):
    root = os.path.join(reference, "staging", "src", "k8s.io")
    protos = []
    for dp, _dn, files in os.walk(root):
        if "generated.proto" in files and not any(s in dp + "/" for s in SKIP):
            protos.append(dp)
    messages, kinds = {}, {}
    for dp in sorted(protos):
        pkg, msgs = parse_proto(os.path.join(dp, "generated.proto"))
        tags = parse_go_tags(dp)
        version = os.path.basename(dp)
        group_dir = os.path.basename(os.path.dirname(dp))
        for name, fields in msgs.items():
            fq = f"{pkg}.{name}"
            out = []
            for label, typ, key, pname, num in fields:
                jname, inline = tags.get(name, {}).get(pname, (pname, False))
                out.append([jname, num, label, resolve(typ, pkg, messages), key, bool(inline)])
            messages[fq] = out
            # served kinds: top-level objects carry ObjectMeta, lists ListMeta + items
            types = {f[0]: f[3] for f in out}
            meta = types.get("metadata", "")
            if group_dir in GROUPS and (meta.endswith("meta.v1.ObjectMeta") or
                                        (meta.endswith("meta.v1.ListMeta") and "items" in types)):
                g = GROUPS[group_dir]
                kinds[f"{g + '/' if g else ''}{version}/{name}"] = fq
    # metav1.Status is registered unversioned in every group and served as `apiVersion: v1,
    # kind: Status` (apimachinery/pkg/apis/meta/v1/register.go): protobuf ERROR watch frames and
    # error responses carry it in a k8s envelope
    status = "k8s.io.apimachinery.pkg.apis.meta.v1.Status"
    if status in messages:
        kinds["v1/Status"] = status
    return {"messages": dict(sorted(messages.items())), "kinds": dict(sorted(kinds.items()))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--out", default=DEFAULT_OUT)
    a = ap.parse_args()
    schema = generate(a.reference)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(schema, f, separators=(",", ":"), sort_keys=False)
        f.write("\n")
    print(f"{len(schema['messages'])} messages, {len(schema['kinds'])} kinds -> {os.path.relpath(a.out, HERE)}")


if __name__ == "__main__":
    main()
