#!/usr/bin/env python3
"""Static verification tier (the reference's `hack/verify-*.sh`, SURVEY §4 "Static verify").

    python hack/verify.py            # run every check, exit 1 on any failure
    python hack/verify.py --update   # regenerate generated files (hack/update-*.sh)
    python hack/verify.py -c imports -c docs

Checks (reference script in brackets):
  compile     every Python module byte-compiles                        [verify-govet]
  boilerplate every Python module has a docstring, every native source a header comment
                                                                       [verify-boilerplate]
  whitespace  no tabs / trailing whitespace in Python                  [verify-gofmt]
  imports     layering rules between packages                          [verify-import-boss]
  flags       component flags are --dashed, unique, never --under_score [verify-flags-underscore, clicheck]
  docs        docs/cli matches the generated CLI reference             [verify-generated-docs]
  protos      api/generated/*.proto match the runtime wire schemas     [verify-generated-device-plugin,
                                                                        verify-generated-protobuf]
  links       relative links in Markdown resolve                       [linkcheck]
"""
from __future__ import annotations

import argparse
import ast
import json
import os
import py_compile
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kubernetes_amd")
sys.path.insert(0, ROOT)

# import-boss: package -> packages it must NOT import (lower layers never reach up)
LAYERS = {
    "api": ("apiserver", "client", "scheduler", "kubelet", "controllers", "kubectl", "proxy", "cri", "deviceplugin",
            "kubeadm", "addons", "monitoring", "kubemark", "e2e", "cmd"),
    "storage": ("apiserver", "client", "scheduler", "kubelet", "controllers", "kubectl", "cmd"),
    "client": ("apiserver", "scheduler", "kubelet", "controllers", "kubectl", "cmd", "kubemark", "e2e"),
    "scheduler": ("kubelet", "controllers", "kubectl", "cmd", "kubemark", "e2e", "proxy"),
    "controllers": ("kubelet", "scheduler", "kubectl", "cmd", "kubemark", "e2e"),
    "deviceplugin": ("apiserver", "scheduler", "controllers", "kubectl", "cmd", "kubemark"),
    "kubelet": ("apiserver", "scheduler", "controllers", "kubectl", "cmd", "kubemark", "e2e"),
    "proxy": ("apiserver", "scheduler", "kubelet", "controllers", "kubectl", "cmd"),
    "native": ("apiserver", "scheduler", "kubelet", "controllers", "kubectl", "cmd", "client"),
    "utils": ("apiserver", "scheduler", "kubelet", "controllers", "kubectl", "cmd", "client"),
}
# the reference's own exceptions, kept explicit (importer -> allowed module prefixes)
ALLOWED = {
    "kubelet": ("kubernetes_amd.apiserver.registry",),   # qos.GetPodQOS lives with the pod strategy
    # pkg/controller/daemon runs the scheduler's predicates to decide where daemons fit
    "controllers": ("kubernetes_amd.scheduler.cache", "kubernetes_amd.scheduler.predicates", "kubernetes_amd.scheduler"),
    # plugin/pkg/scheduler/volumebinder uses the PV controller's claim/volume matching
    "scheduler": ("kubernetes_amd.controllers.volume",),
}

PROTO_MODULES = [  # (module, attribute with message classes, method tables, output name)
    ("kubernetes_amd.deviceplugin.api", "DP", {"DevicePlugin": "DP_METHODS"}, "deviceplugin_v1alpha.proto"),
    ("kubernetes_amd.deviceplugin.api", "PR", {"Identity": "ID_METHODS"}, "pluginregistration_v1beta.proto"),
    ("kubernetes_amd.cri.api", "MSG", {"RuntimeService": "RUNTIME_METHODS", "ImageService": "IMAGE_METHODS"},
     "cri_runtime_v1alpha1.proto"),
    ("kubernetes_amd.csi.api", "MSG", {"Identity": "IDENTITY_METHODS", "Controller": "CONTROLLER_METHODS",
                                       "Node": "NODE_METHODS"}, "csi_v0.proto"),
]


def py_files(base=PKG):
    for d, _, fs in os.walk(base):
        if "__pycache__" in d:
            continue
        for f in sorted(fs):
            if f.endswith(".py"):
                yield os.path.join(d, f)


def rel(p):
    return os.path.relpath(p, ROOT)


# -- checks ------------------------------------------------------------------
def check_compile():
    errs = []
    for p in list(py_files()) + list(py_files(os.path.join(ROOT, "tests"))) + [os.path.join(ROOT, "bench.py")]:
        try:
            py_compile.compile(p, cfile=os.path.join(tempfile.gettempdir(), "kamd_verify.pyc"), doraise=True)
        except py_compile.PyCompileError as e:
            errs.append(f"{rel(p)}: {e.msg}")
    return errs


def check_boilerplate():
    errs = []
    for p in py_files():
        with open(p) as f:
            src = f.read()
        if not src.strip():
            continue                      # empty package markers
        if ast.get_docstring(ast.parse(src)) is None:
            errs.append(f"{rel(p)}: module has no docstring")
    for d, _, fs in os.walk(os.path.join(ROOT, "native")):
        for f in fs:
            if f.endswith((".cc", ".h", ".hip")):
                with open(os.path.join(d, f)) as fh:
                    first = fh.readline()
                if not first.startswith("//"):
                    errs.append(f"{rel(os.path.join(d, f))}: no header comment")
    return errs


def check_whitespace():
    errs = []
    for p in list(py_files()) + list(py_files(os.path.join(ROOT, "tests"))):
        with open(p) as f:
            for i, line in enumerate(f, 1):
                if "\t" in line:
                    errs.append(f"{rel(p)}:{i}: tab")
                if line.rstrip("\n") != line.rstrip("\n").rstrip():
                    errs.append(f"{rel(p)}:{i}: trailing whitespace")
    return errs


def _imports(path):
    tree = ast.parse(open(path).read())
    mod_parts = rel(path)[:-3].split(os.sep)
    for node in ast.walk(tree):
        if isinstance(node, ast.Import):
            for a in node.names:
                yield a.name
        elif isinstance(node, ast.ImportFrom):
            if node.level:
                base = mod_parts[:len(mod_parts) - node.level]
                name = ".".join(base + ([node.module] if node.module else []))
            else:
                name = node.module or ""
            yield name
            for a in node.names:            # `from .. import client` imports a package too
                yield f"{name}.{a.name}"


def check_imports():
    errs = []
    for p in py_files():
        parts = rel(p).split(os.sep)
        if len(parts) < 3:
            continue
        pkg = parts[1]
        banned = LAYERS.get(pkg)
        if not banned:
            continue
        for name in _imports(p):
            segs = name.split(".")
            if len(segs) >= 2 and segs[0] == "kubernetes_amd" and segs[1] in banned:
                if any(name.startswith(a) for a in ALLOWED.get(pkg, ())):
                    continue
                errs.append(f"{rel(p)}: {pkg} must not import {name}")
    return sorted(set(errs))


def check_flags():
    errs = []
    from kubernetes_amd.cmd import gendocs
    for comp, parser in gendocs.parsers().items():
        seen = set()
        for act in parser._actions:
            for opt in act.option_strings:
                if opt.startswith("--") and "_" in opt:
                    errs.append(f"{comp}: flag {opt} uses underscores")
                if opt in seen:
                    errs.append(f"{comp}: duplicate flag {opt}")
                seen.add(opt)
    return errs


def check_docs(update=False):
    out = os.path.join(ROOT, "docs", "cli")
    if update:
        subprocess.run([sys.executable, "-m", "kubernetes_amd.cmd.gendocs", "--format", "md", "--out", out],
                       cwd=ROOT, check=True, capture_output=True)
        return []
    with tempfile.TemporaryDirectory() as tmp:
        subprocess.run([sys.executable, "-m", "kubernetes_amd.cmd.gendocs", "--format", "md", "--out", tmp],
                       cwd=ROOT, check=True, capture_output=True)
        errs = []
        for f in sorted(os.listdir(tmp)):
            have = os.path.join(out, f)
            if not os.path.exists(have) or open(have).read() != open(os.path.join(tmp, f)).read():
                errs.append(f"docs/cli/{f} is stale (run hack/verify.py --update)")
        return errs


_TYPE = {1: "double", 3: "int64", 4: "uint64", 5: "int32", 8: "bool", 9: "string", 12: "bytes", 13: "uint32"}


def render_proto(modname, attr, services):
    """The wire schema of a runtime-built protobuf package as .proto text."""
    import importlib
    m = importlib.import_module(modname)
    classes = getattr(m, attr)
    fd = next(iter(classes.values())).DESCRIPTOR.file
    lines = ["// Code generated by hack/verify.py --update from the runtime schema. DO NOT EDIT.",
             f"// source: {modname}.{attr}", 'syntax = "proto3";', "", f"package {fd.package};", ""]
    for mt in fd.message_types_by_name.values():
        lines.append(f"message {mt.name} {{")
        for f in mt.fields:
            if f.message_type is not None and f.message_type.GetOptions().map_entry:
                v = f.message_type.fields_by_name["value"]
                vt = v.message_type.name if v.message_type is not None else _TYPE[v.type]
                lines.append(f"  map<string, {vt}> {f.name} = {f.number};")
                continue
            t = f.message_type.name if f.message_type is not None else _TYPE[f.type]
            repeated = f.is_repeated if hasattr(f, "is_repeated") else f.label == f.LABEL_REPEATED
            rep = "repeated " if repeated else ""
            lines.append(f"  {rep}{t} {f.name} = {f.number};")
        lines.append("}")
        lines.append("")
    for svc, table in services.items():
        lines.append(f"service {svc} {{")
        for meth, (req, resp, stream) in getattr(m, table).items():
            out = f"stream {resp.DESCRIPTOR.name}" if stream else resp.DESCRIPTOR.name
            lines.append(f"  rpc {meth}({req.DESCRIPTOR.name}) returns ({out}) {{}}")
        lines.append("}")
        lines.append("")
    return "\n".join(lines)


def check_protos(update=False):
    out = os.path.join(ROOT, "kubernetes_amd", "api", "generated")
    os.makedirs(out, exist_ok=True)
    errs = []
    for modname, attr, services, name in PROTO_MODULES:
        text = render_proto(modname, attr, services)
        path = os.path.join(out, name)
        if update:
            with open(path, "w") as f:
                f.write(text)
        elif not os.path.exists(path) or open(path).read() != text:
            errs.append(f"{rel(path)} is stale (run hack/verify.py --update)")
    # the protobuf storage schema table, regenerated from the reference generated.proto files
    # when that tree is present (hack/gen_proto_schema.py)
    ref = os.environ.get("KAMD_REFERENCE", "/root/reference")
    if os.path.isdir(os.path.join(ref, "staging", "src", "k8s.io")):
        sys.path.insert(0, os.path.join(ROOT, "hack"))
        import gen_proto_schema
        text = json.dumps(gen_proto_schema.generate(ref), separators=(",", ":")) + "\n"
        path = gen_proto_schema.DEFAULT_OUT
        if update:
            with open(path, "w") as f:
                f.write(text)
        elif not os.path.exists(path) or open(path).read() != text:
            errs.append(f"{rel(path)} is stale (run hack/verify.py --update)")
    return errs


_LINK = re.compile(r"\]\(([^)#\s]+)(#[^)]*)?\)")


def check_links():
    errs = []
    for d, dirs, fs in os.walk(ROOT):
        dirs[:] = [x for x in dirs if not x.startswith(".") and x not in ("gpurun_out", "__pycache__", "node_modules")]
        for f in fs:
            if not f.endswith(".md") or f in ("PAPERS.md", "SNIPPETS.md"):
                continue
            p = os.path.join(d, f)
            for target, _ in _LINK.findall(open(p, errors="replace").read()):
                if re.match(r"^[a-z]+://", target) or target.startswith("mailto:"):
                    continue
                if not os.path.exists(os.path.normpath(os.path.join(d, target))):
                    errs.append(f"{rel(p)}: broken link {target}")
    return errs


CHECKS = {"compile": check_compile, "boilerplate": check_boilerplate, "whitespace": check_whitespace,
          "imports": check_imports, "flags": check_flags, "docs": check_docs, "protos": check_protos,
          "links": check_links}


def main(argv=None):
    ap = argparse.ArgumentParser("verify")
    ap.add_argument("-c", "--check", action="append", choices=sorted(CHECKS))
    ap.add_argument("--update", action="store_true", help="regenerate docs/cli and api/generated/*.proto")
    a = ap.parse_args(argv)
    if a.update:
        check_docs(update=True)
        check_protos(update=True)
        print("updated generated files")
        return 0
    failed = 0
    for name in a.check or CHECKS:
        errs = CHECKS[name]()
        print(f"{'FAIL' if errs else 'ok  '} {name}" + (f" ({len(errs)})" if errs else ""))
        for e in errs[:50]:
            print(f"     {e}")
        failed += bool(errs)
    return 1 if failed else 0


if __name__ == "__main__":
    sys.exit(main())
