"""OpenAPI v2 (`/openapi/v2`, `/swagger.json`) generated from the served resource table.

Parity: `staging/src/k8s.io/apiserver/pkg/server/routes/openapi.go` + `kube-openapi`'s builder
(`pkg/builder/openapi.go`): one path entry per collection / item / watch / status route
with the operation ids the reference emits (`listCoreV1NamespacedPod`, `createCoreV1NamespacedPod`,
`readCoreV1NamespacedPod`, `replace…`, `patch…`, `delete…`, `deleteCollection…`, `watch…`),
and a definition per kind named `io.k8s.api.<group>.<version>.<Kind>` carrying
`x-kubernetes-group-version-kind`. CRD resources appear with their openAPIV3Schema when set.
The document is rebuilt only when the resource table changes.
"""
from __future__ import annotations

import json

from ..api import meta as m

_GROUP_PKG = {"": "core", "apps": "apps", "batch": "batch", "extensions": "extensions", "policy": "policy",
              "rbac.authorization.k8s.io": "rbac", "storage.k8s.io": "storage", "autoscaling": "autoscaling",
              "networking.k8s.io": "networking", "scheduling.k8s.io": "scheduling", "settings.k8s.io": "settings",
              "certificates.k8s.io": "certificates", "admissionregistration.k8s.io": "admissionregistration",
              "authentication.k8s.io": "authentication", "authorization.k8s.io": "authorization",
              "events.k8s.io": "events", "apiextensions.k8s.io": "apiextensions", "apiregistration.k8s.io": "apiregistration",
              "metrics.k8s.io": "metrics"}

_OBJECT_META = {"$ref": "#/definitions/io.k8s.apimachinery.pkg.apis.meta.v1.ObjectMeta"}
_LIST_META = {"$ref": "#/definitions/io.k8s.apimachinery.pkg.apis.meta.v1.ListMeta"}

_META_DEFS = {
    "io.k8s.apimachinery.pkg.apis.meta.v1.ObjectMeta": {
        "type": "object", "properties": {k: {"type": t} for k, t in (
            ("name", "string"), ("generateName", "string"), ("namespace", "string"), ("uid", "string"),
            ("resourceVersion", "string"), ("generation", "integer"), ("creationTimestamp", "string"),
            ("deletionTimestamp", "string"), ("labels", "object"), ("annotations", "object"),
            ("ownerReferences", "array"), ("finalizers", "array"), ("initializers", "object"))}},
    "io.k8s.apimachinery.pkg.apis.meta.v1.ListMeta": {
        "type": "object", "properties": {"resourceVersion": {"type": "string"}, "continue": {"type": "string"},
                                         "selfLink": {"type": "string"}}},
    "io.k8s.apimachinery.pkg.apis.meta.v1.Status": {
        "type": "object", "properties": {"status": {"type": "string"}, "message": {"type": "string"},
                                         "reason": {"type": "string"}, "code": {"type": "integer"}}},
    "io.k8s.apimachinery.pkg.apis.meta.v1.WatchEvent": {
        "type": "object", "required": ["type", "object"],
        "properties": {"type": {"type": "string"}, "object": {"type": "object"}}},
    "io.k8s.apimachinery.pkg.apis.meta.v1.Patch": {"type": "object"},
    "io.k8s.apimachinery.pkg.apis.meta.v1.DeleteOptions": {
        "type": "object", "properties": {"gracePeriodSeconds": {"type": "integer"},
                                         "propagationPolicy": {"type": "string"}, "preconditions": {"type": "object"}}},
}


def def_name(ri):
    if ri.group in _GROUP_PKG:
        return f"io.k8s.api.{_GROUP_PKG[ri.group]}.{ri.version}.{ri.kind}"
    rev = ".".join(reversed(ri.group.split(".")))
    return f"{rev}.{ri.version}.{ri.kind}"


def _camel_gv(ri):
    g = _GROUP_PKG.get(ri.group) or ri.group.split(".")[0]
    return g[:1].upper() + g[1:] + ri.version[:1].upper() + ri.version[1:]


def _op(op_id, ri, kind_ref, action, params=(), body=False, ok_ref=None):
    o = {"operationId": op_id, "tags": [f"{_GROUP_PKG.get(ri.group, ri.group)}_{ri.version}"],
         "consumes": ["*/*"], "produces": ["application/json", "application/yaml", "application/vnd.kubernetes.protobuf"],
         "schemes": ["https"], "parameters": list(params),
         "responses": {"200": {"description": "OK", "schema": ok_ref or kind_ref}, "401": {"description": "Unauthorized"}},
         "x-kubernetes-action": action,
         "x-kubernetes-group-version-kind": {"group": ri.group, "version": ri.version, "kind": ri.kind}}
    if body:
        o["parameters"].insert(0, {"name": "body", "in": "body", "required": True, "schema": kind_ref})
    return o


_NAME = {"name": "name", "in": "path", "required": True, "type": "string", "uniqueItems": True}
_NS = {"name": "namespace", "in": "path", "required": True, "type": "string", "uniqueItems": True}
_LIST_Q = [{"name": n, "in": "query", "type": t, "uniqueItems": True} for n, t in (
    ("labelSelector", "string"), ("fieldSelector", "string"), ("limit", "integer"), ("continue", "string"),
    ("resourceVersion", "string"), ("timeoutSeconds", "integer"), ("watch", "boolean"))]


def build(schemas=None, version="v1.9.0"):
    """`schemas`: {(group, version, kind): openAPIV3Schema} for CRDs."""
    schemas = schemas or {}
    paths, defs = {}, dict(_META_DEFS)
    for ri in m.RESOURCES:
        if ri.plural in getattr(m, "VIRTUAL", ()):
            continue
        dn = def_name(ri)
        ref = {"$ref": f"#/definitions/{dn}"}
        lref = {"$ref": f"#/definitions/{dn}List"}
        props = {"apiVersion": {"type": "string"}, "kind": {"type": "string"}, "metadata": _OBJECT_META}
        custom = schemas.get((ri.group, ri.version, ri.kind))
        if custom:
            props.update({k: v for k, v in (custom.get("properties") or {}).items() if k not in props})
        else:
            props.update({"spec": {"type": "object"}, "status": {"type": "object"}})
        defs[dn] = {"type": "object", "properties": props,
                    "x-kubernetes-group-version-kind": [{"group": ri.group, "version": ri.version, "kind": ri.kind}]}
        defs[dn + "List"] = {"type": "object", "required": ["items"],
                             "properties": {"apiVersion": {"type": "string"}, "kind": {"type": "string"},
                                            "metadata": _LIST_META, "items": {"type": "array", "items": ref}},
                             "x-kubernetes-group-version-kind": [{"group": ri.group, "version": ri.version,
                                                                  "kind": ri.kind + "List"}]}
        base = "/api/v1" if not ri.group else f"/apis/{ri.group}/{ri.version}"
        gv = _camel_gv(ri)
        nsd = "Namespaced" if ri.namespaced else ""
        coll = f"{base}/namespaces/{{namespace}}/{ri.plural}" if ri.namespaced else f"{base}/{ri.plural}"
        item = coll + "/{name}"
        pp = [_NS] if ri.namespaced else []
        paths[coll] = {
            "get": _op(f"list{gv}{nsd}{ri.kind}", ri, ref, "list", _LIST_Q, ok_ref=lref),
            "post": _op(f"create{gv}{nsd}{ri.kind}", ri, ref, "post", (), body=True),
            "delete": _op(f"deletecollection{gv}{nsd}{ri.kind}", ri, ref, "deletecollection", _LIST_Q,
                          ok_ref={"$ref": "#/definitions/io.k8s.apimachinery.pkg.apis.meta.v1.Status"}),
            "parameters": pp}
        paths[item] = {
            "get": _op(f"read{gv}{nsd}{ri.kind}", ri, ref, "get"),
            "put": _op(f"replace{gv}{nsd}{ri.kind}", ri, ref, "put", (), body=True),
            "patch": dict(_op(f"patch{gv}{nsd}{ri.kind}", ri, ref, "patch", ({"name": "body", "in": "body", "required": True,
                                                                             "schema": {"$ref": "#/definitions/io.k8s.apimachinery.pkg.apis.meta.v1.Patch"}},)),
                          consumes=["application/json-patch+json", "application/merge-patch+json",
                                    "application/strategic-merge-patch+json"]),
            "delete": _op(f"delete{gv}{nsd}{ri.kind}", ri, ref, "delete",
                          ({"name": "body", "in": "body", "schema": {"$ref": "#/definitions/io.k8s.apimachinery.pkg.apis.meta.v1.DeleteOptions"}},),
                          ok_ref={"$ref": "#/definitions/io.k8s.apimachinery.pkg.apis.meta.v1.Status"}),
            "parameters": [_NAME] + pp}
        paths[item + "/status"] = {"get": _op(f"read{gv}{nsd}{ri.kind}Status", ri, ref, "get"),
                                   "put": _op(f"replace{gv}{nsd}{ri.kind}Status", ri, ref, "put", (), body=True),
                                   "parameters": [_NAME] + pp}
        wcoll = (f"{base}/watch/namespaces/{{namespace}}/{ri.plural}" if ri.namespaced else f"{base}/watch/{ri.plural}")
        paths[wcoll] = {"get": _op(f"watch{gv}{nsd}{ri.kind}List", ri, ref, "watchlist", _LIST_Q,
                                   ok_ref={"$ref": "#/definitions/io.k8s.apimachinery.pkg.apis.meta.v1.WatchEvent"}),
                        "parameters": pp}
        if ri.namespaced:
            allp = f"{base}/{ri.plural}"
            paths[allp] = {"get": _op(f"list{gv}{ri.kind}ForAllNamespaces", ri, ref, "list", _LIST_Q, ok_ref=lref)}
    return {"swagger": "2.0", "info": {"title": "Kubernetes (MI355X)", "version": version},
            "paths": dict(sorted(paths.items())), "definitions": dict(sorted(defs.items())),
            "securityDefinitions": {"BearerToken": {"type": "apiKey", "name": "authorization", "in": "header"}},
            "security": [{"BearerToken": []}]}


class OpenAPICache:
    def __init__(self, version="v1.9.0"):
        self.version = version
        self._key = None
        self._body = None

    def get(self, schemas=None):
        key = (len(m.RESOURCES), tuple(r.plural for r in m.RESOURCES[-8:]), json.dumps(sorted(("/".join(k), v) for k, v in (schemas or {}).items()), sort_keys=True))
        if key != self._key:
            self._body = json.dumps(build(schemas, self.version), separators=(",", ":")).encode()
            self._key = key
        return self._body
