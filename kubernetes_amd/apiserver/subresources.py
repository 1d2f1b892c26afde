"""Workload and proxy subresources of the API server.

* `{deployments,replicasets,statefulsets,replicationcontrollers}/scale` — GET/PUT/PATCH of a
  Scale object whose writes land in the owner's `spec.replicas` (the reference's ScaleREST in
  `pkg/registry/{apps,extensions}/*/storage/storage.go` and `pkg/registry/core/
  replicationcontroller/storage/storage.go`). The Scale's group/version follows the request:
  `autoscaling/v1` (selector as a string) for core and apps/v1, `extensions/v1beta1` /
  `apps/v1beta1` / `apps/v1beta2` (selector map + `targetSelector`) for those groups. The
  Scale's resourceVersion is the owner's, and a PUT carrying one is a precondition on it.
* `deployments/rollback` (extensions/v1beta1, apps/v1beta1) — DeploymentRollback recorded as
  `spec.rollbackTo` plus `updatedAnnotations` for the deployment controller to execute
  (`pkg/registry/extensions/deployment/storage/storage.go` RollbackREST).
* `{pods,services,nodes}/proxy[/path]` with `[scheme:]name[:port]` — HTTP relayed to the pod IP,
  a ready endpoint of the service port, or the node's kubelet (`pkg/registry/core/{pod,service,
  node}/strategy.go` ResourceLocation, `rest.go`); upgrade requests are spliced. The deprecated
  `/api/v1/proxy/namespaces/<ns>/<resource>/<name>/...` form is rewritten to the subresource.
"""
from __future__ import annotations

import random

from ..api import codec
from ..api import meta as m
from ..api.labels import selector_to_string
from ..utils.httpserver import Response
from ..utils.patch import JSONPatchError, apply_patch
from .registry import APIError, bad_request, not_found

SCALABLE = ("deployments", "replicasets", "statefulsets", "replicationcontrollers")
ROLLBACK_VERSIONS = ("extensions/v1beta1", "apps/v1beta1")


def scale_group_version(ri, served_gv: str) -> str:
    gv = served_gv or ri.group_version
    if ri.plural != "replicationcontrollers" and gv in ("extensions/v1beta1", "apps/v1beta1", "apps/v1beta2"):
        return gv
    return "autoscaling/v1"


def to_scale(ri, obj, gv: str) -> dict:
    md, spec, st = obj.get("metadata") or {}, obj.get("spec") or {}, obj.get("status") or {}
    sel = spec.get("selector") or {}
    if ri.plural == "replicationcontrollers":
        sel = {"matchLabels": sel}
    out_md = {k: md[k] for k in ("name", "namespace", "uid", "resourceVersion", "creationTimestamp") if k in md}
    status = {"replicas": int(st.get("replicas") or 0)}
    if gv == "autoscaling/v1":
        status["selector"] = selector_to_string(sel)
    else:
        if sel.get("matchLabels") and not sel.get("matchExpressions"):
            status["selector"] = dict(sel["matchLabels"])
        status["targetSelector"] = selector_to_string(sel)
    return {"kind": "Scale", "apiVersion": gv, "metadata": out_md,
            "spec": {"replicas": int(spec["replicas"]) if spec.get("replicas") is not None else 1}, "status": status}


def _validate_scale(scale) -> None:
    r = (scale.get("spec") or {}).get("replicas", 0)
    if isinstance(r, bool) or not isinstance(r, int) or r < 0:
        raise APIError(422, "Invalid", f"Scale \"{(scale.get('metadata') or {}).get('name', '')}\" is invalid: "
                                       f"spec.replicas: Invalid value: {r!r}: must be greater than or equal to 0")


async def handle_scale(server, req, ri, ns, name, user):
    """GET / PUT / PATCH `<resource>/<name>/scale`."""
    gv = scale_group_version(ri, getattr(req, "served_gv", "") or "")
    verb = {"GET": "get", "HEAD": "get", "PUT": "update", "PATCH": "patch"}.get(req.method)
    if verb is None:
        raise APIError(405, "MethodNotAllowed", f"method {req.method} not allowed on scale")
    server._authorize(user, verb, ns, ri.plural, "scale", name, ri.group, req.path)
    _, cur = await server._aexisting(ri, ns, name)
    if verb == "get":
        return _scale_response(to_scale(ri, cur.obj, gv))
    if verb == "patch":
        try:
            scale = apply_patch(req.headers.get("content-type", "application/merge-patch+json"),
                                to_scale(ri, cur.obj, gv), codec.loads(req.body))
        except (JSONPatchError, ValueError) as e:
            raise APIError(422, "Invalid", f"the patch could not be applied: {e}")
    else:
        scale = codec.loads(req.body)
    if not isinstance(scale, dict):
        raise bad_request("body must be a Scale object")
    smd = scale.get("metadata") or {}
    if smd.get("name") and smd["name"] != name:
        raise bad_request("the name of the object does not match the name on the URL")
    _validate_scale(scale)
    obj = dict(cur.obj)
    obj["metadata"] = dict(obj["metadata"])
    if smd.get("resourceVersion"):
        obj["metadata"]["resourceVersion"] = smd["resourceVersion"]     # precondition on the owner
    obj["spec"] = dict(obj.get("spec") or {}, replicas=int((scale.get("spec") or {}).get("replicas", 0)))
    e = await server.update(ri, ns, name, obj, user)
    return _scale_response(to_scale(ri, e.obj, gv))


def _scale_response(scale):
    return Response(200, codec.dumpb(scale), "application/json")


async def handle_rollback(server, req, ri, ns, name, user):
    """POST `deployments/<name>/rollback` (extensions/v1beta1, apps/v1beta1)."""
    gv = getattr(req, "served_gv", "") or ri.group_version
    if gv not in ROLLBACK_VERSIONS:
        raise APIError(404, "NotFound", f"the server could not find the requested resource (post deployments.{gv} {name}/rollback)")
    server._authorize(user, "create", ns, "deployments", "rollback", name, ri.group, req.path)
    body = codec.loads(req.body) if req.body else {}
    if body.get("name") and body["name"] != name:
        raise bad_request("the name of the DeploymentRollback does not match the name on the URL")
    rev = (body.get("rollbackTo") or {}).get("revision", 0)
    if isinstance(rev, bool) or not isinstance(rev, int) or rev < 0:
        raise APIError(422, "Invalid", f"DeploymentRollback \"{name}\" is invalid: rollbackTo.revision: "
                                       f"Invalid value: {rev!r}: must be greater than or equal to 0")
    _, cur = await server._aexisting(ri, ns, name)
    obj = dict(cur.obj)
    md = obj["metadata"] = dict(obj["metadata"])
    ann = body.get("updatedAnnotations") or {}
    if ann:
        md["annotations"] = dict(md.get("annotations") or {}, **ann)
    obj["spec"] = dict(obj.get("spec") or {}, rollbackTo={"revision": rev})
    await server.update(ri, ns, name, obj, user)
    return Response(200, codec.dumpb({"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Success",
                                      "message": f'rollback request for deployment "{name}" succeeded', "code": 200}),
                    "application/json")


# ------------------------------------------------------------------------------------------------
# proxy
PROXY_VERBS = {"GET": "get", "HEAD": "get", "POST": "create", "PUT": "update", "PATCH": "patch", "DELETE": "delete",
               "OPTIONS": "get"}
# hop-by-hop headers (RFC 7230 §6.1) are never forwarded
_HOP = {"connection", "keep-alive", "proxy-authenticate", "proxy-authorization", "te", "trailer",
        "transfer-encoding", "upgrade", "host", "content-length", "authorization"}


def split_scheme_name_port(ident: str):
    """`[scheme:]name[:port]` (`pkg/util/net` SplitSchemeNamePort) -> (scheme, name, port)."""
    parts = ident.split(":")
    if len(parts) == 1:
        return "", parts[0], ""
    if len(parts) == 2:
        return "", parts[0], parts[1]
    if len(parts) == 3 and parts[0] in ("http", "https"):
        return parts[0], parts[1], parts[2]
    raise bad_request(f"invalid service request {ident!r}")


def legacy_proxy_path(path: str) -> str | None:
    """`/api/v1/proxy/namespaces/<ns>/<res>/<name>/<rest>` -> `/api/v1/namespaces/<ns>/<res>/<name>/proxy/<rest>`
    (and the cluster-scoped `/api/v1/proxy/nodes/<name>/<rest>`)."""
    parts = path.split("/")
    if len(parts) < 4 or parts[1:4] != ["api", "v1", "proxy"]:
        return None
    rest = parts[4:]
    if rest[:1] == ["namespaces"] and len(rest) >= 4:
        head, tail = rest[:4], rest[4:]
    elif rest[:1] == ["nodes"] and len(rest) >= 2:
        head, tail = rest[:2], rest[2:]
    else:
        return None
    return "/" + "/".join(["api", "v1"] + head + ["proxy"] + tail)


async def resolve_proxy_target(server, ri, ns, ident):
    """-> base URL (scheme://host:port) for `<ri>/<ident>/proxy`."""
    scheme, name, port = split_scheme_name_port(ident)
    scheme = scheme or (server.kubelet_scheme if ri.plural == "nodes" else "http")
    if ri.plural == "pods":
        _, e = await server._aexisting(ri, ns, name)
        ip = ((e.obj.get("status") or {}).get("podIP") or "")
        if not ip:
            raise bad_request(f"address not allowed: pod {name} has no IP yet")
        host = f"[{ip}]" if ":" in ip else ip
        return f"{scheme}://{host}:{port}" if port else f"{scheme}://{host}"
    if ri.plural == "services":
        _, e = await server._aexisting(ri, ns, name)
        svc = e.obj
        if port.isdigit():
            want = None
            for p in (svc.get("spec") or {}).get("ports") or ():
                if int(p.get("port", 0)) == int(port):
                    want = p.get("name", "")
                    break
            if want is None:
                raise APIError(503, "ServiceUnavailable", f"no service port {port} found for service \"{name}\"")
            port = want
        ep = server.get_object("endpoints", ns, name)
        if ep is None:
            try:
                _, ee = await server._aexisting(m.BY_PLURAL["endpoints"], ns, name)
                ep = ee.obj
            except APIError:
                ep = None
        subsets = list((ep or {}).get("subsets") or ())
        random.shuffle(subsets)
        for ss in subsets:
            for p in ss.get("ports") or ():
                if (p.get("name") or "") == (port or "") and ss.get("addresses"):
                    a = random.choice(ss["addresses"])["ip"]
                    host = f"[{a}]" if ":" in a else a
                    return f"{scheme}://{host}:{p['port']}"
        raise APIError(503, "ServiceUnavailable", f"no endpoints available for service \"{name}\"")
    if ri.plural == "nodes":
        node = server.get_object("nodes", None, name)
        if node is None:
            raise not_found(ri, name)
        st = node.get("status") or {}
        addr = ""
        for kind in ("InternalIP", "ExternalIP", "Hostname"):
            for a in st.get("addresses") or ():
                if a.get("type") == kind and not addr:
                    addr = a.get("address", "")
        addr = addr or "127.0.0.1"
        kport = port or str(((st.get("daemonEndpoints") or {}).get("kubeletEndpoint") or {}).get("Port") or "")
        if not kport:
            raise APIError(503, "ServiceUnavailable", f"node {name} has no kubelet endpoint")
        host = f"[{addr}]" if ":" in addr else addr
        return f"{scheme}://{host}:{kport}"
    raise APIError(404, "NotFound", f"{ri.plural} do not have a proxy subresource")


async def handle_proxy(server, req, ri, ns, ident, sub, user):
    """Any method on `<resource>/<ident>/proxy[/path]`."""
    verb = PROXY_VERBS.get(req.method)
    if verb is None:
        raise APIError(405, "MethodNotAllowed", f"method {req.method} not allowed")
    _, name, _ = split_scheme_name_port(ident)
    server._authorize(user, verb, ns, ri.plural, "proxy", name, ri.group, req.path)
    base = await resolve_proxy_target(server, ri, ns, ident)
    path = sub[len("proxy"):] or "/"
    if not path.startswith("/"):
        path = "/" + path
    if req.path.endswith("/") and not path.endswith("/"):
        path += "/"
    target = base + path + (f"?{req.qs}" if req.qs else "")
    from ..cri.remotecommand import is_upgrade_request, upgrade_proxy_response
    # kubelets: the configured kubelet TLS; https pods / services: not verified (the reference's
    # proxy transport for those has no CA to check against either)
    ctx = None
    if base.startswith("https://"):
        from ..utils.tlsutil import unverified_client_context
        ctx = server.kubelet_ssl if (ri.plural == "nodes" and server.kubelet_ssl is not None) else unverified_client_context()
    if is_upgrade_request(req.headers):
        return upgrade_proxy_response(req, target, ssl_context=ctx)
    from ..client.http import HTTPClient, HTTPError
    c = HTTPClient(base, ssl_context=ctx, timeout=30.0)
    try:
        hdrs = {k: v for k, v in req.headers.items() if k.lower() not in _HOP and k.lower() != "content-type"}
        st, rh, body = await c.request_full(req.method, path + (f"?{req.qs}" if req.qs else ""), req.body or None,
                                   req.headers.get("content-type") or "application/octet-stream", headers=hdrs)
    except (OSError, ConnectionError, HTTPError) as e:
        raise APIError(503, "ServiceUnavailable", f"error trying to reach {ri.kind.lower()}: {e}")
    finally:
        await c.close()
    return Response(st, body, rh.get("content-type") or "application/octet-stream")


# ------------------------------------------------------------------------------------------------
# server-side printing
def wants_table(accept: str) -> bool:
    """`Accept: application/json;as=Table;v=v1alpha1;g=meta.k8s.io` (kubectl get
    --experimental-server-print, `endpoints/handlers/rest.go` transformResponseObject)."""
    return "as=Table" in accept.replace(" ", "")


def to_table(obj: dict, kind: str, include: str = "Metadata") -> dict:
    """A GET / LIST response as a meta.k8s.io/v1alpha1 Table: the same columns `kubectl get`
    prints (`kubectl/printers.py`, the TableGenerator of `pkg/printers`), one row per object
    carrying the object (`includeObject=Object`), its PartialObjectMetadata (the default) or
    nothing (`None`)."""
    from ..kubectl import printers
    is_list = isinstance(obj.get("items"), list)
    items = obj["items"] if is_list else [obj]
    rows, headers = printers.rows_for(kind, items)
    cols = [{"name": h.title() if h != "NAME" else "Name", "type": "string", "format": "name" if h == "NAME" else "",
             "description": "", "priority": 0} for h in headers]
    out_rows = []
    for cells, o in zip(rows, items):
        row = {"cells": [str(c) for c in cells]}
        if include == "Object":
            row["object"] = o
        elif include != "None":
            row["object"] = {"kind": "PartialObjectMetadata", "apiVersion": "meta.k8s.io/v1alpha1",
                             "metadata": o.get("metadata") or {}}
        out_rows.append(row)
    md = {"resourceVersion": (obj.get("metadata") or {}).get("resourceVersion", "")}
    if is_list and (obj.get("metadata") or {}).get("continue"):
        md["continue"] = obj["metadata"]["continue"]
    return {"kind": "Table", "apiVersion": "meta.k8s.io/v1alpha1", "metadata": md, "columnDefinitions": cols,
            "rows": out_rows}
