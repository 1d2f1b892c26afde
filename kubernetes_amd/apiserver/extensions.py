"""API server extension points: admission webhooks, CustomResourceDefinitions, API aggregation.

Admission webhooks — `staging/src/k8s.io/apiserver/pkg/admission/plugin/webhook`:
  * MutatingWebhookConfiguration / ValidatingWebhookConfiguration (admissionregistration.k8s.io
    v1beta1); a hook is called when one of its `rules` matches (operations, apiGroups,
    apiVersions, resources incl. `res/sub` and `*`, `rules/rules.go:33-95`) and its
    `namespaceSelector` matches the namespace labels (`namespace/matcher.go:89-117`: cluster
    scoped non-namespace objects always match);
  * request = AdmissionReview v1beta1 (`request/admissionreview.go:29-71`), POSTed to
    `clientConfig.url` or `clientConfig.service` (resolved through the service's endpoints,
    HTTPS verified against `caBundle`);
  * mutating hooks run in order and apply the returned base64 JSONPatch
    (`mutating/admission.go:199-321`); validating hooks run after all mutation and validation
    (`validating/admission.go`), all relevant ones in parallel; `failurePolicy: Ignore` (the
    v1beta1 default) fails open on call errors, `Fail` rejects; a denial returns the hook's
    `result` status (403 by default).
CustomResourceDefinitions — `staging/src/k8s.io/apiextensions-apiserver`:
  * a CRD named `<plural>.<group>` installs `/apis/<group>/<version>/[namespaces/<ns>/]<plural>`
    with discovery; names are checked against existing resources and the CRD's status gets
    `acceptedNames`, `NamesAccepted` and `Established` (`controller/status/naming_controller.go`);
  * custom objects are validated against `spec.validation.openAPIV3Schema` (type, required,
    properties, items, enum, minimum/maximum, minLength/maxLength, pattern);
  * deleting a CRD deletes all of its custom objects first (`controller/finalizer`).
API aggregation — `staging/src/k8s.io/kube-aggregator`:
  * APIService `<version>.<group>` with `spec.service` proxies `/apis/<group>/<version>/...` to
    the service's endpoint; the group appears in `/apis` discovery; status condition
    `Available` follows whether the service has endpoints (`available_controller.go`).
"""
from __future__ import annotations

import asyncio
import base64
import json
import logging
import re
import ssl

from ..api import meta as m
from ..api.labels import label_selector_as_selector
from .registry import APIError

log = logging.getLogger("apiserver.extensions")

MUTATING = "mutatingwebhookconfigurations"
VALIDATING = "validatingwebhookconfigurations"


# ------------------------------------------------------------------------------------ webhooks
def _rule_matches(rule, op, group, version, resource, sub):
    ops = rule.get("operations") or []
    if "*" not in ops and op not in ops:
        return False
    if not any(g in ("*", group) for g in rule.get("apiGroups") or []):
        return False
    if not any(v in ("*", version) for v in rule.get("apiVersions") or []):
        return False
    for r in rule.get("resources") or []:
        res, _, rsub = r.partition("/")
        if res in ("*", resource) and (rsub in ("*", sub) if "/" in r else sub == ""):
            return True
    return False


class WebhookDispatcher:
    def __init__(self, server):
        self.server = server
        self.calls = 0

    def _hooks(self, plural):
        out = []
        for cfg in sorted(self.server.list_objects(plural), key=m.name_of):
            out.extend(cfg.get("webhooks") or [])
        return out

    def has_any(self):
        s = self.server
        return bool(s.caches[MUTATING].by_key) or bool(s.caches[VALIDATING].by_key)

    def _ns_labels(self, a):
        if a.resource == "namespaces" and not a.subresource and a.obj is not None:
            return (a.obj.get("metadata") or {}).get("labels") or {}
        ns = self.server.get_object("namespaces", None, a.namespace)
        if ns is None:
            raise APIError(404, "NotFound", f'namespaces "{a.namespace}" not found')
        return (ns.get("metadata") or {}).get("labels") or {}

    def _relevant(self, hook, a, ri):
        if not any(_rule_matches(r, a.operation, ri.group, ri.version, ri.plural, a.subresource or "")
                   for r in hook.get("rules") or []):
            return False
        if not a.namespace and a.resource != "namespaces":
            return True
        sel = hook.get("namespaceSelector")
        if not sel:
            return True
        return label_selector_as_selector(sel).matches(self._ns_labels(a))

    def _review(self, a, ri):
        u = a.user
        user = {"username": getattr(u, "name", "") or "", "uid": getattr(u, "uid", "") or "",
                "groups": list(getattr(u, "groups", ()) or ()), "extra": dict(getattr(u, "extra", {}) or {})}
        req = {"uid": m.new_uid(), "kind": {"group": ri.group, "version": ri.version, "kind": ri.kind},
               "resource": {"group": ri.group, "version": ri.version, "resource": ri.plural},
               "subResource": a.subresource or "", "name": a.name or "", "namespace": a.namespace or "",
               "operation": a.operation, "userInfo": user, "object": a.obj, "oldObject": a.old}
        return {"kind": "AdmissionReview", "apiVersion": "admission.k8s.io/v1beta1", "request": req}

    def _endpoint(self, cc):
        """clientConfig -> (base URL, ssl context or None, path)."""
        ca = cc.get("caBundle")
        ctx = None
        if cc.get("url"):
            url = cc["url"]
            if url.startswith("https://"):
                ctx = ssl.create_default_context(cadata=base64.b64decode(ca).decode() if ca else None)
                ctx.check_hostname = False
            scheme_host, _, path = url.partition("://")[2].partition("/")
            return f"{url.split('://')[0]}://{scheme_host}", ctx, "/" + path
        svc = cc.get("service") or {}
        ns, name = svc.get("namespace", "default"), svc.get("name", "")
        ep = self.server.get_object("endpoints", ns, name)
        for ss in (ep or {}).get("subsets") or ():
            for addr in ss.get("addresses") or ():
                port = (ss.get("ports") or [{}])[0].get("port", 443)
                scheme = "https" if ca else "http"
                if ca:
                    ctx = ssl.create_default_context(cadata=base64.b64decode(ca).decode())
                    ctx.check_hostname = False
                return f"{scheme}://{addr['ip']}:{port}", ctx, svc.get("path") or "/"
        raise ConnectionError(f"service {ns}/{name} has no endpoints")

    async def _call(self, hook, review):
        from ..client.http import HTTPClient
        base, ctx, path = self._endpoint(hook.get("clientConfig") or {})
        c = HTTPClient(base, ssl_context=ctx, timeout=float(hook.get("timeoutSeconds") or 30))
        try:
            st, body = await c.request("POST", path, json.dumps(review).encode())
        finally:
            await c.close()
        if st != 200:
            raise ConnectionError(f"webhook returned HTTP {st}")
        return (json.loads(body) or {}).get("response") or {}

    async def _ask(self, hook, a, ri):
        """One webhook call: its response, or None when it failed open."""
        self.calls += 1
        try:
            resp = await self._call(hook, self._review(a, ri))
        except (ConnectionError, OSError, asyncio.TimeoutError, ValueError) as e:
            if hook.get("failurePolicy", "Ignore") != "Fail":
                log.warning("failed calling webhook %s, failing open: %s", hook.get("name"), e)
                return None
            raise APIError(500, "InternalError", f'Internal error occurred: failed calling admission webhook "{hook.get("name")}": {e}')
        if not resp.get("allowed"):
            res = resp.get("result") or {}
            raise APIError(int(res.get("code") or 403), res.get("reason") or "Forbidden",
                           f'admission webhook "{hook.get("name")}" denied the request: {res.get("message", "without explanation")}')
        return resp

    async def run(self, a, ri, mutating):
        hooks = [h for h in self._hooks(MUTATING if mutating else VALIDATING) if self._relevant(h, a, ri)]
        if not mutating:
            # validating/admission.go: every relevant hook is called in parallel; the first
            # error (in hook order) is returned
            results = await asyncio.gather(*(self._ask(h, a, ri) for h in hooks), return_exceptions=True)
            for r in results:
                if isinstance(r, BaseException):
                    raise r
            return
        for hook in hooks:
            resp = await self._ask(hook, a, ri)
            if resp is None:
                continue
            if resp.get("patch"):
                from ..utils.patch import json_patch
                try:
                    a.obj = json_patch(a.obj, json.loads(base64.b64decode(resp["patch"])))
                except Exception as e:
                    raise APIError(500, "InternalError", f"webhook {hook.get('name')} returned an invalid patch: {e}")


# ------------------------------------------------------------------------------------ CRDs
def crd_resource_info(crd):
    sp = crd.get("spec") or {}
    names = sp.get("names") or {}
    return m.ResourceInfo(sp.get("group", ""), sp.get("version") or ((sp.get("versions") or [{}])[0].get("name", "v1")),
                          names.get("kind", ""), names.get("plural", ""), sp.get("scope", "Namespaced") == "Namespaced",
                          tuple(names.get("shortNames") or ()))


def validate_crd(crd):
    from ..api import validation as v
    errs = v.validate_object_meta(crd, False)
    sp = crd.get("spec") or {}
    names = sp.get("names") or {}
    for f in ("group",):
        if not sp.get(f):
            errs.append(v.required(f"spec.{f}"))
    if not (sp.get("version") or sp.get("versions")):
        errs.append(v.required("spec.version"))
    for f in ("plural", "kind"):
        if not names.get(f):
            errs.append(v.required(f"spec.names.{f}"))
    if sp.get("scope", "Namespaced") not in ("Namespaced", "Cluster"):
        errs.append(v.not_supported("spec.scope", sp.get("scope")))
    if names.get("plural") and sp.get("group") and m.name_of(crd) != f"{names['plural']}.{sp['group']}":
        errs.append(v.invalid("metadata.name", f"must be spec.names.plural+\".\"+spec.group"))
    return errs


def _type_ok(val, t):
    return {"object": isinstance(val, dict), "array": isinstance(val, list), "string": isinstance(val, str),
            "integer": isinstance(val, int) and not isinstance(val, bool),
            "number": isinstance(val, (int, float)) and not isinstance(val, bool),
            "boolean": isinstance(val, bool)}.get(t, True)


def validate_schema(val, schema, path="", errs=None):
    """The openAPIV3Schema subset the 1.9 CRD validation supports."""
    errs = [] if errs is None else errs
    if not schema:
        return errs
    t = schema.get("type")
    if t and not _type_ok(val, t):
        errs.append(f"{path or '<root>'}: Invalid value: must be of type {t}")
        return errs
    if "enum" in schema and val not in schema["enum"]:
        errs.append(f"{path}: Unsupported value: {val!r}: supported values: {schema['enum']}")
    if isinstance(val, (int, float)) and not isinstance(val, bool):
        if "minimum" in schema and val < schema["minimum"]:
            errs.append(f"{path}: Invalid value: {val}: must be greater than or equal to {schema['minimum']}")
        if "maximum" in schema and val > schema["maximum"]:
            errs.append(f"{path}: Invalid value: {val}: must be less than or equal to {schema['maximum']}")
    if isinstance(val, str):
        if "minLength" in schema and len(val) < schema["minLength"]:
            errs.append(f"{path}: Invalid value: should be at least {schema['minLength']} chars long")
        if "maxLength" in schema and len(val) > schema["maxLength"]:
            errs.append(f"{path}: Invalid value: should be at most {schema['maxLength']} chars long")
        if "pattern" in schema and not re.search(schema["pattern"], val):
            errs.append(f"{path}: Invalid value: {val!r}: should match {schema['pattern']!r}")
    if isinstance(val, dict):
        for r in schema.get("required") or ():
            if r not in val:
                errs.append(f"{path + '.' if path else ''}{r}: Required value")
        for k, sub in (schema.get("properties") or {}).items():
            if k in val:
                validate_schema(val[k], sub, f"{path + '.' if path else ''}{k}", errs)
    if isinstance(val, list) and schema.get("items"):
        for i, item in enumerate(val):
            validate_schema(item, schema["items"], f"{path}[{i}]", errs)
    return errs


class CRDManager:
    def __init__(self, server):
        self.server = server
        self.installed: dict[str, m.ResourceInfo] = {}   # crd name -> ResourceInfo
        self.schemas: dict[str, dict] = {}               # plural -> openAPIV3Schema

    def names_conflict(self, crd):
        ri = crd_resource_info(crd)
        existing = self.server.caches.get(ri.plural)
        if existing is None:
            return None
        owner = next((n for n, r in self.installed.items() if r.plural == ri.plural), None)
        if owner != m.name_of(crd):
            return f'"{ri.plural}" is already in use'
        return None

    def prepare(self, crd):
        """Set acceptedNames + NamesAccepted / Established (naming controller, done synchronously)."""
        from ..api.meta import now_rfc3339
        conflict = self.names_conflict(crd)
        st = crd.setdefault("status", {})
        now = now_rfc3339()
        names = (crd.get("spec") or {}).get("names") or {}
        if conflict:
            st["conditions"] = [{"type": "NamesAccepted", "status": "False", "reason": "PluralConflict",
                                 "message": conflict, "lastTransitionTime": now},
                                {"type": "Established", "status": "False", "reason": "NotAccepted",
                                 "message": "not all names are accepted", "lastTransitionTime": now}]
            st["acceptedNames"] = {}
        else:
            st["acceptedNames"] = dict(names, listKind=names.get("listKind") or names.get("kind", "") + "List",
                                       singular=names.get("singular") or names.get("kind", "").lower())
            st["conditions"] = [{"type": "NamesAccepted", "status": "True", "reason": "NoConflicts",
                                 "message": "no conflicts found", "lastTransitionTime": now},
                                {"type": "Established", "status": "True", "reason": "InitialNamesAccepted",
                                 "message": "the initial names have been accepted", "lastTransitionTime": now}]

    def observe(self, crd, deleted=False):
        name = m.name_of(crd)
        if deleted:
            ri = self.installed.pop(name, None)
            if ri is not None:
                self.server.uninstall_resource(ri)
                self.schemas.pop(ri.plural, None)
            return
        est = any(c.get("type") == "Established" and c.get("status") == "True"
                  for c in (crd.get("status") or {}).get("conditions") or ())
        if not est or name in self.installed:
            if name in self.installed:
                self.schemas[self.installed[name].plural] = ((crd.get("spec") or {}).get("validation") or {}).get("openAPIV3Schema") or {}
            return
        ri = crd_resource_info(crd)
        self.installed[name] = ri
        self.schemas[ri.plural] = ((crd.get("spec") or {}).get("validation") or {}).get("openAPIV3Schema") or {}
        self.server.install_resource(ri)

    def validate_object(self, ri, obj):
        schema = self.schemas.get(ri.plural)
        if not schema:
            return []
        body = {k: v for k, v in obj.items() if k not in ("apiVersion", "kind", "metadata")}
        sch = dict(schema)
        props = dict(sch.get("properties") or {})
        for k in ("apiVersion", "kind", "metadata"):
            props.pop(k, None)
        sch["properties"] = props
        sch["required"] = [r for r in sch.get("required") or () if r not in ("apiVersion", "kind", "metadata")]
        return validate_schema(body, sch)


# ------------------------------------------------------------------------------------ aggregation
class Aggregator:
    def __init__(self, server):
        self.server = server

    def _services(self):
        return self.server.list_objects("apiservices") if "apiservices" in self.server.caches else []

    def lookup(self, group, version):
        for a in self._services():
            sp = a.get("spec") or {}
            if sp.get("group") == group and sp.get("version") == version and sp.get("service"):
                return a
        return None

    def groups(self):
        out = {}
        for a in self._services():
            sp = a.get("spec") or {}
            if sp.get("service") and sp.get("group"):
                out.setdefault(sp["group"], set()).add(sp.get("version", "v1"))
        return out

    def backend(self, apisvc):
        svc = (apisvc.get("spec") or {}).get("service") or {}
        ep = self.server.get_object("endpoints", svc.get("namespace", "default"), svc.get("name", ""))
        for ss in (ep or {}).get("subsets") or ():
            for addr in ss.get("addresses") or ():
                port = (ss.get("ports") or [{}])[0].get("port", 443)
                return addr["ip"], port
        return None

    def available(self, apisvc):
        return self.backend(apisvc) is not None

    async def proxy(self, req, apisvc):
        from ..client.http import HTTPClient
        from ..utils.httpserver import Response
        be = self.backend(apisvc)
        if be is None:
            raise APIError(503, "ServiceUnavailable", f"service unavailable for {m.name_of(apisvc)}")
        sp = apisvc.get("spec") or {}
        scheme = "http" if sp.get("insecureSkipTLSVerify") or not sp.get("caBundle") else "https"
        ctx = None
        if scheme == "https":
            ctx = ssl.create_default_context(cadata=base64.b64decode(sp["caBundle"]).decode())
            ctx.check_hostname = False
            pc = getattr(self.server, "proxy_client_cert", None)
            if pc:       # --proxy-client-cert-file/--proxy-client-key-file: the front-proxy identity
                ctx.load_cert_chain(pc[0], pc[1])
        c = HTTPClient(f"{scheme}://{be[0]}:{be[1]}", ssl_context=ctx)
        u = getattr(req, "user", None)
        hdrs = {"X-Remote-User": getattr(u, "name", "") or ""}
        groups = list(getattr(u, "groups", ()) or ())
        if groups:       # one header, values comma-joined (what repeated headers become on the wire)
            hdrs["X-Remote-Group"] = ", ".join(groups)
        try:
            path = req.raw_path + (("?" + req.qs) if req.qs else "")
            st, body = await c.request(req.method, path, req.body or None,
                                       req.headers.get("content-type", "application/json"), hdrs)
        except OSError as e:
            raise APIError(503, "ServiceUnavailable", f"error trying to reach service: {e}")
        finally:
            await c.close()
        return Response(st, body)
