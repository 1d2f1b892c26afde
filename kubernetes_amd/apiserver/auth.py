"""Authentication and authorization.

Parity: token-file authenticator (`staging/src/k8s.io/apiserver/plugin/pkg/authenticator/token/tokenfile`),
anonymous user, authorizer modes AlwaysAllow / AlwaysDeny / RBAC
(`plugin/pkg/auth/authorizer/rbac`) / Node (`plugin/pkg/auth/authorizer/node`).
"""
from __future__ import annotations

import csv
from dataclasses import dataclass, field

from ..api import core


@dataclass
class User:
    name: str
    uid: str = ""
    groups: list = field(default_factory=list)
    impersonated_by: object = field(default=None, repr=False, compare=False)   # the requesting user


ANONYMOUS = User("system:anonymous", groups=["system:unauthenticated"])


class TokenAuthenticator:
    """CSV: token,user,uid,"group1,group2" (`--token-auth-file`)."""

    def __init__(self, path=None, tokens=None):
        self.tokens = dict(tokens or {})
        if path:
            with open(path) as f:
                for row in csv.reader(f):
                    if len(row) < 3 or row[0].startswith("#"):
                        continue
                    groups = row[3].split(",") if len(row) > 3 and row[3] else []
                    self.tokens[row[0]] = User(row[1], row[2], groups + ["system:authenticated"])

    def authenticate_token(self, token):
        return self.tokens.get(token)

    def authenticate(self, headers):
        h = headers.get("authorization", "")
        if h.lower().startswith("bearer "):
            u = self.tokens.get(h[7:].strip())
            if u is None:
                return None  # 401
            return u
        return ANONYMOUS


class AttributesRecord:
    __slots__ = ("user", "verb", "namespace", "resource", "subresource", "name", "group", "path", "resource_request")

    def __init__(self, user, verb, namespace, resource, subresource, name, group, path, resource_request=True):
        self.user, self.verb, self.namespace, self.resource = user, verb, namespace, resource
        self.subresource, self.name, self.group, self.path = subresource, name, group, path
        self.resource_request = resource_request


class AlwaysAllow:
    def authorize(self, a):
        return True, ""


class AlwaysDeny:
    def authorize(self, a):
        return False, "AlwaysDeny"


def _rule_matches(rule, a):
    verbs = rule.get("verbs") or []
    if "*" not in verbs and a.verb not in verbs:
        return False
    if not a.resource_request:
        urls = rule.get("nonResourceURLs") or []
        return any(u == "*" or u == a.path or (u.endswith("*") and a.path.startswith(u[:-1])) for u in urls)
    groups = rule.get("apiGroups") or []
    if "*" not in groups and a.group not in groups:
        return False
    res = rule.get("resources") or []
    full = a.resource + ("/" + a.subresource if a.subresource else "")
    if "*" not in res and full not in res and not (a.subresource and f"{a.resource}/*" in res):
        return False
    names = rule.get("resourceNames") or []
    return not names or a.name in names


class RBACAuthorizer:
    """Evaluates Role/ClusterRole + bindings read live from the API server's cache."""

    def __init__(self, server):
        self.server = server
        # --authorization-rbac-super-user: this user passes every RBAC check
        self.super_user = getattr(server, "rbac_super_user", None)

    def _subject_matches(self, s, user):
        k = s.get("kind")
        if k == "User":
            return s.get("name") == user.name
        if k == "Group":
            return s.get("name") in user.groups
        if k == "ServiceAccount":
            return user.name == f"system:serviceaccount:{s.get('namespace')}:{s.get('name')}"
        return False

    def _rules(self, ref, ns):
        kind, name = ref.get("kind"), ref.get("name")
        if kind == "ClusterRole":
            r = self.server.get_object("clusterroles", None, name)
        else:
            r = self.server.get_object("roles", ns, name)
        return (r or {}).get("rules") or []

    def authorize(self, a):
        u = a.user
        if "system:masters" in (u.groups or []) or (self.super_user and u.name == self.super_user):
            return True, ""
        for b in self.server.list_objects("clusterrolebindings"):
            if any(self._subject_matches(s, u) for s in b.get("subjects") or ()):
                if any(_rule_matches(r, a) for r in self._rules(b.get("roleRef") or {}, None)):
                    return True, ""
        if a.namespace:
            for b in self.server.list_objects("rolebindings", a.namespace):
                if any(self._subject_matches(s, u) for s in b.get("subjects") or ()):
                    if any(_rule_matches(r, a) for r in self._rules(b.get("roleRef") or {}, a.namespace)):
                        return True, ""
        return False, f'User "{u.name}" cannot {a.verb} {a.resource} in the namespace "{a.namespace}"'


class NodeAuthorizer:
    """`plugin/pkg/auth/authorizer/node/node_authorizer.go`: a node (`system:node:<name>` in
    `system:nodes`) may `get` a secret / configmap / PVC / PV only when a pod bound to it
    references the object (the reference walks a pod -> object graph; here the graph is read from
    the API server's pod cache); the rest of the node's working set (its Node, pods, events,
    endpoints, services, leases, CSRs) is allowed; anything else defers to the next authorizer."""

    GRAPH = {"secrets", "configmaps", "persistentvolumeclaims", "persistentvolumes"}
    RESOURCES = {"nodes", "pods", "events", "endpoints", "services", "leases", "certificatesigningrequests"}

    def __init__(self, server=None):
        self.server = server

    def _related(self, node, a):
        if self.server is None:
            return True
        for p in self.server.list_objects("pods"):
            if (p.get("spec") or {}).get("nodeName") != node:
                continue
            sp = p.get("spec") or {}
            ns = p["metadata"].get("namespace")
            if a.resource == "persistentvolumes":
                for v in sp.get("volumes") or ():
                    c = (v.get("persistentVolumeClaim") or {}).get("claimName")
                    pvc = self.server.get_object("persistentvolumeclaims", ns, c) if c else None
                    if pvc and (pvc.get("spec") or {}).get("volumeName") == a.name:
                        return True
                continue
            if ns != a.namespace:
                continue
            if a.resource == "secrets":
                names = set(core.pod_secret_names(p))
            elif a.resource == "configmaps":
                names = {(v.get("configMap") or {}).get("name") for v in sp.get("volumes") or ()}
                for c in (sp.get("containers") or []) + (sp.get("initContainers") or []):
                    for e in c.get("env") or ():
                        names.add(((e.get("valueFrom") or {}).get("configMapKeyRef") or {}).get("name"))
                    for ef in c.get("envFrom") or ():
                        names.add((ef.get("configMapRef") or {}).get("name"))
                for v in sp.get("volumes") or ():
                    for src in (v.get("projected") or {}).get("sources") or ():
                        names.add((src.get("configMap") or {}).get("name"))
            else:
                names = {(v.get("persistentVolumeClaim") or {}).get("claimName") for v in sp.get("volumes") or ()}
            if a.name in names:
                return True
        return False

    def authorize(self, a):
        u = a.user
        if not u.name.startswith("system:node:") or "system:nodes" not in (u.groups or []):
            return None, ""
        node = u.name[len("system:node:"):]
        if a.resource in self.GRAPH:
            if a.verb == "get" and a.name and self._related(node, a):
                return True, ""
            return False, f'no path found to object {a.resource}/{a.name} from node "{node}"'
        if a.resource in self.RESOURCES:
            return True, ""
        return None, ""


class ABACAuthorizer:
    """`pkg/auth/authorizer/abac/abac.go`: one JSON policy per line
    (`{"apiVersion":"abac.authorization.kubernetes.io/v1beta1","kind":"Policy","spec":{...}}`);
    spec fields user / group / namespace / resource / apiGroup / readonly / nonResourcePath,
    `*` wildcards; the first matching policy allows."""

    READONLY = {"get", "list", "watch"}

    def __init__(self, path=None, policies=None):
        self.policies = list(policies or [])
        if path:
            import json
            with open(path) as f:
                for line in f:
                    line = line.strip()
                    if line and not line.startswith("#"):
                        p = json.loads(line)
                        self.policies.append(p.get("spec", p))

    @staticmethod
    def _m(want, have):
        return want == "*" or want == have

    def authorize(self, a):
        u = a.user
        for p in self.policies:
            if p.get("user") and not self._m(p["user"], u.name):
                continue
            if p.get("group") and not (p["group"] == "*" or p["group"] in (u.groups or [])):
                continue
            if not p.get("user") and not p.get("group"):
                continue
            if p.get("readonly") and a.verb not in self.READONLY:
                continue
            if a.resource_request:
                if not (self._m(p.get("namespace", ""), a.namespace) and self._m(p.get("resource", ""), a.resource)
                        and self._m(p.get("apiGroup", ""), a.group)):
                    continue
            else:
                np = p.get("nonResourcePath", "")
                if not (np == "*" or np == a.path or (np.endswith("*") and a.path.startswith(np[:-1]))):
                    continue
            return True, ""
        return None, ""


class WebhookAuthorizer:
    """`staging/src/k8s.io/apiserver/plugin/pkg/authorizer/webhook`: SubjectAccessReview POSTed to
    a remote service; allowed answers cached 5 min, denied 30 s."""

    def __init__(self, url, allow_ttl=300.0, deny_ttl=30.0, ssl_context=None):
        self.url, self.allow_ttl, self.deny_ttl, self.ssl = url, allow_ttl, deny_ttl, ssl_context
        self.cache = {}

    def authorize(self, a):
        import json
        import time
        import urllib.request
        u = a.user
        spec = {"user": u.name, "groups": list(u.groups or ()), "uid": u.uid or ""}
        if a.resource_request:
            spec["resourceAttributes"] = {"namespace": a.namespace, "verb": a.verb, "group": a.group,
                                          "resource": a.resource, "subresource": a.subresource, "name": a.name}
        else:
            spec["nonResourceAttributes"] = {"path": a.path, "verb": a.verb}
        key = json.dumps(spec, sort_keys=True)
        hit = self.cache.get(key)
        now = time.monotonic()
        if hit is not None and now < hit[1]:
            return hit[0]
        body = json.dumps({"apiVersion": "authorization.k8s.io/v1", "kind": "SubjectAccessReview", "spec": spec}).encode()
        try:
            req = urllib.request.Request(self.url, body, {"Content-Type": "application/json"})
            with urllib.request.urlopen(req, timeout=10, context=self.ssl) as r:
                st = json.loads(r.read()).get("status") or {}
        except OSError as e:
            return False, f"webhook authorizer error: {e}"
        res = (True, "") if st.get("allowed") else ((False, st.get("reason", "")) if st.get("denied") else (None, st.get("reason", "")))
        self.cache[key] = (res, now + (self.allow_ttl if res[0] else self.deny_ttl))
        return res


class UnionAuthorizer:
    def __init__(self, authorizers):
        self.authorizers = authorizers

    def authorize(self, a):
        reason = ""
        for az in self.authorizers:
            ok, why = az.authorize(a)
            if ok:
                return True, ""
            if ok is False and why:
                reason = why
        return False, reason or "forbidden"


def build_authorizer(modes, server):
    azs = []
    for m in modes:
        if m == "AlwaysAllow":
            azs.append(AlwaysAllow())
        elif m == "AlwaysDeny":
            azs.append(AlwaysDeny())
        elif m == "RBAC":
            azs.append(RBACAuthorizer(server))
        elif m == "Node":
            azs.append(NodeAuthorizer(server))
        elif m == "ABAC":
            azs.append(ABACAuthorizer(getattr(server, "abac_policy_file", None)))
        elif m == "Webhook":
            cfg = getattr(server, "authz_webhook", None)
            if cfg is not None:       # --authorization-webhook-config-file (kubeconfig format)
                azs.append(WebhookAuthorizer(cfg[0], cfg[2], cfg[3], cfg[1]))
            else:
                azs.append(WebhookAuthorizer(getattr(server, "authorization_webhook_url", None)))
        else:
            raise ValueError(f"unknown authorization mode {m}")
    return UnionAuthorizer(azs)
