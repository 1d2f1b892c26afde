"""Authentication and authorization.

Parity: token-file authenticator (`staging/src/k8s.io/apiserver/plugin/pkg/authenticator/token/tokenfile`),
anonymous user, authorizer modes AlwaysAllow / AlwaysDeny / RBAC
(`plugin/pkg/auth/authorizer/rbac`) / Node (`plugin/pkg/auth/authorizer/node`).
"""
from __future__ import annotations

import csv
from dataclasses import dataclass, field


@dataclass
class User:
    name: str
    uid: str = ""
    groups: list = field(default_factory=list)


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
        if "system:masters" in (u.groups or []):
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
    """Nodes may read/write what their pods need; everything else defers to the next authorizer."""

    RESOURCES = {"nodes", "pods", "events", "configmaps", "secrets", "persistentvolumeclaims",
                 "persistentvolumes", "endpoints", "services", "leases"}

    def authorize(self, a):
        u = a.user
        if not u.name.startswith("system:node:") or "system:nodes" not in (u.groups or []):
            return None, ""
        if a.resource in self.RESOURCES:
            return True, ""
        return None, ""


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
            azs.append(NodeAuthorizer())
        else:
            raise ValueError(f"unknown authorization mode {m}")
    return UnionAuthorizer(azs)
