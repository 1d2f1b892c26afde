"""Kubelet API authentication and authorization (`pkg/kubelet/server/auth.go`,
`cmd/kubelet/app/auth.go`).

  * authentication: x509 client certificates (verified by the TLS layer, `--client-ca-file`),
    bearer tokens checked with a TokenReview against the API server
    (`--authentication-token-webhook`, cached `--authentication-token-webhook-cache-ttl`), and
    anonymous requests as `system:anonymous` / `system:unauthenticated` unless
    `--anonymous-auth=false`;
  * authorization: `AlwaysAllow`, or `Webhook` — a SubjectAccessReview per request for the
    `nodes` resource of this node, verb from the HTTP method, subresource from the path
    (`/stats` → stats, `/metrics` → metrics, `/logs` → log, `/spec` → spec, anything else —
    `/pods`, `/exec`, `/containerLogs`, … — `proxy`), cached (`--authorization-webhook-cache-*`).
"""
from __future__ import annotations

import time
from collections import OrderedDict

ANONYMOUS = ("system:anonymous", ("system:unauthenticated",))
VERBS = {"GET": "get", "HEAD": "get", "POST": "create", "PUT": "update", "PATCH": "patch", "DELETE": "delete"}


class TTLCache:
    """Size-bounded LRU with per-entry expiry (the reference's webhook caches are LRUs of 1024
    entries for authn and 10000 for authz, `staging/src/k8s.io/apiserver/pkg/authentication/token/cache`)."""

    def __init__(self, size):
        self.size = size
        self._d: OrderedDict = OrderedDict()

    def get(self, key):
        hit = self._d.get(key)
        if hit is None:
            return None
        if hit[0] <= time.monotonic():
            del self._d[key]
            return None
        self._d.move_to_end(key)
        return hit

    def put(self, key, ttl, value):
        self._d[key] = (time.monotonic() + ttl, value)
        self._d.move_to_end(key)
        while len(self._d) > self.size:
            self._d.popitem(last=False)

    def __len__(self):
        return len(self._d)


def subresource_for(path: str) -> str:
    for prefix, sub in (("/stats", "stats"), ("/metrics", "metrics"), ("/logs", "log"), ("/spec", "spec")):
        if path == prefix or path.startswith(prefix + "/"):
            return sub
    return "proxy"


class KubeletAuth:
    def __init__(self, client, node_name, anonymous=True, token_webhook=False, authz_mode="AlwaysAllow",
                 authn_ttl=120.0, authz_allowed_ttl=300.0, authz_denied_ttl=30.0, authn_cache_size=1024,
                 authz_cache_size=10000):
        self.client = client
        self.node = node_name
        self.anonymous = anonymous
        self.token_webhook = token_webhook
        self.authz_mode = authz_mode
        self.authn_ttl, self.allowed_ttl, self.denied_ttl = authn_ttl, authz_allowed_ttl, authz_denied_ttl
        self._tokens = TTLCache(authn_cache_size)        # token -> (user, groups) or None
        self._decisions = TTLCache(authz_cache_size)     # (user, groups, verb, subresource) -> bool

    async def authenticate(self, req):
        """-> (user, groups) or None (401)."""
        ssl_obj = req.transport.get_extra_info("ssl_object") if req.transport is not None else None
        cert = ssl_obj.getpeercert() if ssl_obj is not None else None
        if cert:
            subj = dict(x[0] for x in cert.get("subject", ()))
            return subj.get("commonName", ""), tuple(v for k, v in (x[0] for x in cert.get("subject", ()))
                                                     if k == "organizationName")
        auth = req.headers.get("authorization", "")
        if auth.lower().startswith("bearer ") and self.token_webhook:
            tok = auth[7:].strip()
            hit = self._tokens.get(tok)
            if hit is not None:
                return hit[1]
            review = await self.client.create("tokenreviews", {"apiVersion": "authentication.k8s.io/v1",
                                                               "kind": "TokenReview", "spec": {"token": tok}})
            st = review.get("status") or {}
            who = None
            if st.get("authenticated"):
                u = st.get("user") or {}
                who = (u.get("username", ""), tuple(u.get("groups") or ()))
            self._tokens.put(tok, self.authn_ttl, who)
            return who
        return ANONYMOUS if self.anonymous else None

    async def authorize(self, user, groups, req) -> bool:
        if self.authz_mode == "AlwaysAllow":
            return True
        verb = VERBS.get(req.method, "get")
        sub = subresource_for(req.path)
        key = (user, groups, verb, sub)
        hit = self._decisions.get(key)
        if hit is not None:
            return hit[1]
        sar = await self.client.create("subjectaccessreviews", {
            "apiVersion": "authorization.k8s.io/v1", "kind": "SubjectAccessReview",
            "spec": {"user": user, "groups": list(groups),
                     "resourceAttributes": {"verb": verb, "resource": "nodes", "subresource": sub, "name": self.node}}})
        ok = bool((sar.get("status") or {}).get("allowed"))
        self._decisions.put(key, self.allowed_ttl if ok else self.denied_ttl, ok)
        return ok

    async def check(self, req):
        """None if the request may proceed, else (status, message)."""
        if req.path in ("/healthz", "/healthz/ping"):
            who = await self.authenticate(req)
            return None if who is not None else (401, "Unauthorized")
        who = await self.authenticate(req)
        if who is None:
            return 401, "Unauthorized"
        user, groups = who
        if not await self.authorize(user, groups, req):
            return 403, (f"Forbidden (user={user}, verb={VERBS.get(req.method, 'get')}, resource=nodes, "
                         f"subresource={subresource_for(req.path)})")
        return None
