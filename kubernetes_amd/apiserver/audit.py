"""Audit logging.

Parity: `staging/src/k8s.io/apiserver/pkg/endpoints/filters/audit.go:41` (`WithAudit`), the policy
checker (`staging/src/k8s.io/apiserver/pkg/audit/policy/checker.go`: first matching rule wins,
levels None < Metadata < Request < RequestResponse, rules match users / userGroups / verbs /
resources{group, resources, resourceNames} / namespaces / nonResourceURLs) and the log backend
(`staging/src/k8s.io/apiserver/plugin/pkg/audit/log/backend.go`: one JSON event per line).

Events are emitted at stage `ResponseComplete`, buffered and flushed once per event-loop turn.
"""
from __future__ import annotations

import asyncio
import json
import os
import threading
import time
import uuid
from datetime import datetime, timezone
from urllib.parse import urlencode

LEVELS = {"None": 0, "Metadata": 1, "Request": 2, "RequestResponse": 3}
_VERBS = {"POST": "create", "PUT": "update", "PATCH": "patch", "DELETE": "delete"}


def _ts():
    return datetime.now(timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")


class Policy:
    def __init__(self, rules=None, level="Metadata"):
        self.rules = rules if rules is not None else [{"level": level}]

    @classmethod
    def load(cls, path):
        import yaml
        with open(path) as f:
            doc = yaml.load(f, Loader=yaml.SafeLoader) or {}
        return cls(doc.get("rules") or [])

    def level_for(self, user, verb, resource, sub, namespace, name, group, path):
        for r in self.rules:
            if r.get("users") and (user is None or user.name not in r["users"]):
                continue
            if r.get("userGroups") and (user is None or not set(user.groups or ()) & set(r["userGroups"])):
                continue
            if r.get("verbs") and verb not in r["verbs"]:
                continue
            if r.get("namespaces") and (namespace or "") not in r["namespaces"]:
                continue
            if r.get("nonResourceURLs"):
                if resource or not any(path == u or (u.endswith("*") and path.startswith(u[:-1]))
                                       for u in r["nonResourceURLs"]):
                    continue
            if r.get("resources"):
                full = f"{resource}/{sub}" if sub else resource
                ok = False
                for gr in r["resources"]:
                    if gr.get("group", "") not in ("", group) and gr.get("group") != "*":
                        continue
                    names = gr.get("resources") or []
                    if names and full not in names and resource not in names and "*" not in names:
                        continue
                    if gr.get("resourceNames") and name not in gr["resourceNames"]:
                        continue
                    ok = True
                    break
                if not ok:
                    continue
            return LEVELS.get(r.get("level", "None"), 0)
        return 0


class AuditLogger:
    def __init__(self, path, policy: Policy | None = None, max_body=64 << 10):
        self.path = path
        self.policy = policy or Policy()
        self.max_body = max_body
        self._buf = []
        self._lock = threading.Lock()
        self._scheduled = False
        self.f = open(path, "a", buffering=1 << 16) if path not in ("-", None) else None

    def log(self, req, method, resource, sub, code, response_body=None):
        parsed_ns = name = None
        parts = [p for p in req.path.split("/") if p]
        if "namespaces" in parts:
            i = parts.index("namespaces")
            if i + 1 < len(parts):
                parsed_ns = parts[i + 1]
        if resource in parts:
            j = parts.index(resource)
            if j + 1 < len(parts):
                name = parts[j + 1]
        group = ""
        if parts and parts[0] == "apis" and len(parts) > 1:
            group = parts[1]
        verb = _VERBS.get(method)
        if verb is None:
            verb = "watch" if (req.query.get("watch") in ("true", "1") or "watch" in parts) else ("get" if name else "list")
        if method == "DELETE" and not name:
            verb = "deletecollection"
        user = getattr(req, "user", None)
        lvl = self.policy.level_for(user, verb, resource, sub, parsed_ns, name, group, req.path)
        if lvl == 0:
            return
        uri = req.raw_path + ("?" + urlencode(req.query) if req.query else "")
        peer = None
        try:
            peer = (req.transport.get_extra_info("peername") or (None,))[0]
        except Exception:
            pass
        ev = {"kind": "Event", "apiVersion": "audit.k8s.io/v1beta1", "level": next(k for k, v in LEVELS.items() if v == lvl),
              "auditID": str(uuid.uuid4()), "stage": "ResponseComplete", "requestURI": uri,
              "verb": verb, "user": {"username": getattr(user, "name", "system:anonymous"),
                                     "groups": list(getattr(user, "groups", ()) or ())},
              "sourceIPs": [peer or "127.0.0.1"],
              "objectRef": {"resource": resource, "namespace": parsed_ns, "name": name, "apiGroup": group,
                            "subresource": sub or None},
              "responseStatus": {"metadata": {}, "code": code},
              "requestReceivedTimestamp": _ts(), "stageTimestamp": _ts()}
        if lvl >= 2 and req.body and len(req.body) <= self.max_body:
            try:
                ev["requestObject"] = json.loads(req.body)
            except ValueError:
                pass
        if lvl >= 3 and response_body and len(response_body) <= self.max_body:
            try:
                ev["responseObject"] = json.loads(response_body)
            except ValueError:
                pass
        line = json.dumps(ev, separators=(",", ":"))
        with self._lock:
            self._buf.append(line)
            if not self._scheduled:
                self._scheduled = True
                try:
                    asyncio.get_running_loop().call_soon(self.flush)
                except RuntimeError:
                    self._scheduled = False
                    self.flush()

    def flush(self):
        with self._lock:
            buf, self._buf = self._buf, []
            self._scheduled = False
        if not buf:
            return
        data = "\n".join(buf) + "\n"
        if self.f is None:
            os.write(1, data.encode())
        else:
            self.f.write(data)
            self.f.flush()

    def close(self):
        self.flush()
        if self.f is not None:
            self.f.close()
            self.f = None


def now():
    return time.time()
