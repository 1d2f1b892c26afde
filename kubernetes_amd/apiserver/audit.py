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
    """Log backend (`plugin/pkg/audit/log`): `format` json (one audit.k8s.io Event per line) or
    legacy (the pre-1.8 `AUDIT: id=... ip=... method=... user=...` request line plus a
    `response="<code>"` line); rotation like the reference's lumberjack writer — past
    `max_size_mb` the file moves to `<name>-<UTC timestamp><ext>`, at most `max_backups` such
    backups are kept and those older than `max_age_days` are removed (0 = no limit)."""

    def __init__(self, path, policy: Policy | None = None, max_body=64 << 10, webhook=None, format="json",
                 max_size_mb=0, max_backups=0, max_age_days=0):
        if format not in ("json", "legacy"):
            raise ValueError(f"unknown audit log format {format!r}")
        self.format = format
        self.max_size = int(max_size_mb) << 20
        self.max_backups, self.max_age = int(max_backups), float(max_age_days) * 86400
        self.path = path
        self.policy = policy or Policy()
        self.max_body = max_body
        self._buf = []
        self._wbuf = []               # JSON events for a batching webhook
        self._lock = threading.Lock()
        self._scheduled = False
        self.stdout = path == "-"
        self.f = open(path, "a", buffering=1 << 16) if path not in ("-", None) else None
        self.webhook = webhook        # WebhookBackend or None

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
        real = getattr(user, "impersonated_by", None)
        if real is not None:      # the event's user is who asked; impersonatedUser who it ran as
            ev["impersonatedUser"] = ev["user"]
            ev["user"] = {"username": real.name, "groups": list(real.groups or ())}
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
        js = json.dumps(ev, separators=(",", ":"))     # the webhook always gets JSON events
        if self.format == "legacy":
            u = ev["user"]
            groups = ",".join(f'\\"{g}\\"' for g in u["groups"])
            line = (f'{ev["requestReceivedTimestamp"]} AUDIT: id="{ev["auditID"]}" ip="{ev["sourceIPs"][0]}" '
                    f'method="{method}" user="{u["username"]}" groups="{groups}" as="<self>" asgroups="<lookup>" '
                    f'namespace="{parsed_ns or "<none>"}" uri="{uri}"\n'
                    f'{ev["stageTimestamp"]} AUDIT: id="{ev["auditID"]}" response="{code}"')
        else:
            line = js
        self._append(line, js)
        return js

    @property
    def blocking(self):
        return self.webhook is not None and self.webhook.blocking

    async def deliver(self, line):
        """Blocking webhook mode: the request waits until its event was POSTed."""
        await asyncio.to_thread(self.webhook.post_now, [line])

    def _append(self, line, js):
        flush_now = False
        with self._lock:
            self._buf.append(line)
            if self.webhook is not None and not self.webhook.blocking:
                self._wbuf.append(js)
            if not self._scheduled:
                self._scheduled = True
                try:
                    asyncio.get_running_loop().call_soon(self.flush)
                except RuntimeError:       # no event loop (tools, tests): write through
                    self._scheduled = False
                    flush_now = True
        if flush_now:
            self.flush()                   # outside the (non-reentrant) lock flush() takes

    def flush(self):
        with self._lock:
            buf, self._buf = self._buf, []
            wbuf, self._wbuf = self._wbuf, []
            self._scheduled = False
        if wbuf:
            self.webhook.enqueue(wbuf)
        if not buf:
            return
        data = "\n".join(buf) + "\n"
        if self.f is not None:
            if self.max_size and self.f.tell() + len(data) > self.max_size and self.f.tell() > 0:
                self._rotate()
            self.f.write(data)
            self.f.flush()
        elif self.stdout:
            os.write(1, data.encode())

    def _rotate(self):
        import glob
        import time as _time
        self.f.close()
        base, ext = os.path.splitext(self.path)
        stamp = _time.strftime("%Y-%m-%dT%H-%M-%S", _time.gmtime()) + f".{int(_time.time() * 1000) % 1000:03d}"
        os.replace(self.path, f"{base}-{stamp}{ext}")
        backups = sorted(glob.glob(f"{glob.escape(base)}-*{ext}"), key=os.path.getmtime, reverse=True)
        now = _time.time()
        for i, b in enumerate(backups):
            if (self.max_backups and i >= self.max_backups) or (self.max_age and now - os.path.getmtime(b) > self.max_age):
                try:
                    os.unlink(b)
                except OSError:
                    pass
        self.f = open(self.path, "a", buffering=1 << 16)

    def close(self):
        self.flush()
        if self.f is not None:
            self.f.close()
            self.f = None
        if self.webhook is not None:
            self.webhook.close()


class WebhookBackend:
    """Audit webhook (`staging/src/k8s.io/apiserver/plugin/pkg/audit/webhook/webhook.go`,
    `--audit-webhook-config-file` kubeconfig naming the remote server).

    mode "batch": events are buffered (`buffer`, 10 000) and POSTed as an `audit.k8s.io/v1beta1`
    EventList in batches of up to `max_batch`, at least every `max_wait` seconds, from a
    background thread so request handling never blocks; batches are throttled to `throttle_qps`
    per second with bursts of `throttle_burst` (0 = unthrottled); a failed batch is retried with
    exponential backoff from `initial_backoff`, then dropped.
    mode "blocking": every request's event is POSTed before its response is sent."""

    def __init__(self, kubeconfig, max_batch=400, max_wait=1.0, buffer=10000, retries=3, mode="batch",
                 throttle_qps=0.0, throttle_burst=0, initial_backoff=0.1):
        if mode not in ("batch", "blocking"):
            raise ValueError(f"unknown audit webhook mode {mode!r}")
        from ..client import clientcmd
        cfg, p = clientcmd.load(kubeconfig)
        r = clientcmd.resolve(cfg, None, os.path.dirname(os.path.abspath(p)))
        if r is None:
            raise ValueError(f"audit webhook kubeconfig {kubeconfig}: no usable context")
        self.url, self.token, self.ssl = r.server, r.token, r.ssl_context
        self.max_batch, self.max_wait, self.buffer, self.retries = max_batch, max_wait, buffer, retries
        self.blocking = mode == "blocking"
        self.initial_backoff = initial_backoff
        self.qps, self.burst = float(throttle_qps or 0), max(1, int(throttle_burst or 1))
        self._tokens, self._last = float(self.burst), time.monotonic()
        self._q = []
        self._cv = threading.Condition()
        self._closed = False
        self.sent = self.dropped = self.posts = 0
        self._t = None
        if not self.blocking:
            self._t = threading.Thread(target=self._run, name="audit-webhook", daemon=True)
            self._t.start()

    def _throttle(self):
        """Token bucket over batch POSTs (`--audit-webhook-batch-throttle-qps/-burst`)."""
        if self.qps <= 0:
            return
        now = time.monotonic()
        self._tokens = min(float(self.burst), self._tokens + (now - self._last) * self.qps)
        self._last = now
        if self._tokens < 1.0:
            time.sleep((1.0 - self._tokens) / self.qps)
            self._tokens = 0.0
            self._last = time.monotonic()
        else:
            self._tokens -= 1.0

    def post_now(self, lines):
        self._post(lines)

    def enqueue(self, lines):
        with self._cv:
            room = self.buffer - len(self._q)
            if room < len(lines):
                self.dropped += len(lines) - max(room, 0)
                lines = lines[:max(room, 0)]
            self._q.extend(lines)
            if len(self._q) >= self.max_batch:
                self._cv.notify()

    def _post(self, batch):
        import urllib.request
        body = ('{"kind":"EventList","apiVersion":"audit.k8s.io/v1beta1","metadata":{},"items":[' +
                ",".join(batch) + "]}").encode()
        hdr = {"Content-Type": "application/json"}
        if self.token:
            hdr["Authorization"] = f"Bearer {self.token}"
        delay = self.initial_backoff
        for _ in range(self.retries):
            try:
                req = urllib.request.Request(self.url, data=body, headers=hdr, method="POST")
                with urllib.request.urlopen(req, timeout=10, context=self.ssl) as r:
                    r.read()
                self.sent += len(batch)
                self.posts += 1
                return
            except OSError:
                time.sleep(delay)
                delay *= 2
        self.dropped += len(batch)

    def _run(self):
        while True:
            with self._cv:
                if not self._q and not self._closed:
                    self._cv.wait(self.max_wait)
                batch, self._q = self._q[:self.max_batch], self._q[self.max_batch:]
                done = self._closed and not self._q
            if batch:
                self._throttle()
                self._post(batch)
            if done:
                return

    def close(self, timeout=10.0):
        with self._cv:
            self._closed = True
            self._cv.notify()
        if self._t is not None:
            self._t.join(timeout)


def now():
    return time.time()
