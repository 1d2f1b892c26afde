"""HTTP scheduler extenders.

Parity: `plugin/pkg/scheduler/core/extender.go` (`HTTPExtender`: `Filter` POSTs ExtenderArgs
{pod, nodes | nodenames} to `<urlPrefix>/<filterVerb>` and gets ExtenderFilterResult {nodes |
nodenames, failedNodes, error}; `Prioritize` gets a HostPriorityList whose scores are multiplied
by `weight`; `IsInterested` via `managedResources`; `ignorable`; `Bind` / `IsBinder`, :198-223)
and the Policy config `plugin/pkg/scheduler/api/types.go:129` (`ExtenderConfig`, `BindVerb`).

Calls are synchronous with a timeout, like the reference's (the scheduling loop is serial);
the scheduler runs `bind` off the event loop. A binder extender takes over writing the binding
(`factory.go:886` getBinder): ExtenderBindingArgs keeps the reference's untagged Go field names
(`PodName`, `PodNamespace`, `PodUID`, `Node`) and, GPU-aware, adds `ExtendedResourceBindings` —
the device IDs the scheduler allocated — so the extender can write a complete binding.
"""
from __future__ import annotations

import http.client
import json
import logging
from urllib.parse import urlparse

from ..api import core

log = logging.getLogger("scheduler.extender")


class ExtenderError(Exception):
    pass


class HTTPExtender:
    def __init__(self, url_prefix, filter_verb="", prioritize_verb="", weight=1, http_timeout=5.0,
                 node_cache_capable=False, managed_resources=None, ignorable=False, bind_verb=""):
        u = urlparse(url_prefix)
        self.host, self.port = u.hostname or "127.0.0.1", u.port or (443 if u.scheme == "https" else 80)
        self.https = u.scheme == "https"
        self.base = u.path.rstrip("/")
        self.filter_verb, self.prioritize_verb = filter_verb, prioritize_verb
        self.weight = weight
        self.timeout = http_timeout
        self.node_cache_capable = node_cache_capable
        self.managed = {m["name"] if isinstance(m, dict) else m for m in (managed_resources or ())}
        self.ignorable = ignorable
        self.bind_verb = bind_verb

    @classmethod
    def from_config(cls, cfg: dict):
        to = cfg.get("httpTimeout")
        if isinstance(to, (int, float)) and to > 1000:   # Go duration in ns
            to = to / 1e9
        return cls(cfg["urlPrefix"], cfg.get("filterVerb", ""), cfg.get("prioritizeVerb", ""),
                   int(cfg.get("weight", 1)), float(to or 5.0), bool(cfg.get("nodeCacheCapable")),
                   cfg.get("managedResources"), bool(cfg.get("ignorable")),
                   cfg.get("bindVerb") or cfg.get("BindVerb") or "")

    def is_binder(self) -> bool:
        return bool(self.bind_verb)

    def bind(self, namespace, name, uid, node, erb=None):
        """Delegate the binding (extender.go:198 Bind); raises ExtenderError on failure."""
        if not self.is_binder():
            raise ExtenderError("Unexpected empty bindVerb in extender")
        args = {"PodName": name, "PodNamespace": namespace, "PodUID": uid or "", "Node": node}
        if erb:
            args["ExtendedResourceBindings"] = erb
        res = self._post(self.bind_verb, args) or {}
        err = res.get("Error") or res.get("error")
        if err:
            raise ExtenderError(err)

    def is_interested(self, pod) -> bool:
        if not self.managed:
            return True
        spec = pod.get("spec") or {}
        for c in (spec.get("containers") or []) + (spec.get("initContainers") or []):
            res = c.get("resources") or {}
            if self.managed & (set(res.get("limits") or {}) | set(res.get("requests") or {})):
                return True
        for per in spec.get("extendedResources") or ():
            try:
                if core.pod_extended_resource_name(per) in self.managed:
                    return True
            except ValueError:
                pass
        return False

    def _post(self, verb, body):
        cls = http.client.HTTPSConnection if self.https else http.client.HTTPConnection
        conn = cls(self.host, self.port, timeout=self.timeout)
        try:
            conn.request("POST", f"{self.base}/{verb}", json.dumps(body), {"Content-Type": "application/json"})
            r = conn.getresponse()
            data = r.read()
            if r.status != 200:
                raise ExtenderError(f"extender {verb}: HTTP {r.status}")
            return json.loads(data)
        except (OSError, ValueError) as e:
            raise ExtenderError(f"extender {verb}: {e}") from e
        finally:
            conn.close()

    def _args(self, pod, nodes):
        if self.node_cache_capable:
            return {"pod": pod, "nodenames": [n.name for n in nodes]}
        return {"pod": pod, "nodes": {"items": [n.node for n in nodes]}}

    def filter(self, pod, nodes):
        """Returns (kept NodeInfos, {node: reason})."""
        if not self.filter_verb or not self.is_interested(pod):
            return nodes, {}
        try:
            res = self._post(self.filter_verb, self._args(pod, nodes))
        except ExtenderError:
            if self.ignorable:
                log.warning("ignorable extender failed; skipping", exc_info=True)
                return nodes, {}
            raise
        if res.get("error"):
            raise ExtenderError(res["error"])
        if res.get("nodenames") is not None:
            keep = set(res["nodenames"])
        else:
            keep = {n["metadata"]["name"] for n in ((res.get("nodes") or {}).get("items") or [])}
        failed = dict(res.get("failedNodes") or {})
        return [n for n in nodes if n.name in keep], failed

    def prioritize(self, pod, nodes):
        """Returns {node: weighted score}."""
        if not self.prioritize_verb or not self.is_interested(pod):
            return {}
        try:
            res = self._post(self.prioritize_verb, self._args(pod, nodes))
        except ExtenderError:
            log.warning("extender prioritize failed; ignoring its scores", exc_info=True)
            return {}
        return {h["host"]: int(h.get("score", 0)) * self.weight for h in res or ()}
