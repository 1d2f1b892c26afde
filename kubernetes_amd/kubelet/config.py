"""Static pods from a manifest directory, mirrored into the API.

Parity: `pkg/kubelet/config/file.go` (poll `--pod-manifest-path` every 20 s; JSON or YAML pod
manifests; the pod name gets `-<nodeName>`, namespace defaults to `default`, a hash of the
manifest identifies the version) and `pkg/kubelet/pod/mirror_client.go` (a mirror pod with the
`kubernetes.io/config.mirror` annotation represents the static pod in the API; it is re-created
when deleted and replaced when the manifest changes; removing the file deletes it).

Here the mirror pod is also how the pod is run: it is created bound to this node
(`spec.nodeName`), so the kubelet's normal informer path admits and starts it.
"""
from __future__ import annotations

import asyncio
import hashlib
import json
import logging
import os

from ..client.rest import APIStatusError

log = logging.getLogger("kubelet.config")

CONFIG_SOURCE = "kubernetes.io/config.source"
CONFIG_HASH = "kubernetes.io/config.hash"
CONFIG_MIRROR = "kubernetes.io/config.mirror"


def load_manifests(path):
    out = []
    if not path or not os.path.isdir(path):
        return out
    for fn in sorted(os.listdir(path)):
        if fn.startswith(".") or not fn.endswith((".json", ".yaml", ".yml")):
            continue
        full = os.path.join(path, fn)
        try:
            with open(full) as f:
                text = f.read()
            if fn.endswith(".json"):
                doc = json.loads(text)
            else:
                import yaml
                doc = yaml.load(text, Loader=yaml.SafeLoader)
        except (OSError, ValueError, Exception) as e:   # a bad file must not stop the others
            log.warning("static pod manifest %s: %s", full, e)
            continue
        if isinstance(doc, dict) and doc.get("kind", "Pod") == "Pod":
            out.append((full, doc, hashlib.sha256(text.encode()).hexdigest()[:16]))
    return out


def parse_manifest_text(text, origin):
    """One pod, or a List / v1 PodList of pods, in JSON or YAML."""
    import yaml
    try:
        doc = json.loads(text) if text.lstrip().startswith("{") else yaml.load(text, Loader=yaml.SafeLoader)
    except (ValueError, yaml.YAMLError) as e:
        log.warning("pod manifest from %s: %s", origin, e)
        return []
    docs = doc.get("items") or [] if isinstance(doc, dict) and doc.get("kind", "").endswith("List") else [doc]
    return [(origin, d, hashlib.sha256(json.dumps(d, sort_keys=True).encode()).hexdigest()[:16])
            for d in docs if isinstance(d, dict) and d.get("kind", "Pod") == "Pod"]


def load_url(url, headers=None, timeout=10.0):
    """`pkg/kubelet/config/http.go`: GET --manifest-url (with --manifest-url-header) every poll."""
    import urllib.request
    req = urllib.request.Request(url, headers=dict(headers or {}))
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return parse_manifest_text(r.read().decode(), url)


class StaticPodSource:
    def __init__(self, kubelet, path, period=20.0, url=None, url_headers=None):
        self.kl = kubelet
        self.path = path
        self.url, self.url_headers = url, url_headers
        self.period = period
        self.known: dict[tuple, str] = {}     # (ns, name) -> hash
        self._task = None
        self._stopped = False

    def start(self):
        self._stopped = False
        self._task = asyncio.ensure_future(self._loop())

    def stop(self):
        # the flag as well as the cancel: a cancellation that lands inside an HTTP call can be
        # turned into an ordinary error by the client, which the loop below would survive
        self._stopped = True
        if self._task:
            self._task.cancel()

    async def _loop(self):
        while not self._stopped:
            try:
                await self.sync()
            except Exception:
                if self._stopped:
                    return
                log.exception("static pod sync failed")
            await asyncio.sleep(self.period)

    def _mirror(self, doc, h, source="file"):
        pod = json.loads(json.dumps(doc))
        md = pod.setdefault("metadata", {})
        # common.go applyDefaults: generatePodName (lower-cased node name), namespace default
        md["name"] = f"{md.get('name', 'static')}-{str(self.kl.node_name).lower()}"
        if not md.get("namespace"):
            md["namespace"] = "default"
        ann = md.setdefault("annotations", {})
        ann.update({CONFIG_SOURCE: source, CONFIG_HASH: h, CONFIG_MIRROR: h})
        for k in ("uid", "resourceVersion", "creationTimestamp"):
            md.pop(k, None)
        pod.setdefault("spec", {})["nodeName"] = self.kl.node_name
        if source == "file":
            # static pods from files tolerate every NoExecute taint, so node problems do not
            # evict them (AddOrUpdateTolerationInPod)
            tols = pod["spec"].setdefault("tolerations", [])
            want = {"operator": "Exists", "effect": "NoExecute"}
            if not any(t.get("operator") == "Exists" and t.get("effect") == "NoExecute" and not t.get("key")
                       for t in tols):
                tols.append(want)
        pod.pop("status", None)
        pod["apiVersion"], pod["kind"] = "v1", "Pod"
        return pod

    async def _sources(self):
        out = [(d, h, "file") for _, d, h in load_manifests(self.path)] if self.path else []
        if self.url:
            try:
                got = await asyncio.get_running_loop().run_in_executor(None, load_url, self.url, self.url_headers)
            except OSError as e:
                log.warning("manifest url %s: %s", self.url, e)
                # an unreachable URL keeps the pods it last served (http.go only replaces on success)
                return out, True
            out += [(d, h, "http") for _, d, h in got]
        return out, False

    async def sync(self):
        c = self.kl.client
        seen = set()
        sources, url_failed = await self._sources()
        for doc, h, src in sources:
            pod = self._mirror(doc, h, src)
            key = (pod["metadata"]["namespace"], pod["metadata"]["name"])
            seen.add(key)
            try:
                cur = await c.get("pods", key[1], key[0])
            except APIStatusError as e:
                if e.code != 404:
                    raise
                cur = None
            if cur is not None and ((cur["metadata"].get("annotations") or {}).get(CONFIG_MIRROR) != h
                                    or cur["metadata"].get("deletionTimestamp")):
                if not cur["metadata"].get("deletionTimestamp"):
                    await c.delete("pods", key[1], key[0], grace_period=0)
                continue     # re-created on the next pass once gone
            if cur is None:
                try:
                    await c.create("pods", pod, key[0])
                except APIStatusError as e:
                    if e.code != 409:
                        log.warning("creating mirror pod %s/%s: %s", key[0], key[1], e)
            self.known[key] = h
        for key in [k for k in self.known if k not in seen]:
            if url_failed:
                continue
            self.known.pop(key)
            try:
                await c.delete("pods", key[1], key[0], grace_period=0)
            except APIStatusError as e:
                if e.code != 404:
                    log.warning("deleting mirror pod %s/%s: %s", key[0], key[1], e)
