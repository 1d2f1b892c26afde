"""Runtime hook service: choose the low-level runtime per container.

Parity (fork F11): `pkg/kubelet/dockershim/docker_hooks.go:38-264` — JSON hooks in a directory,
each `{"runtime": "...", "annotations": {k: v}, "images": ["prefix", ...]}`; a hook is valid
only if its runtime is installed; on container creation the first hook whose annotation
matches the container's annotations, or whose image prefix matches the image, selects the
runtime. The reference used this to route GPU containers to nvidia-container-runtime; on
MI355X no vendor runtime exists, so the default hook set is EMPTY and GPU containers run on
the default runtime with devices injected by the kubelet (`runtime/oci.py`). The service is
kept as a generic annotation/image → runtime selector (e.g. to pick a sandboxed runtime).
"""
from __future__ import annotations

import asyncio
import json
import logging
import os

from .base import Runtime

log = logging.getLogger("hooks")

HOOKS_DIR = "/usr/share/containers/kubernetes-amd/hooks.d"


class HookService:
    def __init__(self, hooks_dir=HOOKS_DIR, available_runtimes=("process", "stub")):
        self.dir = hooks_dir
        self.available = set(available_runtimes)
        self.hooks: dict[str, dict] = {}

    def load(self):
        self._loaded = self._snapshot()      # what the hook set reflects (watch() compares to it)
        self.hooks.clear()
        if not os.path.isdir(self.dir):
            return self
        for f in sorted(os.listdir(self.dir)):
            if not f.endswith(".json"):
                continue
            h = self.read_hook(os.path.join(self.dir, f))
            if h is not None and self.is_valid(h):
                self.hooks[f] = h
        return self

    @staticmethod
    def read_hook(path):
        try:
            with open(path) as fh:
                h = json.load(fh)
        except (OSError, ValueError) as e:
            log.warning("invalid hook %s: %s", path, e)
            return None
        if not isinstance(h, dict) or not h.get("runtime"):
            return None
        h.setdefault("annotations", {})
        h.setdefault("images", [])
        return h

    def _snapshot(self):
        try:
            return sorted((f, os.stat(os.path.join(self.dir, f)).st_mtime_ns) for f in os.listdir(self.dir)
                          if f.endswith(".json"))
        except OSError:
            return []

    async def watch(self, period=1.0):
        """fsnotify equivalent (`docker_hooks.go` Start: Create/Write/Remove events reload the
        hooks): the directory is re-scanned when its JSON files or their mtimes change."""
        while True:
            await asyncio.sleep(period)
            if self._snapshot() != getattr(self, "_loaded", None):
                self.load()
                log.info("hooks reloaded: %s", {k: v["runtime"] for k, v in self.hooks.items()})

    def is_valid(self, h):
        return h["runtime"] in self.available

    def get_runtime(self, image: str, annotations: dict, repo_tags=()) -> str | None:
        tags = list(repo_tags) or [image]
        for _, h in sorted(self.hooks.items()):
            for k, v in h["annotations"].items():
                if annotations.get(k) == v:
                    return h["runtime"]
            for prefix in h["images"]:
                if any(t.startswith(prefix) for t in tags):
                    return h["runtime"]
        return None


class HookedRuntime(Runtime):
    """The dockershim side of F11: several low-level runtimes behind one CRI runtime, the hook
    service picking one per container (`docker_container.go:116-133` sets HostConfig.Runtime).
    Sandboxes start in the default runtime; a container routed elsewhere gets a companion
    sandbox there (created on first use), and every later call for it goes to that runtime."""

    def __init__(self, runtimes: dict, default: str, hooks: HookService):
        super().__init__()
        self.runtimes = runtimes
        self.default = default
        self.hooks = hooks
        self.name = runtimes[default].name
        self.sandboxes: dict[str, dict] = {}      # sid -> {runtime name: sid in that runtime}
        self.owner: dict[str, str] = {}           # container id -> runtime name
        self.chosen: dict[str, str] = {}          # container id -> runtime chosen by a hook (audit)
        self.images = getattr(runtimes[default], "images", None)
        for rt in runtimes.values():
            rt.on_exit(self._fire_exit)

    def _rt(self, cid):
        return self.runtimes[self.owner.get(cid, self.default)]

    async def version(self):
        return await self.runtimes[self.default].version()

    async def run_pod_sandbox(self, pod, annotations):
        sid = await self.runtimes[self.default].run_pod_sandbox(pod, annotations)
        self.sandboxes[sid] = {self.default: sid, "_pod": pod, "_ann": dict(annotations or {})}
        return sid

    async def stop_pod_sandbox(self, sid):
        for name, sub in list((self.sandboxes.get(sid) or {self.default: sid}).items()):
            if not name.startswith("_"):
                await self.runtimes[name].stop_pod_sandbox(sub)

    async def remove_pod_sandbox(self, sid):
        for name, sub in list((self.sandboxes.pop(sid, None) or {self.default: sid}).items()):
            if not name.startswith("_"):
                await self.runtimes[name].remove_pod_sandbox(sub)

    async def create_container(self, sid, pod, container, opts):
        ann = {a["name"]: a["value"] for a in opts.annotations}
        name = self.hooks.get_runtime(container.get("image", ""), ann) or self.default
        if name not in self.runtimes:
            name = self.default
        sb = self.sandboxes.setdefault(sid, {self.default: sid, "_pod": pod, "_ann": {}})
        if name not in sb:
            sb[name] = await self.runtimes[name].run_pod_sandbox(sb["_pod"], sb["_ann"])
        cid = await self.runtimes[name].create_container(sb[name], pod, container, opts)
        self.owner[cid] = name
        if name != self.default:
            self.chosen[cid] = name
        return cid

    async def start_container(self, cid):
        await self._rt(cid).start_container(cid)

    async def stop_container(self, cid, timeout):
        await self._rt(cid).stop_container(cid, timeout)

    async def remove_container(self, cid):
        await self._rt(cid).remove_container(cid)
        self.owner.pop(cid, None)
        self.chosen.pop(cid, None)

    def container_status(self, cid):
        return self._rt(cid).container_status(cid)

    async def container_logs(self, cid, tail=None):
        return await self._rt(cid).container_logs(cid, tail)

    def log_path(self, cid):
        rt = self._rt(cid)
        return rt.log_path(cid) if hasattr(rt, "log_path") else None

    async def exec_sync(self, cid, cmd, timeout):
        return await self._rt(cid).exec_sync(cid, cmd, timeout)

    async def exec_interactive(self, cid, cmd, stdin, stdout, stderr, tty, resize):
        return await self._rt(cid).exec_interactive(cid, cmd, stdin, stdout, stderr, tty, resize)

    async def attach(self, cid, stdin, stdout, stderr, tty, resize):
        return await self._rt(cid).attach(cid, stdin, stdout, stderr, tty, resize)

    def list_containers(self):
        return [c for rt in self.runtimes.values() for c in rt.list_containers()]

    def container_pids(self):
        out = {}
        for rt in self.runtimes.values():
            out.update(rt.container_pids())
        return out

    def isolation_status(self):
        return self.runtimes[self.default].isolation_status()
