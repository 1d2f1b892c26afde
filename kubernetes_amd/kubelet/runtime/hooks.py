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

import json
import logging
import os

log = logging.getLogger("hooks")

HOOKS_DIR = "/usr/share/containers/kubernetes-amd/hooks.d"


class HookService:
    def __init__(self, hooks_dir=HOOKS_DIR, available_runtimes=("process", "stub")):
        self.dir = hooks_dir
        self.available = set(available_runtimes)
        self.hooks: dict[str, dict] = {}

    def load(self):
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
