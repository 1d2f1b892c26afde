"""Checksummed JSON checkpoints.

Parity: `pkg/kubelet/util/store` + `pkg/kubelet/dockershim/docker_checkpoint.go:89-148`
(`PodSandboxCheckpoint{Version, Name, Namespace, Data{PortMappings, HostNetwork}, CheckSum}`:
the checksum covers the object with CheckSum zeroed; a corrupt file is reported and removed)
and `pkg/kubelet/checkpoint/checkpoint.go:67-145` (bootstrap pod checkpoints). Writes are
atomic (temp file + rename), keys are file names.
"""
from __future__ import annotations

import hashlib
import json
import os
import re

_KEY = re.compile(r"^[A-Za-z0-9._-]+$")


class CorruptCheckpoint(ValueError):
    pass


def _checksum(obj):
    body = dict(obj, checksum=0)
    return int(hashlib.sha256(json.dumps(body, sort_keys=True, separators=(",", ":")).encode()).hexdigest()[:8], 16)


class CheckpointManager:
    def __init__(self, root):
        self.root = root
        os.makedirs(root, exist_ok=True)

    def _path(self, key):
        if not _KEY.match(key):
            raise ValueError(f"invalid checkpoint key {key!r}")
        return os.path.join(self.root, key)

    def create(self, key, obj):
        obj = dict(obj)
        obj["checksum"] = _checksum(obj)
        p = self._path(key)
        tmp = p + ".tmp"
        with open(tmp, "w") as f:
            json.dump(obj, f, sort_keys=True)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, p)

    def get(self, key):
        p = self._path(key)
        with open(p) as f:
            try:
                obj = json.load(f)
            except ValueError as e:
                raise CorruptCheckpoint(f"checkpoint {key}: {e}")
        if obj.get("checksum") != _checksum(obj):
            raise CorruptCheckpoint(f"checkpoint {key} is corrupted (checksum mismatch)")
        obj.pop("checksum", None)
        return obj

    def remove(self, key):
        try:
            os.unlink(self._path(key))
        except FileNotFoundError:
            pass

    def list(self):
        return sorted(k for k in os.listdir(self.root) if _KEY.match(k) and not k.endswith(".tmp"))

    def load_all(self):
        """(key, obj) for every valid checkpoint; corrupt ones are removed (reference behaviour)."""
        out = []
        for k in self.list():
            try:
                out.append((k, self.get(k)))
            except (CorruptCheckpoint, OSError):
                self.remove(k)
        return out
