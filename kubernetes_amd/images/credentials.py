"""Pull-secret keyrings (`pkg/credentialprovider/keyring.go`, `config.go`): the kubelet turns a
pod's `imagePullSecrets` (types `kubernetes.io/dockerconfigjson` and legacy
`kubernetes.io/dockercfg`) into a keyring and looks up the credentials for an image:

  * keys are registry URLs (`https://index.docker.io/v1/`, `registry.local:5000`,
    `gcr.io/project`), normalised to host + path; Docker Hub keys match `docker.io` images;
  * a key matches when its host matches the image's registry (labels may be `*` globs, as in
    `*.example.com`, port must match) and its path is a prefix of the repository;
  * more specific keys (longer) come first; the kubelet tries each matching credential in turn.
"""
from __future__ import annotations

import base64
import fnmatch
import json

from . import reference
from .registry import Auth

DOCKER_HUB_KEYS = ("index.docker.io", "docker.io", "registry-1.docker.io")


def _split_key(key: str):
    k = key.split("://", 1)[-1].rstrip("/")
    host, _, path = k.partition("/")
    if host in DOCKER_HUB_KEYS:
        host = reference.DEFAULT_REGISTRY
        if path in ("v1", "v2"):
            path = ""
    return host, path


def _host_matches(pattern: str, host: str) -> bool:
    ph, _, pport = pattern.partition(":")
    hh, _, hport = host.partition(":")
    if pport != hport:
        return False
    pl, hl = ph.split("."), hh.split(".")
    return len(pl) == len(hl) and all(fnmatch.fnmatchcase(h, p) for p, h in zip(pl, hl))


class Keyring:
    def __init__(self):
        self.entries: list[tuple[str, str, Auth]] = []   # (host pattern, path prefix, auth)

    def add(self, key: str, cred: dict):
        host, path = _split_key(key)
        self.entries.append((host, path, Auth(cred.get("username", ""), cred.get("password", ""),
                                              cred.get("auth", ""), cred.get("identitytoken", ""),
                                              cred.get("registrytoken", ""))))
        self.entries.sort(key=lambda e: len(e[0]) + len(e[1]), reverse=True)

    def lookup(self, image: str) -> list[Auth]:
        ref = reference.parse(image)
        out = []
        for host, path, auth in self.entries:
            if _host_matches(host, ref.registry) and (not path or ref.repository == path
                                                       or ref.repository.startswith(path + "/")):
                out.append(auth)
        return out


def keyring_from_secrets(secrets) -> Keyring:
    """Secrets as API objects (data base64-encoded)."""
    kr = Keyring()
    for s in secrets:
        data = s.get("data") or {}
        try:
            if ".dockerconfigjson" in data:
                cfg = json.loads(base64.b64decode(data[".dockerconfigjson"]))
                auths = cfg.get("auths") or {}
            elif ".dockercfg" in data:
                auths = json.loads(base64.b64decode(data[".dockercfg"]))
            else:
                continue
        except (ValueError, TypeError):
            continue
        for key, cred in auths.items():
            if isinstance(cred, dict):
                kr.add(key, cred)
    return kr
