"""Docker image references (`github.com/docker/distribution/reference` as used by the kubelet's
`pkg/kubelet/dockershim/libdocker` and `pkg/util/parsers/parsers.go` ParseImageName):

    [registry[:port]/]repository[:tag][@sha256:digest]

The registry is the first component when it contains "." or ":" or is "localhost"; otherwise the
image is on Docker Hub (`docker.io`, and one-component names live under `library/`). The tag
defaults to `latest` when there is no digest.
"""
from __future__ import annotations

import re

DEFAULT_REGISTRY = "docker.io"
DOCKER_HUB_API = "registry-1.docker.io"
_COMPONENT = re.compile(r"^[a-z0-9]+(?:(?:[._]|__|-+)[a-z0-9]+)*$")
_TAG = re.compile(r"^[\w][\w.-]{0,127}$")
_DIGEST = re.compile(r"^[a-z0-9]+(?:[.+_-][a-z0-9]+)*:[a-fA-F0-9]{32,}$")


class InvalidReference(ValueError):
    pass


class Reference:
    __slots__ = ("registry", "repository", "tag", "digest")

    def __init__(self, registry, repository, tag=None, digest=None):
        self.registry, self.repository, self.tag, self.digest = registry, repository, tag, digest

    @property
    def name(self) -> str:
        """Fully qualified repository name: registry/repository."""
        return f"{self.registry}/{self.repository}"

    @property
    def api_host(self) -> str:
        return DOCKER_HUB_API if self.registry == DEFAULT_REGISTRY else self.registry

    def tagged(self) -> str:
        return f"{self.name}:{self.tag or 'latest'}"

    def __str__(self):
        s = self.name
        if self.tag:
            s += ":" + self.tag
        if self.digest:
            s += "@" + self.digest
        return s

    def familiar(self) -> str:
        """The short form users write (`busybox:1.28`, `amd/rocm:6`), as repo tags are shown."""
        name = self.name
        if self.registry == DEFAULT_REGISTRY:
            name = self.repository[len("library/"):] if self.repository.startswith("library/") else self.repository
        return f"{name}:{self.tag or 'latest'}"


def parse(ref: str) -> Reference:
    if not ref or ref != ref.strip():
        raise InvalidReference(f"invalid reference format: {ref!r}")
    rest, digest = ref, None
    if "@" in rest:
        rest, digest = rest.split("@", 1)
        if not _DIGEST.match(digest):
            raise InvalidReference(f"invalid digest in {ref!r}")
    tag = None
    slash = rest.rfind("/")
    colon = rest.rfind(":")
    if colon > slash:
        rest, tag = rest[:colon], rest[colon + 1:]
        if not _TAG.match(tag):
            raise InvalidReference(f"invalid tag in {ref!r}")
    parts = rest.split("/")
    if len(parts) > 1 and ("." in parts[0] or ":" in parts[0] or parts[0] == "localhost"):
        registry, repo_parts = parts[0], parts[1:]
    else:
        registry, repo_parts = DEFAULT_REGISTRY, parts
    if registry in ("index.docker.io", "registry-1.docker.io"):
        registry = DEFAULT_REGISTRY
    if registry == DEFAULT_REGISTRY and len(repo_parts) == 1:
        repo_parts = ["library"] + repo_parts
    for c in repo_parts:
        if not _COMPONENT.match(c):
            raise InvalidReference(f"invalid reference format: repository name must be lowercase: {ref!r}")
    if tag is None and digest is None:
        tag = "latest"
    return Reference(registry, "/".join(repo_parts), tag, digest)


def normalize(ref: str) -> str:
    """Canonical `registry/repo:tag` (or `@digest`) string used as the store's key."""
    r = parse(ref)
    return f"{r.name}@{r.digest}" if r.digest and not r.tag else (
        f"{r.name}:{r.tag}@{r.digest}" if r.digest else r.tagged())
