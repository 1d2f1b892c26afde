"""The node's image service (CRI ImageService semantics: PullImage / ImageStatus / ListImages /
RemoveImage / ImageFsInfo) over three sources, most specific first:

  1. the OCI store (`store.py`) — images pulled from a registry or imported from an OCI layout;
  2. built-in images — the framework's own workloads (`kubernetes-amd/hip-vector-add`, …) that
     resolve to binaries built in this tree (`cri/server.ImageStore` with a resolver);
  3. a registry pull (`registry.py`), when the service has a registry client.

Container creation asks `image_config(image)` (the OCI config: Entrypoint, Cmd, Env, WorkingDir,
User) and `rootfs(image)` (the unpacked layers an overlay is built on). `command_for` applies the
Kubernetes command/args rules over the image's entrypoint (`pkg/kubelet/kuberuntime` +
dockershim's Entrypoint=command, Cmd=args: a `command` replaces both the image ENTRYPOINT and
CMD, `args` alone replace only CMD).
"""
from __future__ import annotations

import os

from . import reference
from .registry import Auth, RegistryClient
from .store import OCIStore, secure_join


class ImageService:
    def __init__(self, store: OCIStore | None = None, builtins=None, registry: RegistryClient | None = None):
        self.store, self.builtins, self.registry = store, builtins, registry

    def _oci(self, image):
        if self.store is None:
            return None
        try:
            return self.store.image(image)
        except (reference.InvalidReference, OSError, ValueError, KeyError):
            return None

    async def pull_image(self, image, auth: Auth | None = None):
        if self.registry is not None and self.store is not None and not self._builtin(image):
            await self.registry.pull(image, self.store, auth)
            return self.store.image(image)["id"]
        img = self._oci(image)
        if img is not None:
            return img["id"]
        if self.builtins is not None:
            try:
                return self.builtins.pull(image)
            except LookupError as e:
                from ..kubelet.runtime.base import RuntimeError_
                raise RuntimeError_(str(e)) from None
        from ..kubelet.runtime.base import RuntimeError_
        raise RuntimeError_(f"pull access denied for {image}: no registry configured")

    def _builtin(self, image) -> bool:
        if self.builtins is None:
            return False
        from ..kubelet.runtime.process import builtin_argv
        return builtin_argv(self.builtins.normalize(image).rsplit(":", 1)[0]) is not None

    async def image_status(self, image):
        img = self._oci(image)
        if img is not None:
            return {"id": img["id"], "repoTags": img["repo_tags"], "repoDigests": img["repo_digests"], "size": img["size"]}
        if self.builtins is not None:
            i = self.builtins.status(image)
            if i is not None:
                return {"id": i["id"], "repoTags": list(i["repo_tags"]), "size": i["size"]}
        return None

    async def list_images(self):
        out = []
        if self.store is not None:
            out += [{"id": i["id"], "repoTags": i["repo_tags"], "repoDigests": i["repo_digests"], "size": i["size"]}
                    for i in self.store.images()]
        if self.builtins is not None:
            out += [{"id": i["id"], "repoTags": list(i["repo_tags"]), "size": i["size"]}
                    for i in self.builtins.images.values()]
        return out

    async def remove_image(self, image):
        if self.store is not None and self._oci(image) is not None:
            self.store.remove(image)
        elif self.builtins is not None:
            self.builtins.remove(image)

    async def image_fs_info(self):
        used = (self.store.used_bytes() if self.store is not None else 0) + \
            (self.builtins.used_bytes() if self.builtins is not None else 0)
        n = (len(self.store.images()) if self.store is not None else 0) + \
            (len(self.builtins.images) if self.builtins is not None else 0)
        return {"usedBytes": used, "inodesUsed": n}

    # -- container creation helpers ----------------------------------------------------------------
    def image_config(self, image) -> dict | None:
        img = self._oci(image)
        return None if img is None else (img["config"].get("config") or {})

    def rootfs(self, image) -> str | None:
        if self._oci(image) is None:
            return None
        return self.store.rootfs(image)


def command_for(container, cfg) -> list:
    """Entrypoint/command resolution (Kubernetes `command`/`args` over ENTRYPOINT/CMD)."""
    cmd = list(container.get("command") or [])
    args = list(container.get("args") or [])
    if cmd:
        return cmd + args
    ep = list(cfg.get("Entrypoint") or [])
    return ep + (args if args else list(cfg.get("Cmd") or []))


def env_for(cfg, base: dict) -> dict:
    """Image ENV under the container's own variables (the container wins)."""
    env = {}
    for kv in cfg.get("Env") or ():
        k, _, v = kv.partition("=")
        env[k] = v
    env.update(base)
    return env


def user_for(cfg, rootfs: str | None):
    """The image USER as (uid, gid) or None: numeric `uid[:gid]`, or names looked up in the
    image's /etc/passwd and /etc/group."""
    u = (cfg.get("User") or "").strip()
    if not u:
        return None
    name, _, group = u.partition(":")

    def lookup(path, key):
        if rootfs is None:
            return None
        try:
            with open(secure_join(rootfs, path)) as f:
                for ln in f:
                    parts = ln.strip().split(":")
                    if parts and parts[0] == key and len(parts) > 3:
                        return parts
        except OSError:
            return None
        return None
    if name.isdigit():
        uid, gid = int(name), 0
    else:
        pw = lookup("/etc/passwd", name)
        if pw is None:
            raise ValueError(f"unable to find user {name} in the image")
        uid, gid = int(pw[2]), int(pw[3])
    if group:
        if group.isdigit():
            gid = int(group)
        else:
            gr = lookup("/etc/group", group)
            if gr is None:
                raise ValueError(f"unable to find group {group} in the image")
            gid = int(gr[2])
    return uid, gid


def node_image_service(root_dir: str, pull=True, insecure_registries=()):
    """The image service of a process-runtime node: an OCI store under root_dir, the built-in
    images, and (pull=True) registry pulls for everything else."""
    from ..cri.server import ImageStore, host_image_resolver
    return ImageService(OCIStore(root_dir), ImageStore(host_image_resolver),
                        RegistryClient(insecure_registries) if pull else None)
