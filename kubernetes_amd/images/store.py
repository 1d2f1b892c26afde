"""Node-local OCI image store: content-addressed blobs, repository tags, unpacked root
filesystems.

Parity: the image side of the container runtime behind the reference kubelet (dockershim's
`docker_image.go` ListImages / ImageStatus / PullImage / RemoveImage over docker's image store,
and the layer store docker keeps under /var/lib/docker) — here on-disk and native to this
framework:

    <root>/blobs/sha256/<hex>          manifests, configs, layer tarballs (digest-verified)
    <root>/repositories.json           {"registry/repo:tag": manifest digest, ...}
    <root>/rootfs/<image id hex>/      the image's layers applied in order (whiteouts honoured),
                                       the read-only lower layer of every container's overlay

Layer application follows the OCI image spec (`layer.md`): `.wh.<name>` deletes `<name>` from
lower layers, `.wh..wh..opq` makes a directory opaque; every path is resolved inside the rootfs
(symlinks are followed only within it), device nodes are skipped unless the store runs as root.
"""
from __future__ import annotations

import gzip
import hashlib
import io
import json
import os
import shutil
import stat
import tarfile
import tempfile
import threading

from . import reference

MANIFEST_TYPES = ("application/vnd.oci.image.manifest.v1+json",
                  "application/vnd.docker.distribution.manifest.v2+json")
INDEX_TYPES = ("application/vnd.oci.image.index.v1+json",
               "application/vnd.docker.distribution.manifest.list.v2+json")


class ImageNotFound(LookupError):
    pass


class DigestMismatch(ValueError):
    pass


def sha256_digest(data: bytes) -> str:
    return "sha256:" + hashlib.sha256(data).hexdigest()


def secure_join(root: str, path: str, max_links=40) -> str:
    """Resolve `path` as if `root` were `/`: symlinks (absolute or relative) are followed inside
    root and `..` never climbs above it (the `securejoin` semantics container runtimes use)."""
    root = os.path.abspath(root)
    parts = [p for p in path.split("/") if p not in ("", ".")]
    cur = root
    links = 0
    while parts:
        p = parts.pop(0)
        if p == "..":
            cur = os.path.dirname(cur) if cur != root else root
            if not (cur + "/").startswith(root + "/"):
                cur = root
            continue
        nxt = os.path.join(cur, p)
        try:
            st = os.lstat(nxt)
        except FileNotFoundError:
            cur = nxt
            continue
        if stat.S_ISLNK(st.st_mode):
            links += 1
            if links > max_links:
                raise OSError(f"too many levels of symbolic links resolving {path}")
            target = os.readlink(nxt)
            if target.startswith("/"):
                cur = root
            parts = [x for x in target.split("/") if x not in ("", ".")] + parts
            continue
        cur = nxt
    return cur


def _rm(path):
    try:
        st = os.lstat(path)
    except FileNotFoundError:
        return
    if stat.S_ISDIR(st.st_mode):
        shutil.rmtree(path)
    else:
        os.unlink(path)


def _clean(name: str) -> str:
    while name.startswith("./"):
        name = name[2:]
    name = name.lstrip("/")
    return "" if name in (".", "") else name


_BAD_BASES = ("", ".", "..")


def _strictly_inside(root: str, path: str) -> bool:
    root = os.path.abspath(root)
    path = os.path.abspath(path)
    return path != root and path.startswith(root + "/")


def apply_layer(rootfs: str, fileobj, as_root=None):
    """Apply one layer tarball (plain or gzip) to rootfs.

    Untrusted layers (pulled from any registry): an entry whose base name, or whose whiteout
    target, is '', '.' or '..' is rejected — `.wh..` / `.wh...` / `a/..` would otherwise remove or
    overwrite the directory above the layer root (the store's other images) — and every path
    that is created, removed or written must resolve strictly inside rootfs."""
    as_root = (os.geteuid() == 0) if as_root is None else as_root
    rootfs = os.path.abspath(rootfs)
    with tarfile.open(fileobj=fileobj, mode="r:*") as tf:
        for m in tf:
            name = _clean(m.name)
            if not name:
                continue
            parent, base = os.path.split(name.rstrip("/"))
            if base in _BAD_BASES:
                raise ValueError(f"layer entry {m.name!r}: invalid path")
            pdir = secure_join(rootfs, parent)
            if pdir != rootfs and not _strictly_inside(rootfs, pdir):
                raise ValueError(f"layer entry {m.name!r} escapes the rootfs")
            if base == ".wh..wh..opq":
                if os.path.isdir(pdir):
                    for e in os.listdir(pdir):
                        _rm(os.path.join(pdir, e))
                continue
            if base.startswith(".wh."):
                victim = base[4:]
                if victim in _BAD_BASES or "/" in victim:
                    raise ValueError(f"layer entry {m.name!r}: invalid whiteout")
                _rm(os.path.join(pdir, victim))
                continue
            os.makedirs(pdir, exist_ok=True)
            dst = os.path.join(pdir, base)
            if m.isdir():
                # an existing directory symlink is kept and followed, inside the rootfs only
                dst = secure_join(rootfs, name.rstrip("/"))
                if not _strictly_inside(rootfs, dst):
                    continue   # a directory entry that resolves to the rootfs itself: nothing to make
                if os.path.lexists(dst) and not stat.S_ISDIR(os.lstat(dst).st_mode):
                    _rm(dst)
                os.makedirs(dst, exist_ok=True)
            else:
                if os.path.lexists(dst) and not (m.isfile() and os.path.isfile(dst) and not os.path.islink(dst)):
                    _rm(dst)
                if m.isfile():
                    src = tf.extractfile(m)
                    with open(dst, "wb") as f:
                        shutil.copyfileobj(src, f, 1 << 20)
                elif m.issym():
                    os.symlink(m.linkname, dst)
                elif m.islnk():
                    target = secure_join(rootfs, _clean(m.linkname))
                    if not (target + "/").startswith(os.path.abspath(rootfs) + "/") or not os.path.exists(target):
                        continue
                    os.link(target, dst)
                elif (m.ischr() or m.isblk()) and as_root:
                    mode = (stat.S_IFCHR if m.ischr() else stat.S_IFBLK) | (m.mode & 0o7777)
                    os.mknod(dst, mode, os.makedev(m.devmajor, m.devminor))
                elif m.isfifo():
                    os.mkfifo(dst, m.mode & 0o7777)
                else:
                    continue
            if as_root:
                try:
                    os.lchown(dst, m.uid, m.gid)
                except OSError:
                    pass
            if not m.issym():
                os.chmod(dst, m.mode & (0o7777 if as_root else 0o777))
                try:
                    os.utime(dst, (m.mtime, m.mtime))
                except OSError:
                    pass


class OCIStore:
    def __init__(self, root: str):
        self.root = root
        self.blob_dir = os.path.join(root, "blobs", "sha256")
        self.rootfs_dir = os.path.join(root, "rootfs")
        os.makedirs(self.blob_dir, exist_ok=True)
        os.makedirs(self.rootfs_dir, exist_ok=True)
        self._lock = threading.RLock()
        self._repos_path = os.path.join(root, "repositories.json")
        try:
            with open(self._repos_path) as f:
                self.repos: dict[str, str] = json.load(f)
        except (OSError, ValueError):
            self.repos = {}

    # -- blobs -------------------------------------------------------------------------------------
    def blob_path(self, digest: str) -> str:
        algo, _, hexd = digest.partition(":")
        if algo != "sha256" or len(hexd) != 64 or any(c not in "0123456789abcdef" for c in hexd):
            raise ValueError(f"unsupported digest {digest}")
        return os.path.join(self.blob_dir, hexd)

    def has_blob(self, digest) -> bool:
        return os.path.exists(self.blob_path(digest))

    def read_blob(self, digest) -> bytes:
        with open(self.blob_path(digest), "rb") as f:
            return f.read()

    def put_blob(self, data: bytes, digest: str | None = None) -> str:
        d = sha256_digest(data)
        if digest is not None and d != digest:
            raise DigestMismatch(f"content digest {d} does not match {digest}")
        path = self.blob_path(d)
        if not os.path.exists(path):
            fd, tmp = tempfile.mkstemp(dir=self.blob_dir)
            with os.fdopen(fd, "wb") as f:
                f.write(data)
            os.replace(tmp, path)
        return d

    def blob_writer(self, digest: str):
        return _BlobWriter(self, digest)

    # -- repositories ------------------------------------------------------------------------------
    def _save(self):
        tmp = self._repos_path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(self.repos, f, indent=1, sort_keys=True)
        os.replace(tmp, self._repos_path)

    def tag(self, ref: str, manifest_digest: str):
        with self._lock:
            self.repos[reference.normalize(ref)] = manifest_digest
            self._save()

    def resolve(self, ref: str) -> str | None:
        """-> manifest digest of ref (a tag, a digest reference, or an image id)."""
        if ref.startswith("sha256:"):
            for d in self.repos.values():
                if d == ref or self.manifest(d)["config"]["digest"] == ref:
                    return d
            return None
        try:
            r = reference.parse(ref)
        except reference.InvalidReference:
            return None
        if r.digest:
            pinned = self.repos.get(reference.normalize(ref))
            if pinned is not None:
                return pinned
            return r.digest if self.has_blob(r.digest) and "config" in self.manifest(r.digest) else None
        return self.repos.get(r.tagged())

    def manifest(self, digest) -> dict:
        return json.loads(self.read_blob(digest))

    def image(self, ref: str) -> dict | None:
        """{id, repo_tags, repo_digests, size, config, manifest_digest} or None."""
        md = self.resolve(ref)
        if md is None:
            return None
        man = self.manifest(md)
        cfg_digest = man["config"]["digest"]
        tags = sorted(reference.parse(t).familiar() for t, d in self.repos.items() if d == md)
        names = sorted({reference.parse(t).name for t, d in self.repos.items() if d == md})
        size = man["config"].get("size", 0) + sum(l.get("size", 0) for l in man.get("layers") or ())
        return {"id": cfg_digest, "repo_tags": tags, "repo_digests": [f"{n}@{md}" for n in names],
                "size": size, "config": json.loads(self.read_blob(cfg_digest)), "manifest_digest": md}

    def images(self) -> list[dict]:
        seen, out = set(), []
        for d in sorted(set(self.repos.values())):
            if d in seen:
                continue
            seen.add(d)
            tag = next(t for t, x in self.repos.items() if x == d)
            img = self.image(tag)
            if img is not None:
                out.append(img)
        return out

    # -- root filesystems --------------------------------------------------------------------------
    def rootfs(self, ref: str) -> str:
        """The unpacked rootfs of an image (created on first use)."""
        md = self.resolve(ref)
        if md is None:
            raise ImageNotFound(ref)
        man = self.manifest(md)
        hexd = man["config"]["digest"].split(":", 1)[1]
        path = os.path.join(self.rootfs_dir, hexd)
        with self._lock:
            if os.path.isdir(path):
                return path
            tmp = tempfile.mkdtemp(dir=self.rootfs_dir, prefix=".unpack-")
            try:
                for layer in man.get("layers") or ():
                    with open(self.blob_path(layer["digest"]), "rb") as f:
                        apply_layer(tmp, f)
                os.chmod(tmp, 0o755)
                os.replace(tmp, path)
            except BaseException:
                shutil.rmtree(tmp, ignore_errors=True)
                raise
        return path

    # -- removal / accounting ----------------------------------------------------------------------
    def remove(self, ref: str) -> bool:
        """Untag ref (every tag of the image when ref is an id or digest); once no tag names
        the manifest its rootfs and the blobs no other manifest uses are deleted."""
        with self._lock:
            md = self.resolve(ref)
            if md is None:
                return False
            if ref.startswith("sha256:") or "@" in ref:
                for t in [t for t, d in self.repos.items() if d == md]:
                    del self.repos[t]
            else:
                self.repos.pop(reference.parse(ref).tagged(), None)
            self._save()
            if md not in self.repos.values():
                self._collect()
            return True

    def _collect(self):
        live = set()
        for md in set(self.repos.values()):
            man = self.manifest(md)
            live.add(md)
            live.add(man["config"]["digest"])
            live.update(l["digest"] for l in man.get("layers") or ())
        for hexd in os.listdir(self.blob_dir):
            if len(hexd) == 64 and "sha256:" + hexd not in live:
                os.unlink(os.path.join(self.blob_dir, hexd))
        for hexd in os.listdir(self.rootfs_dir):
            if not hexd.startswith(".") and "sha256:" + hexd not in live:
                shutil.rmtree(os.path.join(self.rootfs_dir, hexd), ignore_errors=True)

    def used_bytes(self) -> int:
        total = 0
        for d, _dn, fs in os.walk(self.root):
            for f in fs:
                try:
                    total += os.lstat(os.path.join(d, f)).st_size
                except OSError:
                    pass
        return total

    # -- OCI image layout import ---------------------------------------------------------------------
    def import_layout(self, path: str, tag: str | None = None) -> list[str]:
        """Load an OCI image layout (directory or tar: `oci-layout`, `index.json`, `blobs/`),
        e.g. for air-gapped nodes. Images are tagged from the `org.opencontainers.image.ref.name`
        annotation (or `tag`). Returns the tags added."""
        if os.path.isdir(path):
            def read(name):
                with open(os.path.join(path, name), "rb") as f:
                    return f.read()
        else:
            tf = tarfile.open(path)

            def read(name):
                return tf.extractfile(name).read()
        index = json.loads(read("index.json"))
        added = []
        for desc in index.get("manifests") or ():
            md = desc["digest"]
            man_bytes = read("blobs/sha256/" + md.split(":", 1)[1])
            self.put_blob(man_bytes, md)
            man = json.loads(man_bytes)
            if man.get("mediaType") in INDEX_TYPES or "manifests" in man:
                raise ValueError("nested image indexes in a layout are not supported; export one platform")
            for d in [man["config"]["digest"]] + [l["digest"] for l in man.get("layers") or ()]:
                if not self.has_blob(d):
                    self.put_blob(read("blobs/sha256/" + d.split(":", 1)[1]), d)
            name = (desc.get("annotations") or {}).get("org.opencontainers.image.ref.name") or tag
            if name:
                self.tag(name, md)
                added.append(reference.normalize(name))
        return added


class _BlobWriter:
    """Streaming blob ingest with digest verification (registry pulls)."""

    def __init__(self, store: OCIStore, digest: str):
        self.store, self.digest = store, digest
        self.h = hashlib.sha256()
        fd, self.tmp = tempfile.mkstemp(dir=store.blob_dir)
        self.f = os.fdopen(fd, "wb")
        self.size = 0

    def write(self, data: bytes):
        self.h.update(data)
        self.f.write(data)
        self.size += len(data)

    def commit(self) -> str:
        self.f.close()
        d = "sha256:" + self.h.hexdigest()
        if d != self.digest:
            os.unlink(self.tmp)
            raise DigestMismatch(f"blob digest {d} does not match {self.digest}")
        os.replace(self.tmp, self.store.blob_path(d))
        return d

    def abort(self):
        try:
            self.f.close()
            os.unlink(self.tmp)
        except OSError:
            pass


def build_image(store: OCIStore, tag: str, files: dict, config: dict | None = None, base: str | None = None) -> str:
    """Build a one-layer image (on top of `base`'s layers) from {path: bytes | (bytes, mode) |
    ("symlink", target)}; returns the manifest digest. Used by tests, the local registry add-on
    and `kamd image build`."""
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w") as tf:
        dirs = set()
        for p in sorted(files):
            parts = p.strip("/").split("/")
            for i in range(1, len(parts)):
                d = "/".join(parts[:i])
                if d not in dirs:
                    dirs.add(d)
                    ti = tarfile.TarInfo(d)
                    ti.type, ti.mode = tarfile.DIRTYPE, 0o755
                    tf.addfile(ti)
            v = files[p]
            ti = tarfile.TarInfo(p.strip("/"))
            if isinstance(v, tuple) and v[0] == "symlink":
                ti.type, ti.linkname = tarfile.SYMTYPE, v[1]
                tf.addfile(ti)
                continue
            data, mode = (v if isinstance(v, tuple) else (v, 0o644))
            ti.size, ti.mode = len(data), mode
            tf.addfile(ti, io.BytesIO(data))
    raw = buf.getvalue()
    gz = gzip.compress(raw, mtime=0)
    layers, diff_ids = [], []
    if base is not None:
        bman = store.manifest(store.resolve(base))
        bcfg = json.loads(store.read_blob(bman["config"]["digest"]))
        layers = list(bman["layers"])
        diff_ids = list(bcfg["rootfs"]["diff_ids"])
        cfg = dict(bcfg.get("config") or {})
    else:
        cfg = {}
    cfg.update(config or {})
    ld = store.put_blob(gz)
    layers.append({"mediaType": "application/vnd.oci.image.layer.v1.tar+gzip", "digest": ld, "size": len(gz)})
    diff_ids.append(sha256_digest(raw))
    config_blob = json.dumps({"architecture": "amd64", "os": "linux", "config": cfg,
                              "rootfs": {"type": "layers", "diff_ids": diff_ids}}, sort_keys=True).encode()
    cd = store.put_blob(config_blob)
    man = json.dumps({"schemaVersion": 2, "mediaType": MANIFEST_TYPES[0],
                      "config": {"mediaType": "application/vnd.oci.image.config.v1+json", "digest": cd,
                                 "size": len(config_blob)},
                      "layers": layers}, sort_keys=True).encode()
    md = store.put_blob(man)
    store.tag(tag, md)
    return md
