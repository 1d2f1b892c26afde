"""Pod volumes and container environment, kubelet side.

Parity:
  * network / block volumes (nfs, cephfs, glusterfs, iscsi, fc, rbd) in `volume_plugins.py`;
  * `pkg/kubelet/volumemanager` + the in-tree plugins that need no cloud or network storage:
    `pkg/volume/empty_dir` (node disk or `medium: Memory` = tmpfs, here /dev/shm),
    `pkg/volume/host_path` (with `type: DirectoryOrCreate|FileOrCreate|Directory|File`),
    `pkg/volume/configmap`, `pkg/volume/secret` (keys → files, `items` remap, `defaultMode`),
    `pkg/volume/downwardapi` and `pkg/volume/projected` (a mix of the three);
  * `pkg/kubelet/kubelet_pods.go` `makeEnvironmentVariables` — `env[].valueFrom` (fieldRef,
    resourceFieldRef, configMapKeyRef, secretKeyRef) and `envFrom` (configMapRef/secretRef with
    `prefix`), `$(VAR)` expansion against earlier entries.

A volume is materialised under `<pods dir>/<pod uid>/volumes/<name>`; each `volumeMount` becomes a
bind mount {containerPath, hostPath, readOnly} in the container's run options (the OCI bundle's
`mounts`). The process runtime has no mount namespace, so it also exports each mount's host path
as `KUBERNETES_VOLUME_<NAME>` to the process.
"""
from __future__ import annotations

import base64
import logging
import os
import re
import shutil
import stat

from ..api.quantity import parse_quantity
from ..client.rest import APIStatusError
from .volume_plugins import NETWORK_KINDS

_ENV_NAME = re.compile(r"^[-._a-zA-Z][-._a-zA-Z0-9]*$")   # IsEnvVarName (1.9 C_IDENTIFIER relaxed)
log = logging.getLogger("kubelet.volumes")


class VolumeError(Exception):
    pass


def _rmtree_no_mounts(path, mounter):
    """Remove a pod directory but never descend into a mount point (a network volume that failed
    to unmount must not lose its remote files)."""
    if not os.path.lexists(path):
        return
    if mounter.is_mount_point(path):
        return
    if os.path.isdir(path) and not os.path.islink(path):
        for e in os.listdir(path):
            _rmtree_no_mounts(os.path.join(path, e), mounter)
        try:
            os.rmdir(path)
        except OSError:
            pass
    else:
        try:
            os.unlink(path)
        except OSError:
            pass


def _write_files(d, data: dict, items=None, mode=0o644, binary=False, optional=False) -> set:
    """Project `data` into files under d: every key, or `items` ({key, path, mode}) — an item's
    own `mode` beats `defaultMode` (`pkg/volume/util/atomic_writer.go` payloads). A file is only
    rewritten when its content or mode changed (atomic rename). Returns the relative paths."""
    os.makedirs(d, exist_ok=True)
    if items:
        keys = [(i["key"], i.get("path", i["key"]), i.get("mode")) for i in items]
    else:
        keys = [(k, k, None) for k in data]
    out = set()
    for k, rel, item_mode in keys:
        if k not in data:
            if optional:
                continue
            raise VolumeError(f"key {k!r} not found")
        p = os.path.join(d, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        v = data[k]
        raw = base64.b64decode(v) if binary else str(v).encode()
        want = int(item_mode) if item_mode is not None else mode
        out.add(rel)
        try:
            st = os.stat(p)
            with open(p, "rb") as f:
                if f.read() == raw and (st.st_mode & 0o7777) == want:
                    continue
        except OSError:
            pass
        tmp = p + ".tmp"
        with open(tmp, "wb") as f:
            f.write(raw)
        os.chmod(tmp, want)
        os.replace(tmp, p)
    return out


# volume kinds whose files the kubelet owns, so `fsGroup` applies (SetVolumeOwnership callers)
_OWNED = ("emptyDir", "configMap", "secret", "downwardAPI", "projected")
_READONLY = ("configMap", "secret", "downwardAPI", "projected")


def set_volume_ownership(d, fs_group, readonly):
    """`pkg/volume/volume_linux.go` SetVolumeOwnership: every file and directory of the volume
    gets group `fs_group` and group access (rw, r for the read-only kinds); directories get the
    setgid bit (new files inherit the group) and group search.

    Every entry is opened with O_PATH | O_NOFOLLOW and changed through that descriptor
    (`/proc/self/fd/N`), never by path: a container that can write the volume cannot swap a file
    for a symlink between the check and the chmod and have the kubelet change a host file."""
    mask = 0o440 if readonly else 0o660
    for root, dirs, files in os.walk(d):
        for p in [root] + [os.path.join(root, x) for x in files]:
            try:
                fd = os.open(p, os.O_PATH | os.O_NOFOLLOW | os.O_CLOEXEC)
            except OSError as e:
                log.debug("fsGroup ownership of %s: %s", p, e)
                continue
            try:
                st = os.fstat(fd)
                if stat.S_ISLNK(st.st_mode) or not (stat.S_ISDIR(st.st_mode) or stat.S_ISREG(st.st_mode)):
                    continue          # O_PATH|O_NOFOLLOW on a symlink opens the link itself
                via = f"/proc/self/fd/{fd}"
                os.chown(via, -1, int(fs_group))
                m = stat.S_IMODE(st.st_mode) | mask
                if stat.S_ISDIR(st.st_mode):
                    m |= stat.S_ISGID | 0o110
                os.chmod(via, m)
            except OSError as e:       # not permitted (an unprivileged kubelet outside the group)
                log.debug("fsGroup ownership of %s: %s", p, e)
            finally:
                os.close(fd)


def _fs_group(pod):
    return ((pod.get("spec") or {}).get("securityContext") or {}).get("fsGroup")


def _prune(d, keep: set):
    """Remove projected files no longer in the payload (a key deleted from its ConfigMap, an
    optional source that went away)."""
    for root, _dirs, files in os.walk(d, topdown=False):
        for f in files:
            rel = os.path.relpath(os.path.join(root, f), d)
            if rel not in keep:
                try:
                    os.unlink(os.path.join(root, f))
                except OSError:
                    pass
        if root != d and not os.listdir(root):
            try:
                os.rmdir(root)
            except OSError:
                pass


def _field(pod, path, node_name=None, pod_ip=None, host_ip=None):
    md = pod.get("metadata") or {}
    if path == "metadata.name":
        return md.get("name", "")
    if path == "metadata.namespace":
        return md.get("namespace", "")
    if path == "metadata.uid":
        return md.get("uid", "")
    if path == "spec.nodeName":
        return node_name or (pod.get("spec") or {}).get("nodeName", "")
    if path == "spec.serviceAccountName":
        return (pod.get("spec") or {}).get("serviceAccountName", "")
    if path == "status.podIP":
        return pod_ip or (pod.get("status") or {}).get("podIP", "")
    if path == "status.hostIP":
        # the kubelet's own node address: the status carrying hostIP may not be written yet
        return (pod.get("status") or {}).get("hostIP") or host_ip or ""
    if path in ("metadata.labels", "metadata.annotations"):
        m = md.get(path.split(".")[1]) or {}
        return "\n".join(f'{k}="{v}"' for k, v in sorted(m.items()))
    mm = re.fullmatch(r"metadata\.(labels|annotations)\['(.+)'\]", path)
    if mm:
        return (md.get(mm.group(1)) or {}).get(mm.group(2), "")
    raise VolumeError(f"unsupported fieldRef {path!r}")


def _resource_field(container, ref, allocatable=None):
    """`resourceFieldRef` (`pkg/api/v1/resource/helpers.go` ExtractContainerResourceValue): a
    missing limit is the node's allocatable (`kubelet_resources.go` defaultPodLimitsForDownwardAPI),
    a missing request falls back to the limit."""
    res = container.get("resources") or {}
    r = ref["resource"]
    kind, name = r.split(".", 1)
    q = (res.get(kind) or {}).get(name)
    if q is None and kind == "requests":
        q = (res.get("limits") or {}).get(name)
    if q is None and kind == "limits" and allocatable:
        q = allocatable.get(name)
    if q is None:
        return "0"
    v = parse_quantity(str(q)).value / parse_quantity(str(ref.get("divisor", "1"))).value   # Fractions
    # round up like the reference (ExtractResourceValueByContainerName)
    return str(-(-v.numerator // v.denominator))


def validate_path_no_backsteps(p):
    """`volumevalidation.ValidatePathNoBacksteps`."""
    if ".." in p.split(os.sep):
        raise VolumeError("must not contain '..'")


def make_absolute_path(p):
    """`makeAbsolutePath` (linux): a relative container path is taken from the root."""
    return p if p.startswith("/") else "/" + p


def _within(path, root):
    return path == root or path.startswith(root.rstrip(os.sep) + os.sep)


def make_mounts(container, vols: dict):
    """Each volumeMount becomes {containerPath, hostPath, readOnly}. A subPath must be relative,
    without '..', and must resolve (symlinks included) inside the volume; a missing subPath
    directory is created with the volume directory's mode (`SafeMakeDir`), never through a
    symlink that leaves the volume (the reference's `PrepareSafeSubpath` guarantee)."""
    out = []
    name = container.get("name", "")
    for m in container.get("volumeMounts") or ():
        hp = vols.get(m["name"])
        if hp is None:
            raise VolumeError(f'cannot find volume "{m["name"]}" to mount into container "{name}"')
        sub = m.get("subPath") or ""
        if sub:
            if os.path.isabs(sub):
                raise VolumeError(f"error SubPath `{sub}` must not be an absolute path")
            try:
                validate_path_no_backsteps(sub)
            except VolumeError as e:
                raise VolumeError(f"unable to provision SubPath `{sub}`: {e}") from None
            try:
                perm = os.lstat(hp).st_mode & 0o7777
            except OSError as e:
                raise VolumeError(str(e)) from None
            vol = os.path.realpath(hp)
            target = os.path.join(vol, sub)
            fail = VolumeError(f'failed to prepare subPath for volumeMount "{m["name"]}" of container "{name}"')
            if not os.path.lexists(target):
                # create component by component, refusing any existing symlink on the way
                cur = vol
                for part in sub.split(os.sep):
                    if not part or part == ".":
                        continue
                    cur = os.path.join(cur, part)
                    if os.path.islink(cur) and not _within(os.path.realpath(cur), vol):
                        raise fail
                    if not os.path.lexists(cur):
                        os.mkdir(cur)
                        os.chmod(cur, perm or 0o755)
            if not _within(os.path.realpath(target), vol):
                raise fail
            hp = os.path.realpath(target)
        out.append({"containerPath": make_absolute_path(m["mountPath"]), "hostPath": hp,
                    "readOnly": bool(m.get("readOnly"))})
    return out


class VolumeManager:
    def __init__(self, client, root, csi_plugins_dir=None, node_name=None, attach_timeout=60.0,
                 flex_plugins_dir="/usr/libexec/kubernetes/kubelet-plugins/volume/exec", mounter=None):
        from .volume_plugins import Mounter
        self.mounter = mounter or Mounter()               # nfs / cephfs / glusterfs / iscsi / fc / rbd
        self.net_mounted: dict[str, list] = {}           # pod uid -> [plugin state]
        self.flex_dir = flex_plugins_dir
        self.flex_mounted: dict[str, list] = {}      # pod uid -> [(driver path, target)]
        self.flex_inited: dict[str, dict] = {}       # driver path -> init capabilities
        self.client = client
        self.root = root
        self.csi_dir = csi_plugins_dir
        self.node_name = node_name
        self.attach_timeout = attach_timeout
        self.csi_published: dict[str, list] = {}     # pod uid -> [(driver, volume handle, target)]
        self.in_use: dict[str, set] = {}             # pod uid -> unique names of its attachable volumes
        self.on_in_use_change = None                 # callback: node status should report volumesInUse
        self.allocatable = None                      # node allocatable: default downward-API limits
        self.host_ip = None                          # the node's address (status.hostIP)
        self.recorder = None                         # (obj, type, reason, message): pod events

    def _traversable(self, path):
        """Make the kubelet-owned directories above a volume traversable (0711: no listing) so a
        container running as another uid can reach the volume at its host path — the process
        runtime's containers on the host root read volumes there (KUBERNETES_VOLUME_<NAME>)."""
        stop = os.path.dirname(os.path.dirname(os.path.abspath(self.root)))    # up to the kubelet root
        p = os.path.abspath(path)
        while p.startswith(stop + os.sep) and p != stop:
            try:
                st = os.stat(p)
                if st.st_uid == os.geteuid() and (st.st_mode & 0o111) != 0o111:
                    os.chmod(p, (st.st_mode & 0o7777) | 0o111)
            except OSError:
                pass
            p = os.path.dirname(p)

    def pod_dir(self, pod):
        return os.path.join(self.root, pod["metadata"]["uid"])

    async def _get(self, kind, ns, name, optional):
        try:
            return await self.client.get(kind, name, ns)
        except APIStatusError as e:
            if e.code == 404 and optional:
                return None
            raise VolumeError(f"{kind[:-1]} {ns}/{name} not found" if e.code == 404 else str(e))

    async def setup(self, pod, node_name=None, pod_ip=None) -> dict:
        """Materialise every volume of the pod; returns {volume name: host path}."""
        ns = pod["metadata"].get("namespace", "default")
        base = os.path.join(self.pod_dir(pod), "volumes")
        out = {}
        for v in (pod.get("spec") or {}).get("volumes") or ():
            name = v["name"]
            d = os.path.join(base, name)
            if "emptyDir" in v:
                if (v["emptyDir"] or {}).get("medium") == "Memory":
                    d = await self._memory_dir(pod, name, d, (v["emptyDir"] or {}).get("sizeLimit"))
                os.makedirs(d, exist_ok=True)
                os.chmod(d, 0o777)          # `empty_dir.go` setupDir: world-writable, any runAsUser
            elif "hostPath" in v:
                hp = v["hostPath"]
                d = hp["path"]
                t = hp.get("type", "")
                if t == "DirectoryOrCreate":
                    os.makedirs(d, exist_ok=True)
                elif t == "FileOrCreate" and not os.path.exists(d):
                    os.makedirs(os.path.dirname(d), exist_ok=True)
                    open(d, "a").close()
                elif t == "Directory" and not os.path.isdir(d):
                    raise VolumeError(f"hostPath {d} is not a directory")
                elif t == "File" and not os.path.isfile(d):
                    raise VolumeError(f"hostPath {d} is not a file")
            elif "configMap" in v or "secret" in v:
                await self._cm_secret(ns, v, d)
            elif "downwardAPI" in v:
                self._downward(pod, v["downwardAPI"], d, node_name, pod_ip)
            elif "persistentVolumeClaim" in v:
                d = await self._pvc_path(ns, v["persistentVolumeClaim"], pod, name, node_name)
            elif "flexVolume" in v:
                d = await self._flex_mount(pod, name, v["flexVolume"], d)
            elif "gitRepo" in v:
                await self._git_repo(v["gitRepo"], d)
            elif any(k in v for k in NETWORK_KINDS):
                kind = next(k for k in NETWORK_KINDS if k in v)
                d = await self._net_mount(pod, kind, v[kind], d)
            elif "projected" in v:
                dm = v["projected"].get("defaultMode")
                os.makedirs(d, exist_ok=True)
                for src in v["projected"].get("sources") or ():
                    if "configMap" in src or "secret" in src:
                        await self._cm_secret(ns, src, d, dm)
                    elif "downwardAPI" in src:
                        self._downward(pod, src["downwardAPI"], d, node_name, pod_ip, dm)
            else:
                raise VolumeError(f"volume {name}: unsupported volume source {sorted(k for k in v if k != 'name')}")
            if _fs_group(pod) is not None and any(k in v for k in _OWNED):
                set_volume_ownership(d, _fs_group(pod), any(k in v for k in _READONLY))
            out[name] = d
        if out:
            self._traversable(base)
        return out

    async def _pvc_path(self, ns, src, pod=None, vol_name=None, node_name=None):
        """persistentVolumeClaim -> the bound PV's hostPath / local path, or a CSI volume
        published by its driver (`pkg/volume/util/operationexecutor` mounts the PV the claim is
        bound to)."""
        pvc = await self._get("persistentvolumeclaims", ns, src.get("claimName", ""), False)
        vol = (pvc.get("spec") or {}).get("volumeName")
        if not vol or (pvc.get("status") or {}).get("phase") != "Bound":
            raise VolumeError(f"persistentvolumeclaim {ns}/{src.get('claimName')} is not bound")
        pv = await self._get("persistentvolumes", None, vol, False)
        sp = pv.get("spec") or {}
        if sp.get("flexVolume") and pod is not None:
            d = os.path.join(self.pod_dir(pod), "volumes", "flexvolume", vol)
            return await self._flex_mount(pod, vol, sp["flexVolume"], d)
        if sp.get("csi"):
            return await self._csi_publish(pod, vol, sp, node_name or self.node_name, pv)
        kind = next((k for k in NETWORK_KINDS if sp.get(k)), None)
        if kind is not None and pod is not None:
            # PV mount options: spec.mountOptions, or the 1.9 beta annotation
            opts = list(sp.get("mountOptions") or ())
            ann = ((pv.get("metadata") or {}).get("annotations") or {}).get("volume.beta.kubernetes.io/mount-options")
            if ann and not opts:
                opts = [o.strip() for o in ann.split(",") if o.strip()]
            target = os.path.join(self.pod_dir(pod), "volumes", f"kubernetes.io~{kind}", vol)
            return await self._net_mount(pod, kind, sp[kind], target, opts)
        path = (sp.get("hostPath") or {}).get("path") or (sp.get("local") or {}).get("path")
        if not path:
            raise VolumeError(f"persistentvolume {vol}: only hostPath / local volumes can be mounted on this node")
        os.makedirs(path, exist_ok=True)
        return path

    async def _csi_publish(self, pod, pv_name, sp, node_name, pv=None):
        """`pkg/volume/csi/csi_attacher.go` WaitForAttach (the VolumeAttachment the attach/detach
        controller created must report `attached`) then `csi_mounter.go` SetUpAt:
        NodePublishVolume to `<pod dir>/volumes/kubernetes.io~csi/<pv>/mount`."""
        import asyncio
        from ..csi import api as CSI
        from ..csi.driver import CSIClient, volume_attributes
        src = sp["csi"]
        driver, handle = src["driver"], src["volumeHandle"]
        # reported in use before the mount (`MarkVolumesAsReportedInUse`): from now on the
        # attach/detach controller will not detach it under us
        self._mark_in_use(pod, f"kubernetes.io/csi/{driver}^{handle}")
        va_name = CSI.attachment_name(pv_name, driver, node_name)
        deadline = asyncio.get_running_loop().time() + self.attach_timeout
        info = {}
        while True:
            try:
                va = await self.client.get("volumeattachments", va_name)
                st = va.get("status") or {}
                if st.get("attached"):
                    info = st.get("attachmentMetadata") or {}
                    break
                if st.get("attachError"):
                    raise VolumeError(f"attach of {pv_name} failed: {st['attachError'].get('message')}")
            except APIStatusError as e:
                if e.code != 404:
                    raise
            if asyncio.get_running_loop().time() > deadline:
                raise VolumeError(f"volume {pv_name} is not attached to {node_name} (VolumeAttachment {va_name})")
            await asyncio.sleep(0.05)
        target = os.path.join(self.pod_dir(pod), "volumes", "kubernetes.io~csi", pv_name, "mount")
        c = CSIClient(CSI.socket_path(self.csi_dir, driver))
        try:
            await c.node_publish(handle, target, bool(src.get("readOnly")), info, volume_attributes(pv),
                                 sp.get("accessModes"), src.get("fsType", ""))
        except Exception as e:  # noqa: BLE001 - surfaced as a mount failure, retried by the kubelet
            raise VolumeError(f"NodePublishVolume {handle} via {driver}: {e}")
        finally:
            await c.close()
        self.csi_published.setdefault(pod["metadata"]["uid"], []).append((driver, handle, target))
        return target

    async def _net_mount(self, pod, kind, src, target, mount_options=()):
        """nfs / cephfs / glusterfs / iscsi / fc / rbd (`kubelet/volume_plugins.py`)."""
        from .volume_plugins import MOUNT, MountError, PluginContext
        ctx = PluginContext(self.client, pod["metadata"].get("namespace", "default"), self.mounter,
                            os.path.join(self.root, "..", "plugins", f"kubernetes.io~{kind}"), mount_options)
        if self.mounter.is_mount_point(target):
            return target                          # already set up (pod resync)
        try:
            state = await MOUNT[kind](src, target, ctx)
        except (MountError, APIStatusError, KeyError, ValueError) as e:
            raise VolumeError(f"{kind} volume: {e}")
        state["kind"] = kind
        self.net_mounted.setdefault(pod["metadata"]["uid"], []).append(state)
        return target

    async def _flex_call(self, driver_path, *args):
        """`pkg/volume/flexvolume/driver-call.go`: exec the driver, parse its JSON status."""
        import asyncio
        import json as _json
        p = await asyncio.create_subprocess_exec(driver_path, *args, stdout=asyncio.subprocess.PIPE,
                                                 stderr=asyncio.subprocess.PIPE)
        out, err = await p.communicate()
        try:
            st = _json.loads(out or b"{}")
        except ValueError:
            raise VolumeError(f"flexvolume {driver_path} {args[0]}: invalid output {out[:200]!r} {err[:200]!r}")
        if st.get("status") == "Not supported":
            return st
        if st.get("status") != "Success":
            raise VolumeError(f"flexvolume {driver_path} {args[0]} failed: {st.get('message', '')}")
        return st

    async def _flex_mount(self, pod, vol_name, src, target):
        """FlexVolume (`pkg/volume/flexvolume`): `init` once per driver, then
        `mount <target> <json options>` with the user options plus the kubernetes.io/* keys
        (fsType, readwrite, pod name/namespace/uid, serviceAccount.name, pvOrVolumeName, secret/*)."""
        import json as _json
        vendor_driver = src.get("driver", "")
        vendor, _, drv = vendor_driver.rpartition("/")
        path = os.path.join(self.flex_dir, f"{vendor}~{drv}" if vendor else drv, drv)
        if not os.access(path, os.X_OK):
            raise VolumeError(f"flexvolume driver {vendor_driver} not found at {path}")
        if path not in self.flex_inited:
            self.flex_inited[path] = (await self._flex_call(path, "init")).get("capabilities") or {}
        md = pod["metadata"]
        opts = dict(src.get("options") or {})
        opts.update({"kubernetes.io/fsType": src.get("fsType", ""),
                     "kubernetes.io/readwrite": "ro" if src.get("readOnly") else "rw",
                     "kubernetes.io/pod.name": md["name"], "kubernetes.io/pod.namespace": md.get("namespace", "default"),
                     "kubernetes.io/pod.uid": md["uid"], "kubernetes.io/pvOrVolumeName": vol_name,
                     "kubernetes.io/serviceAccount.name": (pod.get("spec") or {}).get("serviceAccountName", "default")})
        if src.get("secretRef"):
            sec = await self._get("secrets", md.get("namespace", "default"), src["secretRef"]["name"], False)
            for k, v in (sec.get("data") or {}).items():
                opts[f"kubernetes.io/secret/{k}"] = v
        os.makedirs(target, exist_ok=True)
        await self._flex_call(path, "mount", target, _json.dumps(opts))
        self.flex_mounted.setdefault(md["uid"], []).append((path, target))
        return target

    async def _git_repo(self, src, d):
        """gitRepo volume (`pkg/volume/git_repo`): `git clone -- <repo> [<directory>]`, then
        `git checkout <revision>` + `git reset --hard` when a revision is given."""
        import asyncio
        os.makedirs(d, exist_ok=True)
        if os.listdir(d):
            return
        args = ["clone", "--", src["repository"]] + ([src["directory"]] if src.get("directory") else [])
        p = await asyncio.create_subprocess_exec("git", *args, cwd=d, stdout=asyncio.subprocess.PIPE,
                                                 stderr=asyncio.subprocess.PIPE)
        _, err = await p.communicate()
        if p.returncode != 0:
            raise VolumeError(f"git clone {src['repository']}: {err.decode(errors='replace').strip()}")
        if src.get("revision"):
            sub = src.get("directory") or os.path.basename(src["repository"].rstrip("/")).removesuffix(".git")
            repo = d if src.get("directory") == "." else os.path.join(d, sub)
            for cmd in (["checkout", src["revision"]], ["reset", "--hard"]):
                p = await asyncio.create_subprocess_exec("git", *cmd, cwd=repo, stdout=asyncio.subprocess.PIPE,
                                                         stderr=asyncio.subprocess.PIPE)
                _, err = await p.communicate()
                if p.returncode != 0:
                    raise VolumeError(f"git {' '.join(cmd)}: {err.decode(errors='replace').strip()}")

    async def unpublish(self, pod):
        """FlexVolume `unmount`, CSI NodeUnpublishVolume and network/block unmount + detach for
        the pod's volumes (TearDownAt / UnmountDevice)."""
        from .volume_plugins import MountError, PluginContext, detach
        states = self.net_mounted.pop(pod["metadata"]["uid"], [])

        def still_used(key):
            for sts in self.net_mounted.values():
                for st in sts:
                    if ("iscsi", st.get("iscsi", (None, None))[1]) == key or ("rbd", st.get("rbd")) == key:
                        return True
            return False
        for st in states:
            ctx = PluginContext(self.client, pod["metadata"].get("namespace", "default"), self.mounter, "")
            try:
                await detach(ctx, st, still_used)
            except MountError:
                pass
        for path, target in self.flex_mounted.pop(pod["metadata"]["uid"], []):
            try:
                await self._flex_call(path, "unmount", target)
            except VolumeError:
                pass
        from ..csi import api as CSI
        from ..csi.driver import CSIClient
        for driver, handle, target in self.csi_published.pop(pod["metadata"]["uid"], []):
            c = CSIClient(CSI.socket_path(self.csi_dir, driver))
            try:
                await c.node_unpublish(handle, target)
            except Exception:  # noqa: BLE001 - best effort like the reference's unmount retries
                pass
            finally:
                await c.close()
        if self.in_use.pop(pod["metadata"]["uid"], None) and self.on_in_use_change:
            self.on_in_use_change()

    def _mark_in_use(self, pod, name):
        s = self.in_use.setdefault(pod["metadata"]["uid"], set())
        if name not in s:
            s.add(name)
            if self.on_in_use_change:
                self.on_in_use_change()

    def volumes_in_use(self):
        """node.status.volumesInUse: unique names of the attachable volumes mounted (or being
        mounted) for this node's pods."""
        return sorted(set().union(*self.in_use.values())) if self.in_use else []

    async def refresh(self, pod, node_name=None, pod_ip=None):
        """Re-project the pod's configMap / secret / downwardAPI / projected volumes into their
        directories (the kubelet's periodic pod sync, `--sync-frequency`): updated keys, new
        keys, removed keys, an optional source that appeared or went away, changed labels and
        annotations all reach the running container."""
        ns = pod["metadata"].get("namespace", "default")
        base = os.path.join(self.pod_dir(pod), "volumes")
        for v in (pod.get("spec") or {}).get("volumes") or ():
            d = os.path.join(base, v["name"])
            if not os.path.isdir(d):
                continue
            if "configMap" in v or "secret" in v:
                _prune(d, await self._cm_secret(ns, v, d))
            elif "downwardAPI" in v:
                _prune(d, self._downward(pod, v["downwardAPI"], d, node_name, pod_ip))
            elif "projected" in v:
                keep = set()
                for src in v["projected"].get("sources") or ():
                    if "configMap" in src or "secret" in src:
                        keep |= await self._cm_secret(ns, src, d, v["projected"].get("defaultMode"))
                    elif "downwardAPI" in src:
                        keep |= self._downward(pod, src["downwardAPI"], d, node_name, pod_ip,
                                               v["projected"].get("defaultMode"))
                _prune(d, keep)
            if _fs_group(pod) is not None and any(k in v for k in _READONLY):
                set_volume_ownership(d, _fs_group(pod), True)

    async def _cm_secret(self, ns, v, d, default_mode=None):
        if "configMap" in v:
            src = v["configMap"]
            obj = await self._get("configmaps", ns, src["name"], src.get("optional"))
            data = dict((obj or {}).get("data") or {})
            binary = False
            if obj and obj.get("binaryData"):
                for k, b in obj["binaryData"].items():
                    data[k] = base64.b64decode(b).decode("latin-1")
        else:
            src = v["secret"]
            obj = await self._get("secrets", ns, src.get("secretName") or src.get("name"), src.get("optional"))
            data = dict((obj or {}).get("data") or {})
            for k, s in ((obj or {}).get("stringData") or {}).items():
                data[k] = base64.b64encode(s.encode()).decode()
            binary = True
        mode = src.get("defaultMode", default_mode if default_mode is not None else 0o644)
        return _write_files(d, data, src.get("items"), int(mode), binary, optional=bool(src.get("optional")))

    def _downward(self, pod, spec, d, node_name, pod_ip, default_mode=None):
        data = {}
        items = []
        ctrs = {c["name"]: c for c in (pod.get("spec") or {}).get("containers") or ()}
        for it in spec.get("items") or ():
            if "fieldRef" in it:
                data[it["path"]] = _field(pod, it["fieldRef"]["fieldPath"], node_name, pod_ip, self.host_ip)
            elif "resourceFieldRef" in it:
                ref = it["resourceFieldRef"]
                c = ctrs.get(ref.get("containerName")) or next(iter(ctrs.values()), {})
                data[it["path"]] = _resource_field(c, ref, self.allocatable)
            items.append({"key": it["path"], "path": it["path"], "mode": it.get("mode")})
        mode = spec.get("defaultMode", default_mode if default_mode is not None else 0o644)
        return _write_files(d, data, items, int(mode))

    def mounts_for(self, container, vols: dict):
        """`makeMounts` (kubelet_pods.go:167) for the container's volumeMounts."""
        return make_mounts(container, vols)

    async def _memory_dir(self, pod, name, d, size_limit=None):
        """`medium: Memory` (`empty_dir.go` setupTmpfs): a tmpfs mounted on the volume directory
        when the kubelet may mount (root) — visible at the same path to every container, also
        one whose /dev is private — else a directory under /dev/shm."""
        if os.geteuid() == 0 and shutil.which("mount"):
            os.makedirs(d, exist_ok=True)
            if self.mounter.is_mount_point(d):
                return d
            opts = ["mode=0777"]
            if size_limit:
                opts.append(f"size={int(parse_quantity(str(size_limit)).value)}")
            try:
                await self.mounter.mount("tmpfs", d, "tmpfs", opts)
                return d
            except Exception:  # noqa: BLE001 - no mount privilege after all: /dev/shm below
                pass
        if os.path.isdir("/dev/shm"):
            return os.path.join("/dev/shm", "kamd-" + pod["metadata"]["uid"], name)
        return d

    def teardown(self, pod):
        vdir = os.path.join(self.pod_dir(pod), "volumes")
        for v in (pod.get("spec") or {}).get("volumes") or ():
            p = os.path.join(vdir, v["name"])
            if "emptyDir" in v and (v["emptyDir"] or {}).get("medium") == "Memory" and self.mounter.is_mount_point(p):
                import subprocess
                subprocess.run(["umount", p], capture_output=True, timeout=10)
        _rmtree_no_mounts(self.pod_dir(pod), self.mounter)
        shm = os.path.join("/dev/shm", "kamd-" + pod["metadata"]["uid"])
        if os.path.isdir(shm):
            shutil.rmtree(shm, ignore_errors=True)

    async def env_for(self, pod, container, node_name=None, pod_ip=None, base_env=()):
        """Resolved container environment (list of {name, value}). `base_env` (the service
        variables) comes first: envFrom and the container's own env override it, and `$(VAR)`
        references can name it (`kubelet_pods.go` makeEnvironmentVariables)."""
        ns = pod["metadata"].get("namespace", "default")
        env: dict[str, str] = {}
        order = []

        from .kubelet import expand
        svc = {e["name"]: e["value"] for e in base_env}

        def put(k, v):
            if k not in env:
                order.append(k)
            env[k] = v
        for ef in container.get("envFrom") or ():
            pre = ef.get("prefix", "")
            kind, ref = ("configmaps", ef["configMapRef"]) if "configMapRef" in ef else \
                (("secrets", ef["secretRef"]) if "secretRef" in ef else (None, None))
            if kind is None:
                continue
            obj = await self._get(kind, ns, ref["name"], ref.get("optional"))
            invalid = []
            for k, v in sorted(((obj or {}).get("data") or {}).items()):
                if not _ENV_NAME.match(pre + k):
                    invalid.append(k)       # makeEnvironmentVariables: skipped, not fatal
                    continue
                put(pre + k, base64.b64decode(v).decode(errors="replace") if kind == "secrets" else str(v))
            if invalid:
                what = "configMap" if kind == "configmaps" else "secret"
                msg = (f"Keys [{', '.join(sorted(invalid))}] from the EnvFrom {what} {ns}/{ref['name']} were skipped "
                       f"since they are considered invalid environment variable names.")
                rec = getattr(self, "recorder", None)
                if rec is not None:
                    rec(pod, "Warning", "InvalidEnvironmentVariableNames", msg)
                else:
                    log.warning("%s", msg)
        for e in container.get("env") or ():
            name = e["name"]
            if "value" in e:
                # expansion.MappingFuncFor(env so far, service env): `$(VAR)` from earlier entries
                put(name, expand(e["value"], env, svc))
                continue
            vf = e.get("valueFrom") or {}
            if "fieldRef" in vf:
                put(name, _field(pod, vf["fieldRef"]["fieldPath"], node_name, pod_ip, self.host_ip))
            elif "resourceFieldRef" in vf:
                put(name, _resource_field(container, vf["resourceFieldRef"], self.allocatable))
            elif "configMapKeyRef" in vf:
                r = vf["configMapKeyRef"]
                obj = await self._get("configmaps", ns, r["name"], r.get("optional"))
                if obj is not None:
                    if r["key"] not in (obj.get("data") or {}):
                        if not r.get("optional"):
                            raise VolumeError(f"Couldn't find key {r['key']} in ConfigMap {ns}/{r['name']}")
                    else:
                        put(name, str(obj["data"][r["key"]]))
            elif "secretKeyRef" in vf:
                r = vf["secretKeyRef"]
                obj = await self._get("secrets", ns, r["name"], r.get("optional"))
                if obj is not None:
                    if r["key"] not in (obj.get("data") or {}):
                        if not r.get("optional"):
                            raise VolumeError(f"Couldn't find key {r['key']} in Secret {ns}/{r['name']}")
                    else:
                        put(name, base64.b64decode(obj["data"][r["key"]]).decode(errors="replace"))
        # the service variables come last and never override the container's own (kubelet_pods.go)
        for k, v in svc.items():
            if k not in env:
                put(k, v)
        return [{"name": k, "value": env[k]} for k in order]
