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
import os
import re
import shutil

from ..api.quantity import parse_quantity
from ..client.rest import APIStatusError
from .volume_plugins import NETWORK_KINDS


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


def _write_files(d, data: dict, items=None, mode=0o644, binary=False):
    os.makedirs(d, exist_ok=True)
    keys = {i["key"]: i.get("path", i["key"]) for i in items} if items else {k: k for k in data}
    for k, rel in keys.items():
        if k not in data:
            raise VolumeError(f"key {k!r} not found")
        p = os.path.join(d, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        v = data[k]
        raw = base64.b64decode(v) if binary else str(v).encode()
        tmp = p + ".tmp"
        with open(tmp, "wb") as f:
            f.write(raw)
        os.chmod(tmp, mode)
        os.replace(tmp, p)


def _field(pod, path, node_name=None, pod_ip=None):
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
        return (pod.get("status") or {}).get("hostIP", "")
    if path in ("metadata.labels", "metadata.annotations"):
        m = md.get(path.split(".")[1]) or {}
        return "\n".join(f'{k}="{v}"' for k, v in sorted(m.items()))
    mm = re.fullmatch(r"metadata\.(labels|annotations)\['(.+)'\]", path)
    if mm:
        return (md.get(mm.group(1)) or {}).get(mm.group(2), "")
    raise VolumeError(f"unsupported fieldRef {path!r}")


def _resource_field(container, ref):
    res = container.get("resources") or {}
    r = ref["resource"]
    kind, name = r.split(".", 1)
    q = (res.get(kind) or {}).get(name)
    if q is None and kind == "requests":
        q = (res.get("limits") or {}).get(name)
    if q is None:
        return "0"
    v = parse_quantity(str(q)).value / parse_quantity(str(ref.get("divisor", "1"))).value   # Fractions
    # round up like the reference (ExtractResourceValueByContainerName)
    return str(-(-v.numerator // v.denominator))


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
                if (v["emptyDir"] or {}).get("medium") == "Memory" and os.path.isdir("/dev/shm"):
                    d = os.path.join("/dev/shm", "kamd-" + pod["metadata"]["uid"], name)
                os.makedirs(d, exist_ok=True)
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
                for src in v["projected"].get("sources") or ():
                    if "configMap" in src or "secret" in src:
                        await self._cm_secret(ns, src, d)
                    elif "downwardAPI" in src:
                        self._downward(pod, src["downwardAPI"], d, node_name, pod_ip)
            else:
                raise VolumeError(f"volume {name}: unsupported volume source {sorted(k for k in v if k != 'name')}")
            out[name] = d
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

    async def _cm_secret(self, ns, v, d):
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
        _write_files(d, data, src.get("items"), int(src.get("defaultMode", 0o644)), binary)

    def _downward(self, pod, spec, d, node_name, pod_ip):
        data = {}
        items = []
        for it in spec.get("items") or ():
            if "fieldRef" in it:
                data[it["path"]] = _field(pod, it["fieldRef"]["fieldPath"], node_name, pod_ip)
            items.append({"key": it["path"], "path": it["path"]})
        _write_files(d, data, items, int(spec.get("defaultMode", 0o644)))

    def mounts_for(self, container, vols: dict):
        out = []
        for m in container.get("volumeMounts") or ():
            hp = vols.get(m["name"])
            if hp is None:
                raise VolumeError(f"volumeMount {m['name']!r} refers to no pod volume")
            if m.get("subPath"):
                hp = os.path.join(hp, m["subPath"])
                os.makedirs(hp, exist_ok=True)
            out.append({"containerPath": m["mountPath"], "hostPath": hp, "readOnly": bool(m.get("readOnly"))})
        return out

    def teardown(self, pod):
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

        def put(k, v):
            if k not in env:
                order.append(k)
            env[k] = v
        for e in base_env:
            put(e["name"], e["value"])
        for ef in container.get("envFrom") or ():
            pre = ef.get("prefix", "")
            if "configMapRef" in ef:
                r = ef["configMapRef"]
                obj = await self._get("configmaps", ns, r["name"], r.get("optional"))
                for k, v in ((obj or {}).get("data") or {}).items():
                    put(pre + k, str(v))
            elif "secretRef" in ef:
                r = ef["secretRef"]
                obj = await self._get("secrets", ns, r["name"], r.get("optional"))
                for k, v in ((obj or {}).get("data") or {}).items():
                    put(pre + k, base64.b64decode(v).decode(errors="replace"))
        for e in container.get("env") or ():
            name = e["name"]
            if "value" in e:
                val = re.sub(r"\$\(([A-Za-z_][A-Za-z0-9_]*)\)", lambda m: env.get(m.group(1), m.group(0)), str(e["value"]))
                put(name, val)
                continue
            vf = e.get("valueFrom") or {}
            if "fieldRef" in vf:
                put(name, _field(pod, vf["fieldRef"]["fieldPath"], node_name, pod_ip))
            elif "resourceFieldRef" in vf:
                put(name, _resource_field(container, vf["resourceFieldRef"]))
            elif "configMapKeyRef" in vf:
                r = vf["configMapKeyRef"]
                obj = await self._get("configmaps", ns, r["name"], r.get("optional"))
                if obj is not None:
                    if r["key"] not in (obj.get("data") or {}):
                        if not r.get("optional"):
                            raise VolumeError(f"configmap {r['name']} has no key {r['key']}")
                    else:
                        put(name, str(obj["data"][r["key"]]))
            elif "secretKeyRef" in vf:
                r = vf["secretKeyRef"]
                obj = await self._get("secrets", ns, r["name"], r.get("optional"))
                if obj is not None:
                    if r["key"] not in (obj.get("data") or {}):
                        if not r.get("optional"):
                            raise VolumeError(f"secret {r['name']} has no key {r['key']}")
                    else:
                        put(name, base64.b64decode(obj["data"][r["key"]]).decode(errors="replace"))
        return [{"name": k, "value": env[k]} for k in order]
