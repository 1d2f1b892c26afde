"""PersistentVolume binder / provisioner / reclaimer and PVC protection.

Parity: `pkg/controller/volume/persistentvolume/pv_controller.go`:
  * `syncClaim` — an unbound claim binds to the smallest Available volume that satisfies it
    (same storageClassName, access modes superset, capacity >= request, label selector,
    volumeMode) — `index.go findBestMatchForClaim`; pre-bound volumes (`claimRef`) / claims
    (`volumeName`) are honoured; the bind writes `pv.spec.claimRef` + `pv.status.phase=Bound`,
    then `pvc.spec.volumeName` + annotation `pv.kubernetes.io/bind-completed` + `Bound` status;
  * dynamic provisioning — no match and the claim's StorageClass has a provisioner this
    controller runs (`kubernetes.io/host-path`, like the reference's hostpath provisioner used by
    local-up-cluster, `pkg/volume/host_path/host_path.go` Provisioner): a hostPath PV is created
    pre-bound to the claim with the class's reclaimPolicy (default Delete);
  * `syncVolume` — a Bound volume whose claim disappeared becomes Released; reclaimPolicy
    Delete deletes it (and its provisioned directory), Recycle scrubs it back to Available,
    Retain leaves it Released;
  * `pkg/controller/volume/pvcprotection` — finalizer `kubernetes.io/pvc-protection` on every
    claim, removed only once no active pod uses the claim.
"""
from __future__ import annotations

import json
import os
import shutil

from ..api.labels import label_selector_as_selector
from ..api.quantity import parse_quantity
from ..client.rest import APIStatusError, is_not_found
from .base import Controller, split_key

# the 1.9 alpha PV node-affinity annotation (spec.nodeAffinity is 1.10+); read by scheduler/volumes.py
NODE_AFFINITY_ANN = "volume.alpha.kubernetes.io/node-affinity"

BIND_COMPLETED = "pv.kubernetes.io/bind-completed"
BOUND_BY_CONTROLLER = "pv.kubernetes.io/bound-by-controller"
PROVISIONED_BY = "pv.kubernetes.io/provisioned-by"
HOSTPATH_PROVISIONER = "kubernetes.io/host-path"
PVC_PROTECTION = "kubernetes.io/pvc-protection"
SELECTED_NODE = "volume.kubernetes.io/selected-node"


def md_ann(o):
    return o["metadata"].get("annotations") or {}


def _cap(obj, path):
    q = ((obj.get("spec") or {}).get(path) or {}).get("storage") if path == "capacity" else \
        (((obj.get("spec") or {}).get("resources") or {}).get("requests") or {}).get("storage")
    return parse_quantity(str(q)).value if q is not None else 0


def claim_class(pvc):
    sp = pvc.get("spec") or {}
    return sp.get("storageClassName") or (pvc["metadata"].get("annotations") or {}).get(
        "volume.beta.kubernetes.io/storage-class", "")


def volume_class(pv):
    sp = pv.get("spec") or {}
    return sp.get("storageClassName") or (pv["metadata"].get("annotations") or {}).get(
        "volume.beta.kubernetes.io/storage-class", "")


def matches(pv, pvc):
    sp, cs = pv.get("spec") or {}, pvc.get("spec") or {}
    if volume_class(pv) != claim_class(pvc):
        return False
    if not set(cs.get("accessModes") or ()) <= set(sp.get("accessModes") or ()):
        return False
    if _cap(pv, "capacity") < _cap(pvc, "requests"):
        return False
    if (sp.get("volumeMode") or "Filesystem") != (cs.get("volumeMode") or "Filesystem"):
        return False
    sel = cs.get("selector")
    if sel and not label_selector_as_selector(sel).matches(pv["metadata"].get("labels") or {}):
        return False
    return True


def best_match(pvs, pvc):
    cands = [pv for pv in pvs if (pv.get("status") or {}).get("phase", "Available") == "Available"
             and not (pv.get("spec") or {}).get("claimRef") and matches(pv, pvc)]
    cands.sort(key=lambda pv: (_cap(pv, "capacity"), pv["metadata"]["name"]))
    return cands[0] if cands else None


class PersistentVolumeController(Controller):
    name = "persistentvolume-binder"
    workers = 1      # binding decisions are serialized, like the reference's single sync loop

    def __init__(self, client, factory, hostpath_root=None, enable_dynamic_provisioning=True, **kw):
        super().__init__(client, factory, **kw)
        self.hostpath_root = hostpath_root or os.path.join(os.environ.get("TMPDIR", "/tmp"), "kamd-hostpath-pv")
        # --enable-dynamic-provisioning=false: claims only bind to existing volumes
        self.enable_dynamic_provisioning = enable_dynamic_provisioning

    def resync_keys(self):
        return (["claim:" + _key(c) for c in self.pvc_inf.list()] +
                ["volume:" + v["metadata"]["name"] for v in self.pv_inf.list()])

    def setup(self):
        self.pv_inf = self.factory.get("persistentvolumes")
        self.pvc_inf = self.factory.get("persistentvolumeclaims")
        self.sc_inf = self.factory.get("storageclasses")
        self.pvc_inf.add_handler(lambda c: self.enqueue("claim:" + _key(c)), lambda o, n: self.enqueue("claim:" + _key(n)),
                                 self._claim_deleted)
        self.pv_inf.add_handler(self._pv_event, lambda o, n: self._pv_event(n), None)

    def _claim_deleted(self, pvc):
        for pv in self.pv_inf.list():
            ref = (pv.get("spec") or {}).get("claimRef") or {}
            if ref.get("uid") == pvc["metadata"].get("uid"):
                self.enqueue("volume:" + pv["metadata"]["name"])

    def _pv_event(self, pv):
        self.enqueue("volume:" + pv["metadata"]["name"])
        for c in self.pvc_inf.list():
            if (c.get("status") or {}).get("phase") != "Bound":
                self.enqueue("claim:" + _key(c))

    async def sync(self, key):
        kind, _, k = key.partition(":")
        if kind == "claim":
            await self.sync_claim(k)
        else:
            await self.sync_volume(k)

    async def sync_claim(self, key):
        pvc = self.pvc_inf.get(key)
        if pvc is None or pvc["metadata"].get("deletionTimestamp"):
            return
        ns, name = split_key(key)
        sp = pvc.get("spec") or {}
        if (pvc.get("status") or {}).get("phase") == "Bound" and sp.get("volumeName"):
            pv = self.pv_inf.get(sp["volumeName"])
            if pv is not None and ((pv.get("spec") or {}).get("claimRef") or {}).get("uid") == pvc["metadata"]["uid"]:
                return
        pv = None
        if sp.get("volumeName"):
            pv = self.pv_inf.get(sp["volumeName"])
            if pv is None:
                await self._claim_status(pvc, "Pending")
                return
        else:
            for cand in self.pv_inf.list():     # pre-bound volume waiting for this claim
                ref = (cand.get("spec") or {}).get("claimRef") or {}
                if ref.get("namespace") == ns and ref.get("name") == name and ref.get("uid") in (None, "", pvc["metadata"]["uid"]):
                    pv = cand
                    break
            if pv is None and self._delayed(pvc):
                # WaitForFirstConsumer: the scheduler picks the PV (claimRef) or the node
                # (selected-node annotation) once a consuming pod is placed
                if not (md_ann(pvc).get(SELECTED_NODE)):
                    await self._claim_status(pvc, "Pending")
                    return
            elif pv is None:
                pv = best_match(self.pv_inf.list(), pvc)
        if pv is None:
            pv = await self._provision(pvc)
            if pv is None:
                await self._claim_status(pvc, "Pending")
                return
        await self._bind(pv, pvc)

    def _delayed(self, pvc):
        sc = self.sc_inf.get(claim_class(pvc)) if claim_class(pvc) else None
        return bool(sc) and sc.get("volumeBindingMode") == "WaitForFirstConsumer"

    async def _claim_status(self, pvc, phase):
        if (pvc.get("status") or {}).get("phase") != phase:
            await self.client.patch("persistentvolumeclaims", pvc["metadata"]["name"], {"status": {"phase": phase}},
                                    pvc["metadata"]["namespace"], "merge", "status")

    async def _provision(self, pvc):
        if not self.enable_dynamic_provisioning:
            return None
        cls = claim_class(pvc)
        sc = self.sc_inf.get(cls) if cls else None
        if sc is None or sc.get("provisioner") != HOSTPATH_PROVISIONER:
            return None
        md = pvc["metadata"]
        name = f"pvc-{md['uid']}"
        path = os.path.join(self.hostpath_root, name)
        os.makedirs(path, exist_ok=True)
        sp = pvc.get("spec") or {}
        ann = {PROVISIONED_BY: HOSTPATH_PROVISIONER}
        if md_ann(pvc).get(SELECTED_NODE):
            # node-pinned volume: the 1.9 alpha node-affinity annotation (v1.NodeAffinity JSON,
            # staging/src/k8s.io/api/core/v1/types.go:464) — spec.nodeAffinity is 1.10+
            ann[NODE_AFFINITY_ANN] = json.dumps({"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [
                {"matchExpressions": [{"key": "kubernetes.io/hostname", "operator": "In",
                                       "values": [md_ann(pvc)[SELECTED_NODE]]}]}]}})
        pv = {"apiVersion": "v1", "kind": "PersistentVolume",
              "metadata": {"name": name, "annotations": ann},
              "spec": {"capacity": {"storage": ((sp.get("resources") or {}).get("requests") or {}).get("storage", "1Gi")},
                       "accessModes": sp.get("accessModes") or ["ReadWriteOnce"],
                       "persistentVolumeReclaimPolicy": sc.get("reclaimPolicy") or "Delete",
                       "storageClassName": cls, "hostPath": {"path": path},
                       "claimRef": {"kind": "PersistentVolumeClaim", "apiVersion": "v1", "namespace": md["namespace"],
                                    "name": md["name"], "uid": md["uid"]}}}
        try:
            return await self.client.create("persistentvolumes", pv)
        except APIStatusError as e:
            if e.code == 409:
                return await self.client.get("persistentvolumes", name)
            raise

    async def _bind(self, pv, pvc):
        md = pvc["metadata"]
        ref = {"kind": "PersistentVolumeClaim", "apiVersion": "v1", "namespace": md["namespace"], "name": md["name"],
               "uid": md["uid"], "resourceVersion": md.get("resourceVersion", "")}
        if ((pv.get("spec") or {}).get("claimRef") or {}).get("uid") != md["uid"] or (pv.get("status") or {}).get("phase") != "Bound":
            pv = await self.client.patch("persistentvolumes", pv["metadata"]["name"],
                                         {"metadata": {"annotations": {BOUND_BY_CONTROLLER: "yes"}}, "spec": {"claimRef": ref}})
            await self.client.patch("persistentvolumes", pv["metadata"]["name"], {"status": {"phase": "Bound"}}, None,
                                    "merge", "status")
        await self.client.patch("persistentvolumeclaims", md["name"],
                                {"metadata": {"annotations": {BIND_COMPLETED: "yes", BOUND_BY_CONTROLLER: "yes"}},
                                 "spec": {"volumeName": pv["metadata"]["name"]}}, md["namespace"])
        await self.client.patch("persistentvolumeclaims", md["name"], {"status": {
            "phase": "Bound", "accessModes": (pv.get("spec") or {}).get("accessModes") or [],
            "capacity": (pv.get("spec") or {}).get("capacity") or {}}}, md["namespace"], "merge", "status")

    async def sync_volume(self, name):
        pv = self.pv_inf.get(name)
        if pv is None:
            return
        sp = pv.get("spec") or {}
        ref = sp.get("claimRef")
        phase = (pv.get("status") or {}).get("phase", "Available")
        if not ref:
            if phase != "Available":
                await self.client.patch("persistentvolumes", name, {"status": {"phase": "Available"}}, None, "merge", "status")
            return
        pvc = self.pvc_inf.get(f"{ref.get('namespace')}/{ref.get('name')}")
        if pvc is not None and (not ref.get("uid") or pvc["metadata"].get("uid") == ref.get("uid")):
            return
        if pvc is None and phase == "Available" and not ref.get("uid"):
            return     # pre-bound to a claim that does not exist yet
        # claim is gone: release and reclaim
        if phase != "Released":
            await self.client.patch("persistentvolumes", name, {"status": {"phase": "Released"}}, None, "merge", "status")
        policy = sp.get("persistentVolumeReclaimPolicy") or "Retain"
        if policy == "Delete":
            if (pv["metadata"].get("annotations") or {}).get(PROVISIONED_BY) == HOSTPATH_PROVISIONER:
                p = (sp.get("hostPath") or {}).get("path", "")
                if p.startswith(self.hostpath_root):
                    shutil.rmtree(p, ignore_errors=True)
            try:
                await self.client.delete("persistentvolumes", name)
            except APIStatusError as e:
                if not is_not_found(e):
                    raise
        elif policy == "Recycle":
            p = (sp.get("hostPath") or {}).get("path", "")
            if p and os.path.isdir(p):
                for entry in os.listdir(p):
                    full = os.path.join(p, entry)
                    shutil.rmtree(full, ignore_errors=True) if os.path.isdir(full) else os.unlink(full)
            await self.client.patch("persistentvolumes", name, {"spec": {"claimRef": None}})
            await self.client.patch("persistentvolumes", name, {"status": {"phase": "Available"}}, None, "merge", "status")


class ExpandController(Controller):
    """`pkg/controller/volume/expand/expand_controller.go`: a bound claim whose requested size
    exceeds `status.capacity` is expanded — the volume plugin grows the backing volume
    (`ExpandVolumeDevice`; host-path and local volumes are directories, so that is a no-op,
    CSI volumes would call the driver), the PV's `spec.capacity` is raised, and the claim's
    `status.capacity` is updated. Volumes that need a file-system resize on the node get the
    `FileSystemResizePending` condition instead, which the kubelet clears after resizing."""
    name = "expand"
    workers = 1
    FS_RESIZE = ()       # plugin kinds whose file system is grown by the kubelet after the device

    def setup(self):
        self.pvc_inf = self.factory.get("persistentvolumeclaims")
        self.pv_inf = self.factory.get("persistentvolumes")
        self.pvc_inf.add_handler(self._maybe, lambda o, n: self._maybe(n), None)

    def _maybe(self, pvc):
        if (pvc.get("status") or {}).get("phase") == "Bound" and _cap(pvc, "requests") > self._status_cap(pvc):
            self.enqueue("/".join((pvc["metadata"]["namespace"], pvc["metadata"]["name"])))

    @staticmethod
    def _status_cap(pvc):
        q = ((pvc.get("status") or {}).get("capacity") or {}).get("storage")
        return parse_quantity(str(q)).value if q is not None else 0

    async def sync(self, key):
        pvc = self.pvc_inf.get(key)
        if pvc is None or (pvc.get("status") or {}).get("phase") != "Bound":
            return
        want = ((pvc.get("spec") or {}).get("resources") or {}).get("requests", {}).get("storage")
        if _cap(pvc, "requests") <= self._status_cap(pvc):
            return
        pv = self.pv_inf.get((pvc.get("spec") or {}).get("volumeName", ""))
        if pv is None:
            return
        if _cap(pv, "capacity") < _cap(pvc, "requests"):
            await self.client.patch("persistentvolumes", pv["metadata"]["name"], {"spec": {"capacity": {"storage": want}}})
        ns, name = split_key(key)
        kind = next((k for k in ("hostPath", "local", "csi") if k in (pv.get("spec") or {})), "")
        if kind in self.FS_RESIZE:
            await self.client.patch("persistentvolumeclaims", name, {"status": {"conditions": [
                {"type": "FileSystemResizePending", "status": "True",
                 "message": "Waiting for user to (re-)start a pod to finish file system resize of volume on node."}]}},
                ns, "merge", "status")
            return
        await self.client.patch("persistentvolumeclaims", name, {"status": {"capacity": {"storage": want},
                                                                            "conditions": None}}, ns, "merge", "status")
        self.recorder.event(pvc, "Normal", "VolumeResizeSuccessful", f"volume {pv['metadata']['name']} resized to {want}")


class PVCProtectionController(Controller):
    name = "pvc-protection"
    workers = 1

    def setup(self):
        self.pvc_inf = self.factory.get("persistentvolumeclaims")
        self.pod_inf = self.factory.get("pods")
        self.pvc_inf.add_handler(self.enqueue, lambda o, n: self.enqueue(n), None)
        self.pod_inf.add_handler(None, lambda o, n: self._pod(n), self._pod)

    def _pod(self, pod):
        ns = pod["metadata"].get("namespace")
        for v in (pod.get("spec") or {}).get("volumes") or ():
            c = (v.get("persistentVolumeClaim") or {}).get("claimName")
            if c:
                self.enqueue(f"{ns}/{c}")

    def _in_use(self, ns, name):
        for p in self.pod_inf.list():
            if p["metadata"].get("namespace") != ns or (p.get("status") or {}).get("phase") in ("Succeeded", "Failed"):
                continue
            if any((v.get("persistentVolumeClaim") or {}).get("claimName") == name for v in (p.get("spec") or {}).get("volumes") or ()):
                return True
        return False

    async def sync(self, key):
        pvc = self.pvc_inf.get(key)
        if pvc is None:
            return
        ns, name = split_key(key)
        fins = list(pvc["metadata"].get("finalizers") or [])
        if pvc["metadata"].get("deletionTimestamp"):
            if PVC_PROTECTION in fins and not self._in_use(ns, name):
                fins.remove(PVC_PROTECTION)
                await self.client.patch("persistentvolumeclaims", name, {"metadata": {"finalizers": fins}}, ns)
            return
        if PVC_PROTECTION not in fins:
            await self.client.patch("persistentvolumeclaims", name, {"metadata": {"finalizers": fins + [PVC_PROTECTION]}}, ns)


def _key(o):
    return f"{o['metadata'].get('namespace', '')}/{o['metadata']['name']}"
