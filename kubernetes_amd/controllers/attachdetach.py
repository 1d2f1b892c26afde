"""Attach/detach controller and the CSI external attacher.

Parity:
  * `pkg/controller/volume/attachdetach/attach_detach_controller.go` (desired state = volumes of
    scheduled, non-terminated pods per node; the reconciler attaches what is desired and not
    attached, detaches what is attached and no longer desired; `node.status.volumesAttached`
    is maintained from the actual state) with the CSI attacher of
    `pkg/volume/csi/csi_attacher.go` (an attach is a `storage.k8s.io/v1beta1` VolumeAttachment
    named `csi-<sha256(pv + driver + node)>`, `spec{attacher, nodeName,
    source.persistentVolumeName}`; attached when `status.attached` is true).
  * the external-attacher sidecar (kubernetes-csi/external-attacher, paired with the alpha CSI
    support in 1.9): VolumeAttachments for its driver → `ControllerPublishVolume` → status
    `attached: true` + `attachmentMetadata`; a deleted attachment → `ControllerUnpublishVolume`.
"""
from __future__ import annotations

from ..csi.driver import volume_attributes

import logging

from ..client.rest import APIStatusError, is_not_found
from ..csi import api as CSI
from .base import Controller

VA = "volumeattachments"
log = logging.getLogger("attachdetach")


def csi_source(pv):
    return ((pv or {}).get("spec") or {}).get("csi")


CONTROLLER_MANAGED_ATTACH = "volumes.kubernetes.io/controller-managed-attach-detach"
KEEP_TERMINATED_POD_VOLUMES = "volumes.kubernetes.io/keep-terminated-pod-volumes"


def unique_volume_name(driver, handle):
    """`GetUniqueVolumeNameFromSpec` for CSI: `kubernetes.io/csi/<driver>^<handle>`."""
    return f"kubernetes.io/csi/{driver}^{handle}"


def multi_attach_forbidden(pv):
    """`isMultiAttachForbidden`: a PV whose access modes are all single-node (no ROX / RWX)."""
    modes = ((pv or {}).get("spec") or {}).get("accessModes") or ()
    return bool(modes) and not any(md in ("ReadWriteMany", "ReadOnlyMany") for md in modes)


class AttachDetachController(Controller):
    """`pkg/controller/volume/attachdetach`: desired state = the attachable (CSI) volumes of
    scheduled, non-terminated pods on nodes that hand attach/detach to the controller (the
    kubelet's `controller-managed-attach-detach` annotation; `keep-terminated-pod-volumes`
    keeps a terminated pod's volumes attached); actual state = the VolumeAttachments. The
    reconciler (`reconciler.go`):

      * detaches what is attached but no longer desired only once the node no longer reports
        the volume in `status.volumesInUse` — or, after `max_wait_for_unmount` (6 min), anyway
        (a force detach, logged);
      * attaches what is desired and not attached, except a single-node (RWO) volume already
        attached to another node: a Multi-Attach error event (FailedAttachVolume) on the pods
        that want it;
      * keeps `node.status.volumesAttached` equal to the attached set of every managed node
        (an empty list once the last volume is gone)."""
    name = "attachdetach"
    workers = 1
    disable_reconcile_sync = False   # --disable-attach-detach-reconcile-sync
    max_wait_for_unmount = 360.0     # reconciler maxWaitForUnmountDuration

    def resync_keys(self):
        return [] if self.disable_reconcile_sync else ["reconcile"]

    def setup(self):
        self.pods = self.factory.get("pods")
        self.pvcs = self.factory.get("persistentvolumeclaims")
        self.pvs = self.factory.get("persistentvolumes")
        self.vas = self.factory.get(VA)
        self.nodes = self.factory.get("nodes")
        self.detach_requested: dict[str, float] = {}     # attachment -> first time it was undesired
        self.multi_attach_reported: set = set()
        kick = lambda *a: self.enqueue("reconcile")   # noqa: E731 - one global reconcile key
        for inf in (self.pods, self.pvcs, self.pvs, self.vas, self.nodes):
            inf.add_handler(kick, kick, kick)

    def _managed(self, node_name):
        node = self.nodes.get(node_name)
        return node is not None and CONTROLLER_MANAGED_ATTACH in ((node.get("metadata") or {}).get("annotations") or {})

    def desired(self):
        """{attachment name: (pv name, driver, node, [pods])} for scheduled pods on managed
        nodes."""
        out = {}
        for p in self.pods.list():
            node = (p.get("spec") or {}).get("nodeName")
            if not node or not self._managed(node):
                continue
            phase = (p.get("status") or {}).get("phase")
            keep = ((self.nodes.get(node) or {}).get("metadata") or {}).get("annotations", {}).get(
                KEEP_TERMINATED_POD_VOLUMES) == "true"
            if phase in ("Succeeded", "Failed") and not keep:
                continue
            ns = p["metadata"].get("namespace", "default")
            for v in (p.get("spec") or {}).get("volumes") or ():
                claim = (v.get("persistentVolumeClaim") or {}).get("claimName")
                if not claim:
                    continue
                pvc = self.pvcs.get(f"{ns}/{claim}")
                vol = ((pvc or {}).get("spec") or {}).get("volumeName")
                src = csi_source(self.pvs.get(vol)) if vol else None
                if src:
                    ent = out.setdefault(CSI.attachment_name(vol, src["driver"], node), (vol, src["driver"], node, []))
                    ent[3].append(p)
        return out

    def _in_use(self, node_name, pv_name):
        src = csi_source(self.pvs.get(pv_name)) or {}
        name = unique_volume_name(src.get("driver", ""), src.get("volumeHandle", ""))
        return name in (((self.nodes.get(node_name) or {}).get("status") or {}).get("volumesInUse") or ())

    async def sync(self, key):
        import time as _time
        now = _time.monotonic()
        want = self.desired()
        have = {va["metadata"]["name"]: va for va in self.vas.list()}
        requeue = None
        # detach: attached, no longer desired, and not mounted (or waited long enough)
        for name, va in have.items():
            if not name.startswith("csi-") or name in want or va["metadata"].get("deletionTimestamp"):
                continue
            node, pv = va["spec"].get("nodeName"), (va["spec"].get("source") or {}).get("persistentVolumeName", "")
            since = self.detach_requested.setdefault(name, now)
            timed_out = now - since > self.max_wait_for_unmount
            if self._in_use(node, pv) and not timed_out:
                left = self.max_wait_for_unmount - (now - since)
                requeue = left if requeue is None else min(requeue, left)
                continue
            if timed_out:
                log.warning("volume %s is not safe to detach from %s, but maxWaitForUnmountDuration %.0fs expired: "
                            "force detaching", pv, node, self.max_wait_for_unmount)
            try:
                await self.client.delete(VA, name)
            except APIStatusError as e:
                if not is_not_found(e):
                    raise
            self.detach_requested.pop(name, None)
        # attach what is desired and not attached (single-node volumes once only)
        attached_nodes: dict = {}
        for va in have.values():
            if not va["metadata"].get("deletionTimestamp"):
                attached_nodes.setdefault((va["spec"].get("source") or {}).get("persistentVolumeName"), set()).add(
                    va["spec"].get("nodeName"))
        for name, (pv, driver, node, pods) in want.items():
            self.detach_requested.pop(name, None)
            if name in have:
                continue
            others = attached_nodes.get(pv, set()) - {node}
            if others and multi_attach_forbidden(self.pvs.get(pv)):
                if name not in self.multi_attach_reported:
                    self.multi_attach_reported.add(name)
                    for p in pods:
                        self.recorder.event(p, "Warning", "FailedAttachVolume",
                                            f'Multi-Attach error for volume "{pv}" Volume is already exclusively '
                                            f"attached to one node and can't be attached to another")
                continue
            self.multi_attach_reported.discard(name)
            try:
                await self.client.create(VA, {"apiVersion": "storage.k8s.io/v1beta1", "kind": "VolumeAttachment",
                                              "metadata": {"name": name},
                                              "spec": {"attacher": driver, "nodeName": node,
                                                       "source": {"persistentVolumeName": pv}}})
            except APIStatusError as e:
                if e.code != 409:
                    raise
            attached_nodes.setdefault(pv, set()).add(node)
        await self._update_node_statuses()
        if requeue is not None:
            self.queue.add_after("reconcile", max(0.05, requeue))

    async def _update_node_statuses(self):
        """node.status.volumesAttached from the actual state, for every managed node."""
        per_node: dict = {}
        for va in self.vas.list():
            if (va.get("status") or {}).get("attached") and not va["metadata"].get("deletionTimestamp"):
                pv = self.pvs.get(va["spec"]["source"].get("persistentVolumeName", ""))
                src = csi_source(pv) or {}
                per_node.setdefault(va["spec"]["nodeName"], []).append(
                    {"name": unique_volume_name(va["spec"]["attacher"], src.get("volumeHandle", "")),
                     "devicePath": (va["status"].get("attachmentMetadata") or {}).get("devicePath", "")})
        for node in self.nodes.list():
            nn = node["metadata"]["name"]
            if CONTROLLER_MANAGED_ATTACH not in (node["metadata"].get("annotations") or {}):
                continue
            vols = sorted(per_node.get(nn, []), key=lambda v: v["name"])
            if ((node.get("status") or {}).get("volumesAttached") or []) == vols:
                continue
            try:
                await self.client.patch("nodes", nn, {"status": {"volumesAttached": vols or None}}, None, "merge",
                                        "status")
            except APIStatusError as e:
                if not is_not_found(e):
                    raise


class ExternalAttacher(Controller):
    """Sidecar next to a CSI controller plugin (runs per driver, not in the controller manager)."""
    name = "csi-attacher"
    workers = 1

    def __init__(self, client, factory, driver=None, endpoint=None, **kw):
        super().__init__(client, factory, **kw)
        self.driver, self.endpoint = driver, endpoint
        self.csi = None
        self.published: dict[str, tuple] = {}     # attachment -> (volume handle, node)

    def setup(self):
        self.vas = self.factory.get(VA)
        self.pvs = self.factory.get("persistentvolumes")
        self.vas.add_handler(lambda va: self.enqueue(va["metadata"]["name"]),
                             lambda o, n: self.enqueue(n["metadata"]["name"]),
                             lambda va: self.enqueue(va["metadata"]["name"]))

    async def sync(self, key):
        from ..csi.driver import CSIClient
        if self.csi is None:
            self.csi = CSIClient(self.endpoint)
        va = self.vas.get(key)
        if va is None or va["metadata"].get("deletionTimestamp"):
            pub = self.published.pop(key, None)
            if pub is not None:
                await self.csi.controller_unpublish(*pub)
            return
        if va["spec"].get("attacher") != self.driver or (va.get("status") or {}).get("attached"):
            return
        pv = self.pvs.get(va["spec"]["source"].get("persistentVolumeName", ""))
        src = csi_source(pv)
        if not src:
            return
        try:
            info = await self.csi.controller_publish(src["volumeHandle"], va["spec"]["nodeName"], bool(src.get("readOnly")),
                                                     volume_attributes(pv), (pv.get("spec") or {}).get("accessModes"))
        except Exception as e:  # noqa: BLE001 - reported in status.attachError, retried
            await self.client.patch(VA, key, {"status": {"attached": False, "attachError": {"message": str(e)}}}, None,
                                    "merge", "status")
            raise
        self.published[key] = (src["volumeHandle"], va["spec"]["nodeName"])
        await self.client.patch(VA, key, {"status": {"attached": True, "attachmentMetadata": info}}, None, "merge", "status")

    def stop(self):
        super().stop()
        if self.csi is not None:
            from ..utils.tasks import spawn
            spawn(self.csi.close())
