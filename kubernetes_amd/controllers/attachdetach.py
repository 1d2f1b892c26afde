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

from ..client.rest import APIStatusError, is_not_found
from ..csi import api as CSI
from .base import Controller

VA = "volumeattachments"


def csi_source(pv):
    return ((pv or {}).get("spec") or {}).get("csi")


class AttachDetachController(Controller):
    name = "attachdetach"
    workers = 1
    disable_reconcile_sync = False   # --disable-attach-detach-reconcile-sync

    def resync_keys(self):
        return [] if self.disable_reconcile_sync else ["reconcile"]

    def setup(self):
        self.pods = self.factory.get("pods")
        self.pvcs = self.factory.get("persistentvolumeclaims")
        self.pvs = self.factory.get("persistentvolumes")
        self.vas = self.factory.get(VA)
        kick = lambda *a: self.enqueue("reconcile")   # noqa: E731 - one global reconcile key
        for inf in (self.pods, self.pvcs, self.pvs, self.vas):
            inf.add_handler(kick, kick, kick)

    def desired(self):
        """{attachment name: (pv name, driver, node)} for scheduled, live pods."""
        out = {}
        for p in self.pods.list():
            node = (p.get("spec") or {}).get("nodeName")
            phase = (p.get("status") or {}).get("phase")
            if not node or phase in ("Succeeded", "Failed"):
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
                    out[CSI.attachment_name(vol, src["driver"], node)] = (vol, src["driver"], node)
        return out

    async def sync(self, key):
        want = self.desired()
        have = {va["metadata"]["name"]: va for va in self.vas.list()}
        for name, (pv, driver, node) in want.items():
            if name in have:
                continue
            try:
                await self.client.create(VA, {"apiVersion": "storage.k8s.io/v1beta1", "kind": "VolumeAttachment",
                                              "metadata": {"name": name},
                                              "spec": {"attacher": driver, "nodeName": node,
                                                       "source": {"persistentVolumeName": pv}}})
            except APIStatusError as e:
                if e.code != 409:
                    raise
        for name, va in have.items():
            if name.startswith("csi-") and name not in want and not va["metadata"].get("deletionTimestamp"):
                try:
                    await self.client.delete(VA, name)
                except APIStatusError as e:
                    if not is_not_found(e):
                        raise
        # node.status.volumesAttached from the actual state
        per_node = {}
        for va in self.vas.list():
            if (va.get("status") or {}).get("attached"):
                pv = self.pvs.get(va["spec"]["source"].get("persistentVolumeName", ""))
                src = csi_source(pv) or {}
                per_node.setdefault(va["spec"]["nodeName"], []).append(
                    {"name": f"kubernetes.io/csi/{va['spec']['attacher']}^{src.get('volumeHandle', '')}",
                     "devicePath": (va["status"].get("attachmentMetadata") or {}).get("devicePath", "")})
        for node, vols in per_node.items():
            try:
                await self.client.patch("nodes", node, {"status": {"volumesAttached": sorted(vols, key=lambda v: v["name"])}},
                                        None, "merge", "status")
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
