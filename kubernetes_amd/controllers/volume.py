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
import re
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
PV_PROTECTION = "kubernetes.io/pv-protection"      # `pkg/volume/util/finalizer.go:28`
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


def volume_mode_mismatch(pv, pvc) -> bool:
    return ((pv.get("spec") or {}).get("volumeMode") or "Filesystem") != \
        ((pvc.get("spec") or {}).get("volumeMode") or "Filesystem")


def check_volume_satisfy_claim(pv, pvc):
    """`checkVolumeSatisfyClaim`: an error message, or None."""
    if _cap(pv, "capacity") < _cap(pvc, "requests"):
        return f"Storage capacity of volume[{pv['metadata']['name']}] requested by claim[{_key(pvc)}] is not enough"
    if volume_class(pv) != claim_class(pvc):
        return f"Class of volume[{pv['metadata']['name']}] is not the same as claim[{_key(pvc)}]"
    if volume_mode_mismatch(pv, pvc):
        return f"VolumeMode of volume[{pv['metadata']['name']}] is incompatible with VolumeMode of claim[{_key(pvc)}]"
    return None


def is_volume_bound_to_claim(pv, pvc) -> bool:
    """`isVolumeBoundToClaim`: the claimRef names the claim (with its UID, or no UID yet)."""
    ref = (pv.get("spec") or {}).get("claimRef")
    if not ref:
        return False
    md = pvc["metadata"]
    return ref.get("name") == md["name"] and ref.get("namespace") == md.get("namespace") and \
        ref.get("uid") in (None, "", md.get("uid"))


def matches(pv, pvc):
    """An unclaimed volume that would satisfy the claim (class, access modes, size, mode,
    selector) — the scheduler's volume binder uses this too."""
    sp, cs = pv.get("spec") or {}, pvc.get("spec") or {}
    if volume_class(pv) != claim_class(pvc):
        return False
    if not set(cs.get("accessModes") or ()) <= set(sp.get("accessModes") or ()):
        return False
    if _cap(pv, "capacity") < _cap(pvc, "requests"):
        return False
    if volume_mode_mismatch(pv, pvc):
        return False
    sel = cs.get("selector")
    if sel and not label_selector_as_selector(sel).matches(pv["metadata"].get("labels") or {}):
        return False
    return True


def _find_matching_volume(pvs, pvc, delay_binding):
    """`findMatchingVolume` over one access-mode group: a volume pre-bound to the claim wins if
    it is big enough; otherwise (unless binding waits for the first consumer) the smallest
    unclaimed volume of the claim's class matching its selector."""
    want = _cap(pvc, "requests")
    cls = claim_class(pvc)
    sel = (pvc.get("spec") or {}).get("selector")
    selector = label_selector_as_selector(sel) if sel else None
    best = None
    for pv in pvs:
        if volume_mode_mismatch(pv, pvc):
            continue
        size = _cap(pv, "capacity")
        if is_volume_bound_to_claim(pv, pvc):
            if size < want:
                continue
            return pv
        if delay_binding:
            continue          # the scheduler picks the volume together with the node
        if (pv.get("spec") or {}).get("claimRef"):
            continue
        if selector is not None and not selector.matches(pv["metadata"].get("labels") or {}):
            continue
        if volume_class(pv) != cls:
            continue
        if size >= want and (best is None or size < _cap(best, "capacity")):
            best = pv
    return best


def best_match(pvs, pvc, delay_binding=False):
    """`findBestMatchForClaim` (index.go): volumes grouped by their access-mode set; the groups
    that include every mode the claim asks for are tried fewest-modes first, so a claim gets the
    most specific volume kind before a more capable one."""
    want = set((pvc.get("spec") or {}).get("accessModes") or ())
    groups: dict = {}
    for pv in pvs:
        groups.setdefault(frozenset((pv.get("spec") or {}).get("accessModes") or ()), []).append(pv)
    for modes in sorted((g for g in groups if want <= g), key=lambda g: (len(g), sorted(g))):
        pv = _find_matching_volume(sorted(groups[modes], key=lambda v: v["metadata"]["name"]), pvc, delay_binding)
        if pv is not None:
            return pv
    return None


ANN_STORAGE_PROVISIONER = "volume.beta.kubernetes.io/storage-provisioner"
_HOSTPATH_DELETABLE = re.compile(r"^/tmp/.+$")


class PersistentVolumeController(Controller):
    """`pkg/controller/volume/persistentvolume/pv_controller.go`, the same state machine:

      * syncClaim: claims without `bind-completed` go through `syncUnboundClaim` (best match,
        pre-bound volumes, provisioning through the claim's StorageClass — in-tree
        `kubernetes.io/host-path`, else the `storage-provisioner` annotation and an
        ExternalProvisioning event —, WaitForFirstConsumer, VolumeMismatch for a pre-bound
        volume that does not satisfy the claim), bound ones through `syncBoundClaim` (ClaimLost
        when the volume or the reference is gone, ClaimMisbound when the volume is someone
        else's);
      * bind: volume claimRef (+ `bound-by-controller` when the controller chose it) → volume
        Bound → claim volumeName (+ `bound-by-controller` when it chose) + `bind-completed` →
        claim Bound with the volume's access modes and capacity; every step is idempotent, so a
        crash between steps is completed by the next sync;
      * syncVolume: no claimRef / no UID → Available; claim gone (or another UID) → Released and
        reclaimed (Retain / Recycle / Delete, unknown policy → Failed); claim binding in progress
        → the claim is queued; claim bound elsewhere → a dynamically provisioned Delete volume is
        released and deleted, otherwise unbound (claimRef dropped when the controller bound it,
        only its UID when the user pre-bound it);
      * reclaim: the host-path plugin deletes / scrubs only /tmp/.+ directories (and this
        controller's own provisioning root); volumes without a deleter or recycler go Failed
        with VolumeFailedDelete / VolumeFailedRecycle."""
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
            pvc = self.pvc_inf.get(k)
            if pvc is not None:
                await self.sync_claim(pvc)
        else:
            pv = self.pv_inf.get(k)
            if pv is not None:
                await self.sync_volume(pv)

    # -- claims ------------------------------------------------------------------------------
    async def sync_claim(self, pvc):
        if BIND_COMPLETED not in md_ann(pvc):
            await self.sync_unbound_claim(pvc)
        else:
            await self.sync_bound_claim(pvc)

    def _delayed(self, pvc):
        sc = self.sc_inf.get(claim_class(pvc)) if claim_class(pvc) else None
        return bool(sc) and sc.get("volumeBindingMode") == "WaitForFirstConsumer"

    async def sync_unbound_claim(self, pvc):
        vn = (pvc.get("spec") or {}).get("volumeName")
        if not vn:
            # WaitForFirstConsumer: the scheduler pre-binds a volume (claimRef) or names the node
            # (selected-node annotation) once a consuming pod is placed
            delay = self._delayed(pvc) and not md_ann(pvc).get(SELECTED_NODE)
            pv = best_match(self.pv_inf.list(), pvc, delay)
            if pv is not None:
                await self.bind(pv, pvc)
                return
            if delay:
                self.recorder.event(pvc, "Normal", "WaitForFirstConsumer",
                                    "waiting for first consumer to be created before binding")
            elif claim_class(pvc):
                await self.provision_claim(pvc)
                return
            else:
                self.recorder.event(pvc, "Normal", "FailedBinding",
                                    "no persistent volumes available for this claim and no storage class is set")
            await self.update_claim_status(pvc, "Pending", None)
            return
        pv = self.pv_inf.get(vn)
        if pv is None:
            await self.update_claim_status(pvc, "Pending", None)
            return
        if not (pv.get("spec") or {}).get("claimRef"):
            if check_volume_satisfy_claim(pv, pvc):
                self.recorder.event(pvc, "Warning", "VolumeMismatch",
                                    "Volume's size is smaller than requested or volume's class does not match with claim")
                await self.update_claim_status(pvc, "Pending", None)
            else:
                await self.bind(pv, pvc)
        elif is_volume_bound_to_claim(pv, pvc):
            await self.bind(pv, pvc)
        elif BOUND_BY_CONTROLLER not in md_ann(pvc):
            await self.update_claim_status(pvc, "Pending", None)      # the user pre-bound it: wait
        else:
            ref = (pv.get("spec") or {}).get("claimRef") or {}
            raise RuntimeError(f"Invalid binding of claim {_key(pvc)!r} to volume {vn!r}: volume already claimed by "
                               f"{ref.get('namespace')}/{ref.get('name')}")

    async def sync_bound_claim(self, pvc):
        vn = (pvc.get("spec") or {}).get("volumeName")
        if not vn:
            await self.update_claim_status_with_event(pvc, "Lost", None, "Warning", "ClaimLost",
                                                      "Bound claim has lost reference to PersistentVolume. "
                                                      "Data on the volume is lost!")
            return
        pv = self.pv_inf.get(vn)
        if pv is None:
            await self.update_claim_status_with_event(pvc, "Lost", None, "Warning", "ClaimLost",
                                                      "Bound claim has lost its PersistentVolume. Data on the volume "
                                                      "is lost!")
            return
        ref = (pv.get("spec") or {}).get("claimRef")
        if not ref or ref.get("uid") == pvc["metadata"].get("uid"):
            await self.bind(pv, pvc)
        else:
            await self.update_claim_status_with_event(pvc, "Lost", None, "Warning", "ClaimMisbound",
                                                      "Two claims are bound to the same volume, this one is bound "
                                                      "incorrectly")

    async def update_claim_status(self, pvc, phase, pv):
        """`updateClaimStatus`: phase, and the volume's access modes / capacity (both dropped
        without a volume); written only when something changed."""
        st = pvc.get("status") or {}
        patch = {}
        if st.get("phase") != phase:
            patch["phase"] = phase
        if pv is None:
            if st.get("accessModes") is not None:
                patch["accessModes"] = None
            if st.get("capacity") is not None:
                patch["capacity"] = None
        else:
            modes = (pv.get("spec") or {}).get("accessModes")
            if st.get("accessModes") != modes:
                patch["accessModes"] = modes
            if st.get("phase") != phase:
                cap = (pv.get("spec") or {}).get("capacity") or {}
                if "storage" not in cap:
                    raise RuntimeError(f"PersistentVolume {pv['metadata']['name']!r} is without a storage capacity")
                cur = (st.get("capacity") or {}).get("storage")
                if cur is None or parse_quantity(str(cur)) != parse_quantity(str(cap["storage"])):
                    patch["capacity"] = cap
        if not patch:
            return pvc
        return await self.client.patch("persistentvolumeclaims", pvc["metadata"]["name"], {"status": patch},
                                       pvc["metadata"]["namespace"], "merge", "status")

    async def update_claim_status_with_event(self, pvc, phase, pv, etype, reason, message):
        if (pvc.get("status") or {}).get("phase") == phase:
            return pvc
        pvc = await self.update_claim_status(pvc, phase, pv)
        self.recorder.event(pvc, etype, reason, message)
        return pvc

    # -- volumes -----------------------------------------------------------------------------
    async def update_volume_phase(self, pv, phase, message=""):
        if (pv.get("status") or {}).get("phase") == phase:
            return pv
        return await self.client.patch("persistentvolumes", pv["metadata"]["name"],
                                       {"status": {"phase": phase, "message": message or None}}, None, "merge",
                                       "status")

    async def update_volume_phase_with_event(self, pv, phase, etype, reason, message):
        if (pv.get("status") or {}).get("phase") == phase:
            return pv
        pv = await self.update_volume_phase(pv, phase, message)
        self.recorder.event(pv, etype, reason, message)
        return pv

    async def bind(self, pv, pvc):
        """`bind`: the four idempotent steps, each re-read from the previous write."""
        pv = await self.bind_volume_to_claim(pv, pvc)
        pv = await self.update_volume_phase(pv, "Bound")
        pvc = await self.bind_claim_to_volume(pvc, pv)
        await self.update_claim_status(pvc, "Bound", pv)

    async def bind_volume_to_claim(self, pv, pvc):
        md = pvc["metadata"]
        ref = (pv.get("spec") or {}).get("claimRef") or {}
        patch = {}
        if (ref.get("name"), ref.get("namespace"), ref.get("uid")) != (md["name"], md.get("namespace"), md.get("uid")):
            patch["spec"] = {"claimRef": {"kind": "PersistentVolumeClaim", "apiVersion": "v1",
                                          "namespace": md["namespace"], "name": md["name"], "uid": md["uid"],
                                          "resourceVersion": md.get("resourceVersion", "")}}
        if not is_volume_bound_to_claim(pv, pvc) and BOUND_BY_CONTROLLER not in md_ann(pv):
            patch["metadata"] = {"annotations": {BOUND_BY_CONTROLLER: "yes"}}
        if not patch:
            return pv
        return await self.client.patch("persistentvolumes", pv["metadata"]["name"], patch, None, "merge")

    async def bind_claim_to_volume(self, pvc, pv):
        ann = {}
        spec = {}
        if (pvc.get("spec") or {}).get("volumeName") != pv["metadata"]["name"]:
            spec["volumeName"] = pv["metadata"]["name"]
            if BOUND_BY_CONTROLLER not in md_ann(pvc):
                ann[BOUND_BY_CONTROLLER] = "yes"
        if BIND_COMPLETED not in md_ann(pvc):
            ann[BIND_COMPLETED] = "yes"
        if not ann and not spec:
            return pvc
        patch = {}
        if ann:
            patch["metadata"] = {"annotations": ann}
        if spec:
            patch["spec"] = spec
        return await self.client.patch("persistentvolumeclaims", pvc["metadata"]["name"], patch,
                                       pvc["metadata"]["namespace"], "merge")

    async def unbind_volume(self, pv):
        """`unbindVolume`: a controller binding is undone completely; a user pre-binding keeps
        its claim name and loses only the UID."""
        if BOUND_BY_CONTROLLER in md_ann(pv):
            patch = {"spec": {"claimRef": None}, "metadata": {"annotations": {BOUND_BY_CONTROLLER: None}}}
        else:
            patch = {"spec": {"claimRef": {"uid": None}}}
        pv = await self.client.patch("persistentvolumes", pv["metadata"]["name"], patch, None, "merge")
        return await self.update_volume_phase(pv, "Available")

    async def sync_volume(self, pv):
        sp = pv.get("spec") or {}
        ref = sp.get("claimRef")
        if not ref or not ref.get("uid"):
            await self.update_volume_phase(pv, "Available")
            return
        pvc = self.pvc_inf.get(f"{ref.get('namespace')}/{ref.get('name')}")
        if pvc is not None and pvc["metadata"].get("uid") != ref.get("uid"):
            pvc = None
        phase = (pv.get("status") or {}).get("phase")
        if pvc is None:
            if phase not in ("Released", "Failed"):
                pv = await self.update_volume_phase(pv, "Released")
            await self.reclaim_volume(pv)
            return
        vn = (pvc.get("spec") or {}).get("volumeName")
        if not vn:
            self.enqueue("claim:" + _key(pvc))      # binding in progress / dangling: syncClaim fixes it
            return
        if vn == pv["metadata"]["name"]:
            await self.update_volume_phase(pv, "Bound")
            return
        if PROVISIONED_BY in md_ann(pv) and sp.get("persistentVolumeReclaimPolicy") == "Delete":
            if phase not in ("Released", "Failed"):
                pv = await self.update_volume_phase(pv, "Released")
            await self.reclaim_volume(pv)
            return
        await self.unbind_volume(pv)

    # -- reclaim -----------------------------------------------------------------------------
    async def reclaim_volume(self, pv):
        policy = (pv.get("spec") or {}).get("persistentVolumeReclaimPolicy") or "Retain"
        if policy == "Retain":
            return
        if policy == "Recycle":
            await self.recycle_volume(pv)
        elif policy == "Delete":
            await self.delete_volume(pv)
        else:
            await self.update_volume_phase_with_event(pv, "Failed", "Warning", "VolumeUnknownReclaimPolicy",
                                                      "Volume has unrecognized PersistentVolumeReclaimPolicy")

    def is_volume_released(self, pv) -> bool:
        """`isVolumeReleased`: the claimRef's claim (by UID) is gone or bound elsewhere."""
        ref = (pv.get("spec") or {}).get("claimRef") or {}
        if not ref or not ref.get("uid"):
            return False
        pvc = self.pvc_inf.get(f"{ref.get('namespace')}/{ref.get('name')}")
        if pvc is not None and pvc["metadata"].get("uid") == ref.get("uid"):
            vn = (pvc.get("spec") or {}).get("volumeName")
            return bool(vn) and vn != pv["metadata"]["name"]
        return True

    def _host_dir(self, pv):
        """The directory the host-path plugin may delete / scrub (`host_path.go`: /tmp/.+ only),
        or None."""
        p = ((pv.get("spec") or {}).get("hostPath") or {}).get("path") or ""
        if not p:
            return None
        root = os.path.realpath(self.hostpath_root)
        real = os.path.realpath(p)
        if real.startswith(root + os.sep) or _HOSTPATH_DELETABLE.match(p):
            return real
        return None

    async def delete_volume(self, pv):
        try:
            pv = await self.client.get("persistentvolumes", pv["metadata"]["name"])
        except APIStatusError:
            return
        if not self.is_volume_released(pv):
            return
        if "hostPath" not in (pv.get("spec") or {}):
            await self.update_volume_phase_with_event(
                pv, "Failed", "Warning", "VolumeFailedDelete",
                f"Error getting deleter volume plugin for volume {pv['metadata']['name']!r}: no volume plugin matched")
            return
        d = self._host_dir(pv)
        if d is None:
            await self.update_volume_phase_with_event(
                pv, "Failed", "Warning", "VolumeFailedDelete",
                f"host_path deleter only supports /tmp/.+ but received provided "
                f"{((pv.get('spec') or {}).get('hostPath') or {}).get('path')}")
            return
        shutil.rmtree(d, ignore_errors=True)
        try:
            await self.client.delete("persistentvolumes", pv["metadata"]["name"])
        except APIStatusError as e:
            if not is_not_found(e):
                raise

    async def recycle_volume(self, pv):
        try:
            pv = await self.client.get("persistentvolumes", pv["metadata"]["name"])
        except APIStatusError:
            return
        if not self.is_volume_released(pv):
            return
        d = self._host_dir(pv) if "hostPath" in (pv.get("spec") or {}) else None
        if d is None:
            await self.update_volume_phase_with_event(pv, "Failed", "Warning", "VolumeFailedRecycle",
                                                      "No recycler plugin found for the volume!")
            return
        if os.path.isdir(d):
            for entry in os.listdir(d):          # the recycler pod's `rm -rf <dir>/*`
                full = os.path.join(d, entry)
                if os.path.isdir(full) and not os.path.islink(full):
                    shutil.rmtree(full, ignore_errors=True)
                else:
                    try:
                        os.unlink(full)
                    except OSError:
                        pass
        self.recorder.event(pv, "Normal", "VolumeRecycled", "Volume recycled")
        await self.unbind_volume(pv)

    # -- provisioning ------------------------------------------------------------------------
    async def provision_claim(self, pvc):
        """`provisionClaimOperation`."""
        if not self.enable_dynamic_provisioning:
            return
        cls = claim_class(pvc)
        sc = self.sc_inf.get(cls) if cls else None
        if sc is None:
            self.recorder.event(pvc, "Warning", "ProvisioningFailed", f'storageclass.storage.k8s.io "{cls}" not found')
            return
        prov = sc.get("provisioner", "")
        if md_ann(pvc).get(ANN_STORAGE_PROVISIONER) != prov:
            pvc = await self.client.patch("persistentvolumeclaims", pvc["metadata"]["name"],
                                          {"metadata": {"annotations": {ANN_STORAGE_PROVISIONER: prov}}},
                                          pvc["metadata"]["namespace"], "merge")
        if prov != HOSTPATH_PROVISIONER:
            self.recorder.event(pvc, "Normal", "ExternalProvisioning",
                                f"waiting for a volume to be created, either by external provisioner {prov!r} or "
                                f"manually created by system administrator")
            return
        if sc.get("mountOptions"):
            self.recorder.event(pvc, "Warning", "ProvisioningFailed",
                                f"Mount options are not supported by the provisioner but StorageClass "
                                f"{sc['metadata']['name']!r} has mount options {sc['mountOptions']}")
            return
        md = pvc["metadata"]
        name = f"pvc-{md['uid']}"
        if self.pv_inf.get(name) is not None:
            return
        path = os.path.join(self.hostpath_root, name)
        os.makedirs(path, exist_ok=True)
        sp = pvc.get("spec") or {}
        ann = {PROVISIONED_BY: HOSTPATH_PROVISIONER, BOUND_BY_CONTROLLER: "yes"}
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
                                    "name": md["name"], "uid": md["uid"],
                                    "resourceVersion": md.get("resourceVersion", "")}}}
        try:
            await self.client.create("persistentvolumes", pv)
        except APIStatusError as e:
            if e.code != 409:
                self.recorder.event(pvc, "Warning", "ProvisioningFailed",
                                    f"Error creating provisioned PV object for claim {_key(pvc)}: {e}. "
                                    f"Deleting the volume.")
                shutil.rmtree(path, ignore_errors=True)
                return
        self.recorder.event(pvc, "Normal", "ProvisioningSucceeded",
                            f"Successfully provisioned volume {name} using {HOSTPATH_PROVISIONER}")


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


def pod_is_terminated(pod):
    """`volumehelper.IsPodTerminated`: Failed/Succeeded, or deleted with no container running."""
    st = pod.get("status") or {}
    if st.get("phase") in ("Failed", "Succeeded"):
        return True
    if not pod["metadata"].get("deletionTimestamp"):
        return False
    return all((cs.get("state") or {}).get("terminated") is not None or (cs.get("state") or {}).get("waiting") is not None
               for cs in st.get("containerStatuses") or ())


class PVCProtectionController(Controller):
    """`pkg/controller/volume/pvcprotection/pvc_protection_controller.go`: a claim being deleted
    keeps its `kubernetes.io/pvc-protection` finalizer while a scheduled, non-terminated pod in
    its namespace uses it (`isBeingUsed` :213 — unscheduled pods do not block); a live claim
    without the finalizer gets it (the admission plugin normally adds it, :174). Pod events
    only enqueue claims when the pod could unblock them: deleted, terminated or unscheduled
    (`podAddedDeletedUpdated` :272)."""
    name = "pvc-protection"
    workers = 1

    def setup(self):
        self.pvc_inf = self.factory.get("persistentvolumeclaims")
        self.pod_inf = self.factory.get("pods")
        self.pvc_inf.add_handler(self.enqueue, lambda o, n: self.enqueue(n), None)
        self.pod_inf.add_handler(self._pod, lambda o, n: self._pod(n), lambda p: self._pod(p, deleted=True))
        if "namespace" not in self.pod_inf.store.indexers:
            self.pod_inf.store.add_indexer("namespace", lambda p: [p["metadata"].get("namespace", "")])

    def _pod(self, pod, deleted=False):
        if not deleted and not pod_is_terminated(pod) and (pod.get("spec") or {}).get("nodeName"):
            return
        ns = pod["metadata"].get("namespace")
        for v in (pod.get("spec") or {}).get("volumes") or ():
            c = (v.get("persistentVolumeClaim") or {}).get("claimName")
            if c:
                self.enqueue(f"{ns}/{c}")

    def _in_use(self, ns, name):
        for p in self.pod_inf.store.by_index("namespace", ns):
            if not (p.get("spec") or {}).get("nodeName") or pod_is_terminated(p):
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
                await self._write(pvc, fins)
            return
        if PVC_PROTECTION not in fins:
            await self._write(pvc, fins + [PVC_PROTECTION])

    async def _write(self, pvc, fins):
        """An update of the cached object (the controller's role may update claims, not patch
        them); a conflict re-queues the key."""
        upd = dict(pvc, metadata=dict(pvc["metadata"], finalizers=fins))
        try:
            await self.client.update("persistentvolumeclaims", upd, pvc["metadata"].get("namespace"))
        except APIStatusError as e:
            if not is_not_found(e):
                raise


class PVProtectionController(Controller):
    """`pkg/controller/volume/pvprotection/pv_protection_controller.go`: a PersistentVolume being
    deleted keeps its `kubernetes.io/pv-protection` finalizer while it is Bound (`isBeingUsed`);
    once released the finalizer is removed with an update of the live object so the deletion
    completes. Only deletion candidates are queued (`pvAddedUpdated`)."""
    name = "pv-protection"
    workers = 1

    def setup(self):
        self.pv_inf = self.factory.get("persistentvolumes")
        self.pv_inf.add_handler(self._pv, lambda o, n: self._pv(n), None)

    def _pv(self, pv):
        if pv["metadata"].get("deletionTimestamp") and PV_PROTECTION in (pv["metadata"].get("finalizers") or ()):
            self.enqueue(pv["metadata"]["name"])

    async def sync(self, key):
        pv = self.pv_inf.get(key)
        if pv is None or not pv["metadata"].get("deletionTimestamp") or \
                PV_PROTECTION not in (pv["metadata"].get("finalizers") or ()):
            return
        if (pv.get("status") or {}).get("phase") == "Bound":
            return
        live = dict(pv, metadata=dict(pv["metadata"]))
        live["metadata"]["finalizers"] = [f for f in pv["metadata"]["finalizers"] if f != PV_PROTECTION]
        try:
            await self.client.update("persistentvolumes", live)
        except APIStatusError as e:
            if not is_not_found(e):
                raise


def _key(o):
    return f"{o['metadata'].get('namespace', '')}/{o['metadata']['name']}"
