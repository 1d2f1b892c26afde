"""PersistentVolume binder: the `pkg/controller/volume/persistentvolume/binder_test.go` TestSync
table (sets 1-4 and 13: unbound claims, pre-bound claims and volumes, bound claims, volume
phases, storage classes) and TestSyncAlphaBlockVolume's volumeMode cases, plus reclaim
(`delete_test.go` / `recycle_test.go` outcomes for volumes without a plugin). Each case: start
volumes + claims, one syncClaim or syncVolume, then compare the resulting volumes, claims and
events with the reference's expectations."""
import asyncio
import copy

import pytest

from kubernetes_amd.client.fake import FakeClient
from kubernetes_amd.client.informer import InformerFactory
from kubernetes_amd.controllers.volume import BIND_COMPLETED, BOUND_BY_CONTROLLER, PersistentVolumeController

NS = "default"
BBC, BC = BOUND_BY_CONTROLLER, BIND_COMPLETED
EMPTY, GOLD, SILVER, WAIT = "", "gold", "silver", "wait"
MODES = ["ReadWriteOnce", "ReadOnlyMany"]


def vol(name, cap, uid, claim, phase, policy="Retain", cls=EMPTY, *anns, labels=None, mode=None, path=None):
    v = {"apiVersion": "v1", "kind": "PersistentVolume", "metadata": {"name": name},
         "spec": {"capacity": {"storage": cap}, "accessModes": list(MODES), "persistentVolumeReclaimPolicy": policy,
                  "storageClassName": cls, "gcePersistentDisk": {"pdName": name}},
         "status": {"phase": phase}}
    if path is not None:
        del v["spec"]["gcePersistentDisk"]
        v["spec"]["hostPath"] = {"path": path}
    if claim:
        v["spec"]["claimRef"] = {"kind": "PersistentVolumeClaim", "apiVersion": "v1", "namespace": NS, "name": claim,
                                 "uid": uid}
    if anns:
        v["metadata"]["annotations"] = {a: "yes" for a in anns}
    if labels:
        v["metadata"]["labels"] = dict(labels)
    if mode:
        v["spec"]["volumeMode"] = mode
    return v


def claim(name, uid, cap, volume, phase, cls=None, *anns, selector=None, mode=None, status_cap=None):
    c = {"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": name, "namespace": NS, "uid": uid},
         "spec": {"accessModes": list(MODES), "resources": {"requests": {"storage": cap}}},
         "status": {"phase": phase}}
    if volume:
        c["spec"]["volumeName"] = volume
    if cls is not None:
        c["spec"]["storageClassName"] = cls
    if anns:
        c["metadata"]["annotations"] = {a: "yes" for a in anns}
    if selector:
        c["spec"]["selector"] = {"matchLabels": dict(selector)}
    if mode:
        c["spec"]["volumeMode"] = mode
    if phase == "Bound":
        c["status"]["accessModes"] = list(MODES)
        c["status"]["capacity"] = {"storage": status_cap or cap}
    return c


LABELS = {"foo": "true", "bar": "false"}
SC_WAIT = {"apiVersion": "storage.k8s.io/v1", "kind": "StorageClass", "metadata": {"name": WAIT},
           "provisioner": "kubernetes.io/no-provisioner", "volumeBindingMode": "WaitForFirstConsumer"}

# name: (initial volumes, expected volumes, initial claims, expected claims, events, error?, "claim"|"volume")
CASES = {
    "1-1 - successful bind": (
        [vol("volume1-1", "1Gi", "", "", "Pending")], [vol("volume1-1", "1Gi", "uid1-1", "claim1-1", "Bound", "Retain", EMPTY, BBC)],
        [claim("claim1-1", "uid1-1", "1Gi", "", "Pending")], [claim("claim1-1", "uid1-1", "1Gi", "volume1-1", "Bound", None, BBC, BC)],
        [], False, "claim"),
    "1-2 - noop": (
        [vol("volume1-2", "1Gi", "", "", "Pending")], [vol("volume1-2", "1Gi", "", "", "Pending")],
        [claim("claim1-2", "uid1-2", "10Gi", "", "Pending")], [claim("claim1-2", "uid1-2", "10Gi", "", "Pending")],
        ["Normal FailedBinding"], False, "claim"),
    "1-3 - reset to Pending": (
        [vol("volume1-3", "1Gi", "", "", "Pending")], [vol("volume1-3", "1Gi", "", "", "Pending")],
        [claim("claim1-3", "uid1-3", "10Gi", "", "Bound")], [claim("claim1-3", "uid1-3", "10Gi", "", "Pending")],
        ["Normal FailedBinding"], False, "claim"),
    "1-4 - smallest volume": (
        [vol("volume1-4_1", "10Gi", "", "", "Pending"), vol("volume1-4_2", "1Gi", "", "", "Pending")],
        [vol("volume1-4_1", "10Gi", "", "", "Pending"), vol("volume1-4_2", "1Gi", "uid1-4", "claim1-4", "Bound", "Retain", EMPTY, BBC)],
        [claim("claim1-4", "uid1-4", "1Gi", "", "Pending")], [claim("claim1-4", "uid1-4", "1Gi", "volume1-4_2", "Bound", None, BBC, BC)],
        [], False, "claim"),
    "1-5 - prebound volume by name - success": (
        [vol("volume1-5_1", "10Gi", "", "claim1-5", "Pending"), vol("volume1-5_2", "1Gi", "", "", "Pending")],
        [vol("volume1-5_1", "10Gi", "uid1-5", "claim1-5", "Bound"), vol("volume1-5_2", "1Gi", "", "", "Pending")],
        [claim("claim1-5", "uid1-5", "1Gi", "", "Pending")],
        [claim("claim1-5", "uid1-5", "1Gi", "volume1-5_1", "Bound", None, BBC, BC, status_cap="10Gi")],
        [], False, "claim"),
    "1-6 - prebound volume by UID - success": (
        [vol("volume1-6_1", "10Gi", "uid1-6", "claim1-6", "Pending"), vol("volume1-6_2", "1Gi", "", "", "Pending")],
        [vol("volume1-6_1", "10Gi", "uid1-6", "claim1-6", "Bound"), vol("volume1-6_2", "1Gi", "", "", "Pending")],
        [claim("claim1-6", "uid1-6", "1Gi", "", "Pending")],
        [claim("claim1-6", "uid1-6", "1Gi", "volume1-6_1", "Bound", None, BBC, BC, status_cap="10Gi")],
        [], False, "claim"),
    "1-7 - prebound volume to different claim": (
        [vol("volume1-7", "10Gi", "uid1-777", "claim1-7", "Pending")], [vol("volume1-7", "10Gi", "uid1-777", "claim1-7", "Pending")],
        [claim("claim1-7", "uid1-7", "1Gi", "", "Pending")], [claim("claim1-7", "uid1-7", "1Gi", "", "Pending")],
        ["Normal FailedBinding"], False, "claim"),
    "1-8 - complete bind after crash - PV bound": (
        [vol("volume1-8", "1Gi", "uid1-8", "claim1-8", "Pending", "Retain", EMPTY, BBC)],
        [vol("volume1-8", "1Gi", "uid1-8", "claim1-8", "Bound", "Retain", EMPTY, BBC)],
        [claim("claim1-8", "uid1-8", "1Gi", "", "Pending")], [claim("claim1-8", "uid1-8", "1Gi", "volume1-8", "Bound", None, BBC, BC)],
        [], False, "claim"),
    "1-9 - complete bind after crash - PV status saved": (
        [vol("volume1-9", "1Gi", "uid1-9", "claim1-9", "Bound", "Retain", EMPTY, BBC)],
        [vol("volume1-9", "1Gi", "uid1-9", "claim1-9", "Bound", "Retain", EMPTY, BBC)],
        [claim("claim1-9", "uid1-9", "1Gi", "", "Pending")], [claim("claim1-9", "uid1-9", "1Gi", "volume1-9", "Bound", None, BBC, BC)],
        [], False, "claim"),
    "1-10 - complete bind after crash - PVC bound": (
        [vol("volume1-10", "1Gi", "uid1-10", "claim1-10", "Bound", "Retain", EMPTY, BBC)],
        [vol("volume1-10", "1Gi", "uid1-10", "claim1-10", "Bound", "Retain", EMPTY, BBC)],
        [claim("claim1-10", "uid1-10", "1Gi", "volume1-10", "Pending", None, BBC, BC)],
        [claim("claim1-10", "uid1-10", "1Gi", "volume1-10", "Bound", None, BBC, BC)],
        [], False, "claim"),
    "1-11 - bind when selector matches": (
        [vol("volume1-1", "1Gi", "", "", "Pending", labels=LABELS)],
        [vol("volume1-1", "1Gi", "uid1-1", "claim1-1", "Bound", "Retain", EMPTY, BBC, labels=LABELS)],
        [claim("claim1-1", "uid1-1", "1Gi", "", "Pending", selector=LABELS)],
        [claim("claim1-1", "uid1-1", "1Gi", "volume1-1", "Bound", None, BBC, BC, selector=LABELS)],
        [], False, "claim"),
    "1-12 - do not bind when selector does not match": (
        [vol("volume1-1", "1Gi", "", "", "Pending")], [vol("volume1-1", "1Gi", "", "", "Pending")],
        [claim("claim1-1", "uid1-1", "1Gi", "", "Pending", selector=LABELS)],
        [claim("claim1-1", "uid1-1", "1Gi", "", "Pending", selector=LABELS)],
        ["Normal FailedBinding"], False, "claim"),
    "1-13 - delayed binding": (
        [vol("volume1-1", "1Gi", "", "", "Pending", "Retain", WAIT)], [vol("volume1-1", "1Gi", "", "", "Pending", "Retain", WAIT)],
        [claim("claim1-1", "uid1-1", "1Gi", "", "Pending", WAIT)], [claim("claim1-1", "uid1-1", "1Gi", "", "Pending", WAIT)],
        ["Normal WaitForFirstConsumer"], False, "claim"),
    "1-14 - successful prebound PV": (
        [vol("volume1-1", "1Gi", "", "claim1-1", "Pending", "Retain", WAIT)],
        [vol("volume1-1", "1Gi", "uid1-1", "claim1-1", "Bound", "Retain", WAIT)],
        [claim("claim1-1", "uid1-1", "1Gi", "", "Pending", WAIT)],
        [claim("claim1-1", "uid1-1", "1Gi", "volume1-1", "Bound", WAIT, BBC, BC)],
        [], False, "claim"),
    "2-1 - claim prebound to non-existing volume - noop": (
        [], [], [claim("claim2-1", "uid2-1", "10Gi", "volume2-1", "Pending")],
        [claim("claim2-1", "uid2-1", "10Gi", "volume2-1", "Pending")], [], False, "claim"),
    "2-2 - claim prebound to non-existing volume - reset status": (
        [], [], [claim("claim2-2", "uid2-2", "10Gi", "volume2-2", "Bound")],
        [claim("claim2-2", "uid2-2", "10Gi", "volume2-2", "Pending")], [], False, "claim"),
    "2-3 - claim prebound to unbound volume": (
        [vol("volume2-3", "1Gi", "", "", "Pending")], [vol("volume2-3", "1Gi", "uid2-3", "claim2-3", "Bound", "Retain", EMPTY, BBC)],
        [claim("claim2-3", "uid2-3", "1Gi", "volume2-3", "Pending")],
        [claim("claim2-3", "uid2-3", "1Gi", "volume2-3", "Bound", None, BC)], [], False, "claim"),
    "2-4 - claim prebound to prebound volume by name": (
        [vol("volume2-4", "1Gi", "", "claim2-4", "Pending")], [vol("volume2-4", "1Gi", "uid2-4", "claim2-4", "Bound")],
        [claim("claim2-4", "uid2-4", "1Gi", "volume2-4", "Pending")],
        [claim("claim2-4", "uid2-4", "1Gi", "volume2-4", "Bound", None, BC)], [], False, "claim"),
    "2-5 - claim prebound to prebound volume by UID": (
        [vol("volume2-5", "1Gi", "uid2-5", "claim2-5", "Pending")], [vol("volume2-5", "1Gi", "uid2-5", "claim2-5", "Bound")],
        [claim("claim2-5", "uid2-5", "1Gi", "volume2-5", "Pending")],
        [claim("claim2-5", "uid2-5", "1Gi", "volume2-5", "Bound", None, BC)], [], False, "claim"),
    "2-6 - claim prebound to already bound volume": (
        [vol("volume2-6", "1Gi", "uid2-6_1", "claim2-6_1", "Bound")], [vol("volume2-6", "1Gi", "uid2-6_1", "claim2-6_1", "Bound")],
        [claim("claim2-6", "uid2-6", "1Gi", "volume2-6", "Bound")], [claim("claim2-6", "uid2-6", "1Gi", "volume2-6", "Pending")],
        [], False, "claim"),
    "2-7 - claim bound by controller to already bound volume": (
        [vol("volume2-7", "1Gi", "uid2-7_1", "claim2-7_1", "Bound")], [vol("volume2-7", "1Gi", "uid2-7_1", "claim2-7_1", "Bound")],
        [claim("claim2-7", "uid2-7", "1Gi", "volume2-7", "Bound", None, BBC)],
        [claim("claim2-7", "uid2-7", "1Gi", "volume2-7", "Bound", None, BBC)], [], True, "claim"),
    "2-8 - claim prebound to unbound volume that does not match the selector": (
        [vol("volume2-8", "1Gi", "", "", "Pending")], [vol("volume2-8", "1Gi", "uid2-8", "claim2-8", "Bound", "Retain", EMPTY, BBC)],
        [claim("claim2-8", "uid2-8", "1Gi", "volume2-8", "Pending", selector=LABELS)],
        [claim("claim2-8", "uid2-8", "1Gi", "volume2-8", "Bound", None, BC, selector=LABELS)], [], False, "claim"),
    "2-9 - claim prebound to unbound volume that size is smaller than requested": (
        [vol("volume2-9", "1Gi", "", "", "Pending")], [vol("volume2-9", "1Gi", "", "", "Pending")],
        [claim("claim2-9", "uid2-9", "2Gi", "volume2-9", "Bound")], [claim("claim2-9", "uid2-9", "2Gi", "volume2-9", "Pending")],
        ["Warning VolumeMismatch"], False, "claim"),
    "2-10 - claim prebound to unbound volume that class is different": (
        [vol("volume2-10", "1Gi", "1", "", "Pending", "Retain", GOLD)], [vol("volume2-10", "1Gi", "", "", "Pending", "Retain", GOLD)],
        [claim("claim2-10", "uid2-10", "1Gi", "volume2-10", "Bound")],
        [claim("claim2-10", "uid2-10", "1Gi", "volume2-10", "Pending")], ["Warning VolumeMismatch"], False, "claim"),
    "3-1 - bound claim with missing VolumeName": (
        [], [], [claim("claim3-1", "uid3-1", "10Gi", "", "Bound", None, BBC, BC)],
        [claim("claim3-1", "uid3-1", "10Gi", "", "Lost", None, BBC, BC)], ["Warning ClaimLost"], False, "claim"),
    "3-2 - bound claim with missing volume": (
        [], [], [claim("claim3-2", "uid3-2", "10Gi", "volume3-2", "Bound", None, BBC, BC)],
        [claim("claim3-2", "uid3-2", "10Gi", "volume3-2", "Lost", None, BBC, BC)], ["Warning ClaimLost"], False, "claim"),
    "3-3 - bound claim with unbound volume": (
        [vol("volume3-3", "10Gi", "", "", "Pending")], [vol("volume3-3", "10Gi", "uid3-3", "claim3-3", "Bound", "Retain", EMPTY, BBC)],
        [claim("claim3-3", "uid3-3", "10Gi", "volume3-3", "Pending", None, BBC, BC)],
        [claim("claim3-3", "uid3-3", "10Gi", "volume3-3", "Bound", None, BBC, BC)], [], False, "claim"),
    "3-4 - bound claim with prebound volume": (
        [vol("volume3-4", "10Gi", "claim3-4-x", "claim3-4", "Pending")],
        [vol("volume3-4", "10Gi", "claim3-4-x", "claim3-4", "Pending")],
        [claim("claim3-4", "uid3-4", "10Gi", "volume3-4", "Pending", None, BBC, BC)],
        [claim("claim3-4", "uid3-4", "10Gi", "volume3-4", "Lost", None, BBC, BC)], ["Warning ClaimMisbound"], False, "claim"),
    "3-5 - bound claim with bound volume": (
        [vol("volume3-5", "10Gi", "uid3-5", "claim3-5", "Pending")], [vol("volume3-5", "10Gi", "uid3-5", "claim3-5", "Bound")],
        [claim("claim3-5", "uid3-5", "10Gi", "volume3-5", "Pending", None, BC)],
        [claim("claim3-5", "uid3-5", "10Gi", "volume3-5", "Bound", None, BC)], [], False, "claim"),
    "3-6 - bound claim with bound volume": (
        [vol("volume3-6", "10Gi", "uid3-6-x", "claim3-6-x", "Pending")],
        [vol("volume3-6", "10Gi", "uid3-6-x", "claim3-6-x", "Pending")],
        [claim("claim3-6", "uid3-6", "10Gi", "volume3-6", "Pending", None, BC)],
        [claim("claim3-6", "uid3-6", "10Gi", "volume3-6", "Lost", None, BC)], ["Warning ClaimMisbound"], False, "claim"),
    "3-7 - bound claim with unbound volume where selector doesn't match": (
        [vol("volume3-3", "10Gi", "", "", "Pending")], [vol("volume3-3", "10Gi", "uid3-3", "claim3-3", "Bound", "Retain", EMPTY, BBC)],
        [claim("claim3-3", "uid3-3", "10Gi", "volume3-3", "Pending", None, BBC, BC, selector=LABELS)],
        [claim("claim3-3", "uid3-3", "10Gi", "volume3-3", "Bound", None, BBC, BC, selector=LABELS)], [], False, "claim"),
    "4-1 - pending volume": (
        [vol("volume4-1", "10Gi", "", "", "Pending")], [vol("volume4-1", "10Gi", "", "", "Available")], [], [], [], False, "volume"),
    "4-2 - pending prebound volume": (
        [vol("volume4-2", "10Gi", "", "claim4-2", "Pending")], [vol("volume4-2", "10Gi", "", "claim4-2", "Available")], [], [],
        [], False, "volume"),
    "4-3 - bound volume with missing claim": (
        [vol("volume4-3", "10Gi", "uid4-3", "claim4-3", "Bound")], [vol("volume4-3", "10Gi", "uid4-3", "claim4-3", "Released")],
        [], [], [], False, "volume"),
    "4-4 - volume bound to claim with different UID": (
        [vol("volume4-4", "10Gi", "uid4-4", "claim4-4", "Bound")], [vol("volume4-4", "10Gi", "uid4-4", "claim4-4", "Released")],
        [claim("claim4-4", "uid4-4-x", "10Gi", "volume4-4", "Bound", None, BC)],
        [claim("claim4-4", "uid4-4-x", "10Gi", "volume4-4", "Bound", None, BC)], [], False, "volume"),
    "4-5 - volume bound by controller to unbound claim": (
        [vol("volume4-5", "10Gi", "uid4-5", "claim4-5", "Bound", "Retain", EMPTY, BBC)],
        [vol("volume4-5", "10Gi", "uid4-5", "claim4-5", "Bound", "Retain", EMPTY, BBC)],
        [claim("claim4-5", "uid4-5", "10Gi", "", "Pending")], [claim("claim4-5", "uid4-5", "10Gi", "", "Pending")],
        [], False, "volume"),
    "4-5b - volume bound by user to bound claim": (
        [vol("volume4-5", "10Gi", "uid4-5", "claim4-5", "Bound")], [vol("volume4-5", "10Gi", "uid4-5", "claim4-5", "Bound")],
        [claim("claim4-5", "uid4-5", "10Gi", "", "Pending")], [claim("claim4-5", "uid4-5", "10Gi", "", "Pending")],
        [], False, "volume"),
    "4-6 - volume bound by to bound claim": (
        [vol("volume4-6", "10Gi", "uid4-6", "claim4-6", "Available")], [vol("volume4-6", "10Gi", "uid4-6", "claim4-6", "Bound")],
        [claim("claim4-6", "uid4-6", "10Gi", "volume4-6", "Bound")], [claim("claim4-6", "uid4-6", "10Gi", "volume4-6", "Bound")],
        [], False, "volume"),
    "4-7 - volume bound by controller to claim bound somewhere else": (
        [vol("volume4-7", "10Gi", "uid4-7", "claim4-7", "Bound", "Retain", EMPTY, BBC)],
        [vol("volume4-7", "10Gi", "", "", "Available")],
        [claim("claim4-7", "uid4-7", "10Gi", "volume4-7-x", "Bound")],
        [claim("claim4-7", "uid4-7", "10Gi", "volume4-7-x", "Bound")], [], False, "volume"),
    "4-8 - volume bound by user to claim bound somewhere else": (
        [vol("volume4-8", "10Gi", "uid4-8", "claim4-8", "Bound")], [vol("volume4-8", "10Gi", "", "claim4-8", "Available")],
        [claim("claim4-8", "uid4-8", "10Gi", "volume4-8-x", "Bound")],
        [claim("claim4-8", "uid4-8", "10Gi", "volume4-8-x", "Bound")], [], False, "volume"),
    "13-1 - binding to class": (
        [vol("volume13-1-1", "1Gi", "", "", "Pending"), vol("volume13-1-2", "10Gi", "", "", "Pending", "Retain", GOLD)],
        [vol("volume13-1-1", "1Gi", "", "", "Pending"),
         vol("volume13-1-2", "10Gi", "uid13-1", "claim13-1", "Bound", "Retain", GOLD, BBC)],
        [claim("claim13-1", "uid13-1", "1Gi", "", "Pending", GOLD)],
        [claim("claim13-1", "uid13-1", "1Gi", "volume13-1-2", "Bound", GOLD, BBC, BC, status_cap="10Gi")], [], False, "claim"),
    "13-2 - binding without a class": (
        [vol("volume13-2-1", "1Gi", "", "", "Pending", "Retain", GOLD), vol("volume13-2-2", "10Gi", "", "", "Pending")],
        [vol("volume13-2-1", "1Gi", "", "", "Pending", "Retain", GOLD),
         vol("volume13-2-2", "10Gi", "uid13-2", "claim13-2", "Bound", "Retain", EMPTY, BBC)],
        [claim("claim13-2", "uid13-2", "1Gi", "", "Pending")],
        [claim("claim13-2", "uid13-2", "1Gi", "volume13-2-2", "Bound", None, BBC, BC, status_cap="10Gi")], [], False, "claim"),
    "13-3 - binding to specific a class": (
        [vol("volume13-3-1", "1Gi", "", "", "Pending", "Retain", SILVER), vol("volume13-3-2", "10Gi", "", "", "Pending", "Retain", GOLD)],
        [vol("volume13-3-1", "1Gi", "", "", "Pending", "Retain", SILVER),
         vol("volume13-3-2", "10Gi", "uid13-3", "claim13-3", "Bound", "Retain", GOLD, BBC)],
        [claim("claim13-3", "uid13-3", "1Gi", "", "Pending", GOLD)],
        [claim("claim13-3", "uid13-3", "1Gi", "volume13-3-2", "Bound", GOLD, BBC, BC, status_cap="10Gi")], [], False, "claim"),
    "13-4 - empty class": (
        [vol("volume13-4", "1Gi", "", "", "Pending")], [vol("volume13-4", "1Gi", "uid13-4", "claim13-4", "Bound", "Retain", EMPTY, BBC)],
        [claim("claim13-4", "uid13-4", "1Gi", "", "Pending", EMPTY)],
        [claim("claim13-4", "uid13-4", "1Gi", "volume13-4", "Bound", EMPTY, BBC, BC)], [], False, "claim"),
    "14-1 - binding to volumeMode block": (
        [vol("volume14-1", "10Gi", "", "", "Pending", mode="Block")],
        [vol("volume14-1", "10Gi", "uid14-1", "claim14-1", "Bound", "Retain", EMPTY, BBC, mode="Block")],
        [claim("claim14-1", "uid14-1", "10Gi", "", "Pending", mode="Block")],
        [claim("claim14-1", "uid14-1", "10Gi", "volume14-1", "Bound", None, BBC, BC, mode="Block")], [], False, "claim"),
    "14-3 - do not bind pv volumeMode filesystem and pvc volumeMode block": (
        [vol("volume14-3", "10Gi", "", "", "Pending", mode="Filesystem")],
        [vol("volume14-3", "10Gi", "", "", "Pending", mode="Filesystem")],
        [claim("claim14-3", "uid14-3", "10Gi", "", "Pending", mode="Block")],
        [claim("claim14-3", "uid14-3", "10Gi", "", "Pending", mode="Block")], ["Normal FailedBinding"], False, "claim"),
    "14-8 - do not bind when pvc is prebound to pv with mismatching volumeModes": (
        [vol("volume14-8", "10Gi", "", "", "Pending", mode="Block")], [vol("volume14-8", "10Gi", "", "", "Pending", mode="Block")],
        [claim("claim14-8", "uid14-8", "10Gi", "volume14-8", "Pending", mode="Filesystem")],
        [claim("claim14-8", "uid14-8", "10Gi", "volume14-8", "Pending", mode="Filesystem")],
        ["Warning VolumeMismatch"], False, "claim"),
}


def _vol_view(v):
    ref = (v.get("spec") or {}).get("claimRef") or {}
    return (v["metadata"]["name"], ref.get("name") or "", ref.get("uid") or "", (v.get("status") or {}).get("phase"),
            sorted(k for k in (v["metadata"].get("annotations") or {}) if k in (BBC, BC)))


def _claim_view(c):
    st = c.get("status") or {}
    return (c["metadata"]["name"], (c.get("spec") or {}).get("volumeName") or "", st.get("phase"),
            sorted(k for k in (c["metadata"].get("annotations") or {}) if k in (BBC, BC)),
            ((st.get("capacity") or {}).get("storage")), tuple(st.get("accessModes") or ()))


def run_case(volumes, claims, kind, tmp_path=None):
    async def main():
        c = FakeClient(*copy.deepcopy(volumes), *copy.deepcopy(claims), copy.deepcopy(SC_WAIT))
        f = InformerFactory(c)
        ctl = PersistentVolumeController(c, f, hostpath_root=str(tmp_path) if tmp_path else None)
        ctl.setup()
        events = []
        ctl.recorder.event = lambda obj, typ, reason, msg: events.append(f"{typ} {reason}")
        f.start()
        await f.wait_for_cache_sync()
        err = None
        try:
            if kind == "claim":
                await ctl.sync_claim(ctl.pvc_inf.get(f"{NS}/{claims[0]['metadata']['name']}"))
            else:
                await ctl.sync_volume(ctl.pv_inf.get(volumes[0]["metadata"]["name"]))
        except RuntimeError as e:
            err = e
        vols = sorted(c.objects.get("persistentvolumes", {}).values(), key=lambda v: v["metadata"]["name"])
        cls = sorted(c.objects.get("persistentvolumeclaims", {}).values(), key=lambda v: v["metadata"]["name"])
        return vols, cls, events, err
    return asyncio.run(main())


@pytest.mark.parametrize("name", list(CASES))
def test_sync(name):
    vols0, vols1, claims0, claims1, events, want_err, kind = CASES[name]
    vols, cls, got_events, err = run_case(vols0, claims0, kind)
    assert (err is not None) == want_err, (name, err)
    assert [_vol_view(v) for v in vols] == [_vol_view(v) for v in sorted(vols1, key=lambda v: v["metadata"]["name"])], name
    assert [_claim_view(c) for c in cls] == [_claim_view(c) for c in claims1], name
    assert got_events == events, name


def test_best_match_prefers_the_most_specific_access_modes():
    """index.go allPossibleMatchingAccessModes: a claim asking RWO gets the RWO-only volume
    before a bigger-or-smaller RWO+ROX+RWX one."""
    from kubernetes_amd.controllers.volume import best_match
    rwo = vol("rwo", "10Gi", "", "", "Pending")
    rwo["spec"]["accessModes"] = ["ReadWriteOnce"]
    multi = vol("multi", "1Gi", "", "", "Pending")
    multi["spec"]["accessModes"] = ["ReadWriteOnce", "ReadOnlyMany", "ReadWriteMany"]
    c = claim("c", "u", "1Gi", "", "Pending")
    c["spec"]["accessModes"] = ["ReadWriteOnce"]
    assert best_match([multi, rwo], c)["metadata"]["name"] == "rwo"
    c["spec"]["accessModes"] = ["ReadWriteMany"]
    assert best_match([multi, rwo], c)["metadata"]["name"] == "multi"


@pytest.mark.parametrize("policy,spec_kind,phase,event", [
    ("Delete", "gce", "Failed", "Warning VolumeFailedDelete"),          # no deleter plugin
    ("Recycle", "gce", "Failed", "Warning VolumeFailedRecycle"),        # no recycler plugin
    ("Bogus", "gce", "Failed", "Warning VolumeUnknownReclaimPolicy"),
    ("Retain", "gce", "Released", None)])
def test_reclaim_without_a_plugin(policy, spec_kind, phase, event):
    v = vol("volume8", "1Gi", "uid8", "claim8", "Bound", policy)
    vols, _, events, _ = run_case([v], [], "volume")
    assert vols[0]["status"]["phase"] == phase
    assert events == ([event] if event else [])


def test_host_path_delete_and_recycle(tmp_path):
    d = tmp_path / "pv-dir"
    d.mkdir()
    (d / "data").write_text("x")
    v = vol("volume9", "1Gi", "uid9", "claim9", "Bound", "Recycle", path=str(d))
    vols, _, events, _ = run_case([v], [], "volume", tmp_path)
    assert events == ["Normal VolumeRecycled"] and not list(d.iterdir())
    # recycled and unbound: a user pre-binding keeps the claim name and loses the UID
    assert vols[0]["status"]["phase"] == "Available" and not vols[0]["spec"]["claimRef"].get("uid")
    v = vol("volume10", "1Gi", "uid10", "claim10", "Bound", "Delete", path=str(d))
    vols, _, events, _ = run_case([v], [], "volume", tmp_path)
    assert vols == [] and not d.exists()
    # outside /tmp and outside the provisioning root: the host-path deleter refuses
    v = vol("volume11", "1Gi", "uid11", "claim11", "Bound", "Delete", path="/var/lib/precious")
    vols, _, events, _ = run_case([v], [], "volume", tmp_path)
    assert vols[0]["status"]["phase"] == "Failed" and events == ["Warning VolumeFailedDelete"]


def test_external_provisioning_and_missing_class():
    sc = {"apiVersion": "storage.k8s.io/v1", "kind": "StorageClass", "metadata": {"name": GOLD},
          "provisioner": "example.com/nfs"}

    async def main(objs):
        c = FakeClient(*objs)
        f = InformerFactory(c)
        ctl = PersistentVolumeController(c, f)
        ctl.setup()
        events = []
        ctl.recorder.event = lambda obj, typ, reason, msg: events.append(f"{typ} {reason}")
        f.start()
        await f.wait_for_cache_sync()
        await ctl.sync_claim(ctl.pvc_inf.get(f"{NS}/c"))
        return c.objects["persistentvolumeclaims"][(NS, "c")], events
    pvc, events = asyncio.run(main([sc, claim("c", "u", "1Gi", "", "Pending", GOLD)]))
    assert events == ["Normal ExternalProvisioning"]
    assert pvc["metadata"]["annotations"]["volume.beta.kubernetes.io/storage-provisioner"] == "example.com/nfs"
    pvc, events = asyncio.run(main([claim("c", "u", "1Gi", "", "Pending", SILVER)]))
    assert events == ["Warning ProvisioningFailed"]
