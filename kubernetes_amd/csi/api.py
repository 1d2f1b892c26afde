"""CSI v0.1 messages and services, wire-compatible with the spec the reference vendors
(`vendor/github.com/container-storage-interface/spec/lib/go/csi/csi.pb.go`: package `csi`,
services `csi.Identity`, `csi.Controller`, `csi.Node`; the `access_type` oneof of
VolumeCapability is carried as its two optional members `block`=1 / `mount`=2, which is the
same encoding on the wire).
"""
from __future__ import annotations

from ..utils.protodesc import build

S, B, U32, M = "string", "bool", "uint32", "message"


def f(name, num, typ, label="opt", tname=None):
    return (name, num, typ, label, tname)


# VolumeCapability.AccessMode.Mode
UNKNOWN, SINGLE_NODE_WRITER, SINGLE_NODE_READER_ONLY, MULTI_NODE_READER_ONLY, MULTI_NODE_SINGLE_WRITER, \
    MULTI_NODE_MULTI_WRITER = range(6)
K8S_TO_CSI_MODE = {"ReadWriteOnce": SINGLE_NODE_WRITER, "ReadOnlyMany": MULTI_NODE_READER_ONLY,
                   "ReadWriteMany": MULTI_NODE_MULTI_WRITER}

SCHEMA = {
    "Version": [f("major", 1, U32), f("minor", 2, U32), f("patch", 3, U32)],
    "GetSupportedVersionsRequest": [],
    "GetSupportedVersionsResponse": [f("supported_versions", 1, M, "rep", "Version")],
    "GetPluginInfoRequest": [f("version", 1, M, "opt", "Version")],
    "GetPluginInfoResponse": [f("name", 1, S), f("vendor_version", 2, S), f("manifest", 3, S, "map")],
    "VolumeCapability_BlockVolume": [],
    "VolumeCapability_MountVolume": [f("fs_type", 1, S), f("mount_flags", 2, S, "rep")],
    "VolumeCapability_AccessMode": [f("mode", 1, "int32")],
    "VolumeCapability": [f("block", 1, M, "opt", "VolumeCapability_BlockVolume"),
                         f("mount", 2, M, "opt", "VolumeCapability_MountVolume"),
                         f("access_mode", 3, M, "opt", "VolumeCapability_AccessMode")],
    "ControllerPublishVolumeRequest": [f("version", 1, M, "opt", "Version"), f("volume_id", 2, S), f("node_id", 3, S),
                                       f("volume_capability", 4, M, "opt", "VolumeCapability"), f("readonly", 5, B),
                                       f("user_credentials", 6, S, "map"), f("volume_attributes", 7, S, "map")],
    "ControllerPublishVolumeResponse": [f("publish_volume_info", 1, S, "map")],
    "ControllerUnpublishVolumeRequest": [f("version", 1, M, "opt", "Version"), f("volume_id", 2, S), f("node_id", 3, S),
                                         f("user_credentials", 4, S, "map")],
    "ControllerUnpublishVolumeResponse": [],
    "ControllerProbeRequest": [f("version", 1, M, "opt", "Version")],
    "ControllerProbeResponse": [],
    "NodePublishVolumeRequest": [f("version", 1, M, "opt", "Version"), f("volume_id", 2, S),
                                 f("publish_volume_info", 3, S, "map"), f("target_path", 4, S),
                                 f("volume_capability", 5, M, "opt", "VolumeCapability"), f("readonly", 6, B),
                                 f("user_credentials", 7, S, "map"), f("volume_attributes", 8, S, "map")],
    "NodePublishVolumeResponse": [],
    "NodeUnpublishVolumeRequest": [f("version", 1, M, "opt", "Version"), f("volume_id", 2, S), f("target_path", 3, S),
                                   f("user_credentials", 4, S, "map")],
    "NodeUnpublishVolumeResponse": [],
    "GetNodeIDRequest": [f("version", 1, M, "opt", "Version")],
    "GetNodeIDResponse": [f("node_id", 1, S)],
    "NodeProbeRequest": [f("version", 1, M, "opt", "Version")],
    "NodeProbeResponse": [],
}

MSG = build("csi", "csi/csi.proto", SCHEMA)
VERSION = MSG["Version"](major=0, minor=1, patch=0)

IDENTITY, CONTROLLER, NODE = "csi.Identity", "csi.Controller", "csi.Node"


def _m(req, resp):
    return (MSG[req], MSG[resp], False)


IDENTITY_METHODS = {"GetSupportedVersions": _m("GetSupportedVersionsRequest", "GetSupportedVersionsResponse"),
                    "GetPluginInfo": _m("GetPluginInfoRequest", "GetPluginInfoResponse")}
CONTROLLER_METHODS = {"ControllerPublishVolume": _m("ControllerPublishVolumeRequest", "ControllerPublishVolumeResponse"),
                      "ControllerUnpublishVolume": _m("ControllerUnpublishVolumeRequest",
                                                      "ControllerUnpublishVolumeResponse"),
                      "ControllerProbe": _m("ControllerProbeRequest", "ControllerProbeResponse")}
NODE_METHODS = {"NodePublishVolume": _m("NodePublishVolumeRequest", "NodePublishVolumeResponse"),
                "NodeUnpublishVolume": _m("NodeUnpublishVolumeRequest", "NodeUnpublishVolumeResponse"),
                "GetNodeID": _m("GetNodeIDRequest", "GetNodeIDResponse"),
                "NodeProbe": _m("NodeProbeRequest", "NodeProbeResponse")}


def socket_path(plugins_dir, driver):
    """`pkg/volume/csi/csi_plugin.go` csiAddrTemplate: /var/lib/kubelet/plugins/<driver>/csi.sock."""
    import os
    return os.path.join(plugins_dir, driver, "csi.sock")


def attachment_name(pv_name, driver, node):
    """`csi_attacher.go:269` getAttachmentName: csi-<sha256(volName + driver + node)>."""
    import hashlib
    return "csi-" + hashlib.sha256(f"{pv_name}{driver}{node}".encode()).hexdigest()
