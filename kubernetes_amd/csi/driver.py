"""A host-path CSI driver (the reference's test driver pattern, `csi-hostpath`) serving the
Identity, Controller and Node services on a unix socket.

Volumes live under `<root>/volumes/<volume_id>`. ControllerPublishVolume records which node a
volume is attached to (single-node-writer volumes refuse a second node); NodePublishVolume makes
the volume visible at `target_path` (a symlink: no mount privileges needed) and
NodeUnpublishVolume removes it. This is what the e2e and unit tests drive, and it is a working
template for a real MI355X-node storage driver (NVMe scratch, parallel FS).
"""
from __future__ import annotations

import os

import grpc

from ..deviceplugin.api import generic_handler
from . import api as A


class HostPathDriver:
    def __init__(self, name, root, node_id):
        self.name, self.root, self.node_id = name, root, node_id
        self.attached: dict[str, str] = {}       # volume id -> node id
        self.published: dict[str, set] = {}      # volume id -> target paths
        self.server = None

    # Identity
    async def GetSupportedVersions(self, req, ctx):
        return A.MSG["GetSupportedVersionsResponse"](supported_versions=[A.VERSION])

    async def GetPluginInfo(self, req, ctx):
        return A.MSG["GetPluginInfoResponse"](name=self.name, vendor_version="0.1.0", manifest={"runtime": "kubernetes-amd"})

    # Controller
    async def ControllerProbe(self, req, ctx):
        return A.MSG["ControllerProbeResponse"]()

    async def ControllerPublishVolume(self, req, ctx):
        cur = self.attached.get(req.volume_id)
        mode = req.volume_capability.access_mode.mode if req.HasField("volume_capability") else A.SINGLE_NODE_WRITER
        if cur and cur != req.node_id and mode in (A.SINGLE_NODE_WRITER, A.SINGLE_NODE_READER_ONLY):
            await ctx.abort(grpc.StatusCode.FAILED_PRECONDITION,
                            f"volume {req.volume_id} is already published to node {cur}")
        self.attached[req.volume_id] = req.node_id
        return A.MSG["ControllerPublishVolumeResponse"](publish_volume_info={"devicePath": self._vol(req.volume_id)})

    async def ControllerUnpublishVolume(self, req, ctx):
        if self.attached.get(req.volume_id) in (req.node_id, None) or not req.node_id:
            self.attached.pop(req.volume_id, None)
        return A.MSG["ControllerUnpublishVolumeResponse"]()

    # Node
    def _vol(self, vid):
        return os.path.join(self.root, "volumes", vid.replace("/", "_"))

    async def NodeProbe(self, req, ctx):
        return A.MSG["NodeProbeResponse"]()

    async def GetNodeID(self, req, ctx):
        return A.MSG["GetNodeIDResponse"](node_id=self.node_id)

    async def NodePublishVolume(self, req, ctx):
        if not req.volume_id or not req.target_path:
            await ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, "volume_id and target_path are required")
        src = self._vol(req.volume_id)
        os.makedirs(src, exist_ok=True)
        os.makedirs(os.path.dirname(req.target_path), exist_ok=True)
        if os.path.islink(req.target_path):
            if os.readlink(req.target_path) != src:
                await ctx.abort(grpc.StatusCode.ALREADY_EXISTS, f"{req.target_path} is published from another volume")
        else:
            if os.path.isdir(req.target_path) and not os.listdir(req.target_path):
                os.rmdir(req.target_path)
            os.symlink(src, req.target_path)
        self.published.setdefault(req.volume_id, set()).add(req.target_path)
        return A.MSG["NodePublishVolumeResponse"]()

    async def NodeUnpublishVolume(self, req, ctx):
        if os.path.islink(req.target_path):
            os.unlink(req.target_path)
        self.published.get(req.volume_id, set()).discard(req.target_path)
        return A.MSG["NodeUnpublishVolumeResponse"]()

    async def start(self, socket_path):
        os.makedirs(os.path.dirname(socket_path), exist_ok=True)
        if os.path.exists(socket_path):
            os.unlink(socket_path)
        self.server = grpc.aio.server()
        self.server.add_generic_rpc_handlers((generic_handler(A.IDENTITY, A.IDENTITY_METHODS, self),
                                              generic_handler(A.CONTROLLER, A.CONTROLLER_METHODS, self),
                                              generic_handler(A.NODE, A.NODE_METHODS, self)))
        self.server.add_insecure_port("unix://" + socket_path)
        await self.server.start()
        return self

    async def stop(self):
        if self.server is not None:
            await self.server.stop(0)


class CSIClient:
    """`pkg/volume/csi/csi_client.go`: the kubelet / attacher side of the socket."""

    def __init__(self, endpoint, timeout=15.0):
        from ..deviceplugin.api import _Stub
        target = endpoint if endpoint.startswith("unix:") else "unix://" + endpoint
        self.channel = grpc.aio.insecure_channel(target)
        self.identity = _Stub(self.channel, A.IDENTITY, A.IDENTITY_METHODS)
        self.controller = _Stub(self.channel, A.CONTROLLER, A.CONTROLLER_METHODS)
        self.node = _Stub(self.channel, A.NODE, A.NODE_METHODS)
        self.timeout = timeout

    async def assert_supported_version(self):
        r = await self.identity.GetSupportedVersions(A.MSG["GetSupportedVersionsRequest"](), timeout=self.timeout)
        if not any(v.major == 0 and v.minor == 1 for v in r.supported_versions):
            raise RuntimeError("CSI driver does not support version 0.1.x")

    @staticmethod
    def capability(access_modes=("ReadWriteOnce",), fs_type=""):
        mode = A.K8S_TO_CSI_MODE.get((access_modes or ["ReadWriteOnce"])[0], A.SINGLE_NODE_WRITER)
        return A.MSG["VolumeCapability"](mount=A.MSG["VolumeCapability_MountVolume"](fs_type=fs_type),
                                         access_mode=A.MSG["VolumeCapability_AccessMode"](mode=mode))

    async def node_publish(self, volume_id, target, readonly=False, publish_info=None, attributes=None,
                           access_modes=None, fs_type=""):
        await self.node.NodePublishVolume(A.MSG["NodePublishVolumeRequest"](
            version=A.VERSION, volume_id=volume_id, target_path=target, readonly=readonly,
            publish_volume_info=publish_info or {}, volume_attributes=attributes or {},
            volume_capability=self.capability(access_modes, fs_type)), timeout=self.timeout)

    async def node_unpublish(self, volume_id, target):
        await self.node.NodeUnpublishVolume(A.MSG["NodeUnpublishVolumeRequest"](
            version=A.VERSION, volume_id=volume_id, target_path=target), timeout=self.timeout)

    async def controller_publish(self, volume_id, node_id, readonly=False, attributes=None, access_modes=None):
        r = await self.controller.ControllerPublishVolume(A.MSG["ControllerPublishVolumeRequest"](
            version=A.VERSION, volume_id=volume_id, node_id=node_id, readonly=readonly,
            volume_attributes=attributes or {}, volume_capability=self.capability(access_modes)), timeout=self.timeout)
        return dict(r.publish_volume_info)

    async def controller_unpublish(self, volume_id, node_id):
        await self.controller.ControllerUnpublishVolume(A.MSG["ControllerUnpublishVolumeRequest"](
            version=A.VERSION, volume_id=volume_id, node_id=node_id), timeout=self.timeout)

    async def close(self):
        await self.channel.close()


# CSIPersistentVolumeSource in this API version (staging/src/k8s.io/api/core/v1/types.go:1693) has
# driver / volumeHandle / readOnly only; the attributes handed to the driver's ControllerPublish
# and NodePublish travel in this PV annotation (JSON map) — spec.csi.volumeAttributes is 1.10+.
VOLUME_ATTRIBUTES_ANNOTATION = "csi.volume.kubernetes.io/volume-attributes"


def volume_attributes(pv) -> dict:
    import json
    ann = ((pv or {}).get("metadata") or {}).get("annotations") or {}
    raw = ann.get(VOLUME_ATTRIBUTES_ANNOTATION)
    if not raw:
        return {}
    try:
        v = json.loads(raw)
    except ValueError:
        return {}
    return {str(k): str(x) for k, x in v.items()} if isinstance(v, dict) else {}
