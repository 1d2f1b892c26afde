"""Device plugin server base: serves DevicePlugin + Identity on one unix socket.

Transport: `utils/grpclite` (gRPC over HTTP/2 on the event loop; a unary call costs a fraction
of grpc.aio's CPU, which matters because AdmitPod/InitContainer run for every GPU pod) or
`transport="grpc"` (grpc.aio). Both speak the same wire protocol to any gRPC kubelet.

Parity: the reference's test double `DevicePluginStub` (pkg/kubelet/cm/devicemanager/device_plugin_stub.go:41-276)
doubles as the production base class here: `update(devices)` pushes a new device list to every
open ListAndWatch stream, `admit_fn` / `init_fn` are pluggable (`InitStubFunc`).

Socket layout (`pkg/kubelet/apis/deviceplugin/v1alpha/constants.go:31-35`, watcher rules
`pkg/kubelet/apis/pluginregistration/v1beta/plugin_watcher.go:222-244`):
    <plugins_dir>/<vendor domain>/<socket>       e.g. .../plugins/amd.com/amdgpu.sock
"""
from __future__ import annotations

import asyncio
import logging
import os

import grpc

from ..utils import grpclite
from . import api

log = logging.getLogger("deviceplugin")


def device(id_, health=api.HEALTHY, attributes=None):
    return api.DP["Device"](ID=id_, health=health, Attributes=attributes or {})


class DevicePluginServer:
    def __init__(self, resource_name: str, socket_path: str, devices=None, init_timeout=10,
                 supported_versions=(api.VERSION,), labels=None, transport="lite"):
        self.resource_name = resource_name
        self.socket_path = socket_path
        self.devices = list(devices or [])
        self.init_timeout = init_timeout
        self.supported_versions = list(supported_versions)
        self.labels = dict(labels or {})
        self.transport = transport
        self.registration_status = None      # last PluginRegistrationStatus from the kubelet
        self.registered = asyncio.Event()
        self._streams: set[asyncio.Queue] = set()
        self._server = None
        self.admit_calls = 0
        self.init_calls = 0

    # -- hooks for subclasses ------------------------------------------------
    async def admit_pod(self, request) -> dict:
        """Return pod annotations (AdmitPodResponse.pod.annotations)."""
        return {}

    async def init_container(self, container) -> dict:
        """Return {"envs":{}, "mounts":[{...}], "devices":[{...}], "annotations":{}}."""
        return {}

    # -- device list updates ---------------------------------------------------
    def update(self, devices):
        self.devices = list(devices)
        for q in list(self._streams):
            q.put_nowait(list(self.devices))

    # -- DevicePlugin service ---------------------------------------------------
    async def GetPluginInfo(self, request, context):
        return api.DP["GetPluginInfoResponse"](init_timeout=self.init_timeout, labels=self.labels)

    async def ListAndWatch(self, request, context):
        q: asyncio.Queue = asyncio.Queue()
        self._streams.add(q)
        try:
            yield api.DP["ListAndWatchResponse"](devices=self.devices)
            while True:
                devs = await q.get()
                if devs is None:
                    return
                yield api.DP["ListAndWatchResponse"](devices=devs)
        finally:
            self._streams.discard(q)

    async def AdmitPod(self, request, context):
        self.admit_calls += 1
        ann = await self.admit_pod(request)
        return api.DP["AdmitPodResponse"](pod=api.DP["PodSpec"](annotations=ann or {}))

    async def InitContainer(self, request, context):
        self.init_calls += 1
        spec = await self.init_container(request.container)
        cs = api.DP["ContainerSpec"](envs=spec.get("envs") or {}, annotations=spec.get("annotations") or {})
        for m in spec.get("mounts") or ():
            cs.mounts.add(**m)
        for d in spec.get("devices") or ():
            cs.devices.add(**d)
        return api.DP["InitContainerResponse"](spec=cs)

    # -- Identity service ----------------------------------------------------------
    async def GetSupportedVersions(self, request, context):
        return api.PR["GetSupportedVersionsResponse"](supported_versions=self.supported_versions)

    async def GetPluginIdentity(self, request, context):
        return api.PR["GetPluginIdentityResponse"](resource_name=self.resource_name)

    async def PluginRegistrationStatus(self, request, context):
        self.registration_status = (request.success, request.error)
        if request.success:
            self.registered.set()
        else:
            log.error("plugin %s registration failed: %s", self.resource_name, request.error)
        return api.PR["Empty"]()

    # -- lifecycle -----------------------------------------------------------------
    async def start(self):
        os.makedirs(os.path.dirname(self.socket_path), exist_ok=True)
        if os.path.exists(self.socket_path):
            os.unlink(self.socket_path)
        if self.transport == "grpc":
            self._server = grpc.aio.server(options=[("grpc.so_reuseport", 0)])
            self._server.add_generic_rpc_handlers((
                api.generic_handler(api.DP_SERVICE, api.DP_METHODS, self),
                api.generic_handler(api.ID_SERVICE, api.ID_METHODS, self),
            ))
        else:
            self._server = grpclite.Server()
            self._server.add_service(api.DP_SERVICE, api.DP_METHODS, self)
            self._server.add_service(api.ID_SERVICE, api.ID_METHODS, self)
        self._server.add_insecure_port("unix://" + self.socket_path)
        await self._server.start()
        return self

    async def stop(self, grace=0.1):
        for q in list(self._streams):
            q.put_nowait(None)
        if self._server is not None:
            await self._server.stop(grace)
            self._server = None
        try:
            os.unlink(self.socket_path)
        except FileNotFoundError:
            pass
