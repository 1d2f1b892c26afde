"""Registration validator, per-plugin endpoint and the endpoint handler.

Parity:
  * Validator (`pkg/kubelet/apis/pluginregistration/v1beta/validation.go:32-141`): dial the unix
    socket (1 s), GetSupportedVersions must contain the kubelet's version, GetPluginIdentity
    resource name must be an extended resource name AND start with the directory domain,
    then PluginRegistrationStatus tells the plugin the outcome.
  * endpoint (`pkg/kubelet/cm/devicemanager/endpoint.go:34-223`): GetPluginInfo (1 s) gives
    init_timeout; Run consumes ListAndWatch and, when the stream ends, reports every device
    deleted; InitContainer is bounded by init_timeout. Fix: AdmitPod is
    bounded too (the reference has no timeout).
  * endpointHandler/endpointStore (`endpoint_handler.go:30-248`): a re-registering plugin
    inherits the old endpoint's device store; the old endpoint is silenced and stopped;
    `track_endpoint` removes an endpoint whose stream ended unless it was replaced.
"""
from __future__ import annotations

import asyncio
import logging

from ...api.core import is_extended_resource_name
from ...deviceplugin import api
from ...utils import grpclite
from .stores import AlwaysEmptyDeviceStore, DeviceStore

log = logging.getLogger("devicemanager")

ADMIT_TIMEOUT = 10.0


class RegistrationError(Exception):
    pass


class Validator:
    def __init__(self, version: str, domain: str):
        self.version = version
        self.domain = domain

    async def connect(self, socket_path: str, timeout=1.0):
        # grpclite: gRPC over HTTP/2 on the kubelet's loop (utils/grpclite.py); any gRPC plugin
        # server answers it
        ch = grpclite.Channel("unix://" + socket_path)
        try:
            await asyncio.wait_for(ch.channel_ready(), timeout)
        except (asyncio.TimeoutError, grpclite.RpcError):
            await ch.close()
            raise RegistrationError(f"failed to dial device plugin {socket_path}")
        return ch

    async def validate_endpoint(self, ch) -> str:
        ident = api.identity_stub(ch)
        vs = await ident.GetSupportedVersions(api.PR["GetSupportedVersionsRequest"](), timeout=1.0)
        if self.version not in vs.supported_versions:
            raise RegistrationError(f"kubelet version {self.version} not in plugin supported versions {list(vs.supported_versions)}")
        idr = await ident.GetPluginIdentity(api.PR["GetPluginIdentityRequest"](version=self.version), timeout=1.0)
        name = idr.resource_name
        if not is_extended_resource_name(name):
            raise RegistrationError(f"invalid name of device plugin socket: {name} is not an extended resource name")
        if not name.startswith(self.domain):
            raise RegistrationError(f"resource name {name} does not start with the plugin domain {self.domain}")
        return name

    async def notify(self, ch, err: Exception | None):
        ident = api.identity_stub(ch)
        try:
            await ident.PluginRegistrationStatus(api.PR["RegistrationStatus"](success=err is None, error=str(err or "")), timeout=1.0)
        except grpclite.RpcError as e:
            log.warning("could not notify plugin of registration status: %s", e.code())


class Endpoint:
    def __init__(self, channel, resource_name: str, socket_path: str):
        self.channel = channel
        self.resource_name = resource_name
        self.socket_path = socket_path
        self.stub = api.device_plugin_stub(channel)
        self.store: DeviceStore = DeviceStore()
        self.init_timeout = 1
        self.labels = {}
        self._call = None
        self._stopped = False
        self.superseded = False      # a re-registration took over this endpoint's device store

    async def init(self):
        info = await self.stub.GetPluginInfo(api.DP["GetPluginInfoRequest"](), timeout=1.0)
        self.init_timeout = info.init_timeout or 1
        self.labels = dict(info.labels)

    async def run(self):
        """Consume ListAndWatch until the stream ends; then report all devices deleted."""
        try:
            self._call = self.stub.ListAndWatch(api.DP["ListAndWatchRequest"]())
            async for resp in self._call:
                added, updated, deleted = self.store.update(resp.devices)
                if added or updated or deleted:
                    self.store.fire(self.resource_name, added, updated, deleted)
        except grpclite.RpcError as e:
            if not self._stopped:
                log.warning("ListAndWatch %s ended: %s", self.resource_name, e.code())
        except asyncio.CancelledError:
            pass
        finally:
            # the stream ended: report every device deleted — unless a re-registering endpoint
            # already owns this store (its devices live on under the new plugin)
            if not self.superseded:
                _, _, deleted = self.store.update([])
                if deleted:
                    self.store.fire(self.resource_name, [], [], deleted)

    async def init_container(self, req):
        return await self.stub.InitContainer(req, timeout=float(self.init_timeout))

    async def admit_pod(self, req):
        return await self.stub.AdmitPod(req, timeout=ADMIT_TIMEOUT)

    async def stop(self):
        self._stopped = True
        if self._call is not None:
            self._call.cancel()
        await self.channel.close()


class EndpointHandler:
    def __init__(self, callback, version=api.VERSION):
        self.callback = callback
        self.version = version
        self.endpoints: dict[str, Endpoint] = {}
        self._tasks: dict[Endpoint, asyncio.Task] = {}
        self.swap_hook = None  # test shim: awaited between store hand-over and swap (endpointStoreShim)

    def endpoint(self, resource):
        return self.endpoints.get(resource)

    async def new_endpoint(self, socket_path: str, domain: str) -> Endpoint:
        v = Validator(self.version, domain)
        ch = await v.connect(socket_path, 1.0)
        try:
            name = await v.validate_endpoint(ch)
        except (RegistrationError, grpclite.RpcError) as e:
            await v.notify(ch, e)
            await ch.close()
            raise RegistrationError(str(e)) from e
        await v.notify(ch, None)
        e = Endpoint(ch, name, socket_path)
        try:
            await e.init()
        except grpclite.RpcError as err:
            await ch.close()
            raise RegistrationError(f"GetPluginInfo failed: {err.code()}") from err
        old = self.endpoints.get(name)
        if old is not None:
            e.store = old.store           # carry devices over to the new endpoint
            old.superseded = True         # its stream ending from now on must not delete them
        else:
            e.store = DeviceStore(self.callback)
        if self.swap_hook is not None:
            await self.swap_hook(e)
        # the old endpoint may have ended (and left the table) while we were suspended
        cur = self.endpoints.get(name)
        self.endpoints[name] = e
        self._tasks[e] = asyncio.ensure_future(self._track(e))
        for o in {x for x in (old, cur) if x is not None and x is not e}:
            o.superseded = True
            o.store = AlwaysEmptyDeviceStore()     # silence before stopping
            await o.stop()
        return e

    async def _track(self, e: Endpoint):
        await e.run()
        self._tasks.pop(e, None)
        if self.endpoints.get(e.resource_name) is e:
            del self.endpoints[e.resource_name]

    async def stop(self):
        for e in list(self.endpoints.values()):
            await e.stop()
        for t in list(self._tasks.values()):
            t.cancel()
        self.endpoints.clear()

    def devices(self):
        return {n: e.store.devices_list() for n, e in self.endpoints.items()}
