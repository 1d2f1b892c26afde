"""Kubelet DeviceManager (fork F9) and its no-op stub.

Parity: `pkg/kubelet/cm/devicemanager/manager.go:46-339` (`ManagerImpl`: Start / run /
AdmitPod / GetCapacity / admitPod / PodResources / InitContainer / lazyPodDelete / Stop),
`manager_stub.go:28-71`, metric `kubelet_device_plugin_alloc_latency_microseconds`
(`pkg/kubelet/metrics/metrics.go:147-152`, observed around AdmitPod at manager.go:229-231).

Fixes over the reference:
  * item 1: AdmitPod rejects a pod whose assigned device is already held by another active pod
    (the reference only checks existence + health).
  * item 4: kubelet-restart race — an already-bound pod whose plugin has not re-registered yet
    waits up to `registration_grace` seconds instead of failing admission immediately.
  * registration count metric is actually incremented (quirk Q4).
"""
from __future__ import annotations

import asyncio
import logging
import os
import time

from ...api import core
from ...deviceplugin import api
from ...utils.metrics import MICRO_BUCKETS
from .endpoint import EndpointHandler, RegistrationError
from .stores import ManagerStore, PodCache, merge_init_responses
from .watcher import PluginWatcher

log = logging.getLogger("devicemanager")


class AdmitError(Exception):
    pass


class ManagerImpl:
    def __init__(self, plugins_dir=api.DEVICE_PLUGINS_PATH, metrics=None, registration_grace=10.0):
        self.plugins_dir = os.path.abspath(plugins_dir)
        self.store = ManagerStore()
        self.handler = EndpointHandler(self.store.update_capacity)
        self.watcher = PluginWatcher(self.plugins_dir)
        self.pod_cache = PodCache()
        self.active_pods = lambda: []
        self.registration_grace = registration_grace
        self._task = None
        self._registered = asyncio.Event()
        self.m_latency = self.m_reg = None
        if metrics is not None:
            self.m_latency = metrics.histogram("kubelet_device_plugin_alloc_latency_microseconds",
                                               "Duration in microseconds to serve a device plugin allocation request",
                                               ("resource_name",), MICRO_BUCKETS)
            self.m_reg = metrics.counter("kubelet_device_plugin_registration_count",
                                         "Cumulative number of device plugin registrations", ("resource_name",))

    # -- lifecycle ------------------------------------------------------------
    async def start(self, active_pods=None):
        if active_pods is not None:
            self.active_pods = active_pods
        self.watcher.start()
        self._task = asyncio.ensure_future(self._run())

    async def _run(self):
        while True:
            path = await self.watcher.added.get()
            domain = os.path.relpath(os.path.dirname(path), self.plugins_dir).strip("/")
            try:
                e = await self.handler.new_endpoint(path, domain)
            except (RegistrationError, OSError) as err:
                log.error("could not register endpoint %s: %s", path, err)
                continue
            except Exception:
                log.exception("endpoint registration crashed for %s", path)
                continue
            log.info("registered device plugin %s at %s", e.resource_name, path)
            if self.m_reg is not None:
                self.m_reg.labels(e.resource_name).inc()
            self._registered.set()

    async def stop(self):
        await self.handler.stop()
        self.watcher.stop()
        if self._task:
            self._task.cancel()

    # -- capacity -------------------------------------------------------------
    def get_capacity(self):
        return self.store.get_capacity()

    def add_capacity_listener(self, fn):
        self.store.listeners.append(fn)

    # -- admission ------------------------------------------------------------
    def _lazy_pod_delete(self):
        active = {p["metadata"]["uid"] for p in self.active_pods()}
        for uid in list(self.pod_cache.list_pods()):
            if uid not in active:
                self.pod_cache.delete_pod(uid)

    async def _wait_registered(self, rname):
        # the resource exists once the plugin registered AND its first ListAndWatch snapshot
        # landed; registration alone (the event) can precede the snapshot, so re-check on every
        # registration and at least every 10 ms
        deadline = time.monotonic() + self.registration_grace
        while not self.store.has_resource(rname) and time.monotonic() < deadline:
            self._registered.clear()
            try:
                await asyncio.wait_for(self._registered.wait(), max(0.0, min(0.01, deadline - time.monotonic())))
            except asyncio.TimeoutError:
                pass

    async def admit_pod(self, pod):
        self._lazy_pod_delete()
        rnames = []
        ers = (pod.get("spec") or {}).get("extendedResources") or []
        for per in ers:
            try:
                rname = core.pod_extended_resource_name(per)
            except ValueError as e:
                raise AdmitError(str(e))
            if not self.store.has_resource(rname) and self.registration_grace > 0:
                await self._wait_registered(rname)
            try:
                self.store.has_devices(rname, per.get("assigned") or [])
            except LookupError as e:
                raise AdmitError(str(e))
            if rname not in rnames:
                rnames.append(rname)
        if not rnames:
            return
        # duplicate assignment across active pods
        mine = core.pod_assigned_devices(pod)
        uid = pod["metadata"]["uid"]
        for other in self.active_pods():
            if other["metadata"]["uid"] == uid or core.pod_is_terminal(other):
                continue
            theirs = core.pod_assigned_devices(other)
            for rn, ids in mine.items():
                clash = set(ids) & set(theirs.get(rn, ()))
                if clash:
                    raise AdmitError(f"device(s) {sorted(clash)} of {rn} already assigned to pod "
                                     f"{other['metadata'].get('namespace')}/{other['metadata']['name']}")
        for rname in rnames:
            await self._admit_one(pod, rname)

    async def _admit_one(self, pod, rname):
        spec = pod.get("spec") or {}
        req = api.DP["AdmitPodRequest"](pod_name=pod["metadata"]["name"])
        for key, field in (("initContainers", req.init_containers), ("containers", req.containers)):
            for c in spec.get(key) or ():
                devs = core.pod_extended_resource_assigned(rname, c, pod)
                field[c["name"]].name = c["name"]
                field[c["name"]].devices.extend(devs)
        e = self.handler.endpoint(rname)
        if e is None:
            raise AdmitError(f"could not find Endpoint for {rname}")
        t0 = time.perf_counter()
        try:
            resp = await e.admit_pod(req)
        except Exception as err:  # grpc errors, timeouts
            raise AdmitError(f"device plugin {rname} rejected pod: {getattr(err, 'details', lambda: err)()}")
        finally:
            if self.m_latency is not None:
                self.m_latency.labels(rname).observe((time.perf_counter() - t0) * 1e6)
        self.pod_cache.cache_pod_resources(pod, resp)

    def pod_resources(self, pod):
        return self.pod_cache.pod_resources(pod)

    def delete_pod(self, uid):
        self.pod_cache.delete_pod(uid)

    async def init_container(self, pod, container):
        ers = (pod.get("spec") or {}).get("extendedResources") or []
        requests: dict[str, object] = {}
        for r in container.get("extendedResourceRequests") or ():
            i = core.pod_extended_resource_index(r, ers)
            rname = core.pod_extended_resource_name(ers[i])
            req = requests.get(rname)
            if req is None:
                req = requests[rname] = api.DP["InitContainerRequest"]()
                req.container.name = container["name"]
            req.container.devices.extend(ers[i].get("assigned") or [])
        responses = []
        for rname, req in requests.items():
            e = self.handler.endpoint(rname)
            if e is None:
                raise AdmitError(f"could not find Endpoint for {rname}")
            responses.append(await e.init_container(req))
        return merge_init_responses(responses)


class ManagerStub:
    """No-op manager used when the DevicePlugins feature gate is off (manager_stub.go:28-71)."""

    async def start(self, active_pods=None):
        pass

    async def stop(self):
        pass

    def get_capacity(self):
        return {}, []

    def add_capacity_listener(self, fn):
        pass

    async def admit_pod(self, pod):
        pass

    def pod_resources(self, pod):
        return None

    def delete_pod(self, uid):
        pass

    async def init_container(self, pod, container):
        return {"envs": [], "devices": [], "mounts": [], "annotations": []}
