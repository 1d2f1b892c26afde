"""Device manager data stores.

  * DeviceStore   — per endpoint; diffs each ListAndWatch snapshot into added / updated
                    (health change only) / deleted and invokes the manager callback
                    (`pkg/kubelet/cm/devicemanager/device_store.go:25-183`, incl.
                    `alwaysEmptyDeviceStore` to silence a replaced endpoint).
  * ManagerStore  — node-level ExtendedResourceMap (`manager_store.go:29-130`): GetCapacity
                    returns a clone plus resource names removed since the last call;
                    HasDevices requires existence AND Healthy.
  * PodCache      — pod UID -> RunPodOptions{annotations} from AdmitPod (`cache.go:26-101`);
                    a None response is tolerated (reference quirk Q7 dereferenced it).
  * merge_init_responses — `DeviceRunContainerOptionsFromInitResponses`
                    (`device_run_container_options.go:24-113`): first value wins on conflict.
"""
from __future__ import annotations

import logging
import threading

from ...deviceplugin import api

log = logging.getLogger("devicemanager")


def plugin_device_to_v1(d) -> dict:
    return {"id": d.ID, "health": d.health, "attributes": dict(d.Attributes)}


class DeviceStore:
    def __init__(self, callback=None):
        self.devices: dict[str, object] = {}
        self.callback = callback
        self._lock = threading.Lock()

    def update(self, devs):
        added, updated, deleted = [], [], []
        new = {}
        with self._lock:
            for d in devs:
                new[d.ID] = d
                old = self.devices.get(d.ID)
                if old is None:
                    self.devices[d.ID] = d
                    added.append(d)
                elif d.health != old.health or dict(d.Attributes) != dict(old.Attributes):
                    # the reference only propagates health changes; attribute changes (e.g. the
                    # ECC counter) are propagated too so Node.status stays truthful
                    self.devices[d.ID] = d
                    updated.append(d)
            for did in [k for k in self.devices if k not in new]:
                deleted.append(self.devices.pop(did))
        return added, updated, deleted

    def devices_list(self):
        with self._lock:
            return list(self.devices.values())

    def fire(self, resource, added, updated, deleted):
        if self.callback is not None:
            self.callback(resource, added, updated, deleted)


class AlwaysEmptyDeviceStore(DeviceStore):
    def update(self, devs):
        return [], [], []

    def fire(self, *a):
        pass


class ManagerStore:
    def __init__(self):
        self.resources: dict[str, dict] = {}   # rname -> {"resources": {id: ExtendedResource}}
        self.removed: list[str] = []
        self._lock = threading.Lock()
        self.listeners = []                   # called after every capacity change

    def update_capacity(self, res, added, updated, deleted):
        with self._lock:
            dom = self.resources.setdefault(res, {"resources": {}})
            for d in list(added) + list(updated):
                dom["resources"][d.ID] = plugin_device_to_v1(d)
            for d in deleted:
                dom["resources"].pop(d.ID, None)
            if not dom["resources"]:
                del self.resources[res]
                self.removed.append(res)
        for fn in self.listeners:
            try:
                fn(res)
            except Exception:
                log.exception("capacity listener failed")

    def get_capacity(self):
        with self._lock:
            clone = {k: {"resources": {i: {"id": r["id"], "health": r["health"], "attributes": dict(r["attributes"])}
                                       for i, r in v["resources"].items()}} for k, v in self.resources.items()}
            removed, self.removed = self.removed, []
        return clone, removed

    def has_devices(self, res, ids):
        with self._lock:
            dom = self.resources.get(res)
            if dom is None:
                raise LookupError(f"resource {res} not available on this node")
            for i in ids:
                r = dom["resources"].get(i)
                if r is None:
                    raise LookupError(f"resource {res}/{i} not available on this node")
                if r["health"] != api.HEALTHY:
                    raise LookupError(f"resource {res}/{i} is unhealthy on this node")

    def has_resource(self, res) -> bool:
        with self._lock:
            return res in self.resources


class PodCache:
    def __init__(self):
        self.pods: dict[str, dict] = {}
        self._lock = threading.Lock()

    def cache_pod_resources(self, pod, resp):
        uid = pod["metadata"]["uid"]
        ann = dict(resp.pod.annotations) if (resp is not None and resp.HasField("pod")) else {}
        with self._lock:
            cur = self.pods.setdefault(uid, {"annotations": {}})
            for k, v in ann.items():
                cur["annotations"].setdefault(k, v)

    def pod_resources(self, pod):
        with self._lock:
            r = self.pods.get(pod["metadata"]["uid"])
            return {"annotations": dict(r["annotations"])} if r else None

    def delete_pod(self, uid):
        with self._lock:
            self.pods.pop(uid, None)

    def list_pods(self):
        with self._lock:
            return dict(self.pods)


def merge_init_responses(responses) -> dict:
    opts = {"envs": [], "devices": [], "mounts": [], "annotations": []}
    envs, devs, mounts, anns = {}, {}, {}, {}
    for resp in responses:
        spec = resp.spec
        for k, v in spec.envs.items():
            if k in envs:
                if envs[k] != v:
                    log.error("Environment variable %s has conflicting setting: %s and %s", k, envs[k], v)
                continue
            envs[k] = v
            opts["envs"].append({"name": k, "value": v})
        for d in spec.devices:
            if d.container_path in devs:
                if devs[d.container_path] != d.host_path:
                    log.error("Container device %s has conflicting mapping host devices: %s and %s",
                              d.container_path, devs[d.container_path], d.host_path)
                continue
            devs[d.container_path] = d.host_path
            opts["devices"].append({"pathOnHost": d.host_path, "pathInContainer": d.container_path,
                                    "permissions": d.permissions})
        for m in spec.mounts:
            if m.container_path in mounts:
                if mounts[m.container_path] != m.host_path:
                    log.error("Container mount %s has conflicting mapping host mounts: %s and %s",
                              m.container_path, mounts[m.container_path], m.host_path)
                continue
            mounts[m.container_path] = m.host_path
            opts["mounts"].append({"name": m.container_path, "containerPath": m.container_path,
                                   "hostPath": m.host_path, "readOnly": m.read_only})
        for k, v in spec.annotations.items():
            if k in anns:
                if anns[k] != v:
                    log.error("Annotation %s has conflicting setting: %s and %s", k, anns[k], v)
                continue
            anns[k] = v
            opts["annotations"].append({"name": k, "value": v})
    return opts
