"""Controller framework: shared informers + rate-limited work queue + N async workers.

Parity: the pattern every controller in `pkg/controller/*` follows (informer event handlers
enqueue keys; `processNextWorkItem` → `syncHandler(key)`; errors re-queued with
`AddRateLimited`, success `Forget`) and `controller.ControllerExpectations`
(`pkg/controller/controller_utils.go`) which stops a controller from acting twice on the same
intent before its informer has observed the result.
"""
from __future__ import annotations

import asyncio
import logging
import time

from ..api import meta as m
from ..api.labels import label_selector_as_selector
from ..client.events import EventRecorder
from ..parallel.workqueue import RateLimitingQueue

log = logging.getLogger("controller")


class Expectations:
    """Per-key outstanding creates/deletes; satisfied when both reach 0 or the entry expires."""

    TTL = 300.0

    def __init__(self):
        self._e: dict[str, list] = {}   # key -> [adds, dels, timestamp]

    def expect(self, key, adds=0, dels=0):
        self._e[key] = [adds, dels, time.monotonic()]

    def raise_(self, key, adds=0, dels=0):
        e = self._e.setdefault(key, [0, 0, time.monotonic()])
        e[0] += adds
        e[1] += dels

    def observe_add(self, key):
        e = self._e.get(key)
        if e:
            e[0] -= 1

    def observe_del(self, key):
        e = self._e.get(key)
        if e:
            e[1] -= 1

    def satisfied(self, key):
        e = self._e.get(key)
        if e is None:
            return True
        if e[0] <= 0 and e[1] <= 0:
            return True
        return time.monotonic() - e[2] > self.TTL

    def delete(self, key):
        self._e.pop(key, None)


class Controller:
    name = "controller"
    workers = 4
    # full resync (`--deployment-controller-sync-period`, `--namespace-sync-period`,
    # `--resource-quota-sync-period`, `--pvclaimbinder-sync-period`, `--service-sync-period`,
    # `--attach-detach-reconcile-sync-period`): every `resync_period` seconds each key from
    # resync_keys() is queued again, whether or not a watch event touched it; 0 = off
    resync_period = 0.0
    primary = None            # resource whose objects are the controller's keys

    def __init__(self, client, factory, recorder: EventRecorder | None = None):
        self.client = client
        self.factory = factory
        self.queue = RateLimitingQueue(self.name)
        self.recorder = recorder or EventRecorder(client, f"{self.name}-controller")
        self._tasks = []
        self.syncs = 0

    # subclasses: register informers/handlers in setup(), implement sync(key)
    def setup(self):
        raise NotImplementedError

    async def sync(self, key):
        raise NotImplementedError

    def enqueue(self, obj_or_key):
        key = obj_or_key if isinstance(obj_or_key, str) else m.ns_name(obj_or_key)
        self.queue.add(key)

    async def _worker(self):
        while True:
            key, shutdown = await self.queue.get()
            if shutdown:
                return
            try:
                # a sync returning False keeps the key's backoff history (the job controller counts
                # consecutive failed-pod retries against backoffLimit); anything else forgets it
                if await self.sync(key) is not False:
                    self.queue.forget(key)
                self.syncs += 1
            except asyncio.CancelledError:
                raise
            except Exception as e:
                log.debug("%s sync %s failed: %s", self.name, key, e)
                self.queue.add_rate_limited(key)
            finally:
                self.queue.done(key)

    def resync_keys(self):
        if self.primary is None:
            return []
        return [m.ns_name(o) for o in self.factory.get(self.primary).list()]

    async def _resync(self):
        while True:
            await asyncio.sleep(self.resync_period)
            for k in self.resync_keys():
                self.queue.add(k)

    def start(self):
        self.recorder.start()
        self._tasks = [asyncio.ensure_future(self._worker()) for _ in range(self.workers)]
        if self.resync_period > 0:
            self._tasks.append(asyncio.ensure_future(self._resync()))

    def stop(self):
        self.queue.shutdown()
        for t in self._tasks:
            t.cancel()
        self.recorder.stop()


def split_key(key):
    if "/" in key:
        ns, name = key.split("/", 1)
        return ns, name
    return None, key


def controller_ref(obj):
    return m.controller_of(obj)


def selector_of(obj):
    return label_selector_as_selector((obj.get("spec") or {}).get("selector"))


def pod_is_active(pod):
    st = (pod.get("status") or {}).get("phase")
    return st not in ("Succeeded", "Failed") and not (pod.get("metadata") or {}).get("deletionTimestamp")


def pod_is_ready(pod):
    for c in (pod.get("status") or {}).get("conditions") or ():
        if c.get("type") == "Ready":
            return c.get("status") == "True"
    return False


async def claim_objects(client, owner, resource, candidates, matches, ignore=None):
    """`ControllerRefManager.ClaimObject` over `candidates` (same namespace as `owner`):
    objects the owner controls stay claimed while they match and are released (their owner
    reference patched away) when they stop matching; orphans that match are adopted unless the
    owner is being deleted. `ignore(obj)` skips objects (e.g. terminating pods) for adoption and
    release. Returns the claimed objects (adopted ones as patched)."""
    uid = m.uid_of(owner)
    out = []
    for o in candidates:
        ref = controller_ref(o)
        ok = matches(o)
        if ref is not None:
            if ref.get("uid") != uid:
                continue
            if ok:
                out.append(o)
            elif not o["metadata"].get("deletionTimestamp") and not (ignore and ignore(o)):
                refs = [r for r in o["metadata"].get("ownerReferences") or () if r.get("uid") != uid]
                try:
                    await client.patch(resource, m.name_of(o), {"metadata": {"ownerReferences": refs or None,
                                                                             "uid": m.uid_of(o)}}, m.namespace_of(o))
                except Exception as e:      # noqa: BLE001 - a vanished or changed object is simply not ours
                    if getattr(e, "code", None) not in (404, 409, 422):
                        raise
            continue
        if not ok or owner["metadata"].get("deletionTimestamp") or o["metadata"].get("deletionTimestamp") or \
                (ignore and ignore(o)):
            continue
        refs = list(o["metadata"].get("ownerReferences") or ()) + [m.owner_reference(owner)]
        try:
            out.append(await client.patch(resource, m.name_of(o), {"metadata": {"ownerReferences": refs,
                                                                                "uid": m.uid_of(o)}},
                                          m.namespace_of(o)))
        except Exception as e:              # noqa: BLE001
            if getattr(e, "code", None) not in (404, 409, 422):
                raise
    return out


def _ready_time(pod):
    for c in (pod.get("status") or {}).get("conditions") or ():
        if c.get("type") == "Ready" and c.get("status") == "True":
            return m.parse_rfc3339(c.get("lastTransitionTime"))
    return None


def active_pods_key(pod):
    """Sort key of `controller.ActivePods` (`controller_utils.go:731`): pods to delete first
    sort first — unassigned < assigned; Pending < Unknown < Running; not ready < ready; among
    ready pods, ready for less time first (no transition time first of all); more container
    restarts first; newer first (no creation time first of all)."""
    st = pod.get("status") or {}
    ready = pod_is_ready(pod)
    phase = {"Pending": 0, "Unknown": 1, "Running": 2}.get(st.get("phase"), 0)
    if ready:
        rt = _ready_time(pod)
        ready_key = (0, 0.0) if rt is None else (1, -rt)
    else:
        ready_key = (0, 0.0)
    restarts = max((int(cs.get("restartCount") or 0) for cs in st.get("containerStatuses") or ()), default=0)
    ct = m.parse_rfc3339((pod.get("metadata") or {}).get("creationTimestamp"))
    created_key = (0, 0.0) if ct is None else (1, -ct)
    return (1 if (pod.get("spec") or {}).get("nodeName") else 0, phase, 1 if ready else 0, ready_key, -restarts,
            created_key)


def pod_is_available(pod, min_ready_seconds=0, now=None):
    """`podutil.IsPodAvailable`: Ready, and Ready for at least minReadySeconds."""
    for c in (pod.get("status") or {}).get("conditions") or ():
        if c.get("type") == "Ready":
            if c.get("status") != "True":
                return False
            if not min_ready_seconds:
                return True
            since = m.parse_rfc3339(c.get("lastTransitionTime"))
            if since is None:
                return False
            return since + int(min_ready_seconds) < (time.time() if now is None else now)
    return False


def pod_from_template(template, owner, generate_name, namespace):
    tmd = (template or {}).get("metadata") or {}
    pod = {"apiVersion": "v1", "kind": "Pod",
           "metadata": {"generateName": generate_name, "namespace": namespace,
                        "labels": dict(tmd.get("labels") or {}), "annotations": dict(tmd.get("annotations") or {}),
                        "ownerReferences": [m.owner_reference(owner)]},
           "spec": m.fast_copy((template or {}).get("spec") or {})}
    if not pod["metadata"]["annotations"]:
        del pod["metadata"]["annotations"]
    return pod
