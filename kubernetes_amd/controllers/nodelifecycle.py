"""Node lifecycle: node health monitoring, zone disruption, rate-limited evictions and the
NoExecute taint manager.

Parity: `pkg/controller/node/node_controller.go` and `pkg/controller/node/scheduler/`.

  * monitor pass every `monitor_period` (`monitorNodeStatus`, :619): the local time of the last
    heartbeat change per node is tracked (never the node's own clock); a node silent for longer
    than `grace` (`startup_grace` if it never posted a Ready condition) gets Ready and the
    pressure conditions set to Unknown (`tryUpdateNodeStatus`, :916); a Ready -> not-Ready
    transition records NodeNotReady and marks every pod on the node not ready
    (`MarkAllPodsNotReady`).
  * zones (`failure-domain.beta.kubernetes.io/region` + `/zone`), each with a rate-limited timed
    queue of nodes (`RateLimitedTimedQueue`, token bucket of burst 1). Zone state from the Ready
    conditions (`ComputeZoneState`, :1183): FullDisruption when no node is Ready,
    PartialDisruption when more than 2 and at least `unhealthy_zone_threshold` of them are not
    Ready, Normal otherwise. Rates (`setLimiterInZone`, :887): Normal -> `eviction_rate`;
    Partial -> `secondary_eviction_rate` above `large_cluster_threshold` nodes, else 0 (stop);
    Full -> `eviction_rate`; every zone fully disrupted -> all evictions stop and queued ones are
    cancelled (the master is the likely partitioned party); leaving that mode resets the probe
    timestamps of all nodes (`handleDisruption`, :789).
  * eviction mode (TaintBasedEvictions off, the 1.9 default): a node NotReady / Unknown for
    `pod_eviction_timeout` is queued; the eviction pass (every 100 ms) deletes its pods except
    DaemonSet pods, setting reason NodeLost first (`util.DeletePods`); a Ready node is removed
    from the queue (`cancelPodEviction`).
  * taint mode (TaintBasedEvictions on): the queue rate-limits adding the `not-ready` /
    `unreachable` NoExecute taints (mutually exclusive, swapped at once); a Ready node loses
    both (`doNoExecuteTaintingPass`, :515, `markNodeAsReachable`).
  * NoExecute taint manager (`taint_controller.go`): a pod on a node with NoExecute taints it
    does not all tolerate is deleted at once; otherwise at the minimum `tolerationSeconds` of the
    tolerations used (never, when none has a limit); removed taints cancel scheduled deletions.
  * TaintNodesByCondition: NoSchedule taints mirror MemoryPressure / DiskPressure / OutOfDisk /
    NetworkUnavailable (`doNoScheduleTaintingPass`, :487); deprecated
    `node.alpha.kubernetes.io/{notReady,unreachable}` keys are rewritten
    (`doFixDeprecatedTaintKeyPass`, :450).

GPU pods evicted here release their device IDs through the normal delete path.
"""
from __future__ import annotations

import asyncio
import heapq
import itertools
import logging
import time

from ..api import core
from ..api.meta import now_rfc3339
from ..client.rest import APIStatusError, is_not_found
from ..utils.features import DefaultFeatureGate
from .base import Controller, controller_ref

log = logging.getLogger("nodelifecycle")

NOT_READY_TAINT = "node.kubernetes.io/not-ready"
UNREACHABLE_TAINT = "node.kubernetes.io/unreachable"
DEPRECATED_TAINTS = {"node.alpha.kubernetes.io/notReady": NOT_READY_TAINT,
                     "node.alpha.kubernetes.io/unreachable": UNREACHABLE_TAINT}
CONDITION_TAINTS = {"MemoryPressure": "node.kubernetes.io/memory-pressure",
                    "OutOfDisk": "node.kubernetes.io/out-of-disk",
                    "DiskPressure": "node.kubernetes.io/disk-pressure",
                    "NetworkUnavailable": "node.kubernetes.io/network-unavailable"}
ZONE_LABEL = "failure-domain.beta.kubernetes.io/zone"
REGION_LABEL = "failure-domain.beta.kubernetes.io/region"
INITIAL, NORMAL, FULL, PARTIAL = "Initial", "Normal", "FullDisruption", "PartialDisruption"
NODE_LOST = "NodeLost"


def zone_key(node) -> str:
    """`utilnode.GetZoneKey`: "" when the node carries neither label."""
    labels = (node.get("metadata") or {}).get("labels") or {}
    region, zone = labels.get(REGION_LABEL, ""), labels.get(ZONE_LABEL, "")
    return f"{region}:\x00:{zone}" if region or zone else ""


class TokenBucket:
    """`flowcontrol.NewTokenBucketRateLimiter(qps, burst)`; qps <= 0 never admits."""

    def __init__(self, qps, burst=1, clock=time.monotonic):
        self.qps, self.burst, self.clock = float(qps), burst, clock
        self.tokens, self.last = float(burst), clock()

    def try_accept(self) -> bool:
        if self.qps <= 0:
            return False
        now = self.clock()
        self.tokens = min(self.burst, self.tokens + (now - self.last) * self.qps)
        self.last = now
        if self.tokens >= 1:
            self.tokens -= 1
            return True
        return False


class RateLimitedTimedQueue:
    """`scheduler.RateLimitedTimedQueue`: unique values ordered by process time; an entry stays
    known after it was processed (so it is not queued again) until `remove` forgets it."""

    def __init__(self, qps, clock=time.monotonic):
        self.clock = clock
        self.qps = qps
        self.limiter = TokenBucket(qps, 1, clock)
        self.heap: list = []
        self.items: dict[str, list] = {}      # value -> [process_at, seq, uid, added_at, queued]
        self._seq = itertools.count()

    def add(self, value, uid="") -> bool:
        if value in self.items:
            return False
        now = self.clock()
        e = [now, next(self._seq), uid, now, True]
        self.items[value] = e
        heapq.heappush(self.heap, (e[0], e[1], value))
        return True

    def remove(self, value) -> bool:
        return self.items.pop(value, None) is not None

    def swap_limiter(self, qps):
        if qps == self.qps:
            return
        self.qps = qps
        self.limiter = TokenBucket(qps, 1, self.clock)

    def queued(self):
        return [v for v, e in self.items.items() if e[4]]

    async def try_(self, fn):
        """fn(value, uid) -> (done, retry_after). Process due entries while tokens last."""
        while self.heap:
            at, seq, value = self.heap[0]
            e = self.items.get(value)
            if e is None or e[1] != seq or not e[4]:
                heapq.heappop(self.heap)        # forgotten or superseded entry
                continue
            now = self.clock()
            if now < at:
                return
            if not self.limiter.try_accept():
                return
            heapq.heappop(self.heap)
            done, wait = await fn(value, e[2])
            if value not in self.items:
                continue
            if done:
                e[4] = False
            else:
                e[0], e[1] = now + wait + 0.001, next(self._seq)
                heapq.heappush(self.heap, (e[0], e[1], value))


def compute_zone_state(ready_conditions, unhealthy_threshold=0.55):
    ready = sum(1 for c in ready_conditions if c is not None and c.get("status") == "True")
    not_ready = len(ready_conditions) - ready
    if ready == 0 and not_ready > 0:
        return not_ready, FULL
    if not_ready > 2 and not_ready / (not_ready + ready) >= unhealthy_threshold:
        return not_ready, PARTIAL
    return not_ready, NORMAL


def min_toleration_time(used):
    """`getMinTolerationTime`: 0 with no tolerations, None for 'forever'."""
    if not used:
        return 0.0
    best = None
    for t in used:
        s = t.get("tolerationSeconds")
        if s is None:
            continue
        if s <= 0:
            return 0.0
        best = s if best is None else min(best, s)
    return None if best is None else float(best)


def matching_tolerations(taints, tolerations):
    """`v1helper.GetMatchingTolerations` -> (all tolerated, tolerations used)."""
    used = []
    for taint in taints:
        hit = [t for t in tolerations or () if core.tolerates([t], taint)]
        if not hit:
            return False, []
        used += hit
    return True, used


class NodeLifecycleController(Controller):
    name = "nodelifecycle"
    workers = 2

    def __init__(self, client, factory, recorder=None, monitor_period=5.0, grace=40.0, startup_grace=60.0,
                 pod_eviction_timeout=300.0, eviction_rate=0.1, secondary_eviction_rate=0.01,
                 large_cluster_threshold=50, unhealthy_zone_threshold=0.55, taint_based_evictions=None,
                 taint_manager=True, taint_nodes_by_condition=None, eviction_period=0.1, clock=time.monotonic):
        super().__init__(client, factory, recorder)
        self.monitor_period, self.grace, self.startup_grace = monitor_period, grace, startup_grace
        self.eviction_timeout = pod_eviction_timeout
        self.eviction_rate, self.secondary_rate = eviction_rate, secondary_eviction_rate
        self.large_cluster, self.unhealthy_threshold = large_cluster_threshold, unhealthy_zone_threshold
        self.taint_mode = (DefaultFeatureGate("TaintBasedEvictions") if taint_based_evictions is None
                           else taint_based_evictions)
        self.by_condition = (DefaultFeatureGate("TaintNodesByCondition") if taint_nodes_by_condition is None
                             else taint_nodes_by_condition)
        self.run_taint_manager = taint_manager
        self.eviction_period = eviction_period
        self.clock = clock
        # name -> {"ready": observed Ready condition, "probe": t, "transition": t}
        self.status: dict[str, dict] = {}
        self.known: dict[str, dict] = {}
        self.zone_states: dict[str, str] = {}
        self.zone_queues: dict[str, RateLimitedTimedQueue] = {}
        self.tainted: dict[str, list] = {}     # taint manager: node -> NoExecute taints
        self.scheduled: dict[str, tuple] = {}  # pod key -> (created, trigger, timer handle)
        self._loops = []

    # -- wiring -----------------------------------------------------------------------------
    def setup(self):
        self.node_inf = self.factory.get("nodes")
        self.pod_inf = self.factory.get("pods")
        self.ds_inf = self.factory.get("daemonsets")
        if "nodeName" not in self.pod_inf.store.indexers:
            self.pod_inf.store.add_indexer("nodeName", lambda p: [(p.get("spec") or {}).get("nodeName", "")])
        if self.run_taint_manager:
            self.node_inf.add_handler(lambda n: self.enqueue("node/" + n["metadata"]["name"]),
                                      self._node_updated, lambda n: self.enqueue("node/" + n["metadata"]["name"]))
            self.pod_inf.add_handler(self._pod_event, lambda o, n: self._pod_updated(o, n), self._pod_deleted)

    def start(self):
        super().start()
        self._loops = [asyncio.ensure_future(self._every(self.monitor_period, self.monitor)),
                       asyncio.ensure_future(self._every(self.eviction_period, self._queue_pass))]

    def stop(self):
        super().stop()
        for t in self._loops:
            t.cancel()
        for _c, _t, h in self.scheduled.values():
            h.cancel()
        self.scheduled.clear()

    async def _every(self, period, fn):
        while True:
            await asyncio.sleep(period)
            try:
                await fn()
            except APIStatusError as e:
                log.warning("node lifecycle pass: %s", e)

    # -- monitor --------------------------------------------------------------------------------
    def _queue_for(self, zone):
        q = self.zone_queues.get(zone)
        if q is None:
            q = self.zone_queues[zone] = RateLimitedTimedQueue(self.eviction_rate, self.clock)
            self.zone_states.setdefault(zone, INITIAL)
        return q

    async def monitor(self):
        nodes = self.node_inf.list()
        names = {n["metadata"]["name"] for n in nodes}
        for n in nodes:
            name = n["metadata"]["name"]
            self._queue_for(zone_key(n))
            if name not in self.known:
                self.known[name] = n
                self.recorder.event(n, "Normal", "RegisteredNode", f"Registered Node {name} in Controller")
                if self.taint_mode:
                    await self._mark_reachable(n)
                else:
                    self._cancel_eviction(n)
        for name in list(self.known):
            if name not in names:
                self.recorder.event(self.known.pop(name), "Normal", "RemovingNode", f"Removing Node {name} from Controller")
                self.status.pop(name, None)
        zone_conditions: dict[str, list] = {}
        for n in nodes:
            name = n["metadata"]["name"]
            if any(t.get("key") in DEPRECATED_TAINTS for t in (n.get("spec") or {}).get("taints") or ()):
                n = await self._fix_deprecated_taints(n)
            if self.by_condition:
                n = await self._condition_taints(n)
            try:
                observed, current = await self._update_status(n)
            except APIStatusError as e:
                if is_not_found(e):
                    continue
                raise
            zone_conditions.setdefault(zone_key(n), []).append(current)
            now = self.clock()
            st = self.status[name]
            status = observed.get("status")
            if status == "False":
                if self.taint_mode:
                    if self._has_taint(n, UNREACHABLE_TAINT):
                        await self._swap_taints(n, NOT_READY_TAINT, UNREACHABLE_TAINT)
                    else:
                        self._queue_for(zone_key(n)).add(name, n["metadata"].get("uid", ""))
                elif now > st["transition"] + self.eviction_timeout:
                    self._queue_for(zone_key(n)).add(name, n["metadata"].get("uid", ""))
            elif status == "Unknown":
                if self.taint_mode:
                    if self._has_taint(n, NOT_READY_TAINT):
                        await self._swap_taints(n, UNREACHABLE_TAINT, NOT_READY_TAINT)
                    else:
                        self._queue_for(zone_key(n)).add(name, n["metadata"].get("uid", ""))
                elif now > st["probe"] + self.eviction_timeout:
                    self._queue_for(zone_key(n)).add(name, n["metadata"].get("uid", ""))
            elif status == "True":
                if self.taint_mode:
                    await self._mark_reachable(n)
                else:
                    self._cancel_eviction(n)
            if current is not None and current.get("status") != "True" and status == "True":
                self.recorder.event(n, "Normal", "NodeNotReady", f"Node {name} status is now: NodeNotReady")
                await self._mark_pods_not_ready(name)
        await self._handle_disruption(zone_conditions, nodes)

    async def _update_status(self, node):
        """`tryUpdateNodeStatus` -> (observed Ready condition, current Ready condition after the
        update, None when the kubelet never posted one)."""
        name = node["metadata"]["name"]
        now = self.clock()
        status = node.get("status") or {}
        current = core.get_condition(status, "Ready")
        if current is None:
            observed = {"type": "Ready", "status": "Unknown"}
            grace = self.startup_grace
        else:
            observed = dict(current)
            grace = self.grace
        saved = self.status.get(name)
        if saved is None or (saved["ready"] is None) != (current is None):
            saved = {"ready": current and dict(current), "probe": now, "transition": now}
        elif current is not None and saved["ready"].get("lastHeartbeatTime") != current.get("lastHeartbeatTime"):
            transition = now if saved["ready"].get("lastTransitionTime") != current.get("lastTransitionTime") \
                else saved["transition"]
            saved = {"ready": dict(current), "probe": now, "transition": transition}
        self.status[name] = saved
        if now <= saved["probe"] + grace:
            return observed, current
        conds = [dict(c) for c in status.get("conditions") or ()]
        stamp = now_rfc3339()
        by_type = {c.get("type"): c for c in conds}
        changed = False
        for ctype in ("Ready", "MemoryPressure", "DiskPressure"):
            c = by_type.get(ctype)
            if c is None:
                conds.append({"type": ctype, "status": "Unknown", "reason": "NodeStatusNeverUpdated",
                              "message": "Kubelet never posted node status.",
                              "lastHeartbeatTime": node["metadata"].get("creationTimestamp"),
                              "lastTransitionTime": stamp})
                changed = changed or ctype == "Ready"
            elif c.get("status") != "Unknown":
                c.update(status="Unknown", reason="NodeStatusUnknown", message="Kubelet stopped posting node status.",
                         lastTransitionTime=stamp)
                changed = changed or ctype == "Ready"
        if changed:
            await self.client.patch("nodes", name, {"status": {"conditions": conds}}, None, "merge", "status")
            self.status[name] = {"ready": saved["ready"], "probe": saved["probe"], "transition": now}
            current = next(c for c in conds if c.get("type") == "Ready")
        return observed, current

    async def _handle_disruption(self, zone_conditions, nodes):
        new_states = {}
        all_full = True
        for zone, conds in zone_conditions.items():
            _unhealthy, st = compute_zone_state(conds, self.unhealthy_threshold)
            all_full = all_full and st == FULL
            new_states[zone] = st
            self.zone_states.setdefault(zone, INITIAL)
        all_were_full = True
        for zone in list(self.zone_states):
            if zone not in zone_conditions:
                del self.zone_states[zone]
                continue
            if self.zone_states[zone] != FULL:
                all_were_full = False
        if not zone_conditions:
            return
        if all_full and all_were_full:
            return
        if all_full:
            log.warning("all nodes are not Ready: entering master disruption mode, evictions stopped")
            for n in nodes:
                if self.taint_mode:
                    await self._mark_reachable(n)
                else:
                    self._cancel_eviction(n)
            for zone in self.zone_states:
                self._queue_for(zone).swap_limiter(0)
                self.zone_states[zone] = FULL
            return
        if all_were_full:
            log.warning("some nodes are Ready again: leaving master disruption mode")
            now = self.clock()
            for n in nodes:
                s = self.status.get(n["metadata"]["name"])
                if s is not None:
                    s["probe"] = s["transition"] = now
            for zone in self.zone_states:
                self._set_limiter(zone, len(zone_conditions.get(zone, ())), new_states[zone])
                self.zone_states[zone] = new_states[zone]
            return
        for zone, st in list(self.zone_states.items()):
            if st != new_states[zone]:
                log.info("zone %r is now in state %s", zone, new_states[zone])
                self._set_limiter(zone, len(zone_conditions[zone]), new_states[zone])
                self.zone_states[zone] = new_states[zone]

    def _set_limiter(self, zone, size, state):
        q = self._queue_for(zone)
        if state == NORMAL or state == FULL:
            q.swap_limiter(self.eviction_rate)
        elif state == PARTIAL:
            q.swap_limiter(self.secondary_rate if size > self.large_cluster else 0)

    # -- queue passes -------------------------------------------------------------------------
    async def _queue_pass(self):
        fn = self._taint_node if self.taint_mode else self._evict_node
        for q in list(self.zone_queues.values()):
            await q.try_(fn)

    async def _evict_node(self, name, uid):
        """`util.DeletePods`: every pod of the node but DaemonSet pods -> (done, retry)."""
        pods = [p for p in self.pod_inf.store.by_index("nodeName", name) if (p.get("spec") or {}).get("nodeName") == name]
        if pods:
            node = self.node_inf.get(name) or {"kind": "Node", "metadata": {"name": name, "uid": uid}}
            self.recorder.event(node, "Normal", "DeletingAllPods", f"Deleting all Pods from Node {name}.")
        for p in pods:
            md = p["metadata"]
            try:
                if (p.get("status") or {}).get("reason") != NODE_LOST:
                    await self.client.patch("pods", md["name"], {"status": {
                        "reason": NODE_LOST, "message": f"Node {name} which was running pod {md['name']} is unresponsive"}},
                        md["namespace"], "merge", "status")
                if md.get("deletionTimestamp"):
                    continue
                ref = controller_ref(p)
                if ref and ref.get("kind") == "DaemonSet":
                    continue
                self.recorder.event(p, "Normal", "NodeControllerEviction",
                                    f"Marking for deletion Pod {md['name']} from Node {name}")
                await self.client.delete("pods", md["name"], md["namespace"])
            except APIStatusError as e:
                if not is_not_found(e):
                    log.warning("unable to evict %s/%s: %s", md["namespace"], md["name"], e)
                    return False, 0.0
        return True, 0.0

    async def _taint_node(self, name, uid):
        node = self.node_inf.get(name)
        if node is None:
            return True, 0.0
        st = (core.get_condition(node.get("status"), "Ready") or {}).get("status")
        if st == "False":
            return await self._swap_taints(node, NOT_READY_TAINT, UNREACHABLE_TAINT), 0.0
        if st == "Unknown":
            return await self._swap_taints(node, UNREACHABLE_TAINT, NOT_READY_TAINT), 0.0
        return True, 0.0        # Ready again: nothing to taint

    def _cancel_eviction(self, node):
        return self._queue_for(zone_key(node)).remove(node["metadata"]["name"])

    # -- taint helpers --------------------------------------------------------------------------
    @staticmethod
    def _has_taint(node, key):
        return any(t.get("key") == key and t.get("effect") == "NoExecute" for t in (node.get("spec") or {}).get("taints") or ())

    async def _set_taints(self, node, taints):
        name = node["metadata"]["name"]
        try:
            await self.client.patch("nodes", name, {"spec": {"taints": taints or None}})
        except APIStatusError as e:
            if is_not_found(e):
                return False
            raise
        return True

    async def _swap_taints(self, node, add_key, del_key):
        """`SwapNodeControllerTaint`: add one NoExecute taint, drop its opposite."""
        fresh = self.node_inf.get(node["metadata"]["name"]) or node
        taints = [t for t in (fresh.get("spec") or {}).get("taints") or ()
                  if not (t.get("key") == del_key and t.get("effect") == "NoExecute")]
        if not any(t.get("key") == add_key and t.get("effect") == "NoExecute" for t in taints):
            taints.append({"key": add_key, "effect": "NoExecute", "timeAdded": now_rfc3339()})
        elif len(taints) == len((fresh.get("spec") or {}).get("taints") or ()):
            return True
        return await self._set_taints(fresh, taints)

    async def _mark_reachable(self, node):
        fresh = self.node_inf.get(node["metadata"]["name"]) or node
        old = (fresh.get("spec") or {}).get("taints") or []
        taints = [t for t in old if not (t.get("key") in (NOT_READY_TAINT, UNREACHABLE_TAINT) and t.get("effect") == "NoExecute")]
        if len(taints) != len(old):
            await self._set_taints(fresh, taints)
        return self._queue_for(zone_key(fresh)).remove(fresh["metadata"]["name"])

    async def _fix_deprecated_taints(self, node):
        taints = []
        for t in (node.get("spec") or {}).get("taints") or ():
            t = dict(t)
            t["key"] = DEPRECATED_TAINTS.get(t.get("key"), t.get("key"))
            taints.append(t)
        await self._set_taints(node, taints)
        return dict(node, spec=dict(node.get("spec") or {}, taints=taints))

    async def _condition_taints(self, node):
        want = {CONDITION_TAINTS[c["type"]] for c in (node.get("status") or {}).get("conditions") or ()
                if c.get("type") in CONDITION_TAINTS and c.get("status") == "True"}
        managed = set(CONDITION_TAINTS.values())
        old = (node.get("spec") or {}).get("taints") or []
        have = {t["key"] for t in old if t.get("key") in managed and t.get("effect") == "NoSchedule"}
        if want == have:
            return node
        taints = [t for t in old if not (t.get("key") in managed and t.get("effect") == "NoSchedule")]
        taints += [{"key": k, "effect": "NoSchedule"} for k in sorted(want)]
        await self._set_taints(node, taints)
        return dict(node, spec=dict(node.get("spec") or {}, taints=taints))

    async def _mark_pods_not_ready(self, name):
        """`util.MarkAllPodsNotReady`."""
        for p in self.pod_inf.store.by_index("nodeName", name):
            cond = core.get_condition(p.get("status"), "Ready")
            if cond is None or cond.get("status") == "False":
                continue
            conds = [dict(c, status="False", lastTransitionTime=now_rfc3339()) if c.get("type") == "Ready" else c
                     for c in (p.get("status") or {}).get("conditions") or ()]
            try:
                await self.client.patch("pods", p["metadata"]["name"], {"status": {"conditions": conds}},
                                        p["metadata"]["namespace"], "merge", "status")
            except APIStatusError as e:
                if not is_not_found(e):
                    log.warning("unable to mark pod %s not ready: %s", p["metadata"]["name"], e)

    # -- NoExecute taint manager -----------------------------------------------------------------
    def _node_updated(self, old, new):
        if (old.get("spec") or {}).get("taints") != (new.get("spec") or {}).get("taints"):
            self.enqueue("node/" + new["metadata"]["name"])

    def _pod_event(self, pod):
        if (pod.get("spec") or {}).get("nodeName"):
            self.enqueue(f"pod/{pod['metadata']['namespace']}/{pod['metadata']['name']}")

    def _pod_updated(self, old, new):
        if (old.get("spec") or {}).get("nodeName") != (new.get("spec") or {}).get("nodeName") or \
                (old.get("spec") or {}).get("tolerations") != (new.get("spec") or {}).get("tolerations"):
            self._pod_event(new)

    def _pod_deleted(self, pod):
        self._cancel(f"{pod['metadata']['namespace']}/{pod['metadata']['name']}", event=False)

    async def sync(self, key):
        kind, _, rest = key.partition("/")
        if kind == "node":
            node = self.node_inf.get(rest)
            taints = [t for t in ((node or {}).get("spec") or {}).get("taints") or () if t.get("effect") == "NoExecute"]
            if taints:
                self.tainted[rest] = taints
            else:
                self.tainted.pop(rest, None)
            for p in self.pod_inf.store.by_index("nodeName", rest):
                self._process_pod(p, taints)
        elif kind == "pod":
            ns, _, name = rest.partition("/")
            pod = self.pod_inf.store.get(f"{ns}/{name}")
            if pod is None:
                self._cancel(rest, event=False)
                return
            node = (pod.get("spec") or {}).get("nodeName")
            if node and node in self.tainted:
                self._process_pod(pod, self.tainted[node])

    def _process_pod(self, pod, taints):
        key = f"{pod['metadata']['namespace']}/{pod['metadata']['name']}"
        if not taints:
            self._cancel(key)
            return
        if pod["metadata"].get("deletionTimestamp") or core.pod_is_terminal(pod):
            return
        ok, used = matching_tolerations(taints, (pod.get("spec") or {}).get("tolerations") or ())
        now = self.clock()
        if not ok:
            self._cancel(key, event=False)
            self._schedule(key, now, now)
            return
        wait = min_toleration_time(used)
        if wait is None:
            return          # tolerated forever: an already scheduled deletion is kept
        if key in self.scheduled:
            return          # an earlier scheduled deletion stands (processPodOnNode keeps it)
        self._schedule(key, now, now + wait)

    def _schedule(self, key, created, trigger):
        loop = asyncio.get_event_loop()
        h = loop.call_later(max(0.0, trigger - self.clock()), lambda: asyncio.ensure_future(self._taint_evict(key)))
        self.scheduled[key] = (created, trigger, h)

    def _cancel(self, key, event=True):
        cur = self.scheduled.pop(key, None)
        if cur is not None:
            cur[2].cancel()
            if event:
                ns, _, name = key.partition("/")
                self.recorder.event({"kind": "Pod", "metadata": {"name": name, "namespace": ns}}, "Normal",
                                    "TaintManagerEviction", f"Cancelling deletion of Pod {key}")

    async def _taint_evict(self, key):
        self.scheduled.pop(key, None)
        ns, _, name = key.partition("/")
        self.recorder.event({"kind": "Pod", "metadata": {"name": name, "namespace": ns}}, "Normal",
                            "TaintManagerEviction", f"Marking for deletion Pod {key}")
        try:
            await self.client.delete("pods", name, ns)
        except APIStatusError as e:
            if not is_not_found(e):
                log.warning("taint manager: unable to delete %s: %s", key, e)
