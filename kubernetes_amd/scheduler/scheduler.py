"""kube-scheduler equivalent: informers → queue → scheduleOne → assume → async bind.

Parity: `plugin/pkg/scheduler/scheduler.go:170-497` (`Run`, `scheduleOne`, `schedule`, `assume`,
`bind` in a goroutine), the factory's informer wiring and cache handlers
(`plugin/pkg/scheduler/factory/factory.go:554-829`, scheduled-pod field selector
`spec.nodeName!=,status.phase!=Succeeded,status.phase!=Failed`), the binder with the fork's
`Target.ExtendedResources` (`scheduler.go:481-492`, `factory.go:1241-1244`), events
`Scheduled` / `FailedScheduling` and the metrics of `plugin/pkg/scheduler/metrics/metrics.go:33-50`.

Scale-out (MI355X clusters with many nodes): `shard_count > 1` runs several scheduler
processes in parallel over a PARTITION of the cluster, so no shard processes every pod event:
  * nodes: shard i owns every node whose index in the sorted node-name list is i mod n, and
    keeps pod accounting only for those, fed by one `spec.nodeName=<node>` watch per owned
    node (served by the store's node-indexed fan-out);
  * pods: shard i lists/watches only the unassigned pods selected by `?kamdShard=i/n`
    ((crc32(namespace/name) + offset label) mod n, api/sharding.py), evaluated server side;
  * a pod that fits none of the shard's nodes is handed to the next shard by bumping its
    `scheduler.kamd.io/shard-offset` label (`scheduler.kamd.io/shard-hops` counts the hops);
    after a full round it is reported unschedulable (and preemption is tried) on the last shard,
    and it is offered to the next shard again after `rehandoff_period` seconds, doubling per round
    up to 10 s (the capacity it needs may have freed on another shard's nodes).
Per-shard work is O(cluster pods / n). Trade-off: inter-pod (anti-)affinity is evaluated
against the pods on the shard's own nodes. GPU double assignment stays impossible: the API
server's device-claim guard rejects a conflicting bind (409) and the shard retries.

Fix: `assume()` writes the device binding into the assumed pod's
`spec.extendedResources[].assigned` before `AssumePod`, so the cache reserves those devices
immediately and the next pod in the same burst cannot receive them.
"""
from __future__ import annotations

import asyncio
import logging
import time
import zlib

from ..api import core
from ..api.meta import ns_name, now_rfc3339
from ..api.sharding import QUERY_PARAM, SHARD_OFFSET_LABEL, offset_of
from ..client.events import EventRecorder
from ..client.informer import Informer
from ..client.rest import APIStatusError, is_not_found
from ..utils.httpserver import HTTPServer, Response
from ..utils.metrics import MICRO_BUCKETS, Registry
from ..utils.trace import Trace
from .cache import PodInfo, SchedulerCache
from .extender import ExtenderError
from .generic import FitError, GenericScheduler
from .queue import SchedulingQueue
from .volumes import SELECTED_NODE_ANN, plan_bindings
from ..utils.tasks import spawn

log = logging.getLogger("scheduler")

DEFAULT_SCHEDULER = "default-scheduler"
SHARD_HOPS_ANNOTATION = "scheduler.kamd.io/shard-hops"


class Scheduler:
    def __init__(self, client, scheduler_name=DEFAULT_SCHEDULER, predicates=None, priorities=None,
                 percentage_of_nodes_to_score=100, emit_events=True, extenders=None, max_binds_in_flight=256,
                 update_unschedulable_status=True, shard_index=0, shard_count=1, preemption=True,
                 rehandoff_period=0.2, hard_pod_affinity_symmetric_weight=1, failure_domains=None):
        self.client = client
        self.name = scheduler_name
        self.profiling = True         # --profiling: /debug/pprof on the metrics port
        self.cache = SchedulerCache()
        self.cache.hard_pod_affinity_weight = hard_pod_affinity_symmetric_weight
        if failure_domains:
            self.cache.failure_domains = tuple(failure_domains)
        self.queue = SchedulingQueue()
        self.algo = GenericScheduler(self.cache, predicates, priorities, percentage_of_nodes_to_score, extenders)
        # factory.go:886 getBinder: the first extender with a bindVerb writes bindings
        self.binder = next((e for e in extenders or () if getattr(e, "is_binder", lambda: False)()), None)
        self.algo.queue = self.queue
        self.shard_index, self.shard_count = shard_index, shard_count
        self.partitioned = shard_count > 1
        self.rehandoff_period = rehandoff_period
        self.all_nodes: dict[str, dict] = {}          # partitioned: every node object
        self.owned: dict[str, Informer] = {}          # partitioned: owned node -> its pod informer
        self._owned_ready: set = set()
        self._rehandoff_delay: dict = {}             # pod key -> current re-offer delay (doubling)
        self.handoffs = 0
        self.conflicts = 0
        self.recorder = EventRecorder(client, scheduler_name, enabled=emit_events)
        self.update_unschedulable_status = update_unschedulable_status
        self.metrics = Registry()
        self.m_e2e = self.metrics.histogram("scheduler_e2e_scheduling_latency_microseconds",
                                            "E2e scheduling latency (scheduling algorithm + binding)", (), MICRO_BUCKETS)
        self.m_algo = self.metrics.histogram("scheduler_scheduling_algorithm_latency_microseconds",
                                             "Scheduling algorithm latency", (), MICRO_BUCKETS)
        self.m_bind = self.metrics.histogram("scheduler_binding_latency_microseconds", "Binding latency", (), MICRO_BUCKETS)
        self.m_attempts = self.metrics.counter("scheduler_schedule_attempts_total", "Scheduling attempts", ("result",))
        self.m_pending = self.metrics.gauge("scheduler_pending_pods", "Pods in the scheduling queue", ("queue",))
        self.m_preemptions = self.metrics.counter("scheduler_total_preemption_attempts", "Preemptions that evicted victims")
        self.preemption = preemption
        self.scheduled = 0
        self.bind_sem = asyncio.Semaphore(max_binds_in_flight)
        self._tasks = []
        self._binds = set()
        self.http = None
        if self.partitioned:
            # only this shard's unassigned pods; assigned pods come from the per-node informers
            self.pod_informer = Informer(client, "pods",
                                         field_selector="spec.nodeName=,status.phase!=Succeeded,status.phase!=Failed",
                                         extra_query={QUERY_PARAM: f"{shard_index}/{shard_count}"})
        else:
            self.pod_informer = Informer(client, "pods", field_selector="status.phase!=Succeeded,status.phase!=Failed")
        self.node_informer = Informer(client, "nodes")
        self.pvc_informer = Informer(client, "persistentvolumeclaims")
        self.pv_informer = Informer(client, "persistentvolumes")
        self.sc_informer = Informer(client, "storageclasses")
        # services: SelectorSpread / ServiceSpreading / ServiceAffinity / ServiceAntiAffinity
        self.svc_informer = Informer(client, "services")
        # preemption: PDB-aware victim selection (the reference scheduler cache's ListPDBs)
        self.pdbs: dict[str, dict] = {}
        self.pdb_informer = Informer(client, "poddisruptionbudgets") if preemption else None

    # -- informer handlers -------------------------------------------------
    def _responsible(self, pod):
        # partitioned shards get only their pods from the server (kamdShard selection)
        return (pod.get("spec") or {}).get("schedulerName", DEFAULT_SCHEDULER) == self.name

    # -- partitioned shards: unassigned pods + owned nodes --------------------------
    def _on_unassigned_add(self, pod):
        if not (pod.get("spec") or {}).get("nodeName") and self._responsible(pod) \
                and not pod["metadata"].get("deletionTimestamp"):
            self.queue.add(pod)

    def _on_unassigned_update(self, old, new):
        if not self._responsible(new):
            return
        if new["metadata"].get("deletionTimestamp") or (new.get("spec") or {}).get("nodeName"):
            self.queue.delete(new)
        else:
            self.queue.update(old, new)

    def _on_unassigned_delete(self, pod):
        # bound (now on some node's informer), deleted, or handed to another shard
        self.queue.delete(pod)
        if (pod.get("spec") or {}).get("nodeName") or pod["metadata"].get("deletionTimestamp"):
            self._rehandoff_delay.pop(ns_name(pod), None)

    def _on_owned_pod_add(self, pod):
        self.cache.add_pod(pod)
        self.queue.assigned_pod_added(pod)

    def _on_owned_pod_delete(self, pod):
        self.cache.remove_pod(pod)
        self.queue.move_all_to_active()   # capacity was freed

    def _owns(self, names):
        return {n for i, n in enumerate(sorted(names)) if i % self.shard_count == self.shard_index}

    def _rebalance(self):
        want = self._owns(self.all_nodes)
        for name in [n for n in self.owned if n not in want]:
            self.owned.pop(name).stop()
            self._owned_ready.discard(name)
            self.cache.drop_node(name)
        for name in want:
            if name in self.owned:
                continue
            inf = Informer(self.client, "pods", field_selector=f"spec.nodeName={name},status.phase!=Succeeded,"
                                                               "status.phase!=Failed")
            inf.add_handler(self._on_owned_pod_add, lambda old, new: self._on_owned_pod_add(new), self._on_owned_pod_delete)
            self.owned[name] = inf
            inf.start()
            spawn(self._node_ready(name, inf))

    async def _node_ready(self, name, inf):
        """A node becomes schedulable for this shard once its pods are known."""
        while not inf.has_synced():
            if self.owned.get(name) is not inf:
                return
            await asyncio.sleep(0.01)
        if self.owned.get(name) is inf and name in self.all_nodes:
            self._owned_ready.add(name)
            self.cache.add_node(self.all_nodes[name])
            self.queue.move_all_to_active()

    def _on_part_node_add(self, node):
        name = node["metadata"]["name"]
        known = name in self.all_nodes
        self.all_nodes[name] = node
        if not known:
            self._rebalance()
        elif name in self._owned_ready:
            self.cache.add_node(node)

    def _on_part_node_update(self, old, new):
        name = new["metadata"]["name"]
        self.all_nodes[name] = new
        if name in self._owned_ready:
            self.cache.add_node(new)
            if _node_capacity_changed(old, new):
                self.queue.move_all_to_active()

    def _on_part_node_delete(self, node):
        if self.all_nodes.pop(node["metadata"]["name"], None) is not None:
            self._rebalance()

    def _handoff(self, pod, msg):
        """Pass a pod this shard cannot place to the next shard; False once it has been
        through every shard (then it is unschedulable here)."""
        md = pod["metadata"]
        hops = int((md.get("annotations") or {}).get(SHARD_HOPS_ANNOTATION, "0") or 0)
        if hops >= self.shard_count - 1:
            return False
        self.queue.delete(pod)
        self.handoffs += 1
        spawn(self._patch_shard(pod, offset_of(md.get("labels")) + 1, hops + 1))
        return True

    async def _patch_shard(self, pod, offset, hops):
        md = pod["metadata"]
        try:
            await self.client.patch("pods", md["name"], {"metadata": {
                "labels": {SHARD_OFFSET_LABEL: str(offset)},
                "annotations": {SHARD_HOPS_ANNOTATION: str(hops)}}}, md.get("namespace"))
        except APIStatusError as e:
            if not is_not_found(e):
                log.warning("handing %s to the next shard failed: %s", ns_name(pod), e)
                self.queue.add_backoff(pod)

    async def _rehandoff_loop(self):
        """Unschedulable pods are offered to the next shard again (its capacity may have freed)."""
        tick = max(0.02, self.rehandoff_period / 4)
        while True:
            await asyncio.sleep(tick)
            now = time.monotonic()
            for pod, since in list(self.queue.unschedulable_since()):
                key = ns_name(pod)
                delay = self._rehandoff_delay.get(key, self.rehandoff_period)
                if now - since < delay:
                    continue
                self._rehandoff_delay[key] = min(delay * 2, 10.0)
                if len(self._rehandoff_delay) > 100_000:
                    self._rehandoff_delay.clear()
                self.queue.delete(pod)
                self.handoffs += 1
                spawn(self._patch_shard(pod, offset_of(pod["metadata"].get("labels")) + 1, 0))

    def _on_pod_add(self, pod):
        if (pod.get("spec") or {}).get("nodeName"):
            self.cache.add_pod(pod)
            self.queue.assigned_pod_added(pod)
            return
        if self._responsible(pod) and not pod["metadata"].get("deletionTimestamp"):
            self.queue.add(pod)

    def _on_pod_update(self, old, new):
        assigned_new = bool((new.get("spec") or {}).get("nodeName"))
        if assigned_new:
            if not (old.get("spec") or {}).get("nodeName"):
                self.queue.delete(old)
            self.cache.add_pod(new)
            self.queue.assigned_pod_added(new)
            return
        if self._responsible(new):
            if new["metadata"].get("deletionTimestamp"):
                self.queue.delete(new)
            else:
                self.queue.update(old, new)

    def _on_pod_delete(self, pod):
        if (pod.get("spec") or {}).get("nodeName") or self.cache.get_pod(ns_name(pod)) is not None:
            self.cache.remove_pod(pod)
            self.queue.move_all_to_active()   # capacity was freed
        else:
            self.queue.delete(pod)

    def _on_node_add(self, node):
        self.cache.add_node(node)
        self.queue.move_all_to_active()

    def _on_node_update(self, old, new):
        self.cache.add_node(new)
        if _node_capacity_changed(old, new):
            self.queue.move_all_to_active()

    def _on_node_delete(self, node):
        self.cache.remove_node(node)

    def _volume_handlers(self):
        vl = self.cache.volumes

        def key(o):
            md = o["metadata"]
            return f"{md['namespace']}/{md['name']}" if md.get("namespace") else md["name"]

        def put(d, moved=True):
            def h(*objs):
                o = objs[-1]
                d[key(o)] = o
                if d is vl.pvs and ((o.get("spec") or {}).get("claimRef")):
                    vl.assumed_pvs.pop(key(o), None)
                if moved:
                    self.queue.move_all_to_active()
            return h

        def drop(d):
            def h(o):
                d.pop(key(o), None)
                vl.assumed_pvs.pop(key(o), None)
            return h
        self.pvc_informer.add_handler(put(vl.pvcs), put(vl.pvcs), drop(vl.pvcs))
        self.pv_informer.add_handler(put(vl.pvs), put(vl.pvs), drop(vl.pvs))
        self.sc_informer.add_handler(put(vl.classes), put(vl.classes), drop(vl.classes))
        self.svc_informer.add_handler(self.cache.set_service, lambda old, new: self.cache.set_service(new),
                                      self.cache.remove_service)
        if self.pdb_informer is not None:
            self.pdb_informer.add_handler(put(self.pdbs, False), put(self.pdbs, False), drop(self.pdbs))

    def _aux_informers(self):
        out = [self.pvc_informer, self.pv_informer, self.sc_informer, self.svc_informer]
        if self.pdb_informer is not None:
            out.append(self.pdb_informer)
        return out

    # -- scheduling loop ---------------------------------------------------------
    async def run(self, metrics_port=None, metrics_address="127.0.0.1"):
        self.recorder.start()
        if self.partitioned:
            self.node_informer.add_handler(self._on_part_node_add, self._on_part_node_update, self._on_part_node_delete)
            self.pod_informer.add_handler(self._on_unassigned_add, self._on_unassigned_update,
                                          self._on_unassigned_delete)
            self._tasks.append(asyncio.ensure_future(self._rehandoff_loop()))
        else:
            self.node_informer.add_handler(self._on_node_add, self._on_node_update, self._on_node_delete)
            self.pod_informer.add_handler(self._on_pod_add, self._on_pod_update, self._on_pod_delete)
        self._volume_handlers()
        for inf in self._aux_informers():
            inf.start()
        self.node_informer.start()
        await self.node_informer.wait_synced(60)
        if self.partitioned:
            t = time.monotonic()
            while len(self._owned_ready) < len(self.owned) and time.monotonic() - t < 60:
                await asyncio.sleep(0.01)
        for inf in self._aux_informers():
            await inf.wait_synced(60)
        self.pod_informer.start()
        await self.pod_informer.wait_synced(60)
        if metrics_port is not None:
            self.http = HTTPServer(self._http)
            try:
                await self.http.start(metrics_address, metrics_port)
            except OSError as e:     # another scheduler on this host holds the port: not fatal
                log.warning("healthz/metrics endpoint %s:%s not started: %s", metrics_address, metrics_port, e)
                self.http = None
        self._tasks.append(asyncio.ensure_future(self._housekeeping()))
        while True:
            ent = await self.queue.pop()
            if ent is None:
                return
            self.schedule_one(*ent[:2])
            # yield so informer deliveries and bind completions interleave with the loop
            await asyncio.sleep(0)

    async def _housekeeping(self):
        while True:
            await asyncio.sleep(1.0)
            self.cache.cleanup_expired()
            self.queue.flush_unschedulable_leftover()
            self.m_pending.labels("active").set(len(self.queue.active))
            self.m_pending.labels("unschedulable").set(len(self.queue.unschedulable))

    def schedule_one(self, pod, pi):
        if pi is None:
            pi = PodInfo(pod)
        tr = Trace(f"Scheduling {ns_name(pod)}")
        t0 = tr.start
        try:
            host, erb = self.algo.schedule(pod, pi)
            tr.step(f"Computing predicates, device allocation and priorities -> {host}")
            tr.log_if_long(0.1, log)
        except FitError as e:
            if self.partitioned and self._handoff(pod, str(e)):
                return None
            self.m_attempts.labels("unschedulable").inc()
            self.recorder.event(pod, "Warning", "FailedScheduling", str(e))
            self.queue.add_unschedulable(pod)
            if self.update_unschedulable_status:
                spawn(self._set_unschedulable(pod, str(e)))
            if self.preemption:
                self._try_preempt(pod, pi, e)
            return None
        except Exception as e:  # pragma: no cover - defensive
            log.exception("scheduling %s failed", ns_name(pod))
            self.m_attempts.labels("error").inc()
            self.queue.add_backoff(pod)
            self.recorder.event(pod, "Warning", "FailedScheduling", str(e))
            return None
        self.m_algo.observe((time.perf_counter() - t0) * 1e6)
        # the assumed copy shares everything but spec (nodeName) and the per-resource entries
        # that get device IDs: the cache never mutates a pod it holds
        assumed = dict(pod)
        spec = assumed["spec"] = dict(pod["spec"])
        spec["nodeName"] = host
        ers = spec.get("extendedResources")
        if ers:
            spec["extendedResources"] = [dict(per, assigned=list(erb[per.get("name")]["resources"]))
                                         if per.get("name") in erb else per for per in ers]
        try:
            self.cache.assume_pod(assumed, pi)
        except ValueError as e:
            log.warning("assume failed: %s", e)
            return None
        vplan = None
        if pi is not None and pi.volumes.claims:
            # volumebinder AssumePodVolumes: reserve the chosen PVs in the cache now
            vplan = plan_bindings(self.cache.volumes, pod, self.cache.nodes[host].labels, host)
            for kind, pvc, pv in vplan:
                if kind == "bind":
                    self.cache.volumes.assumed_pvs[pv["metadata"]["name"]] = pvc
        t = asyncio.ensure_future(self._bind(pod, assumed, host, erb, t0, vplan))
        self._binds.add(t)
        t.add_done_callback(self._binds.discard)
        return host

    async def _bind_volumes(self, plan, host):
        """volumebinder BindPodVolumes: pre-bind PVs (claimRef) / mark claims for provisioning."""
        for kind, pvc, pv in plan:
            md = pvc["metadata"]
            if kind == "bind":
                ref = {"kind": "PersistentVolumeClaim", "apiVersion": "v1", "namespace": md["namespace"],
                       "name": md["name"], "uid": md.get("uid")}
                await self.client.patch("persistentvolumes", pv["metadata"]["name"], {"spec": {"claimRef": ref}})
            else:
                await self.client.patch("persistentvolumeclaims", md["name"],
                                        {"metadata": {"annotations": {SELECTED_NODE_ANN: host}}}, md["namespace"])

    async def _bind(self, pod, assumed, host, erb, t0, vplan=None):
        md = pod["metadata"]
        async with self.bind_sem:
            tb = time.perf_counter()
            try:
                if vplan:
                    await self._bind_volumes(vplan, host)
                if self.binder is not None:
                    await asyncio.get_running_loop().run_in_executor(
                        None, self.binder.bind, md.get("namespace", "default"), md["name"], md.get("uid"), host,
                        erb or None)
                else:
                    await self.client.bind(md.get("namespace", "default"), md["name"], host, erb or None, decode=False)
            except (APIStatusError, ExtenderError, ConnectionError, OSError, asyncio.TimeoutError) as e:
                self.cache.forget_pod(assumed)
                for kind, _pvc, pv in vplan or ():
                    if kind == "bind":
                        self.cache.volumes.assumed_pvs.pop(pv["metadata"]["name"], None)
                self.m_attempts.labels("error").inc()
                if isinstance(e, APIStatusError) and e.code == 409 and "already assigned" in str(e):
                    # lost a device race to another scheduler shard: retry soon, no event spam
                    self.conflicts += 1
                    self.queue.add_backoff(pod, conflict=True)
                    return
                self.recorder.event(pod, "Warning", "FailedScheduling", f"Binding rejected: {e}")
                if not (isinstance(e, APIStatusError) and is_not_found(e)):
                    self.queue.add_backoff(pod)
                return
            self.cache.finish_binding(assumed)
        now = time.perf_counter()
        self.m_bind.observe((now - tb) * 1e6)
        self.m_e2e.observe((now - t0) * 1e6)
        self.m_attempts.labels("scheduled").inc()
        self.scheduled += 1
        self.queue.backoff.forget(ns_name(pod))
        self.queue.conflict_backoff.forget(ns_name(pod))
        self.recorder.event(pod, "Normal", "Scheduled", f"Successfully assigned {md['name']} to {host}")

    def _try_preempt(self, pod, pi, fit_error=None):
        """scheduler.go preempt() (:209-253): pick a node and the minimal lower-priority victims
        (`preemption.preempt`), then — in order — write the `NominatedNodeName` annotation on
        the preemptor, delete the victims, and clear the nominations of lower-priority pods
        nominated to that node. The preemptor is retried when the victims' deletions free their
        resources (pod delete events re-activate the queue); meanwhile the queue's nominated
        index holds the freed devices for it."""
        from .preemption import preempt
        try:
            node, victims, clear = preempt(self.algo, pod, pi, fit_error, list(self.pdbs.values()), self.queue)
        except Exception:  # pragma: no cover - defensive
            log.exception("preemption for %s failed", ns_name(pod))
            return
        if node is not None:
            if victims:
                self.m_preemptions.inc()
            # index the nomination now; the informer's copy of the annotated pod replaces it
            self.queue.nominate(pod, node)
        if node is not None or clear:
            spawn(self._preempt_writes(pod, node, victims, clear))

    async def _preempt_writes(self, pod, node, victims, clear):
        md = pod["metadata"]
        if node is not None:
            if not await self._set_nomination(pod, node):
                self.queue.nominate(pod, "")
                return
            for v in victims:
                vmd = v["metadata"]
                if not await self._delete_victim(vmd.get("namespace"), vmd["name"]):
                    return
                self.recorder.event(v, "Normal", "Preempted", f"by {md.get('namespace')}/{md['name']} on node {node}")
        for p in clear:
            # a failure here is not critical (scheduler.go:245-251)
            self.queue.nominate(p, "")
            await self._set_nomination(p, "")

    async def _set_nomination(self, pod, node):
        """podPreemptor.UpdatePodAnnotations / RemoveNominatedNodeAnnotation
        (factory.go:1271-1300): a merge patch of the annotation through pods/status; "" clears."""
        from .preemption import NOMINATED_ANNOTATION
        md = pod["metadata"]
        try:
            await self.client.patch("pods", md["name"], {"metadata": {"annotations": {NOMINATED_ANNOTATION: node}}},
                                    md.get("namespace"), "merge", "status")
            return True
        except APIStatusError as e:
            if not is_not_found(e):
                log.warning("could not %s nominated node of %s/%s: %s", "set" if node else "clear",
                            md.get("namespace"), md["name"], e)
        except Exception as e:  # noqa: BLE001 - connection errors: the pod is retried anyway
            log.warning("could not update nominated node of %s/%s: %s", md.get("namespace"), md["name"], e)
        return False

    async def _delete_victim(self, ns, name):
        try:
            await self.client.delete("pods", name, ns)
        except APIStatusError as e:
            if not is_not_found(e):
                log.warning("deleting preemption victim %s/%s: %s", ns, name, e)
                return False
        except Exception as e:  # noqa: BLE001
            log.warning("deleting preemption victim %s/%s: %s", ns, name, e)
            return False
        return True

    async def _set_unschedulable(self, pod, msg):
        md = pod["metadata"]
        cond = {"type": core.COND_POD_SCHEDULED, "status": "False", "reason": "Unschedulable", "message": msg,
                "lastProbeTime": None, "lastTransitionTime": now_rfc3339()}
        old = core.get_condition(pod.get("status"), core.COND_POD_SCHEDULED)
        if old and old.get("status") == "False" and old.get("message") == msg:
            return
        try:
            await self.client.patch("pods", md["name"], {"status": {"conditions": [cond]}}, md.get("namespace"),
                                    "strategic", "status")
        except Exception as e:
            log.debug("could not update pod condition: %s", e)

    async def _http(self, req):
        if req.path == "/metrics":
            return Response(200, self.metrics.render(), "text/plain; version=0.0.4")
        if req.path == "/healthz":
            return Response(200, b"ok", "text/plain")
        if req.path.startswith("/debug/pprof") and self.profiling:
            from ..utils.profiling import handle_debug
            return await handle_debug(req)
        return Response(404, b"not found", "text/plain")

    async def stop(self):
        self.queue.close()
        for t in self._tasks:
            t.cancel()
        self.pod_informer.stop()
        self.node_informer.stop()
        for inf in self.owned.values():
            inf.stop()
        for inf in self._aux_informers():
            inf.stop()
        self.recorder.stop()
        if self.http:
            await self.http.stop()

    async def wait_binds(self):
        while self._binds:
            await asyncio.gather(*list(self._binds), return_exceptions=True)


def shard_of(key: str, count: int) -> int:
    return zlib.crc32(key.encode()) % count


def _node_capacity_changed(old, new):
    os_, ns = old.get("status") or {}, new.get("status") or {}
    return (os_.get("allocatable") != ns.get("allocatable") or os_.get("extendedResources") != ns.get("extendedResources")
            or (old.get("spec") or {}) != (new.get("spec") or {})
            or old["metadata"].get("labels") != new["metadata"].get("labels")
            or [c.get("status") for c in os_.get("conditions") or ()] != [c.get("status") for c in ns.get("conditions") or ()])
