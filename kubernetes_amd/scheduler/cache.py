"""Scheduler cache: NodeInfo aggregation, the fork's per-device ER manager, assumed pods.

Parity:
  * `plugin/pkg/scheduler/schedulercache/cache.go:40-462` — AssumePod / FinishBinding /
    ForgetPod / AddPod / UpdatePod / RemovePod, assumed-pod TTL expiry, node add/update/remove.
  * `plugin/pkg/scheduler/schedulercache/node_info.go` — requested / non-zero requested /
    allocatable, host ports, taints, conditions, generation.
  * `plugin/pkg/scheduler/schedulercache/extended_resources.go:25-210` (fork F5) — per node
    allocatable / available / used device maps; SetNode reconciles from
    `Node.status.extendedResources`; AddPod / RemovePod move `Assigned` IDs.

Fixes: assumed pods carry their device assignment (item 1) so back-to-back
bin-packing can never double-assign; the reference deep-copied `Available()` per node per
pod — here allocation works on the live map with a scratch "taken" set (item 9);
RemoveNode actually drops state (quirk Q8).
"""
from __future__ import annotations

import time

from ..api import core
from ..api.meta import ns_name
from ..api.quantity import Quantity, parse_quantity
from .volumes import VolumeLister, VolumeInfo

DEFAULT_MILLI_CPU = 100                 # priorities/util/non_zero.go
DEFAULT_MEMORY = 200 * 1024 * 1024


def _q(v) -> Quantity:
    return parse_quantity(v) if isinstance(v, str) else Quantity(v)


class PodInfo:
    """Parsed, cached resource view of a pod (computed once per pod version)."""
    __slots__ = ("milli_cpu", "memory", "ephemeral", "scalars", "nz_cpu", "nz_mem", "ports", "er", "assigned", "volumes",
                 "limits")

    def __init__(self, pod):
        req = core.pod_requests(pod)
        self.milli_cpu = req["cpu"].milli_value() if "cpu" in req else 0
        self.memory = req["memory"].int_value() if "memory" in req else 0
        self.ephemeral = req["ephemeral-storage"].int_value() if "ephemeral-storage" in req else 0
        # `calculateResource`: scalar resources are extended (domain-qualified) names and
        # hugepages; any other key a container names is not accounted
        self.scalars = {k: v.int_value() for k, v in req.items()
                        if k not in ("cpu", "memory", "ephemeral-storage", "pods")
                        and (core.is_extended_resource_name(k) or k.startswith("hugepages-"))}
        spec = pod.get("spec") or {}
        # `priorities/util/non_zero.go` GetNonzeroRequests: per container, a request that is not
        # set counts as 100m / 200Mi (an explicit zero stays zero); init containers do not count
        nzc = nzm = 0
        for c in spec.get("containers") or ():
            r = (c.get("resources") or {}).get("requests") or {}
            nzc += _q(r["cpu"]).milli_value() if "cpu" in r else DEFAULT_MILLI_CPU
            nzm += _q(r["memory"]).int_value() if "memory" in r else DEFAULT_MEMORY
        self.nz_cpu, self.nz_mem = nzc, nzm
        ports = []
        for c in spec.get("containers") or ():
            for p in c.get("ports") or ():
                if p.get("hostPort"):
                    ports.append((p.get("hostIP", "0.0.0.0"), p.get("protocol", "TCP"), p["hostPort"]))
        self.ports = ports
        er = []
        for per in spec.get("extendedResources") or ():
            try:
                rn = core.pod_extended_resource_name(per)
                n = core.pod_extended_resource_count(per)
            except (ValueError, KeyError):
                continue
            er.append((per.get("name"), rn, n, (per.get("affinity") or {}).get("required") or []))
        self.er = er
        self.assigned = core.pod_assigned_devices(pod)
        self.volumes = VolumeInfo(pod)
        lim_cpu = lim_mem = 0
        for c in spec.get("containers") or ():
            lim = (c.get("resources") or {}).get("limits") or {}
            if "cpu" in lim:
                lim_cpu += _q(lim["cpu"]).milli_value()
            if "memory" in lim:
                lim_mem += _q(lim["memory"]).int_value()
        self.limits = (lim_cpu, lim_mem)

    def with_assigned(self, pod):
        """This pod's info for its assumed copy: everything parsed stays, only the devices the
        scheduler just assigned change (no second parse per scheduled pod)."""
        out = object.__new__(PodInfo)
        for s in PodInfo.__slots__:
            setattr(out, s, getattr(self, s))
        out.assigned = core.pod_assigned_devices(pod)
        return out


def _hive(dev):
    return (dev.get("attributes") or {}).get(core.ATTR_HIVE, "")


def _healthy(dev):
    return dev.get("health", core.HEALTHY) == core.HEALTHY


class ERManager:
    """Per-node device accounting. Besides the reference's allocatable/available/used maps it
    keeps, per resource, the healthy free devices grouped by xGMI hive (`hive_free`) and their
    count (`nfree`), maintained incrementally so the scheduler's filter is O(hives), not
    O(devices), per node."""

    __slots__ = ("allocatable", "available", "used", "hive_free", "nfree")

    def __init__(self):
        self.allocatable: dict[str, dict[str, dict]] = {}
        self.available: dict[str, dict[str, dict]] = {}
        self.used: dict[str, dict[str, str]] = {}              # rname -> {device id: pod key}
        self.hive_free: dict[str, dict[str, dict]] = {}        # rname -> {hive: {id: dev}} (healthy, free)
        self.nfree: dict[str, int] = {}

    def clone(self):
        c = ERManager()
        c.allocatable = {k: dict(v) for k, v in self.allocatable.items()}
        c.available = {k: dict(v) for k, v in self.available.items()}
        c.used = {k: dict(v) for k, v in self.used.items()}
        c.hive_free = {k: {h: dict(d) for h, d in v.items()} for k, v in self.hive_free.items()}
        c.nfree = dict(self.nfree)
        return c

    def _take(self, rn, i):
        avail = self.available.get(rn)
        if avail is None:
            return
        dev = avail.pop(i, None)
        if dev is not None and _healthy(dev):
            hf = self.hive_free[rn].get(_hive(dev))
            if hf is not None and hf.pop(i, None) is not None:
                self.nfree[rn] -= 1

    def _give(self, rn, i):
        dev = self.allocatable.get(rn, {}).get(i)
        if dev is None:
            return
        self.available.setdefault(rn, {})[i] = dev
        if _healthy(dev):
            self.hive_free.setdefault(rn, {}).setdefault(_hive(dev), {})[i] = dev
            self.nfree[rn] = self.nfree.get(rn, 0) + 1

    def add_pod(self, key, assigned: dict):
        for rn, ids in assigned.items():
            used = self.used.setdefault(rn, {})
            for i in ids:
                used[i] = key
                self._take(rn, i)

    def remove_pod(self, key, assigned: dict):
        for rn, ids in assigned.items():
            used = self.used.get(rn)
            if not used:
                continue
            for i in ids:
                if used.get(i) == key:
                    del used[i]
                    self._give(rn, i)
            if not used:
                del self.used[rn]

    def set_node(self, node):
        ers = ((node.get("status") or {}).get("extendedResources")) or {}
        self.allocatable = {rn: dict((dom or {}).get("resources") or {}) for rn, dom in ers.items()}
        self.available = {}
        self.hive_free = {}
        self.nfree = {}
        for rn, devs in self.allocatable.items():
            used = self.used.get(rn, {})
            av = self.available[rn] = {}
            hf = self.hive_free[rn] = {}
            n = 0
            for i, d in devs.items():
                if i in used:
                    continue
                av[i] = d
                if _healthy(d):
                    hf.setdefault(_hive(d), {})[i] = d
                    n += 1
            self.nfree[rn] = n

    def free_count(self, rname, healthy_only=True) -> int:
        if healthy_only:
            return self.nfree.get(rname, 0)
        return len(self.available.get(rname) or ())


DEFAULT_FAILURE_DOMAINS = ("kubernetes.io/hostname", "failure-domain.beta.kubernetes.io/zone",
                           "failure-domain.beta.kubernetes.io/region")


class NodeInfo:
    __slots__ = ("node", "name", "labels", "taints", "alloc_cpu", "alloc_mem", "alloc_eph", "alloc_pods", "alloc_scalars",
                 "req_cpu", "req_mem", "req_eph", "req_scalars", "nz_cpu", "nz_mem", "pods", "ports", "er", "generation",
                 "ready", "unschedulable", "mem_pressure", "disk_pressure", "gpu_total", "images", "cond_reason")

    def __init__(self, name=""):
        self.node = None
        self.name = name
        self.labels = {}
        self.taints = []
        self.alloc_cpu = self.alloc_mem = self.alloc_eph = self.alloc_pods = 0
        self.alloc_scalars = {}
        self.req_cpu = self.req_mem = self.req_eph = 0
        self.req_scalars = {}
        self.nz_cpu = self.nz_mem = 0
        self.pods: dict[str, tuple] = {}   # key -> (pod, PodInfo)
        self.ports = set()
        self.er = ERManager()
        self.generation = 0
        self.ready = True
        self.cond_reason = None     # OutOfDisk / NetworkUnavailable not False (CheckNodeConditionPredicate)
        self.unschedulable = False
        self.mem_pressure = False
        self.disk_pressure = False
        self.gpu_total = 0
        self.images = {}

    def set_node(self, node):
        self.node = node
        self.name = node["metadata"]["name"]
        self.labels = node["metadata"].get("labels") or {}
        spec = node.get("spec") or {}
        st = node.get("status") or {}
        self.taints = spec.get("taints") or []
        self.unschedulable = bool(spec.get("unschedulable"))
        alloc = st.get("allocatable") or st.get("capacity") or {}
        self.alloc_cpu = _q(alloc["cpu"]).milli_value() if "cpu" in alloc else 0
        self.alloc_mem = _q(alloc["memory"]).int_value() if "memory" in alloc else 0
        self.alloc_eph = _q(alloc["ephemeral-storage"]).int_value() if "ephemeral-storage" in alloc else 0
        self.alloc_pods = _q(alloc["pods"]).int_value() if "pods" in alloc else 110
        self.alloc_scalars = {k: _q(v).int_value() for k, v in alloc.items()
                              if k not in ("cpu", "memory", "ephemeral-storage", "pods")}
        self.ready = True
        self.cond_reason = None
        self.mem_pressure = self.disk_pressure = False
        for c in st.get("conditions") or ():
            t, s = c.get("type"), c.get("status")
            if t == "Ready":
                self.ready = s == "True"
            elif t == "OutOfDisk" and s != "False":
                self.cond_reason = self.cond_reason or "node(s) were out of disk space"
            elif t == "NetworkUnavailable" and s != "False":
                self.cond_reason = self.cond_reason or "node(s) had unavailable network"
            elif t == "MemoryPressure":
                self.mem_pressure = s == "True"
            elif t == "DiskPressure":
                self.disk_pressure = s == "True"
        self.er.set_node(node)
        self.gpu_total = len(self.er.allocatable.get(core.AMD_GPU, {}))
        imgs = {}
        for im in (node.get("status") or {}).get("images") or ():
            for n in im.get("names") or ():
                imgs[n] = im.get("sizeBytes", 0)
        self.images = imgs
        self.generation += 1

    def clone(self):
        """Independent copy for what-if evaluation (preemption)."""
        c = NodeInfo(self.name)
        for s in ("node", "labels", "taints", "alloc_cpu", "alloc_mem", "alloc_eph", "alloc_pods", "alloc_scalars",
                  "req_cpu", "req_mem", "req_eph", "nz_cpu", "nz_mem", "generation", "ready", "unschedulable",
                  "mem_pressure", "disk_pressure", "gpu_total", "images", "cond_reason"):
            setattr(c, s, getattr(self, s))
        c.req_scalars = dict(self.req_scalars)
        c.pods = dict(self.pods)
        c.ports = set(self.ports)
        c.er = self.er.clone()
        return c

    def add_pod(self, key, pod, pi: PodInfo):
        if key in self.pods:
            self.remove_pod(key)
        self.pods[key] = (pod, pi)
        self.req_cpu += pi.milli_cpu
        self.req_mem += pi.memory
        self.req_eph += pi.ephemeral
        for k, v in pi.scalars.items():
            self.req_scalars[k] = self.req_scalars.get(k, 0) + v
        self.nz_cpu += pi.nz_cpu
        self.nz_mem += pi.nz_mem
        for p in pi.ports:
            self.ports.add(p)
        self.er.add_pod(key, pi.assigned)
        self.generation += 1

    def remove_pod(self, key):
        ent = self.pods.pop(key, None)
        if ent is None:
            return False
        _, pi = ent
        self.req_cpu -= pi.milli_cpu
        self.req_mem -= pi.memory
        self.req_eph -= pi.ephemeral
        for k, v in pi.scalars.items():
            self.req_scalars[k] = self.req_scalars.get(k, 0) - v
        self.nz_cpu -= pi.nz_cpu
        self.nz_mem -= pi.nz_mem
        for p in pi.ports:
            self.ports.discard(p)
        self.er.remove_pod(key, pi.assigned)
        self.generation += 1
        return True


class SchedulerCache:
    def __init__(self, assumed_ttl=30.0):
        self.nodes: dict[str, NodeInfo] = {}
        self.pod_states: dict[str, tuple] = {}   # key -> (pod, node name)
        self.assumed: dict[str, float] = {}      # key -> deadline (0 until binding finished)
        self.ttl = assumed_ttl
        self.anti_pods: dict[str, dict] = {}     # pods with required anti-affinity (symmetry check)
        # pods whose own affinity terms score incoming pods (interpod_affinity.go "existing pod"
        # branch): any podAffinity, or preferred podAntiAffinity
        self.affinity_pods: dict[str, dict] = {}
        self.hard_pod_affinity_weight = 1        # --hard-pod-affinity-symmetric-weight
        # --failure-domains: the topology an EMPTY topologyKey of a preferred pod (anti-)affinity
        # term stands for — nodes are in one domain when they share any of these labels' values
        # (`algorithm/priorities/util/topologies.go` NodesHaveSameTopologyKey)
        self.failure_domains = DEFAULT_FAILURE_DOMAINS
        self.volumes = VolumeLister()
        self.services: dict[str, dict[str, dict | None]] = {}   # namespace -> service -> selector

    # -- services (spreading / service affinity) -----------------------------
    def set_service(self, svc):
        md = svc["metadata"]
        self.services.setdefault(md.get("namespace", "default"), {})[md["name"]] = \
            (svc.get("spec") or {}).get("selector")

    def remove_service(self, svc):
        md = svc["metadata"]
        d = self.services.get(md.get("namespace", "default"))
        if d is not None:
            d.pop(md["name"], None)
            if not d:
                self.services.pop(md.get("namespace", "default"), None)

    def _track(self, key, pod):
        aff = (pod.get("spec") or {}).get("affinity") or {}
        anti = aff.get("podAntiAffinity") or {}
        if anti.get("requiredDuringSchedulingIgnoredDuringExecution"):
            self.anti_pods[key] = pod
        else:
            self.anti_pods.pop(key, None)
        if aff.get("podAffinity") or anti.get("preferredDuringSchedulingIgnoredDuringExecution"):
            self.affinity_pods[key] = pod
        else:
            self.affinity_pods.pop(key, None)

    def _node(self, name):
        ni = self.nodes.get(name)
        if ni is None:
            ni = self.nodes[name] = NodeInfo(name)
        return ni

    # -- pods ---------------------------------------------------------------
    def assume_pod(self, pod, pi=None):
        key = ns_name(pod)
        if key in self.pod_states:
            raise ValueError(f"pod {key} is in the cache, so can't be assumed")
        node = pod["spec"]["nodeName"]
        self._node(node).add_pod(key, pod, pi.with_assigned(pod) if pi is not None else PodInfo(pod))
        self.pod_states[key] = (pod, node)
        self.assumed[key] = 0.0
        self._track(key, pod)

    def finish_binding(self, pod):
        key = ns_name(pod)
        if key in self.assumed:
            self.assumed[key] = time.monotonic() + self.ttl

    def _drop_empty(self, name):
        """`removePod`: a NodeInfo with neither a node nor pods is deleted."""
        ni = self.nodes.get(name)
        if ni is not None and ni.node is None and not ni.pods:
            del self.nodes[name]

    def forget_pod(self, pod):
        key = ns_name(pod)
        st = self.pod_states.get(key)
        if st is None or key not in self.assumed:
            return
        self._node(st[1]).remove_pod(key)
        self._drop_empty(st[1])
        del self.pod_states[key]
        del self.assumed[key]
        self.anti_pods.pop(key, None)
        self.affinity_pods.pop(key, None)

    def add_pod(self, pod):
        """Confirmed (bound) pod from the informer. An assumed pod is replaced by the API
        object; unlike the reference (cache.go:232-245) its devices are re-added, which is a
        no-op when the assumed copy already carried them (our assume() sets them)."""
        key = ns_name(pod)
        node = pod["spec"]["nodeName"]
        st = self.pod_states.get(key)
        if st is not None and st[1] == node:
            old = st[0]
            if old.get("spec") == pod.get("spec") and \
                    (old.get("metadata") or {}).get("labels") == (pod.get("metadata") or {}).get("labels"):
                # the bound copy of an assumed pod, or a status / metadata-only update (kubelet
                # status, graceful deletion): nothing the scheduler accounts for changed — keep
                # the parsed PodInfo, swap the object
                ni = self._node(node)
                ent = ni.pods.get(key)
                if ent is not None:
                    ni.pods[key] = (pod, ent[1])
                    self.pod_states[key] = (pod, node)
                    self.assumed.pop(key, None)
                    self._track(key, pod)
                    return
        if st is not None:
            self._node(st[1]).remove_pod(key)
            self._drop_empty(st[1])
        self._node(node).add_pod(key, pod, PodInfo(pod))
        self.pod_states[key] = (pod, node)
        self.assumed.pop(key, None)
        self._track(key, pod)

    def update_pod(self, old, new):
        self.add_pod(new)

    def remove_pod(self, pod):
        key = ns_name(pod)
        st = self.pod_states.pop(key, None)
        self.assumed.pop(key, None)
        self.anti_pods.pop(key, None)
        self.affinity_pods.pop(key, None)
        if st is not None:
            ni = self.nodes.get(st[1])
            if ni is not None:
                ni.remove_pod(key)
                if ni.node is None and not ni.pods:
                    del self.nodes[st[1]]

    def is_assumed(self, pod):
        return ns_name(pod) in self.assumed

    def get_pod(self, key):
        st = self.pod_states.get(key)
        return st[0] if st else None

    def cleanup_expired(self, now=None):
        now = time.monotonic() if now is None else now
        for key, dl in list(self.assumed.items()):
            if dl and dl < now:
                pod, node = self.pod_states[key]
                self._node(node).remove_pod(key)
                self._drop_empty(node)
                del self.pod_states[key]
                del self.assumed[key]
                self.anti_pods.pop(key, None)
                self.affinity_pods.pop(key, None)

    # -- nodes --------------------------------------------------------------
    def add_node(self, node):
        self._node(node["metadata"]["name"]).set_node(node)

    update_node = lambda self, old, new: self.add_node(new)  # noqa: E731

    def remove_node(self, node):
        name = node["metadata"]["name"]
        ni = self.nodes.get(name)
        if ni is None:
            return
        if ni.pods:
            # keep pod accounting until the pods are deleted (cache.go RemoveNode)
            ni.node = None
            ni.er = ERManager()
            ni.generation += 1
        else:
            del self.nodes[name]

    def node_list(self):
        return [ni for ni in self.nodes.values() if ni.node is not None]

    def drop_node(self, name):
        """Forget a node and every pod accounted on it (a partitioned scheduler shard that no
        longer owns the node)."""
        ni = self.nodes.pop(name, None)
        if ni is None:
            return
        for key in list(ni.pods):
            self.pod_states.pop(key, None)
            self.assumed.pop(key, None)
            self.anti_pods.pop(key, None)
