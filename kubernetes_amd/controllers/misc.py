"""ServiceAccount, Endpoints, ResourceQuota (status) and Disruption (PDB status) controllers.

Parity: `pkg/controller/serviceaccount` (a `default` ServiceAccount in every namespace),
`pkg/controller/endpoint/endpoints_controller.go` (Endpoints = ready / not-ready pod IPs of
the service selector, per port), `pkg/controller/resourcequota` (status.used recomputed —
including the fork's pod-level GPU requests, see admission/plugins.pod_usage),
`pkg/controller/disruption/disruption.go` (PDB currentHealthy / desiredHealthy /
disruptionsAllowed).
"""
from __future__ import annotations

import time

from ..api import meta as m
from ..api.labels import label_selector_as_selector, selector_from_set
from ..api.quantity import Quantity
from ..client.rest import APIStatusError, is_already_exists, is_not_found
from .base import Controller, controller_ref, pod_is_ready, split_key


class ServiceAccountController(Controller):
    name = "serviceaccount"
    workers = 1

    def setup(self):
        self.ns_inf = self.factory.get("namespaces")
        self.sa_inf = self.factory.get("serviceaccounts")
        # `serviceaccounts_controller.go`: namespace adds and updates (a namespace that stopped
        # terminating), account deletions re-create the default account
        self.ns_inf.add_handler(lambda n: self.enqueue(n["metadata"]["name"]),
                                lambda o, n: self.enqueue(n["metadata"]["name"]), None)
        self.sa_inf.add_handler(None, None, lambda sa: self.enqueue(sa["metadata"]["namespace"]))

    async def sync(self, key):
        ns = self.ns_inf.get(key)
        if ns is None or ns["metadata"].get("deletionTimestamp"):
            return
        if self.sa_inf.get(f"{key}/default") is not None:
            return
        try:
            await self.client.create("serviceaccounts", {"metadata": {"name": "default", "namespace": key}}, key)
        except APIStatusError as e:
            if not (is_already_exists(e) or e.code in (403, 404)):
                raise


def _semantic(o):
    """apiequality.Semantic.DeepEqual for wire objects: empty values (omitted on the wire, e.g.
    by the protobuf codec) compare equal to absent ones."""
    if isinstance(o, dict):
        return {k: _semantic(v) for k, v in o.items() if v not in (None, "", [], {})}
    if isinstance(o, list):
        return [_semantic(v) for v in o]
    return o


TOLERATE_UNREADY = "service.alpha.kubernetes.io/tolerate-unready-endpoints"
LEADER_ANNOTATION = "control-plane.alpha.kubernetes.io/leader"


def should_pod_be_in_endpoints(pod) -> bool:
    """`shouldPodBeInEndpoints`: a not-ready pod is listed as notReady unless it can never run
    again (Never: Failed/Succeeded; OnFailure: Succeeded)."""
    policy = (pod.get("spec") or {}).get("restartPolicy", "Always")
    phase = (pod.get("status") or {}).get("phase")
    if policy == "Never":
        return phase not in ("Failed", "Succeeded")
    if policy == "OnFailure":
        return phase != "Succeeded"
    return True


def repack_subsets(entries):
    """`endpoints.RepackSubsets` + `SortSubsets`: entries are (address, port, ready); addresses
    are de-duplicated by (ip, targetRef uid) keeping "ready" once seen ready; ports offered by
    the same set of addresses (with the same readiness) share one subset."""
    addrs, by_port = {}, {}
    for addr, port, ready in entries:
        key = (addr["ip"], (addr.get("targetRef") or {}).get("uid"))
        addrs.setdefault(key, addr)
        pk = (port.get("name", ""), port["port"], port.get("protocol", "TCP"))
        cur = by_port.setdefault(pk, {})
        cur[key] = cur.get(key, False) or ready
    groups = {}
    for pk, amap in by_port.items():
        groups.setdefault(tuple(sorted(amap.items())), []).append(pk)
    out = []
    for amap, ports in groups.items():
        ss = {}
        ready = sorted((addrs[k] for k, r in amap if r), key=lambda a: (a["ip"], (a.get("targetRef") or {}).get("uid", "")))
        not_ready = sorted((addrs[k] for k, r in amap if not r),
                           key=lambda a: (a["ip"], (a.get("targetRef") or {}).get("uid", "")))
        if ready:
            ss["addresses"] = ready
        if not_ready:
            ss["notReadyAddresses"] = not_ready
        ss["ports"] = [{"name": n, "port": p, "protocol": pr} if n else {"port": p, "protocol": pr}
                       for n, p, pr in sorted(ports)]
        out.append(ss)
    out.sort(key=lambda ss: repr(ss["ports"]))
    return out


class EndpointsController(Controller):
    """`pkg/controller/endpoint/endpoints_controller.go` syncService: for a service with a
    selector, every selected pod with an IP becomes an address for each service port it has
    (`FindPort`; a headless service without ports gets port-less addresses), ready or
    notReady (`shouldPodBeInEndpoints`) — all ready when the service tolerates unready
    endpoints (the `tolerate-unready-endpoints` annotation or spec.publishNotReadyAddresses),
    which also keeps terminating pods; the hostname is published when the pod's
    hostname/subdomain name this service; subsets are repacked (`RepackSubsets`). Endpoints
    carry the service's labels and are written only on a change; a deleted service's endpoints
    are deleted, and leftover endpoints (no service, not a leader-election record) are queued at
    start (`checkLeftoverEndpoints`)."""
    name = "endpoint"

    def setup(self):
        self.svc_inf = self.factory.get("services")
        self.pod_inf = self.factory.get("pods")
        self.ep_inf = self.factory.get("endpoints")
        self.svc_inf.add_handler(self.enqueue, lambda o, n: self.enqueue(n), self.enqueue)
        self.pod_inf.add_handler(self._pod, self._pod_update, self._pod)

    def start(self):
        super().start()
        for ep in self.ep_inf.list():
            if LEADER_ANNOTATION not in ((ep.get("metadata") or {}).get("annotations") or {}):
                self.enqueue(ep)

    def _services_for(self, pod):
        ns = pod["metadata"].get("namespace")
        labels = pod["metadata"].get("labels") or {}
        for svc in self.svc_inf.list():
            sel = (svc.get("spec") or {}).get("selector")
            if svc["metadata"].get("namespace") == ns and sel is not None and selector_from_set(sel).matches(labels):
                yield svc

    def _pod(self, pod):
        for svc in self._services_for(pod):
            self.enqueue(svc)

    def _pod_update(self, old, new):
        """`updatePod`: nothing to do unless something endpoints show changed; a label change
        re-syncs the services of both label sets."""
        if old.get("metadata", {}).get("resourceVersion") == new.get("metadata", {}).get("resourceVersion"):
            return
        if (old["metadata"].get("labels") or {}) != (new["metadata"].get("labels") or {}):
            self._pod(old)
        self._pod(new)

    async def sync(self, key):
        ns, name = split_key(key)
        svc = self.svc_inf.get(key)
        if svc is None:
            try:
                await self.client.delete("endpoints", name, ns)
            except APIStatusError as e:
                if not is_not_found(e):
                    raise
            return
        spec = svc.get("spec") or {}
        sel = spec.get("selector")
        if sel is None:
            return          # endpoints of a selector-less service are managed by the user
        ann = svc["metadata"].get("annotations") or {}
        tolerate = str(ann.get(TOLERATE_UNREADY, "")).lower() in ("true", "1", "t") or \
            bool(spec.get("publishNotReadyAddresses"))
        s = selector_from_set(sel)
        svc_ports = spec.get("ports") or ()
        entries = []
        for p in self.pod_inf.list():
            md = p["metadata"]
            if md.get("namespace") != ns or not s.matches(md.get("labels") or {}):
                continue
            ip = (p.get("status") or {}).get("podIP")
            if not ip or (not tolerate and md.get("deletionTimestamp")):
                continue
            pspec = p.get("spec") or {}
            addr = {"ip": ip, "nodeName": pspec.get("nodeName"),
                    "targetRef": {"kind": "Pod", "namespace": ns, "name": md["name"], "uid": md.get("uid"),
                                  "resourceVersion": md.get("resourceVersion")}}
            if pspec.get("hostname") and pspec.get("subdomain") == name:
                addr["hostname"] = pspec["hostname"]
            ready = tolerate or pod_is_ready(p)
            if not ready and not should_pod_be_in_endpoints(p):
                continue
            if not svc_ports:
                if spec.get("clusterIP") == "None":
                    entries.append((addr, {"port": 0, "protocol": "TCP"}, ready))
                continue
            for sp in svc_ports:
                port = find_port(p, sp)
                if port is None:          # a named port the pod lacks: not an endpoint for it
                    continue
                entries.append((addr, {"name": sp.get("name", ""), "port": port,
                                       "protocol": sp.get("protocol", "TCP")}, ready))
        subsets = repack_subsets(entries)
        labels = svc["metadata"].get("labels") or {}
        cur = self.ep_inf.get(key)
        if cur is not None and _semantic(cur.get("subsets") or []) == _semantic(subsets) and \
                (cur["metadata"].get("labels") or {}) == labels:
            return
        if cur is None:
            ep = {"apiVersion": "v1", "kind": "Endpoints",
                  "metadata": {"name": name, "namespace": ns, "labels": labels}, "subsets": subsets}
            try:
                await self.client.create("endpoints", ep, ns)
                return
            except APIStatusError as e:
                if not is_already_exists(e):
                    raise
                cur = await self.client.get("endpoints", name, ns)
        new = dict(cur, subsets=subsets)
        new["metadata"] = dict(cur["metadata"], labels=labels)
        await self.client.update("endpoints", new, ns)


def find_port(pod, svc_port):
    """`podutil.FindPort`: the service port's targetPort as a number — an int (or digits) as
    is, a name looked up among the pod's container ports of the same protocol; None when the
    pod has no such named port."""
    tp = svc_port.get("targetPort", svc_port.get("port"))
    if isinstance(tp, int):
        return tp
    if isinstance(tp, str) and tp.isdigit():
        return int(tp)
    proto = svc_port.get("protocol", "TCP")
    for c in (pod.get("spec") or {}).get("containers") or ():
        for cp in c.get("ports") or ():
            if cp.get("name") == tp and cp.get("protocol", "TCP") == proto:
                return int(cp["containerPort"])
    return None


class ResourceQuotaController(Controller):
    """`pkg/controller/resourcequota/resource_quota_controller.go` syncResourceQuota: status.hard
    mirrors spec.hard and status.used is recounted for every hard name by the quota evaluators
    (`kubernetes_amd.quota`), respecting the quota's scopes, then masked to the hard names; the
    status is written only when hard or used changed. Replenishment: any change to an object
    the static evaluators count (pods, services, PVCs, configmaps, secrets,
    replicationcontrollers, resourcequotas) re-queues the quotas of its namespace; other
    `count/<resource>.<group>` names are recounted from a live list at sync time and on the
    periodic resync (`--resource-quota-sync-period`, 5 min)."""
    name = "resourcequota"
    primary = "resourcequotas"
    workers = 2
    resync_period = 300.0
    WATCHED = ("pods", "services", "persistentvolumeclaims", "configmaps", "secrets", "replicationcontrollers")

    def setup(self):
        from ..quota import Registry
        self.registry = Registry()
        self.rq_inf = self.factory.get("resourcequotas")
        self.rq_inf.add_handler(self.enqueue, self._rq_update, None)
        self.infs = {"resourcequotas": self.rq_inf}
        for r in self.WATCHED:
            inf = self.infs[r] = self.factory.get(r)
            inf.add_handler(self._obj, lambda o, n: self._obj(n), self._obj)

    def _rq_update(self, old, new):
        # our own status writes come back as updates: only spec changes need a recount
        if (old.get("spec") or {}) != (new.get("spec") or {}) or not (new.get("status") or {}).get("used"):
            self.enqueue(new)

    def _obj(self, obj):
        ns = (obj.get("metadata") or {}).get("namespace")
        if not ns:
            return
        for q in self.rq_inf.list():
            if q["metadata"].get("namespace") == ns:
                self.enqueue(q)

    async def _objects(self, ns, hard):
        """{(group, resource): objects in ns} for every kind some hard name counts."""
        out = {}
        for n in hard:
            ev = self.registry.for_name(n)
            if ev is None or (ev.group, ev.resource) in out:
                continue
            if not ev.group and ev.resource in self.infs:
                out[("", ev.resource)] = [o for o in self.infs[ev.resource].list()
                                          if o["metadata"].get("namespace") == ns]
                continue
            ri = await self._resource_info(ev.group, ev.resource)
            if ri is None:
                out[(ev.group, ev.resource)] = []
                continue
            try:
                out[(ev.group, ev.resource)] = (await self.client.list(ri, ns if ri.namespaced else None))["items"]
            except APIStatusError as e:
                if e.code not in (403, 404, 405):
                    raise
                out[(ev.group, ev.resource)] = []
        return out

    async def _resource_info(self, group, resource):
        """Built-in resources from the local table; anything else (custom resources) through
        API discovery, cached per resync."""
        ri = m.BY_PLURAL.get(resource)
        if ri is not None and ri.group == group:
            return ri
        cache = getattr(self, "_discovered", None)
        if cache is None or time.monotonic() - cache[0] > self.resync_period:
            from .garbagecollector import deletable_resources, discover
            try:
                infos = deletable_resources(await discover(self.client), ignored=())
            except APIStatusError:
                infos = []
            cache = self._discovered = (time.monotonic(), {(r.group, r.plural): r for r in infos})
        return cache[1].get((group, resource))

    async def sync(self, key):
        from .. import quota
        q = self.rq_inf.get(key)
        if q is None:
            return
        ns, name = split_key(key)
        spec = q.get("spec") or {}
        hard = dict(spec.get("hard") or {})
        st0 = q.get("status") or {}
        objs = await self._objects(ns, hard)
        used = dict(st0.get("used") or {})
        used.update(quota.calculate_usage(lambda g, r: objs.get((g, r), ()), spec.get("scopes") or (), hard,
                                          self.registry))
        used = quota.to_strings(quota.mask(used, hard))
        dirty = (st0.get("hard") is None or st0.get("used") is None
                 or not quota.equals(st0.get("hard") or {}, hard)
                 or not quota.equals(st0.get("used") or {}, used))
        if not dirty:
            return
        body = dict(q, status={"hard": hard, "used": used})
        await self.client.update_status("resourcequotas", body, ns)


class DisruptionController(Controller):
    """`pkg/controller/disruption/disruption.go`: a budget's expected pod count is the pods it
    selects for an integer minAvailable, and the summed scale of their controllers
    (ReplicaSet / ReplicationController / StatefulSet / Deployment) for a percentage or any
    maxUnavailable (`getExpectedPodCount`, `getExpectedScale`); healthy pods are Ready ones not
    already counted as disrupted; status.disruptedPods entries (written by the eviction
    subresource) are dropped once the pod is deleted or after DeletionTimeout (2 min), when the
    budget is looked at again."""
    name = "disruption"
    workers = 2
    DELETION_TIMEOUT = 120.0

    def setup(self):
        self.pdb_inf = self.factory.get("poddisruptionbudgets")
        self.pod_inf = self.factory.get("pods")
        self.infs = {k: self.factory.get(r) for k, r in (("ReplicaSet", "replicasets"),
                                                           ("ReplicationController", "replicationcontrollers"),
                                                           ("StatefulSet", "statefulsets"),
                                                           ("Deployment", "deployments"))}
        self.pdb_inf.add_handler(self.enqueue, lambda o, n: self.enqueue(n), None)
        self.pod_inf.add_handler(self._pod, lambda o, n: self._pod(n), self._pod)

    def _pod(self, pod):
        for pdb in self.pdb_inf.list():
            if pdb["metadata"].get("namespace") == pod["metadata"].get("namespace"):
                self.enqueue(pdb)

    def expected_scale(self, pods):
        """Sum of the scale of every controller that owns a selected pod (each counted once);
        a pod without a (known) controller makes the count unknowable -> None."""
        seen = {}
        for p in pods:
            ref = controller_ref(p)
            if ref is None:
                return None
            kind = ref.get("kind")
            key = (kind, ref.get("uid"))
            if key in seen:
                continue
            ctl = None
            if kind == "ReplicaSet":
                rs = self.infs["ReplicaSet"].get(f"{m.namespace_of(p)}/{ref['name']}")
                dref = controller_ref(rs) if rs is not None else None
                if dref is not None and dref.get("kind") == "Deployment":
                    d = self.infs["Deployment"].get(f"{m.namespace_of(p)}/{dref['name']}")
                    if d is not None and m.uid_of(d) == dref.get("uid"):
                        key, ctl = ("Deployment", m.uid_of(d)), d
                        if key in seen:
                            continue
                if ctl is None:
                    ctl = rs
            elif kind in self.infs:
                ctl = self.infs[kind].get(f"{m.namespace_of(p)}/{ref['name']}")
            if ctl is None or m.uid_of(ctl) != key[1]:
                return None
            seen[key] = int((ctl.get("spec") or {}).get("replicas", 1))
        return sum(seen.values())

    async def sync(self, key):
        pdb = self.pdb_inf.get(key)
        if pdb is None:
            return
        ns, name = split_key(key)
        spec = pdb.get("spec") or {}
        raw_sel = spec.get("selector") or {}
        sel = label_selector_as_selector(raw_sel)
        # getPodsForPdb: an empty selector selects nothing
        pods = [] if not (raw_sel.get("matchLabels") or raw_sel.get("matchExpressions")) else \
            [p for p in self.pod_inf.list() if p["metadata"].get("namespace") == ns
             and sel.matches(p["metadata"].get("labels") or {})]
        now = time.time()
        st0 = pdb.get("status") or {}
        # disruptedPods: kept while the evicted pod still exists, undeleted, within the timeout
        by_name = {m.name_of(p): p for p in pods}
        disrupted, recheck = {}, None
        for pname, ts in (st0.get("disruptedPods") or {}).items():
            p = by_name.get(pname)
            t = m.parse_rfc3339(ts) or 0
            if p is None or p["metadata"].get("deletionTimestamp") or t + self.DELETION_TIMEOUT < now:
                continue
            disrupted[pname] = ts
            left = t + self.DELETION_TIMEOUT - now
            recheck = left if recheck is None else min(recheck, left)
        healthy = sum(1 for p in pods if not p["metadata"].get("deletionTimestamp")
                      and pod_is_ready(p) and m.name_of(p) not in disrupted)
        min_avail, max_unavail = spec.get("minAvailable"), spec.get("maxUnavailable")
        failed = False
        if max_unavail is not None:
            expected = self.expected_scale(pods)
            failed = expected is None
            expected = expected or 0
            desired = max(0, expected - _abs(max_unavail, expected, round_up=True))
        elif min_avail is not None and isinstance(min_avail, str) and min_avail.endswith("%"):
            expected = self.expected_scale(pods)
            failed = expected is None
            expected = expected or 0
            desired = _abs(min_avail, expected, round_up=True)
        else:
            expected = len(pods)
            desired = _abs(min_avail, expected) if min_avail is not None else expected
        allowed = 0 if failed else max(0, healthy - desired)
        st = {"currentHealthy": healthy, "desiredHealthy": desired, "expectedPods": expected,
              "disruptionsAllowed": allowed, "observedGeneration": pdb["metadata"].get("generation", 1),
              "disruptedPods": disrupted or None}
        if recheck is not None:
            self.queue.add_after(key, recheck + 0.05)
        cur = {k: st0.get(k) for k in st}
        if cur.get("disruptedPods") == {}:
            cur["disruptedPods"] = None
        if cur == st:
            return
        patch = dict(st)
        if disrupted:          # a merge patch merges maps: dropped entries are nulled explicitly
            patch["disruptedPods"] = dict({k: None for k in st0.get("disruptedPods") or ()}, **disrupted)
        await self.client.patch("poddisruptionbudgets", name, {"status": patch}, ns, "merge", "status")


def _abs(v, total, round_up=True):
    """intstr.GetValueFromIntOrPercent (the disruption controller rounds up)."""
    if isinstance(v, str) and v.endswith("%"):
        import math
        x = float(v[:-1]) * total / 100.0
        return int(math.ceil(x) if round_up else math.floor(x))
    return int(v)
