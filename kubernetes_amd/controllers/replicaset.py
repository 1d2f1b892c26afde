"""ReplicaSet / ReplicationController controller.

Parity: `pkg/controller/replicaset/replica_set.go` (manageReplicas with expectations and
slow-start batches, adoption of orphans and release of non-matching pods via
ControllerRefManager, deletion order `controller.ActivePods`: unscheduled < pending < not-ready <
ready for less time < more restarts < newer, status calculation with ReplicaFailure) and `pkg/controller/replication` (same logic over
ReplicationController with a map selector).
"""
from __future__ import annotations

import asyncio

from ..api import meta as m
from ..api.labels import selector_from_set
from ..client.rest import APIStatusError, is_not_found
from .base import (Controller, Expectations, active_pods_key, claim_objects, controller_ref, pod_from_template,
                   pod_is_active, pod_is_available, pod_is_ready, selector_of, split_key)

BURST = 500  # slowStartBatch upper bound per sync


class ReplicaSetController(Controller):
    name = "replicaset"
    resource = "replicasets"
    kind = "ReplicaSet"

    def setup(self):
        self.exp = Expectations()
        self.rs_inf = self.factory.get(self.resource)
        self.pod_inf = self.factory.get("pods")
        self.rs_inf.add_handler(self.enqueue, lambda o, n: self.enqueue(n), self._rs_deleted)
        self.pod_inf.add_handler(self._pod_added, self._pod_updated, self._pod_deleted)
        if "controllerUID" not in self.pod_inf.store.indexers:
            self.pod_inf.store.add_indexer("controllerUID", lambda p: [r["uid"] for r in (p["metadata"].get("ownerReferences") or ()) if r.get("controller")])
        if "namespace" not in self.pod_inf.store.indexers:
            self.pod_inf.store.add_indexer("namespace", lambda p: [p["metadata"].get("namespace", "")])

    def _selector(self, rs):
        if self.kind == "ReplicationController":
            return selector_from_set((rs.get("spec") or {}).get("selector") or ((rs.get("spec") or {}).get("template") or {}).get("metadata", {}).get("labels"))
        return selector_of(rs)

    def _owner_key(self, pod):
        ref = controller_ref(pod)
        if ref is None or ref.get("kind") != self.kind:
            return None
        return f"{pod['metadata'].get('namespace')}/{ref['name']}"

    def _rs_deleted(self, rs):
        self.exp.delete(m.ns_name(rs))

    def _pod_added(self, pod):
        k = self._owner_key(pod)
        if k:
            self.exp.observe_add(k)
            self.enqueue(k)
        elif not controller_ref(pod):
            self._enqueue_matching(pod)

    def _pod_updated(self, old, new):
        k = self._owner_key(new)
        if k:
            self.enqueue(k)
            ok = self._owner_key(old)
            if ok and ok != k:
                self.enqueue(ok)
        elif not controller_ref(new):
            self._enqueue_matching(new)

    def _pod_deleted(self, pod):
        k = self._owner_key(pod)
        if k:
            self.exp.observe_del(k)
            self.enqueue(k)

    def _enqueue_matching(self, pod):
        labels = pod["metadata"].get("labels") or {}
        ns = pod["metadata"].get("namespace")
        for rs in self.rs_inf.list():
            if rs["metadata"].get("namespace") == ns and self._selector(rs).matches(labels):
                self.enqueue(rs)

    async def sync(self, key):
        rs = self.rs_inf.get(key)
        if rs is None:
            self.exp.delete(key)
            return
        ns, name = split_key(key)
        sel = self._selector(rs)
        # claim pods (ControllerRefManager): keep matching owned pods, release owned pods whose
        # labels stopped matching, adopt matching active orphans
        owned = await claim_objects(self.client, rs, "pods", self.pod_inf.store.by_index("namespace", ns),
                                    lambda p: sel.matches(p["metadata"].get("labels") or {}),
                                    ignore=lambda p: not pod_is_active(p))
        active = [p for p in owned if pod_is_active(p)]
        err = None
        if self.exp.satisfied(key) and not rs["metadata"].get("deletionTimestamp"):
            try:
                await self._manage(rs, active, key)
            except APIStatusError as e:
                err = e
        await self._update_status(rs, owned, active, err)
        if err is not None:
            raise err

    async def _manage(self, rs, active, key):
        ns = rs["metadata"]["namespace"]
        want = int((rs.get("spec") or {}).get("replicas", 1))
        diff = len(active) - want
        if diff < 0:
            n = min(-diff, BURST)
            self.exp.expect(key, adds=n)
            tmpl = (rs.get("spec") or {}).get("template") or {}
            gen = rs["metadata"]["name"] + "-"
            # slow start batches (1, 2, 4, ...) like the reference's slowStartBatch
            batch, done = 1, 0
            while done < n:
                b = min(batch, n - done)
                res = await asyncio.gather(*(self.client.create("pods", pod_from_template(tmpl, rs, gen, ns), ns)
                                             for _ in range(b)), return_exceptions=True)
                errs = [r for r in res if isinstance(r, Exception)]
                for _ in errs:
                    self.exp.observe_add(key)
                done += b
                if errs:
                    for _ in range(n - done):
                        self.exp.observe_add(key)
                    self.recorder.event(rs, "Warning", "FailedCreate", f"Error creating: {errs[0]}")
                    raise errs[0]
                batch *= 2
            self.recorder.event(rs, "Normal", "SuccessfulCreate", f"Created {n} pods")
        elif diff > 0:
            victims = sorted(active, key=active_pods_key)[:min(diff, BURST)]
            self.exp.expect(key, dels=len(victims))

            async def rm(p):
                try:
                    await self.client.delete("pods", p["metadata"]["name"], ns)
                except APIStatusError as e:
                    self.exp.observe_del(key)
                    if not is_not_found(e):
                        raise
            await asyncio.gather(*(rm(p) for p in victims))
            self.recorder.event(rs, "Normal", "SuccessfulDelete", f"Deleted {len(victims)} pods")

    async def _update_status(self, rs, owned, active, manage_err=None):
        tmpl_labels = ((rs.get("spec") or {}).get("template") or {}).get("metadata", {}).get("labels") or {}
        ready = [p for p in active if pod_is_ready(p)]
        # availableReplicas: Ready for minReadySeconds (replica_set_utils.go calculateStatus)
        mrs = int((rs.get("spec") or {}).get("minReadySeconds") or 0)
        available = sum(1 for p in ready if pod_is_available(p, mrs))
        st = {"replicas": len(active),
              "fullyLabeledReplicas": sum(1 for p in active if all((p["metadata"].get("labels") or {}).get(k) == v for k, v in tmpl_labels.items())),
              "readyReplicas": len(ready), "availableReplicas": available,
              "observedGeneration": rs["metadata"].get("generation", 1)}
        if mrs and len(ready) != available:
            # look again once the newest ready pod has been ready for minReadySeconds
            self.queue.add_after(m.ns_name(rs), float(mrs))
        cur = rs.get("status") or {}
        # ReplicaFailure while pods cannot be created / deleted (replica_set_utils.go:105-118)
        conds = [c for c in cur.get("conditions") or ()]
        failure = next((c for c in conds if c.get("type") == "ReplicaFailure"), None)
        if manage_err is not None and failure is None:
            reason = "FailedCreate" if len(active) < int((rs.get("spec") or {}).get("replicas", 1)) else "FailedDelete"
            conds = conds + [{"type": "ReplicaFailure", "status": "True", "reason": reason,
                              "message": str(manage_err), "lastTransitionTime": m.now_rfc3339()}]
        elif manage_err is None and failure is not None:
            conds = [c for c in conds if c.get("type") != "ReplicaFailure"]
        if conds != (cur.get("conditions") or []):
            st["conditions"] = conds or None
        if all(cur.get(k, 0) == v for k, v in st.items() if k != "conditions") and "conditions" not in st:
            return
        try:
            await self.client.patch(self.resource, rs["metadata"]["name"], {"status": st}, rs["metadata"]["namespace"], "merge", "status")
        except APIStatusError as e:
            if not is_not_found(e):
                raise


class ReplicationControllerController(ReplicaSetController):
    name = "replicationcontroller"
    resource = "replicationcontrollers"
    kind = "ReplicationController"
