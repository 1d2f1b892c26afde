"""Deployment controller: ReplicaSets per pod-template hash, RollingUpdate / Recreate, status,
revision annotations and rollback to a revision.

Parity: `pkg/controller/deployment/{deployment_controller.go,sync.go,rolling.go,recreate.go,
rollback.go,util/deployment_util.go}` — `pod-template-hash` label, `deployment.kubernetes.io/revision`
annotation, maxSurge / maxUnavailable arithmetic, conditions Available / Progressing.
"""
from __future__ import annotations

import hashlib
import json
import math

from ..api import meta as m
from ..api.meta import now_rfc3339
from ..client.rest import APIStatusError, is_already_exists, is_not_found
from .base import Controller, controller_ref, split_key

REVISION = "deployment.kubernetes.io/revision"
HASH_LABEL = "pod-template-hash"


def template_hash(tmpl) -> str:
    h = hashlib.sha256(json.dumps(tmpl, sort_keys=True).encode()).hexdigest()
    return str(int(h[:8], 16) % (10 ** 10))


def _resolve(v, total, round_up):
    if v is None:
        return 0
    if isinstance(v, str) and v.endswith("%"):
        x = float(v[:-1]) * total / 100.0
        return int(math.ceil(x) if round_up else math.floor(x))
    return int(v)


class DeploymentController(Controller):
    name = "deployment"
    primary = "deployments"
    workers = 2

    def setup(self):
        self.d_inf = self.factory.get("deployments")
        self.rs_inf = self.factory.get("replicasets")
        self.d_inf.add_handler(self.enqueue, lambda o, n: self.enqueue(n), None)
        self.rs_inf.add_handler(self._rs_event, lambda o, n: self._rs_event(n), self._rs_event)

    def _rs_event(self, rs):
        ref = controller_ref(rs)
        if ref and ref.get("kind") == "Deployment":
            self.enqueue(f"{rs['metadata']['namespace']}/{ref['name']}")

    def _owned_rs(self, d):
        uid = d["metadata"]["uid"]
        ns = d["metadata"]["namespace"]
        return [rs for rs in self.rs_inf.list() if rs["metadata"].get("namespace") == ns and (controller_ref(rs) or {}).get("uid") == uid]

    async def sync(self, key):
        d = self.d_inf.get(key)
        if d is None or d["metadata"].get("deletionTimestamp"):
            return
        ns, name = split_key(key)
        spec = d.get("spec") or {}
        if spec.get("paused"):
            return
        rollback = (spec.get("rollbackTo") or {}).get("revision") if spec.get("rollbackTo") else None
        rss = self._owned_rs(d)
        if rollback is not None:
            await self._rollback(d, rss, int(rollback))
            return
        tmpl = spec.get("template") or {}
        h = template_hash(tmpl)
        new_rs = next((rs for rs in rss if (rs["metadata"].get("labels") or {}).get(HASH_LABEL) == h), None)
        old = [rs for rs in rss if rs is not new_rs]
        max_rev = max([int((rs["metadata"].get("annotations") or {}).get(REVISION, "0")) for rs in rss] + [0])
        replicas = int(spec.get("replicas", 1))
        if new_rs is None:
            new_rs = await self._create_rs(d, tmpl, h, max_rev + 1, 0 if old and spec.get("strategy", {}).get("type") != "Recreate" else 0)
        elif int((new_rs["metadata"].get("annotations") or {}).get(REVISION, "0")) < max_rev:
            new_rs = await self._patch_rs(new_rs, annotations={REVISION: str(max_rev + 1)})
        strategy = (spec.get("strategy") or {}).get("type", "RollingUpdate")
        if strategy == "Recreate":
            active_old = [rs for rs in old if int((rs.get("spec") or {}).get("replicas", 0)) > 0]
            for rs in active_old:
                await self._scale(rs, 0)
            if any(int((rs.get("status") or {}).get("replicas", 0)) > 0 for rs in old):
                return  # wait for old pods to terminate
            await self._scale(new_rs, replicas)
        else:
            ru = (spec.get("strategy") or {}).get("rollingUpdate") or {}
            surge = _resolve(ru.get("maxSurge", "25%"), replicas, True)
            unavail = _resolve(ru.get("maxUnavailable", "25%"), replicas, False)
            if surge == 0 and unavail == 0:
                unavail = 1
            new_cur = int((new_rs.get("spec") or {}).get("replicas", 0))
            old_total = sum(int((rs.get("spec") or {}).get("replicas", 0)) for rs in old)
            # scale up new within surge
            max_total = replicas + surge
            if new_cur < replicas:
                up = min(replicas - new_cur, max(0, max_total - (new_cur + old_total)))
                if not old:
                    up = replicas - new_cur
                if up > 0:
                    new_rs = await self._scale(new_rs, new_cur + up)
                    new_cur += up
            elif new_cur > replicas:
                new_rs = await self._scale(new_rs, replicas)
                new_cur = replicas
            # scale down old keeping availability
            avail_new = int((new_rs.get("status") or {}).get("availableReplicas", 0))
            avail_old = sum(int((rs.get("status") or {}).get("availableReplicas", 0)) for rs in old)
            min_avail = replicas - unavail
            can_remove = max(0, avail_new + avail_old - min_avail)
            # pods that are not available in old RSes can always go
            for rs in sorted(old, key=lambda r: int((r["metadata"].get("annotations") or {}).get(REVISION, "0"))):
                cur = int((rs.get("spec") or {}).get("replicas", 0))
                if cur == 0:
                    continue
                unavail_old = max(0, cur - int((rs.get("status") or {}).get("availableReplicas", 0)))
                dec = min(cur, unavail_old + can_remove)
                if dec > 0:
                    await self._scale(rs, cur - dec)
                    can_remove = max(0, can_remove - max(0, dec - unavail_old))
        await self._cleanup(d, old)
        await self._status(d, new_rs, old)

    async def _create_rs(self, d, tmpl, h, revision, replicas):
        ns = d["metadata"]["namespace"]
        labels = dict((tmpl.get("metadata") or {}).get("labels") or {})
        labels[HASH_LABEL] = h
        t = m.fast_copy(tmpl)
        t.setdefault("metadata", {})["labels"] = labels
        sel = m.fast_copy((d.get("spec") or {}).get("selector") or {"matchLabels": dict(labels)})
        sel.setdefault("matchLabels", {})[HASH_LABEL] = h
        rs = {"apiVersion": "apps/v1", "kind": "ReplicaSet",
              "metadata": {"name": f"{d['metadata']['name']}-{h}", "namespace": ns, "labels": labels,
                           "annotations": {REVISION: str(revision)}, "ownerReferences": [m.owner_reference(d)]},
              "spec": {"replicas": replicas, "selector": sel, "template": t}}
        try:
            out = await self.client.create("replicasets", rs, ns)
            self.recorder.event(d, "Normal", "ScalingReplicaSet", f"Created new replica set {rs['metadata']['name']}")
            return out
        except APIStatusError as e:
            if is_already_exists(e):
                return await self.client.get("replicasets", rs["metadata"]["name"], ns)
            raise

    async def _patch_rs(self, rs, annotations=None):
        return await self.client.patch("replicasets", rs["metadata"]["name"], {"metadata": {"annotations": annotations}},
                                       rs["metadata"]["namespace"])

    async def _scale(self, rs, n):
        if int((rs.get("spec") or {}).get("replicas", 0)) == n:
            return rs
        try:
            return await self.client.patch("replicasets", rs["metadata"]["name"], {"spec": {"replicas": n}}, rs["metadata"]["namespace"])
        except APIStatusError as e:
            if is_not_found(e):
                return rs
            raise

    async def _cleanup(self, d, old):
        limit = (d.get("spec") or {}).get("revisionHistoryLimit", 10)
        dead = [rs for rs in old if int((rs.get("spec") or {}).get("replicas", 0)) == 0 and int((rs.get("status") or {}).get("replicas", 0)) == 0]
        dead.sort(key=lambda r: int((r["metadata"].get("annotations") or {}).get(REVISION, "0")))
        for rs in dead[:max(0, len(dead) - int(limit))]:
            try:
                await self.client.delete("replicasets", rs["metadata"]["name"], rs["metadata"]["namespace"])
            except APIStatusError:
                pass

    async def _rollback(self, d, rss, revision):
        target = None
        if revision == 0:
            revs = sorted(rss, key=lambda r: int((r["metadata"].get("annotations") or {}).get(REVISION, "0")))
            target = revs[-2] if len(revs) >= 2 else None
        else:
            target = next((r for r in rss if (r["metadata"].get("annotations") or {}).get(REVISION) == str(revision)), None)
        # the template is replaced as a whole (a merge patch would keep labels the target lacks),
        # guarded by the resourceVersion the decision was made on
        ops = [{"op": "test", "path": "/metadata/resourceVersion", "value": d["metadata"]["resourceVersion"]},
               {"op": "remove", "path": "/spec/rollbackTo"}]
        if target is not None:
            t = m.fast_copy((target.get("spec") or {}).get("template") or {})
            (t.get("metadata") or {}).get("labels", {}).pop(HASH_LABEL, None)
            ops.append({"op": "replace", "path": "/spec/template", "value": t})
            rev = (target["metadata"].get("annotations") or {}).get(REVISION, str(revision))
            self.recorder.event(d, "Normal", "DeploymentRollback", f"Rolled back deployment {d['metadata']['name']} to revision {rev}")
        else:
            self.recorder.event(d, "Warning", "DeploymentRollbackRevisionNotFound", "Unable to find the revision to rollback to.")
        await self.client.patch("deployments", d["metadata"]["name"], ops, d["metadata"]["namespace"], "json")

    async def _status(self, d, new_rs, old):
        allrs = [new_rs] + old
        replicas = int((d.get("spec") or {}).get("replicas", 1))
        tot = sum(int((r.get("status") or {}).get("replicas", 0)) for r in allrs)
        ready = sum(int((r.get("status") or {}).get("readyReplicas", 0)) for r in allrs)
        avail = sum(int((r.get("status") or {}).get("availableReplicas", 0)) for r in allrs)
        upd = int((new_rs.get("status") or {}).get("replicas", 0))
        unavail = max(0, replicas - avail)
        now = now_rfc3339()
        conds = [{"type": "Available", "status": "True" if avail >= replicas - _resolve(
            ((d.get("spec") or {}).get("strategy") or {}).get("rollingUpdate", {}).get("maxUnavailable", "25%"), replicas, False) else "False",
                  "reason": "MinimumReplicasAvailable", "lastUpdateTime": now, "lastTransitionTime": now},
                 {"type": "Progressing", "status": "True",
                  "reason": "NewReplicaSetAvailable" if upd == replicas and avail == replicas else "ReplicaSetUpdated",
                  "message": f'ReplicaSet "{new_rs["metadata"]["name"]}" is progressing.', "lastUpdateTime": now,
                  "lastTransitionTime": now}]
        st = {"observedGeneration": d["metadata"].get("generation", 1), "replicas": tot, "updatedReplicas": upd,
              "readyReplicas": ready, "availableReplicas": avail, "unavailableReplicas": unavail}
        cur = d.get("status") or {}
        if all(cur.get(k) == v for k, v in st.items()):
            return
        st["conditions"] = conds
        try:
            await self.client.patch("deployments", d["metadata"]["name"], {"status": st}, d["metadata"]["namespace"], "merge", "status")
        except APIStatusError as e:
            if not is_not_found(e):
                raise
