"""Deployment controller.

Parity: `pkg/controller/deployment/`
  * `deployment_controller.go:syncDeployment` (`:560-640`): claim ReplicaSets (adopt orphans that
    match the selector, release owned ones that stop matching); an empty selector selects
    nothing; a deleted deployment only has its status synced; paused deployments still *scale*
    (`sync`) but do not roll out (`:622`); `rollbackTo` is handled before anything else; a scaling
    event (an active RS whose desired-replicas annotation differs from spec.replicas,
    `isScalingEvent`) is a proportional scale, not a rollout;
  * `sync.go`: `getNewReplicaSet` (create the RS for the current template or bump the existing
    one's revision / minReadySeconds, with the Progressing condition FoundNewReplicaSet /
    NewReplicaSetCreated / ReplicaSetCreateError), `scale` (`:385`: proportional scaling across
    every active RS using the max-replicas annotation, leftovers to the largest),
    `scaleReplicaSet` (replicas plus desired/max-replicas annotations), `cleanupDeployment`
    (revisionHistoryLimit), `calculateStatus` (Available = availableReplicas >= replicas -
    maxUnavailable: MinimumReplicasAvailable / MinimumReplicasUnavailable);
  * `rolling.go`: reconcileNewReplicaSet / reconcileOldReplicaSets (cleanupUnhealthyReplicas, then
    scaleDownOldReplicaSetsForRollingUpdate);
  * `recreate.go`: scale every old RS to 0, wait until no old pod is running, then scale up;
  * `rollback.go`: rollbackTo.revision (0 = the previous revision) copies that RS's template
    and annotations, then clears rollbackTo;
  * `progress.go`: `syncRolloutStatus` — Progressing=True ReplicaSetUpdated while the rollout
    moves, NewReplicaSetAvailable when complete, Progressing=False ProgressDeadlineExceeded when
    no progress was made for progressDeadlineSeconds (`DeploymentTimedOut`); stuck deployments
    are requeued for the moment their deadline passes (`requeueStuckDeployment`); ReplicaSet
    ReplicaFailure conditions surface on the deployment; paused/resumed conditions
    (`checkPausedConditions`).
"""
from __future__ import annotations

from ..api import meta as m
from ..api.labels import label_selector_as_selector
from ..api.meta import now_rfc3339, parse_rfc3339
from ..client.rest import APIStatusError, is_already_exists, is_not_found
from . import deployment_util as U
from .base import Controller, controller_ref, split_key
from .deployment_util import HASH_LABEL, REVISION, template_hash  # noqa: F401  (re-export)


class DeploymentController(Controller):
    name = "deployment"
    primary = "deployments"
    workers = 5                      # --concurrent-deployment-syncs

    def setup(self):
        self.d_inf = self.factory.get("deployments")
        self.rs_inf = self.factory.get("replicasets")
        self.pod_inf = self.factory.get("pods")
        self.d_inf.add_handler(self.enqueue, lambda o, n: self.enqueue(n), self.enqueue)
        self.rs_inf.add_handler(self._rs_added, self._rs_updated, self._rs_deleted)
        self.pod_inf.add_handler(None, None, self._pod_deleted)

    # -- event handlers (deployment_controller.go:160-380) --------------------------------------
    def _owner_key(self, rs):
        ref = controller_ref(rs)
        if ref and ref.get("kind") == "Deployment":
            return f"{m.namespace_of(rs)}/{ref['name']}"
        return None

    def _deployments_for_orphan(self, rs):
        labels = rs["metadata"].get("labels") or {}
        for d in self.d_inf.list():
            if m.namespace_of(d) != m.namespace_of(rs):
                continue
            sel = label_selector_as_selector((d.get("spec") or {}).get("selector"))
            if not sel.empty() and sel.matches(labels):
                self.enqueue(d)

    def _rs_added(self, rs):
        k = self._owner_key(rs)
        if k:
            self.enqueue(k)
        elif controller_ref(rs) is None:
            self._deployments_for_orphan(rs)

    def _rs_updated(self, old, new):
        k, ok = self._owner_key(new), self._owner_key(old)
        if ok and ok != k:
            self.enqueue(ok)
        if k:
            self.enqueue(k)
        elif controller_ref(new) is None:
            self._deployments_for_orphan(new)

    def _rs_deleted(self, rs):
        k = self._owner_key(rs)
        if k:
            self.enqueue(k)

    def _pod_deleted(self, pod):
        """A Recreate deployment waits for the last old pod to go (`deletePod`, `:339`)."""
        ref = controller_ref(pod)
        if not ref or ref.get("kind") != "ReplicaSet":
            return
        rs = self.rs_inf.get(f"{m.namespace_of(pod)}/{ref['name']}")
        if rs is None:
            return
        k = self._owner_key(rs)
        if not k:
            return
        d = self.d_inf.get(k)
        if d is not None and ((d.get("spec") or {}).get("strategy") or {}).get("type") == "Recreate":
            self.enqueue(k)

    # -- claiming ----------------------------------------------------------------------------
    async def claim_replica_sets(self, d, sel):
        ns, uid = m.namespace_of(d), m.uid_of(d)
        out = []
        for rs in self.rs_inf.list():
            if m.namespace_of(rs) != ns:
                continue
            ref = controller_ref(rs)
            matches = sel.matches(rs["metadata"].get("labels") or {})
            if ref is not None:
                if ref.get("uid") != uid:
                    continue
                if matches:
                    out.append(rs)
                elif not rs["metadata"].get("deletionTimestamp"):
                    refs = [r for r in rs["metadata"].get("ownerReferences") or () if r.get("uid") != uid]
                    await self._patch_rs_meta(rs, {"ownerReferences": refs or None})
                continue
            if matches and not d["metadata"].get("deletionTimestamp") and not rs["metadata"].get("deletionTimestamp"):
                refs = list(rs["metadata"].get("ownerReferences") or ()) + [m.owner_reference(d)]
                adopted = await self._patch_rs_meta(rs, {"ownerReferences": refs, "uid": m.uid_of(rs)})
                if adopted is not None:
                    out.append(adopted)
        return out

    async def _patch_rs_meta(self, rs, md):
        try:
            return await self.client.patch("replicasets", m.name_of(rs), {"metadata": md}, m.namespace_of(rs))
        except APIStatusError as e:
            if is_not_found(e):
                return None
            raise

    def pods_by_rs(self, rss):
        uids = {m.uid_of(rs) for rs in rss}
        out = {u: [] for u in uids}
        for p in self.pod_inf.list():
            ref = controller_ref(p)
            if ref and ref.get("uid") in uids:
                out[ref["uid"]].append(p)
        return out

    # -- syncDeployment ----------------------------------------------------------------------
    async def sync(self, key):
        cached = self.d_inf.get(key)
        if cached is None:
            return
        d = m.fast_copy(cached)
        spec = d.get("spec") or {}
        sel_spec = spec.get("selector")
        if not sel_spec or not (sel_spec.get("matchLabels") or sel_spec.get("matchExpressions")):
            self.recorder.event(d, "Warning", "SelectingAll",
                                "This deployment is selecting all pods. A non-empty selector is required.")
            if (d.get("status") or {}).get("observedGeneration", 0) < d["metadata"].get("generation", 0):
                await self._write_status(d, dict(d.get("status") or {},
                                                 observedGeneration=d["metadata"].get("generation", 1)))
            return
        sel = label_selector_as_selector(sel_spec)
        rss = await self.claim_replica_sets(d, sel)
        if d["metadata"].get("deletionTimestamp"):
            await self.sync_status_only(d, rss)
            return
        d = await self.check_paused_conditions(d)
        if spec.get("paused"):
            await self.sync_scale(d, rss)
            return
        if spec.get("rollbackTo") is not None:
            await self.rollback(d, rss)
            return
        if await self.is_scaling_event(d, rss):
            await self.sync_scale(d, rss)
            return
        if (spec.get("strategy") or {}).get("type", "RollingUpdate") == "Recreate":
            await self.rollout_recreate(d, rss)
        else:
            await self.rollout_rolling(d, rss)

    # -- sync.go -----------------------------------------------------------------------------
    async def sync_status_only(self, d, rss):
        new_rs, old_rss = await self.get_all_replica_sets_and_sync_revision(d, rss, False)
        await self.sync_deployment_status([r for r in old_rss + [new_rs] if r is not None], new_rs, d)

    async def sync_scale(self, d, rss):
        """`sync`: scaling and status only (paused deployments, scaling events)."""
        new_rs, old_rss = await self.get_all_replica_sets_and_sync_revision(d, rss, False)
        await self.scale(d, new_rs, old_rss)
        if (d.get("spec") or {}).get("paused") and (d.get("spec") or {}).get("rollbackTo") is None:
            await self.cleanup_deployment(old_rss, d)
        await self.sync_deployment_status([r for r in old_rss + [new_rs] if r is not None], new_rs, d)

    async def is_scaling_event(self, d, rss):
        new_rs, old_rss = await self.get_all_replica_sets_and_sync_revision(d, rss, False)
        for rs in U.filter_active(old_rss + [new_rs]):
            desired = U.annotations_of(rs).get(U.DESIRED_REPLICAS)
            if desired is None:
                continue
            try:
                if int(desired) != U.replicas_of(d):
                    return True
            except ValueError:
                continue
        return False

    async def get_all_replica_sets_and_sync_revision(self, d, rss, create):
        _, all_old = U.find_old_replica_sets(d, rss)
        new_rs = await self.get_new_replica_set(d, rss, all_old, create)
        return new_rs, all_old

    async def get_new_replica_set(self, d, rss, old_rss, create):
        existing = U.find_new_replica_set(d, rss)
        max_old = max((U.revision_of(rs) for rs in old_rss), default=0)
        new_revision = str(max_old + 1)
        spec = d.get("spec") or {}
        if existing is not None:
            rs = m.fast_copy(existing)
            ann_changed = U.set_new_replica_set_annotations(d, rs, new_revision, True)
            mrs_changed = int((rs.get("spec") or {}).get("minReadySeconds") or 0) != int(spec.get("minReadySeconds") or 0)
            if ann_changed or mrs_changed:
                rs["spec"]["minReadySeconds"] = int(spec.get("minReadySeconds") or 0)
                return await self._update_rs(rs)
            needs = self._set_deployment_revision(d, U.annotations_of(rs).get(REVISION, ""))
            if U.has_progress_deadline(d) and U.get_condition(d.get("status"), "Progressing") is None:
                st = dict(d.get("status") or {})
                U.set_condition(st, U.new_condition("Progressing", "True", U.FOUND_NEW_RS,
                                                    f'Found new replica set "{m.name_of(rs)}"'))
                d["status"] = st
                needs = True
            if needs:
                await self._write_deployment(d)
            return rs
        if not create:
            return None
        tmpl = m.fast_copy(spec.get("template") or {})
        collisions = int((d.get("status") or {}).get("collisionCount") or 0)
        h = template_hash(spec.get("template") or {}, collisions)
        tmpl.setdefault("metadata", {}).setdefault("labels", {})[HASH_LABEL] = h
        sel = m.fast_copy(spec.get("selector") or {})
        sel.setdefault("matchLabels", {})[HASH_LABEL] = h
        labels = dict(tmpl["metadata"]["labels"])
        rs = {"apiVersion": "apps/v1", "kind": "ReplicaSet",
              "metadata": {"name": f"{m.name_of(d)}-{h}", "namespace": m.namespace_of(d), "labels": labels,
                           "ownerReferences": [m.owner_reference(d)]},
              "spec": {"replicas": 0, "minReadySeconds": int(spec.get("minReadySeconds") or 0),
                       "selector": sel, "template": tmpl}}
        all_rss = [r for r in old_rss]
        rs["spec"]["replicas"] = U.new_rs_new_replicas(d, all_rss, rs)
        U.set_new_replica_set_annotations(d, rs, new_revision, False)
        try:
            created = await self.client.create("replicasets", rs, m.namespace_of(d))
        except APIStatusError as e:
            if is_already_exists(e):
                cur = None
                try:
                    cur = await self.client.get("replicasets", m.name_of(rs), m.namespace_of(d))
                except APIStatusError:
                    pass
                if cur is not None and (controller_ref(cur) or {}).get("uid") == m.uid_of(d) and \
                        U.equal_ignore_hash((cur.get("spec") or {}).get("template"), spec.get("template")):
                    return cur       # our own RS from an earlier sync, not yet in the cache
                # a hash collision: bump the collision count and retry with another name
                st = dict(d.get("status") or {})
                st["collisionCount"] = collisions + 1
                d["status"] = st
                await self._write_status(d, st)
                raise
            if U.has_progress_deadline(d):
                st = dict(d.get("status") or {})
                U.set_condition(st, U.new_condition("Progressing", "False", U.FAILED_RS_CREATE,
                                                    f'Failed to create new replica set "{m.name_of(rs)}": {e}'))
                d["status"] = st
                await self._write_status(d, st)
            raise
        if U.replicas_of(created) > 0:
            self.recorder.event(d, "Normal", "ScalingReplicaSet",
                                f"Scaled up replica set {m.name_of(created)} to {U.replicas_of(created)}")
        needs = self._set_deployment_revision(d, new_revision)
        if U.has_progress_deadline(d):
            st = dict(d.get("status") or {})
            U.set_condition(st, U.new_condition("Progressing", "True", U.NEW_RS_CREATED,
                                                f'Created new replica set "{m.name_of(created)}"'))
            d["status"] = st
            needs = True
        if needs:
            await self._write_deployment(d)
        return created

    def _set_deployment_revision(self, d, revision):
        ann = d["metadata"].setdefault("annotations", {})
        if revision and ann.get(REVISION) != revision:
            ann[REVISION] = revision
            return True
        return False

    async def scale(self, d, new_rs, old_rss):
        """`scale` (sync.go:385): proportional scaling of every active ReplicaSet."""
        n = U.replicas_of(d)
        active_or_latest = U.find_active_or_latest(new_rs, old_rss)
        if active_or_latest is not None:
            if U.replicas_of(active_or_latest) == n:
                return
            await self.scale_replica_set_and_record_event(active_or_latest, n, d)
            return
        if U.is_saturated(d, new_rs):
            for old in U.filter_active(old_rss):
                await self.scale_replica_set_and_record_event(old, 0, d)
            return
        if not U.is_rolling(d):
            return
        all_rss = U.filter_active(old_rss + [new_rs])
        allowed = n + U.max_surge(d) if n > 0 else 0
        to_add = allowed - U.replica_count(all_rss)
        # largest first; ties: newer first when adding (ReplicaSetsBySizeNewer), older first when
        # removing (ReplicaSetsBySizeOlder)
        all_rss.sort(key=U.creation_key, reverse=to_add > 0)
        all_rss.sort(key=lambda r: -U.replicas_of(r))
        op = "up" if to_add > 0 else "down" if to_add < 0 else ""
        added = 0
        sizes = {}
        for rs in all_rss:
            if to_add != 0:
                p = U.get_proportion(rs, d, to_add, added)
                sizes[m.name_of(rs)] = U.replicas_of(rs) + p
                added += p
            else:
                sizes[m.name_of(rs)] = U.replicas_of(rs)
        if to_add != 0 and all_rss:
            name0 = m.name_of(all_rss[0])
            sizes[name0] = max(0, sizes[name0] + to_add - added)
        for rs in all_rss:
            await self.scale_replica_set(rs, sizes[m.name_of(rs)], d, op)

    async def scale_replica_set_and_record_event(self, rs, new_scale, d):
        if U.replicas_of(rs) == new_scale:
            return False, rs
        op = "up" if U.replicas_of(rs) < new_scale else "down"
        return await self.scale_replica_set(rs, new_scale, d, op)

    async def scale_replica_set(self, rs, new_scale, d, op):
        size_changed = U.replicas_of(rs) != new_scale
        desired, maxr = U.replicas_of(d), U.replicas_of(d) + U.max_surge(d)
        ann_changed = U.replicas_annotations_need_update(rs, desired, maxr)
        if not (size_changed or ann_changed):
            return False, rs
        rs = m.fast_copy(rs)
        rs.setdefault("spec", {})["replicas"] = new_scale
        U.set_replicas_annotations(rs, desired, maxr)
        rs = await self._update_rs(rs)
        if size_changed:
            self.recorder.event(d, "Normal", "ScalingReplicaSet",
                                f"Scaled {op} replica set {m.name_of(rs)} to {new_scale}")
        return True, rs

    async def _update_rs(self, rs):
        return await self.client.update("replicasets", rs, m.namespace_of(rs))

    async def cleanup_deployment(self, old_rss, d):
        limit = (d.get("spec") or {}).get("revisionHistoryLimit")
        if limit is None:
            return
        cleanable = sorted((rs for rs in old_rss if rs is not None and not rs["metadata"].get("deletionTimestamp")),
                           key=U.creation_key)
        diff = len(cleanable) - int(limit)
        for rs in cleanable[:max(0, diff)]:
            if U.status_of(rs, "replicas") != 0 or U.replicas_of(rs) != 0 or \
                    rs["metadata"].get("generation", 0) > (rs.get("status") or {}).get("observedGeneration", 0):
                continue
            try:
                await self.client.delete("replicasets", m.name_of(rs), m.namespace_of(rs))
            except APIStatusError as e:
                if not is_not_found(e):
                    raise

    def calculate_status(self, all_rss, new_rs, d):
        available = U.available_replica_count(all_rss)
        total = U.replica_count(all_rss)
        st = dict(d.get("status") or {})
        st.update({"observedGeneration": d["metadata"].get("generation", 1),
                   "replicas": U.actual_replica_count(all_rss),
                   "updatedReplicas": U.actual_replica_count([new_rs]) if new_rs is not None else 0,
                   "readyReplicas": U.ready_replica_count(all_rss),
                   "availableReplicas": available,
                   "unavailableReplicas": max(0, total - available)})
        st["conditions"] = [dict(c) for c in st.get("conditions") or ()]
        if available >= U.replicas_of(d) - U.max_unavailable(d):
            U.set_condition(st, U.new_condition("Available", "True", U.MIN_AVAILABLE,
                                                "Deployment has minimum availability."))
        else:
            U.set_condition(st, U.new_condition("Available", "False", U.MIN_UNAVAILABLE,
                                                "Deployment does not have minimum availability."))
        return st

    async def sync_deployment_status(self, all_rss, new_rs, d):
        st = self.calculate_status(all_rss, new_rs, d)
        if _status_equal(d.get("status"), st):
            return
        await self._write_status(d, st)

    # -- rolling.go --------------------------------------------------------------------------
    async def rollout_rolling(self, d, rss):
        new_rs, old_rss = await self.get_all_replica_sets_and_sync_revision(d, rss, True)
        all_rss = old_rss + [new_rs]
        if await self.reconcile_new_replica_set(all_rss, new_rs, d):
            await self.sync_rollout_status(all_rss, new_rs, d)
            return
        if await self.reconcile_old_replica_sets(all_rss, U.filter_active(old_rss), new_rs, d):
            await self.sync_rollout_status(all_rss, new_rs, d)
            return
        if U.deployment_complete(d, d.get("status") or {}):
            await self.cleanup_deployment(old_rss, d)
        await self.sync_rollout_status(all_rss, new_rs, d)

    async def reconcile_new_replica_set(self, all_rss, new_rs, d):
        n = U.replicas_of(d)
        if U.replicas_of(new_rs) == n:
            return False
        if U.replicas_of(new_rs) > n:
            scaled, _ = await self.scale_replica_set_and_record_event(new_rs, n, d)
            return scaled
        count = U.new_rs_new_replicas(d, all_rss, new_rs)
        scaled, _ = await self.scale_replica_set_and_record_event(new_rs, count, d)
        return scaled

    async def reconcile_old_replica_sets(self, all_rss, old_rss, new_rs, d):
        if U.replica_count(old_rss) == 0:
            return False
        all_pods = U.replica_count(all_rss)
        min_available = U.replicas_of(d) - U.max_unavailable(d)
        new_unavailable = U.replicas_of(new_rs) - U.status_of(new_rs, "availableReplicas")
        max_scaled_down = all_pods - min_available - new_unavailable
        if max_scaled_down <= 0:
            return False
        old_rss, cleaned = await self.cleanup_unhealthy_replicas(old_rss, d, max_scaled_down)
        scaled = await self.scale_down_old_replica_sets_for_rolling_update(old_rss + [new_rs], old_rss, d)
        return cleaned + scaled > 0

    async def cleanup_unhealthy_replicas(self, old_rss, d, max_cleanup):
        out, total = [], 0
        for rs in sorted(old_rss, key=U.creation_key):
            if total >= max_cleanup:
                out.append(rs)
                continue
            cur, avail = U.replicas_of(rs), U.status_of(rs, "availableReplicas")
            if cur == 0 or cur == avail:
                out.append(rs)
                continue
            down = min(max_cleanup - total, cur - avail)
            _, rs = await self.scale_replica_set_and_record_event(rs, cur - down, d)
            total += down
            out.append(rs)
        return out, total

    async def scale_down_old_replica_sets_for_rolling_update(self, all_rss, old_rss, d):
        min_available = U.replicas_of(d) - U.max_unavailable(d)
        available = U.available_replica_count(all_rss)
        if available <= min_available:
            return 0
        want = available - min_available
        total = 0
        for rs in sorted(old_rss, key=U.creation_key):
            if total >= want:
                break
            cur = U.replicas_of(rs)
            if cur == 0:
                continue
            down = min(cur, want - total)
            await self.scale_replica_set_and_record_event(rs, cur - down, d)
            total += down
        return total

    # -- recreate.go -------------------------------------------------------------------------
    async def rollout_recreate(self, d, rss):
        new_rs, old_rss = await self.get_all_replica_sets_and_sync_revision(d, rss, False)
        all_rss = [r for r in old_rss + [new_rs] if r is not None]
        if await self.scale_down_old_replica_sets_for_recreate(U.filter_active(old_rss), d):
            await self.sync_rollout_status(all_rss, new_rs, d)
            return
        if self.old_pods_running(new_rs, old_rss, self.pods_by_rs(rss)):
            await self.sync_rollout_status(all_rss, new_rs, d)
            return
        if new_rs is None:
            new_rs, old_rss = await self.get_all_replica_sets_and_sync_revision(d, rss, True)
            all_rss = old_rss + [new_rs]
        await self.scale_replica_set_and_record_event(new_rs, U.replicas_of(d), d)
        if U.deployment_complete(d, d.get("status") or {}):
            await self.cleanup_deployment(old_rss, d)
        await self.sync_rollout_status(all_rss, new_rs, d)

    async def scale_down_old_replica_sets_for_recreate(self, old_rss, d):
        scaled = False
        for i, rs in enumerate(old_rss):
            if U.replicas_of(rs) == 0:
                continue
            changed, new = await self.scale_replica_set_and_record_event(rs, 0, d)
            if changed:
                old_rss[i] = new
                scaled = True
        return scaled

    @staticmethod
    def old_pods_running(new_rs, old_rss, pods_by_rs):
        if U.actual_replica_count(old_rss) > 0:
            return True
        for uid, pods in pods_by_rs.items():
            if new_rs is not None and m.uid_of(new_rs) == uid:
                continue
            for p in pods:
                if (p.get("status") or {}).get("phase") in ("Failed", "Succeeded"):
                    continue
                return True
        return False

    # -- rollback.go -------------------------------------------------------------------------
    async def rollback(self, d, rss):
        new_rs, old_rss = await self.get_all_replica_sets_and_sync_revision(d, rss, True)
        all_rss = [r for r in old_rss + [new_rs] if r is not None]
        to = int(((d.get("spec") or {}).get("rollbackTo") or {}).get("revision") or 0)
        if to == 0:
            to = U.last_revision(all_rss)
            if to == 0:
                self.recorder.event(d, "Warning", "DeploymentRollbackRevisionNotFound",
                                    "Unable to find last revision.")
                await self._clear_rollback_to(d)
                return
        for rs in all_rss:
            if U.revision_of(rs) != to:
                continue
            tmpl = (rs.get("spec") or {}).get("template") or {}
            performed = False
            if not U.equal_ignore_hash(d["spec"].get("template"), tmpl):
                t = m.fast_copy(tmpl)
                ((t.get("metadata") or {}).get("labels") or {}).pop(HASH_LABEL, None)
                d["spec"]["template"] = t
                U.set_deployment_annotations_to(d, rs)
                performed = True
            else:
                self.recorder.event(d, "Warning", "DeploymentRollbackTemplateUnchanged",
                                    f'The rollback revision contains the same template as current deployment "{m.name_of(d)}"')
            await self._clear_rollback_to(d)
            if performed:
                self.recorder.event(d, "Normal", "DeploymentRollback",
                                    f"Rolled back deployment {m.name_of(d)} to revision {to}")
            return
        self.recorder.event(d, "Warning", "DeploymentRollbackRevisionNotFound",
                            "Unable to find the revision to rollback to.")
        await self._clear_rollback_to(d)

    async def _clear_rollback_to(self, d):
        d["spec"].pop("rollbackTo", None)
        await self.client.update("deployments", d, m.namespace_of(d))

    # -- progress.go -------------------------------------------------------------------------
    async def check_paused_conditions(self, d):
        if not U.has_progress_deadline(d):
            return d
        cond = U.get_condition(d.get("status"), "Progressing")
        if cond is not None and cond.get("reason") == U.TIMED_OUT:
            return d
        paused_exists = cond is not None and cond.get("reason") == U.PAUSED
        st = dict(d.get("status") or {})
        st["conditions"] = [dict(c) for c in st.get("conditions") or ()]
        if (d.get("spec") or {}).get("paused") and not paused_exists:
            U.set_condition(st, U.new_condition("Progressing", "Unknown", U.PAUSED, "Deployment is paused"))
        elif not (d.get("spec") or {}).get("paused") and paused_exists:
            U.set_condition(st, U.new_condition("Progressing", "Unknown", U.RESUMED, "Deployment is resumed"))
        else:
            return d
        d["status"] = st
        await self._write_status(d, st)
        return d

    def rollout_status(self, all_rss, new_rs, d):
        """The status `syncRolloutStatus` writes (pure; the table tests check it)."""
        st = self.calculate_status(all_rss, new_rs, d)
        if not U.has_progress_deadline(d):
            U.remove_condition(st, "Progressing")
        cur = U.get_condition(d.get("status"), "Progressing")
        complete = st["replicas"] == st["updatedReplicas"] and cur is not None and \
            cur.get("reason") == U.NEW_RS_AVAILABLE
        if U.has_progress_deadline(d) and not complete:
            if U.deployment_complete(d, st):
                msg = (f'ReplicaSet "{m.name_of(new_rs)}" has successfully progressed.' if new_rs is not None
                       else f'Deployment "{m.name_of(d)}" has successfully progressed.')
                U.set_condition(st, U.new_condition("Progressing", "True", U.NEW_RS_AVAILABLE, msg))
            elif U.deployment_progressing(d, st):
                msg = (f'ReplicaSet "{m.name_of(new_rs)}" is progressing.' if new_rs is not None
                       else f'Deployment "{m.name_of(d)}" is progressing.')
                cond = U.new_condition("Progressing", "True", U.REPLICA_SET_UPDATED, msg)
                if cur is not None and cur.get("status") == "True":
                    cond["lastTransitionTime"] = cur.get("lastTransitionTime")
                U.remove_condition(st, "Progressing")
                U.set_condition(st, cond)
            elif U.deployment_timed_out(d, st):
                msg = (f'ReplicaSet "{m.name_of(new_rs)}" has timed out progressing.' if new_rs is not None
                       else f'Deployment "{m.name_of(d)}" has timed out progressing.')
                U.set_condition(st, U.new_condition("Progressing", "False", U.TIMED_OUT, msg))
        failures = self.replica_failures(all_rss, new_rs)
        if failures:
            U.set_condition(st, failures[0])
        else:
            U.remove_condition(st, "ReplicaFailure")
        return st

    async def sync_rollout_status(self, all_rss, new_rs, d):
        all_rss = [r for r in all_rss if r is not None]
        st = self.rollout_status(all_rss, new_rs, d)
        if _status_equal(d.get("status"), st):
            after = self.requeue_stuck_deployment(d, st)
            if after == 0:
                self.queue.add_rate_limited(m.ns_name(d))
            elif after is not None:
                self.queue.add_after(m.ns_name(d), after + 1.0)
            return st
        d["status"] = st
        await self._write_status(d, st)
        return st

    @staticmethod
    def replica_failures(all_rss, new_rs):
        """`getReplicaFailures`: the new RS's ReplicaFailure condition first, then any other's."""
        ordered = ([new_rs] if new_rs is not None else []) + [r for r in all_rss if r is not new_rs]
        for rs in ordered:
            for c in (rs.get("status") or {}).get("conditions") or ():
                if c.get("type") == "ReplicaFailure":
                    return [{"type": "ReplicaFailure", "status": c.get("status"), "reason": c.get("reason"),
                             "message": c.get("message"), "lastUpdateTime": c.get("lastTransitionTime"),
                             "lastTransitionTime": c.get("lastTransitionTime")}]
        return []

    def requeue_stuck_deployment(self, d, new_status):
        """Seconds until this deployment's progress deadline passes (0 = now), None = never."""
        cur = U.get_condition(d.get("status"), "Progressing")
        if not U.has_progress_deadline(d) or cur is None:
            return None
        if U.deployment_complete(d, new_status) or cur.get("reason") == U.TIMED_OUT:
            return None
        last = parse_rfc3339(cur.get("lastUpdateTime"))
        if last is None:
            return None
        after = last + int(d["spec"]["progressDeadlineSeconds"]) - U.now_fn()
        return 0 if after < 1 else after

    # -- writes ------------------------------------------------------------------------------
    async def _write_status(self, d, st):
        d["status"] = st
        try:
            await self.client.patch("deployments", m.name_of(d), {"status": st}, m.namespace_of(d),
                                    "merge", "status")
        except APIStatusError as e:
            if not is_not_found(e):
                raise

    async def _write_deployment(self, d):
        """The revision annotation (metadata) and, through the status subresource, conditions."""
        try:
            await self.client.patch("deployments", m.name_of(d),
                                    {"metadata": {"annotations": {REVISION: U.annotations_of(d).get(REVISION)}}},
                                    m.namespace_of(d))
        except APIStatusError as e:
            if not is_not_found(e):
                raise
        if d.get("status"):
            await self._write_status(d, d["status"])


def _status_equal(a, b):
    """Status equality ignoring condition timestamps' churn (`reflect.DeepEqual` on the rest)."""
    a, b = dict(a or {}), dict(b or {})
    ca, cb = a.pop("conditions", None) or [], b.pop("conditions", None) or []
    if {k: v for k, v in a.items() if v not in (None, 0)} != {k: v for k, v in b.items() if v not in (None, 0)}:
        return False
    key = lambda c: (c.get("type"), c.get("status"), c.get("reason"), c.get("message"))   # noqa: E731
    return sorted(map(key, ca)) == sorted(map(key, cb))


__all__ = ["DeploymentController", "template_hash", "HASH_LABEL", "REVISION", "now_rfc3339"]
