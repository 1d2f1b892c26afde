"""StatefulSet controller.

Parity: `pkg/controller/statefulset/`
  * identity & storage (`stateful_set_utils.go`): pod `<set>-<ordinal>` with the
    `statefulset.kubernetes.io/pod-name` label, hostname = pod name, subdomain = serviceName; one
    PersistentVolumeClaim per volumeClaimTemplate per ordinal named `<claim>-<set>-<ordinal>`
    (`getPersistentVolumeClaimName`, `:144`), labelled with the selector's matchLabels and owned by
    nobody (claims outlive the set), mounted as the pod volume named after the template
    (`updateStorage`, `:180`); a pod whose identity or volumes drifted is repaired in place
    (`UpdateStatefulPod`);
  * pod control (`stateful_pod_control.go:179 createPersistentVolumeClaims`): claims are created
    before their pod;
  * revisions (`stateful_set_control.go:182-239 getStatefulSetRevisions`): the update revision is
    the ControllerRevision of the current template (reused, or re-numbered on a rollback); the
    current revision is the one `status.currentRevision` names; new pods below the partition get
    the current revision's template (`newVersionedStatefulSetPod`);
  * the update loop (`updateStatefulSet`, `:240-495`): OrderedReady creates one missing ordinal at
    a time and only after every lower ordinal is Running and Ready, recreates Failed pods, scales
    down from the highest ordinal, then — RollingUpdate — deletes the highest-ordinal pod at or
    above `rollingUpdate.partition` that is not on the update revision, one at a time, waiting
    for health; OnDelete leaves existing pods alone; Parallel lifts the ordering constraints;
  * status (`updateStatefulSetStatus`, `completeRollingUpdate`, `inconsistentStatus`): replicas /
    ready / current / updated counts; when every replica is updated and ready the current
    revision rolls forward to the update revision;
  * history (`truncateHistory`): revisions that are neither current, update, nor any pod's are
    deleted oldest first beyond `revisionHistoryLimit`;
  * adoption (`stateful_set.go getPodsForStatefulSet` / ControllerRefManager): orphan pods that
    match the selector and carry the set's name + ordinal are adopted, owned pods that stop
    matching are released.
"""
from __future__ import annotations

import re

from ..api import meta as m
from ..api.labels import label_selector_as_selector
from ..client.rest import APIStatusError, is_already_exists, is_conflict, is_not_found
from .base import Controller, controller_ref, pod_from_template, pod_is_ready, split_key
from .history import ensure_revision, revisions_of, truncate_history

POD_NAME_LABEL = "statefulset.kubernetes.io/pod-name"
REVISION_LABEL = "controller-revision-hash"
_ORDINAL = re.compile(r"^(.*)-([0-9]+)$")


# -- stateful_set_utils.go ------------------------------------------------------------------
def parent_and_ordinal(pod):
    mt = _ORDINAL.match(m.name_of(pod))
    if not mt:
        return "", -1
    try:
        return mt.group(1), int(mt.group(2))
    except ValueError:
        return "", -1


def ordinal_of(pod):
    return parent_and_ordinal(pod)[1]


def pod_name(ss, ordinal):
    return f"{m.name_of(ss)}-{ordinal}"


def claim_name(ss, claim, ordinal):
    return f"{m.name_of(claim)}-{m.name_of(ss)}-{ordinal}"


def is_member_of(ss, pod):
    return parent_and_ordinal(pod)[0] == m.name_of(ss)


def identity_matches(ss, pod):
    parent, ordinal = parent_and_ordinal(pod)
    return (ordinal >= 0 and parent == m.name_of(ss) and m.name_of(pod) == pod_name(ss, ordinal)
            and m.namespace_of(pod) == m.namespace_of(ss)
            and (pod["metadata"].get("labels") or {}).get(POD_NAME_LABEL) == m.name_of(pod))


def _claim_templates(ss):
    return (ss.get("spec") or {}).get("volumeClaimTemplates") or ()


def storage_matches(ss, pod):
    ordinal = ordinal_of(pod)
    if ordinal < 0:
        return False
    vols = {v.get("name"): v for v in (pod.get("spec") or {}).get("volumes") or ()}
    for claim in _claim_templates(ss):
        v = vols.get(m.name_of(claim))
        if v is None or (v.get("persistentVolumeClaim") or {}).get("claimName") != claim_name(ss, claim, ordinal):
            return False
    return True


def persistent_volume_claims(ss, ordinal):
    """{template name: the claim object for this ordinal} (`getPersistentVolumeClaims`)."""
    match = dict(((ss.get("spec") or {}).get("selector") or {}).get("matchLabels") or {})
    out = {}
    for tmpl in _claim_templates(ss):
        claim = m.fast_copy(tmpl)
        md = claim.setdefault("metadata", {})
        md["name"] = claim_name(ss, tmpl, ordinal)
        md["namespace"] = m.namespace_of(ss)
        md["labels"] = dict(match)
        for k in ("uid", "resourceVersion", "creationTimestamp", "selfLink"):
            md.pop(k, None)
        claim.pop("status", None)
        claim["apiVersion"], claim["kind"] = "v1", "PersistentVolumeClaim"
        out[m.name_of(tmpl)] = claim
    return out


def update_storage(ss, pod):
    claims = persistent_volume_claims(ss, ordinal_of(pod))
    spec = pod.setdefault("spec", {})
    vols = [{"name": n, "persistentVolumeClaim": {"claimName": c["metadata"]["name"]}} for n, c in claims.items()]
    vols += [v for v in spec.get("volumes") or () if v.get("name") not in claims]
    spec["volumes"] = vols


def update_identity(ss, pod):
    md = pod["metadata"]
    md["name"] = pod_name(ss, ordinal_of(pod))
    md["namespace"] = m.namespace_of(ss)
    md.setdefault("labels", {})[POD_NAME_LABEL] = md["name"]


def is_running_and_ready(pod):
    return (pod.get("status") or {}).get("phase") == "Running" and pod_is_ready(pod)


def is_failed(pod):
    return (pod.get("status") or {}).get("phase") == "Failed"


def is_terminating(pod):
    return bool(pod["metadata"].get("deletionTimestamp"))


def is_healthy(pod):
    return is_running_and_ready(pod) and not is_terminating(pod)


def pod_revision(pod):
    return (pod["metadata"].get("labels") or {}).get(REVISION_LABEL, "")


def apply_revision(ss, rev):
    """`ApplyRevision`: the set with the revision's pod template."""
    out = dict(ss)
    out["spec"] = dict(ss.get("spec") or {})
    tmpl = (((rev or {}).get("data") or {}).get("spec") or {}).get("template")
    if tmpl is not None:
        out["spec"]["template"] = tmpl
    return out


def new_stateful_pod(ss, ordinal):
    spec = ss.get("spec") or {}
    pod = pod_from_template(spec.get("template"), ss, "", m.namespace_of(ss))
    pod["metadata"].pop("generateName", None)
    pod["metadata"]["name"] = pod_name(ss, ordinal)
    update_identity(ss, pod)
    pod["spec"]["hostname"] = pod["metadata"]["name"]
    if spec.get("serviceName"):
        pod["spec"]["subdomain"] = spec["serviceName"]
    update_storage(ss, pod)
    return pod


def new_versioned_pod(current_set, update_set, current_rev, update_rev, ordinal):
    """`newVersionedStatefulSetPod`: ordinals below the partition stay on the current revision."""
    us = (current_set.get("spec") or {}).get("updateStrategy") or {}
    ru = us.get("rollingUpdate")
    rolling = us.get("type", "RollingUpdate") == "RollingUpdate"
    if (rolling and ru is None and ordinal < int((current_set.get("status") or {}).get("currentReplicas") or 0)) or \
            (ru is not None and ordinal < int(ru.get("partition") or 0)):
        pod = new_stateful_pod(current_set, ordinal)
        pod["metadata"]["labels"][REVISION_LABEL] = current_rev
        return pod
    pod = new_stateful_pod(update_set, ordinal)
    pod["metadata"]["labels"][REVISION_LABEL] = update_rev
    return pod


def complete_rolling_update(ss, status):
    us = (ss.get("spec") or {}).get("updateStrategy") or {}
    if us.get("type", "RollingUpdate") == "RollingUpdate" and \
            status["updatedReplicas"] == status["replicas"] and status["readyReplicas"] == status["replicas"]:
        status["currentReplicas"] = status["updatedReplicas"]
        status["currentRevision"] = status["updateRevision"]


STATUS_FIELDS = ("replicas", "readyReplicas", "currentReplicas", "updatedReplicas", "currentRevision",
                 "updateRevision")


def inconsistent_status(ss, status):
    cur = ss.get("status") or {}
    if cur.get("observedGeneration") is None or status["observedGeneration"] > cur["observedGeneration"]:
        return True
    return any((cur.get(k) or (0 if k.endswith("Replicas") or k == "replicas" else "")) != status[k]
               for k in STATUS_FIELDS)


class StatefulSetController(Controller):
    name = "statefulset"
    workers = 2

    def setup(self):
        self.ss_inf = self.factory.get("statefulsets")
        self.pod_inf = self.factory.get("pods")
        self.rev_inf = self.factory.get("controllerrevisions")
        self.pvc_inf = self.factory.get("persistentvolumeclaims")
        self.ss_inf.add_handler(self.enqueue, lambda o, n: self.enqueue(n), None)
        self.pod_inf.add_handler(self._pod, lambda o, n: self._pod_update(o, n), self._pod)
        self.rev_inf.add_handler(None, None, self._rev_deleted)

    def _sets_for_orphan(self, pod):
        labels = pod["metadata"].get("labels") or {}
        for ss in self.ss_inf.list():
            if m.namespace_of(ss) != m.namespace_of(pod):
                continue
            sel = label_selector_as_selector((ss.get("spec") or {}).get("selector"))
            if not sel.empty() and sel.matches(labels):
                yield ss

    def _pod(self, pod):
        ref = controller_ref(pod)
        if ref is not None:
            if ref.get("kind") == "StatefulSet":
                self.enqueue(f"{m.namespace_of(pod)}/{ref['name']}")
            return
        for ss in self._sets_for_orphan(pod):
            self.enqueue(ss)

    def _pod_update(self, old, new):
        self._pod(new)
        o, n = controller_ref(old), controller_ref(new)
        if o is not None and (n is None or o.get("uid") != n.get("uid")) and o.get("kind") == "StatefulSet":
            self.enqueue(f"{m.namespace_of(old)}/{o['name']}")

    def _rev_deleted(self, rev):
        ref = controller_ref(rev)
        if ref and ref.get("kind") == "StatefulSet":
            self.enqueue(f"{m.namespace_of(rev)}/{ref['name']}")

    # -- pod claiming (ControllerRefManager) --------------------------------------------------
    async def claim_pods(self, ss):
        ns, uid = m.namespace_of(ss), m.uid_of(ss)
        sel = label_selector_as_selector((ss.get("spec") or {}).get("selector"))
        out = []
        for p in self.pod_inf.list():
            if m.namespace_of(p) != ns:
                continue
            ref = controller_ref(p)
            labels = p["metadata"].get("labels") or {}
            matches = not sel.empty() and sel.matches(labels) and is_member_of(ss, p)
            if ref is not None:
                if ref.get("uid") != uid:
                    continue
                if matches:
                    out.append(p)
                elif not is_terminating(p):
                    await self._release(p, uid)
                continue
            if matches and not is_terminating(p) and not ss["metadata"].get("deletionTimestamp"):
                adopted = await self._adopt(ss, p)
                if adopted is not None:
                    out.append(adopted)
        return out

    async def _adopt(self, ss, pod):
        refs = list(pod["metadata"].get("ownerReferences") or ()) + [m.owner_reference(ss)]
        try:
            return await self.client.patch("pods", m.name_of(pod),
                                           {"metadata": {"ownerReferences": refs, "uid": m.uid_of(pod)}},
                                           m.namespace_of(pod))
        except APIStatusError as e:
            if is_not_found(e):
                return None
            raise

    async def _release(self, pod, uid):
        refs = [r for r in pod["metadata"].get("ownerReferences") or () if r.get("uid") != uid]
        try:
            await self.client.patch("pods", m.name_of(pod), {"metadata": {"ownerReferences": refs or None}},
                                    m.namespace_of(pod))
        except APIStatusError as e:
            if not is_not_found(e):
                raise

    # -- pod control (stateful_pod_control.go) -------------------------------------------
    async def create_claims(self, ss, ordinal):
        errs = []
        for claim in persistent_volume_claims(ss, ordinal).values():
            if self.pvc_inf.get(f"{m.namespace_of(ss)}/{claim['metadata']['name']}") is not None:
                continue
            try:
                await self.client.create("persistentvolumeclaims", claim, m.namespace_of(ss))
                self.recorder.event(ss, "Normal", "SuccessfulCreate",
                                    f"create Claim {claim['metadata']['name']} Pod {pod_name(ss, ordinal)} "
                                    f"in StatefulSet {m.name_of(ss)} success")
            except APIStatusError as e:
                if not is_already_exists(e):
                    self.recorder.event(ss, "Warning", "FailedCreate",
                                        f"create Claim {claim['metadata']['name']} for Pod {pod_name(ss, ordinal)} "
                                        f"in StatefulSet {m.name_of(ss)} failed error: {e}")
                    errs.append(e)
        if errs:
            raise errs[0]

    async def create_pod(self, ss, pod):
        await self.create_claims(ss, ordinal_of(pod))
        try:
            await self.client.create("pods", pod, m.namespace_of(ss))
        except APIStatusError as e:
            if not is_already_exists(e):
                self._pod_event("create", ss, pod, e)
            raise
        self._pod_event("create", ss, pod)

    async def update_pod(self, ss, pod):
        """`UpdateStatefulPod`: repair identity and storage, retrying on conflicts."""
        for _ in range(5):
            pod = m.fast_copy(pod)
            consistent = True
            if not identity_matches(ss, pod):
                update_identity(ss, pod)
                consistent = False
            if not storage_matches(ss, pod):
                update_storage(ss, pod)
                consistent = False
                await self.create_claims(ss, ordinal_of(pod))
            if consistent:
                return
            try:
                await self.client.update("pods", pod, m.namespace_of(ss))
                self._pod_event("update", ss, pod)
                return
            except APIStatusError as e:
                if not is_conflict(e):
                    self._pod_event("update", ss, pod, e)
                    raise
                pod = await self.client.get("pods", m.name_of(pod), m.namespace_of(pod))
        raise RuntimeError(f"updating pod {m.name_of(pod)}: too many conflicts")

    async def delete_pod(self, ss, pod):
        try:
            await self.client.delete("pods", m.name_of(pod), m.namespace_of(pod))
        except APIStatusError as e:
            if is_not_found(e):
                return
            self._pod_event("delete", ss, pod, e)
            raise
        self._pod_event("delete", ss, pod)

    def _pod_event(self, verb, ss, pod, err=None):
        if err is None:
            self.recorder.event(ss, "Normal", f"Successful{verb.title()}",
                                f"{verb} Pod {m.name_of(pod)} in StatefulSet {m.name_of(ss)} successful")
        else:
            self.recorder.event(ss, "Warning", f"Failed{verb.title()}",
                                f"{verb} Pod {m.name_of(pod)} in StatefulSet {m.name_of(ss)} failed error: {err}")

    # -- the control loop -----------------------------------------------------------------
    async def sync(self, key):
        ss = self.ss_inf.get(key)
        if ss is None:
            return
        pods = await self.claim_pods(ss)
        spec = ss.get("spec") or {}
        revisions = revisions_of(self.rev_inf.list(), m.uid_of(ss))
        update_rev = await ensure_revision(self.client, ss, "StatefulSet", spec.get("template") or {}, revisions,
                                           limit=None)
        cur_name = (ss.get("status") or {}).get("currentRevision")
        current_rev = next((r for r in revisions if m.name_of(r) == cur_name), None) or update_rev
        status = await self.update_stateful_set(ss, current_rev, update_rev, pods)
        complete_rolling_update(ss, status)
        if inconsistent_status(ss, status):
            ns, name = split_key(key)
            try:
                await self.client.patch("statefulsets", name, {"status": status}, ns, "merge", "status")
            except APIStatusError as e:
                if not is_not_found(e):
                    raise
        live = {m.name_of(current_rev), m.name_of(update_rev)} | {pod_revision(p) for p in pods}
        await truncate_history(self.client, revisions_of(self.rev_inf.list(), m.uid_of(ss)) or revisions, live,
                               int(spec.get("revisionHistoryLimit", 10)))

    async def update_stateful_set(self, ss, current_rev, update_rev, pods):
        current_set = apply_revision(ss, current_rev)
        update_set = apply_revision(ss, update_rev)
        cur_name, upd_name = m.name_of(current_rev), m.name_of(update_rev)
        spec = ss.get("spec") or {}
        status = {"observedGeneration": ss["metadata"].get("generation", 1), "replicas": 0, "readyReplicas": 0,
                  "currentReplicas": 0, "updatedReplicas": 0, "currentRevision": cur_name,
                  "updateRevision": upd_name,
                  "collisionCount": int((ss.get("status") or {}).get("collisionCount") or 0)}
        n = int(spec.get("replicas", 1))
        replicas = [None] * n
        created = set()
        condemned = []

        def count(pod, d):
            rev = pod_revision(pod)
            if rev == cur_name:
                status["currentReplicas"] += d
            elif rev == upd_name:
                status["updatedReplicas"] += d

        for p in pods:
            status["replicas"] += 1
            if is_running_and_ready(p):
                status["readyReplicas"] += 1
            if not is_terminating(p):
                count(p, 1)
            o = ordinal_of(p)
            if 0 <= o < n:
                replicas[o] = p
                created.add(o)
            elif o >= n:
                condemned.append(p)
        for o in range(n):
            if replicas[o] is None:
                replicas[o] = new_versioned_pod(current_set, update_set, cur_name, upd_name, o)
        condemned.sort(key=ordinal_of)
        unhealthy = [p for p in replicas + condemned if not is_healthy(p)]    # placeholders included
        first_unhealthy = min(unhealthy, key=ordinal_of) if unhealthy else None
        if ss["metadata"].get("deletionTimestamp"):
            return status
        monotonic = spec.get("podManagementPolicy") != "Parallel"

        for o in range(n):
            pod = replicas[o]
            if o in created and is_failed(pod):
                await self.delete_pod(ss, pod)
                count(pod, -1)
                status["replicas"] -= 1
                created.discard(o)
                pod = replicas[o] = new_versioned_pod(current_set, update_set, cur_name, upd_name, o)
            if o not in created:
                await self.create_pod(ss, pod)
                status["replicas"] += 1
                count(pod, 1)
                if monotonic:
                    return status
                continue
            if is_terminating(pod) and monotonic:
                return status
            if not is_running_and_ready(pod) and monotonic:
                return status
            if identity_matches(ss, pod) and storage_matches(ss, pod):
                continue
            await self.update_pod(update_set, pod)

        for pod in reversed(condemned):
            if is_terminating(pod):
                if monotonic:
                    return status
                continue
            if not is_running_and_ready(pod) and monotonic and pod is not first_unhealthy:
                return status
            await self.delete_pod(ss, pod)
            count(pod, -1)
            if monotonic:
                return status

        us = spec.get("updateStrategy") or {}
        if us.get("type", "RollingUpdate") == "OnDelete":
            return status
        update_min = int((us.get("rollingUpdate") or {}).get("partition") or 0)
        for o in range(n - 1, update_min - 1, -1):
            pod = replicas[o]
            if pod_revision(pod) != upd_name and not is_terminating(pod):
                await self.delete_pod(ss, pod)
                status["currentReplicas"] -= 1
                return status
            if not is_healthy(pod):
                return status
        return status
