"""Deployment helpers: replica arithmetic, annotations, conditions, progress predicates.

Parity: `pkg/controller/deployment/util/deployment_util.go` — revision / desired-replicas /
max-replicas annotations (`:50-60`) and the annotation copy rules (`SetNewReplicaSetAnnotations`
`:245`, `annotationsToSkip` `:296`); `ResolveFenceposts`, `MaxSurge`, `MaxUnavailable`;
`NewRSNewReplicas`; proportional scaling (`GetProportion` `:453`, `getReplicaSetFraction`
`:475`); `FindActiveOrLatest` `:356`, `FindNewReplicaSet` `:658` / `EqualIgnoreHash` `:638`,
`IsSaturated` `:910`; condition helpers and the progress predicates `DeploymentComplete`,
`DeploymentProgressing`, `DeploymentTimedOut` (`:836-905`). Objects are plain dicts.
"""
from __future__ import annotations

import hashlib
import json
import math
import re
import time

from ..api import meta as m
from ..api.meta import now_rfc3339, parse_rfc3339

REVISION = "deployment.kubernetes.io/revision"
REVISION_HISTORY = "deployment.kubernetes.io/revision-history"
DESIRED_REPLICAS = "deployment.kubernetes.io/desired-replicas"
MAX_REPLICAS = "deployment.kubernetes.io/max-replicas"
LAST_APPLIED = "kubectl.kubernetes.io/last-applied-configuration"
HASH_LABEL = "pod-template-hash"
MAX_INT32 = 2 ** 31 - 1

# condition reasons (deployment_util.go:70-93)
REPLICA_SET_UPDATED = "ReplicaSetUpdated"
FAILED_RS_CREATE = "ReplicaSetCreateError"
NEW_RS_CREATED = "NewReplicaSetCreated"
FOUND_NEW_RS = "FoundNewReplicaSet"
NEW_RS_AVAILABLE = "NewReplicaSetAvailable"
TIMED_OUT = "ProgressDeadlineExceeded"
PAUSED = "DeploymentPaused"
RESUMED = "DeploymentResumed"
MIN_AVAILABLE = "MinimumReplicasAvailable"
MIN_UNAVAILABLE = "MinimumReplicasUnavailable"

_SKIP = {LAST_APPLIED, REVISION, REVISION_HISTORY, DESIRED_REPLICAS, MAX_REPLICAS}

# tests replace this to pin "now" (the reference's `nowFn`)
now_fn = time.time


def replicas_of(obj) -> int:
    v = (obj.get("spec") or {}).get("replicas")
    return 1 if v is None and obj.get("kind") == "Deployment" else int(v or 0)


def status_of(obj, field) -> int:
    return int((obj.get("status") or {}).get(field) or 0)


def annotations_of(obj):
    return (obj.get("metadata") or {}).get("annotations") or {}


def revision_of(obj) -> int:
    try:
        return int(annotations_of(obj).get(REVISION) or 0)
    except ValueError:
        return 0


# -- int-or-percent (intstr.GetValueFromIntOrPercent) -----------------------------------------
_PCT = re.compile(r"^(\d+)%$")


def value_from_int_or_percent(v, total, round_up):
    if v is None:
        return 0
    if isinstance(v, bool):
        raise ValueError(f"invalid value {v!r}")
    if isinstance(v, int):
        return v
    s = str(v)
    if s.isdigit():
        return int(s)
    mt = _PCT.match(s)
    if not mt:
        raise ValueError(f"invalid value for IntOrString: invalid value {s!r}")
    x = int(mt.group(1)) * total / 100.0
    return int(math.ceil(x) if round_up else math.floor(x))


def is_rolling(d):
    return ((d.get("spec") or {}).get("strategy") or {}).get("type", "RollingUpdate") == "RollingUpdate"


def _rolling(d):
    return ((d.get("spec") or {}).get("strategy") or {}).get("rollingUpdate") or {}


def resolve_fenceposts(max_surge, max_unavailable, desired):
    """-> (surge, unavailable); both 0 would deadlock a rollout, so unavailable becomes 1."""
    surge = value_from_int_or_percent(max_surge if max_surge is not None else 0, desired, True)
    unavail = value_from_int_or_percent(max_unavailable if max_unavailable is not None else 0, desired, False)
    if surge == 0 and unavail == 0:
        unavail = 1
    return surge, unavail


def max_surge(d):
    if not is_rolling(d):
        return 0
    ru = _rolling(d)
    return resolve_fenceposts(ru.get("maxSurge"), ru.get("maxUnavailable"), replicas_of(d))[0]


def max_unavailable(d):
    n = replicas_of(d)
    if not is_rolling(d) or n == 0:
        return 0
    ru = _rolling(d)
    return min(resolve_fenceposts(ru.get("maxSurge"), ru.get("maxUnavailable"), n)[1], n)


# -- replica set sets -----------------------------------------------------------------------
def creation_key(rs):
    return (parse_rfc3339((rs.get("metadata") or {}).get("creationTimestamp")) or 0.0, m.name_of(rs))


def filter_active(rss):
    return [rs for rs in rss if rs is not None and replicas_of(rs) > 0]


def replica_count(rss):
    return sum(replicas_of(rs) for rs in rss if rs is not None)


def actual_replica_count(rss):
    return sum(status_of(rs, "replicas") for rs in rss if rs is not None)


def ready_replica_count(rss):
    return sum(status_of(rs, "readyReplicas") for rs in rss if rs is not None)


def available_replica_count(rss):
    return sum(status_of(rs, "availableReplicas") for rs in rss if rs is not None)


def _strip_hash(tmpl):
    t = m.fast_copy(tmpl or {})
    labels = (t.get("metadata") or {}).get("labels")
    if labels is not None:
        labels.pop(HASH_LABEL, None)
        if not labels:
            t["metadata"].pop("labels")
    md = t.get("metadata")
    if md is not None and not md:
        t.pop("metadata")
    return t


def equal_ignore_hash(t1, t2):
    return _strip_hash(t1) == _strip_hash(t2)


def find_new_replica_set(d, rss):
    """The oldest RS whose template equals the deployment's, ignoring the hash label."""
    tmpl = (d.get("spec") or {}).get("template") or {}
    for rs in sorted(rss, key=creation_key):
        if equal_ignore_hash((rs.get("spec") or {}).get("template"), tmpl):
            return rs
    return None


def find_old_replica_sets(d, rss):
    """-> (old RSs with pods, all old RSs)."""
    new = find_new_replica_set(d, rss)
    old = [rs for rs in rss if rs is not new]
    return [rs for rs in old if replicas_of(rs) > 0], old


def find_active_or_latest(new_rs, old_rss):
    if new_rs is None and not old_rss:
        return None
    old_sorted = sorted(old_rss, key=creation_key, reverse=True)
    active = filter_active(old_sorted + [new_rs])
    if not active:
        return new_rs if new_rs is not None else old_sorted[0]
    if len(active) == 1:
        return active[0]
    return None


def is_saturated(d, rs):
    if rs is None:
        return False
    try:
        desired = int(annotations_of(rs).get(DESIRED_REPLICAS, ""))
    except ValueError:
        return False
    n = replicas_of(d)
    return replicas_of(rs) == n and desired == n and status_of(rs, "availableReplicas") == n


def last_revision(rss):
    """The second-highest revision (what a rollback to revision 0 restores)."""
    top = sec = 0
    for rs in rss:
        v = revision_of(rs)
        if v >= top:
            top, sec = v, top
        elif v > sec:
            sec = v
    return sec


def new_rs_new_replicas(d, all_rss, new_rs):
    """`NewRSNewReplicas`: the new RS's size this step (RollingUpdate: bounded by maxSurge)."""
    n = replicas_of(d)
    if not is_rolling(d):
        return n
    surge = value_from_int_or_percent(_rolling(d).get("maxSurge", 0) or 0, n, True)
    current = replica_count(all_rss)
    max_total = n + surge
    if current >= max_total:
        return replicas_of(new_rs)
    return replicas_of(new_rs) + min(max_total - current, n - replicas_of(new_rs))


# -- annotations ----------------------------------------------------------------------------
def set_replicas_annotations(rs, desired, max_replicas):
    ann = rs.setdefault("metadata", {}).setdefault("annotations", {})
    changed = False
    for k, v in ((DESIRED_REPLICAS, str(desired)), (MAX_REPLICAS, str(max_replicas))):
        if ann.get(k) != v:
            ann[k] = v
            changed = True
    return changed


def replicas_annotations_need_update(rs, desired, max_replicas):
    ann = annotations_of(rs)
    return ann.get(DESIRED_REPLICAS) != str(desired) or ann.get(MAX_REPLICAS) != str(max_replicas)


def copy_deployment_annotations_to_rs(d, rs):
    ann = rs.setdefault("metadata", {}).setdefault("annotations", {})
    changed = False
    for k, v in annotations_of(d).items():
        if k in _SKIP or ann.get(k) == v:
            continue
        ann[k] = v
        changed = True
    return changed


def set_new_replica_set_annotations(d, rs, new_revision, exists):
    changed = copy_deployment_annotations_to_rs(d, rs)
    ann = rs["metadata"].setdefault("annotations", {})
    had = REVISION in ann
    old = ann.get(REVISION, "")
    try:
        old_i = int(old) if old else 0
    except ValueError:
        return False
    if old_i < int(new_revision):
        ann[REVISION] = str(new_revision)
        changed = True
    if had and changed:
        hist = ann.get(REVISION_HISTORY, "")
        ann[REVISION_HISTORY] = f"{hist},{old}" if hist else old
    if not exists and set_replicas_annotations(rs, replicas_of(d), replicas_of(d) + max_surge(d)):
        changed = True
    return changed


def set_deployment_annotations_to(d, rollback_rs):
    """`SetDeploymentAnnotationsTo`: the deployment takes the rolled-back RS's annotations."""
    keep = {k: v for k, v in annotations_of(d).items() if k in _SKIP}
    new = {k: v for k, v in annotations_of(rollback_rs).items() if k not in _SKIP}
    d["metadata"]["annotations"] = {**new, **keep}


# -- proportional scaling -------------------------------------------------------------------
def _max_replicas_annotation(rs):
    try:
        return int(annotations_of(rs)[MAX_REPLICAS])
    except (KeyError, ValueError):
        return None


def replica_set_fraction(rs, d):
    n = replicas_of(d)
    if n == 0:
        return -replicas_of(rs)
    deployment_replicas = n + max_surge(d)
    annotated = _max_replicas_annotation(rs)
    if annotated is None:
        annotated = status_of(d, "replicas")      # the deployment's size before the scaling event
    if not annotated:
        return 0
    new_size = replicas_of(rs) * deployment_replicas / annotated
    return int(math.floor(new_size + 0.5)) - replicas_of(rs)   # Go's math.Round: half away from zero


def get_proportion(rs, d, to_add, added):
    if rs is None or replicas_of(rs) == 0 or to_add == 0 or to_add == added:
        return 0
    frac = replica_set_fraction(rs, d)
    allowed = to_add - added
    return min(frac, allowed) if to_add > 0 else max(frac, allowed)


# -- conditions -----------------------------------------------------------------------------
def new_condition(ctype, status, reason, message, now=None):
    t = now or now_rfc3339(now_fn())
    return {"type": ctype, "status": status, "lastUpdateTime": t, "lastTransitionTime": t,
            "reason": reason, "message": message}


def get_condition(status, ctype):
    for c in (status or {}).get("conditions") or ():
        if c.get("type") == ctype:
            return c
    return None


def set_condition(status, cond):
    """`SetDeploymentCondition`: same status and reason -> keep the existing one; same status ->
    keep its lastTransitionTime."""
    cur = get_condition(status, cond["type"])
    if cur is not None and cur.get("status") == cond["status"] and cur.get("reason") == cond["reason"]:
        return
    if cur is not None and cur.get("status") == cond["status"]:
        cond = dict(cond, lastTransitionTime=cur.get("lastTransitionTime"))
    status["conditions"] = [c for c in status.get("conditions") or () if c.get("type") != cond["type"]] + [cond]


def remove_condition(status, ctype):
    status["conditions"] = [c for c in status.get("conditions") or () if c.get("type") != ctype]


def has_progress_deadline(d):
    pds = (d.get("spec") or {}).get("progressDeadlineSeconds")
    return pds is not None and int(pds) != MAX_INT32


def deployment_complete(d, new_status):
    n = replicas_of(d)
    return (int(new_status.get("updatedReplicas") or 0) == n and int(new_status.get("replicas") or 0) == n and
            int(new_status.get("availableReplicas") or 0) == n and
            int(new_status.get("observedGeneration") or 0) >= int((d.get("metadata") or {}).get("generation") or 0))


def deployment_progressing(d, new_status):
    old = d.get("status") or {}
    old_old = int(old.get("replicas") or 0) - int(old.get("updatedReplicas") or 0)
    new_old = int(new_status.get("replicas") or 0) - int(new_status.get("updatedReplicas") or 0)
    return (int(new_status.get("updatedReplicas") or 0) > int(old.get("updatedReplicas") or 0) or
            new_old < old_old or
            int(new_status.get("readyReplicas") or 0) > int(old.get("readyReplicas") or 0) or
            int(new_status.get("availableReplicas") or 0) > int(old.get("availableReplicas") or 0))


def deployment_timed_out(d, new_status):
    if not has_progress_deadline(d):
        return False
    cond = get_condition(new_status, "Progressing")
    if cond is None:
        return False
    if cond.get("reason") == NEW_RS_AVAILABLE:
        return False
    if cond.get("reason") == TIMED_OUT:
        return True
    frm = parse_rfc3339(cond.get("lastUpdateTime"))
    if frm is None:
        return False
    return frm + int(d["spec"]["progressDeadlineSeconds"]) < now_fn()


def template_hash(tmpl, collision_count=None) -> str:
    """`ComputeHash`: a stable hash of the pod template (+ the collision count when set)."""
    data = json.dumps(tmpl or {}, sort_keys=True)
    if collision_count:
        data += str(collision_count)
    h = hashlib.sha256(data.encode()).hexdigest()
    return str(int(h[:8], 16) % (10 ** 10))
