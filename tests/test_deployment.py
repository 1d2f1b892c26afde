"""Deployment controller: tables ported from `pkg/controller/deployment/{sync,rolling,recreate,
progress}_test.go` and `util/deployment_util_test.go`, run against the fake client, plus live
checks of what the tables cannot see: a stuck rollout reports ProgressDeadlineExceeded (and
`kubectl rollout status` fails), a paused deployment still scales, minimum availability is
reported with the right reason.
"""
import asyncio
import copy
import datetime as dt

import pytest

from kubernetes_amd.api import meta as m
from kubernetes_amd.client.fake import FakeClient
from kubernetes_amd.client.informer import InformerFactory
from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.controllers import deployment_util as U
from kubernetes_amd.controllers.deployment import DeploymentController


def ts(h, mi=0, s=0, y=2016, mo=5, d=20):
    return dt.datetime(y, mo, d, h, mi, s, tzinfo=dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


NEW, OLD, OLDER = ts(2), ts(1), ts(0)


def rs(name, replicas, selector=None, timestamp=None, available=None, status_replicas=None):
    r = {"apiVersion": "apps/v1", "kind": "ReplicaSet",
         "metadata": {"name": name, "namespace": "default", "uid": f"uid-{name}"},
         "spec": {"replicas": replicas, "selector": {"matchLabels": dict(selector or {})}, "template": {}}}
    if timestamp:
        r["metadata"]["creationTimestamp"] = timestamp
    st = {}
    if available is not None:
        st["availableReplicas"] = available
    if status_replicas is not None:
        st["replicas"] = status_replicas
    if st:
        r["status"] = st
    return r


def deployment(name, replicas, history=None, surge=0, unavailable=0, selector=None, strategy="RollingUpdate",
               pds=None):
    d = {"apiVersion": "apps/v1", "kind": "Deployment",
         "metadata": {"name": name, "namespace": "default", "uid": f"uid-{name}", "annotations": {}, "generation": 1},
         "spec": {"replicas": replicas, "selector": {"matchLabels": dict(selector or {})},
                  "strategy": {"type": strategy},
                  "template": {"metadata": {"labels": dict(selector or {})},
                               "spec": {"containers": [{"name": "c", "image": "foo/bar"}]}}}}
    if strategy == "RollingUpdate":
        d["spec"]["strategy"]["rollingUpdate"] = {"maxSurge": surge, "maxUnavailable": unavailable}
    if history is not None:
        d["spec"]["revisionHistoryLimit"] = history
    if pds is not None:
        d["spec"]["progressDeadlineSeconds"] = pds
    return d


class Recorder:
    """A controller on an empty fake client whose RS updates / deletes are answered and recorded
    (the reference's `fake.Clientset{}` + `Actions()`)."""

    def __init__(self):
        self.c = FakeClient()
        self.updates, self.deletes = [], []

        def upd(a):
            self.updates.append(copy.deepcopy(a.obj))
            return True, copy.deepcopy(a.obj)

        def dele(a):
            self.deletes.append(a.name)
            return True, {"kind": "Status"}
        self.c.prepend_reactor("update", "replicasets", upd)
        self.c.prepend_reactor("delete", "replicasets", dele)
        self.c.prepend_reactor("patch", "deployments", lambda a: (True, {}))
        self.dc = DeploymentController(self.c, InformerFactory(self.c))
        self.dc.setup()


def _go(coro):
    return asyncio.run(coro)


# -- sync_test.go: TestScale --------------------------------------------------------------------
def _updated(d, **kw):
    d = deployment("foo", **kw)
    d["spec"]["template"]["metadata"]["labels"]["another"] = "label"
    return d


SCALE = [
    ("normal scaling event: 10 -> 12", deployment("foo", 12), deployment("foo", 10),
     rs("foo-v1", 10, None, NEW), [], 12, [], set(), {}),
    ("normal scaling event: 10 -> 5", deployment("foo", 5), deployment("foo", 10),
     rs("foo-v1", 10, None, NEW), [], 5, [], set(), {}),
    ("proportional scaling: 5 -> 10", deployment("foo", 10), deployment("foo", 5),
     rs("foo-v2", 2, None, NEW), [rs("foo-v1", 3, None, OLD)], 4, [6], set(), {}),
    ("proportional scaling: 5 -> 3", deployment("foo", 3), deployment("foo", 5),
     rs("foo-v2", 2, None, NEW), [rs("foo-v1", 3, None, OLD)], 1, [2], set(), {}),
    ("proportional scaling: 9 -> 4", deployment("foo", 4), deployment("foo", 9),
     rs("foo-v2", 8, None, NEW), [rs("foo-v1", 1, None, OLD)], 4, [0], set(), {}),
    ("proportional scaling: 7 -> 10", deployment("foo", 10), deployment("foo", 7),
     rs("foo-v3", 2, None, NEW), [rs("foo-v2", 3, None, OLD), rs("foo-v1", 2, None, OLDER)], 3, [4, 3], set(), {}),
    ("proportional scaling: 13 -> 8", deployment("foo", 8), deployment("foo", 13),
     rs("foo-v3", 2, None, NEW), [rs("foo-v2", 8, None, OLD), rs("foo-v1", 3, None, OLDER)], 1, [5, 2], set(), {}),
    ("leftover distribution: 3 -> 4", deployment("foo", 4), deployment("foo", 3),
     rs("foo-v3", 1, None, NEW), [rs("foo-v2", 1, None, OLD), rs("foo-v1", 1, None, OLDER)], 2, [1, 1], set(), {}),
    ("leftover distribution: 3 -> 2", deployment("foo", 2), deployment("foo", 3),
     rs("foo-v3", 1, None, NEW), [rs("foo-v2", 1, None, OLD), rs("foo-v1", 1, None, OLDER)], 1, [1, 0], set(), {}),
    ("proportional scaling (no new rs): 4 -> 5", deployment("foo", 5), deployment("foo", 4),
     None, [rs("foo-v2", 2, None, OLD), rs("foo-v1", 2, None, OLDER)], None, [3, 2], set(), {}),
    ("proportional scaling: 6 -> 0", deployment("foo", 0), deployment("foo", 6),
     rs("foo-v3", 3, None, NEW), [rs("foo-v2", 2, None, OLD), rs("foo-v1", 1, None, OLDER)], 0, [0, 0], set(), {}),
    ("proportional scaling: 0 -> 6", deployment("foo", 6), deployment("foo", 6),
     rs("foo-v3", 0, None, NEW), [rs("foo-v2", 0, None, OLD), rs("foo-v1", 0, None, OLDER)], 6, [0, 0],
     {"foo-v2", "foo-v1"}, {}),
    ("failed rs update", deployment("foo", 5), deployment("foo", 5),
     rs("foo-v3", 2, None, NEW), [rs("foo-v2", 1, None, OLD), rs("foo-v1", 1, None, OLDER)], 2, [2, 1],
     {"foo-v3", "foo-v1"}, {"foo-v2": 3}),
    ("deployment with surge pods", deployment("foo", 20, surge=2), deployment("foo", 10, surge=2),
     rs("foo-v2", 6, None, NEW), [rs("foo-v1", 6, None, OLD)], 11, [11], set(), {}),
    ("change both surge and size", deployment("foo", 50, surge=6), deployment("foo", 10, surge=3),
     rs("foo-v2", 5, None, NEW), [rs("foo-v1", 8, None, OLD)], 22, [34], set(), {}),
    ("change both size and template", _updated(None, replicas=14, selector={"foo": "bar"}),
     deployment("foo", 10, selector={"foo": "bar"}),
     None, [rs("foo-v2", 7, None, NEW), rs("foo-v1", 3, None, OLD)], None, [10, 4], set(), {}),
    ("saturated but broken new replica set does not affect old pods", deployment("foo", 2, surge=1, unavailable=1),
     deployment("foo", 2, surge=1, unavailable=1),
     rs("foo-v2", 2, None, NEW, available=0), [rs("foo-v1", 1, None, OLD)], 2, [1], set(), {}),
]


@pytest.mark.parametrize("case", SCALE, ids=[c[0] for c in SCALE])
def test_scale(case):
    name, d, old_d, new_rs, old_rss, exp_new, exp_old, wasnt, desired_ann = copy.deepcopy(case)
    for r in ([new_rs] if new_rs else []) + old_rss:
        want = desired_ann.get(r["metadata"]["name"], U.replicas_of(old_d))
        U.set_replicas_annotations(r, want, want + U.max_surge(old_d))
    if old_d["spec"]["replicas"] != d["spec"]["replicas"]:
        d.setdefault("status", {})["replicas"] = old_d["spec"]["replicas"]
    h = Recorder()
    _go(h.dc.scale(d, new_rs, old_rss))
    sizes = {r["metadata"]["name"]: U.replicas_of(r) for r in ([new_rs] if new_rs else []) + old_rss}
    for u in h.updates:
        if u["metadata"]["name"] not in wasnt:
            sizes[u["metadata"]["name"]] = U.replicas_of(u)
    if exp_new is not None and new_rs is not None:
        assert sizes[new_rs["metadata"]["name"]] == exp_new, name
    assert [sizes[r["metadata"]["name"]] for r in old_rss] == exp_old, name


# -- sync_test.go: cleanupDeployment -------------------------------------------------------------
def _rs_status(name, spec, status, deleted=False):
    r = rs(name, spec, {"foo": "bar"}, status_replicas=status)
    if deleted:
        r["metadata"]["deletionTimestamp"] = ts(3)
    return r


@pytest.mark.parametrize("old,limit,expected", [
    ([_rs_status("foo-1", 0, 0), _rs_status("foo-2", 0, 0), _rs_status("foo-3", 0, 0)], 1, 2),
    ([_rs_status("foo-1", 0, 0), _rs_status("foo-2", 0, 1), _rs_status("foo-3", 1, 0), _rs_status("foo-4", 1, 1)], 0, 1),
    ([_rs_status("foo-1", 0, 0), _rs_status("foo-2", 0, 0)], 0, 2),
    ([_rs_status("foo-1", 1, 1), _rs_status("foo-2", 1, 1)], 0, 0),
    ([_rs_status("foo-1", 0, 0, deleted=True)], 0, 0),
])
def test_cleanup_deployment(old, limit, expected):
    h = Recorder()
    _go(h.dc.cleanup_deployment(old, deployment("foo", 1, history=limit, selector={"foo": "bar"})))
    assert len(h.deletes) == expected


# -- rolling_test.go ----------------------------------------------------------------------------
@pytest.mark.parametrize("replicas,surge,old,new,expected", [
    (10, 0, 10, 0, None), (10, 2, 10, 0, 2), (10, 2, 5, 0, 7), (10, 2, 10, 2, None), (10, 2, 2, 11, 10)])
def test_reconcile_new_replica_set(replicas, surge, old, new, expected):
    h = Recorder()
    new_rs, old_rs = rs("foo-v2", new), rs("foo-v2", old)
    d = deployment("foo", replicas, surge=surge, unavailable=0, selector={"foo": "bar"})
    scaled = _go(h.dc.reconcile_new_replica_set([new_rs, old_rs], new_rs, d))
    if expected is None:
        assert not scaled and not h.updates
    else:
        assert scaled and len(h.updates) == 1 and U.replicas_of(h.updates[0]) == expected


@pytest.mark.parametrize("replicas,unavail,old,new,ready_old,ready_new,scale", [
    (10, 0, 10, 0, 10, 0, True), (10, 2, 10, 0, 10, 0, True), (10, 2, 10, 0, 8, 0, True),
    (10, 2, 10, 0, 9, 0, True), (10, 2, 8, 2, 8, 0, False)])
def test_reconcile_old_replica_sets(replicas, unavail, old, new, ready_old, ready_new, scale):
    h = Recorder()
    new_rs = rs("foo-new", new, {"foo": "new"}, available=ready_new)
    old_rs = rs("foo-old", old, {"foo": "old"}, available=ready_old)
    d = deployment("foo", replicas, surge=0, unavailable=unavail, selector={"foo": "new"})
    assert _go(h.dc.reconcile_old_replica_sets([old_rs, new_rs], [old_rs], new_rs, d)) == scale


@pytest.mark.parametrize("old,ready,max_cleanup,expected", [(10, 8, 1, 1), (10, 8, 3, 2), (10, 8, 0, 0), (10, 10, 3, 0)])
def test_cleanup_unhealthy_replicas(old, ready, max_cleanup, expected):
    h = Recorder()
    d = deployment("foo", 10, surge=2, unavailable=2)
    _, count = _go(h.dc.cleanup_unhealthy_replicas([rs("foo-v2", old, available=ready)], d, max_cleanup))
    assert count == expected


@pytest.mark.parametrize("replicas,unavail,ready,old,expected", [
    (10, 0, 10, 10, 9), (10, 2, 10, 10, 8), (10, 2, 8, 10, None), (10, 2, 10, 0, None), (10, 2, 1, 10, None)])
def test_scale_down_old_replica_sets_for_rolling_update(replicas, unavail, ready, old, expected):
    h = Recorder()
    old_rs = rs("foo-v2", old, available=ready)
    d = deployment("foo", replicas, surge=0, unavailable=unavail, selector={"foo": "bar"})
    scaled = _go(h.dc.scale_down_old_replica_sets_for_rolling_update([old_rs], [old_rs], d))
    if expected is None:
        assert scaled == 0 and not h.updates
    else:
        assert scaled and U.replicas_of(h.updates[0]) == expected


# -- recreate_test.go -----------------------------------------------------------------------------
def test_scale_down_old_replica_sets_for_recreate():
    h = Recorder()
    d = deployment("foo", 3, selector={"foo": "bar"}, strategy="Recreate")
    olds = [rs("foo-0", 3, {"foo": "bar"})]
    assert _go(h.dc.scale_down_old_replica_sets_for_recreate(olds, d))
    assert all(U.replicas_of(r) == 0 for r in olds)


def _pods(*phases):
    return [{"metadata": {"name": f"p{i}"}, "status": {"phase": ph}} for i, ph in enumerate(phases)]


@pytest.mark.parametrize("name,new_rs,old_rss,pods,expected", [
    ("no old RSs", None, [], {}, False),
    ("old RSs with running pods", None, [rs("a", 1), rs("b", 1)],
     {"uid-a": _pods("Running"), "uid-b": _pods("Running")}, True),
    ("old RSs without pods but with non-zero status replicas", None, [rs("rs-1", 0, status_replicas=1)], {}, True),
    ("old RSs without pods or non-zero status replicas", None, [rs("rs-1", 0, status_replicas=0)], {}, False),
    ("terminal pods only", None, [rs("rs-1", 0, status_replicas=0)], {"uid-1": _pods("Failed", "Succeeded")}, False),
    ("pod in unknown phase", None, [rs("rs-1", 0, status_replicas=0)], {"uid-1": _pods("Unknown")}, True),
    ("pending pod", None, [rs("rs-1", 0, status_replicas=0)], {"uid-1": _pods("Pending")}, True),
    ("new RS pods do not count", rs("new", 1), [rs("rs-1", 0, status_replicas=0)], {"uid-new": _pods("Running")}, False),
])
def test_old_pods_running(name, new_rs, old_rss, pods, expected):
    assert DeploymentController.old_pods_running(new_rs, old_rss, pods) == expected, name


# -- progress_test.go -----------------------------------------------------------------------------
TEST_TIME = ts(18, 49, 0, 2017, 2, 15)


def current_deployment(pds, replicas, st_replicas, updated, available, conditions):
    d = {"kind": "Deployment", "metadata": {"name": "progress-test", "namespace": "default", "uid": "u"},
         "spec": {"replicas": replicas, "strategy": {"type": "Recreate"}},
         "status": {"replicas": st_replicas, "updatedReplicas": updated, "availableReplicas": available,
                    "conditions": copy.deepcopy(conditions or [])}}
    if pds is not None:
        d["spec"]["progressDeadlineSeconds"] = pds
    return d


def cond(status, reason, t=None):
    c = {"type": "Progressing", "status": status, "reason": reason}
    if t:
        c["lastUpdateTime"] = c["lastTransitionTime"] = t
    return c


FAILED = cond("False", U.TIMED_OUT)
NEW_RS_AVAILABLE = cond("True", U.NEW_RS_AVAILABLE, TEST_TIME)
RS_UPDATED = cond("True", U.REPLICA_SET_UPDATED, TEST_TIME)
STUCK = {"type": "Progressing", "status": "True", "lastUpdateTime": TEST_TIME}


@pytest.fixture
def pinned_now():
    saved = U.now_fn
    yield lambda t: setattr(U, "now_fn", lambda: m.parse_rfc3339(t) if isinstance(t, str) else t)
    U.now_fn = saved


@pytest.mark.parametrize("name,d,status,now,expected", [
    ("no progressDeadlineSeconds specified", current_deployment(None, 4, 3, 3, 2, None), (3, 3, 2), None, None),
    ("no progressing condition found", current_deployment(60, 4, 3, 3, 2, None), (3, 3, 2), None, None),
    ("complete deployment does not need to be requeued", current_deployment(60, 3, 3, 3, 3, None), (3, 3, 3), None, None),
    ("already failed deployment does not need to be requeued", current_deployment(60, 3, 3, 3, 0, [FAILED]),
     (3, 3, 0), None, None),
    ("stuck deployment - 30s", current_deployment(60, 3, 3, 3, 1, [STUCK]), (3, 3, 1), ts(18, 49, 30, 2017, 2, 15), 30),
    ("stuck deployment - 1s", current_deployment(60, 3, 3, 3, 1, [STUCK]), (3, 3, 1), ts(18, 49, 59, 2017, 2, 15), 1),
    ("failed deployment - less than a second => now", current_deployment(60, 3, 3, 3, 1, [STUCK]), (3, 3, 1),
     m.parse_rfc3339(ts(18, 49, 59, 2017, 2, 15)) + 1e-3, 0),   # Go: +1ns; float64 epoch seconds: +1ms
    ("failed deployment - now", current_deployment(60, 3, 3, 3, 1, [STUCK]), (3, 3, 1), ts(18, 50, 0, 2017, 2, 15), 0),
    ("failed deployment - 1s after deadline", current_deployment(60, 3, 3, 3, 1, [STUCK]), (3, 3, 1),
     ts(18, 50, 1, 2017, 2, 15), 0),
    ("failed deployment - 60s after deadline", current_deployment(60, 3, 3, 3, 1, [STUCK]), (3, 3, 1),
     ts(18, 51, 0, 2017, 2, 15), 0),
])
def test_requeue_stuck_deployment(name, d, status, now, expected, pinned_now):
    if now is not None:
        pinned_now(now)
    h = Recorder()
    st = {"replicas": status[0], "updatedReplicas": status[1], "availableReplicas": status[2]}
    got = h.dc.requeue_stuck_deployment(d, st)
    assert got == expected if expected is None else got == pytest.approx(expected, abs=1e-6), name


def rs_avail(name, spec, st, avail):
    return rs(name, spec, status_replicas=st, available=avail)


SYNC_ROLLOUT = [
    ("General: remove Progressing condition if no Progress Deadline", current_deployment(None, 3, 2, 2, 2, [RS_UPDATED]),
     [rs_avail("bar", 0, 1, 1)], rs_avail("foo", 3, 2, 2), None, None, None, False),
    ("General: do not estimate progress of deployment with only one active ReplicaSet",
     current_deployment(60, 3, 3, 3, 3, [NEW_RS_AVAILABLE]), [rs_avail("bar", 3, 3, 3)], None,
     "True", U.NEW_RS_AVAILABLE, True, True),
    ("DeploymentProgressing: dont update lastTransitionTime if deployment already has Progressing=True",
     current_deployment(60, 3, 2, 2, 2, [RS_UPDATED]), [rs_avail("bar", 0, 1, 1)], rs_avail("foo", 3, 2, 2),
     "True", U.REPLICA_SET_UPDATED, False, True),
    ("DeploymentProgressing: update everything if deployment has Progressing=False",
     current_deployment(60, 3, 2, 2, 2, [FAILED]), [rs_avail("bar", 0, 1, 1)], rs_avail("foo", 3, 2, 2),
     "True", U.REPLICA_SET_UPDATED, False, False),
    ("DeploymentProgressing: create Progressing condition if it does not exist",
     current_deployment(60, 3, 2, 2, 2, []), [rs_avail("bar", 0, 1, 1)], rs_avail("foo", 3, 2, 2),
     "True", U.REPLICA_SET_UPDATED, False, False),
    ("DeploymentComplete: dont update lastTransitionTime if deployment already has Progressing=True",
     current_deployment(60, 3, 3, 3, 3, [RS_UPDATED]), [], rs_avail("foo", 3, 3, 3),
     "True", U.NEW_RS_AVAILABLE, False, True),
    ("DeploymentComplete: update everything if deployment has Progressing=False",
     current_deployment(60, 3, 3, 3, 3, [FAILED]), [], rs_avail("foo", 3, 3, 3),
     "True", U.NEW_RS_AVAILABLE, False, False),
    ("DeploymentComplete: create Progressing condition if it does not exist",
     current_deployment(60, 3, 3, 3, 3, []), [], rs_avail("foo", 3, 3, 3), "True", U.NEW_RS_AVAILABLE, False, False),
    ("DeploymentComplete: defend against NPE when newRS=nil", current_deployment(60, 0, 3, 3, 3, [RS_UPDATED]),
     [rs_avail("foo", 0, 0, 0)], None, "True", U.NEW_RS_AVAILABLE, False, False),
    ("DeploymentTimedOut: update status if rollout exceeds Progress Deadline",
     current_deployment(60, 3, 2, 2, 2, [RS_UPDATED]), [], rs_avail("foo", 3, 2, 2),
     "False", U.TIMED_OUT, False, False),
    ("DeploymentTimedOut: do not update status if deployment has existing timedOut condition",
     current_deployment(60, 3, 2, 2, 2, [dict(FAILED, lastUpdateTime=TEST_TIME, lastTransitionTime=TEST_TIME)]), [],
     rs_avail("foo", 3, 2, 2), "False", U.TIMED_OUT, True, True),
]


@pytest.mark.parametrize("case", SYNC_ROLLOUT, ids=[c[0] for c in SYNC_ROLLOUT])
def test_sync_rollout_status(case):
    name, d, all_rss, new_rs, status, reason, keep_update, keep_transition = copy.deepcopy(case)
    if new_rs is not None:
        all_rss.append(new_rs)
    h = Recorder()
    st = h.dc.rollout_status(all_rss, new_rs, d)
    c = U.get_condition(st, "Progressing")
    if status is None:
        assert c is None, name
        return
    assert c is not None and (c["status"], c["reason"]) == (status, reason), (name, c)
    if keep_update:
        assert c["lastUpdateTime"] == TEST_TIME, name
    if keep_transition:
        assert c["lastTransitionTime"] == TEST_TIME, name


# -- util/deployment_util_test.go -----------------------------------------------------------------
@pytest.mark.parametrize("surge,unavail,desired,exp", [
    ("0%", "0%", 0, (0, 1)), ("39%", "39%", 10, (4, 3)), ("oops", "39%", 10, None), ("55%", "urg", 10, None)])
def test_resolve_fenceposts(surge, unavail, desired, exp):
    if exp is None:
        with pytest.raises(ValueError):
            U.resolve_fenceposts(surge, unavail, desired)
    else:
        assert U.resolve_fenceposts(surge, unavail, desired) == exp


@pytest.mark.parametrize("name,strategy,dep,new,surge,expected", [
    ("can not scale up - to newRSReplicas", "RollingUpdate", 1, 5, 1, 5),
    ("scale up - to depReplicas", "RollingUpdate", 6, 2, 10, 6),
    ("recreate - to depReplicas", "Recreate", 3, 1, 1, 3)])
def test_new_rs_new_replicas(name, strategy, dep, new, surge, expected):
    d = deployment("nginx", dep, surge=surge, unavailable=1)
    d["spec"]["strategy"]["type"] = strategy
    assert U.new_rs_new_replicas(d, [rs("rs5", 5)], rs("new", new)) == expected, name


@pytest.mark.parametrize("desired,current,updated,available,unavail,surge,expected", [
    (5, 5, 5, 4, 1, 0, False), (5, 5, 5, 3, 1, 0, False), (5, 5, 5, 5, 0, 0, True), (5, 5, 4, 5, 0, 0, False),
    (1, 2, 1, 1, 0, 1, False), (1, 1, 1, 0, 1, 1, False)])
def test_deployment_complete(desired, current, updated, available, unavail, surge, expected):
    d = deployment("d", desired, surge=surge, unavailable=unavail)
    d["metadata"]["generation"] = 0
    st = {"replicas": current, "updatedReplicas": updated, "availableReplicas": available}
    assert U.deployment_complete(d, st) == expected


def _st(cur, upd, ready, avail):
    return {"replicas": cur, "updatedReplicas": upd, "readyReplicas": ready, "availableReplicas": avail}


@pytest.mark.parametrize("old,new,expected", [
    (_st(10, 4, 4, 4), _st(10, 6, 4, 4), True), (_st(10, 4, 4, 4), _st(10, 4, 4, 4), False),
    (_st(10, 4, 6, 6), _st(8, 4, 6, 6), True), (_st(10, 7, 3, 3), _st(10, 6, 3, 3), False),
    (_st(10, 4, 7, 7), _st(8, 8, 5, 5), True), (_st(10, 10, 9, 8), _st(10, 10, 10, 8), True),
    (_st(10, 10, 10, 9), _st(10, 10, 10, 10), True)])
def test_deployment_progressing(old, new, expected):
    assert U.deployment_progressing({"status": old}, new) == expected


def _tf(mi, s):
    return ts(0, mi, s, 2016, 1, 1)


@pytest.mark.parametrize("name,pds,reason,frm,now,expected", [
    ("no progressDeadlineSeconds specified - no timeout", None, "", _tf(1, 9), _tf(1, 20), False),
    ("progressDeadlineSeconds: 10s, 11s elapsed", 10, "", _tf(1, 9), _tf(1, 20), True),
    ("progressDeadlineSeconds: 10s, 9s elapsed", 10, "", _tf(1, 11), _tf(1, 20), False),
    ("previous status was a complete deployment", None, U.NEW_RS_AVAILABLE, None, None, False)])
def test_deployment_timed_out(name, pds, reason, frm, now, expected, pinned_now):
    if now:
        pinned_now(now)
    d = {"spec": {}, "status": {"conditions": [{"type": "Progressing", "status": "True", "reason": reason,
                                                "lastUpdateTime": frm}]}}
    if pds is not None:
        d["spec"]["progressDeadlineSeconds"] = pds
    assert U.deployment_timed_out(d, d["status"]) == expected, name


@pytest.mark.parametrize("replicas,unavail,expected", [
    (10, 5, 5), (10, 10, 10), (5, 10, 5), (0, 10, 0), (10, "50%", 5), (10, "100%", 10), (5, "100%", 5)])
def test_max_unavailable(replicas, unavail, expected):
    assert U.max_unavailable(deployment("d", replicas, surge=1, unavailable=unavail)) == expected


def test_max_unavailable_recreate():
    assert U.max_unavailable({"spec": {"strategy": {"type": "Recreate"}}}) == 0


def test_annotation_utils_and_rollback_history():
    d = deployment("d", 3, surge=1)
    d["metadata"]["annotations"] = {"team": "gpu", U.REVISION: "9", U.LAST_APPLIED: "{}"}
    r = rs("r", 3)
    assert U.set_new_replica_set_annotations(d, r, "1", False)
    ann = r["metadata"]["annotations"]
    assert ann == {"team": "gpu", U.REVISION: "1", U.DESIRED_REPLICAS: "3", U.MAX_REPLICAS: "4"}
    # a rollback to this RS: the old revision goes to the history annotation
    assert U.set_new_replica_set_annotations(d, r, "4", True)
    assert ann[U.REVISION] == "4" and ann[U.REVISION_HISTORY] == "1"
    assert U.set_new_replica_set_annotations(d, r, "6", True) and ann[U.REVISION_HISTORY] == "1,4"
    assert not U.set_new_replica_set_annotations(d, r, "5", True)       # never lowers a revision
    assert U.last_revision([rs("a", 0), r, dict(rs("b", 0), metadata={"annotations": {U.REVISION: "5"}})]) == 5


def test_empty_selector_selects_nothing(run):
    async def main():
        d = deployment("foo", 1)
        d["spec"]["selector"] = {}
        d["metadata"]["generation"] = 2
        c = FakeClient(d)
        dc = DeploymentController(c, InformerFactory(c))
        dc.setup()
        dc.factory.start()
        await dc.factory.wait_for_cache_sync()
        await dc.sync("default/foo")
        assert not [a for a in c.actions if a.resource == "replicasets" and a.verb == "create"]
        assert (await c.get("deployments", "foo", "default"))["status"]["observedGeneration"] == 2
    run(main())


# -- live cluster ---------------------------------------------------------------------------------
def _live_deploy(name, replicas, gpus=0, pds=None, paused=False):
    c = {"name": "c", "image": "kubernetes-amd/pause"}
    if gpus:
        c["resources"] = {"limits": {"amd.com/gpu": str(gpus)}}
    d = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": name, "namespace": "default"},
         "spec": {"replicas": replicas, "selector": {"matchLabels": {"app": name}}, "paused": paused,
                  "template": {"metadata": {"labels": {"app": name}}, "spec": {"containers": [c]}}}}
    if pds is not None:
        d["spec"]["progressDeadlineSeconds"] = pds
    return d


def test_progress_deadline_paused_scaling_and_availability_live(run, tmp_path):
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=2, controllers=["deployment", "replicaset"]) as cl:
            c = cl.client

            def conds(d):
                return {x["type"]: x for x in (d.get("status") or {}).get("conditions") or ()}
            # unschedulable (asks for more GPUs than the node has): stuck -> ProgressDeadlineExceeded
            await c.create("deployments", _live_deploy("stuck", 1, gpus=8, pds=2))

            async def timed_out():
                d = await c.get("deployments", "stuck", "default")
                p = conds(d).get("Progressing")
                return d if p and p["reason"] == U.TIMED_OUT and p["status"] == "False" else None
            d = await cl.wait_for(timed_out, timeout=20)
            av = conds(d)["Available"]
            assert (av["status"], av["reason"]) == ("False", U.MIN_UNAVAILABLE)
            from kubernetes_amd.kubectl.cli import rollout_status
            with pytest.raises(SystemExit) as ei:
                rollout_status(d)
            assert "exceeded its progress deadline" in str(ei.value)
            # a paused deployment still scales (and reports DeploymentPaused)
            await c.create("deployments", _live_deploy("web", 2, paused=True))

            async def n_pods(app, n):
                ps = (await c.list("pods", "default", label_selector=f"app={app}"))["items"]
                return len([p for p in ps if not p["metadata"].get("deletionTimestamp")]) == n
            await asyncio.sleep(1.0)
            assert not (await c.list("replicasets", "default", label_selector="app=web"))["items"]
            await c.patch("deployments", "web", {"spec": {"paused": False}}, "default")
            await cl.wait_for(lambda: n_pods("web", 2), timeout=20)
            await c.patch("deployments", "web", {"spec": {"paused": True}}, "default")

            async def paused_cond():
                p = conds(await c.get("deployments", "web", "default")).get("Progressing")
                return p and p["reason"] == U.PAUSED
            await cl.wait_for(paused_cond, timeout=10)
            await c.patch("deployments", "web", {"spec": {"replicas": 4}}, "default")
            await cl.wait_for(lambda: n_pods("web", 4), timeout=20)
            rss = (await c.list("replicasets", "default", label_selector="app=web"))["items"]
            assert len(rss) == 1 and U.annotations_of(rss[0])[U.DESIRED_REPLICAS] == "4"
            # a paused template change does not roll out
            await c.patch("deployments", "web", {"spec": {"template": {"metadata": {"annotations": {"x": "1"}}}}},
                          "default")
            await asyncio.sleep(1.0)
            assert len((await c.list("replicasets", "default", label_selector="app=web"))["items"]) == 1
            await c.patch("deployments", "web", {"spec": {"paused": False}}, "default")

            async def rolled():
                d = await c.get("deployments", "web", "default")
                p = conds(d).get("Progressing")
                st = d.get("status") or {}
                return p and p["reason"] == U.NEW_RS_AVAILABLE and st.get("updatedReplicas") == 4 and \
                    st.get("replicas") == 4 and st.get("availableReplicas") == 4
            await cl.wait_for(rolled, timeout=40)
            d = await c.get("deployments", "web", "default")
            assert U.annotations_of(d)[U.REVISION] == "2"
            av = conds(d)["Available"]
            assert (av["status"], av["reason"]) == ("True", U.MIN_AVAILABLE)
    run(main(), timeout=120)
