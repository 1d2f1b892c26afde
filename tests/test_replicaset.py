"""ReplicaSet controller: `controller_utils_test.go` TestSortingActivePods (the deletion order)
and `replica_set_test.go` cases over the fake client — nothing to do at the right count,
deletes of the lowest-ranked pods, slow-start creates that stop at the first failing batch with a
ReplicaFailure condition, adoption of matching orphans, release of owned pods whose labels
stopped matching, and pods of other controllers left alone."""
import asyncio
import random
import time

from kubernetes_amd.api.meta import now_rfc3339
from kubernetes_amd.client.fake import FakeClient
from kubernetes_amd.client.informer import InformerFactory
from kubernetes_amd.client.rest import APIStatusError
from kubernetes_amd.controllers.base import active_pods_key
from kubernetes_amd.controllers.replicaset import ReplicaSetController

UID = "rs-uid"


def rs(replicas):
    return {"apiVersion": "apps/v1", "kind": "ReplicaSet",
            "metadata": {"name": "foobar", "namespace": "default", "uid": UID, "generation": 1},
            "spec": {"replicas": replicas, "selector": {"matchLabels": {"app": "web"}},
                     "template": {"metadata": {"labels": {"app": "web"}},
                                  "spec": {"containers": [{"name": "c", "image": "foo/bar"}]}}}}


def pod(name, owner=True, labels=None, node="node-a", phase="Running", ready=True, ready_at=None, restarts=(0,),
        created=None):
    p = {"apiVersion": "v1", "kind": "Pod",
         "metadata": {"name": name, "namespace": "default", "uid": f"{name}-uid",
                      "labels": {"app": "web"} if labels is None else labels},
         "spec": {"nodeName": node} if node else {},
         "status": {"phase": phase, "containerStatuses": [{"name": f"c{i}", "restartCount": r}
                                                          for i, r in enumerate(restarts)]}}
    if ready:
        cond = {"type": "Ready", "status": "True"}
        if ready_at is not None:
            cond["lastTransitionTime"] = ready_at
        p["status"]["conditions"] = [cond]
    if created is not None:
        p["metadata"]["creationTimestamp"] = created
    if owner:
        p["metadata"]["ownerReferences"] = [{"apiVersion": "apps/v1", "kind": "ReplicaSet", "name": "foobar",
                                             "uid": UID, "controller": True}]
    return p


def test_sorting_active_pods():
    now = now_rfc3339()
    then = now_rfc3339(time.time() - 30 * 86400)
    pods = [pod("p0", node="", phase="Pending", ready=False),
            pod("p1", node="bar", phase="Pending", ready=False),
            pod("p2", phase="Unknown", ready=False),
            pod("p3", phase="Running", ready=False),
            pod("p4", ready_at=None, restarts=(3, 0)),
            pod("p5", ready_at=now, restarts=(3, 0)),
            pod("p6", ready_at=then, restarts=(3, 0)),
            pod("p7", ready_at=then, restarts=(2, 1), created=now),
            pod("p8", ready_at=then, restarts=(2, 1), created=then)]
    want = [p["metadata"]["name"] for p in pods]
    for _ in range(20):
        shuffled = pods[:]
        random.shuffle(shuffled)
        assert [p["metadata"]["name"] for p in sorted(shuffled, key=active_pods_key)] == want


def run_sync(*objs, fail_creates_after=None):
    async def main():
        c = FakeClient(*objs)
        n = {"creates": 0}

        def on_create(a):
            n["creates"] += 1
            if fail_creates_after is not None and n["creates"] > fail_creates_after:
                raise APIStatusError(500, {"message": "fake error"})
            return False, None
        c.prepend_reactor("create", "pods", on_create)
        f = InformerFactory(c)
        rc = ReplicaSetController(c, f)
        rc.setup()
        events = []
        rc.recorder.event = lambda obj, typ, reason, msg: events.append((typ, reason))
        f.start()
        await f.wait_for_cache_sync()
        err = None
        try:
            await rc.sync("default/foobar")
        except APIStatusError as e:
            err = e
        acts = [(a.verb, a.resource) for a in c.actions if a.verb in ("create", "delete", "patch", "update")]
        return c, acts, events, err, n["creates"]
    return asyncio.run(main())


def test_sync_does_nothing_at_the_right_count():
    c, acts, events, err, _ = run_sync(rs(2), pod("a"), pod("b"))
    assert err is None and ("create", "pods") not in acts and ("delete", "pods") not in acts and not events


def test_sync_deletes_the_lowest_ranked():
    c, acts, events, err, _ = run_sync(rs(2), pod("a"), pod("b"), pod("pending", node="", phase="Pending", ready=False))
    deleted = [a for a in c.actions if a.verb == "delete" and a.resource == "pods"]
    assert [a.name for a in deleted] == ["pending"] and ("Normal", "SuccessfulDelete") in events


def test_slow_start_stops_at_the_first_failing_batch():
    c, acts, events, err, attempts = run_sync(rs(10), fail_creates_after=3)
    # batches of 1, 2 succeed (3 pods), the batch of 4 fails: 7 attempts, no fourth batch
    assert attempts == 7 and err is not None and ("Warning", "FailedCreate") in events
    st = (c.objects["replicasets"][("default", "foobar")]).get("status") or {}
    conds = [x for x in st.get("conditions") or () if x["type"] == "ReplicaFailure"]
    assert conds and conds[0]["reason"] == "FailedCreate"


def test_orphans_are_adopted_and_mismatches_released():
    other = pod("theirs")
    other["metadata"]["ownerReferences"][0].update(uid="other-uid", name="other")
    c, acts, events, err, _ = run_sync(rs(2), pod("orphan", owner=False), pod("stray", labels={"app": "db"}),
                                       pod("kept"), other)
    objs = c.objects["pods"]
    assert objs[("default", "orphan")]["metadata"]["ownerReferences"][0]["uid"] == UID
    assert not objs[("default", "stray")]["metadata"].get("ownerReferences")
    assert objs[("default", "theirs")]["metadata"]["ownerReferences"][0]["uid"] == "other-uid"
    # orphan + kept make 2: nothing created or deleted
    assert ("create", "pods") not in acts and ("delete", "pods") not in acts


def test_terminal_orphans_are_not_adopted():
    done = pod("done", owner=False, phase="Succeeded", ready=False)
    c, acts, events, err, _ = run_sync(rs(1), done, pod("a"))
    assert not c.objects["pods"][("default", "done")]["metadata"].get("ownerReferences")
