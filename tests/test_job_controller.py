"""Job controller: `pkg/controller/job/job_controller_test.go` TestControllerSyncJob table (plus
the active-deadline and orphan-adoption cases), over the fake client — one sync, then the
creations / deletions it issued and the status it wrote."""
import asyncio
import copy

import pytest

from kubernetes_amd.client.fake import FakeClient
from kubernetes_amd.client.informer import InformerFactory
from kubernetes_amd.client.rest import APIStatusError
from kubernetes_amd.controllers.job import JobController

UID = "job-uid"


def new_job(parallelism, completions, backoff, deleting=False):
    j = {"apiVersion": "batch/v1", "kind": "Job",
         "metadata": {"name": "foobar", "namespace": "default", "uid": UID},
         "spec": {"parallelism": parallelism, "backoffLimit": backoff,
                  "selector": {"matchLabels": {"controller-uid": UID}},
                  "template": {"metadata": {"labels": {"controller-uid": UID, "job-name": "foobar"}},
                               "spec": {"restartPolicy": "Never", "containers": [{"name": "c", "image": "foo/bar"}]}}}}
    if completions >= 0:
        j["spec"]["completions"] = completions
    if deleting:
        j["metadata"]["deletionTimestamp"] = "2017-01-01T00:00:00Z"
    return j


def pods(n, phase, start=0):
    out = []
    for i in range(start, start + n):
        out.append({"apiVersion": "v1", "kind": "Pod",
                    "metadata": {"name": f"pod-{phase}-{i}", "namespace": "default",
                                 "labels": {"controller-uid": UID, "job-name": "foobar"},
                                 "ownerReferences": [{"apiVersion": "batch/v1", "kind": "Job", "name": "foobar",
                                                      "uid": UID, "controller": True}]},
                    "spec": {}, "status": {"phase": phase}})
    return out


# name: (parallelism, completions, backoffLimit, deleting, controller error, pending, active, succeeded, failed,
#        creations, deletions, active, succeeded, failed, condition, reason)
CASES = {
    "job start": (2, 5, 6, False, False, 0, 0, 0, 0, 2, 0, 2, 0, 0, None, ""),
    "WQ job start": (2, -1, 6, False, False, 0, 0, 0, 0, 2, 0, 2, 0, 0, None, ""),
    "pending pods": (2, 5, 6, False, False, 2, 0, 0, 0, 0, 0, 2, 0, 0, None, ""),
    "correct # of pods": (2, 5, 6, False, False, 0, 2, 0, 0, 0, 0, 2, 0, 0, None, ""),
    "WQ job: correct # of pods": (2, -1, 6, False, False, 0, 2, 0, 0, 0, 0, 2, 0, 0, None, ""),
    "too few active pods": (2, 5, 6, False, False, 0, 1, 1, 0, 1, 0, 2, 1, 0, None, ""),
    "too few active pods with a dynamic job": (2, -1, 6, False, False, 0, 1, 0, 0, 1, 0, 2, 0, 0, None, ""),
    "too few active pods, with controller error": (2, 5, 6, False, True, 0, 1, 1, 0, 1, 0, 1, 1, 0, None, ""),
    "too many active pods": (2, 5, 6, False, False, 0, 3, 0, 0, 0, 1, 2, 0, 0, None, ""),
    "too many active pods, with controller error": (2, 5, 6, False, True, 0, 3, 0, 0, 0, 1, 3, 0, 0, None, ""),
    "failed pod": (2, 5, 6, False, True, 0, 1, 1, 1, 1, 0, 1, 1, 1, None, ""),
    "job finish": (2, 5, 6, False, False, 0, 0, 5, 0, 0, 0, 0, 5, 0, "Complete", ""),
    "WQ job finishing": (2, -1, 6, False, False, 0, 1, 1, 0, 0, 0, 1, 1, 0, None, ""),
    "WQ job all finished": (2, -1, 6, False, False, 0, 0, 2, 0, 0, 0, 0, 2, 0, "Complete", ""),
    "WQ job all finished despite one failure": (2, -1, 6, False, False, 0, 0, 1, 1, 0, 0, 0, 1, 1, "Complete", ""),
    "more active pods than completions": (2, 5, 6, False, False, 0, 10, 0, 0, 0, 8, 2, 0, 0, None, ""),
    "status change": (2, 5, 6, False, False, 0, 2, 2, 0, 0, 0, 2, 2, 0, None, ""),
    "deleting job": (2, 5, 6, True, False, 1, 1, 1, 0, 0, 0, 2, 1, 0, None, ""),
    "to many job sync failure": (2, 5, 0, True, False, 0, 0, 0, 1, 0, 0, 0, 0, 1, "Failed", "BackoffLimitExceeded"),
}


@pytest.mark.parametrize("name", list(CASES))
def test_controller_sync_job(name):
    (par, comp, backoff, deleting, ctl_err, pending, active, succ, failed,
     exp_create, exp_delete, exp_active, exp_succ, exp_failed, exp_cond, exp_reason) = CASES[name]

    async def main():
        objs = [new_job(par, comp, backoff, deleting)]
        objs += pods(pending, "Pending") + pods(active, "Running") + pods(succ, "Succeeded") + pods(failed, "Failed")
        c = FakeClient(*objs)
        creates, deletes = [], []

        def on(kind):
            def fn(a):
                (creates if kind == "create" else deletes).append(a.name)
                if ctl_err:
                    raise APIStatusError(500, {"message": "Fake error"})
                return False, None
            return fn
        c.prepend_reactor("create", "pods", on("create"))
        c.prepend_reactor("delete", "pods", on("delete"))
        f = InformerFactory(c)
        jc = JobController(c, f)
        jc.setup()
        f.start()
        await f.wait_for_cache_sync()
        try:
            await jc.sync("default/foobar")
        except Exception:          # noqa: BLE001 - failed pods / controller errors re-queue the job
            pass
        st = (await c.get("jobs", "foobar", "default")).get("status") or {}
        return creates, deletes, st
    creates, deletes, st = asyncio.run(main())
    assert len(creates) == exp_create, (name, creates)
    assert len(deletes) == exp_delete, (name, deletes)
    if exp_create or exp_delete or st:
        assert (st.get("active", 0), st.get("succeeded", 0), st.get("failed", 0)) == (exp_active, exp_succ, exp_failed), \
            (name, st)
    conds = [x for x in st.get("conditions") or () if x.get("status") == "True"]
    if exp_cond is None:
        assert not conds, (name, conds)
    else:
        assert conds and conds[-1]["type"] == exp_cond and conds[-1].get("reason", "") == exp_reason, (name, conds)


def test_past_active_deadline_fails_the_job_and_deletes_active_pods():
    async def main():
        j = new_job(1, 1, 6)
        j["spec"]["activeDeadlineSeconds"] = 10
        j["status"] = {"startTime": "2017-01-01T00:00:00Z", "active": 1}
        c = FakeClient(j, *pods(1, "Running"))
        f = InformerFactory(c)
        jc = JobController(c, f)
        jc.setup()
        f.start()
        await f.wait_for_cache_sync()
        await jc.sync("default/foobar")
        st = (await c.get("jobs", "foobar", "default"))["status"]
        return st, c.objects.get("pods", {})
    st, left = asyncio.run(main())
    failed = [x for x in st["conditions"] if x["type"] == "Failed"]
    assert failed and failed[0]["reason"] == "DeadlineExceeded"
    assert st["active"] == 0 and st["failed"] == 1 and not left


def test_job_start_requeues_for_its_active_deadline():
    async def main():
        j = new_job(1, 1, 6)
        j["spec"]["activeDeadlineSeconds"] = 30
        c = FakeClient(j)
        f = InformerFactory(c)
        jc = JobController(c, f)
        jc.setup()
        f.start()
        await f.wait_for_cache_sync()
        await jc.sync("default/foobar")
        return jc.queue._heap
    heap = asyncio.run(main())
    assert any(item == "default/foobar" for _, _, item in heap)


def test_orphan_pod_matching_the_selector_is_adopted():
    async def main():
        orphan = pods(1, "Running")[0]
        orphan["metadata"].pop("ownerReferences")
        c = FakeClient(new_job(1, 1, 6), orphan)
        f = InformerFactory(c)
        jc = JobController(c, f)
        jc.setup()
        f.start()
        await f.wait_for_cache_sync()
        await jc.sync("default/foobar")
        p = await c.get("pods", orphan["metadata"]["name"], "default")
        creates = [a for a in c.actions if a.verb == "create"]
        return p, creates
    p, creates = asyncio.run(main())
    assert p["metadata"]["ownerReferences"][0]["uid"] == UID and not creates
