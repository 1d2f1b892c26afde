"""CronJob controller: the `pkg/controller/cronjob/cronjob_controller_test.go` TestSyncOne table
(concurrency policy x suspend x schedule validity x starting deadline x previous/active runs x
"now", counting creates, deletes, events, warnings and the final active list), the history
limits (TestCleanupFinishedJobs: oldest finished jobs by start time go first) and the cron
parser (`?`, names, steps)."""
import asyncio
import datetime as dt

import pytest

from kubernetes_amd.client.fake import FakeClient
from kubernetes_amd.client.informer import InformerFactory
from kubernetes_amd.controllers.job import CronJobController, cron_matches, job_from_template

ON_THE_HOUR, ERROR_SCHEDULE = "0 * * * ?", "obvious error schedule"
SHORT, MEDIUM, LONG, NONE = 10, 2 * 60 * 60, 1000000, None
A, F, R = "Allow", "Forbid", "Replace"


def ts(s):
    return dt.datetime.strptime(s, "%Y-%m-%dT%H:%M:%SZ").replace(tzinfo=dt.timezone.utc)


JUST_BEFORE, JUST_AFTER = ts("2016-05-19T09:59:00Z"), ts("2016-05-19T10:01:00Z")
WEEK_AFTER = ts("2016-05-26T10:00:00Z")
BEFORE_PRIOR, AFTER_PRIOR = ts("2016-05-19T08:59:00Z"), ts("2016-05-19T09:01:00Z")


def rfc(t):
    return t.strftime("%Y-%m-%dT%H:%M:%SZ")


def cron_job(policy=A, suspend=False, schedule=ON_THE_HOUR, deadline=NONE):
    spec = {"schedule": schedule, "concurrencyPolicy": policy, "suspend": suspend,
            "jobTemplate": {"metadata": {"labels": {"a": "b"}, "annotations": {"x": "y"}},
                            "spec": {"template": {"spec": {"containers": [{"name": "c", "image": "foo/bar"}]}}}}}
    if deadline is not None:
        spec["startingDeadlineSeconds"] = deadline
    return {"apiVersion": "batch/v1beta1", "kind": "CronJob",
            "metadata": {"name": "mycronjob", "namespace": "snazzycats", "uid": "1a2b3c",
                         "creationTimestamp": rfc(JUST_BEFORE)}, "spec": spec}


# name: (policy, suspend, schedule, deadline, ran previously, still active, now,
#        expect create, expect delete, expect active, expected warnings)
T, Fa = True, False
CASES = {
    "never ran, not valid schedule, A": (A, Fa, ERROR_SCHEDULE, NONE, Fa, Fa, JUST_BEFORE, Fa, Fa, 0, 1),
    "never ran, not valid schedule, F": (F, Fa, ERROR_SCHEDULE, NONE, Fa, Fa, JUST_BEFORE, Fa, Fa, 0, 1),
    "never ran, not time, A": (A, Fa, ON_THE_HOUR, NONE, Fa, Fa, JUST_BEFORE, Fa, Fa, 0, 0),
    "never ran, not time, R": (R, Fa, ON_THE_HOUR, NONE, Fa, Fa, JUST_BEFORE, Fa, Fa, 0, 0),
    "never ran, is time, A": (A, Fa, ON_THE_HOUR, NONE, Fa, Fa, JUST_AFTER, T, Fa, 1, 0),
    "never ran, is time, F": (F, Fa, ON_THE_HOUR, NONE, Fa, Fa, JUST_AFTER, T, Fa, 1, 0),
    "never ran, is time, R": (R, Fa, ON_THE_HOUR, NONE, Fa, Fa, JUST_AFTER, T, Fa, 1, 0),
    "never ran, is time, suspended": (A, T, ON_THE_HOUR, NONE, Fa, Fa, JUST_AFTER, Fa, Fa, 0, 0),
    "never ran, is time, past deadline": (A, Fa, ON_THE_HOUR, SHORT, Fa, Fa, JUST_AFTER, Fa, Fa, 0, 0),
    "never ran, is time, not past deadline": (A, Fa, ON_THE_HOUR, LONG, Fa, Fa, JUST_AFTER, T, Fa, 1, 0),
    "prev ran but done, not time, A": (A, Fa, ON_THE_HOUR, NONE, T, Fa, JUST_BEFORE, Fa, Fa, 0, 0),
    "prev ran but done, is time, A": (A, Fa, ON_THE_HOUR, NONE, T, Fa, JUST_AFTER, T, Fa, 1, 0),
    "prev ran but done, is time, F": (F, Fa, ON_THE_HOUR, NONE, T, Fa, JUST_AFTER, T, Fa, 1, 0),
    "prev ran but done, is time, R": (R, Fa, ON_THE_HOUR, NONE, T, Fa, JUST_AFTER, T, Fa, 1, 0),
    "prev ran but done, is time, suspended": (A, T, ON_THE_HOUR, NONE, T, Fa, JUST_AFTER, Fa, Fa, 0, 0),
    "prev ran but done, is time, past deadline": (A, Fa, ON_THE_HOUR, SHORT, T, Fa, JUST_AFTER, Fa, Fa, 0, 0),
    "prev ran but done, is time, not past deadline": (A, Fa, ON_THE_HOUR, LONG, T, Fa, JUST_AFTER, T, Fa, 1, 0),
    "still active, not time, A": (A, Fa, ON_THE_HOUR, NONE, T, T, JUST_BEFORE, Fa, Fa, 1, 0),
    "still active, not time, R": (R, Fa, ON_THE_HOUR, NONE, T, T, JUST_BEFORE, Fa, Fa, 1, 0),
    "still active, is time, A": (A, Fa, ON_THE_HOUR, NONE, T, T, JUST_AFTER, T, Fa, 2, 0),
    "still active, is time, F": (F, Fa, ON_THE_HOUR, NONE, T, T, JUST_AFTER, Fa, Fa, 1, 0),
    "still active, is time, R": (R, Fa, ON_THE_HOUR, NONE, T, T, JUST_AFTER, T, T, 1, 0),
    "still active, is time, suspended": (A, T, ON_THE_HOUR, NONE, T, T, JUST_AFTER, Fa, Fa, 1, 0),
    "still active, is time, past deadline": (A, Fa, ON_THE_HOUR, SHORT, T, T, JUST_AFTER, Fa, Fa, 1, 0),
    "still active, is time, not past deadline": (A, Fa, ON_THE_HOUR, LONG, T, T, JUST_AFTER, T, Fa, 2, 0),
    "prev ran but done, long overdue, not past deadline, A": (A, Fa, ON_THE_HOUR, LONG, T, Fa, WEEK_AFTER, Fa, Fa, 0, 1),
    "prev ran but done, long overdue, no deadline, R": (R, Fa, ON_THE_HOUR, NONE, T, Fa, WEEK_AFTER, Fa, Fa, 0, 1),
    "prev ran but done, long overdue, past medium deadline, A": (A, Fa, ON_THE_HOUR, MEDIUM, T, Fa, WEEK_AFTER, T, Fa, 1, 0),
    "prev ran but done, long overdue, past short deadline, F": (F, Fa, ON_THE_HOUR, SHORT, T, Fa, WEEK_AFTER, T, Fa, 1, 0),
}


@pytest.mark.parametrize("name", list(CASES))
def test_sync_one(name):
    (policy, suspend, schedule, deadline, ran, active, now,
     exp_create, exp_delete, exp_active, exp_warnings) = CASES[name]
    cj = cron_job(policy, suspend, schedule, deadline)
    jobs = []
    if ran:
        cj["metadata"]["creationTimestamp"] = rfc(BEFORE_PRIOR)
        cj["status"] = {"lastScheduleTime": rfc(AFTER_PRIOR)}
        job = job_from_template(cj, AFTER_PRIOR)
        job["metadata"]["uid"] = "1234"
        job["spec"]["parallelism"] = 1
        job["spec"]["selector"] = {"matchLabels": {"controller-uid": "1234"}}
        if active:
            cj["status"]["active"] = [{"kind": "Job", "name": job["metadata"]["name"], "namespace": "snazzycats",
                                       "uid": "1234"}]
            jobs.append(job)

    async def main():
        c = FakeClient(cj, *jobs)
        f = InformerFactory(c)
        ctl = CronJobController(c, f)
        ctl.setup()
        events = []
        ctl.recorder.event = lambda obj, typ, reason, msg: events.append((typ, reason))
        f.start()
        await f.wait_for_cache_sync()
        await ctl.sync_one(await c.get("cronjobs", "mycronjob", "snazzycats"), jobs, now.timestamp())
        creates = [a for a in c.actions if a.verb == "create" and a.resource == "jobs"]
        deletes = [a for a in c.actions if a.verb == "delete" and a.resource == "jobs"]
        final = await c.get("cronjobs", "mycronjob", "snazzycats")
        return creates, deletes, events, final, c
    creates, deletes, events, final, c = asyncio.run(main())
    assert len(creates) == (1 if exp_create else 0), (name, creates)
    assert len(deletes) == (1 if exp_delete else 0), (name, deletes)
    warnings = [e for e in events if e[0] == "Warning"]
    assert len(warnings) == exp_warnings, (name, events)
    assert len(events) == int(exp_create) + int(exp_delete) + exp_warnings, (name, events)
    assert len((final.get("status") or {}).get("active") or ()) == exp_active, (name, final.get("status"))
    if exp_create:
        made = [o for (ns, n), o in c.objects["jobs"].items() if o["metadata"].get("uid") != "1234"][0]
        ref = made["metadata"]["ownerReferences"][0]
        assert (ref["apiVersion"], ref["kind"], ref["name"], ref["uid"], ref["controller"]) == \
            ("batch/v1beta1", "CronJob", "mycronjob", "1a2b3c", True)
        assert made["metadata"]["labels"] == {"a": "b"} and made["metadata"]["annotations"] == {"x": "y"}
        assert final["status"]["lastScheduleTime"] == rfc(now.replace(minute=0, second=0))


def _finished(name, kind, start):
    j = {"apiVersion": "batch/v1", "kind": "Job",
         "metadata": {"name": name, "namespace": "snazzycats", "uid": f"u-{name}",
                      "ownerReferences": [{"apiVersion": "batch/v1beta1", "kind": "CronJob", "name": "mycronjob",
                                           "uid": "1a2b3c", "controller": True}]},
         "spec": {"parallelism": 1, "selector": {"matchLabels": {"job": name}}},
         "status": {"conditions": [{"type": kind, "status": "True"}]}}
    if start:
        j["status"]["startTime"] = start
    return j


def test_cleanup_finished_jobs_keeps_the_newest():
    cj = cron_job()
    cj["spec"]["successfulJobsHistoryLimit"] = 1
    cj["spec"]["failedJobsHistoryLimit"] = 1
    jobs = [_finished("s1", "Complete", "2016-05-19T04:00:00Z"), _finished("s2", "Complete", "2016-05-19T05:00:00Z"),
            _finished("s3", "Complete", None),
            _finished("f1", "Failed", "2016-05-19T04:00:00Z"), _finished("f2", "Failed", "2016-05-19T06:00:00Z")]

    async def main():
        c = FakeClient(cj, *jobs)
        f = InformerFactory(c)
        ctl = CronJobController(c, f)
        ctl.setup()
        f.start()
        await f.wait_for_cache_sync()
        await ctl.cleanup_finished_jobs(cj, jobs)
        return sorted(n for (_, n) in c.objects.get("jobs", {}))
    # byJobStartTime puts unstarted jobs last: s3 is "newest" and survives
    assert asyncio.run(main()) == ["f2", "s3"]


def test_no_history_limit_keeps_everything():
    cj = cron_job()
    jobs = [_finished("s1", "Complete", "2016-05-19T04:00:00Z"), _finished("s2", "Complete", "2016-05-19T05:00:00Z")]

    async def main():
        c = FakeClient(cj, *jobs)
        f = InformerFactory(c)
        ctl = CronJobController(c, f)
        ctl.setup()
        f.start()
        await f.wait_for_cache_sync()
        await ctl.cleanup_finished_jobs(cj, jobs)
        return len(c.objects.get("jobs", {}))
    assert asyncio.run(main()) == 2


@pytest.mark.parametrize("expr,when,want", [
    ("0 * * * ?", "2016-05-19T10:00:00Z", True), ("0 * * * ?", "2016-05-19T10:01:00Z", False),
    ("*/15 9-17 * * mon-fri", "2016-05-19T09:45:00Z", True), ("*/15 9-17 * * mon-fri", "2016-05-21T09:45:00Z", False),
    ("0 0 1 jan *", "2017-01-01T00:00:00Z", True), ("5/20 * * * *", "2016-05-19T10:45:00Z", True),
    ("@hourly", "2016-05-19T10:00:00Z", True)])
def test_cron_matches(expr, when, want):
    assert cron_matches(expr, ts(when)) is want


@pytest.mark.parametrize("expr", ["obvious error schedule", "61 * * * *", "* * * * 9", "*/0 * * * *"])
def test_cron_rejects(expr):
    with pytest.raises(ValueError):
        cron_matches(expr, ts("2016-05-19T10:00:00Z"))
