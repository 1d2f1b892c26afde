"""Job and CronJob controllers.

Parity: `pkg/controller/job/job_controller.go` (parallelism / completions / backoffLimit /
activeDeadlineSeconds, conditions Complete / Failed, succeeded / failed / active counts) and
`pkg/controller/cronjob/cronjob_controller.go` + `utils.go` (5-field cron schedule,
concurrencyPolicy Allow / Forbid / Replace, successful/failed history limits, suspend).

GPU jobs are the main MI355X use: a Job whose template requests `amd.com/gpu` runs
`completions` GPU pods, `parallelism` at a time, each admitted with its own device IDs.
"""
from __future__ import annotations

import asyncio
import datetime as dt
import time

from ..api import meta as m
from ..api.meta import now_rfc3339, parse_rfc3339
from ..client.rest import APIStatusError, is_already_exists, is_not_found
from ..api.labels import selector_to_string
from .base import Controller, Expectations, active_pods_key, controller_ref, pod_from_template, split_key


DEFAULT_JOB_BACKOFF = 10.0       # job_controller.go DefaultJobBackOff
MAX_JOB_BACKOFF = 360.0          # MaxJobBackOff


def job_finished(job):
    return any(c.get("type") in ("Complete", "Failed") and c.get("status") == "True"
               for c in (job.get("status") or {}).get("conditions") or ())


def active_pod_rank(p):
    """`controller.ActivePods` order (the pods to delete first come first)."""
    return active_pods_key(p)


class JobController(Controller):
    """`pkg/controller/job/job_controller.go`: pods claimed through the job's selector (orphans
    adopted, non-matching released); a new pod failure re-queues the job with exponential
    backoff (10 s doubling to 360 s) and the job fails with BackoffLimitExceeded once the
    consecutive retries pass backoffLimit; activeDeadlineSeconds is checked at the deadline
    (the job is re-queued for it when it starts); manageJob keeps `parallelism` pods active
    (work-queue jobs — no completions — stop adding pods after the first success) creating in
    slow-start batches and deleting not-ready / unscheduled pods first."""
    name = "job"

    def __init__(self, client, factory, recorder=None, backoff=DEFAULT_JOB_BACKOFF, max_backoff=MAX_JOB_BACKOFF):
        super().__init__(client, factory, recorder)
        from ..parallel.workqueue import ItemExponentialFailureRateLimiter, RateLimitingQueue
        self.queue = RateLimitingQueue(self.name, ItemExponentialFailureRateLimiter(backoff, max_backoff))
        self.backoff, self.max_backoff = backoff, max_backoff

    def setup(self):
        self.exp = Expectations()
        self.job_inf = self.factory.get("jobs")
        self.pod_inf = self.factory.get("pods")
        self.job_inf.add_handler(self.enqueue, self._job_updated, lambda j: self.exp.delete(m.ns_name(j)))
        self.pod_inf.add_handler(self._pod_add, self._pod_update, self._pod_del)

    def _job_updated(self, old, new):
        self.enqueue(new)
        # activeDeadlineSeconds changed on a started job: look again when it passes
        ad = (new.get("spec") or {}).get("activeDeadlineSeconds")
        start = parse_rfc3339((new.get("status") or {}).get("startTime"))
        if ad is not None and start and ad != (old.get("spec") or {}).get("activeDeadlineSeconds"):
            self.queue.add_after(m.ns_name(new), max(0.0, start + int(ad) - time.time()))

    def _job_key(self, pod):
        ref = controller_ref(pod)
        if ref and ref.get("kind") == "Job":
            return f"{pod['metadata']['namespace']}/{ref['name']}"
        return None

    def _jobs_for_orphan(self, pod):
        from ..api.labels import label_selector_as_selector
        labels = pod["metadata"].get("labels") or {}
        for j in self.job_inf.list():
            if m.namespace_of(j) == m.namespace_of(pod):
                sel = label_selector_as_selector((j.get("spec") or {}).get("selector"))
                if not sel.empty() and sel.matches(labels):
                    self.enqueue(j)

    def _enqueue_backoff(self, key, immediate):
        """`enqueueController(job, immediate)`: a pod failure waits out the current backoff."""
        if immediate:
            self.queue.add(key)
            return
        n = self.queue.num_requeues(key)
        delay = 0.0 if n <= 0 else min(self.max_backoff, self.backoff * (2 ** (n - 1)))
        self.queue.add_after(key, delay)

    def _pod_add(self, pod):
        if pod["metadata"].get("deletionTimestamp"):
            self._pod_del(pod)
            return
        k = self._job_key(pod)
        if k:
            self.exp.observe_add(k)
            self.enqueue(k)
        elif controller_ref(pod) is None:
            self._jobs_for_orphan(pod)

    def _pod_update(self, old, new):
        k, ok = self._job_key(new), self._job_key(old)
        if ok and ok != k:
            self.queue.add(ok)
        if k:
            self._enqueue_backoff(k, (new.get("status") or {}).get("phase") != "Failed")
        elif controller_ref(new) is None:
            self._jobs_for_orphan(new)

    def _pod_del(self, pod):
        k = self._job_key(pod)
        if k:
            self.exp.observe_del(k)
            self.enqueue(k)

    async def claim_pods(self, job):
        from ..api.labels import label_selector_as_selector
        sel = label_selector_as_selector((job.get("spec") or {}).get("selector"))
        uid, ns = m.uid_of(job), m.namespace_of(job)
        out = []
        for p in self.pod_inf.list():
            if m.namespace_of(p) != ns:
                continue
            ref = controller_ref(p)
            matches = not sel.empty() and sel.matches(p["metadata"].get("labels") or {})
            if ref is not None:
                if ref.get("uid") != uid:
                    continue
                if matches:
                    out.append(p)
                elif not p["metadata"].get("deletionTimestamp"):
                    refs = [r for r in p["metadata"].get("ownerReferences") or () if r.get("uid") != uid]
                    await self._patch_pod(p, {"metadata": {"ownerReferences": refs or None}})
                continue
            if matches and not job["metadata"].get("deletionTimestamp") and not p["metadata"].get("deletionTimestamp"):
                refs = list(p["metadata"].get("ownerReferences") or ()) + [m.owner_reference(job)]
                adopted = await self._patch_pod(p, {"metadata": {"ownerReferences": refs, "uid": m.uid_of(p)}})
                if adopted is not None:
                    out.append(adopted)
        return out

    async def _patch_pod(self, p, patch):
        try:
            return await self.client.patch("pods", m.name_of(p), patch, m.namespace_of(p))
        except APIStatusError as e:
            if is_not_found(e):
                return None
            raise

    async def _delete(self, p):
        try:
            await self.client.delete("pods", m.name_of(p), m.namespace_of(p))
            return None
        except APIStatusError as e:
            return None if is_not_found(e) else e

    async def sync(self, key):
        job = self.job_inf.get(key)
        if job is None:
            self.exp.delete(key)
            return None
        if job_finished(job):
            return None
        ns, name = split_key(key)
        spec = job.get("spec") or {}
        st = job.get("status") or {}
        previous_retry = self.queue.num_requeues(key)
        needs_sync = self.exp.satisfied(key)
        pods = await self.claim_pods(job)
        active_pods = [p for p in pods if (p.get("status") or {}).get("phase") not in ("Succeeded", "Failed")
                       and not p["metadata"].get("deletionTimestamp")]
        active = len(active_pods)
        succeeded = sum(1 for p in pods if (p.get("status") or {}).get("phase") == "Succeeded")
        failed = sum(1 for p in pods if (p.get("status") or {}).get("phase") == "Failed")
        conds = list(st.get("conditions") or [])
        n_conds = len(conds)
        start = st.get("startTime")
        status_new = {}
        if not start:
            start = now_rfc3339()
            status_new["startTime"] = start
            if spec.get("activeDeadlineSeconds") is not None:
                self.queue.add_after(key, float(spec["activeDeadlineSeconds"]))
        now = now_rfc3339()
        backoff_limit = int(spec.get("backoffLimit", 6))
        new_failure = failed > int(st.get("failed") or 0)
        reason = None
        if new_failure and previous_retry + 1 > backoff_limit:
            reason, msg = "BackoffLimitExceeded", "Job has reached the specified backoff limit"
        elif spec.get("activeDeadlineSeconds") is not None and \
                time.time() - (parse_rfc3339(start) or time.time()) >= int(spec["activeDeadlineSeconds"]):
            reason, msg = "DeadlineExceeded", "Job was active longer than specified deadline"
        manage_err = None
        if reason is not None:
            errs = [e for e in await asyncio.gather(*(self._delete(p) for p in active_pods)) if e is not None]
            manage_err = errs[0] if errs else None
            failed += active
            active = 0
            conds.append({"type": "Failed", "status": "True", "lastProbeTime": now, "lastTransitionTime": now,
                          "reason": reason, "message": msg})
            self.recorder.event(job, "Warning", reason, msg)
        else:
            if needs_sync and not job["metadata"].get("deletionTimestamp"):
                active, manage_err = await self.manage_job(job, key, active_pods, succeeded)
            completions = spec.get("completions")
            complete = False
            if completions is None:
                complete = succeeded > 0 and active == 0
            elif succeeded >= int(completions):
                complete = True
                if active > 0:
                    self.recorder.event(job, "Warning", "TooManyActivePods",
                                        "Too many active pods running after completion count reached")
                if succeeded > int(completions):
                    self.recorder.event(job, "Warning", "TooManySucceededPods",
                                        "Too many succeeded pods running after completion count reached")
            if complete:
                conds.append({"type": "Complete", "status": "True", "lastProbeTime": now, "lastTransitionTime": now})
                status_new["completionTime"] = now
                self.recorder.event(job, "Normal", "Completed", "Job completed")
        forget = False
        if (int(st.get("active") or 0), int(st.get("succeeded") or 0), int(st.get("failed") or 0)) != \
                (active, succeeded, failed) or len(conds) != n_conds or status_new:
            status_new.update({"active": active, "succeeded": succeeded, "failed": failed, "conditions": conds})
            try:
                await self.client.patch("jobs", name, {"status": status_new}, ns, "merge", "status")
            except APIStatusError as e:
                if not is_not_found(e):
                    raise
            if new_failure and not any(c.get("type") in ("Complete", "Failed") for c in conds):
                # re-queue after the backoff period (the retry counts toward backoffLimit)
                raise RuntimeError(f"failed pod(s) detected for job key {key!r}")
            forget = True
        if manage_err is not None:
            raise manage_err
        return None if forget else False

    async def manage_job(self, job, key, active_pods, succeeded):
        spec = job.get("spec") or {}
        ns, name = split_key(key)
        active = len(active_pods)
        parallelism = int(spec.get("parallelism", 1))
        errs = []
        if active > parallelism:
            diff = active - parallelism
            self.exp.expect(key, dels=diff)
            victims = sorted(active_pods, key=active_pod_rank)[:diff]
            res = await asyncio.gather(*(self._delete(p) for p in victims))
            for e in res:
                if e is not None:
                    self.exp.observe_del(key)
                    errs.append(e)
            active -= diff - sum(1 for e in res if e is not None)
        elif active < parallelism:
            completions = spec.get("completions")
            if completions is None:
                want = active if succeeded > 0 else parallelism
            else:
                want = min(int(completions) - succeeded, parallelism)
            diff = max(0, want - active)
            self.exp.expect(key, adds=diff)
            tmpl = spec.get("template") or {}
            batch = min(diff, 1)
            created = 0
            while diff > 0:
                res = await asyncio.gather(*(self.client.create("pods", pod_from_template(tmpl, job, f"{name}-", ns), ns)
                                             for _ in range(batch)), return_exceptions=True)
                bad = [r for r in res if isinstance(r, Exception)]
                for _ in bad:
                    self.exp.observe_add(key)
                created += batch - len(bad)
                errs += bad
                diff -= batch
                if bad and diff > 0:
                    for _ in range(diff):          # slow start: the rest waits for the next sync
                        self.exp.observe_add(key)
                    break
                batch = min(2 * batch, diff)
            if created:
                self.recorder.event(job, "Normal", "SuccessfulCreate", f"Created {created} pods")
            if errs:
                self.recorder.event(job, "Warning", "FailedCreate", f"Error creating: {errs[0]}")
            active += created
        return active, (errs[0] if errs else None)


# ---------------------------------------------------------------------------
_MONTHS = {n: i + 1 for i, n in enumerate(("jan", "feb", "mar", "apr", "may", "jun", "jul", "aug", "sep", "oct",
                                            "nov", "dec"))}
_DOWS = {n: i for i, n in enumerate(("sun", "mon", "tue", "wed", "thu", "fri", "sat"))}


def _field_match(spec, value, lo, hi, names=None):
    """One cron field (robfig/cron `ParseStandard`): `*` / `?`, lists, ranges, steps and, for
    month and day-of-week, three-letter names."""
    def num(x):
        x = x.strip().lower()
        if names and x in names:
            return names[x]
        v = int(x)
        if not lo <= v <= hi:
            raise ValueError(f"cron value {v} out of range [{lo}, {hi}]")
        return v
    for part in spec.split(","):
        step = 1
        if "/" in part:
            part, s = part.split("/", 1)
            step = int(s)
            if step <= 0:
                raise ValueError(f"invalid cron step {s!r}")
        if part in ("*", "?"):
            a, b = lo, hi
        elif "-" in part:
            a, b = (num(x) for x in part.split("-", 1))
        else:
            a = num(part)
            b = hi if step > 1 else a
        if a <= value <= b and (value - a) % step == 0:
            return True
    return False


def cron_matches(expr: str, t: dt.datetime) -> bool:
    """Standard 5-field cron (minute hour dom month dow); @hourly/@daily/@every-minute aliases."""
    aliases = {"@hourly": "0 * * * *", "@daily": "0 0 * * *", "@midnight": "0 0 * * *", "@weekly": "0 0 * * 0",
               "@monthly": "0 0 1 * *", "@yearly": "0 0 1 1 *", "@annually": "0 0 1 1 *"}
    expr = aliases.get(expr.strip(), expr)
    f = expr.split()
    if len(f) != 5:
        raise ValueError(f"invalid cron schedule {expr!r}")
    dow = (t.weekday() + 1) % 7
    return (_field_match(f[0], t.minute, 0, 59) and _field_match(f[1], t.hour, 0, 23) and
            _field_match(f[2], t.day, 1, 31) and _field_match(f[3], t.month, 1, 12, _MONTHS) and
            _field_match(f[4], dow, 0, 6, _DOWS))


class TooManyMissed(ValueError):
    pass


def missed_schedules(expr, since: float, now: float, cap=100):
    """Scheduled times in (since, now], minute resolution (`getRecentUnmetScheduleTimes`);
    more than `cap` raises TooManyMissed — the reference refuses to guess which to start."""
    out = []
    t = dt.datetime.fromtimestamp(since, dt.timezone.utc).replace(second=0, microsecond=0) + dt.timedelta(minutes=1)
    end = dt.datetime.fromtimestamp(now, dt.timezone.utc)
    while t <= end:
        if cron_matches(expr, t):
            out.append(t)
            if len(out) > cap:
                raise TooManyMissed("Too many missed start time (> 100). Set or decrease .spec.startingDeadlineSeconds "
                                    "or check clock skew.")
        t += dt.timedelta(minutes=1)
    return out


def unmet_schedule_times(cj, now: float):
    """`getRecentUnmetScheduleTimes`: from lastScheduleTime (else creation), but no earlier than
    now - startingDeadlineSeconds."""
    spec = cj.get("spec") or {}
    try:                      # cron.ParseStandard first: an unparseable schedule is an error
        cron_matches(spec.get("schedule", ""), dt.datetime.fromtimestamp(now, dt.timezone.utc))
    except ValueError as e:
        raise ValueError(f"Unparseable schedule: {spec.get('schedule', '')} : {e}") from None
    earliest = parse_rfc3339((cj.get("status") or {}).get("lastScheduleTime")) or \
        parse_rfc3339(cj["metadata"].get("creationTimestamp")) or now
    sds = spec.get("startingDeadlineSeconds")
    if sds is not None:
        earliest = max(earliest, now - int(sds))
    if earliest > now:
        return []
    return missed_schedules(spec.get("schedule", ""), earliest, now)


def finished_status(job):
    """(finished, "Complete" | "Failed" | None) — `getFinishedStatus`."""
    for c in (job.get("status") or {}).get("conditions") or ():
        if c.get("type") in ("Complete", "Failed") and c.get("status") == "True":
            return True, c["type"]
    return False, None


def job_from_template(cj, scheduled: dt.datetime):
    """`getJobFromTemplate`: the template's labels and annotations, a name deterministic in the
    scheduled time (`<cronjob>-<unix seconds>`: the same start is never created twice), and a
    controller reference to the CronJob."""
    jt = (cj.get("spec") or {}).get("jobTemplate") or {}
    md = jt.get("metadata") or {}
    return {"apiVersion": "batch/v1", "kind": "Job",
            "metadata": {"name": f"{m.name_of(cj)}-{int(scheduled.timestamp())}", "namespace": m.namespace_of(cj),
                         "labels": dict(md.get("labels") or {}), "annotations": dict(md.get("annotations") or {}),
                         "ownerReferences": [m.owner_reference(cj)]},
            "spec": m.fast_copy(jt.get("spec") or {})}


def _job_ref(job):
    md = job["metadata"]
    return {"kind": "Job", "namespace": md.get("namespace"), "name": md["name"], "uid": md.get("uid"),
            "apiVersion": "batch/v1", "resourceVersion": md.get("resourceVersion")}


class CronJobController(Controller):
    """`pkg/controller/cronjob/cronjob_controller.go`: every 10 s each CronJob is synced
    (`syncAll` → `syncOne` + `cleanupFinishedJobs`):

      * status.active is reconciled with the jobs the CronJob controls — finished ones leave it
        (SawCompletedJob), vanished ones too (MissingJob), unknown running ones are reported
        (UnexpectedJob);
      * deleting or suspended: nothing starts;
      * the latest unmet schedule time starts, unless it is past startingDeadlineSeconds, more than
        100 were missed (FailedNeedsStart), or a run is active under Forbid; under Replace the
        active jobs are deleted first (parallelism 0, their pods, then the job);
      * the created job joins status.active and lastScheduleTime advances;
      * finished jobs beyond successful/failedJobsHistoryLimit are deleted oldest first
        (by status.startTime, then name)."""
    name = "cronjob"
    workers = 1
    SYNC_PERIOD = 10.0

    def setup(self):
        self.cj_inf = self.factory.get("cronjobs")
        self.job_inf = self.factory.get("jobs")
        self.cj_inf.add_handler(self.enqueue, lambda o, n: self.enqueue(n), None)
        self._tick = None

    def start(self):
        super().start()
        self._tick = asyncio.ensure_future(self._ticker())

    def stop(self):
        super().stop()
        if self._tick:
            self._tick.cancel()

    async def _ticker(self):
        while True:
            await asyncio.sleep(self.SYNC_PERIOD)
            for cj in self.cj_inf.list():
                self.enqueue(cj)

    async def _update_status(self, cj, status):
        if (cj.get("status") or {}) == status:
            return cj
        body = dict(cj, status=status)
        return await self.client.update_status("cronjobs", body, m.namespace_of(cj))

    async def delete_job(self, cj, job, reason=""):
        """`deleteJob`: stop the job (parallelism 0), delete its pods, then the job."""
        ns = m.namespace_of(job)
        try:
            if ((job.get("spec") or {}).get("parallelism", 1)) != 0:
                job = m.fast_copy(job)
                job["spec"]["parallelism"] = 0
                job = await self.client.update("jobs", job, ns)
            sel = selector_to_string((job.get("spec") or {}).get("selector") or {})
            for pod in (await self.client.list("pods", ns, label_selector=sel))["items"] if sel else ():
                try:
                    await self.client.delete("pods", m.name_of(pod), ns)
                except APIStatusError as e:
                    if not is_not_found(e):
                        raise
            await self.client.delete("jobs", m.name_of(job), ns)
        except APIStatusError as e:
            self.recorder.event(cj, "Warning", "FailedDelete", f"Deleted job: {e}")
            return False
        self.recorder.event(cj, "Normal", "SuccessfulDelete", f"Deleted job {m.name_of(job)}")
        return True

    async def sync(self, key, now=None):
        cj = self.cj_inf.get(key)
        if cj is None:
            return
        now = now or time.time()
        uid = m.uid_of(cj)
        jobs = [j for j in self.job_inf.list() if (controller_ref(j) or {}).get("uid") == uid]
        await self.sync_one(cj, jobs, now)
        await self.cleanup_finished_jobs(cj, jobs)

    async def sync_one(self, cj, jobs, now):
        status = m.fast_copy(cj.get("status") or {})
        active = list(status.get("active") or ())
        active_uids = {a.get("uid") for a in active}
        children = set()
        for j in jobs:
            children.add(m.uid_of(j))
            done, _ = finished_status(j)
            found = m.uid_of(j) in active_uids
            if not found and not done:
                self.recorder.event(cj, "Warning", "UnexpectedJob",
                                    f"Saw a job that the controller did not create or forgot: {m.name_of(j)}")
            elif found and done:
                active = [a for a in active if a.get("uid") != m.uid_of(j)]
                self.recorder.event(cj, "Normal", "SawCompletedJob", f"Saw completed job: {m.name_of(j)}")
        for a in list(active):
            if a.get("uid") not in children:
                self.recorder.event(cj, "Normal", "MissingJob", f"Active job went missing: {a.get('name')}")
                active = [x for x in active if x.get("uid") != a.get("uid")]
        if active:
            status["active"] = active
        else:
            status.pop("active", None)
        cj = await self._update_status(cj, status)
        spec = cj.get("spec") or {}
        if cj["metadata"].get("deletionTimestamp") or spec.get("suspend"):
            return
        try:
            times = unmet_schedule_times(cj, now)
        except ValueError as e:
            self.recorder.event(cj, "Warning", "FailedNeedsStart", f"Cannot determine if job needs to be started: {e}")
            return
        if not times:
            return
        sched = times[-1]
        sds = spec.get("startingDeadlineSeconds")
        if sds is not None and sched.timestamp() + int(sds) < now:
            return             # missed the starting window
        pol = spec.get("concurrencyPolicy", "Allow")
        if pol == "Forbid" and active:
            return
        if pol == "Replace":
            for a in list(active):
                job = self.job_inf.get(f"{a.get('namespace')}/{a.get('name')}")
                if job is None:
                    try:
                        job = await self.client.get("jobs", a.get("name"), a.get("namespace"))
                    except APIStatusError as e:
                        self.recorder.event(cj, "Warning", "FailedGet", f"Get job: {e}")
                        return
                if not await self.delete_job(cj, job):
                    return
                active = [x for x in active if x.get("uid") != m.uid_of(job)]
        job = job_from_template(cj, sched)
        try:
            created = await self.client.create("jobs", job, m.namespace_of(cj))
        except APIStatusError as e:
            self.recorder.event(cj, "Warning", "FailedCreate", f"Error creating job: {e}")
            if is_already_exists(e):
                return
            raise
        self.recorder.event(cj, "Normal", "SuccessfulCreate", f"Created job {m.name_of(created)}")
        status = m.fast_copy(cj.get("status") or {})
        status["active"] = active + [_job_ref(created)]
        status["lastScheduleTime"] = sched.strftime("%Y-%m-%dT%H:%M:%SZ")
        await self._update_status(cj, status)

    async def cleanup_finished_jobs(self, cj, jobs):
        spec = cj.get("spec") or {}
        for kind, field in (("Complete", "successfulJobsHistoryLimit"), ("Failed", "failedJobsHistoryLimit")):
            lim = spec.get(field)
            if lim is None:
                continue
            done = [j for j in jobs if finished_status(j) == (True, kind)]
            extra = len(done) - int(lim)
            if extra <= 0:
                continue
            # byJobStartTime: started jobs by start time (unstarted last), then name
            done.sort(key=lambda j: (parse_rfc3339((j.get("status") or {}).get("startTime")) is None,
                                     parse_rfc3339((j.get("status") or {}).get("startTime")) or 0, m.name_of(j)))
            for j in done[:extra]:
                await self.delete_job(cj, j, "history limit reached")
