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
from .base import Controller, Expectations, controller_ref, pod_from_template, split_key


DEFAULT_JOB_BACKOFF = 10.0       # job_controller.go DefaultJobBackOff
MAX_JOB_BACKOFF = 360.0          # MaxJobBackOff


def job_finished(job):
    return any(c.get("type") in ("Complete", "Failed") and c.get("status") == "True"
               for c in (job.get("status") or {}).get("conditions") or ())


def active_pod_rank(p):
    """`controller.ActivePods` order: unassigned < assigned, pending < unknown < running,
    not-ready < ready, newer first — the pods to delete first come first."""
    st = p.get("status") or {}
    phase = {"Pending": 0, "Unknown": 1, "Running": 2}.get(st.get("phase"), 0)
    ready = any(c.get("type") == "Ready" and c.get("status") == "True" for c in st.get("conditions") or ())
    return (1 if (p.get("spec") or {}).get("nodeName") else 0, phase, 1 if ready else 0,
            -(parse_rfc3339(p["metadata"].get("creationTimestamp")) or 0))


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
def _field_match(spec, value, lo, hi):
    for part in spec.split(","):
        step = 1
        if "/" in part:
            part, s = part.split("/", 1)
            step = int(s)
        if part == "*":
            a, b = lo, hi
        elif "-" in part:
            a, b = (int(x) for x in part.split("-", 1))
        else:
            a = b = int(part)
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
            _field_match(f[2], t.day, 1, 31) and _field_match(f[3], t.month, 1, 12) and _field_match(f[4], dow, 0, 6))


def missed_schedules(expr, since: float, now: float, cap=100):
    """Scheduled times in (since, now], minute resolution (getRecentUnmetScheduleTimes)."""
    out = []
    t = dt.datetime.fromtimestamp(since, dt.timezone.utc).replace(second=0, microsecond=0) + dt.timedelta(minutes=1)
    end = dt.datetime.fromtimestamp(now, dt.timezone.utc)
    while t <= end and len(out) < cap:
        if cron_matches(expr, t):
            out.append(t)
        t += dt.timedelta(minutes=1)
    return out


class CronJobController(Controller):
    name = "cronjob"
    workers = 1

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
            await asyncio.sleep(10)   # reference syncs every 10 s
            for cj in self.cj_inf.list():
                self.enqueue(cj)

    async def sync(self, key, now=None):
        cj = self.cj_inf.get(key)
        if cj is None:
            return
        ns, name = split_key(key)
        spec = cj.get("spec") or {}
        now = now or time.time()
        uid = cj["metadata"]["uid"]
        jobs = [j for j in self.job_inf.list() if (controller_ref(j) or {}).get("uid") == uid]
        running = [j for j in jobs if not any(c.get("type") in ("Complete", "Failed") and c.get("status") == "True"
                                             for c in (j.get("status") or {}).get("conditions") or ())]
        # history limits
        for kind, lim in (("Complete", spec.get("successfulJobsHistoryLimit", 3)), ("Failed", spec.get("failedJobsHistoryLimit", 1))):
            done = [j for j in jobs if any(c.get("type") == kind and c.get("status") == "True" for c in (j.get("status") or {}).get("conditions") or ())]
            done.sort(key=lambda j: j["metadata"].get("creationTimestamp", ""))
            for j in done[:max(0, len(done) - int(lim))]:
                try:
                    await self.client.delete("jobs", j["metadata"]["name"], ns, propagation="Background")
                except APIStatusError:
                    pass
        if spec.get("suspend"):
            return
        last = parse_rfc3339((cj.get("status") or {}).get("lastScheduleTime")) or parse_rfc3339(cj["metadata"].get("creationTimestamp")) or now
        times = missed_schedules(spec.get("schedule", ""), last, now)
        if not times:
            return
        sched = times[-1]
        sds = spec.get("startingDeadlineSeconds")
        if sds is not None and now - sched.timestamp() > int(sds):
            return
        pol = spec.get("concurrencyPolicy", "Allow")
        if running and pol == "Forbid":
            return
        if running and pol == "Replace":
            for j in running:
                try:
                    await self.client.delete("jobs", j["metadata"]["name"], ns, propagation="Background")
                except APIStatusError:
                    pass
        jt = spec.get("jobTemplate") or {}
        jname = f"{name}-{int(sched.timestamp() // 60)}"
        job = {"apiVersion": "batch/v1", "kind": "Job",
               "metadata": {"name": jname, "namespace": ns, "labels": dict((jt.get("metadata") or {}).get("labels") or {}),
                            "annotations": {"cronjob.kubernetes.io/scheduled-time": sched.strftime("%Y-%m-%dT%H:%M:%SZ")},
                            "ownerReferences": [m.owner_reference(cj)]},
               "spec": m.fast_copy(jt.get("spec") or {})}
        try:
            await self.client.create("jobs", job, ns)
            self.recorder.event(cj, "Normal", "SuccessfulCreate", f"Created job {jname}")
        except APIStatusError as e:
            if not is_already_exists(e):
                raise
        await self.client.patch("cronjobs", name, {"status": {"lastScheduleTime": sched.strftime("%Y-%m-%dT%H:%M:%SZ")}},
                                ns, "merge", "status")
