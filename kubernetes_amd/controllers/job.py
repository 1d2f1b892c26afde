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


class JobController(Controller):
    name = "job"

    def setup(self):
        self.exp = Expectations()
        self.job_inf = self.factory.get("jobs")
        self.pod_inf = self.factory.get("pods")
        self.job_inf.add_handler(self.enqueue, lambda o, n: self.enqueue(n), lambda j: self.exp.delete(m.ns_name(j)))
        self.pod_inf.add_handler(self._pod_add, lambda o, n: self._pod_touch(n), self._pod_del)
        if "controllerUID" not in self.pod_inf.store.indexers:
            self.pod_inf.store.add_indexer("controllerUID", lambda p: [r["uid"] for r in (p["metadata"].get("ownerReferences") or ()) if r.get("controller")])

    def _job_key(self, pod):
        ref = controller_ref(pod)
        if ref and ref.get("kind") == "Job":
            return f"{pod['metadata']['namespace']}/{ref['name']}"
        return None

    def _pod_add(self, pod):
        k = self._job_key(pod)
        if k:
            self.exp.observe_add(k)
            self.enqueue(k)

    def _pod_touch(self, pod):
        k = self._job_key(pod)
        if k:
            self.enqueue(k)

    def _pod_del(self, pod):
        k = self._job_key(pod)
        if k:
            self.exp.observe_del(k)
            self.enqueue(k)

    async def sync(self, key):
        job = self.job_inf.get(key)
        if job is None:
            self.exp.delete(key)
            return
        ns, name = split_key(key)
        st = job.get("status") or {}
        if any(c.get("type") in ("Complete", "Failed") and c.get("status") == "True" for c in st.get("conditions") or ()):
            return
        spec = job.get("spec") or {}
        pods = self.pod_inf.store.by_index("controllerUID", job["metadata"]["uid"])
        active = [p for p in pods if (p.get("status") or {}).get("phase") not in ("Succeeded", "Failed")
                  and not p["metadata"].get("deletionTimestamp")]
        succeeded = sum(1 for p in pods if (p.get("status") or {}).get("phase") == "Succeeded")
        failed = sum(1 for p in pods if (p.get("status") or {}).get("phase") == "Failed")
        completions = spec.get("completions")
        parallelism = int(spec.get("parallelism", 1))
        backoff = int(spec.get("backoffLimit", 6))
        start = st.get("startTime") or now_rfc3339()
        now = now_rfc3339()
        conds = list(st.get("conditions") or [])
        finished = None
        deadline = spec.get("activeDeadlineSeconds")
        if deadline is not None and time.time() - (parse_rfc3339(start) or time.time()) > int(deadline):
            finished = ("Failed", "DeadlineExceeded", "Job was active longer than specified deadline")
        elif failed > backoff:
            finished = ("Failed", "BackoffLimitExceeded", "Job has reached the specified backoff limit")
        elif completions is not None and succeeded >= int(completions):
            finished = ("Complete", None, None)
        elif completions is None and succeeded > 0 and not active:
            finished = ("Complete", None, None)
        if finished is not None:
            for p in active:
                try:
                    await self.client.delete("pods", p["metadata"]["name"], ns)
                except APIStatusError:
                    pass
            c = {"type": finished[0], "status": "True", "lastProbeTime": now, "lastTransitionTime": now}
            if finished[1]:
                c["reason"], c["message"] = finished[1], finished[2]
            conds.append(c)
            self.recorder.event(job, "Normal" if finished[0] == "Complete" else "Warning",
                                finished[1] or "Completed", finished[2] or "Job completed")
            active = []
        elif self.exp.satisfied(key):
            want = parallelism
            if completions is not None:
                want = min(parallelism, int(completions) - succeeded)
            diff = want - len(active)
            if diff > 0:
                self.exp.expect(key, adds=diff)
                tmpl = spec.get("template") or {}
                res = await asyncio.gather(*(self.client.create("pods", pod_from_template(tmpl, job, f"{name}-", ns), ns)
                                             for _ in range(diff)), return_exceptions=True)
                for r in res:
                    if isinstance(r, Exception):
                        self.exp.observe_add(key)
                self.recorder.event(job, "Normal", "SuccessfulCreate", f"Created {diff} pods")
            elif diff < 0:
                for p in active[:(-diff)]:
                    try:
                        await self.client.delete("pods", p["metadata"]["name"], ns)
                    except APIStatusError:
                        pass
        newst = {"active": len(active), "succeeded": succeeded, "failed": failed, "startTime": start,
                 "conditions": conds}
        if finished and finished[0] == "Complete":
            newst["completionTime"] = now
        if {k: st.get(k) for k in newst} != newst:
            try:
                await self.client.patch("jobs", name, {"status": newst}, ns, "merge", "status")
            except APIStatusError as e:
                if not is_not_found(e):
                    raise


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
