"""Density load generator and measurement (kubemark density / scheduler_perf equivalent).

Metric definitions follow the reference:
  * startup latency = watch-observed `Running` minus creation (`test/e2e/scalability/density.go:799-803`);
    measured here with a monotonic client clock (create request sent → Running observed on the
    watch), because `creationTimestamp` has 1 s resolution;
  * throughput = pods per second (saturation: all pods Running) and the scheduled-pods rate
    sampled per second (`test/integration/scheduler_perf/scheduler_test.go:131-182`), reporting
    the average and the worst 1-s interval.
"""
from __future__ import annotations

import asyncio
import collections
import time

from ..api import core
from ..client.rest import APIStatusError, Client


def gpu_pod(name, ns, labels, gpus=1, selector=None, annotations=None):
    c = {"name": "gpu", "image": "kubernetes-amd/hip-vector-add:1", "resources": {"limits": {core.AMD_GPU: str(gpus)}}}
    p = {"apiVersion": "v1", "kind": "Pod",
         "metadata": {"name": name, "namespace": ns, "labels": labels, "annotations": dict(annotations or {})},
         "spec": {"containers": [c], "restartPolicy": "Never", "terminationGracePeriodSeconds": 1}}
    if selector:
        p["spec"]["nodeSelector"] = selector
    return p


def pct(vals, q):
    if not vals:
        return float("nan")
    s = sorted(vals)
    k = min(len(s) - 1, max(0, int(round(q * (len(s) - 1)))))
    return s[k]


class DensityRunner:
    def __init__(self, master, rank=0, namespace="density", pods_per_step=64, gpus_per_pod=1, concurrency=128,
                 annotations=None, client_procs=0, workdir=None):
        self.master = master
        self.client = Client(master, max_conns=64)
        # client_procs > 0: creates/deletes are issued by helper processes (density_client.py)
        self.client_procs = client_procs
        self.workdir = workdir
        self.pool = None
        self.rank = rank
        self.ns = namespace
        self.pods_per_step = pods_per_step
        self.gpus_per_pod = gpus_per_pod
        self.concurrency = concurrency
        self.created: dict[str, float] = {}
        self.scheduled: dict[str, float] = {}
        self.running: dict[str, float] = {}
        self.gone: dict[str, float] = {}
        self.assigned: dict[str, tuple] = {}     # pod -> (node, [device ids]) as observed Running
        self.annotations = dict(annotations or {})
        self._watch_task = None
        self._stream = None
        self._changed = asyncio.Event()
        self.selector = f"density-rank={rank}"

    async def start(self):
        try:
            await self.client.create("namespaces", {"metadata": {"name": self.ns}})
        except APIStatusError as e:
            if e.code != 409:
                raise
        lst = await self.client.list("pods", self.ns, label_selector=self.selector)
        self._stream = await self.client.watch("pods", self.ns, lst["metadata"]["resourceVersion"],
                                               label_selector=self.selector)
        self._watch_task = asyncio.ensure_future(self._watch())
        if self.client_procs:
            import tempfile
            from .density_client import HelperPool
            self.pool = await HelperPool(self.master, self.client_procs, self.workdir or tempfile.gettempdir()).start()

    async def _watch(self):
        async for evs in self._stream.batches():
            now = time.monotonic()      # when this read arrived (one timestamp per batch)
            for etype, pod in evs:
                name = pod["metadata"]["name"]
                if etype == "DELETED":
                    self.gone.setdefault(name, now)
                else:
                    if (pod.get("spec") or {}).get("nodeName") and name not in self.scheduled:
                        self.scheduled[name] = now
                    if (pod.get("status") or {}).get("phase") == core.POD_RUNNING and name not in self.running:
                        self.running[name] = now
                        self.assigned[name] = (pod["spec"].get("nodeName"),
                                               [i for ids in core.pod_assigned_devices(pod).values() for i in ids])
            self._changed.set()

    async def _diagnose(self, names, phase):
        """What the pods that never reached `phase` look like (for the timeout error)."""
        missing = [n for n in names if n not in (self.running if phase == "running" else self.gone)]
        out = collections.Counter()
        for n in missing[:50]:
            try:
                p = await self.client.get("pods", n, self.ns)
                st = (p.get("status") or {})
                out[(st.get("phase"), bool((p.get("spec") or {}).get("nodeName")),
                     bool(p["metadata"].get("deletionTimestamp")))] += 1
            except APIStatusError as e:
                out[("http", e.code)] += 1
        return f"{len(missing)} pods not {phase}; sample (phase, bound, deleting): {dict(out)}; " \
               f"watch alive: {self._watch_task is not None and not self._watch_task.done()}"

    async def _wait(self, pred, timeout, names=(), phase=""):
        end = time.monotonic() + timeout
        while not pred():
            left = end - time.monotonic()
            if left <= 0:
                raise TimeoutError("density step timed out: " + await self._diagnose(names, phase))
            self._changed.clear()
            try:
                await asyncio.wait_for(self._changed.wait(), min(left, 1.0))
            except asyncio.TimeoutError:
                pass

    async def step(self, k, timeout=300):
        names = [f"r{self.rank}-s{k}-{i}" for i in range(self.pods_per_step)]
        labels = {"density-rank": str(self.rank), "density-step": str(k)}
        sem = asyncio.Semaphore(self.concurrency)
        t0 = time.monotonic()

        api_lat = {"create": [], "delete": []}

        async def create(n):
            async with sem:
                self.created[n] = t = time.monotonic()
                await self.client.create("pods", gpu_pod(n, self.ns, labels, self.gpus_per_pod,
                                                         annotations=self.annotations), self.ns)
                api_lat["create"].append(time.monotonic() - t)

        if self.pool is not None:
            sent, api_lat["create"] = await self.pool.call("create", self.ns, names, labels=labels,
                                                           gpus=self.gpus_per_pod, annotations=self.annotations)
            self.created.update(sent)
        else:
            await asyncio.gather(*(create(n) for n in names))
        t_created = time.monotonic()
        await self._wait(_all_in(names, self.running), timeout, names, "running")
        t_running = time.monotonic()

        async def delete(n):
            async with sem:
                t = time.monotonic()
                try:
                    await self.client.delete("pods", n, self.ns)
                except APIStatusError as e:
                    if e.code != 404:
                        raise
                api_lat["delete"].append(time.monotonic() - t)

        if self.pool is not None:
            _, api_lat["delete"] = await self.pool.call("delete", self.ns, names)
        else:
            await asyncio.gather(*(delete(n) for n in names))
        t_deleted = time.monotonic()
        await self._wait(_all_in(names, self.gone), timeout, names, "gone")
        t_gone = time.monotonic()
        lat = [self.running[n] - self.created[n] for n in names]
        sched = sorted(self.scheduled[n] for n in names if n in self.scheduled)
        return {"pods": len(names), "names": names, "create_s": t_created - t0, "to_running_s": t_running - t0,
                "delete_issued_s": t_deleted - t0, "cycle_s": t_gone - t0, "latencies": lat,
                "scheduled_times": [s - t0 for s in sched], "scheduled_at": sched,
                "running_at": sorted(self.running[n] for n in names), "api_latencies": api_lat}

    async def stop(self):
        if self.pool is not None:
            await self.pool.stop()
        if self._stream:
            self._stream.close()
        if self._watch_task:
            self._watch_task.cancel()
        await self.client.close()


def interval_rates(times, bucket=1.0, start=0.0, end=None):
    """Pods per 1-s interval (scheduler_perf samples the scheduled count once per second,
    `test/integration/scheduler_perf/scheduler_test.go:131-182`): (avg, min) over the FULL
    intervals of [start, end]. With no full interval (a run shorter than one second) the min is
    not measurable and is reported as None."""
    if end is None:
        end = max(times) if times else start
    n = int((end - start) // bucket)
    if n < 1:
        return (len(times) / max(end - start, 1e-9) if times else 0.0), None
    counts = [0] * n
    for t in times:
        k = int((t - start) // bucket)
        if 0 <= k < n:
            counts[k] += 1
    return sum(counts) / (n * bucket), min(counts) / bucket


def _all_in(names, seen):
    """A predicate "every name is in `seen`" that re-checks only the names still missing (it is
    evaluated after every watch batch)."""
    pending = list(names)

    def pred():
        pending[:] = [n for n in pending if n not in seen]
        return not pending
    return pred
