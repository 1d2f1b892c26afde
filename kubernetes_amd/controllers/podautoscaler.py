"""HorizontalPodAutoscaler controller.

Parity: `pkg/controller/podautoscaler/horizontal.go` + `replica_calculator.go`:
  * resync every `--horizontal-pod-autoscaler-sync-period` (30 s);
  * metrics: autoscaling/v1 `targetCPUUtilizationPercentage` and v2beta1-style `spec.metrics`
    (`Resource` with `targetAverageUtilization` / `targetAverageValue`); the desired count is the
    max over metrics (`computeReplicasForMetrics`);
  * utilization = sum(usage) / sum(requests) over ready pods; unready pods and pods without
    metrics are treated conservatively (0 % on scale-up, 100 % of request on scale-down for
    missing pods), a change within `tolerance` (0.1) is ignored (`GetResourceReplicas` :56-161);
  * scale-up is limited to max(2 x current, 4) per step (`scaleUpLimitFactor/Minimum` :52-53),
    clamped to [minReplicas (default 1), maxReplicas]; no rescale inside the up-/down-scale
    forbidden windows (3 min / 5 min) after `lastScaleTime` (`shouldScale` :553-575);
  * status: currentReplicas, desiredReplicas, currentCPUUtilizationPercentage, lastScaleTime;
  * the target is read and scaled through its `scale` subresource (autoscaling/v1 Scale:
    replicas + selector string), as `horizontal.go` does with its ScaleNamespacer.
Metrics come from `metrics.k8s.io/v1beta1` PodMetrics through the API server (metrics-server).
MI355X: the resource name `amd.com/gpu` scales on GPU utilization — the per-pod GPU duty cycle
in percent, so `targetAverageUtilization: 70` keeps the pods' MI355Xs ~70 % busy.
"""
from __future__ import annotations

import asyncio
import json
import math
import time

from ..api.labels import parse as parse_labels, selector_to_string
from ..api.meta import now_rfc3339, parse_rfc3339
from ..api.quantity import parse_quantity
from ..client.rest import APIStatusError
from .base import Controller, pod_is_ready, split_key

TARGETS = {"Deployment": "deployments", "ReplicaSet": "replicasets", "ReplicationController": "replicationcontrollers",
           "StatefulSet": "statefulsets"}
GPU = "amd.com/gpu"


selector_string = selector_to_string


def utilization_replicas(current, target_util, usage, requests, ready, unready, missing, tolerance):
    """replica_calculator.GetResourceReplicas; usage/requests in the same unit per pod name."""
    metrics = {p: v for p, v in usage.items() if p in ready}
    if not metrics:
        raise ValueError("did not receive metrics for any ready pods")
    ratio = sum(metrics.values()) / max(1e-12, sum(requests[p] for p in metrics)) * 100 / target_util
    util = int(sum(metrics.values()) * 100 / max(1e-12, sum(requests[p] for p in metrics)))
    rebalance = bool(unready) and ratio > 1.0
    if not rebalance and not missing:
        if abs(1.0 - ratio) <= tolerance:
            return current, util
        return int(math.ceil(ratio * len(metrics))), util
    if missing:
        for p in missing:
            metrics[p] = requests[p] if ratio < 1.0 else 0.0
    if rebalance:
        for p in unready:
            metrics[p] = 0.0
    new_ratio = sum(metrics.values()) / max(1e-12, sum(requests[p] for p in metrics)) * 100 / target_util
    if abs(1.0 - new_ratio) <= tolerance or (ratio < 1.0 < new_ratio) or (ratio > 1.0 > new_ratio):
        return current, util
    return int(math.ceil(new_ratio * len(metrics))), util


class HorizontalController(Controller):
    name = "horizontalpodautoscaling"
    workers = 2

    def __init__(self, client, factory, sync_period=30.0, tolerance=0.1, upscale_window=180.0, downscale_window=300.0,
                 **kw):
        super().__init__(client, factory, **kw)
        self.sync_period = sync_period
        self.tolerance = tolerance
        self.upscale_window = upscale_window
        self.downscale_window = downscale_window
        self._tick = None

    def setup(self):
        self.hpa_inf = self.factory.get("horizontalpodautoscalers")
        self.pod_inf = self.factory.get("pods")
        self.hpa_inf.add_handler(self.enqueue, lambda o, n: self.enqueue(n), None)

    def start(self):
        super().start()
        self._tick = asyncio.ensure_future(self._ticker())

    def stop(self):
        super().stop()
        if self._tick:
            self._tick.cancel()

    async def _ticker(self):
        while True:
            await asyncio.sleep(self.sync_period)
            for h in self.hpa_inf.list():
                self.enqueue(h)

    async def _pod_metrics(self, ns, selector):
        path = f"/apis/metrics.k8s.io/v1beta1/namespaces/{ns}/pods"
        if selector:
            from urllib.parse import quote
            path += "?labelSelector=" + quote(selector)
        st, body = await self.client.raw("GET", path)
        if st != 200:
            raise ValueError(f"unable to get metrics: HTTP {st}")
        return {i["metadata"]["name"]: i for i in json.loads(body).get("items") or ()}

    def _metric_specs(self, spec):
        if spec.get("metrics"):
            return spec["metrics"]
        return [{"type": "Resource", "resource": {"name": "cpu",
                                                  "targetAverageUtilization": spec.get("targetCPUUtilizationPercentage", 80)}}]

    async def sync(self, key):
        hpa = self.hpa_inf.get(key)
        if hpa is None:
            return
        ns, name = split_key(key)
        spec = hpa.get("spec") or {}
        ref = spec.get("scaleTargetRef") or {}
        plural = TARGETS.get(ref.get("kind"))
        if plural is None:
            self.recorder.event(hpa, "Warning", "FailedGetScale", f"unsupported scale target kind {ref.get('kind')}")
            return
        try:
            scale = await self.client.get(plural, ref.get("name"), ns, subresource="scale")
        except APIStatusError as e:
            self.recorder.event(hpa, "Warning", "FailedGetScale", str(e))
            return
        current = int((scale.get("spec") or {}).get("replicas", 1))
        sel_str = (scale.get("status") or {}).get("selector") or ""
        if not sel_str:
            self.recorder.event(hpa, "Warning", "SelectorRequired", "selector is required")
            return
        sel = parse_labels(sel_str)
        pods = [p for p in self.pod_inf.list() if p["metadata"].get("namespace") == ns and
                sel.matches(p["metadata"].get("labels") or {}) and not p["metadata"].get("deletionTimestamp")
                and (p.get("status") or {}).get("phase") not in ("Succeeded", "Failed")]
        desired, cpu_util = current, None
        if current == 0:
            desired = 0     # autoscaling disabled for a target scaled to zero
        else:
            try:
                pm = await self._pod_metrics(ns, sel_str)
                best = 0
                for ms in self._metric_specs(spec):
                    if ms.get("type") != "Resource":
                        continue
                    r, util = self._resource_replicas(current, ms["resource"], pods, pm)
                    if ms["resource"].get("name") == "cpu":
                        cpu_util = util
                    best = max(best, r)
                desired = best or current
            except ValueError as e:
                self.recorder.event(hpa, "Warning", "FailedGetResourceMetric", str(e))
                desired = current
        lo, hi = int(spec.get("minReplicas") or 1), int(spec.get("maxReplicas") or current)
        if desired > current:
            desired = min(desired, max(2 * current, 4))
        desired = max(lo, min(hi, desired))
        st = hpa.get("status") or {}
        now = time.time()
        last = parse_rfc3339(st.get("lastScaleTime")) if st.get("lastScaleTime") else None
        rescale = desired != current
        if rescale and last is not None:
            if desired < current and now - last < self.downscale_window:
                rescale = False
            if desired > current and now - last < self.upscale_window:
                rescale = False
        new_st = {"currentReplicas": current, "desiredReplicas": desired if rescale else current,
                  "observedGeneration": hpa["metadata"].get("generation", 1)}
        if cpu_util is not None:
            new_st["currentCPUUtilizationPercentage"] = cpu_util
        if rescale:
            scale["spec"] = {"replicas": desired}
            try:
                await self.client.update(plural, scale, ns, subresource="scale")
            except APIStatusError as e:
                self.recorder.event(hpa, "Warning", "FailedRescale", f"New size: {desired}; error: {e}")
                raise
            self.recorder.event(hpa, "Normal", "SuccessfulRescale", f"New size: {desired}; reason: metric above/below target")
            new_st["lastScaleTime"] = now_rfc3339()
            new_st["currentReplicas"] = current
        elif st.get("lastScaleTime"):
            new_st["lastScaleTime"] = st["lastScaleTime"]
        if {k: st.get(k) for k in new_st} != new_st:
            await self.client.patch("horizontalpodautoscalers", name, {"status": new_st}, ns, "merge", "status")

    def _resource_replicas(self, current, res, pods, pm):
        rname = res.get("name")
        usage, requests, ready, unready, missing = {}, {}, set(), set(), set()
        for p in pods:
            pn = p["metadata"]["name"]
            if rname == GPU:
                req = 100.0 * sum(1 for _ in (p.get("spec") or {}).get("extendedResources") or ()) or 0.0
                req = req or (100.0 if any(GPU in ((c.get("resources") or {}).get("limits") or {})
                                           for c in (p.get("spec") or {}).get("containers") or ()) else 0.0)
            else:
                req = 0.0
                for c in (p.get("spec") or {}).get("containers") or ():
                    q = ((c.get("resources") or {}).get("requests") or {}).get(rname)
                    if q is None:
                        if "targetAverageUtilization" in res:
                            raise ValueError(f"missing request for {rname} on container {c['name']} in pod {ns_of(p)}/{pn}")
                        continue
                    req += float(parse_quantity(str(q)).value)
            requests[pn] = req
            if (p.get("status") or {}).get("phase") != "Running" or not pod_is_ready(p):
                unready.add(pn)
                continue
            m = pm.get(pn)
            if m is None:
                missing.add(pn)
                continue
            ready.add(pn)
            if rname == GPU:
                vals = [float(c["usage"][GPU]) for c in m.get("containers") or () if GPU in (c.get("usage") or {})]
                usage[pn] = sum(vals) / len(vals) if vals else 0.0
            else:
                usage[pn] = sum(float(parse_quantity(str((c.get("usage") or {}).get(rname, "0"))).value)
                                for c in m.get("containers") or ())
        if "targetAverageValue" in res:
            target = float(parse_quantity(str(res["targetAverageValue"])).value)
            if not usage:
                raise ValueError("did not receive metrics for any ready pods")
            ratio = (sum(usage.values()) / len(usage)) / max(1e-12, target)
            if abs(1 - ratio) <= self.tolerance:
                return current, None
            return int(math.ceil(ratio * len(usage))), None
        return utilization_replicas(current, float(res.get("targetAverageUtilization", 80)), usage, requests,
                                    ready, unready, missing, self.tolerance)


def ns_of(p):
    return p["metadata"].get("namespace", "")
