"""HorizontalPodAutoscaler controller.

Parity: `pkg/controller/podautoscaler/horizontal.go` + `replica_calculator.go` +
`metrics/utilization.go`:
  * resync every `--horizontal-pod-autoscaler-sync-period` (30 s);
  * the target is read and scaled through its `scale` subresource (autoscaling/v1 Scale:
    replicas + selector string), as `horizontal.go` does with its ScaleNamespacer;
    `currentReplicas` is the scale's status, a spec of 0 disables autoscaling (ScalingActive
    False ScalingDisabled), replicas outside [minReplicas, maxReplicas] are brought back first;
  * metrics (`computeReplicasForMetrics`): `Resource` (targetAverageUtilization over the pods'
    requests, or targetAverageValue), `Pods` and `Object` (custom.metrics.k8s.io); the largest
    proposal wins; autoscaling/v1 `targetCPUUtilizationPercentage` is the default CPU metric;
  * replica calculation (`GetResourceReplicas`, `calcPlainMetricReplicas`,
    `GetObjectMetricReplicas`) in integer milli-units like the reference: utilization truncated
    to a whole percent, unready pods (not Running or not Ready) left out and, on a scale-up,
    counted at 0; pods without metrics counted at 100 % of request on a scale-down and 0 % on a
    scale-up; no change within `tolerance` (0.1) or when the correction flips direction;
  * `normalizeDesiredReplicas`: [max(1, minReplicas), min(maxReplicas, max(2 x current, 4))]
    with ScalingLimited (TooFewReplicas / TooManyReplicas / ScaleUpLimit / DesiredWithinRange);
  * forbidden windows after `lastScaleTime` (3 min up, 5 min down: `shouldScale`) with
    AbleToScale BackoffUpscale / BackoffDownscale / BackoffBoth / ReadyForNewScale, and
    SucceededGetScale / FailedGetScale / SucceededRescale / FailedUpdateScale;
  * status: currentReplicas, desiredReplicas, lastScaleTime, currentMetrics, conditions,
    currentCPUUtilizationPercentage (the autoscaling/v1 field), written only on a change;
  * events: SuccessfulRescale / FailedRescale ("New size: N; reason: ..."), FailedGetScale,
    FailedGet{Resource,Pods,Object}Metric, FailedComputeMetricsReplicas, SelectorRequired,
    InvalidSelector, InvalidMetricSourceType.
Metrics come from `metrics.k8s.io/v1beta1` PodMetrics through the API server (metrics-server)
and from `custom.metrics.k8s.io/v1beta1` when an adapter serves it.
MI355X: the resource name `amd.com/gpu` scales on GPU utilization — each pod's request is 100 %
per GPU and its usage the pod's GPU duty cycle in percent (metrics-server reports it per
container, averaged over the container's GPUs), so `targetAverageUtilization: 70` keeps the pods'
MI355Xs ~70 % busy.
"""
from __future__ import annotations

import asyncio
import json
import math
import time
from urllib.parse import quote

from ..api import meta as m
from ..api.labels import SelectorError, parse as parse_labels, selector_to_string
from ..api.meta import now_rfc3339, parse_rfc3339
from ..api.quantity import parse_quantity
from ..client.rest import APIStatusError
from .base import Controller, pod_is_ready, split_key

TARGETS = {"Deployment": "deployments", "ReplicaSet": "replicasets", "ReplicationController": "replicationcontrollers",
           "StatefulSet": "statefulsets"}
GPU = "amd.com/gpu"
SCALE_UP_LIMIT_FACTOR, SCALE_UP_LIMIT_MINIMUM = 2.0, 4.0
CONDITIONS_ANN = "autoscaling.alpha.kubernetes.io/conditions"
CURRENT_METRICS_ANN = "autoscaling.alpha.kubernetes.io/current-metrics"

selector_string = selector_to_string


def milli(q) -> int:
    return int(math.ceil(parse_quantity(str(q)).value * 1000))


# ---------------------------------------------------------------------------- replica calculator
def resource_utilization_ratio(metrics, requests, target_utilization):
    """`GetResourceUtilizationRatio`: (ratio, utilization %, raw average) over the pods that have
    both a metric and a request; utilization is truncated to a whole percent."""
    total = req_total = n = 0
    for pod, v in metrics.items():
        if pod in requests:
            total += v
            req_total += requests[pod]
            n += 1
    if n == 0:
        raise ValueError("no metrics returned matched known pods")
    if req_total <= 0:
        raise ValueError("no pods with a non-zero request")
    util = int(total * 100 // req_total)
    return util / float(target_utilization), util, total // n


def _ready_split(pods, metrics):
    unready, missing, ready = set(), set(), set()
    for p in pods:
        name = p["metadata"]["name"]
        if (p.get("status") or {}).get("phase") != "Running" or not pod_is_ready(p):
            unready.add(name)
            metrics.pop(name, None)
            continue
        if name not in metrics:
            missing.add(name)
            continue
        ready.add(name)
    return ready, unready, missing


def resource_replicas(current, target_utilization, metrics, pods, resource, requests_of, tolerance=0.1):
    """`GetResourceReplicas`: (replicas, utilization %, raw average milli-value). `metrics` maps
    pod name -> usage (milli), `requests_of(pod)` -> the pod's request (milli) or raises."""
    if not pods:
        raise ValueError("no pods returned by selector while calculating replica count")
    metrics = dict(metrics)
    requests = {p["metadata"]["name"]: requests_of(p) for p in pods}
    ready, unready, missing = _ready_split(pods, metrics)
    if not metrics:
        raise ValueError("did not receive metrics for any ready pods")
    ratio, util, raw = resource_utilization_ratio(metrics, requests, target_utilization)
    rebalance = bool(unready) and ratio > 1.0
    if not rebalance and not missing:
        if abs(1.0 - ratio) <= tolerance:
            return current, util, raw
        return int(math.ceil(ratio * len(ready))), util, raw
    if missing and ratio != 1.0:
        for name in missing:
            metrics[name] = requests[name] if ratio < 1.0 else 0
    if rebalance:
        for name in unready:
            metrics[name] = 0
    new_ratio, _, _ = resource_utilization_ratio(metrics, requests, target_utilization)
    if abs(1.0 - new_ratio) <= tolerance or (ratio < 1.0 < new_ratio) or (ratio > 1.0 > new_ratio):
        return current, util, raw
    return int(math.ceil(new_ratio * len(metrics))), util, raw


def plain_metric_replicas(current, target, metrics, pods, tolerance=0.1):
    """`calcPlainMetricReplicas` (targetAverageValue resources, Pods metrics): (replicas,
    average milli-value)."""
    if not pods:
        raise ValueError("no pods returned by selector while calculating replica count")
    metrics = dict(metrics)
    ready, unready, missing = _ready_split(pods, metrics)
    if not metrics:
        raise ValueError("did not receive metrics for any ready pods")
    util = sum(metrics.values()) // len(metrics)
    ratio = util / float(target)
    rebalance = bool(unready) and ratio > 1.0
    if not rebalance and not missing:
        if abs(1.0 - ratio) <= tolerance:
            return current, util
        return int(math.ceil(ratio * len(ready))), util
    if missing and ratio != 1.0:
        for name in missing:
            metrics[name] = target if ratio < 1.0 else 0
    if rebalance:
        for name in unready:
            metrics[name] = 0
    new_ratio = (sum(metrics.values()) // len(metrics)) / float(target)
    if abs(1.0 - new_ratio) <= tolerance or (ratio < 1.0 < new_ratio) or (ratio > 1.0 > new_ratio):
        return current, util
    return int(math.ceil(new_ratio * len(metrics))), util


def object_metric_replicas(current, target, value, tolerance=0.1):
    """`GetObjectMetricReplicas`: scale the current count by value / target."""
    ratio = value / float(target)
    if abs(1.0 - ratio) <= tolerance:
        return current
    return int(math.ceil(ratio * current))


def utilization_replicas(current, target_util, usage, requests, ready, unready, missing, tolerance):
    """Compatibility shim over `resource_replicas` for callers that already split the pods:
    usage / requests per pod name in the same unit."""
    pods = [{"metadata": {"name": n}, "status": {"phase": "Running" if n not in unready else "Pending",
                                                  "conditions": [{"type": "Ready", "status": "True"}]}}
            for n in sorted(set(ready) | set(unready) | set(missing))]
    scaled_usage = {n: int(round(v * 1000)) for n, v in usage.items() if n in ready}
    scaled_req = {n: int(round(v * 1000)) for n, v in requests.items()}
    r, util, _ = resource_replicas(current, target_util, scaled_usage, pods, "", lambda p: scaled_req[p["metadata"]["name"]],
                                   tolerance)
    return r, util


def convert_desired_replicas_with_rules(current, desired, hpa_min, hpa_max):
    """`convertDesiredReplicasWithRules`: (replicas, condition reason, message)."""
    if hpa_min == 0:
        lo, msg = 1, "the desired replica count is zero"
    else:
        lo, msg = hpa_min, "the desired replica count is less than the minimum replica count"
    limit = int(max(SCALE_UP_LIMIT_FACTOR * current, SCALE_UP_LIMIT_MINIMUM))
    if hpa_max > limit:
        hi, cond, msg_hi = limit, "ScaleUpLimit", "the desired replica count is increasing faster than the maximum scale rate"
    else:
        hi, cond, msg_hi = hpa_max, "TooManyReplicas", "the desired replica count is more than the maximum replica count"
    if desired < lo:
        return lo, "TooFewReplicas", msg
    if desired > hi:
        return hi, cond, msg_hi
    return desired, "DesiredWithinRange", "the desired count is within the acceptable range"


def set_condition(status, ctype, cstatus, reason, message):
    """`setConditionInList`: update in place; the transition time moves only on a status flip."""
    conds = status.setdefault("conditions", [])
    cur = next((c for c in conds if c.get("type") == ctype), None)
    if cur is None:
        cur = {"type": ctype}
        conds.append(cur)
    if cur.get("status") != cstatus:
        cur["lastTransitionTime"] = now_rfc3339()
    cur.update(status=cstatus, reason=reason, message=message)


class MetricError(Exception):
    def __init__(self, reason, message):
        super().__init__(message)
        self.reason = reason


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

    # -- metrics clients ------------------------------------------------------------------
    async def _get_json(self, path):
        st, body = await self.client.raw("GET", path)
        if st != 200:
            raise ValueError(f"unable to fetch metrics from API: HTTP {st}")
        return json.loads(body)

    async def resource_metrics(self, resource, ns, selector):
        """pod name -> usage: milli-units summed over containers (`GetResourceMetric`); for
        amd.com/gpu the pod's duty cycle x its GPU count (percent units)."""
        path = f"/apis/metrics.k8s.io/v1beta1/namespaces/{ns}/pods"
        if selector:
            path += "?labelSelector=" + quote(selector)
        items = (await self._get_json(path)).get("items") or ()
        if not items:
            raise ValueError("no metrics returned from resource metrics API")
        out = {}
        for it in items:
            name = it["metadata"]["name"]
            cs = it.get("containers") or ()
            if resource == GPU:
                vals = [float(c["usage"][GPU]) for c in cs if GPU in (c.get("usage") or {})]
                if vals:
                    out[name] = (sum(vals) / len(vals), len(vals))
                continue
            if any(resource not in (c.get("usage") or {}) for c in cs):
                continue         # the reference skips pods with a container lacking the resource
            out[name] = sum(milli(c["usage"][resource]) for c in cs)
        return out

    async def pods_metric(self, metric, ns, selector):
        path = f"/apis/custom.metrics.k8s.io/v1beta1/namespaces/{ns}/pods/*/{quote(metric)}"
        if selector:
            path += "?labelSelector=" + quote(selector)
        items = (await self._get_json(path)).get("items") or ()
        if not items:
            raise ValueError("no metrics returned from custom metrics API")
        return {it["describedObject"]["name"]: milli(it["value"]) for it in items}

    async def object_metric(self, metric, ns, target):
        ri = m.BY_KIND.get(target.get("kind"))
        plural = ri.plural if ri is not None else (target.get("kind") or "").lower() + "s"
        path = f"/apis/custom.metrics.k8s.io/v1beta1/namespaces/{ns}/{plural}/{quote(target.get('name', ''))}/{quote(metric)}"
        items = (await self._get_json(path)).get("items") or ()
        if not items:
            raise ValueError("no metrics returned from custom metrics API")
        return milli(items[0]["value"])

    # -- per metric -----------------------------------------------------------------------
    @staticmethod
    def _metric_specs(spec):
        if spec.get("metrics"):
            return spec["metrics"]
        return [{"type": "Resource", "resource": {"name": "cpu",
                                                  "targetAverageUtilization": spec.get("targetCPUUtilizationPercentage", 80)}}]

    def _requests_of(self, resource):
        def fn(p):
            if resource == GPU:
                n = 0
                for per in (p.get("spec") or {}).get("extendedResources") or ():
                    n += int(per.get("count") or len(per.get("assigned") or ()) or 1)
                if not n:
                    for c in (p.get("spec") or {}).get("containers") or ():
                        res = c.get("resources") or {}
                        n += int((res.get("limits") or {}).get(GPU, (res.get("requests") or {}).get(GPU, 0)) or 0)
                if not n:
                    raise ValueError(f"missing request for {GPU} in pod {m.namespace_of(p)}/{m.name_of(p)}")
                return 100 * n
            total = 0
            for c in (p.get("spec") or {}).get("containers") or ():
                q = ((c.get("resources") or {}).get("requests") or {}).get(resource)
                if q is None:
                    raise ValueError(f"missing request for {resource} on container {c.get('name')} in pod "
                                     f"{m.namespace_of(p)}/{m.name_of(p)}")
                total += milli(q)
            return total
        return fn

    async def compute_replicas_for_metrics(self, hpa, status, current, selector, pods):
        """`computeReplicasForMetrics`: (replicas, metric name, statuses) or MetricError."""
        ns = m.namespace_of(hpa)
        replicas, name, statuses = 0, "", []
        for ms in self._metric_specs(hpa.get("spec") or {}):
            typ = ms.get("type")
            try:
                if typ == "Resource":
                    res = ms.get("resource") or {}
                    rname = res.get("name")
                    metrics = await self.resource_metrics(rname, ns, selector)
                    if rname == GPU:
                        metrics = {k: int(round(duty * n * 1000)) for k, (duty, n) in metrics.items()}
                    if res.get("targetAverageValue") is not None:
                        r, raw = plain_metric_replicas(current, milli(res["targetAverageValue"]), metrics, pods,
                                                       self.tolerance)
                        proposal_name = f"{rname} resource"
                        st = {"type": "Resource", "resource": {"name": rname, "currentAverageValue": f"{raw}m"}}
                    elif res.get("targetAverageUtilization") is not None:
                        req = self._requests_of(rname)
                        if rname == GPU:
                            req = (lambda f: (lambda p: f(p) * 1000))(req)
                        r, util, raw = resource_replicas(current, int(res["targetAverageUtilization"]), metrics, pods,
                                                         rname, req, self.tolerance)
                        proposal_name = f"{rname} resource utilization (percentage of request)"
                        st = {"type": "Resource", "resource": {"name": rname, "currentAverageUtilization": util,
                                                               "currentAverageValue": f"{raw}m"}}
                    else:
                        raise MetricError("FailedGetResourceMetric", "invalid resource metric source: neither a "
                                          "utilization target nor a value target was set")
                elif typ == "Pods":
                    pm = ms.get("pods") or {}
                    metrics = await self.pods_metric(pm.get("metricName", ""), ns, selector)
                    r, util = plain_metric_replicas(current, milli(pm.get("targetAverageValue", "0")), metrics, pods,
                                                    self.tolerance)
                    proposal_name = f"pods metric {pm.get('metricName')}"
                    st = {"type": "Pods", "pods": {"metricName": pm.get("metricName"), "currentAverageValue": f"{util}m"}}
                elif typ == "Object":
                    om = ms.get("object") or {}
                    value = await self.object_metric(om.get("metricName", ""), ns, om.get("target") or {})
                    r = object_metric_replicas(current, milli(om.get("targetValue", "0")), value, self.tolerance)
                    proposal_name = f"{(om.get('target') or {}).get('kind')} metric {om.get('metricName')}"
                    st = {"type": "Object", "object": {"target": om.get("target"), "metricName": om.get("metricName"),
                                                       "currentValue": f"{value}m"}}
                else:
                    raise MetricError("InvalidMetricSourceType", f"unknown metric source type {typ!r}")
            except MetricError:
                raise
            except (ValueError, APIStatusError) as e:
                reason = {"Resource": "FailedGetResourceMetric", "Pods": "FailedGetPodsMetric",
                          "Object": "FailedGetObjectMetric"}.get(typ, "FailedGetResourceMetric")
                raise MetricError(reason, str(e)) from None
            statuses.append(st)
            if replicas == 0 or r > replicas:
                replicas, name = r, proposal_name
        set_condition(status, "ScalingActive", "True", "ValidMetricFound",
                      f"the HPA was able to successfully calculate a replica count from {name}")
        return replicas, name, statuses

    # -- reconcile ------------------------------------------------------------------------
    async def sync(self, key):
        hpa = self.hpa_inf.get(key)
        if hpa is None:
            return
        await self.reconcile(hpa)

    async def reconcile(self, hpa, now=None):
        now = now if now is not None else time.time()
        ns, name = m.namespace_of(hpa), m.name_of(hpa)
        spec = hpa.get("spec") or {}
        original = self.read_status(hpa)
        status = json.loads(json.dumps(original))
        ref = spec.get("scaleTargetRef") or {}
        plural = TARGETS.get(ref.get("kind"))
        try:
            if plural is None:
                raise ValueError(f"unrecognized resource for scale target kind {ref.get('kind')!r}")
            scale = await self.client.get(plural, ref.get("name"), ns, subresource="scale")
        except (ValueError, APIStatusError) as e:
            self.recorder.event(hpa, "Warning", "FailedGetScale", str(e))
            set_condition(status, "AbleToScale", "False", "FailedGetScale",
                          f"the HPA controller was unable to get the target's current scale: {e}")
            await self._write_status(hpa, original, status)
            return
        set_condition(status, "AbleToScale", "True", "SucceededGetScale",
                      "the HPA controller was able to get the target's current scale")
        current = int((scale.get("status") or {}).get("replicas", (scale.get("spec") or {}).get("replicas", 0)) or 0)
        hpa_min = spec.get("minReplicas")
        hpa_max = int(spec.get("maxReplicas") or current)
        statuses = None
        rescale, reason, desired = True, "", 0
        if int((scale.get("spec") or {}).get("replicas", 0) or 0) == 0:
            desired, rescale = 0, False
            set_condition(status, "ScalingActive", "False", "ScalingDisabled",
                          "scaling is disabled since the replica count of the target is zero")
        elif current > hpa_max:
            reason, desired = "Current number of replicas above Spec.MaxReplicas", hpa_max
        elif hpa_min is not None and current < int(hpa_min):
            reason, desired = "Current number of replicas below Spec.MinReplicas", int(hpa_min)
        elif current == 0:
            reason, desired = "Current number of replicas must be greater than 0", 1
        else:
            sel_str = (scale.get("status") or {}).get("selector") or ""
            try:
                if not sel_str:
                    self.recorder.event(hpa, "Warning", "SelectorRequired", "selector is required")
                    raise MetricError("InvalidSelector", "the HPA target's scale is missing a selector")
                try:
                    sel = parse_labels(sel_str)
                except (SelectorError, ValueError) as e:
                    msg = f"couldn't convert selector into a corresponding internal selector object: {e}"
                    self.recorder.event(hpa, "Warning", "InvalidSelector", msg)
                    raise MetricError("InvalidSelector", msg) from None
                pods = [p for p in self.pod_inf.list() if m.namespace_of(p) == ns
                        and sel.matches(p["metadata"].get("labels") or {})]
                metric_desired, metric_name, statuses = await self.compute_replicas_for_metrics(
                    hpa, status, current, sel_str, pods)
            except MetricError as e:
                if e.reason not in ("InvalidSelector",):
                    self.recorder.event(hpa, "Warning", e.reason, str(e))
                set_condition(status, "ScalingActive", "False", e.reason,
                              f"the HPA was unable to compute the replica count: {e}"
                              if e.reason != "InvalidSelector" else str(e))
                status["currentReplicas"] = current
                await self._write_status(hpa, original, status)
                self.recorder.event(hpa, "Warning", "FailedComputeMetricsReplicas", str(e))
                return
            desired = max(0, metric_desired)
            if desired > current:
                reason = f"{metric_name} above target"
            elif desired < current:
                reason = "All metrics below target"
            desired, cond, msg = convert_desired_replicas_with_rules(current, desired, int(hpa_min or 0), hpa_max)
            set_condition(status, "ScalingLimited", "False" if cond == "DesiredWithinRange" else "True", cond, msg)
            rescale = self.should_scale(status, current, desired, now)
            last = parse_rfc3339(status.get("lastScaleTime"))
            back_down = back_up = False
            if last is not None:
                if not last + self.downscale_window < now:
                    set_condition(status, "AbleToScale", "False", "BackoffDownscale",
                                  "the time since the previous scale is still within the downscale forbidden window")
                    back_down = True
                if not last + self.upscale_window < now:
                    back_up = True
                    if back_down:
                        set_condition(status, "AbleToScale", "False", "BackoffBoth",
                                      "the time since the previous scale is still within both the downscale and "
                                      "upscale forbidden windows")
                    else:
                        set_condition(status, "AbleToScale", "False", "BackoffUpscale",
                                      "the time since the previous scale is still within the upscale forbidden window")
            if not back_down and not back_up:
                set_condition(status, "AbleToScale", "True", "ReadyForNewScale",
                              "the last scale time was sufficiently old as to warrant a new scale")
        if rescale:
            scale = dict(scale, spec=dict(scale.get("spec") or {}, replicas=desired))
            try:
                await self.client.update(plural, scale, ns, subresource="scale")
            except APIStatusError as e:
                self.recorder.event(hpa, "Warning", "FailedRescale", f"New size: {desired}; reason: {reason}; error: {e}")
                set_condition(status, "AbleToScale", "False", "FailedUpdateScale",
                              f"the HPA controller was unable to update the target scale: {e}")
                status["currentReplicas"] = current
                await self._write_status(hpa, original, status)
                raise
            set_condition(status, "AbleToScale", "True", "SucceededRescale",
                          f"the HPA controller was able to update the target scale to {desired}")
            self.recorder.event(hpa, "Normal", "SuccessfulRescale", f"New size: {desired}; reason: {reason}")
            status["lastScaleTime"] = now_rfc3339(now)
        else:
            desired = current
        status["currentReplicas"] = current
        status["desiredReplicas"] = desired
        if statuses is not None:
            status["currentMetrics"] = statuses or None
            cpu = next((s["resource"]["currentAverageUtilization"] for s in statuses
                        if s.get("type") == "Resource" and s["resource"].get("name") == "cpu"
                        and "currentAverageUtilization" in s["resource"]), None)
            if cpu is not None:
                status["currentCPUUtilizationPercentage"] = cpu
        status["observedGeneration"] = hpa["metadata"].get("generation", 1)
        await self._write_status(hpa, original, status)

    def should_scale(self, status, current, desired, now):
        """`shouldScale`."""
        if desired == current:
            return False
        last = parse_rfc3339(status.get("lastScaleTime"))
        if last is None:
            return True
        if desired < current and last + self.downscale_window < now:
            return True
        if desired > current and last + self.upscale_window < now:
            return True
        return False

    @staticmethod
    def _v1_shaped(hpa):
        """An autoscaling/v1 object (no v2beta1 `spec.metrics`): like the reference's v1 storage,
        its v2beta1-only status lives in annotations (`autoscaling.alpha.kubernetes.io/conditions`,
        `.../current-metrics`, `pkg/apis/autoscaling/v1/conversion.go`)."""
        return not (hpa.get("spec") or {}).get("metrics")

    def read_status(self, hpa):
        st = json.loads(json.dumps(hpa.get("status") or {}))
        if self._v1_shaped(hpa):
            ann = hpa["metadata"].get("annotations") or {}
            for key, field in ((CONDITIONS_ANN, "conditions"), (CURRENT_METRICS_ANN, "currentMetrics")):
                if key in ann:
                    try:
                        st[field] = json.loads(ann[key])
                    except ValueError:
                        pass
        return st

    async def _write_status(self, hpa, original, status):
        """`updateStatusIfNeeded` (+ the v1 annotation form of conditions / currentMetrics)."""
        status = {k: v for k, v in status.items() if v is not None}
        if status == {k: v for k, v in original.items() if v is not None}:
            return
        ns, name = m.namespace_of(hpa), m.name_of(hpa)
        try:
            if self._v1_shaped(hpa):
                ann = {CONDITIONS_ANN: json.dumps(status.pop("conditions", None) or [], sort_keys=True),
                       CURRENT_METRICS_ANN: json.dumps(status.pop("currentMetrics", None) or [], sort_keys=True)}
                cur = hpa["metadata"].get("annotations") or {}
                if any(cur.get(k) != v for k, v in ann.items()):
                    hpa = await self.client.patch("horizontalpodautoscalers", name, {"metadata": {"annotations": ann}},
                                                  ns, "merge")
            else:
                status.pop("currentCPUUtilizationPercentage", None)       # v1-only field
            if status != {k: v for k, v in (hpa.get("status") or {}).items() if v is not None}:
                await self.client.update_status("horizontalpodautoscalers", dict(hpa, status=status), ns)
        except APIStatusError as e:
            self.recorder.event(hpa, "Warning", "FailedUpdateStatus", str(e))
            raise


def ns_of(p):
    return p["metadata"].get("namespace", "")


__all__ = ["HorizontalController", "resource_replicas", "plain_metric_replicas", "object_metric_replicas",
           "convert_desired_replicas_with_rules", "utilization_replicas", "selector_string", "split_key"]
