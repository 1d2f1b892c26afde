"""HorizontalPodAutoscaler: the `replica_calculator_test.go` table (resource utilization with
unready / missing / superfluous metrics, tolerance, custom pods and object metrics) against the
pure calculator, and `horizontal_test.go` reconcile cases over a fake client with a scale
subresource and a metrics API: scale up / down, the scale-up limit, min / max bounds, zero
replicas, forbidden windows, and the AbleToScale / ScalingActive / ScalingLimited conditions."""
import asyncio
import json
import time

import pytest

from kubernetes_amd.api.meta import now_rfc3339
from kubernetes_amd.client.fake import FakeClient
from kubernetes_amd.client.informer import InformerFactory
from kubernetes_amd.client.rest import APIStatusError
from kubernetes_amd.controllers.podautoscaler import (CONDITIONS_ANN, HorizontalController, object_metric_replicas,
                                                      plain_metric_replicas, resource_replicas)

NS = "test-namespace"


def mkpods(n, requests=None, readiness=None, containers=2, resource="cpu"):
    out = []
    for i in range(n):
        ready = "True" if readiness is None else readiness[i]
        cs = [{"name": f"c{j}"} for j in range(containers)]
        if requests is not None and i < len(requests):
            for c in cs:
                c["resources"] = {"requests": {resource: requests[i]}}
        out.append({"apiVersion": "v1", "kind": "Pod",
                    "metadata": {"name": f"test-pod-{i}", "namespace": NS, "labels": {"name": "test-pod"}},
                    "spec": {"containers": cs},
                    "status": {"phase": "Running", "conditions": [{"type": "Ready", "status": ready}]}})
    return out


def req_of(resource="cpu"):
    from kubernetes_amd.controllers.podautoscaler import milli

    def fn(p):
        total = 0
        for c in p["spec"]["containers"]:
            q = ((c.get("resources") or {}).get("requests") or {}).get(resource)
            if q is None:
                raise ValueError(f"missing request for {resource} on container {c['name']}")
            total += milli(q)
        return total
    return fn


def levels_metrics(levels, names=None, containers=2):
    return {(names[i] if names else f"test-pod-{i}"): lv * containers for i, lv in enumerate(levels)}


# name: (current, expected replicas or error substring, requests, levels, readiness, target, expected util, raw)
RESOURCE_CASES = {
    "ScaleUp": (3, 5, ["1.0"] * 3, [300, 500, 700], None, 30, 50, 2 * 500),
    "ScaleUpUnreadyLessScale": (3, 4, ["1.0"] * 3, [300, 500, 700], ["False", "True", "True"], 30, 60, 2 * 600),
    "ScaleUpUnreadyNoScale": (3, 3, ["1.0"] * 3, [400, 500, 700], ["True", "False", "False"], 30, 40, 2 * 400),
    "ScaleDown": (5, 3, ["1.0"] * 5, [100, 300, 500, 250, 250], None, 50, 28, 2 * 280),
    "ScaleDownIgnoresUnreadyPods": (5, 2, ["1.0"] * 5, [100, 300, 500, 250, 250],
                                    ["True", "True", "True", "False", "False"], 50, 30, 2 * 300),
    "Tolerance": (3, 3, ["0.9", "1.0", "1.1"], [1010, 1030, 1020], None, 100, 102, 2 * 1020),
    "SuperfluousMetrics": (4, 24, ["1.0"] * 4, [4000, 9500, 3000, 7000, 3200, 2000], None, 100, 587, 2 * 5875),
    "MissingMetrics": (4, 3, ["1.0"] * 4, [400, 95], None, 100, 24, 495),
    "MissingMetricsNoChangeEq": (2, 2, ["1.0"] * 2, [1000], None, 100, 100, 2 * 1000),
    "MissingMetricsNoChangeGt": (2, 2, ["1.0"] * 2, [1900], None, 100, 190, 2 * 1900),
    "MissingMetricsNoChangeLt": (2, 2, ["1.0"] * 2, [600], None, 100, 60, 2 * 600),
    "MissingMetricsUnreadyNoChange": (3, 3, ["1.0"] * 3, [100, 450], ["False", "True", "True"], 50, 45, 2 * 450),
    "MissingMetricsUnreadyScaleUp": (3, 4, ["1.0"] * 3, [100, 2000], ["False", "True", "True"], 50, 200, 2 * 2000),
    "MissingMetricsUnreadyScaleDown": (4, 3, ["1.0"] * 4, [100, 100, 100], ["False", "True", "True", "True"], 50, 10,
                                       2 * 100),
    "EmptyCPURequest": (1, "missing request for", [], [200], None, 100, None, None),
}


@pytest.mark.parametrize("name", list(RESOURCE_CASES))
def test_resource_replicas(name):
    current, want, requests, levels, readiness, target, util, raw = RESOURCE_CASES[name]
    pods = mkpods(current, requests, readiness)
    if isinstance(want, str):
        with pytest.raises(ValueError, match=want):
            resource_replicas(current, target, levels_metrics(levels), pods, "cpu", req_of())
        return
    r, got_util, got_raw = resource_replicas(current, target, levels_metrics(levels), pods, "cpu", req_of())
    assert (r, got_util, got_raw) == (want, util, raw)


def test_disjoint_resource_metrics():
    pods = mkpods(1, ["1.0"])
    with pytest.raises(ValueError, match="no metrics returned matched known pods"):
        resource_replicas(1, 100, {"an-older-pod-name": 200}, pods, "cpu", req_of())


def test_computed_tolerance_alg_implementation():
    """TestReplicaCalcComputedToleranceAlgImplementation: a target just past the tolerance
    scales down; one just inside it does not."""
    start, used = 10, 10 * 150
    requested = 2 * used
    per_pod = requested // start
    reqs = [f"{per_pod + d}m" for d in (100, -100, 10, -10, 2, -2, 1, -1, 0, 0)]
    pods = [dict(p, spec={"containers": [{"name": "c0", "resources": {"requests": {"cpu": reqs[i]}}}]})
            for i, p in enumerate(mkpods(start))]
    metrics = {f"test-pod-{i}": used // 10 for i in range(start)}
    ratio_used = float(requested // used)
    target = abs(1 / (ratio_used * (1 - 0.1))) + .01
    final = int(__import__("math").ceil(used / (requested * target) * start))
    r, util, _ = resource_replicas(start, int(target * 100), metrics, pods, "cpu", req_of())
    assert r == final and util == used * 100 // requested
    target = abs(1 / (ratio_used * (1 - 0.1))) + .004
    assert resource_replicas(start, int(target * 100), metrics, pods, "cpu", req_of())[0] == start


@pytest.mark.parametrize("current,want,levels,readiness,target,util", [
    (3, 4, [20000, 10000, 30000], None, 15000, 20000),                          # ScaleUpCM
    (3, 4, [50000, 10000, 30000], ["True", "True", "False"], 15000, 30000),      # ScaleUpCMUnreadyLessScale
    (3, 3, [50000, 15000, 30000], ["False", "True", "False"], 15000, 15000),     # ...NoScaleWouldScaleDown
    (5, 3, [12000] * 5, None, 20000, 12000),                                     # ScaleDownCM
    (3, 3, [20000, 21000, 21000], None, 20000, 20666)])                          # ToleranceCM
def test_pods_metric_replicas(current, want, levels, readiness, target, util):
    pods = mkpods(current, readiness=readiness)
    metrics = {f"test-pod-{i}": v for i, v in enumerate(levels)}
    assert plain_metric_replicas(current, target, metrics, pods) == (want, util)


@pytest.mark.parametrize("current,want,value,target", [(3, 4, 20000, 15000), (5, 3, 12000, 20000), (3, 3, 20666, 20000)])
def test_object_metric_replicas(current, want, value, target):
    assert object_metric_replicas(current, target, value) == want


# --------------------------------------------------------------------------- reconcile
class MetricsClient(FakeClient):
    def __init__(self, *objs, pod_metrics=None, fail_metrics=False):
        super().__init__(*objs)
        self.pod_metrics = pod_metrics or {}
        self.fail_metrics = fail_metrics

    async def raw(self, method, path, body=None, headers=None):
        if self.fail_metrics:
            return 503, b"{}"
        items = [{"metadata": {"name": n, "namespace": NS},
                  "containers": [{"name": f"c{j}", "usage": {"cpu": f"{v}m"}} for j in range(2)]}
                 for n, v in self.pod_metrics.items()]
        return 200, json.dumps({"items": items}).encode()


def hpa(min_r=2, max_r=6, target=30, last_scale=None, metrics=None):
    h = {"apiVersion": "autoscaling/v1", "kind": "HorizontalPodAutoscaler",
         "metadata": {"name": "test-hpa", "namespace": NS, "generation": 1},
         "spec": {"scaleTargetRef": {"apiVersion": "apps/v1", "kind": "Deployment", "name": "test-rc"},
                  "minReplicas": min_r, "maxReplicas": max_r}}
    if metrics is not None:
        h["spec"]["metrics"] = metrics
    else:
        h["spec"]["targetCPUUtilizationPercentage"] = target
    if last_scale is not None:
        h["status"] = {"lastScaleTime": now_rfc3339(last_scale)}
    return h


def reconcile(h, spec_replicas, status_replicas, levels=None, readiness=None, selector="name=test-pod",
              fail_get_scale=False, fail_update_scale=False, fail_metrics=False):
    pods = mkpods(status_replicas, ["1.0"] * status_replicas, readiness)
    metrics = {f"test-pod-{i}": v for i, v in enumerate(levels or [])}

    async def main():
        c = MetricsClient(h, *pods, pod_metrics=metrics, fail_metrics=fail_metrics)
        updates = []

        def get_scale(a):
            if a.subresource != "scale":
                return False, None
            if fail_get_scale:
                raise APIStatusError(404, {"message": "not found"})
            return True, {"apiVersion": "autoscaling/v1", "kind": "Scale", "metadata": {"name": "test-rc", "namespace": NS},
                          "spec": {"replicas": spec_replicas}, "status": {"replicas": status_replicas, "selector": selector}}

        def update_scale(a):
            if a.subresource != "scale":
                return False, None
            if fail_update_scale:
                raise APIStatusError(500, {"message": "boom"})
            updates.append(a.obj["spec"]["replicas"])
            return True, a.obj
        c.prepend_reactor("get", "deployments", get_scale)
        c.prepend_reactor("update", "deployments", update_scale)
        f = InformerFactory(c)
        hc = HorizontalController(c, f)
        hc.setup()
        events = []
        hc.recorder.event = lambda obj, typ, reason, msg: events.append((typ, reason, msg))
        f.start()
        await f.wait_for_cache_sync()
        try:
            await hc.reconcile(hc.hpa_inf.get(f"{NS}/test-hpa"))
        except APIStatusError:
            pass
        final = await c.get("horizontalpodautoscalers", "test-hpa", NS)
        return updates, events, final, hc.read_status(final)
    return asyncio.run(main())


def cond(st, t):
    return next(((c["status"], c["reason"]) for c in st.get("conditions") or () if c["type"] == t), None)


def test_scale_up():
    updates, events, final, st = reconcile(hpa(), 3, 3, [300, 500, 700])
    assert updates == [5] and st["desiredReplicas"] == 5 and st["currentCPUUtilizationPercentage"] == 50
    assert ("Normal", "SuccessfulRescale", "New size: 5; reason: cpu resource utilization (percentage of request) "
            "above target") in events
    assert cond(st, "AbleToScale") == ("True", "SucceededRescale")
    assert cond(st, "ScalingActive") == ("True", "ValidMetricFound")
    assert cond(st, "ScalingLimited") == ("False", "DesiredWithinRange")
    assert st["currentMetrics"][0]["resource"]["currentAverageUtilization"] == 50
    # autoscaling/v1 object: v2beta1-only status kept in annotations, as the reference's v1 storage
    assert CONDITIONS_ANN in final["metadata"]["annotations"] and "conditions" not in final["status"]


def test_scale_down():
    updates, events, final, st = reconcile(hpa(target=50), 5, 5, [100, 300, 500, 250, 250])
    assert updates == [3] and ("Normal", "SuccessfulRescale", "New size: 3; reason: All metrics below target") in events


def test_tolerance_no_scale():
    updates, events, _, st = reconcile(hpa(target=100, min_r=1), 3, 3, [1010, 1030, 1020])
    assert updates == [] and st["desiredReplicas"] == 3 and cond(st, "AbleToScale") == ("True", "ReadyForNewScale")


def test_scale_up_limit():
    updates, _, _, st = reconcile(hpa(min_r=1, max_r=100, target=10), 3, 3, [1000, 1000, 1000])
    assert updates == [6] and cond(st, "ScalingLimited") == ("True", "ScaleUpLimit")


def test_max_replicas_limit():
    updates, _, _, st = reconcile(hpa(min_r=2, max_r=5, target=10), 3, 3, [1000, 1000, 1000])
    assert updates == [5] and cond(st, "ScalingLimited") == ("True", "TooManyReplicas")


def test_min_replicas_limit():
    updates, _, _, st = reconcile(hpa(min_r=2, max_r=5, target=90), 3, 3, [10, 95, 10])
    assert updates == [2] and cond(st, "ScalingLimited") == ("True", "TooFewReplicas")


def test_replicas_outside_the_bounds_are_brought_back():
    updates, events, _, _ = reconcile(hpa(min_r=2, max_r=5), 7, 7, [100] * 7)
    assert updates == [5] and events[-1][2] == "New size: 5; reason: Current number of replicas above Spec.MaxReplicas"
    updates, events, _, _ = reconcile(hpa(min_r=2, max_r=5), 1, 1, [100])
    assert updates == [2] and events[-1][2] == "New size: 2; reason: Current number of replicas below Spec.MinReplicas"


def test_zero_replicas_disable_scaling():
    updates, _, _, st = reconcile(hpa(), 0, 0, [])
    assert updates == [] and cond(st, "ScalingActive") == ("False", "ScalingDisabled")


def test_forbidden_windows():
    updates, _, _, st = reconcile(hpa(last_scale=time.time() - 60), 3, 3, [300, 500, 700])
    assert updates == [] and cond(st, "AbleToScale") == ("False", "BackoffBoth")
    updates, _, _, st = reconcile(hpa(last_scale=time.time() - 240), 3, 3, [300, 500, 700])   # up allowed after 3 min
    assert updates == [5]
    updates, _, _, st = reconcile(hpa(target=50, last_scale=time.time() - 240), 5, 5, [100, 300, 500, 250, 250])
    assert updates == [] and cond(st, "AbleToScale") == ("False", "BackoffDownscale")


def test_condition_failures():
    _, events, _, st = reconcile(hpa(), 3, 3, [300, 500, 700], fail_get_scale=True)
    assert cond(st, "AbleToScale") == ("False", "FailedGetScale") and events[0][1] == "FailedGetScale"
    _, events, _, st = reconcile(hpa(), 3, 3, [300, 500, 700], selector="")
    assert cond(st, "ScalingActive") == ("False", "InvalidSelector") and events[0][1] == "SelectorRequired"
    _, events, _, st = reconcile(hpa(), 3, 3, [300, 500, 700], fail_metrics=True)
    assert cond(st, "ScalingActive") == ("False", "FailedGetResourceMetric")
    assert {e[1] for e in events} >= {"FailedGetResourceMetric", "FailedComputeMetricsReplicas"}
    updates, events, _, st = reconcile(hpa(), 3, 3, [300, 500, 700], fail_update_scale=True)
    assert cond(st, "AbleToScale") == ("False", "FailedUpdateScale") and events[-1][1] == "FailedRescale"


def test_v2_object_keeps_conditions_in_status():
    m = [{"type": "Resource", "resource": {"name": "cpu", "targetAverageUtilization": 30}}]
    updates, _, final, st = reconcile(hpa(metrics=m), 3, 3, [300, 500, 700])
    assert updates == [5] and cond(final["status"], "AbleToScale") == ("True", "SucceededRescale")
    assert "currentCPUUtilizationPercentage" not in final["status"]
