"""metrics-server (metrics.k8s.io via aggregation) + HorizontalPodAutoscaler on CPU and on MI355X
GPU utilization.

Parity: `pkg/controller/podautoscaler/horizontal_test.go` / `replica_calculator_test.go`
(utilization math, tolerance, scale-up limit, unready / missing pods) and
`test/e2e/autoscaling/horizontal_pod_autoscaling.go` (scale a Deployment on CPU).
"""
import asyncio

from kubernetes_amd.client.rest import Client
from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.controllers.podautoscaler import selector_string, utilization_replicas
from kubernetes_amd.metrics_server import MetricsServer


def test_replica_calculator():
    req = {"a": 100.0, "b": 100.0, "c": 100.0}
    # 3 ready pods at 90% with target 50% -> ceil(1.8*3) = 6
    assert utilization_replicas(3, 50, {"a": 90, "b": 90, "c": 90}, req, {"a", "b", "c"}, set(), set(), 0.1) == (6, 90)
    # within tolerance -> unchanged
    assert utilization_replicas(3, 50, {"a": 52, "b": 52, "c": 52}, req, {"a", "b", "c"}, set(), set(), 0.1)[0] == 3
    # scale-up with an unready pod: it counts as 0% -> ceil(((90+90+0)/300)/0.5 * 3) = 4
    assert utilization_replicas(3, 50, {"a": 90, "b": 90}, req, {"a", "b"}, {"c"}, set(), 0.1)[0] == 4
    # scale-down with a missing pod: it counts as 100% of its request -> direction flips -> unchanged
    assert utilization_replicas(3, 50, {"a": 10, "b": 10}, req, {"a", "b"}, set(), {"c"}, 0.1)[0] == 3
    assert selector_string({"matchLabels": {"app": "x"}, "matchExpressions": [{"key": "t", "operator": "In", "values": ["a", "b"]}]}) \
        == "app=x,t in (a,b)"


def _deploy(name, replicas, ann, resources):
    return {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": name, "namespace": "default"},
            "spec": {"replicas": replicas, "selector": {"matchLabels": {"app": name}},
                     "template": {"metadata": {"labels": {"app": name}, "annotations": ann},
                                  "spec": {"containers": [{"name": "c", "image": "img:1", "resources": resources}]}}}}


def test_hpa_scales_on_cpu_and_gpu(run):
    async def main():
        cl = LocalCluster(nodes=1, gpus_per_node=8, kubelet_http=True,
                          controllers=["deployment", "replicaset", "horizontalpodautoscaling"],
                          controller_options={"horizontalpodautoscaling": {"sync_period": 0.2, "upscale_window": 0,
                                                                           "downscale_window": 0}})
        await cl.start()
        ms = await MetricsServer(Client(cl.url), resolution=0.1).start()
        c = cl.client
        try:
            await c.create("deployments", _deploy("cpu", 1, {"kubemark.amd.com/cpu-millicores": "400"},
                                                  {"requests": {"cpu": "200m"}}))
            await c.create("deployments", _deploy("gpu", 1, {"kubemark.amd.com/gpu-utilization": "90"},
                                                  {"limits": {"amd.com/gpu": "1"}}))
            await c.create("horizontalpodautoscalers", {"metadata": {"name": "cpu", "namespace": "default"},
                "spec": {"scaleTargetRef": {"apiVersion": "apps/v1", "kind": "Deployment", "name": "cpu"},
                         "minReplicas": 1, "maxReplicas": 5, "targetCPUUtilizationPercentage": 50}})
            await c.create("horizontalpodautoscalers", {"metadata": {"name": "gpu", "namespace": "default"},
                "spec": {"scaleTargetRef": {"apiVersion": "apps/v1", "kind": "Deployment", "name": "gpu"},
                         "minReplicas": 1, "maxReplicas": 3,
                         "metrics": [{"type": "Resource", "resource": {"name": "amd.com/gpu", "targetAverageUtilization": 45}}]}})
            # metrics API is served through the aggregator
            for _ in range(100):
                st, _ = await c.raw("GET", "/apis/metrics.k8s.io/v1beta1/namespaces/default/pods")
                if st == 200:
                    break
                await asyncio.sleep(0.05)
            assert st == 200

            async def replicas(n):
                return (await c.get("deployments", n, "default"))["spec"]["replicas"]
            for _ in range(300):
                if await replicas("cpu") == 5 and await replicas("gpu") == 3:
                    break
                await asyncio.sleep(0.05)
            assert await replicas("cpu") == 5
            assert await replicas("gpu") == 3
            hpa = await c.get("horizontalpodautoscalers", "cpu", "default")
            assert hpa["status"].get("currentCPUUtilizationPercentage") == 200 and hpa["status"].get("lastScaleTime"), hpa["status"]
            pm = await c.raw("GET", "/apis/metrics.k8s.io/v1beta1/namespaces/default/pods")
            assert b'"amd.com/gpu": "90"' in pm[1] or b'"amd.com/gpu":"90"' in pm[1]
        finally:
            await ms.stop()
            await cl.stop()
    run(main(), timeout=90)
