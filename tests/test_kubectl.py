"""kubectl against a live cluster running on a background event loop."""
import asyncio
import io
import json
import threading
import time

import pytest
import yaml

from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.kubectl.cli import main as kubectl


@pytest.fixture(scope="module")
def cluster():
    loop = asyncio.new_event_loop()
    holder = {}
    ready = threading.Event()

    def run():
        asyncio.set_event_loop(loop)
        cl = LocalCluster(nodes=2, gpus_per_node=8, controllers=["*"])
        loop.run_until_complete(cl.start())
        holder["cl"] = cl
        ready.set()
        loop.run_forever()
        loop.run_until_complete(cl.stop())

    t = threading.Thread(target=run, daemon=True)
    t.start()
    assert ready.wait(60)
    yield holder["cl"]
    loop.call_soon_threadsafe(loop.stop)
    t.join(30)


def k(cluster, *args):
    out = io.StringIO()
    rc = kubectl(["-s", cluster.url] + list(args), out=out)
    return rc, out.getvalue()


def wait(pred, timeout=20):
    t = time.time()
    while time.time() - t < timeout:
        r = pred()
        if r:
            return r
        time.sleep(0.05)
    raise TimeoutError


def test_get_nodes_shows_gpus(cluster):
    rc, out = k(cluster, "get", "nodes", "-o", "wide")
    assert rc == 0
    assert "node-0" in out and "8/8" in out and "MI355X" in out and "gfx950" in out and "288Gi" in out


def test_create_apply_describe_delete(cluster, tmp_path):
    manifest = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "vadd"},
                "spec": {"containers": [{"name": "c", "image": "kubernetes-amd/hip-vector-add",
                                         "resources": {"limits": {"amd.com/gpu": "2"}}}]}}
    f = tmp_path / "pod.yaml"
    f.write_text(yaml.safe_dump(manifest))
    rc, out = k(cluster, "create", "-f", str(f))
    assert rc == 0 and "pod/vadd created" in out
    wait(lambda: "Running" in k(cluster, "get", "pods", "vadd")[1])
    rc, out = k(cluster, "describe", "pod", "vadd")
    assert "Extended Resources:" in out and "Assigned:  GPU-" in out and "amd.com/gpu=2" in out
    rc, out = k(cluster, "get", "pod", "vadd", "-o", "jsonpath={.spec.extendedResources[0].assigned}")
    assert out.count("GPU-") == 2
    rc, out = k(cluster, "top", "nodes")
    assert "GPUS-ALLOCATED" in out
    rc, out = k(cluster, "label", "pod", "vadd", "team=ml")
    assert rc == 0
    rc, out = k(cluster, "get", "pods", "-l", "team=ml", "-o", "name")
    assert out.strip() == "pod/vadd"
    rc, out = k(cluster, "delete", "pod", "vadd", "--grace-period", "0")
    assert 'pod "vadd" deleted' in out


def test_describe_node_lists_devices(cluster):
    rc, out = k(cluster, "describe", "node", "node-1")
    assert rc == 0 and "Extended Resources (amd.com/gpu):" in out and "renderD128" in out and "Healthy" in out


def test_deployment_scale_rollout(cluster, tmp_path):
    d = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "svc"},
         "spec": {"replicas": 2, "selector": {"matchLabels": {"app": "svc"}},
                  "template": {"metadata": {"labels": {"app": "svc"}},
                               "spec": {"containers": [{"name": "c", "image": "x", "resources": {"limits": {"amd.com/gpu": "1"}}}]}}}}
    f = tmp_path / "d.json"
    f.write_text(json.dumps(d))
    assert k(cluster, "apply", "-f", str(f))[0] == 0
    rc, out = k(cluster, "rollout", "status", "deployment/svc", "--timeout", "30")
    assert "successfully rolled out" in out
    assert k(cluster, "scale", "deployment", "svc", "--replicas", "3")[0] == 0
    rc, out = k(cluster, "rollout", "status", "deployment/svc", "--timeout", "30")
    assert "successfully rolled out" in out
    d["spec"]["template"]["metadata"]["labels"]["v"] = "2"
    d["spec"]["selector"]["matchLabels"] = {"app": "svc"}
    f.write_text(json.dumps(d))
    rc, out = k(cluster, "apply", "-f", str(f))
    assert "configured" in out
    wait(lambda: "2" in k(cluster, "rollout", "history", "deployment/svc")[1])
    rc, out = k(cluster, "get", "deploy")
    assert "svc" in out


def test_cordon_taint_drain(cluster):
    assert k(cluster, "cordon", "node-1")[0] == 0
    rc, out = k(cluster, "get", "nodes")
    assert "SchedulingDisabled" in out
    assert k(cluster, "taint", "nodes", "node-1", "gpu=maintenance:NoSchedule")[0] == 0
    rc, out = k(cluster, "describe", "node", "node-1")
    assert "gpu:NoSchedule" in out
    assert k(cluster, "taint", "nodes", "node-1", "gpu-")[0] == 0
    assert k(cluster, "drain", "node-1", "--ignore-daemonsets", "--force")[0] == 0
    assert k(cluster, "uncordon", "node-1")[0] == 0


def test_misc_commands(cluster):
    assert "Server Version" in k(cluster, "version")[1]
    assert "apps/v1" in k(cluster, "api-versions")[1]
    assert "deployments" in k(cluster, "api-resources")[1]
    assert "extendedResources" in k(cluster, "explain", "pods")[1]
    rc, out = k(cluster, "get", "pods", "nope")
    assert rc == 1
