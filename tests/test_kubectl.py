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
    rc, out = k(cluster, "get", "pods", "vadd", "--experimental-server-print")   # columns from the API server
    assert rc == 0 and out.splitlines()[0].split()[:3] == ["NAME", "READY", "STATUS"] and "Running" in out
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
    with pytest.raises(SystemExit, match="Expected replicas to be 7, was 3"):   # --current-replicas precondition
        k(cluster, "scale", "deployment", "svc", "--current-replicas", "7", "--replicas", "1")
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
    # undo through the rollback subresource: the controller restores revision 1's template
    rc, out = k(cluster, "rollout", "undo", "deployment/svc")
    assert rc == 0 and "rolled back" in out

    def restored():
        d = json.loads(k(cluster, "get", "deployment", "svc", "-o", "json")[1])
        return "v" not in d["spec"]["template"]["metadata"]["labels"] and not d["spec"].get("rollbackTo")
    wait(restored)


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


def _get(cluster, *args):
    rc, out = k(cluster, "get", *args, "-o", "json")
    assert rc == 0, out
    return json.loads(out)


def test_create_generators(cluster, tmp_path):
    assert k(cluster, "create", "namespace", "gen")[0] == 0
    assert k(cluster, "-n", "gen", "create", "configmap", "cfg", "--from-literal", "a=1", "--from-literal", "b=2")[0] == 0
    assert _get(cluster, "-n", "gen", "configmap", "cfg")["data"] == {"a": "1", "b": "2"}
    assert k(cluster, "-n", "gen", "create", "secret", "generic", "s1", "--from-literal", "pw=hunter2")[0] == 0
    import base64
    assert base64.b64decode(_get(cluster, "-n", "gen", "secret", "s1")["data"]["pw"]) == b"hunter2"
    assert k(cluster, "-n", "gen", "create", "serviceaccount", "robot")[0] == 0
    assert k(cluster, "-n", "gen", "create", "role", "reader", "--verb", "get", "--verb", "list", "--resource", "pods")[0] == 0
    assert k(cluster, "-n", "gen", "create", "rolebinding", "rb", "--role", "reader", "--serviceaccount", "gen:robot")[0] == 0
    rb = _get(cluster, "-n", "gen", "rolebinding", "rb")
    assert rb["subjects"] == [{"kind": "ServiceAccount", "namespace": "gen", "name": "robot"}]
    assert k(cluster, "-n", "gen", "create", "quota", "q", "--hard", "pods=10,amd.com/gpu=4")[0] == 0
    assert _get(cluster, "-n", "gen", "resourcequota", "q")["spec"]["hard"]["amd.com/gpu"] == "4"
    assert k(cluster, "-n", "gen", "create", "service", "clusterip", "web", "--tcp", "80:8080")[0] == 0
    assert _get(cluster, "-n", "gen", "service", "web")["spec"]["ports"][0]["targetPort"] == 8080
    assert k(cluster, "-n", "gen", "create", "deployment", "trainer", "--image", "rocm/pytorch", "--gpus", "1")[0] == 0
    d = _get(cluster, "-n", "gen", "deployment", "trainer")
    assert d["spec"]["template"]["spec"]["containers"][0]["resources"]["limits"]["amd.com/gpu"] == "1"
    rc, out = k(cluster, "create", "--dry-run", "-o", "yaml", "priorityclass", "high", "--value", "1000")
    assert rc == 0 and yaml.safe_load(out)["value"] == 1000


def test_set_commands(cluster):
    k(cluster, "create", "namespace", "setns")
    assert k(cluster, "-n", "setns", "create", "deployment", "app", "--image", "busybox:1")[0] == 0
    assert k(cluster, "-n", "setns", "set", "image", "deployment/app", "busybox=busybox:2")[0] == 0
    assert k(cluster, "-n", "setns", "set", "resources", "deployment/app", "--limits", "cpu=2,memory=1Gi")[0] == 0
    assert k(cluster, "-n", "setns", "set", "env", "deployment/app", "MODE=fast", "HIP_VISIBLE_DEVICES=0")[0] == 0
    assert k(cluster, "-n", "setns", "set", "env", "deployment/app", "MODE-")[0] == 0
    assert k(cluster, "-n", "setns", "set", "serviceaccount", "deployment/app", "default")[0] == 0
    c = _get(cluster, "-n", "setns", "deployment", "app")["spec"]["template"]["spec"]
    ctr = c["containers"][0]
    assert ctr["image"] == "busybox:2" and ctr["resources"]["limits"] == {"cpu": "2", "memory": "1Gi"}
    assert ctr["env"] == [{"name": "HIP_VISIBLE_DEVICES", "value": "0"}] and c["serviceAccountName"] == "default"


def test_rolling_update_rc(cluster):
    k(cluster, "create", "namespace", "ru")
    rc_obj = {"apiVersion": "v1", "kind": "ReplicationController", "metadata": {"name": "web", "namespace": "ru"},
              "spec": {"replicas": 2, "selector": {"app": "web"},
                       "template": {"metadata": {"labels": {"app": "web"}},
                                    "spec": {"containers": [{"name": "web", "image": "nginx:1"}]}}}}
    import tempfile
    with tempfile.NamedTemporaryFile("w", suffix=".yaml", delete=False) as f:
        yaml.safe_dump(rc_obj, f)
    assert k(cluster, "create", "-f", f.name)[0] == 0
    wait(lambda: (_get(cluster, "-n", "ru", "rc", "web").get("status") or {}).get("readyReplicas") == 2)
    rc, out = k(cluster, "-n", "ru", "rolling-update", "web", "--image", "nginx:2", "--timeout", "60")
    assert rc == 0, out
    assert 'replicationcontroller "web" rolling updated' in out
    cur = _get(cluster, "-n", "ru", "rc", "web")
    assert cur["spec"]["template"]["spec"]["containers"][0]["image"] == "nginx:2" and cur["spec"]["replicas"] == 2

    def settled():
        pods = [p for p in _get(cluster, "-n", "ru", "pods")["items"] if not p["metadata"].get("deletionTimestamp")]
        return len(pods) == 2 and all(p["spec"]["containers"][0]["image"] == "nginx:2" for p in pods)
    wait(settled, 30)


def test_convert_diff_completion_plugin_options_reconcile(cluster, tmp_path, monkeypatch):
    dep = {"apiVersion": "extensions/v1beta1", "kind": "Deployment", "metadata": {"name": "old", "namespace": "default"},
           "spec": {"template": {"metadata": {"labels": {"a": "b"}}, "spec": {"containers": [{"name": "c", "image": "x"}]}}}}
    p = tmp_path / "d.yaml"
    p.write_text(yaml.safe_dump(dep))
    rc, out = k(cluster, "convert", "-f", str(p))
    assert rc == 0 and yaml.safe_load(out)["apiVersion"] == "apps/v1"

    cm = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "difftest", "namespace": "default"}, "data": {"k": "1"}}
    p2 = tmp_path / "cm.yaml"
    p2.write_text(yaml.safe_dump(cm))
    assert k(cluster, "apply", "-f", str(p2))[0] == 0
    rc, out = k(cluster, "alpha", "diff", "-f", str(p2))
    assert rc == 0 and out.strip() == ""
    cm["data"]["k"] = "2"
    p2.write_text(yaml.safe_dump(cm))
    rc, out = k(cluster, "alpha", "diff", "-f", str(p2))
    assert rc == 1 and "-  k: '1'" in out and "+  k: '2'" in out

    rc, out = k(cluster, "completion", "bash")
    assert rc == 0 and "rolling-update" in out and "complete -F _kubectl kubectl" in out
    rc, out = k(cluster, "options")
    assert "--kubeconfig" in out

    plug = tmp_path / "plugins" / "hello"
    plug.mkdir(parents=True)
    (plug / "plugin.yaml").write_text(yaml.safe_dump({"name": "hello", "shortDesc": "says hello",
                                                      "command": "echo hello-$KUBECTL_PLUGINS_CURRENT_NAMESPACE > out.txt"}))
    monkeypatch.setenv("KUBECTL_PLUGINS_PATH", str(tmp_path / "plugins"))
    rc, out = k(cluster, "plugin")
    assert "hello" in out and "says hello" in out
    assert k(cluster, "-n", "kube-system", "plugin", "hello")[0] == 0
    assert (plug / "out.txt").read_text().strip() == "hello-kube-system"

    role = {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole", "metadata": {"name": "recon"},
            "rules": [{"apiGroups": [""], "resources": ["pods"], "verbs": ["get"]}]}
    p3 = tmp_path / "r.yaml"
    p3.write_text(yaml.safe_dump(role))
    assert k(cluster, "auth", "reconcile", "-f", str(p3))[0] == 0
    role["rules"].append({"apiGroups": [""], "resources": ["nodes"], "verbs": ["list"]})
    p3.write_text(yaml.safe_dump(role))
    assert k(cluster, "auth", "reconcile", "-f", str(p3))[0] == 0
    assert len(_get(cluster, "clusterrole", "recon")["rules"]) == 2


def test_daemonset_revisions_rolling_update_and_undo(cluster):
    """ControllerRevision history (pkg/controller/history) + DaemonSet RollingUpdate +
    kubectl rollout history/undo for daemonsets."""
    k(cluster, "create", "namespace", "dsrev")
    ds = {"apiVersion": "apps/v1", "kind": "DaemonSet", "metadata": {"name": "agent", "namespace": "dsrev"},
          "spec": {"selector": {"matchLabels": {"app": "agent"}},
                   "template": {"metadata": {"labels": {"app": "agent"}},
                                "spec": {"containers": [{"name": "c", "image": "agent:v1"}]}}}}
    import tempfile
    with tempfile.NamedTemporaryFile("w", suffix=".yaml", delete=False) as f:
        yaml.safe_dump(ds, f)
    assert k(cluster, "create", "-f", f.name)[0] == 0

    def pods_with(image):
        ps = [p for p in _get(cluster, "-n", "dsrev", "pods")["items"] if not p["metadata"].get("deletionTimestamp")]
        return len(ps) == 2 and all(p["spec"]["containers"][0]["image"] == image for p in ps)
    wait(lambda: pods_with("agent:v1"), 30)
    assert k(cluster, "-n", "dsrev", "set", "image", "daemonset/agent", "c=agent:v2")[0] == 0
    wait(lambda: pods_with("agent:v2"), 60)
    revs = _get(cluster, "-n", "dsrev", "controllerrevisions")["items"]
    assert sorted(r["revision"] for r in revs) == [1, 2]
    rc, out = k(cluster, "-n", "dsrev", "rollout", "history", "daemonset/agent")
    assert rc == 0 and "REVISION" in out and "2" in out
    assert k(cluster, "-n", "dsrev", "rollout", "undo", "daemonset/agent")[0] == 0
    wait(lambda: pods_with("agent:v1"), 60)
    revs = _get(cluster, "-n", "dsrev", "controllerrevisions")["items"]
    assert max(revs, key=lambda r: r["revision"])["data"]["spec"]["template"]["spec"]["containers"][0]["image"] == "agent:v1"


def test_describe_node_shows_partitions_and_burn_in():
    from kubernetes_amd.api import core
    from kubernetes_amd.kubectl.printers import describe
    attrs = {core.ATTR_PRODUCT: "MI355X", core.ATTR_ARCH: "gfx950", core.ATTR_HBM: "36Gi", core.ATTR_HIVE: "h",
             core.ATTR_NUMA: "0", core.ATTR_RENDER_MINOR: "137", core.ATTR_INDEX: "9", core.ATTR_PARTITION: "CPX",
             core.ATTR_PARTITION_ID: "1", core.ATTR_SOCKET: "1", "amd.com/burn-in": "passed",
             "amd.com/mfma-tflops": "1188", "amd.com/mfma-fp8-tflops": "2242", "amd.com/hbm-gbps": "6199"}
    node = {"kind": "Node", "metadata": {"name": "n"}, "spec": {},
            "status": {"extendedResources": {core.AMD_GPU: {"resources": {"g9": {"health": "Healthy", "attributes": attrs}}}}}}
    out = describe(node)
    assert "partition=CPX/1@socket1" in out and "burn-in=passed (bf16 1188 / fp8 2242 TF/s, HBM 6199 GB/s)" in out


def test_drain_retries_while_a_budget_refuses(cluster, tmp_path, monkeypatch):
    """drain.go evictPods: 429 from the eviction API is retried until the budget allows it (or
    --timeout), then the pod's deletion is awaited."""
    from kubernetes_amd.kubectl.cli import Kubectl
    monkeypatch.setattr(Kubectl, "DRAIN_RETRY", 0.2)
    monkeypatch.setattr(Kubectl, "DRAIN_POLL", 0.1)
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "guarded", "labels": {"app": "guarded"}},
           "spec": {"nodeName": "node-0", "containers": [{"name": "c", "image": "x"}]}}
    pdb = {"apiVersion": "policy/v1beta1", "kind": "PodDisruptionBudget", "metadata": {"name": "guard"},
           "spec": {"minAvailable": 1, "selector": {"matchLabels": {"app": "guarded"}}}}
    for name, obj in (("pod.json", pod), ("pdb.json", pdb)):
        (tmp_path / name).write_text(json.dumps(obj))
        assert k(cluster, "create", "-f", str(tmp_path / name))[0] == 0
    wait(lambda: "Running" in k(cluster, "get", "pods", "guarded")[1])
    wait(lambda: json.loads(k(cluster, "get", "pdb", "guard", "-o", "json")[1]).get("status", {}).get("currentHealthy") == 1)
    with pytest.raises(SystemExit, match="Drain did not complete"):
        k(cluster, "drain", "node-0", "--force", "--ignore-daemonsets", "--timeout", "1")
    assert "guarded" in k(cluster, "get", "pods", "guarded")[1]
    assert k(cluster, "delete", "pdb", "guard")[0] == 0          # a budget's spec is immutable in 1.9
    rc, out = k(cluster, "drain", "node-0", "--force", "--ignore-daemonsets", "--timeout", "20")
    assert rc == 0 and "pod/guarded evicted" in out and "node/node-0 drained" in out
    assert k(cluster, "uncordon", "node-0")[0] == 0


def test_get_all_and_reference_columns(cluster):
    """`kubectl get all` (the legacy user-resource category) and the reference printers'
    columns for services, endpoints, service accounts and namespaces."""
    rc, out = k(cluster, "get", "all")
    assert rc == 0 and "svc/kubernetes" in out and "CLUSTER-IP" in out and "443/TCP" in out
    rc, out = k(cluster, "get", "ep", "kubernetes")
    assert out.splitlines()[0].split() == ["NAME", "ENDPOINTS", "AGE"]
    rc, out = k(cluster, "get", "sa", "-n", "kube-system")
    assert out.splitlines()[0].split()[:2] == ["NAME", "SECRETS"]
    rc, out = k(cluster, "get", "ns", "--all-namespaces")
    assert out.splitlines()[0].split() == ["NAME", "STATUS", "AGE"]          # cluster-scoped: no NAMESPACE column


@pytest.mark.parametrize("status,deleting,expect", [
    ({"phase": "Running", "containerStatuses": [{"ready": True, "state": {"running": {}}, "restartCount": 2}]}, False, ("Running", 2)),
    ({"phase": "Pending", "initContainerStatuses": [{"state": {"waiting": {"reason": "PodInitializing"}}}]}, False, ("Init:0/1", 0)),
    ({"phase": "Pending", "initContainerStatuses": [{"state": {"terminated": {"exitCode": 3}}, "restartCount": 1}]}, False,
     ("Init:ExitCode:3", 1)),
    ({"phase": "Running", "containerStatuses": [{"state": {"waiting": {"reason": "CrashLoopBackOff"}}, "restartCount": 4}]},
     False, ("CrashLoopBackOff", 4)),
    ({"phase": "Succeeded", "containerStatuses": [{"state": {"terminated": {"exitCode": 0, "reason": "Completed"}}}]},
     False, ("Completed", 0)),
    ({"phase": "Running", "containerStatuses": [{"ready": True, "state": {"running": {}}},
                                                {"state": {"terminated": {"exitCode": 0, "reason": "Completed"}}}]},
     False, ("Running", 0)),
    ({"phase": "Failed", "containerStatuses": [{"state": {"terminated": {"exitCode": 137, "signal": 9}}}]}, False, ("Signal:9", 0)),
    ({"phase": "Running"}, True, ("Terminating", 0)),
    ({"phase": "Failed", "reason": "Evicted"}, False, ("Evicted", 0)),
])
def test_pod_status_column(status, deleting, expect):
    """printPod's STATUS / RESTARTS columns (`pkg/printers/internalversion/printers_test.go`
    TestPrintPod cases)."""
    from kubernetes_amd.kubectl.printers import pod_status_and_restarts
    p = {"metadata": {"name": "p"}, "spec": {"initContainers": [{"name": "i"}]} if "initContainerStatuses" in status else {},
         "status": status}
    if deleting:
        p["metadata"]["deletionTimestamp"] = "2000-01-01T00:00:00Z"
    assert pod_status_and_restarts(p) == expect


def test_logs_need_a_container_name_for_multi_container_pods(cluster):
    """`log.go` validateContainer: a multi-container pod's logs need a container name."""
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "two"},
           "spec": {"containers": [{"name": "a", "image": "x"}, {"name": "b", "image": "x"}]}}
    import tempfile
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump(pod, f)
    assert k(cluster, "create", "-f", f.name)[0] == 0
    wait(lambda: "Running" in k(cluster, "get", "pods", "two")[1])
    with pytest.raises(SystemExit, match="a container name must be specified for pod two, choose one of: \\[a b\\]"):
        k(cluster, "logs", "two")
    with pytest.raises(SystemExit, match="container c is not valid for pod two"):
        k(cluster, "logs", "two", "-c", "c")
    k(cluster, "delete", "pod", "two", "--grace-period", "0")


def test_get_pods_hides_terminated_unless_show_all(cluster):
    """kubectl 1.9 `filterPods`: lists hide Succeeded / Failed pods unless --show-all; a named
    pod is always printed."""
    import tempfile
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "done", "annotations": {"kubemark.amd.com/run-seconds": "0"}},
           "spec": {"restartPolicy": "Never", "containers": [{"name": "c", "image": "x"}]}}
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump(pod, f)
    assert k(cluster, "create", "-f", f.name)[0] == 0
    wait(lambda: "Completed" in k(cluster, "get", "pod", "done")[1])
    assert "done" not in k(cluster, "get", "pods")[1]
    assert "done" in k(cluster, "get", "pods", "--show-all")[1]
    k(cluster, "delete", "pod", "done", "--grace-period", "0")
