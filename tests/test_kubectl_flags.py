"""kubectl's reference flags against a live local cluster: get (sort-by, label columns,
show-labels, no-headers, ignore-not-found, --raw), label/annotate (--overwrite, -l, --list,
--dry-run, --local), patch (--dry-run/-o), scale -l, taint (--overwrite, removal), drain
(--dry-run, --delete-local-data), rollout pause/resume, run (generators, --dry-run -o,
--expose), expose (port introspection), version -o, cluster-info (dump), explain, logs
(-l, --timestamps, --limit-bytes, -f), edit --output-patch, delete --now.

Parity: `pkg/kubectl/cmd/*.go` (get.go, label.go, annotate.go, patch.go, scale.go, taint.go,
drain.go, rollout/, run.go, expose.go, version.go, clusterinfo*.go, explain.go, logs.go,
edit.go, delete.go).
"""
import asyncio
import io
import json
import os
import sys
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


def wait(pred, timeout=30):
    t = time.time()
    while time.time() - t < timeout:
        r = pred()
        if r:
            return r
        time.sleep(0.05)
    raise TimeoutError


def _pod(name, labels=None, cmd=None, volumes=None):
    c = {"name": "c", "image": "busybox"}
    if cmd:
        c["command"] = cmd
    spec = {"containers": [c]}
    if volumes:
        spec["volumes"] = volumes
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "labels": labels or {}}, "spec": spec}


def _create(cluster, tmp_path, obj):
    f = tmp_path / f"{obj['metadata']['name']}.yaml"
    f.write_text(yaml.safe_dump(obj))
    rc, out = k(cluster, "create", "-f", str(f))
    assert rc == 0, out
    return f


def test_get_printing_flags(cluster, tmp_path):
    for n, tier in (("zeta", "b"), ("alpha", "a"), ("mid", "c")):
        _create(cluster, tmp_path, _pod(f"gp-{n}", {"tier": tier, "grp": "gp"}))
    rc, out = k(cluster, "get", "pods", "-l", "grp=gp", "--sort-by", "{.metadata.labels.tier}", "--no-headers",
                "-L", "tier")
    lines = out.strip().splitlines()
    assert [ln.split()[0] for ln in lines] == ["gp-alpha", "gp-zeta", "gp-mid"]
    assert [ln.split()[-1] for ln in lines] == ["a", "b", "c"] and "NAME" not in out
    rc, out = k(cluster, "get", "pods", "gp-alpha", "--show-labels", "--show-kind")
    assert "LABELS" in out.splitlines()[0] and "grp=gp,tier=a" in out and "pod/gp-alpha" in out
    rc, out = k(cluster, "get", "pods", "nope", "--ignore-not-found")
    assert rc == 0 and out.strip() == ""
    rc, out = k(cluster, "get", "--raw", "/api/v1/namespaces/default/pods/gp-mid")
    assert json.loads(out)["metadata"]["labels"]["tier"] == "c"
    rc, out = k(cluster, "get", "pods", "-l", "grp=gp", "--chunk-size", "1", "-o", "name")
    assert sorted(out.split()) == ["pod/gp-alpha", "pod/gp-mid", "pod/gp-zeta"]


def test_label_annotate_flags(cluster, tmp_path):
    f = _create(cluster, tmp_path, _pod("lb-1", {"app": "lb", "v": "1"}))
    _create(cluster, tmp_path, _pod("lb-2", {"app": "lb"}))
    with pytest.raises(SystemExit, match="already has a value"):
        k(cluster, "label", "pod", "lb-1", "v=2")
    assert k(cluster, "label", "pod", "lb-1", "v=2", "--overwrite")[0] == 0
    rc, out = k(cluster, "label", "pods", "-l", "app=lb", "team=gpu")
    assert rc == 0 and "pod/lb-1 labeled" in out and "pod/lb-2 labeled" in out
    rc, out = k(cluster, "label", "pod", "lb-1", "--list")
    assert "v=2" in out.splitlines() and "team=gpu" in out.splitlines()
    rc, out = k(cluster, "label", "pod", "lb-2", "x=y", "--dry-run", "-o", "json")
    assert json.loads(out)["metadata"]["labels"]["x"] == "y"
    assert "x" not in json.loads(k(cluster, "get", "pod", "lb-2", "-o", "json")[1])["metadata"]["labels"]
    rc, out = k(cluster, "label", "--local", "-f", str(f), "only=local", "-o", "yaml")
    assert yaml.safe_load(out)["metadata"]["labels"]["only"] == "local"
    assert "only" not in json.loads(k(cluster, "get", "pod", "lb-1", "-o", "json")[1])["metadata"]["labels"]
    assert k(cluster, "annotate", "pods", "--all", "note=hi")[0] == 0
    with pytest.raises(SystemExit, match="--overwrite is false"):
        k(cluster, "annotate", "pod", "lb-2", "note=bye")
    assert json.loads(k(cluster, "get", "pod", "lb-2", "-o", "json")[1])["metadata"]["annotations"]["note"] == "hi"


def test_patch_scale_rollout_pause(cluster, tmp_path):
    dep = {"apiVersion": "apps/v1beta1", "kind": "Deployment", "metadata": {"name": "web", "labels": {"tier": "fe"}},
           "spec": {"replicas": 1, "selector": {"matchLabels": {"app": "web"}},
                    "template": {"metadata": {"labels": {"app": "web"}},
                                 "spec": {"containers": [{"name": "c", "image": "busybox",
                                                          "ports": [{"containerPort": 8080}]}]}}}}
    _create(cluster, tmp_path, dep)
    rc, out = k(cluster, "patch", "deployment", "web", "-p", '{"spec":{"replicas":5}}', "--dry-run", "-o", "json")
    assert json.loads(out)["spec"]["replicas"] == 5
    assert json.loads(k(cluster, "get", "deployment", "web", "-o", "json")[1])["spec"]["replicas"] == 1
    rc, out = k(cluster, "scale", "deployments", "-l", "tier=fe", "--replicas", "2", "--timeout", "30")
    assert rc == 0, out
    assert 'deployment "web" scaled' in out, out
    assert k(cluster, "rollout", "pause", "deployment/web")[1].strip() == 'deployment "web" paused'
    assert json.loads(k(cluster, "get", "deployment", "web", "-o", "json")[1])["spec"]["paused"] is True
    assert "already paused" in k(cluster, "rollout", "pause", "deployment/web")[1]
    assert k(cluster, "rollout", "resume", "deployment/web")[1].strip() == 'deployment "web" resumed'
    rc, out = k(cluster, "rollout", "history", "deployment/web", "--revision", "1")
    assert rc == 0 and 'deployment "web" with revision #1' in out and "Image:      busybox" in out
    # expose derives the port from the pod template
    rc, out = k(cluster, "expose", "deployment", "web", "--dry-run", "-o", "json")
    svc = json.loads(out)
    assert svc["spec"]["ports"] == [{"port": 8080, "protocol": "TCP", "targetPort": 8080}]
    assert svc["spec"]["selector"] == {"app": "web"} and svc["metadata"]["labels"] == {"tier": "fe"}
    rc, out = k(cluster, "expose", "deployment", "web", "--port", "80", "--target-port", "8080", "--type", "NodePort",
                "--name", "web-np")
    assert rc == 0, out
    assert "service/web-np exposed" in out, out
    s = json.loads(k(cluster, "get", "svc", "web-np", "-o", "json")[1])
    assert s["spec"]["type"] == "NodePort" and s["spec"]["ports"][0]["targetPort"] == 8080


def test_taint_flags(cluster):
    assert k(cluster, "taint", "nodes", "node-1", "gpu=mi355x:NoSchedule")[0] == 0
    with pytest.raises(SystemExit, match="--overwrite is false"):
        k(cluster, "taint", "nodes", "node-1", "gpu=other:NoSchedule")
    assert k(cluster, "taint", "nodes", "node-1", "gpu=other:NoSchedule", "--overwrite")[0] == 0
    n = json.loads(k(cluster, "get", "node", "node-1", "-o", "json")[1])
    assert [t for t in n["spec"]["taints"] if t["key"] == "gpu"] == [{"key": "gpu", "value": "other", "effect": "NoSchedule"}]
    with pytest.raises(SystemExit, match="invalid taint effect"):
        k(cluster, "taint", "nodes", "node-1", "a=b:Sometimes")
    assert k(cluster, "taint", "nodes", "node-1", "gpu:NoSchedule-")[0] == 0
    assert "node/node-1 cordoned (dry run)" in k(cluster, "cordon", "node-1", "--dry-run")[1]
    assert not json.loads(k(cluster, "get", "node", "node-1", "-o", "json")[1])["spec"].get("unschedulable")
    assert "already uncordoned" in k(cluster, "uncordon", "node-1")[1]
    n = json.loads(k(cluster, "get", "node", "node-1", "-o", "json")[1])
    assert not [t for t in (n["spec"].get("taints") or ()) if t["key"] == "gpu"]


def test_drain_dry_run_and_local_data(cluster, tmp_path):
    p = _pod("scratch", volumes=[{"name": "tmp", "emptyDir": {}}])
    p["spec"]["nodeName"] = "node-0"
    p["metadata"]["ownerReferences"] = []
    _create(cluster, tmp_path, p)
    with pytest.raises(SystemExit, match="not managed by"):
        k(cluster, "drain", "node-0", "--dry-run", "--ignore-daemonsets")
    with pytest.raises(SystemExit, match="local storage"):
        k(cluster, "drain", "node-0", "--dry-run", "--ignore-daemonsets", "--force")
    rc, out = k(cluster, "drain", "node-0", "--dry-run", "--ignore-daemonsets", "--force", "--delete-local-data")
    assert rc == 0 and "pod/scratch evicted (dry run)" in out and "drained (dry run)" in out
    assert not json.loads(k(cluster, "get", "node", "node-0", "-o", "json")[1])["spec"].get("unschedulable")
    k(cluster, "delete", "pod", "scratch", "--now")


def test_run_generators(cluster):
    rc, out = k(cluster, "run", "gen-dep", "--image", "busybox", "--replicas", "3", "--env", "A=1", "--port", "80",
                "--limits", "cpu=200m,memory=64Mi", "--dry-run", "-o", "json")
    d = json.loads(out)
    assert d["kind"] == "Deployment" and d["spec"]["replicas"] == 3
    c = d["spec"]["template"]["spec"]["containers"][0]
    assert c["env"] == [{"name": "A", "value": "1"}] and c["ports"] == [{"containerPort": 80}]
    assert c["resources"]["limits"] == {"cpu": "200m", "memory": "64Mi"}
    assert json.loads(k(cluster, "run", "gen-job", "--image", "busybox", "--restart", "OnFailure", "--dry-run",
                        "-o", "json")[1])["kind"] == "Job"
    assert json.loads(k(cluster, "run", "gen-cj", "--image", "busybox", "--schedule", "*/5 * * * *", "--restart",
                        "OnFailure", "--dry-run", "-o", "json")[1])["kind"] == "CronJob"
    o = json.loads(k(cluster, "run", "gen-pod", "--image", "busybox", "--restart", "Never", "--command", "--dry-run",
                     "-o", "json", "--", "sh", "-c", "true")[1])
    assert o["kind"] == "Pod" and o["spec"]["containers"][0]["command"] == ["sh", "-c", "true"]
    rc, out = k(cluster, "run", "svcd", "--image", "busybox", "--port", "9000", "--expose")
    assert rc == 0 and "service/svcd created" in out and "deployment/svcd created" in out
    s = json.loads(k(cluster, "get", "svc", "svcd", "-o", "json")[1])
    assert s["spec"]["selector"] == {"run": "svcd"} and s["spec"]["ports"][0]["port"] == 9000
    with pytest.raises(SystemExit, match="--rm should only be used"):
        k(cluster, "run", "x", "--image", "busybox", "--rm")


def test_version_cluster_info_explain(cluster, tmp_path):
    rc, out = k(cluster, "version", "-o", "json")
    v = json.loads(out)
    assert v["clientVersion"]["gitVersion"] and v["serverVersion"]["gitVersion"]
    assert "Server" not in k(cluster, "version", "--client", "--short")[1]
    rc, out = k(cluster, "cluster-info")
    assert out.startswith("Kubernetes master is running at")
    d = tmp_path / "dump"
    rc, out = k(cluster, "cluster-info", "dump", "--output-directory", str(d), "--namespaces", "default")
    assert rc == 0 and (d / "nodes.json").exists() and (d / "default" / "pods.json").exists()
    assert json.loads((d / "nodes.json").read_text())["items"]
    rc, out = k(cluster, "explain", "pods")
    assert "KIND:     Pod" in out and "metadata" in out and "FIELDS:" in out
    rc, out = k(cluster, "explain", "pods.metadata")
    assert "RESOURCE: metadata <Object>" in out and "labels" in out
    with pytest.raises(SystemExit, match="does not exist"):
        k(cluster, "explain", "pods.nope")


def test_logs_flags(run, tmp_path):
    """logs needs a real kubelet endpoint: a process-runtime cluster serving kubelet HTTP."""
    from kubernetes_amd.kubectl.cli import Kubectl, build_parser

    async def kc(url, *argv):
        out = io.StringIO()
        kk = Kubectl(build_parser().parse_args(["-s", url, *argv]), out)
        kk.rc = 0
        try:
            await kk.cmd_logs()
        finally:
            await kk.client.close()
        return out.getvalue()

    async def main():
        cl = LocalCluster(nodes=1, gpus_per_node=0, runtime="process", kubelet_http=True, workdir=str(tmp_path / "c"))
        await cl.start()
        try:
            script = "import time\nfor i in range(1, 6): print(f'line-{i}', flush=True)\ntime.sleep(30)"
            follow = "import time\nfor i in range(1, 4): print(f'f-{i}', flush=True); time.sleep(0.3)"
            for name, code in (("talker", script), ("follower", follow)):
                await cl.client.create("pods", {"metadata": {"name": name, "namespace": "default", "labels": {"app": name}},
                                                "spec": {"nodeName": cl.nodes[0].name, "restartPolicy": "Never",
                                                         "containers": [{"name": "c", "image": "busybox",
                                                                         "command": [sys.executable, "-c", code]}]}})
            await cl.wait_pod("talker")
            await cl.wait_pod("follower")
            # -f streams until the container exits
            out = await asyncio.wait_for(kc(cl.url, "logs", "-f", "follower"), 30)
            assert out.split() == ["f-1", "f-2", "f-3"]
            for _ in range(200):
                if "line-5" in await kc(cl.url, "logs", "talker"):
                    break
                await asyncio.sleep(0.05)
            assert "line-1" in await kc(cl.url, "logs", "-l", "app=talker")
            assert (await kc(cl.url, "logs", "talker", "--tail", "2")).split() == ["line-4", "line-5"]
            assert await kc(cl.url, "logs", "talker", "--limit-bytes", "7") == "line-1\n"
            ts, _, text = (await kc(cl.url, "logs", "talker", "--timestamps", "--tail", "1")).strip().partition(" ")
            assert text == "line-5" and ts[:2] == "20" and ts.endswith("Z")
            assert "line-3" in await kc(cl.url, "logs", "talker", "--since", "1h")
            assert "line-3" in await kc(cl.url, "logs", "talker", "c")     # container as the 2nd positional
        finally:
            await cl.stop()
    run(main())


def test_describe_kinds(cluster, tmp_path):
    """Per-kind describers (`pkg/printers/internalversion/describe.go`)."""
    dep = {"apiVersion": "apps/v1beta1", "kind": "Deployment", "metadata": {"name": "dsc"},
           "spec": {"replicas": 2, "selector": {"matchLabels": {"app": "dsc"}},
                    "template": {"metadata": {"labels": {"app": "dsc"}},
                                 "spec": {"containers": [{"name": "c", "image": "busybox", "env": [{"name": "A", "value": "1"}],
                                                          "ports": [{"containerPort": 7000}],
                                                          "resources": {"limits": {"cpu": "100m"}}}]}}}}
    _create(cluster, tmp_path, dep)
    wait(lambda: "2 available" in k(cluster, "describe", "deployment", "dsc")[1])
    out = k(cluster, "describe", "deployment", "dsc")[1]
    assert "2 desired | 2 updated | 2 total | 2 available" in out and "RollingUpdateStrategy:  25% max unavailable" in out
    assert "NewReplicaSet:   dsc-" in out and "A:  1" in out and "Port:       7000/TCP" in out
    rs = json.loads(k(cluster, "get", "rs", "-l", "app=dsc", "-o", "json")[1])["items"][0]["metadata"]["name"]
    assert "Pods Status:  2 Running / 0 Waiting" in k(cluster, "describe", "rs", rs)[1]
    k(cluster, "expose", "deployment", "dsc", "--port", "80", "--target-port", "7000")
    out = wait(lambda: (lambda o: o if "Endpoints:         <none>" not in o else None)(k(cluster, "describe", "svc", "dsc")[1]))
    assert "Type:              ClusterIP" in out and "TargetPort:        7000/TCP" in out and ":7000" in out
    sec = {"apiVersion": "v1", "kind": "Secret", "metadata": {"name": "dsc-s"}, "data": {"pw": "aHVudGVyMg=="}}
    _create(cluster, tmp_path, sec)
    out = k(cluster, "describe", "secret", "dsc-s")[1]
    assert "pw:  7 bytes" in out and "hunter2" not in out and "aHVudGVyMg" not in out
    out = k(cluster, "describe", "namespace", "default")[1]
    assert "Status:  Active" in out and "No resource quota." in out
    out = k(cluster, "describe", "node", "node-0")[1]
    assert "Non-terminated Pods:" in out and "Allocated resources:" in out and "amd.com/gpu" in out


def test_apply_last_applied_and_can_i(cluster, tmp_path):
    cm = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "lac"}, "data": {"a": "1"}}
    f = tmp_path / "cm.yaml"
    f.write_text(yaml.safe_dump(cm))
    assert k(cluster, "apply", "-f", str(f))[0] == 0
    rc, out = k(cluster, "apply", "view-last-applied", "configmap", "lac", "-o", "json")
    assert json.loads(out)["data"] == {"a": "1"}
    cm["data"] = {"a": "2", "b": "3"}
    f.write_text(yaml.safe_dump(cm))
    assert "configmap/lac configured" in k(cluster, "apply", "set-last-applied", "-f", str(f))[1]
    assert yaml.safe_load(k(cluster, "apply", "view-last-applied", "configmap/lac")[1])["data"] == {"a": "2", "b": "3"}
    assert json.loads(k(cluster, "get", "cm", "lac", "-o", "json")[1])["data"] == {"a": "1"}   # only the annotation
    bare = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "bare"}, "data": {}}
    _create(cluster, tmp_path, bare)
    g = tmp_path / "bare.yaml"
    g.write_text(yaml.safe_dump(bare))
    with pytest.raises(SystemExit, match="--create-annotation"):
        k(cluster, "apply", "set-last-applied", "-f", str(g))
    assert k(cluster, "apply", "set-last-applied", "-f", str(g), "--create-annotation")[0] == 0
    # auth can-i answers through a SelfSubjectAccessReview (the local cluster allows everything)
    rc, out = k(cluster, "auth", "can-i", "create", "pods")
    assert rc == 0 and out.strip() == "yes"
    rc, out = k(cluster, "auth", "can-i", "get", "/healthz", "-q")
    assert rc == 0 and out == ""


def test_set_flags(cluster, tmp_path):
    """`kubectl set` (pkg/kubectl/cmd/set): TYPE NAME form, -l, --local -f, --dry-run -o, image
    `*=`, env -e / --from / --list / --overwrite=false."""
    dep = {"apiVersion": "apps/v1beta1", "kind": "Deployment", "metadata": {"name": "setd", "labels": {"grp": "set"}},
           "spec": {"replicas": 1, "selector": {"matchLabels": {"app": "setd"}},
                    "template": {"metadata": {"labels": {"app": "setd"}},
                                 "spec": {"containers": [{"name": "a", "image": "busybox"},
                                                         {"name": "b", "image": "busybox"}]}}}}
    f = _create(cluster, tmp_path, dep)
    rc, out = k(cluster, "set", "image", "deployments", "-l", "grp=set", "*=img:2")
    assert rc == 0 and "deployment/setd image updated" in out
    d = json.loads(k(cluster, "get", "deploy", "setd", "-o", "json")[1])
    assert [c["image"] for c in d["spec"]["template"]["spec"]["containers"]] == ["img:2", "img:2"]
    rc, out = k(cluster, "set", "image", "--local", "-f", str(f), "a=local:1", "-o", "json")
    assert json.loads(out)["spec"]["template"]["spec"]["containers"][0]["image"] == "local:1"
    rc, out = k(cluster, "set", "resources", "deployment", "setd", "--limits", "cpu=2", "--dry-run", "-o", "yaml")
    assert yaml.safe_load(out)["spec"]["template"]["spec"]["containers"][0]["resources"]["limits"]["cpu"] == "2"
    d = json.loads(k(cluster, "get", "deploy", "setd", "-o", "json")[1])
    assert "resources" not in d["spec"]["template"]["spec"]["containers"][0]            # dry run wrote nothing
    cm = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "envsrc"}, "data": {"db-host": "x", "port": "1"}}
    _create(cluster, tmp_path, cm)
    assert k(cluster, "set", "env", "deployment/setd", "-e", "MODE=fast", "--from", "configmap/envsrc", "--prefix",
             "app_")[0] == 0
    rc, out = k(cluster, "set", "env", "deployment/setd", "--list", "-c", "a")
    assert "MODE=fast" in out and "# APP_DB_HOST from configmap envsrc, key db-host" in out
    with pytest.raises(SystemExit, match="--overwrite is false"):
        k(cluster, "set", "env", "deployment/setd", "MODE=slow", "--overwrite=false")
    assert k(cluster, "set", "env", "deployment/setd", "MODE-")[0] == 0
    assert "MODE=" not in k(cluster, "set", "env", "deployment/setd", "--list")[1]
