"""Kubelet: volumes (configMap / secret / downwardAPI / emptyDir / hostPath / projected),
env valueFrom + envFrom, liveness / readiness probes."""
import asyncio
import base64
import json
import os

from kubernetes_amd.cluster import LocalCluster


def test_volumes_and_env_process_runtime(run, tmp_path):
    hp = str(tmp_path / "host")

    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=0, runtime="process") as cl:
            c = cl.client
            await c.create("configmaps", {"metadata": {"name": "cfg", "namespace": "default"},
                                          "data": {"model": "llama-70b", "batch": "32"}})
            await c.create("secrets", {"metadata": {"name": "tok", "namespace": "default"},
                                       "data": {"token": base64.b64encode(b"s3cr3t").decode()}})
            script = ("cat $KUBERNETES_VOLUME_CFG/model; echo; cat $KUBERNETES_VOLUME_SEC/t; echo; "
                      "cat $KUBERNETES_VOLUME_INFO/labels; echo; echo POD=$MY_POD NS=$MY_NS NODE=$MY_NODE "
                      "MODEL=$MODEL TOKEN=$TOKEN B=$CFG_batch CPU=$CPU_LIMIT MSG=$MSG; "
                      "echo hi > $KUBERNETES_VOLUME_SCRATCH/x; ls $KUBERNETES_VOLUME_HOST; cat $KUBERNETES_VOLUME_PROJ/model")
            pod = {"metadata": {"name": "vol", "namespace": "default", "labels": {"app": "train"}},
                   "spec": {"restartPolicy": "Never",
                            "volumes": [{"name": "cfg", "configMap": {"name": "cfg"}},
                                        {"name": "sec", "secret": {"secretName": "tok", "items": [{"key": "token", "path": "t"}]}},
                                        {"name": "info", "downwardAPI": {"items": [{"path": "labels", "fieldRef": {"fieldPath": "metadata.labels"}}]}},
                                        {"name": "scratch", "emptyDir": {}},
                                        {"name": "host", "hostPath": {"path": hp, "type": "DirectoryOrCreate"}},
                                        {"name": "proj", "projected": {"sources": [{"configMap": {"name": "cfg"}}]}}],
                            "containers": [{"name": "c", "image": "busybox", "command": ["/bin/sh", "-c", script],
                                            "resources": {"limits": {"cpu": "2"}},
                                            "volumeMounts": [{"name": n, "mountPath": f"/mnt/{n}"} for n in
                                                             ("cfg", "sec", "info", "scratch", "host", "proj")],
                                            "envFrom": [{"configMapRef": {"name": "cfg"}, "prefix": "CFG_"}],
                                            "env": [{"name": "MY_POD", "valueFrom": {"fieldRef": {"fieldPath": "metadata.name"}}},
                                                    {"name": "MY_NS", "valueFrom": {"fieldRef": {"fieldPath": "metadata.namespace"}}},
                                                    {"name": "MY_NODE", "valueFrom": {"fieldRef": {"fieldPath": "spec.nodeName"}}},
                                                    {"name": "MODEL", "valueFrom": {"configMapKeyRef": {"name": "cfg", "key": "model"}}},
                                                    {"name": "TOKEN", "valueFrom": {"secretKeyRef": {"name": "tok", "key": "token"}}},
                                                    {"name": "CPU_LIMIT", "valueFrom": {"resourceFieldRef": {"resource": "limits.cpu"}}},
                                                    {"name": "MSG", "value": "model=$(MODEL)"}]}]}}
            await c.create("pods", pod)
            p = await cl.wait_pod("vol", phase="Succeeded", timeout=30)
            assert p["status"]["containerStatuses"][0]["state"]["terminated"]["exitCode"] == 0
            rt = cl.nodes[0].runtime
            cs = rt.list_containers()[0]
            log = open(cs.log_path).read()
            assert "llama-70b" in log and "s3cr3t" in log and 'app="train"' in log
            assert "POD=vol NS=default NODE=node-0 MODEL=llama-70b TOKEN=s3cr3t B=32 CPU=2 MSG=model=llama-70b" in log
            assert log.rstrip().endswith("llama-70b")
            spec = json.load(open(os.path.join(os.path.dirname(cs.log_path), "config.json")))
            dests = {m["destination"] for m in spec["mounts"]}
            assert {"/mnt/cfg", "/mnt/sec", "/mnt/scratch"} <= dests
            assert os.path.isdir(hp)
    run(main(), timeout=120)


def test_missing_configmap_blocks_then_recovers(run):
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=0) as cl:
            c = cl.client
            await c.create("pods", {"metadata": {"name": "wait-cm", "namespace": "default"},
                                    "spec": {"volumes": [{"name": "v", "configMap": {"name": "later"}}],
                                             "containers": [{"name": "c", "image": "x",
                                                             "volumeMounts": [{"name": "v", "mountPath": "/v"}]}]}})
            await asyncio.sleep(0.5)
            p = await c.get("pods", "wait-cm", "default")
            assert p["status"]["phase"] == "Pending"
            await c.create("configmaps", {"metadata": {"name": "later", "namespace": "default"}, "data": {"a": "1"}})
            await cl.wait_pod("wait-cm", timeout=10)
    run(main(), timeout=60)


def test_readiness_and_liveness_probes(run):
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=0) as cl:
            c = cl.client
            probe = {"exec": {"command": ["check"]}, "periodSeconds": 1, "failureThreshold": 1}
            await c.create("pods", {"metadata": {"name": "pr", "namespace": "default"},
                                    "spec": {"containers": [{"name": "c", "image": "x", "readinessProbe": probe,
                                                             "livenessProbe": dict(probe, failureThreshold=2)}]}})
            p = await cl.wait_pod("pr")
            uid = p["metadata"]["uid"]

            async def cond(pred):
                for _ in range(600):
                    p = await c.get("pods", "pr", "default")
                    if pred(p):
                        return p
                    await asyncio.sleep(0.02)
                raise AssertionError(p["status"])
            ready = lambda p: any(x["type"] == "Ready" and x["status"] == "True" for x in p["status"]["conditions"])  # noqa: E731
            await cond(ready)
            rt = cl.nodes[0].runtime
            # readiness fails -> Ready=False while the container keeps running (liveness still ok... until it fails too)
            rt.exec_codes[(uid, "c")] = 1
            p = await cond(lambda p: not ready(p) or p["status"]["containerStatuses"][0]["restartCount"] >= 1)
            # liveness failed twice -> container killed and restarted
            p = await cond(lambda p: p["status"]["containerStatuses"][0]["restartCount"] >= 1)
            rt.exec_codes[(uid, "c")] = 0
            p = await cond(lambda p: ready(p) and p["status"]["containerStatuses"][0]["state"].get("running"))
            # the killed instance is the restarted container's lastState (kubectl describe "Last State")
            last = p["status"]["containerStatuses"][0].get("lastState", {}).get("terminated")
            assert last is not None and "exitCode" in last, p["status"]["containerStatuses"][0]
            # prober.go: every failed probe is an Unhealthy event naming the probe type
            emitted = cl.nodes[0].kubelet.recorder.emitted
            assert any(r == "Unhealthy" and m.startswith("Readiness probe failed") for _t, r, m in emitted)
            assert any(r == "Unhealthy" and m.startswith("Liveness probe failed") for _t, r, m in emitted)
    run(main(), timeout=60)


def test_node_status_transitions_images_and_machine_info(run):
    """`kubelet_node_status.go`: lastTransitionTime moves only when a condition's status changes
    (the node controller's NotReady eviction timer depends on it), OutOfDisk is reported, images
    are listed largest first, and the machine / boot identity is filled in."""
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=0) as cl:
            c, k = cl.client, cl.nodes[0].kubelet
            await c.create("pods", {"metadata": {"name": "img", "namespace": "default"},
                                    "spec": {"containers": [{"name": "c", "image": "busybox"}]}})
            await cl.wait_pod("img")

            async def status():
                await k.update_node_status()
                return (await c.get("nodes", k.node_name))["status"]
            s1 = await status()
            await asyncio.sleep(1.1)                       # RFC 3339 timestamps have 1 s resolution
            s2 = await status()
            by = lambda s: {x["type"]: x for x in s["conditions"]}  # noqa: E731
            r1, r2 = by(s1)["Ready"], by(s2)["Ready"]
            assert r1["lastTransitionTime"] == r2["lastTransitionTime"]
            assert r2["lastHeartbeatTime"] > r1["lastHeartbeatTime"]
            assert by(s2)["OutOfDisk"]["status"] == "False"
            assert any(any("busybox" in n for n in i["names"]) for i in s2.get("images") or ())
            assert s2["nodeInfo"]["bootID"] and s2["nodeInfo"]["kernelVersion"]
    run(main(), timeout=60)


def test_pod_is_pending_while_any_container_waits(run):
    """`GetPhase`: one running container does not make the pod Running while another waits
    (here: an image that may never be pulled)."""
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=0) as cl:
            c = cl.client
            await c.create("pods", {"metadata": {"name": "half", "namespace": "default"},
                                    "spec": {"containers": [{"name": "ok", "image": "busybox"},
                                                            {"name": "stuck", "image": "never-pulled:1",
                                                             "imagePullPolicy": "Never"}]}})
            for _ in range(200):
                p = await c.get("pods", "half", "default")
                cs = {s["name"]: s for s in (p.get("status") or {}).get("containerStatuses") or ()}
                if cs.get("ok", {}).get("state", {}).get("running") and cs.get("stuck", {}).get("state", {}).get("waiting"):
                    break
                await asyncio.sleep(0.02)
            assert cs["stuck"]["state"]["waiting"]["reason"] == "ErrImageNeverPull"
            assert p["status"]["phase"] == "Pending"
    run(main(), timeout=60)
