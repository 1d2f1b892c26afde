"""Conformance-style e2e specs (mirrors of `test/e2e/common/*`, `test/e2e/apps/*`,
`test/e2e/network/service.go`, `test/e2e/scheduling/predicates.go`,
`test/e2e/scheduling/nvidia-gpus.go`). Each spec runs in its own namespace."""
from __future__ import annotations

import base64

from ..api import core
from .framework import conformance, spec

BUSYBOX = "busybox"


def _pod(name, cmd, restart="Never", **spec_extra):
    return {"metadata": {"name": name, "labels": {"app": name}},
            "spec": dict({"restartPolicy": restart, "containers": [{"name": "c", "image": BUSYBOX,
                                                                     "command": ["sh", "-c", cmd]}]}, **spec_extra)}


@conformance("Pods should run to completion and expose their logs")
async def pod_logs(f):
    await f.client.create("pods", _pod("hello", "echo hello-e2e"), f.ns)
    await f.pod_phase("hello", ("Succeeded",))
    assert "hello-e2e" in await f.logs("hello")


@conformance("Downward API should provide pod name and namespace as env vars")
async def downward_env(f):
    p = _pod("dapi", "echo $MY_NAME/$MY_NS")
    p["spec"]["containers"][0]["env"] = [
        {"name": "MY_NAME", "valueFrom": {"fieldRef": {"fieldPath": "metadata.name"}}},
        {"name": "MY_NS", "valueFrom": {"fieldRef": {"fieldPath": "metadata.namespace"}}}]
    await f.client.create("pods", p, f.ns)
    await f.pod_phase("dapi", ("Succeeded",))
    assert f"dapi/{f.ns}" in await f.logs("dapi")


@conformance("ConfigMap should be consumable from pods in volume")
async def configmap_volume(f):
    await f.client.create("configmaps", {"metadata": {"name": "cfg"}, "data": {"data-1": "value-1"}}, f.ns)
    # the in-process runtime has no mount namespace: it exposes the volume's host path in
    # KUBERNETES_VOLUME_<NAME>; container runtimes mount it at /etc/cfg
    p = _pod("cm", "cat /etc/cfg/data-1 2>/dev/null || cat $KUBERNETES_VOLUME_V/data-1")
    p["spec"]["containers"][0]["volumeMounts"] = [{"name": "v", "mountPath": "/etc/cfg"}]
    p["spec"]["volumes"] = [{"name": "v", "configMap": {"name": "cfg"}}]
    await f.client.create("pods", p, f.ns)
    await f.pod_phase("cm", ("Succeeded",))
    assert "value-1" in await f.logs("cm")


@conformance("Secrets should be consumable via environment variables")
async def secret_env(f):
    await f.client.create("secrets", {"metadata": {"name": "s"}, "data": {"pw": base64.b64encode(b"s3cr3t").decode()}}, f.ns)
    p = _pod("sec", "echo PW=$PW")
    p["spec"]["containers"][0]["env"] = [{"name": "PW", "valueFrom": {"secretKeyRef": {"name": "s", "key": "pw"}}}]
    await f.client.create("pods", p, f.ns)
    await f.pod_phase("sec", ("Succeeded",))
    assert "PW=s3cr3t" in await f.logs("sec")


@conformance("Deployment should run the requested replicas and roll out a new template")
async def deployment_rollout(f):
    d = {"metadata": {"name": "web"}, "spec": {"replicas": 2, "selector": {"matchLabels": {"app": "web"}},
                                               "template": {"metadata": {"labels": {"app": "web"}},
                                                            "spec": {"containers": [{"name": "c", "image": BUSYBOX,
                                                                                     "command": ["sh", "-c", "sleep 3600"]}]}}}}
    await f.client.create("deployments", d, f.ns)

    async def available(gen=None):
        x = await f.client.get("deployments", "web", f.ns)
        st = x.get("status") or {}
        ok = st.get("availableReplicas") == 2 and st.get("updatedReplicas") == 2 and st.get("replicas") == 2
        return x if ok and (gen is None or st.get("observedGeneration", 0) >= gen) else None
    await f.wait(available, 60, "deployment available")
    cur = await f.client.patch("deployments", "web", {"spec": {"template": {"metadata": {"labels": {"app": "web",
                                                                                                    "v": "2"}}}}}, f.ns)
    await f.wait(lambda: available(cur["metadata"].get("generation")), 60, "rollout of the new template")
    rs = [r for r in (await f.client.list("replicasets", f.ns))["items"] if (r.get("spec") or {}).get("replicas")]
    assert len(rs) == 1 and rs[0]["spec"]["template"]["metadata"]["labels"].get("v") == "2"


@conformance("Service should get a cluster IP and endpoints for ready pods")
async def service_endpoints(f):
    await f.client.create("pods", _pod("backend", "sleep 3600", restart="Always"), f.ns)
    await f.client.create("services", {"metadata": {"name": "svc"}, "spec": {"selector": {"app": "backend"},
                                                                             "ports": [{"port": 80}]}}, f.ns)
    svc = await f.client.get("services", "svc", f.ns)
    assert svc["spec"].get("clusterIP") not in (None, "", "None")
    pod = await f.pod_phase("backend", ("Running",))

    async def ep():
        e = await f.client.get("endpoints", "svc", f.ns)
        ips = [a["ip"] for s in e.get("subsets") or () for a in s.get("addresses") or ()]
        return ips if pod["status"].get("podIP") in ips else None
    await f.wait(ep, 60, "endpoints")


@conformance("Scheduler should respect nodeSelector and report unschedulable pods")
async def node_selector(f):
    nodes = (await f.client.list("nodes"))["items"]
    target = nodes[0]["metadata"]["name"]
    p = _pod("pinned", "true", nodeSelector={"kubernetes.io/hostname": target})
    await f.client.create("pods", p, f.ns)
    got = await f.pod_phase("pinned", ("Running", "Succeeded"))
    assert got["spec"]["nodeName"] == target
    await f.client.create("pods", _pod("nowhere", "true", nodeSelector={"e2e": "no-such-node"}), f.ns)

    async def unsched():
        x = await f.client.get("pods", "nowhere", f.ns)
        c = core.get_condition(x.get("status"), core.COND_POD_SCHEDULED)
        return c if c and c.get("status") == "False" and c.get("reason") == "Unschedulable" else None
    await f.wait(unsched, 30, "PodScheduled=False/Unschedulable")


@conformance("Namespace deletion should remove the namespace's pods")
async def namespace_deletion(f):
    ns = f.ns + "-nsdel"
    await f.client.create("namespaces", {"metadata": {"name": ns}})
    await f.client.create("pods", _pod("victim", "sleep 3600", restart="Always"), ns)
    await f.client.delete("namespaces", ns)

    async def gone():
        try:
            await f.client.get("namespaces", ns)
            return None
        except Exception:  # noqa: BLE001
            return True
    await f.wait(gone, 90, "namespace removal")


@spec("GPU: pods requesting amd.com/gpu get distinct devices and run the HIP vector add", "Feature:GPU")
async def gpu_vector_add(f):
    nodes = (await f.client.list("nodes"))["items"]
    gpus = sum(int((n["status"].get("capacity") or {}).get(core.AMD_GPU, "0")) for n in nodes)
    if gpus < 1:
        raise AssertionError("cluster advertises no amd.com/gpu")
    n = min(2, gpus)        # nvidia-gpus.go runs one pod per GPU; two show distinct assignment
    for i in range(n):
        p = {"metadata": {"name": f"vec-{i}"}, "spec": {"restartPolicy": "Never", "containers": [
            {"name": "c", "image": "kubernetes-amd/hip-vector-add", "resources": {"limits": {core.AMD_GPU: "1"}}}]}}
        await f.client.create("pods", p, f.ns)
    assigned = []
    for i in range(n):
        pod = await f.pod_phase(f"vec-{i}", ("Succeeded",), 180)
        assigned.append(tuple(core.pod_assigned_devices(pod).get(core.AMD_GPU, ())) or
                        tuple(d for per in pod["spec"].get("extendedResources") or () for d in per.get("assigned") or ()))
        assert "Test PASSED" in await f.logs(f"vec-{i}")
    assert all(assigned), assigned
    if n == 2:
        assert set(assigned[0]).isdisjoint(assigned[1]), assigned
