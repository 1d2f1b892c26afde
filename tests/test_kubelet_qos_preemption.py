"""Kubelet QoS / OOM scores, pod & QoS cgroups, critical-pod preemption, sysctl admission and
service environment variables.

Parity: `pkg/kubelet/qos/policy_test.go` (OOM score bands), `pkg/kubelet/cm/helpers_linux_test.go`
(ResourceConfigForPod), `pkg/kubelet/preemption/preemption_test.go` (victim selection by QoS and
distance), `pkg/kubelet/sysctl/whitelist_test.go`, `pkg/kubelet/envvars/envvars_test.go`.
"""
import os

import pytest

from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.kubelet import cgroups as cg
from kubernetes_amd.kubelet import envvars, preemption, qos, sysctl


def pod(name, cpu_req=None, mem_req=None, cpu_lim=None, mem_lim=None, ns="default", ann=None, uid=None, prio=None):
    res = {}
    if cpu_req or mem_req:
        res["requests"] = {k: v for k, v in (("cpu", cpu_req), ("memory", mem_req)) if v}
    if cpu_lim or mem_lim:
        res["limits"] = {k: v for k, v in (("cpu", cpu_lim), ("memory", mem_lim)) if v}
    p = {"metadata": {"name": name, "namespace": ns, "uid": uid or f"uid-{name}", "annotations": dict(ann or {})},
         "spec": {"containers": [{"name": "c", "image": "busybox", "resources": res}]}}
    if prio is not None:
        p["spec"]["priority"] = prio
    return p


GI = 1 << 30


def test_qos_classes_and_oom_score_bands():
    be, bu = pod("be"), pod("bu", cpu_req="100m", mem_req="1Gi")
    gu = pod("gu", cpu_req="1", mem_req="2Gi", cpu_lim="1", mem_lim="2Gi")
    assert (qos.pod_qos(be), qos.pod_qos(bu), qos.pod_qos(gu)) == ("BestEffort", "Burstable", "Guaranteed")
    c = lambda p: p["spec"]["containers"][0]  # noqa: E731
    assert qos.oom_score_adj(be, c(be), 16 * GI) == 1000
    assert qos.oom_score_adj(gu, c(gu), 16 * GI) == -998
    assert qos.oom_score_adj(bu, c(bu), 16 * GI) == 1000 - 1000 // 16        # 938
    huge = pod("huge", cpu_req="1", mem_req="64Gi")
    assert qos.oom_score_adj(huge, c(huge), 16 * GI) == 2                     # never below Burstable's floor
    tiny = pod("tiny", cpu_req="1m", mem_req="1")
    assert qos.oom_score_adj(tiny, c(tiny), 16 * GI) == 999                   # never as high as BestEffort
    crit = pod("dp", ns="kube-system", ann={qos.CRITICAL_POD_ANNOTATION: ""})
    assert qos.is_critical_pod(crit) and qos.oom_score_adj(crit, c(crit), 16 * GI) == 1000   # by class only
    assert not qos.is_critical_pod(pod("x", ann={qos.CRITICAL_POD_ANNOTATION: ""}))   # only in kube-system
    assert qos.is_critical_pod(pod("p", prio=2000001000))


def test_resource_config_for_pod_and_cgroup_tree(tmp_path):
    assert cg.milli_cpu_to_shares(0) == 2 and cg.milli_cpu_to_shares(1000) == 1024 and cg.milli_cpu_to_shares(1) == 2
    assert cg.milli_cpu_to_quota(500) == 50_000 and cg.milli_cpu_to_quota(5) == 1000
    assert cg.shares_to_weight(2) == 1 and cg.shares_to_weight(262144) == 10000 and cg.shares_to_weight(1024) == 39
    gu = pod("gu", cpu_req="1500m", mem_req="2Gi", cpu_lim="1500m", mem_lim="2Gi")
    assert cg.resource_config_for_pod(gu) == {"cpu_shares": 1536, "cpu_quota": 150_000, "memory_limit": 2 * GI}
    bu = pod("bu", cpu_req="250m", mem_req="1Gi", mem_lim="4Gi")     # no cpu limit: no quota
    assert cg.resource_config_for_pod(bu) == {"cpu_shares": 256, "cpu_quota": None, "memory_limit": 4 * GI}
    assert cg.resource_config_for_pod(pod("be")) == {"cpu_shares": 2, "cpu_quota": None, "memory_limit": None}

    m = cg.CgroupManager(str(tmp_path), {"cpu": 15_000, "memory": 60 * GI}).start()
    assert m.read(m.kubepods, "memory.max") == str(60 * GI)
    assert m.read(m.kubepods, "cpu.weight") == str(cg.shares_to_weight(15_360))
    d_gu, d_bu = m.ensure_pod(gu), m.ensure_pod(bu)
    assert d_gu == os.path.join(str(tmp_path), "kubepods", "poduid-gu")
    assert d_bu == os.path.join(str(tmp_path), "kubepods", "burstable", "poduid-bu")
    assert m.read(d_gu, "cpu.max") == "150000 100000" and m.read(d_gu, "memory.max") == str(2 * GI)
    assert m.read(d_bu, "cpu.max") == "max 100000"
    assert m.read(m.qos_dir("Burstable"), "cpu.weight") == str(cg.shares_to_weight(256))
    bu2 = pod("bu2", cpu_req="750m")
    m.ensure_pod(bu2)
    assert m.read(m.qos_dir("Burstable"), "cpu.weight") == str(cg.shares_to_weight(1024))
    m.destroy_pod("uid-bu")
    assert not os.path.exists(d_bu)
    assert m.read(m.qos_dir("Burstable"), "cpu.weight") == str(cg.shares_to_weight(768))


def test_preemption_victim_selection():
    # reference preemption_test.go shapes: prefer BestEffort, then Burstable, then Guaranteed;
    # within a class the pod closest to the shortfall
    be1, be2 = pod("be1"), pod("be2")
    bu_small, bu_big = pod("bus", cpu_req="100m", mem_req="100Mi"), pod("bub", cpu_req="1", mem_req="1Gi")
    gu = pod("gu", cpu_req="2", mem_req="2Gi", cpu_lim="2", mem_lim="2Gi")
    crit = pod("crit", ns="kube-system", ann={qos.CRITICAL_POD_ANNOTATION: ""}, cpu_req="4")
    names = lambda ps: sorted(p["metadata"]["name"] for p in ps)  # noqa: E731
    # one pod slot short: a BestEffort pod goes, never the critical one
    assert len(preemption.pods_to_preempt([be1, bu_big, gu, crit], {"pods": 1})) == 1
    assert names(preemption.pods_to_preempt([be1, bu_big, gu, crit], {"pods": 1})) == ["be1"]
    # 900m cpu short: the 1-cpu Burstable pod covers it alone (BestEffort requests nothing)
    assert names(preemption.pods_to_preempt([be1, be2, bu_small, bu_big, gu], {"cpu": 900})) == ["bub"]
    # 2.5 cpu short: the Guaranteed pod only once both Burstable pods are not enough
    got = names(preemption.pods_to_preempt([be1, bu_small, bu_big, gu], {"cpu": 2500}))
    assert "gu" in got and "bub" in got and "be1" not in got
    with pytest.raises(ValueError):
        preemption.pods_to_preempt([be1, crit], {"cpu": 1000})


def test_sysctl_whitelist():
    h = sysctl.SysctlAdmitHandler(allowed_unsafe=["net.core.somaxconn", "kernel.msg*"])
    ok = pod("ok", ann={sysctl.SAFE_ANNOTATION: "kernel.shm_rmid_forced=1,net.ipv4.tcp_syncookies=1",
                        sysctl.UNSAFE_ANNOTATION: "net.core.somaxconn=1024,kernel.msgmax=65536"})
    assert h.admit(ok) is None
    assert h.pod_sysctls(ok)["net.core.somaxconn"] == "1024"
    bad = pod("bad", ann={sysctl.SAFE_ANNOTATION: "net.core.somaxconn=1024"})     # unsafe under the safe key
    assert h.admit(bad)[0] == "SysctlForbidden"
    assert h.admit(pod("nn", ann={sysctl.UNSAFE_ANNOTATION: "vm.swappiness=1"}))[0] == "SysctlForbidden"
    hostnet = pod("hn", ann={sysctl.SAFE_ANNOTATION: "net.ipv4.tcp_syncookies=1"})
    hostnet["spec"]["hostNetwork"] = True
    assert "host net" in h.admit(hostnet)[1]
    assert h.admit(pod("fmt", ann={sysctl.SAFE_ANNOTATION: "kernel.shm_rmid_forced"}))[0] == "SysctlForbidden"
    with pytest.raises(ValueError):
        sysctl.SysctlAdmitHandler(allowed_unsafe=["vm.*"])          # not namespaced


def test_service_env_vars():
    svcs = [{"metadata": {"name": "kubernetes", "namespace": "default"},
             "spec": {"clusterIP": "10.0.0.1", "ports": [{"name": "https", "port": 443, "protocol": "TCP"}]}},
            {"metadata": {"name": "gpu-metrics", "namespace": "ml"},
             "spec": {"clusterIP": "10.0.0.9", "ports": [{"name": "http-prom", "port": 9400}, {"port": 53, "protocol": "UDP"}]}},
            {"metadata": {"name": "headless", "namespace": "ml"}, "spec": {"clusterIP": "None", "ports": [{"port": 1}]}},
            {"metadata": {"name": "other", "namespace": "other"}, "spec": {"clusterIP": "10.0.0.7", "ports": [{"port": 1}]}}]
    env = {e["name"]: e["value"] for e in envvars.service_env(svcs, "ml")}
    assert env["KUBERNETES_SERVICE_HOST"] == "10.0.0.1" and env["KUBERNETES_SERVICE_PORT"] == "443"
    assert env["KUBERNETES_SERVICE_PORT_HTTPS"] == "443" and env["KUBERNETES_PORT"] == "tcp://10.0.0.1:443"
    assert env["GPU_METRICS_SERVICE_HOST"] == "10.0.0.9" and env["GPU_METRICS_SERVICE_PORT_HTTP_PROM"] == "9400"
    assert env["GPU_METRICS_PORT_53_UDP"] == "udp://10.0.0.9:53" and env["GPU_METRICS_PORT_53_UDP_ADDR"] == "10.0.0.9"
    assert env["GPU_METRICS_PORT_9400_TCP_PROTO"] == "tcp"
    assert not any(k.startswith(("HEADLESS_", "OTHER_")) for k in env)


def test_kubelet_cgroups_env_sysctl_and_critical_preemption(run, tmp_path):
    """End to end on a process-runtime node: service env vars and the pod cgroup reach the
    container process, an unsafe sysctl is rejected, and a critical pod that does not fit
    preempts a Burstable pod (which ends Failed/Preempting)."""
    cgroot = tmp_path / "cgroup"

    async def main():
        cl = LocalCluster(nodes=1, gpus_per_node=0, runtime="process", workdir=str(tmp_path / "c"),
                          kubelet_kwargs={"cpu": "2", "memory": "8Gi", "cgroup_root": str(cgroot)})
        await cl.start()
        c = cl.client
        node = cl.nodes[0].name
        try:
            await c.create("services", {"metadata": {"name": "hip-svc"}, "spec": {"ports": [{"port": 8080}]}}, "default")
            svc = await c.get("services", "hip-svc", "default")

            async def svc_seen():
                return any(s["metadata"]["name"] == "hip-svc" for s in cl.nodes[0].kubelet.svc_informer.list())
            await cl.wait_for(svc_seen, 10)
            await c.create("pods", {"metadata": {"name": "envpod"}, "spec": {"nodeName": node, "containers": [{
                "name": "c", "image": "busybox", "resources": {"requests": {"cpu": "1500m", "memory": "1Gi"}},
                "env": [{"name": "FROM_SVC", "value": "$(HIP_SVC_SERVICE_HOST):$(HIP_SVC_SERVICE_PORT)"}],
                "command": ["sh", "-c", "env; cat /proc/self/oom_score_adj; sleep 60"]}]}}, "default")

            async def running(name, ns="default"):
                p = await c.get("pods", name, ns)
                return p if (p.get("status") or {}).get("phase") == "Running" else None
            p = await cl.wait_for(lambda: running("envpod"), 20)
            kl = cl.nodes[0].kubelet
            st = kl.pods[p["metadata"]["uid"]]
            cid = st.containers["c"]

            async def logged():
                out = (await kl.runtime.container_logs(cid)).decode()
                return out if "FROM_SVC=" in out else None
            out = await cl.wait_for(logged, 10)
            ip = svc["spec"]["clusterIP"]
            assert f"HIP_SVC_SERVICE_HOST={ip}" in out and f"FROM_SVC={ip}:8080" in out
            assert "KUBERNETES_SERVICE_HOST=" in out
            pdir = kl.cgroups.pod_dir(p)
            assert pdir.endswith(os.path.join("kubepods", "burstable", "pod" + p["metadata"]["uid"]))
            # the container runs in its own leaf under the pod cgroup; the pod cgroup itself holds
            # no process (cgroup v2 no-internal-process rule once it delegates cpu/memory)
            leaves = [x for x in os.listdir(pdir) if x.startswith("ctr-")]
            assert leaves and os.path.exists(os.path.join(pdir, leaves[0], "cgroup.procs"))
            assert not (kl.cgroups.read(pdir, "cgroup.procs") or "").strip()
            assert kl.cgroups.read(pdir, "cpu.weight") == str(cg.shares_to_weight(1536))

            # unsafe sysctl without --experimental-allowed-unsafe-sysctls: rejected at admission
            await c.create("pods", {"metadata": {"name": "sysctl", "annotations": {
                sysctl.UNSAFE_ANNOTATION: "net.core.somaxconn=4096"}},
                "spec": {"nodeName": node, "containers": [{"name": "c", "image": "busybox", "command": ["sleep", "5"]}]}},
                "default")

            async def rejected():
                q = await c.get("pods", "sysctl", "default")
                return q if (q.get("status") or {}).get("reason") == "SysctlForbidden" else None
            q = await cl.wait_for(rejected, 20)
            assert q["status"]["phase"] == "Failed"

            # a critical kube-system pod needing 1 cpu on a 2-cpu node that has 1.5 cpu in use
            await c.create("pods", {"metadata": {"name": "critical", "namespace": "kube-system",
                                                 "annotations": {qos.CRITICAL_POD_ANNOTATION: ""}},
                                    "spec": {"nodeName": node, "containers": [{
                                        "name": "c", "image": "busybox", "command": ["sleep", "60"],
                                        "resources": {"requests": {"cpu": "1"}}}]}}, "kube-system")
            await cl.wait_for(lambda: running("critical", "kube-system"), 20)

            async def preempted():
                v = await c.get("pods", "envpod", "default")
                return v if (v.get("status") or {}).get("reason") == "Preempting" else None
            v = await cl.wait_for(preempted, 20)
            assert v["status"]["phase"] == "Failed"
            evs = (await c.list("events", "default"))["items"]
            assert any(e.get("reason") == "Preempting" and e["involvedObject"]["name"] == "envpod" for e in evs)
        finally:
            await cl.stop()
    run(main(), timeout=120)
