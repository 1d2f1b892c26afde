"""DeviceManager + device plugin protocol (fork F7/F8/F9).

Mirrors the reference's unit tests: `manager_test.go:87-171` (TestManagerPluginHandling: two
stub plugins, capacity add/remove, health-only changes), `:173` (re-registration),
`endpoint_test.go`, `device_store_test.go`, `plugin_watcher_test.go:65,119`.
"""
import asyncio
import threading
import os

import pytest

from kubernetes_amd.deviceplugin import api
from kubernetes_amd.deviceplugin.amdgpu import AMDGPUPlugin
from kubernetes_amd.deviceplugin.server import DevicePluginServer, device
from kubernetes_amd.kubelet.devicemanager.manager import AdmitError, ManagerImpl
from kubernetes_amd.kubelet.devicemanager.stores import DeviceStore, merge_init_responses
from kubernetes_amd.kubelet.devicemanager.watcher import PluginWatcher
from kubernetes_amd.native import amdsmi


async def until(pred, timeout=5.0):
    t = asyncio.get_running_loop().time() + timeout
    while not pred():
        if asyncio.get_running_loop().time() > t:
            raise TimeoutError("condition not met")
        await asyncio.sleep(0.01)


def test_device_store_diff():
    s = DeviceStore()
    a, u, d = s.update([device("a"), device("b")])
    assert [x.ID for x in a] == ["a", "b"] and not u and not d
    a, u, d = s.update([device("a", api.UNHEALTHY), device("c")])
    assert [x.ID for x in a] == ["c"] and [x.ID for x in u] == ["a"] and [x.ID for x in d] == ["b"]
    a, u, d = s.update([device("a", api.UNHEALTHY), device("c")])
    assert not a and not u and not d


def test_watcher_layout_rules(tmp_path, run):
    async def main():
        import socket
        w = PluginWatcher(str(tmp_path))
        w.start()
        os.makedirs(tmp_path / "amd.com")
        s = socket.socket(socket.AF_UNIX)
        s.bind(str(tmp_path / "amd.com" / "p.sock"))
        # a socket in the root is ignored; a directory inside a domain is ignored
        s2 = socket.socket(socket.AF_UNIX)
        s2.bind(str(tmp_path / "root.sock"))
        os.makedirs(tmp_path / "amd.com" / "subdir")
        p = await asyncio.wait_for(w.added.get(), 5)
        assert p == str(tmp_path / "amd.com" / "p.sock")
        os.unlink(tmp_path / "amd.com" / "p.sock")
        r = await asyncio.wait_for(w.removed.get(), 5)
        assert r == p
        assert w.added.empty()
        w.stop()
        s.close()
        s2.close()
    run(main())


def test_manager_plugin_handling(tmp_path, run):
    async def main():
        m = ManagerImpl(str(tmp_path))
        await m.start()
        p1 = DevicePluginServer("vendor.com/foo", str(tmp_path / "vendor.com" / "foo.sock"),
                                [device("d1"), device("d2")])
        p2 = DevicePluginServer("vendor.com/bar", str(tmp_path / "vendor.com" / "bar.sock"), [device("x")])
        await p1.start()
        await p2.start()
        await until(lambda: set(m.get_capacity()[0]) == {"vendor.com/foo", "vendor.com/bar"})
        await p1.registered.wait()
        cap, removed = m.get_capacity()
        assert set(cap["vendor.com/foo"]["resources"]) == {"d1", "d2"} and not removed
        # health-only change propagates
        p1.update([device("d1", api.UNHEALTHY), device("d2")])
        await until(lambda: m.get_capacity()[0]["vendor.com/foo"]["resources"]["d1"]["health"] == api.UNHEALTHY)
        # deleting every device removes the resource and reports it once
        p2.update([])
        await until(lambda: "vendor.com/bar" not in m.get_capacity()[0])
        # plugin death: stream ends -> devices deleted
        await p1.stop()
        await until(lambda: "vendor.com/foo" not in m.get_capacity()[0])
        await p2.stop()
        await m.stop()
    run(main())


def test_registration_rejects_wrong_domain_and_version(tmp_path, run):
    async def main():
        m = ManagerImpl(str(tmp_path))
        await m.start()
        bad = DevicePluginServer("other.com/gpu", str(tmp_path / "amd.com" / "bad.sock"), [device("z")])
        await bad.start()
        await until(lambda: bad.registration_status is not None)
        assert bad.registration_status[0] is False and "domain" in bad.registration_status[1]
        old = DevicePluginServer("amd.com/gpu", str(tmp_path / "amd.com" / "old.sock"), [device("z")],
                                 supported_versions=("v1alpha1",))
        await old.start()
        await until(lambda: old.registration_status is not None)
        assert old.registration_status[0] is False
        assert m.get_capacity()[0] == {}
        await bad.stop()
        await old.stop()
        await m.stop()
    run(main())


def test_reregistration_carries_store(tmp_path, run):
    async def main():
        m = ManagerImpl(str(tmp_path))
        await m.start()
        p1 = DevicePluginServer("amd.com/gpu", str(tmp_path / "amd.com" / "a.sock"), [device("g0"), device("g1")])
        await p1.start()
        await until(lambda: "amd.com/gpu" in m.get_capacity()[0])
        e1 = m.handler.endpoint("amd.com/gpu")
        # the same resource re-registers on a new socket with one device changed
        p2 = DevicePluginServer("amd.com/gpu", str(tmp_path / "amd.com" / "b.sock"), [device("g0"), device("g2")])
        await p2.start()
        await until(lambda: m.handler.endpoint("amd.com/gpu") is not e1)
        await until(lambda: set(m.get_capacity()[0]["amd.com/gpu"]["resources"]) == {"g0", "g2"})
        # stopping the OLD plugin must not delete the new endpoint's devices
        await p1.stop()
        await asyncio.sleep(0.2)
        assert set(m.get_capacity()[0]["amd.com/gpu"]["resources"]) == {"g0", "g2"}
        await p2.stop()
        await m.stop()
    run(main())


def _pod(uid, assigned, name="p"):
    return {"metadata": {"name": name, "namespace": "default", "uid": uid},
            "spec": {"containers": [{"name": "c", "extendedResourceRequests": ["er1"]}],
                     "extendedResources": [{"name": "er1", "resources": {"limits": {"amd.com/gpu": str(len(assigned))},
                                                                         "requests": {"amd.com/gpu": str(len(assigned))}},
                                            "assigned": assigned}]}}


def test_amdgpu_plugin_admit_and_init_container(tmp_path, run):
    async def main():
        smi = amdsmi.SMI(fixture=amdsmi.fixture_file(8))
        plugin = AMDGPUPlugin(str(tmp_path), smi=smi, health_interval=0, dev_root="/dev")
        ids = [g.device_id_str for g in plugin.gpus]
        active = []
        m = ManagerImpl(str(tmp_path))
        await m.start(lambda: active)
        await plugin.start()
        await until(lambda: "amd.com/gpu" in m.get_capacity()[0])
        cap = m.get_capacity()[0]["amd.com/gpu"]["resources"]
        assert len(cap) == 8
        attrs = cap[ids[2]]["attributes"]
        assert attrs["amd.com/arch"] == "gfx950" and attrs["amd.com/product"] == "MI355X"
        assert attrs["amd.com/memory"] == "294912" and attrs["amd.com/hbm"] == "288Gi"
        assert attrs["amd.com/render-minor"] == "130"
        pod = _pod("u1", [ids[1], ids[2]])
        await m.admit_pod(pod)
        active.append(pod)
        assert m.pod_resources(pod)["annotations"]["amd.com/gpu-devices"] == f"{ids[1]},{ids[2]}"
        opts = await m.init_container(pod, pod["spec"]["containers"][0])
        paths = [d["pathOnHost"] for d in opts["devices"]]
        assert paths == ["/dev/kfd", "/dev/dri/renderD129", "/dev/dri/renderD130"]
        envs = {e["name"]: e["value"] for e in opts["envs"]}
        assert envs["AMD_VISIBLE_DEVICES"] == "1,2" and envs["AMD_GPU_ARCH"] == "gfx950"
        # duplicate assignment to a second active pod is rejected by the kubelet
        with pytest.raises(AdmitError):
            await m.admit_pod(_pod("u2", [ids[2]], "q"))
        # unknown / unhealthy devices are rejected
        with pytest.raises(AdmitError):
            await m.admit_pod(_pod("u3", ["GPU-nope"], "r"))
        smi.fake_set_ecc(5, 3)
        assert plugin.poll_health()
        await until(lambda: m.get_capacity()[0]["amd.com/gpu"]["resources"][ids[5]]["health"] == api.UNHEALTHY)
        with pytest.raises(AdmitError):
            await m.admit_pod(_pod("u4", [ids[5]], "s"))
        smi.fake_set_ecc(5, 0)
        await plugin.stop()
        await m.stop()
    run(main())


def test_burn_in_gates_devices_and_publishes_measurements(tmp_path, run):
    """With a burn-in configured, GPUs are offered Unhealthy (`amd.com/burn-in=pending`) until
    their acceptance test passes; a GPU that fails stays Unhealthy; measured TFLOP/s and GB/s
    become attributes the scheduler's selectors can use."""
    from kubernetes_amd.deviceplugin.amdgpu import ATTR_BURN_IN, ATTR_HBM_GBPS, ATTR_MFMA_TFLOPS
    from kubernetes_amd.deviceplugin.burnin import BurnIn, BurnInResult
    from kubernetes_amd.scheduler.cache import ERManager
    from kubernetes_amd.scheduler.topology import Request, allocate

    class FakeBurnIn(BurnIn):
        def __init__(self):
            super().__init__(min_tflops=700, min_hbm_gbps=3000)
            self.release = threading.Event()

        def run(self, i):
            self.release.wait(5)
            r = BurnInResult(ok=False, tflops=1400.0 - 100 * i, hbm_gbps=6000.0, mfma_rel_err=1e-4,
                             fp8_tflops=2800.0, fp8_rel_err=1e-5)
            if i == 3:
                r.tflops = 350.0                       # throttled part
            r.reason = self.judge(r)
            r.ok = not r.reason
            return r

    async def main():
        smi = amdsmi.SMI(fixture=amdsmi.fixture_file(4, seed="burn"))
        bi = FakeBurnIn()
        plugin = AMDGPUPlugin(str(tmp_path), smi=smi, health_interval=0, burn_in=bi)
        ids = [g.device_id_str for g in plugin.gpus]
        m = ManagerImpl(str(tmp_path))
        await m.start(lambda: [])
        await plugin.start()
        await until(lambda: "amd.com/gpu" in m.get_capacity()[0])
        cap = m.get_capacity()[0]["amd.com/gpu"]["resources"]
        assert all(d["health"] == api.UNHEALTHY and d["attributes"][ATTR_BURN_IN] == "pending" for d in cap.values())
        with pytest.raises(AdmitError):
            await m.admit_pod(_pod("u0", [ids[0]]))
        bi.release.set()
        await until(lambda: all(d["attributes"][ATTR_BURN_IN] != "pending"
                                for d in m.get_capacity()[0]["amd.com/gpu"]["resources"].values()))
        cap = m.get_capacity()[0]["amd.com/gpu"]["resources"]
        assert [cap[i]["health"] for i in ids] == [api.HEALTHY] * 3 + [api.UNHEALTHY]
        assert cap[ids[3]]["attributes"][ATTR_BURN_IN] == "failed" and "350" in plugin._burn[ids[3]].reason
        assert cap[ids[1]]["attributes"][ATTR_MFMA_TFLOPS] == "1300" and cap[ids[1]]["attributes"][ATTR_HBM_GBPS] == "6000"
        assert cap[ids[1]]["attributes"]["amd.com/mfma-fp8-tflops"] == "2800"
        await m.admit_pod(_pod("u1", [ids[0]]))
        # a pod can ask for the fastest parts only
        er = ERManager()
        er.set_node({"metadata": {"name": "n"}, "status": {"extendedResources": m.get_capacity()[0]}})
        b, _, _ = allocate([Request("er", "amd.com/gpu", 2, [{"key": ATTR_MFMA_TFLOPS, "operator": "Gt",
                                                               "values": ["1250"]}])], er)
        assert sorted(b["er"]["resources"]) == sorted(ids[:2])
        await plugin.stop()
        await m.stop()
    run(main())


def test_admit_waits_for_plugin_after_restart(tmp_path, run):
    async def main():
        m = ManagerImpl(str(tmp_path), registration_grace=5.0)
        await m.start()
        plugin = DevicePluginServer("amd.com/gpu", str(tmp_path / "amd.com" / "g.sock"), [device("g0")])

        async def late():
            await asyncio.sleep(0.3)
            await plugin.start()
        t = asyncio.ensure_future(late())
        await m.admit_pod(_pod("u1", ["g0"]))  # would fail immediately in the reference
        await t
        await plugin.stop()
        await m.stop()
    run(main())


def test_merge_init_responses_first_wins():
    R = api.DP["InitContainerResponse"]
    r1 = R(spec=api.DP["ContainerSpec"](envs={"A": "1"}, devices=[api.DP["DeviceSpec"](container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")]))
    r2 = R(spec=api.DP["ContainerSpec"](envs={"A": "2", "B": "3"}, devices=[api.DP["DeviceSpec"](container_path="/dev/kfd", host_path="/dev/other")]))
    o = merge_init_responses([r1, r2])
    assert o["envs"] == [{"name": "A", "value": "1"}, {"name": "B", "value": "3"}]
    assert [d["pathOnHost"] for d in o["devices"]] == ["/dev/kfd"]


def test_node_status_drops_removed_devices_and_resources(tmp_path, run):
    """Unregistering a plugin (or dropping one of its devices) must reach the API server: the
    node-status patch only adds map keys otherwise, and the scheduler cache would keep
    allocating the stale Healthy IDs. Reference: `kubelet_node_status.go:608-623`
    zeroes removed resources."""
    from kubernetes_amd.cluster import LocalCluster

    async def main():
        import tempfile
        cl = LocalCluster(nodes=1, gpus_per_node=0, emit_events=False,
                          workdir=tempfile.mkdtemp(prefix="kdm", dir="/tmp"))   # unix socket path < 108 chars
        await cl.start()
        n = cl.nodes[0]
        p = DevicePluginServer("amd.com/gpu", os.path.join(n.plugins_dir, "amd.com", "stub.sock"),
                               [device("g0"), device("g1"), device("g2")])
        try:
            await p.start()

            async def server_devs():
                node = await cl.client.get("nodes", n.name)
                dom = (node["status"].get("extendedResources") or {}).get("amd.com/gpu")
                return node, (set(dom["resources"]) if dom else None)
            await cl.wait_for(lambda: _eq(server_devs, {"g0", "g1", "g2"}))
            p.update([device("g0"), device("g2")])
            node = await cl.wait_for(lambda: _eq(server_devs, {"g0", "g2"}))
            assert node["status"]["capacity"]["amd.com/gpu"] == "2"
            ni = cl.scheduler.cache.nodes[n.name]
            await cl.wait_for(lambda: _const(set(ni.er.allocatable.get("amd.com/gpu", {})) == {"g0", "g2"}))
            await p.stop()
            node = await cl.wait_for(lambda: _eq(server_devs, None))
            assert node["status"]["capacity"]["amd.com/gpu"] == "0"
            assert node["status"]["allocatable"]["amd.com/gpu"] == "0"
            await cl.wait_for(lambda: _const("amd.com/gpu" not in cl.scheduler.cache.nodes[n.name].er.allocatable))
        finally:
            try:
                await p.stop()
            finally:
                await cl.stop()
    run(main())


async def _eq(fn, want):
    node, got = await fn()
    return node if got == want else None


async def _const(v):
    return v


def test_reregistration_interleaving_shim(tmp_path, run):
    """`endpoint_handler_test.go:153` TestReRegistration with the instrumented store shim
    (`endpoint_store_shim.go`): the swap is paused, the shim checks that the new endpoint shares
    the old endpoint's device store, and — the harder interleaving — the OLD plugin dies while
    the swap is paused. Re-registration must never report the carried-over devices deleted, and
    the superseded endpoint must still be stopped."""
    from kubernetes_amd.kubelet.devicemanager.endpoint import EndpointHandler

    async def main():
        calls = []
        h = EndpointHandler(lambda n, a, u, d: calls.append((n, [x.ID for x in a], [x.ID for x in u], [x.ID for x in d])))
        dom = tmp_path / "amd.com"
        p1 = DevicePluginServer("amd.com/gpu", str(dom / "p1.sock"), [device("Dev1"), device("Dev2")])
        p2 = DevicePluginServer("amd.com/gpu", str(dom / "p2.sock"), [device("Dev1"), device("Dev2")])
        await p1.start()
        e1 = await h.new_endpoint(p1.socket_path, "amd.com")
        await until(lambda: len(calls) == 1)
        assert calls[0] == ("amd.com/gpu", ["Dev1", "Dev2"], [], [])
        await p2.start()
        seen = {}

        async def shim(new):
            old = h.endpoint("amd.com/gpu")
            seen["old"], seen["new"] = old, new
            assert old is e1 and new.store is old.store and len(old.store.devices_list()) == 2
            await p1.stop()                       # the old plugin dies inside the swap window
            await asyncio.sleep(0.3)
        h.swap_hook = shim
        e2 = await h.new_endpoint(p2.socket_path, "amd.com")
        await asyncio.sleep(0.2)
        assert seen["new"] is e2
        assert not any(c[3] for c in calls), calls                  # nothing reported deleted
        assert h.endpoint("amd.com/gpu") is e2
        assert sorted(d.ID for d in h.devices()["amd.com/gpu"]) == ["Dev1", "Dev2"]
        assert e1._stopped                                           # superseded endpoint stopped
        await e2.stop()                                              # stop time: devices deleted once
        await until(lambda: any(c[3] for c in calls))
        assert [c[3] for c in calls if c[3]] == [["Dev1", "Dev2"]]
        await h.stop()
        await p2.stop()
    run(main())
