"""Cluster DNS add-on (A / SRV / PTR / CNAME / pod records, NXDOMAIN, upstream forwarding,
UDP + TCP) and the add-on manager (Reconcile / EnsureExists / prune)."""
import asyncio

import yaml

from kubernetes_amd.addons import dns as D
from kubernetes_amd.addons.manager import MODE, AddonManager
from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client.rest import APIStatusError, Client


def test_cluster_dns(run):
    async def main():
        s = APIServer()
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        await c.create("namespaces", {"metadata": {"name": "ml"}})
        web = await c.create("services", {"metadata": {"name": "web"}, "spec": {
            "selector": {"app": "web"}, "ports": [{"name": "http", "port": 80, "protocol": "TCP"}]}}, "ml")
        await c.create("services", {"metadata": {"name": "workers"}, "spec": {
            "clusterIP": "None", "selector": {"app": "w"}, "ports": [{"name": "nccl", "port": 29500}]}}, "ml")
        await c.create("endpoints", {"metadata": {"name": "workers"}, "subsets": [{
            "addresses": [{"ip": "10.244.1.7", "hostname": "trainer-0"}, {"ip": "10.244.1.8", "hostname": "trainer-1"}],
            "ports": [{"name": "nccl", "port": 29500}]}]}, "ml")
        await c.create("services", {"metadata": {"name": "ext"}, "spec": {"type": "ExternalName",
                                                                         "externalName": "models.example.com"}}, "ml")
        # an "upstream" resolver answering everything outside the cluster domain
        up = D.DNSServer(None, "upstream.test", records=D.Records("example.com"))
        up.records.services["x/y"] = {"metadata": {"namespace": "x", "name": "y"}, "spec": {"clusterIP": "1.2.3.4"}}
        up_port = await up.start()
        srv = D.DNSServer(c, "cluster.local", [f"127.0.0.1:{up_port}"])
        dport = await srv.start()
        try:
            ip = web["spec"]["clusterIP"]
            rc, ans = await D.resolve("127.0.0.1", dport, "web.ml.svc.cluster.local")
            assert rc == D.NOERROR and ans[0][1:] == (D.A, ip)
            rc, ans = await D.resolve("127.0.0.1", dport, "web.ml.svc.cluster.local", tcp=True)
            assert ans[0][2] == ip
            rc, ans = await D.resolve("127.0.0.1", dport, "workers.ml.svc.cluster.local")
            assert sorted(a[2] for a in ans if a[1] == D.A) == ["10.244.1.7", "10.244.1.8"]
            rc, ans = await D.resolve("127.0.0.1", dport, "trainer-1.workers.ml.svc.cluster.local")
            assert [a[2] for a in ans] == ["10.244.1.8"]
            rc, ans = await D.resolve("127.0.0.1", dport, "_nccl._tcp.workers.ml.svc.cluster.local", D.SRV)
            srvs = sorted(a[2] for a in ans if a[1] == D.SRV)
            assert srvs == [(10, 100, 29500, "trainer-0.workers.ml.svc.cluster.local"),
                            (10, 100, 29500, "trainer-1.workers.ml.svc.cluster.local")]
            assert {a[2] for a in ans if a[1] == D.A} == {"10.244.1.7", "10.244.1.8"}
            rc, ans = await D.resolve("127.0.0.1", dport, "_http._tcp.web.ml.svc.cluster.local", D.SRV)
            assert ans[0][2] == (10, 100, 80, "web.ml.svc.cluster.local")
            rc, ans = await D.resolve("127.0.0.1", dport, "ext.ml.svc.cluster.local")
            assert ans[0][1:] == (D.CNAME, "models.example.com")
            rc, ans = await D.resolve("127.0.0.1", dport, "10-244-3-9.ml.pod.cluster.local")
            assert ans[0][2] == "10.244.3.9"
            rev = ".".join(reversed(ip.split("."))) + ".in-addr.arpa"
            rc, ans = await D.resolve("127.0.0.1", dport, rev, D.PTR)
            assert ans[0][2] == "web.ml.svc.cluster.local"
            rc, ans = await D.resolve("127.0.0.1", dport, "nope.ml.svc.cluster.local")
            assert rc == D.NXDOMAIN and any(a[1] == D.SOA for a in ans)
            rc, ans = await D.resolve("127.0.0.1", dport, "y.x.svc.example.com")       # forwarded upstream
            assert rc == D.NOERROR and ans[0][2] == "1.2.3.4"
            # a new service shows up through the informer
            new = await c.create("services", {"metadata": {"name": "late"}, "spec": {"ports": [{"port": 1}]}}, "ml")
            for _ in range(100):
                rc, ans = await D.resolve("127.0.0.1", dport, "late.ml.svc.cluster.local")
                if ans:
                    break
                await asyncio.sleep(0.02)
            assert ans[0][2] == new["spec"]["clusterIP"]
        finally:
            await srv.stop()
            await up.stop()
            await c.close()
            await s.stop()
    run(main())


def test_addon_manager(run, tmp_path):
    d = tmp_path / "addons"
    d.mkdir()
    rec = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "rec", "labels": {MODE: "Reconcile"}},
           "data": {"v": "1"}}
    ens = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "ens", "labels": {MODE: "EnsureExists"}},
           "data": {"v": "1"}}
    ign = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "ign"}, "data": {"v": "1"}}
    (d / "a.yaml").write_text(yaml.safe_dump_all([rec, ens, ign]))

    async def main():
        s = APIServer()
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        mgr = AddonManager(c, str(d))
        try:
            await mgr.reconcile_once()
            assert (await c.get("configmaps", "rec", "kube-system"))["data"] == {"v": "1"}
            assert (await c.get("configmaps", "ens", "kube-system"))["data"] == {"v": "1"}
            try:
                await c.get("configmaps", "ign", "kube-system")
                raise AssertionError("unlabelled add-ons are ignored")
            except APIStatusError as e:
                assert e.code == 404
            await c.patch("configmaps", "rec", {"data": {"v": "hand-edited"}}, "kube-system")
            await c.patch("configmaps", "ens", {"data": {"v": "hand-edited"}}, "kube-system")
            await mgr.reconcile_once()
            assert (await c.get("configmaps", "rec", "kube-system"))["data"] == {"v": "1"}       # reconciled back
            assert (await c.get("configmaps", "ens", "kube-system"))["data"] == {"v": "hand-edited"}
            (d / "a.yaml").write_text(yaml.safe_dump_all([ens]))
            await mgr.reconcile_once()
            try:
                await c.get("configmaps", "rec", "kube-system")
                raise AssertionError("removed Reconcile add-on must be pruned")
            except APIStatusError as e:
                assert e.code == 404
        finally:
            await c.close()
            await s.stop()
    run(main())


def test_hyperkube_dispatch(capsys):
    from kubernetes_amd.cmd import hyperkube
    assert hyperkube.main(["hyperkube"]) == 2
    assert "kubelet" in capsys.readouterr().err
    assert hyperkube.main(["hyperkube", "kubeadm", "version"]) == 0
    assert "kubeadm version" in capsys.readouterr().out
    assert hyperkube.main(["/usr/local/bin/kubeadm", "token", "generate"]) == 0     # symlink-style invocation
    tok = capsys.readouterr().out.strip()
    assert len(tok) == 23 and tok[6] == "."


def test_default_addons_reconcile(run):
    from kubernetes_amd.addons.manager import default_addons
    import tempfile, os

    async def main():
        s = APIServer()
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        with tempfile.TemporaryDirectory() as d:
            with open(os.path.join(d, "addons.yaml"), "w") as f:
                yaml.safe_dump_all(default_addons("10.0.0.10"), f)
            try:
                await AddonManager(c, d).reconcile_once()
                svc = await c.get("services", "kube-dns", "kube-system")
                assert svc["spec"]["clusterIP"] == "10.0.0.10"
                assert (await c.get("daemonsets", "amd-gpu-device-plugin", "kube-system"))["spec"]["template"]
            finally:
                await c.close()
                await s.stop()
    run(main())


def test_gendocs_all_components(tmp_path):
    from kubernetes_amd.cmd import gendocs
    files = gendocs.generate(str(tmp_path / "md"), "md")
    assert len(files) == len(gendocs.COMPONENTS)
    kubectl = (tmp_path / "md" / "kubectl.md").read_text()
    assert "## kubectl rolling-update" in kubectl and "## kubectl set image" in kubectl
    assert "--feature-gates" in (tmp_path / "md" / "kubelet.md").read_text()
    man = gendocs.generate(str(tmp_path / "man"), "man", ["kubeadm"])
    assert any(p.endswith("kubeadm-join.1") for p in man)
    assert gendocs.generate(str(tmp_path / "y"), "yaml", ["kube-scheduler"])


def test_dashboard_shows_gpu_allocation(run):
    """cluster/addons/dashboard equivalent: per-device allocation, health and pods, as HTML and JSON."""
    import json as _json

    from kubernetes_amd.addons.dashboard import Dashboard
    from kubernetes_amd.cluster import LocalCluster
    from kubernetes_amd.utils.httpserver import HTTPServer  # noqa: F401

    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=4) as cl:
            await cl.client.create("pods", {"metadata": {"name": "g"}, "spec": {"containers": [
                {"name": "c", "image": "x", "resources": {"limits": {"amd.com/gpu": "2"}}}]}})
            pod = await cl.wait_pod("g")
            d = Dashboard(cl.url)
            port = await d.start("127.0.0.1", 0)
            try:
                import asyncio
                r, w = await asyncio.open_connection("127.0.0.1", port)
                w.write(b"GET /api/summary HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
                raw = await r.read()
                w.close()
                body = raw.split(b"\r\n\r\n", 1)[1]
                if b"\r\n" in body[:10]:          # chunked
                    body = body.split(b"\r\n", 1)[1].rsplit(b"\r\n0\r\n", 1)[0]
                s = _json.loads(body)
                assert s["gpus"] == {"total": 4, "allocated": 2, "healthy": 4}, s["gpus"]
                devs = {x["id"]: x["pod"] for x in s["nodes"][0]["devices"]}
                assigned = pod["spec"]["extendedResources"][0]["assigned"]
                assert all(devs[i] == "default/g" for i in assigned)
                r, w = await asyncio.open_connection("127.0.0.1", port)
                w.write(b"GET / HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
                page = (await r.read()).decode()
                w.close()
                assert "GPUs: 2 / 4 allocated" in page and assigned[0] in page
            finally:
                await d.stop()
    run(main(), timeout=60)
