"""Component flags take effect or are refused — none is silently accepted.

Each reference flag is either implemented (a test below shows the effect), a deprecated no-op in
the reference itself (`deprecated_noop`, citing the reference's MarkDeprecated line), or refused
when set to anything but its default (`unsupported`, with the reason in the error).
"""
import asyncio
import glob
import json
import os
import threading
import time
from http.server import BaseHTTPRequestHandler, HTTPServer

import pytest

from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client.informer import Informer
from kubernetes_amd.client.rest import PROTOBUF, Client

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_no_flag_is_accepted_and_ignored():
    for f in glob.glob(os.path.join(ROOT, "kubernetes_amd", "cmd", "*.py")):
        src = open(f).read()
        assert 'help="accepted' not in src, f
        assert "no-ops kept for command-line compatibility" not in src, f


@pytest.mark.parametrize("module,argv,needle", [
    ("apiserver", ["--watch-cache", "false"], "--watch-cache"),
    ("apiserver", ["--etcd-quorum-read", "false"], "linearizable"),
    ("apiserver", ["--tls-sni-cert-key", "a.crt,a.key"], "SNI"),
    ("apiserver", ["--watch-cache-sizes", "pods#0"], "positive"),
    ("controller_manager", ["--flex-volume-plugin-dir", "/x"], "kubelet"),
    ("controller_manager", ["--pv-recycler-minimum-timeout-nfs", "1"], "recycled"),
    ("kubelet", ["--cadvisor-port", "4194"], "cAdvisor"),
    ("kubelet", ["--enforce-node-allocatable", "pods,system-reserved"], "system-reserved"),
    ("kubelet", ["--seccomp-profile-root", "/x"], "seccomp"),
    ("proxy", ["--udp-timeout", "1s"], "UDP"),
])
def test_unsupported_values_are_refused(module, argv, needle, capsys):
    import importlib
    mod = importlib.import_module(f"kubernetes_amd.cmd.{module}")
    with pytest.raises(SystemExit) as e:
        mod.main(argv + ["--master", "http://127.0.0.1:1"] if module != "apiserver" else argv)
    assert e.value.code == 2
    assert needle in capsys.readouterr().err


def test_unsupported_flags_accept_their_default():
    from kubernetes_amd.cmd.apiserver import _parser
    from kubernetes_amd.cmd._common import check_unsupported
    ap = _parser()
    a = ap.parse_args(["--watch-cache", "true", "--etcd-quorum-read", "true", "--master-service-namespace", "default",
                       "--kubelet-read-only-port", "10255", "--ssh-user", "me"])
    check_unsupported(ap, a)      # no error


def test_watch_cache_sizes_and_target_ram():
    from kubernetes_amd.cmd.apiserver import watch_cache_sizes
    assert watch_cache_sizes(0, "") == {}
    s = watch_cache_sizes(60 * 1000, "pods#123,apiservices.apiregistration.k8s.io#77")
    assert s["pods"] == 123 and s["apiservices"] == 77 and s["nodes"] == 5000 and s["endpoints"] == 10000
    srv = APIServer(watch_cache_sizes={"pods": 7})
    assert srv.caches["pods"].events.maxlen == 7 and srv.caches["nodes"].events.maxlen == srv.watch_window


def test_client_protobuf_content_type(run):
    async def main():
        s = APIServer()
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}", content_type=PROTOBUF)
        seen = []
        real = c.http.request

        async def spy(method, path, body=None, content_type="application/json", headers=None):
            st, resp = await real(method, path, body, content_type, headers)
            seen.append((method, content_type, (headers or {}).get("Accept", ""), resp[:4]))
            return st, resp
        c.http.request = spy
        try:
            pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "default",
                                                                   "labels": {"a": "b"}},
                   "spec": {"containers": [{"name": "c", "image": "busybox", "args": ["x", "y"]}]}}
            made = await c.create("pods", pod, "default")
            got = await c.get("pods", "p", "default")
            assert got["spec"]["containers"][0]["args"] == ["x", "y"] and got["metadata"]["uid"] == made["metadata"]["uid"]
            assert seen[0][1] == PROTOBUF and seen[0][3] == b"k8s\x00"        # protobuf both ways
            assert seen[1][2].startswith(PROTOBUF) and seen[1][3] == b"k8s\x00"
            lst = await c.list("pods", "default")
            assert [p["metadata"]["name"] for p in lst["items"]] == ["p"]
            # kinds outside the schema still go as JSON
            await c.create("configmaps", {"metadata": {"name": "cm"}, "data": {"k": "v"}}, "default")
            assert (await c.get("configmaps", "cm", "default"))["data"] == {"k": "v"}
            with pytest.raises(Exception) as e:
                await c.get("pods", "missing", "default")
            assert getattr(e.value, "code", None) == 404
        finally:
            await c.close()
            await s.stop()
    run(main(), timeout=60)
    with pytest.raises(ValueError):
        Client("http://x", content_type="application/yaml")


def test_informer_resync_redelivers_cached_objects(run):
    async def main():
        s = APIServer()
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        await c.create("configmaps", {"metadata": {"name": "cm"}, "data": {}}, "default")
        inf = Informer(c, "configmaps", "default", resync_period=0.1)
        same = []
        inf.add_handler(None, lambda old, new: same.append(old is new), None)
        inf.start()
        await inf.wait_synced()
        await asyncio.sleep(0.45)
        inf.stop()
        await c.close()
        await s.stop()
        assert len(same) >= 2 and all(same)
    run(main(), timeout=30)


def test_controller_full_resync_period(run):
    from kubernetes_amd.client.informer import InformerFactory
    from kubernetes_amd.controllers.base import Controller

    class Probe(Controller):
        name = "probe"
        primary = "configmaps"

        def setup(self):
            self.factory.get("configmaps").add_handler(self.enqueue, None, None)
            self.synced_keys = []

        async def sync(self, key):
            self.synced_keys.append(key)

    async def main():
        s = APIServer()
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        await c.create("configmaps", {"metadata": {"name": "cm"}, "data": {}}, "default")
        f = InformerFactory(c)
        p = Probe(c, f)
        p.resync_period = 0.1
        p.setup()
        f.start()
        await f.wait_for_cache_sync()
        p.start()
        await asyncio.sleep(0.5)
        p.stop()
        f.stop()
        await c.close()
        await s.stop()
        assert p.synced_keys.count("default/cm") >= 3     # the add + periodic resyncs
    run(main(), timeout=30)


def test_etcd_compaction_interval(run):
    async def main():
        s = APIServer(compaction_interval=0.15)
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        for i in range(5):
            await c.create("configmaps", {"metadata": {"name": f"cm{i}"}, "data": {}}, "default")
        await asyncio.sleep(0.5)
        rev = s.store.compacted_revision
        await c.close()
        await s.stop()
        assert s.compactions >= 2 and rev >= 5
    run(main(), timeout=30)


def test_delete_collection_workers(run):
    async def main():
        s = APIServer(delete_collection_workers=4)
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        for i in range(20):
            await c.create("configmaps", {"metadata": {"name": f"cm{i:02d}", "labels": {"x": "y"}}, "data": {}}, "default")
        out = await c.delete_collection("configmaps", "default", "x=y")
        left = (await c.list("configmaps", "default", label_selector="x=y"))["items"]
        await c.close()
        await s.stop()
        assert len(out["items"]) == 20 and not left
        assert [o["metadata"]["name"] for o in out["items"]] == [f"cm{i:02d}" for i in range(20)]
    run(main(), timeout=30)


class _Sink(BaseHTTPRequestHandler):
    got = []

    def do_POST(self):
        body = self.rfile.read(int(self.headers["Content-Length"]))
        _Sink.got.append((time.monotonic(), json.loads(body)))
        self.send_response(200)
        self.end_headers()

    def log_message(self, *a):
        pass


@pytest.fixture
def audit_sink(tmp_path):
    _Sink.got = []
    httpd = HTTPServer(("127.0.0.1", 0), _Sink)
    t = threading.Thread(target=httpd.serve_forever, daemon=True)
    t.start()
    kc = tmp_path / "audit.kubeconfig"
    kc.write_text(json.dumps({
        "apiVersion": "v1", "kind": "Config", "current-context": "a",
        "clusters": [{"name": "a", "cluster": {"server": f"http://127.0.0.1:{httpd.server_port}/audit"}}],
        "users": [{"name": "a", "user": {}}], "contexts": [{"name": "a", "context": {"cluster": "a", "user": "a"}}]}))
    yield str(kc)
    httpd.shutdown()


def test_audit_webhook_blocking_mode(run, audit_sink):
    from kubernetes_amd.apiserver.audit import AuditLogger, WebhookBackend

    async def main():
        wh = WebhookBackend(audit_sink, mode="blocking")
        s = APIServer(audit=AuditLogger(None, webhook=wh))
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        await c.create("configmaps", {"metadata": {"name": "cm"}, "data": {}}, "default")
        n = len(_Sink.got)            # delivered before the response came back
        await c.close()
        await s.stop()
        return n
    n = run(main(), timeout=30)
    assert n >= 1 and _Sink.got[-1][1]["items"][0]["verb"] == "create"


def test_audit_webhook_batch_throttle(audit_sink):
    from kubernetes_amd.apiserver.audit import WebhookBackend
    wh = WebhookBackend(audit_sink, max_batch=1, max_wait=0.01, throttle_qps=10, throttle_burst=1)
    t0 = time.monotonic()
    for i in range(4):
        wh.enqueue([json.dumps({"kind": "Event", "auditID": str(i)})])
    wh.close()
    assert len(_Sink.got) == 4
    assert _Sink.got[-1][0] - t0 >= 0.25       # 4 batches at 10/s with a burst of 1
    with pytest.raises(ValueError):
        WebhookBackend(audit_sink, mode="sometimes")


def test_failure_domains_for_empty_topology_key():
    from kubernetes_amd.scheduler.cache import SchedulerCache
    from kubernetes_amd.scheduler.generic import GenericScheduler

    def node(name, zone):
        return {"metadata": {"name": name, "labels": {"kubernetes.io/hostname": name,
                                                      "failure-domain.beta.kubernetes.io/zone": zone}},
                "spec": {}, "status": {"allocatable": {"cpu": "8", "memory": "16Gi", "pods": "110"},
                                       "conditions": [{"type": "Ready", "status": "True"}]}}

    def pod(name, labels, node_name=None, anti=False):
        p = {"metadata": {"name": name, "namespace": "default", "uid": name, "labels": labels},
             "spec": {"containers": [{"name": "c", "image": "x"}]}}
        if node_name:
            p["spec"]["nodeName"] = node_name
        if anti:
            p["spec"]["affinity"] = {"podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
                {"weight": 100, "podAffinityTerm": {"labelSelector": {"matchLabels": {"app": "web"}},
                                                    "topologyKey": ""}}]}}
        return p

    def place(domains):
        cache = SchedulerCache()
        if domains:
            cache.failure_domains = domains
        for n, z in (("a", "z1"), ("b", "z1"), ("c", "z2")):
            cache.add_node(node(n, z))
        cache.add_pod(pod("web-0", {"app": "web"}, "a"))
        return GenericScheduler(cache).schedule(pod("new", {"app": "x"}, anti=True))[0]
    assert place(None) == "c"                                  # b shares a's zone
    assert place(("kubernetes.io/hostname",)) != "a"            # only a's own host is the domain


def test_nodeipam_skips_the_service_range():
    from kubernetes_amd.controllers.network import CIDRSet
    s = CIDRSet("10.0.0.0/16", 24)
    assert s.exclude("10.0.0.0/24") == 1 and s.exclude("192.168.0.0/16") == 0
    assert s.allocate() == "10.0.1.0/24"
    s2 = CIDRSet("10.0.0.0/16", 24)
    s2.exclude("10.0.4.0/22")
    got = [s2.allocate() for _ in range(8)]
    assert not any(g.startswith(("10.0.4.", "10.0.5.", "10.0.6.", "10.0.7.")) for g in got)


def test_dynamic_provisioning_switch(run):
    from kubernetes_amd.controllers.volume import PersistentVolumeController

    async def main():
        pv = PersistentVolumeController(None, None, enable_dynamic_provisioning=False)
        # provisionClaim returns before touching the class, the claim or the API
        assert await pv.provision_claim({"metadata": {"name": "c", "namespace": "d", "uid": "u"},
                                         "spec": {"storageClassName": "gold"}}) is None
    run(main(), timeout=10)


def test_cpu_cfs_quota_switch(tmp_path):
    from kubernetes_amd.kubelet.cgroups import CgroupManager
    pod = {"metadata": {"name": "g", "namespace": "d", "uid": "u1"},
           "spec": {"containers": [{"name": "c", "resources": {"limits": {"cpu": "2", "memory": "1Gi"},
                                                               "requests": {"cpu": "2", "memory": "1Gi"}}}]}}
    on = CgroupManager(str(tmp_path / "on")).start()
    off = CgroupManager(str(tmp_path / "off"), cpu_cfs_quota=False).start()
    on.ensure_pod(pod)
    off.ensure_pod(pod)
    read = lambda m: open(os.path.join(m.pod_dir(pod), "cpu.max")).read()   # noqa: E731
    assert read(on).startswith("200000 ") and read(off).startswith("max ")


def test_contention_profiler_finds_the_blocking_call(run):
    from kubernetes_amd.utils import profiling

    def stall():
        time.sleep(0.15)

    async def main():
        prof = profiling.BlockProfiler(asyncio.get_running_loop()).start()
        await asyncio.sleep(0.05)
        stall()
        await asyncio.sleep(0.05)
        prof.stop()
        return prof.report()
    rep = run(main(), timeout=10)
    assert "stall" in rep and "blocked" in rep
