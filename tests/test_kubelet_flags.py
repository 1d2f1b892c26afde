"""The reference kubelet's command-line surface: TLS serving (self-signed or given, x509 client
authentication), read-only and healthz ports, debugging handlers, registration options,
privileged / host-namespace admission, soft eviction, image pull throttling, host checks, and
API-server-to-kubelet HTTPS.

Parity: `cmd/kubelet/app/options/options.go` flags and `server.go` (InitializeTLS,
ListenAndServeKubeletReadOnlyServer, healthz), `pkg/kubelet/kubelet.go` canRunPod,
`pkg/kubelet/eviction/helpers.go` (ParseThresholdConfig, thresholdsMetGracePeriod, minimum
reclaim), `pkg/kubelet/images/puller.go` (serial puller, throttleImagePulling).
"""
import asyncio
import json
import os
import ssl
import subprocess
import sys
import threading

import pytest

from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.cmd import kubelet as kcmd
from kubernetes_amd.kubelet import hostchecks as H
from kubernetes_amd.kubelet.eviction import EvictionManager, parse_soft_thresholds, parse_thresholds
from kubernetes_amd.kubelet.images import ImageManager
from kubernetes_amd.native import crypto
from kubernetes_amd.utils.tlsutil import client_context, self_signed_serving_cert


def test_flag_parsers():
    assert kcmd._taints("dedicated=gpu:NoSchedule,maint:NoExecute") == [
        {"key": "dedicated", "value": "gpu", "effect": "NoSchedule"}, {"key": "maint", "effect": "NoExecute"}]
    with pytest.raises(SystemExit):
        kcmd._taints("k=v:Sometimes")
    assert kcmd._duration("1m30s") == 90 and kcmd._duration("2h") == 7200 and kcmd._duration("500ms") == 0.5
    assert kcmd._duration("15") == 15.0


def test_host_checks(tmp_path):
    swaps = tmp_path / "swaps"
    swaps.write_text("Filename\tType\tSize\tUsed\tPriority\n")
    assert not H.swap_enabled(str(swaps))
    H.check_swap(True, str(swaps))
    swaps.write_text("Filename\tType\tSize\tUsed\tPriority\n/swapfile file 1048572 0 -2\n")
    with pytest.raises(H.HostCheckError, match="swap"):
        H.check_swap(True, str(swaps))
    H.check_swap(False, str(swaps))
    root = tmp_path / "sys"
    for k, v in (("vm/overcommit_memory", 0), ("vm/panic_on_oom", 0), ("kernel/panic", 10), ("kernel/panic_on_oops", 1)):
        (root / k).parent.mkdir(parents=True, exist_ok=True)
        (root / k).write_text(f"{v}\n")
    assert H.kernel_default_mismatches(str(root)) == ["vm.overcommit_memory=0 (want 1)"]
    with pytest.raises(H.HostCheckError):
        H.check_kernel_defaults(True, str(root))
    H.check_kernel_defaults(False, str(root))
    # lock file: exclusive, and another open of it is noticed
    lk = H.LockFile(str(tmp_path / "kubelet.lock")).acquire()
    hit = threading.Event()
    lk.watch_contention(hit.set)
    with open(tmp_path / "kubelet.lock"):
        pass
    assert hit.wait(5)
    other = H.LockFile(str(tmp_path / "kubelet.lock"))
    with pytest.raises(BlockingIOError):
        other.acquire(blocking=False)
    lk.release()
    other.acquire(blocking=False).release()


def test_soft_eviction_grace_and_minimum_reclaim():
    now = [0.0]
    avail = [900 << 20]
    th = parse_thresholds("memory.available<100Mi", "memory.available=200Mi") + \
        parse_soft_thresholds("memory.available<1Gi", "memory.available=1m30s")
    with pytest.raises(ValueError, match="grace period must be specified"):
        parse_soft_thresholds("memory.available<1Gi", "")
    em = EvictionManager(th, lambda: {"memory.available": (avail[0], 16 << 30)}, max_pod_grace=20,
                         clock=lambda: now[0])
    pod = {"metadata": {"name": "p", "uid": "u"}, "spec": {"terminationGracePeriodSeconds": 60},
           "status": {"qosClass": "BestEffort"}}
    v, msg, grace = em.select_victim_with_grace([pod])
    assert v is None and em.has("MemoryPressure")          # condition at once, eviction after the grace period
    now[0] = 91.0
    v, msg, grace = em.select_victim_with_grace([pod])
    assert v is pod and grace == 20 and msg == "The node was low on resource: memory."   # soft: --eviction-max-pod-grace-period
    avail[0] = 50 << 20                                      # under the hard threshold: immediate, grace 0
    v, msg, grace = em.select_victim_with_grace([pod])
    assert v is pod and grace == 0
    avail[0] = 250 << 20                                     # above 100Mi but below 100Mi + 200Mi reclaim
    assert any(t.hard for t in em.observe())
    avail[0] = 400 << 20
    assert not any(t.hard for t in em.observe())
    # allocatable only subtracts hard thresholds
    assert em.hard_memory_bytes() == 100 << 20


def test_image_pulls_serialized_and_throttled(run):
    class Svc:
        def __init__(self):
            self.active = self.peak = 0

        async def image_status(self, image):
            return None

        async def pull_image(self, image, auth=None):
            self.active += 1
            self.peak = max(self.peak, self.active)
            await asyncio.sleep(0.05)
            self.active -= 1
            return image

    async def main():
        svc = Svc()
        t = [0.0]
        im = ImageManager(svc, serialize=True, qps=1.0, burst=2, clock=lambda: t[0])
        pod = {"metadata": {"name": "p", "namespace": "default"}, "spec": {}}
        res = await asyncio.gather(*(im.ensure_image_exists(pod, {"image": f"img{i}:v1"}) for i in range(3)),
                                   return_exceptions=True)
        assert svc.peak == 1                                 # serial puller
        errs = [r for r in res if isinstance(r, Exception)]
        assert len(errs) == 1 and "QPS exceeded" in str(errs[0])
        t[0] = 100.0                                         # tokens refilled (and back-off passed)
        assert await im.ensure_image_exists(pod, {"image": "img9:v1"}) == "img9:v1"
        par = ImageManager(Svc(), serialize=False)
        await asyncio.gather(*(par.ensure_image_exists(pod, {"image": f"x{i}:v1"}) for i in range(3)))
        assert par.service.peak == 3
    run(main())


def _get(url, ctx=None, method="GET", cert=None):
    import http.client
    from urllib.parse import urlsplit
    u = urlsplit(url)
    if u.scheme == "https":
        c = http.client.HTTPSConnection(u.hostname, u.port, context=ctx, timeout=10)
    else:
        c = http.client.HTTPConnection(u.hostname, u.port, timeout=10)
    c.request(method, u.path + (("?" + u.query) if u.query else ""))
    r = c.getresponse()
    return r.status, r.read()


def test_kubelet_tls_ports_and_registration(run, tmp_path):
    cert, key = self_signed_serving_cert(str(tmp_path / "pki"), "node-0", ["127.0.0.1"])
    assert self_signed_serving_cert(str(tmp_path / "pki"), "node-0") == (cert, key)    # reused
    ca, ca_key = crypto.self_signed_ca("clients")
    (tmp_path / "ca.crt").write_text(ca)
    ck = crypto.generate_key()
    (tmp_path / "client.key").write_text(ck)
    (tmp_path / "client.crt").write_text(crypto.issue_cert(key_pem=ck, cn="kube-apiserver-kubelet-client",
                                                           orgs=("system:masters",), ca_cert=ca, ca_key=ca_key,
                                                           usage="client"))
    from kubernetes_amd.kubelet.server_auth import KubeletAuth

    async def main():
        kw = {"tls": (cert, key, str(tmp_path / "ca.crt")), "read_only_port": 0, "healthz_port": 0,
              "address": "0.0.0.0", "node_ip": "127.0.0.1", "register_taints": [{"key": "dedicated", "value": "gpu", "effect": "NoSchedule"}],
              "register_schedulable": False, "provider_id": "amd://rack1/node-0", "allow_privileged": False,
              "host_sources": {"hostNetwork": ["file"]}}
        async with LocalCluster(nodes=1, gpus_per_node=0, kubelet_http=True, kubelet_kwargs=kw) as cl:
            kl = cl.nodes[0].kubelet
            kl.auth = KubeletAuth(cl.client, "node-0", anonymous=False)   # x509 only
            node = await cl.client.get("nodes", "node-0")
            assert {"type": "InternalIP", "address": "127.0.0.1"} in node["status"]["addresses"]   # not the bind address
            assert node["spec"]["taints"] == [{"key": "dedicated", "value": "gpu", "effect": "NoSchedule"}]
            assert node["spec"]["unschedulable"] and node["spec"]["providerID"] == "amd://rack1/node-0"
            base = f"https://127.0.0.1:{kl.http_port}"
            plain = await asyncio.to_thread(lambda: _get_or_error(f"http://127.0.0.1:{kl.http_port}/healthz"))
            assert plain != 200                                       # TLS only
            st, _ = await asyncio.to_thread(_get, base + "/pods", client_context())
            assert st == 401                                          # no client certificate, anonymous off
            cctx = client_context(None, str(tmp_path / "client.crt"), str(tmp_path / "client.key"))
            st, body = await asyncio.to_thread(_get, base + "/pods", cctx)
            assert st == 200 and json.loads(body)["kind"] == "PodList"
            # read-only port: no auth, GET only, no debugging handlers
            ro = f"http://127.0.0.1:{kl.read_only_port}"
            st, body = await asyncio.to_thread(_get, ro + "/pods")
            assert st == 200
            st, _ = await asyncio.to_thread(_get, ro + "/containerLogs/default/x/c")
            assert st == 404
            st, _ = await asyncio.to_thread(_get, ro + "/pods", None, "POST")
            assert st == 405
            st, body = await asyncio.to_thread(_get, f"http://127.0.0.1:{kl.healthz_port}/healthz")
            assert st == 200 and body == b"ok"
            # the API server reaches the kubelet over https for the node proxy and pod logs
            cl.api.kubelet_ssl, cl.api.kubelet_scheme = cctx, "https"
            st, body = await cl.client.raw("GET", "/api/v1/nodes/node-0/proxy/healthz")
            assert st == 200 and body == b"ok"
            # canRunPod: privileged and (source-restricted) host networking are refused
            await cl.client.patch("nodes", "node-0", {"spec": {"unschedulable": False, "taints": None}})
            for name, spec in (("priv", {"containers": [{"name": "c", "image": "x", "securityContext": {"privileged": True}}]}),
                               ("hostnet", {"hostNetwork": True, "containers": [{"name": "c", "image": "x"}]})):
                await cl.client.create("pods", {"metadata": {"name": name, "namespace": "default"}, "spec": spec})
                p = await cl.wait_pod(name, phase="Failed", timeout=20)
                assert p["status"]["reason"] == "Forbidden" and "disallowed" in p["status"]["message"]
            await cl.client.create("pods", {"metadata": {"name": "ok", "namespace": "default"},
                                            "spec": {"containers": [{"name": "c", "image": "x"}]}})
            await cl.wait_pod("ok", timeout=20)
            st, body = await cl.client.raw("GET", "/api/v1/namespaces/default/pods/ok/log")
            assert st == 200
    run(main(), timeout=90)


def _get_or_error(url):
    try:
        return _get(url)[0]
    except (OSError, ssl.SSLError, Exception):   # noqa: BLE001 - a TLS port answers plain HTTP with garbage
        return -1


def test_kubelet_debugging_handlers_off(run):
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=0, kubelet_http=True,
                                kubelet_kwargs={"debugging_handlers": False}) as cl:
            kl = cl.nodes[0].kubelet
            base = f"http://127.0.0.1:{kl.http_port}"
            assert (await asyncio.to_thread(_get, base + "/healthz"))[0] == 200
            for p in ("/containerLogs/default/x/c", "/exec/default/x/c", "/configz", "/runningpods/", "/logs/"):
                assert (await asyncio.to_thread(_get, base + p))[0] == 404, p
    run(main(), timeout=60)


@pytest.mark.parametrize("argv,needle", [
    (["--cloud-provider", "aws"], "cloud providers are out of scope"),
    (["--runonce=true"], "not supported"),
    (["--register-with-taints", "k=v:Bogus"], "invalid taint"),
])
def test_kubelet_cli_rejects(argv, needle, tmp_path):
    r = subprocess.run([sys.executable, "-m", "kubernetes_amd.cmd.kubelet", "--root-dir", str(tmp_path), "--fail-swap-on=false",
                        "--master", "http://127.0.0.1:9"] + argv, capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    assert r.returncode != 0 and needle in (r.stderr + r.stdout), r.stderr[-500:]
