"""kube-controller-manager / kube-scheduler / kube-proxy command lines: the health and metrics
endpoints componentstatuses probes (10252 / 10251), controller worker counts, HPA and signing
settings, leader-election lock names, kube-proxy cleanup, conntrack and --write-config-to.

Parity: `cmd/kube-controller-manager/app/options/options.go`, `plugin/cmd/kube-scheduler/app/
server.go` (healthz/metrics servers, lock object flags), `cmd/kube-proxy/app/server.go`
(CleanupLeftovers, conntrack, WriteConfigTo).
"""
import asyncio
import json
import os
import socket
import subprocess
import sys
import time
import urllib.request

import pytest
import yaml

from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.controllers.manager import ControllerManager
from kubernetes_amd.proxy.cleanup import conntrack_max, set_conntrack, strip_kube_rules
from kubernetes_amd.utils.componentserver import ComponentServer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _get(url):
    with urllib.request.urlopen(url, timeout=5) as r:
        return r.status, r.read()


def test_component_server(run):
    async def main():
        class M:
            def render(self):
                return b"x_total 3\n"
        cs = ComponentServer("kubescheduler", metrics=M(), configz=lambda: {"port": 1})
        port = await cs.start("127.0.0.1", 0)
        try:
            st, body = await asyncio.to_thread(_get, f"http://127.0.0.1:{port}/healthz")
            assert (st, body) == (200, b"ok")
            assert (await asyncio.to_thread(_get, f"http://127.0.0.1:{port}/metrics"))[1] == b"x_total 3\n"
            assert json.loads((await asyncio.to_thread(_get, f"http://127.0.0.1:{port}/configz"))[1]) == {"kubescheduler": {"port": 1}}
            # a taken port is not fatal
            assert await ComponentServer("again").start("127.0.0.1", port) is None
        finally:
            await cs.stop()
    run(main())


def test_controller_workers_and_metrics(run):
    async def main():
        api = APIServer()
        from kubernetes_amd.client.rest import Client
        c = Client(f"http://127.0.0.1:{await api.start()}")
        try:
            cm = ControllerManager(c, ["deployment", "replicaset"], workers={"deployment": 2, "replicaset": 7})
            assert {x.name: x.workers for x in cm.controllers}["deployment"] == 2
            await cm.start()
            text = cm.render_metrics().decode()
            assert 'workqueue_depth{name="deployment"}' in text and 'controller_syncs_total{name="replicaset"}' in text
            await cm.stop()
        finally:
            await c.close()
            await api.stop()
    run(main())


def _spawn(args):
    return subprocess.Popen([sys.executable, "-m"] + args, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                            env=dict(os.environ, PYTHONPATH=ROOT))


def _wait_http(url, proc, timeout=60):
    t = time.time()
    while time.time() - t < timeout:
        if proc.poll() is not None:
            raise AssertionError(proc.stderr.read()[-800:])
        try:
            return _get(url)
        except OSError:
            time.sleep(0.1)
    raise TimeoutError(url)


def test_controller_manager_and_scheduler_serve_health(tmp_path):
    pf = tmp_path / "port"
    api = _spawn(["kubernetes_amd.cmd.apiserver", "--port", "0", "--port-file", str(pf), "--storage-engine", "python"])
    procs = [api]
    try:
        t = time.time()
        while not (pf.exists() and pf.read_text().strip()):
            assert time.time() - t < 60 and api.poll() is None
            time.sleep(0.05)
        url = f"http://127.0.0.1:{pf.read_text().strip()}"
        cmp_, sp = _free(), _free()
        cm = _spawn(["kubernetes_amd.cmd.controller_manager", "--master", url, "--port", str(cmp_), "--address", "127.0.0.1",
                     "--concurrent-deployment-syncs", "3", "--horizontal-pod-autoscaler-upscale-delay", "1m"])
        sch = _spawn(["kubernetes_amd.cmd.scheduler", "--master", url, "--port", str(sp), "--address", "127.0.0.1",
                      "--hard-pod-affinity-symmetric-weight", "5"])
        procs += [cm, sch]
        assert _wait_http(f"http://127.0.0.1:{cmp_}/healthz", cm) == (200, b"ok")
        cfg = json.loads(_get(f"http://127.0.0.1:{cmp_}/configz")[1])["componentconfig"]
        assert cfg["concurrent_deployment_syncs"] == 3 and cfg["horizontal_pod_autoscaler_upscale_delay"] == "1m"
        for _ in range(100):
            if b"workqueue_depth" in _get(f"http://127.0.0.1:{cmp_}/metrics")[1]:
                break
            time.sleep(0.1)
        assert b'workqueue_depth{name="deployment"}' in _get(f"http://127.0.0.1:{cmp_}/metrics")[1]
        assert _wait_http(f"http://127.0.0.1:{sp}/healthz", sch) == (200, b"ok")
        assert b"scheduler_e2e_scheduling_latency_microseconds" in _get(f"http://127.0.0.1:{sp}/metrics")[1]
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            p.wait(10)


@pytest.mark.parametrize("argv,needle", [
    (["kubernetes_amd.cmd.controller_manager", "--cloud-provider", "aws"], "out of scope"),
    (["kubernetes_amd.cmd.scheduler", "--hard-pod-affinity-symmetric-weight", "101"], "0..100"),
])
def test_component_cli_rejects(argv, needle):
    r = subprocess.run([sys.executable, "-m"] + argv + ["--master", "http://127.0.0.1:9"], capture_output=True,
                       text=True, timeout=60, env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode != 0 and needle in r.stderr + r.stdout, r.stderr[-500:]


SAVE = """# Generated by iptables-save
*nat
:PREROUTING ACCEPT [0:0]
:OUTPUT ACCEPT [0:0]
:POSTROUTING ACCEPT [0:0]
:DOCKER - [0:0]
:KUBE-SERVICES - [0:0]
:KUBE-SVC-ABC - [0:0]
:KUBE-POSTROUTING - [0:0]
-A PREROUTING -m comment --comment "kubernetes service portals" -j KUBE-SERVICES
-A PREROUTING -m addrtype --dst-type LOCAL -j DOCKER
-A OUTPUT -j KUBE-SERVICES
-A POSTROUTING -j KUBE-POSTROUTING
-A POSTROUTING -s 172.17.0.0/16 ! -o docker0 -j MASQUERADE
-A KUBE-SERVICES -d 10.0.0.1/32 -p tcp -j KUBE-SVC-ABC
-A KUBE-SVC-ABC -j DNAT --to-destination 10.1.0.5:443
COMMIT
"""


def test_proxy_cleanup_and_conntrack(tmp_path):
    out = strip_kube_rules(SAVE)
    assert "KUBE-" not in out
    assert ":DOCKER - [0:0]" in out and "-j DOCKER" in out and "-j MASQUERADE" in out and out.strip().endswith("COMMIT")
    assert conntrack_max(32768, 131072, cpus=2) == 131072 and conntrack_max(32768, 131072, cpus=64) == 2097152
    assert conntrack_max(0, 131072) == 0
    for rel in ("proc/sys/net/netfilter", "sys/module/nf_conntrack/parameters"):
        (tmp_path / rel).mkdir(parents=True)
    (tmp_path / "sys/module/nf_conntrack/parameters/hashsize").write_text("1048576\n")
    failed = set_conntrack(2097152, 86400, root=str(tmp_path))
    assert not failed
    assert (tmp_path / "proc/sys/net/netfilter/nf_conntrack_max").read_text() == "2097152"
    assert (tmp_path / "proc/sys/net/netfilter/nf_conntrack_tcp_timeout_established").read_text() == "86400"
    assert (tmp_path / "sys/module/nf_conntrack/parameters/hashsize").read_text().strip() == "1048576"   # not shrunk


def test_proxy_write_config_to(tmp_path):
    out = tmp_path / "kp.yaml"
    r = subprocess.run([sys.executable, "-m", "kubernetes_amd.cmd.proxy", "--proxy-mode", "ipvs", "--cluster-cidr",
                        "10.244.0.0/16", "--iptables-masquerade-bit", "12", "--healthz-bind-address", "0.0.0.0:20256",
                        "--write-config-to", str(out)], capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stderr[-500:]
    cfg = yaml.safe_load(out.read_text())
    assert cfg["kind"] == "KubeProxyConfiguration" and cfg["mode"] == "ipvs" and cfg["clusterCIDR"] == "10.244.0.0/16"
    assert cfg["iptables"]["masqueradeBit"] == 12 and cfg["healthzBindAddress"].endswith(":20256")
    # the written file is a valid --config input
    from argparse import Namespace
    from kubernetes_amd.cmd.proxy import apply_config_file
    a = Namespace(proxy_mode="iptables", cluster_cidr="", bind_address="127.0.0.1", hostname_override="h",
                  masquerade_all=False, iptables_sync_period=30.0, iptables_min_sync_period=0.0, ipvs_scheduler="rr",
                  healthz_port=10256, metrics_port=10249, kubeconfig=None)
    apply_config_file(a, str(out))
    assert a.proxy_mode == "ipvs" and a.healthz_port == 20256
