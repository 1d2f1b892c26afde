"""Kubelet networking (host-local IPAM, kubenet, CNI exec protocol, DNS / hosts files, host
ports), node IPAM and LoadBalancer controllers, container GC and `logs --previous`.

Reference tests mirrored: pkg/kubelet/network/cni/cni_test.go (fake plugin binary fed the net
config on stdin), kubenet_linux_test.go, dns/dns_test.go, hostport/hostport_manager_test.go,
pkg/controller/node/ipam/cidrset/cidr_set_test.go, container_gc_test.go.
"""
import asyncio
import json
import os
import socket
import stat
import sys

import pytest

from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.controllers.network import CIDRSet
from kubernetes_amd.kubelet import network as net


def pod(name="p", ns="default", **spec):
    return {"metadata": {"name": name, "namespace": ns, "uid": "u-" + name},
            "spec": dict({"containers": [{"name": "c", "image": "busybox"}]}, **spec)}


def test_host_local_ipam(tmp_path):
    ipam = net.HostLocalIPAM(str(tmp_path / "ipam"), "10.9.0.0/29")
    ips = [ipam.allocate(f"c{i}") for i in range(5)]
    assert ips == [f"10.9.0.{i}" for i in range(2, 7)]           # .0 network, .1 gateway, .7 broadcast
    assert ipam.allocate("c0") == "10.9.0.2"                      # idempotent per container
    with pytest.raises(net.NetworkError):
        ipam.allocate("c9")
    ipam.release("c2")
    assert ipam.allocate("c9") == "10.9.0.4"
    # state is on disk: a new allocator (kubelet restart) sees the same reservations
    again = net.HostLocalIPAM(str(tmp_path / "ipam"), "10.9.0.0/29")
    with pytest.raises(net.NetworkError):
        again.allocate("other")


def test_dns_and_hosts(tmp_path, feature_gate):
    rc = tmp_path / "resolv.conf"
    rc.write_text("nameserver 192.168.1.1\nsearch corp.example\noptions timeout:2\n")
    d = net.DNSConfigurer(["10.96.0.10"], "cluster.local", str(rc))
    text = d.resolv_text(pod(ns="ml"))
    assert "nameserver 10.96.0.10" in text
    assert "search ml.svc.cluster.local svc.cluster.local cluster.local corp.example" in text
    assert "options ndots:5" in text
    assert "nameserver 192.168.1.1" in d.resolv_text(pod(dnsPolicy="Default"))
    assert "nameserver 192.168.1.1" in d.resolv_text(pod(hostNetwork=True))           # ClusterFirst + hostNetwork
    assert "nameserver 10.96.0.10" in d.resolv_text(pod(hostNetwork=True, dnsPolicy="ClusterFirstWithHostNet"))
    feature_gate.set("CustomPodDNS=true")
    custom = d.resolv_text(pod(dnsPolicy="None", dnsConfig={
        "nameservers": ["1.1.1.1"], "searches": ["a.b"], "options": [{"name": "ndots", "value": "2"}, {"name": "edns0"}]}))
    assert custom == "nameserver 1.1.1.1\nsearch a.b\noptions ndots:2 edns0\n"
    many = d.pod_dns(pod(dnsConfig={"nameservers": ["1.1.1.1", "2.2.2.2", "3.3.3.3"],
                                    "searches": [f"s{i}.example" for i in range(10)]}))
    assert len(many[0]) == 3 and len(many[1]) == 6
    hosts = d.hosts_text(pod(hostname="w0", subdomain="workers", hostAliases=[{"ip": "10.1.1.1", "hostnames": ["db"]}]),
                         "10.244.1.5")
    assert "10.244.1.5\tw0.workers.default.svc.cluster.local\tw0" in hosts and "10.1.1.1\tdb" in hosts
    mounts = d.write_pod_files(str(tmp_path / "pod"), pod(), "10.244.1.5")
    assert {m["containerPath"] for m in mounts} == {"/etc/hosts", "/etc/resolv.conf"}
    assert "10.244.1.5\tp" in (tmp_path / "pod" / "etc-hosts").read_text()


def test_hostports_hold_and_rules():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    hm = net.HostportManager()
    p1 = pod("a", containers=[{"name": "c", "image": "x", "ports": [{"containerPort": 80, "hostPort": port,
                                                                     "hostIP": "127.0.0.1"}]}])
    p2 = pod("b", containers=[{"name": "c", "image": "x", "ports": [{"containerPort": 81, "hostPort": port,
                                                                     "hostIP": "127.0.0.1"}]}])
    hm.add(p1, "10.244.0.5")
    rules = hm.rules()
    assert f"--dport {port} -j KUBE-HP-" in rules and "DNAT --to-destination 10.244.0.5:80" in rules
    hm2 = net.HostportManager()
    with pytest.raises(net.NetworkError):       # the port is held by the first manager
        hm2.add(p2, "10.244.0.6")
    hm.remove(p1)
    hm2.add(p2, "10.244.0.6")
    hm2.close()
    hm.close()
    assert hm.add(pod("h", hostNetwork=True), "x") == []


FAKE_CNI = r'''#!{py}
import json, os, sys
conf = json.load(sys.stdin)
with open(os.environ["CNI_LOG"], "a") as f:
    f.write(json.dumps({{"cmd": os.environ["CNI_COMMAND"], "type": conf["type"], "id": os.environ["CNI_CONTAINERID"],
                        "args": os.environ["CNI_ARGS"], "prev": conf.get("prevResult"), "subnet": conf.get("ipam", {{}}).get("subnet")}}) + "\n")
if os.environ["CNI_COMMAND"] == "ADD":
    if conf["type"] == "fakebridge":
        print(json.dumps({{"cniVersion": "0.3.1", "ips": [{{"version": "4", "address": "10.88.0.7/24"}}]}}))
    else:
        print(json.dumps(conf["prevResult"]))
'''


def test_cni_plugin_protocol(run, tmp_path, monkeypatch):
    bindir, confdir = tmp_path / "bin", tmp_path / "net.d"
    bindir.mkdir()
    confdir.mkdir()
    for name in ("fakebridge", "fakeportmap"):
        p = bindir / name
        p.write_text(FAKE_CNI.format(py=sys.executable))
        p.chmod(p.stat().st_mode | stat.S_IEXEC)
    (confdir / "10-test.conflist").write_text(json.dumps({
        "cniVersion": "0.3.1", "name": "mi355x-net",
        "plugins": [{"type": "fakebridge", "ipam": {"type": "host-local", "subnet": "usePodCidr"}},
                    {"type": "fakeportmap", "capabilities": {"portMappings": True}}]}))
    log = tmp_path / "cni.log"
    monkeypatch.setenv("CNI_LOG", str(log))
    plugin = net.CNIPlugin(str(confdir), [str(bindir)], pod_cidr="10.88.0.0/24")
    assert plugin.status() is None

    async def main():
        ip = await plugin.setup_pod(pod("web", ns="ml"), "sandbox-1")
        assert ip == "10.88.0.7"
        await plugin.teardown_pod(pod("web", ns="ml"), "sandbox-1")
    run(main())
    calls = [json.loads(x) for x in log.read_text().splitlines()]
    assert [(c["cmd"], c["type"]) for c in calls] == [("ADD", "fakebridge"), ("ADD", "fakeportmap"),
                                                      ("DEL", "fakeportmap"), ("DEL", "fakebridge")]
    assert calls[0]["subnet"] == "10.88.0.0/24" and "K8S_POD_NAMESPACE=ml;K8S_POD_NAME=web" in calls[0]["args"]
    assert calls[1]["prev"]["ips"][0]["address"] == "10.88.0.7/24"        # chained plugins get prevResult
    assert net.CNIPlugin(str(tmp_path / "empty"), [str(bindir)]).status() == "cni config uninitialized"


def test_cidr_set():
    cs = CIDRSet("10.244.0.0/22", 24)
    assert cs.occupy("10.244.1.0/24")
    assert [cs.allocate() for _ in range(3)] == ["10.244.0.0/24", "10.244.2.0/24", "10.244.3.0/24"]
    with pytest.raises(RuntimeError):
        cs.allocate()
    cs.release("10.244.2.0/24")
    assert cs.allocate() == "10.244.2.0/24"
    assert not cs.occupy("192.168.0.0/24")


def test_kubenet_with_node_ipam_end_to_end(run, tmp_path):
    async def main():
        cl = LocalCluster(nodes=0, gpus_per_node=0, workdir=str(tmp_path / "c"), controllers=["nodeipam"],
                          controller_options={"nodeipam": {"cluster_cidr": "10.200.0.0/16"}})
        await cl.start()
        try:
            cl.kubelet_kwargs = {"network_plugin": net.KubenetPlugin(str(tmp_path / "netdata")),
                                 "dns": net.DNSConfigurer(["10.96.0.10"], "cluster.local", ""),
                                 "hostports": net.HostportManager(hold_sockets=False)}
            await cl.add_node("node-0")
            c = cl.client

            async def ready():
                n = await c.get("nodes", "node-0")
                conds = {x["type"]: x["status"] for x in (n.get("status") or {}).get("conditions") or ()}
                return n if n["spec"].get("podCIDR") and conds.get("Ready") == "True" else None
            n = await cl.wait_for(ready, 20)
            assert n["spec"]["podCIDR"] == "10.200.0.0/24"
            await c.create("pods", {"metadata": {"name": "web"}, "spec": {"containers": [
                {"name": "c", "image": "nginx", "ports": [{"containerPort": 80, "hostPort": 8080}]}]}}, "default")

            async def running():
                p = await c.get("pods", "web", "default")
                return p if (p.get("status") or {}).get("podIP") and p["status"].get("phase") == "Running" else None
            p = await cl.wait_for(running, 20)
            assert p["status"]["podIP"].startswith("10.200.0.") and p["status"]["podIP"] != "10.200.0.1"
            kl = cl.nodes[0].kubelet
            resolv = open(os.path.join(kl.root_dir, "pods", p["metadata"]["uid"], "resolv.conf")).read()
            assert "nameserver 10.96.0.10" in resolv and "search default.svc.cluster.local" in resolv
            assert f"DNAT --to-destination {p['status']['podIP']}:80" in kl.hostports.rules()
            await c.delete("pods", "web", "default", grace_period=0)

            async def released():
                return not kl.network.ipam._reserved()
            await cl.wait_for(released, 20)
        finally:
            await cl.stop()
    run(main(), timeout=60)


def test_loadbalancer_pool(run, tmp_path):
    async def main():
        cl = LocalCluster(nodes=0, gpus_per_node=0, workdir=str(tmp_path / "c"), controllers=["service"],
                          controller_options={"service": {"ip_range": "192.0.2.10-192.0.2.11"}})
        await cl.start()
        c = cl.client
        try:
            def svc(name, **spec):
                return {"metadata": {"name": name}, "spec": dict({"type": "LoadBalancer", "selector": {"app": name},
                                                                  "ports": [{"port": 80}]}, **spec)}
            await c.create("services", svc("a"), "default")
            await c.create("services", svc("b", loadBalancerIP="192.0.2.11"), "default")

            async def ingress(name):
                s = await c.get("services", name, "default")
                ing = ((s.get("status") or {}).get("loadBalancer") or {}).get("ingress")
                return ing[0]["ip"] if ing else None
            assert await cl.wait_for(lambda: ingress("b"), 10) == "192.0.2.11"
            assert await cl.wait_for(lambda: ingress("a"), 10) == "192.0.2.10"
            await c.create("services", svc("c"), "default")                        # pool exhausted
            await asyncio.sleep(0.3)
            assert await ingress("c") is None
            await c.patch("services", "a", {"spec": {"type": "ClusterIP"}}, "default")   # releases .10

            async def c_gets_it():
                return await ingress("c") == "192.0.2.10" and await ingress("a") is None
            assert await cl.wait_for(c_gets_it, 10)
        finally:
            await cl.stop()
    run(main(), timeout=60)


def test_crashloop_backoff_container_gc_and_previous_logs(run, tmp_path):
    async def main():
        cl = LocalCluster(nodes=1, gpus_per_node=0, runtime="process", workdir=str(tmp_path / "c"),
                          kubelet_kwargs={"crash_backoff": (0.3, 0.6)})
        await cl.start()
        c = cl.client
        kl = cl.nodes[0].kubelet
        try:
            await c.create("pods", {"metadata": {"name": "crash"}, "spec": {"containers": [
                {"name": "c", "image": "busybox", "command": ["sh", "-c", "echo attempt-$$; exit 3"]}]}}, "default")

            async def backing_off():
                p = await c.get("pods", "crash", "default")
                for cs in (p.get("status") or {}).get("containerStatuses") or ():
                    w = (cs.get("state") or {}).get("waiting") or {}
                    if w.get("reason") == "CrashLoopBackOff":
                        return cs
                return None
            cs = await cl.wait_for(backing_off, 20)
            assert cs["lastState"]["terminated"]["exitCode"] == 3 and "Back-off" in cs["state"]["waiting"]["message"]
            st = next(s for s in kl.pods.values() if s.pod["metadata"]["name"] == "crash")
            await cl.wait_for(lambda: _true(st.restarts.get("c", 0) >= 2 and st.previous.get("c")), 20)
            assert st.backoff["c"][1] in (0.6,)                     # doubled once, then capped
            code, body = await kl_http_logs(cl, "crash", previous=True)
            assert code == 200 and b"attempt-" in body
            # default policy keeps one dead instance per container; the latest instance the pod's
            # status comes from is never removed while the pod lives
            cur = st.containers.get("c")
            assert cur not in await kl.garbage_collect_containers()
            kl.container_gc = {"max_per_pod_container": 0}
            prev = st.previous.get("c")
            cur = st.containers.get("c")
            removed = await kl.garbage_collect_containers()
            assert cur not in removed, (cur, prev, removed)
            assert prev is None or prev == cur or prev in removed, (cur, prev, removed)
        finally:
            await cl.stop()
    run(main(), timeout=60)


async def _true(v):
    return v


async def kl_http_logs(cl, name, previous=False):
    kl = cl.nodes[0].kubelet

    class Req:
        path = f"/containerLogs/default/{name}/c"
        query = {"previous": "true"} if previous else {}
        headers = {}
        method = "GET"
    r = await kl._http(Req())
    return r.status, r.body


def test_kubenet_delegates_to_cni_bridge(run, tmp_path):
    """kubenet with a netns and CNI binaries: the generated bridge config (hairpin, MTU, host-local
    over the pod CIDR) then loopback, as in `kubenet_linux.go` setUpPod."""
    import json as _json
    import stat
    import sys as _sys
    bindir = tmp_path / "bin"
    bindir.mkdir()
    calls = tmp_path / "calls.jsonl"
    script = ("#!" + _sys.executable + "\nimport json,os,sys\nconf=json.load(sys.stdin)\n"
              f"open({str(calls)!r},'a').write(json.dumps({{'cmd':os.environ['CNI_COMMAND'],'conf':conf,"
              "'netns':os.environ['CNI_NETNS']})+'\\n')\n"
              "if os.environ['CNI_COMMAND']=='ADD' and conf['type']=='bridge':\n"
              "    print(json.dumps({'ip4':{'ip':'10.244.1.7/24'}}))\n")
    for name in ("bridge", "host-local", "loopback"):
        f = bindir / name
        f.write_text(script)
        f.chmod(f.stat().st_mode | stat.S_IEXEC)

    async def main():
        k = net.KubenetPlugin(str(tmp_path / "d"), mtu=9000, cni_bin_dirs=[str(bindir)], hairpin_mode="hairpin-veth")
        k.set_pod_cidr("10.244.1.0/24")
        pod = {"metadata": {"name": "p", "namespace": "default"}}
        assert await k.setup_pod(pod, "sb1", "/var/run/netns/x") == "10.244.1.7"
        await k.teardown_pod(pod, "sb1", "/var/run/netns/x")
        recs = [_json.loads(line) for line in calls.read_text().splitlines()]
        assert [(r["cmd"], r["conf"]["type"]) for r in recs] == [("ADD", "bridge"), ("ADD", "loopback"), ("DEL", "bridge")]
        b = recs[0]["conf"]
        assert b["bridge"] == "cbr0" and b["mtu"] == 9000 and b["hairpinMode"] is True and b["isGateway"] is True
        assert b["ipam"]["subnet"] == "10.244.1.0/24" and b["ipMasq"] is False
        # no namespace (process runtime): in-process host-local allocation
        ip = await k.setup_pod(pod, "sb2", "")
        assert ip.startswith("10.244.1.") and len(calls.read_text().splitlines()) == 3
        with pytest.raises(ValueError):
            net.KubenetPlugin(str(tmp_path / "e"), hairpin_mode="bogus")
    run(main())


def test_make_port_mappings():
    """`pkg/kubelet/container/helpers_test.go` TestMakePortMappings."""
    def port(name, proto, cport, hport, ip):
        return {"name": name, "protocol": proto, "containerPort": cport, "hostPort": hport, "hostIP": ip}
    c = {"name": "fooContainer", "ports": [port("", "TCP", 80, 8080, "127.0.0.1"), port("", "TCP", 443, 4343, "192.168.0.1"),
                                           port("foo", "UDP", 555, 5555, ""), port("foo", "UDP", 888, 8888, ""),
                                           port("", "TCP", 80, 8888, "")]}
    got = net.make_port_mappings(c)
    assert [(m["name"], m["protocol"], m["containerPort"], m["hostPort"], m["hostIP"]) for m in got] == [
        ("fooContainer-TCP:80", "TCP", 80, 8080, "127.0.0.1"), ("fooContainer-TCP:443", "TCP", 443, 4343, "192.168.0.1"),
        ("fooContainer-foo", "UDP", 555, 5555, "")]
