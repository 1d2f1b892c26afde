"""Pod DNS ported from `pkg/kubelet/network/dns/dns_test.go` (TestParseResolvConf,
TestFormDNSSearchFitsLimits, TestFormDNSNameserversFitsLimits, TestMergeDNSOptions,
TestGetPodDNSType, TestGetPodDNS, TestGetPodDNSCustom) plus the API validation of
dnsPolicy None / dnsConfig behind the CustomPodDNS gate."""
import pytest

from kubernetes_amd.kubelet import network as net

PARSE = [
    ("", [], [], []), (" ", [], [], []), ("\n", [], [], []), ("\t\n\t", [], [], []),
    ("#comment\n", [], [], []), (" #comment\n", [], [], []), ("#comment\n#comment", [], [], []),
    ("#comment\nnameserver", [], [], []), ("#comment\nnameserver\nsearch", [], [], []),
    ("nameserver 1.2.3.4", ["1.2.3.4"], [], []), (" nameserver 1.2.3.4", ["1.2.3.4"], [], []),
    ("\tnameserver 1.2.3.4", ["1.2.3.4"], [], []), ("nameserver\t1.2.3.4", ["1.2.3.4"], [], []),
    ("nameserver \t 1.2.3.4", ["1.2.3.4"], [], []),
    ("nameserver 1.2.3.4\nnameserver 5.6.7.8", ["1.2.3.4", "5.6.7.8"], [], []),
    ("nameserver 1.2.3.4 #comment", ["1.2.3.4"], [], []),
    ("search foo", [], ["foo"], []), ("search foo bar", [], ["foo", "bar"], []),
    ("search foo bar bat\n", [], ["foo", "bar", "bat"], []), ("search foo\nsearch bar", [], ["bar"], []),
    ("nameserver 1.2.3.4\nsearch foo bar", ["1.2.3.4"], ["foo", "bar"], []),
    ("nameserver 1.2.3.4\nsearch foo\nnameserver 5.6.7.8\nsearch bar", ["1.2.3.4", "5.6.7.8"], ["bar"], []),
    ("#comment\nnameserver 1.2.3.4\n#comment\nsearch foo\ncomment", ["1.2.3.4"], ["foo"], []),
    ("options ndots:5 attempts:2", [], [], ["ndots:5", "attempts:2"]),
    ("options ndots:1\noptions ndots:5 attempts:3", [], [], ["ndots:5", "attempts:3"]),
    ("nameserver 1.2.3.4\nsearch foo\nnameserver 5.6.7.8\nsearch bar\noptions ndots:5 attempts:4",
     ["1.2.3.4", "5.6.7.8"], ["bar"], ["ndots:5", "attempts:4"]),
]


@pytest.mark.parametrize("data,ns,search,opts", PARSE)
def test_parse_resolv_conf(data, ns, search, opts):
    assert net.parse_resolv_conf_text(data) == (ns, search, opts)


def configurer(cluster_dns=(), domain="TEST", resolv=""):
    events = []
    c = net.DNSConfigurer(list(cluster_dns), domain, resolv, recorder=lambda obj, t, r, m: events.append((t, r, m)),
                          node_ref={"kind": "Node", "metadata": {"name": "testNode"}})
    return c, events


POD = {"metadata": {"name": "test_pod", "namespace": "testNS", "uid": ""}, "spec": {}}


@pytest.mark.parametrize("names,want,event", [
    (["testNS.svc.TEST", "svc.TEST", "TEST"], ["testNS.svc.TEST", "svc.TEST", "TEST"], None),
    (["testNS.svc.TEST", "svc.TEST", "TEST", "AAA", "BBB"], ["testNS.svc.TEST", "svc.TEST", "TEST", "AAA", "BBB"], None),
    (["testNS.svc.TEST", "svc.TEST", "TEST", "AAA", "B" * 256, "BBB"], ["testNS.svc.TEST", "svc.TEST", "TEST", "AAA"],
     "Search Line limits were exceeded, some search paths have been omitted, the applied search line is: "
     "testNS.svc.TEST svc.TEST TEST AAA"),
    (["testNS.svc.TEST", "svc.TEST", "TEST", "AAA", "BBB", "CCC", "DDD"],
     ["testNS.svc.TEST", "svc.TEST", "TEST", "AAA", "BBB", "CCC"],
     "Search Line limits were exceeded, some search paths have been omitted, the applied search line is: "
     "testNS.svc.TEST svc.TEST TEST AAA BBB CCC"),
])
def test_form_dns_search_fits_limits(names, want, event):
    c, events = configurer()
    assert c.form_dns_search_fits_limits(names, POD) == want
    assert events == ([("Warning", "DNSConfigForming", event)] if event else [])


@pytest.mark.parametrize("ns,want,event", [
    (["127.0.0.1"], ["127.0.0.1"], False),
    (["127.0.0.1", "10.0.0.10", "8.8.8.8"], ["127.0.0.1", "10.0.0.10", "8.8.8.8"], False),
    (["127.0.0.1", "10.0.0.10", "8.8.8.8", "1.2.3.4"], ["127.0.0.1", "10.0.0.10", "8.8.8.8"], True),
])
def test_form_dns_nameservers_fits_limits(ns, want, event):
    c, events = configurer()
    assert c.form_dns_nameservers_fits_limits(ns, POD) == want
    assert bool(events) == event


@pytest.mark.parametrize("existing,options,want", [
    (["ndots:5", "debug"], None, ["ndots:5", "debug"]),
    (["ndots:5", "debug"], [{"name": "single-request"}, {"name": "attempts", "value": "3"}],
     ["ndots:5", "debug", "single-request", "attempts:3"]),
    (["ndots:5", "debug"], [{"name": "ndots", "value": "3"}, {"name": "debug"}, {"name": "single-request"},
                            {"name": "attempts", "value": "3"}], ["ndots:3", "debug", "single-request", "attempts:3"]),
])
def test_merge_dns_options(existing, options, want):
    assert sorted(net.merge_dns_options(existing, options)) == sorted(want)


@pytest.mark.parametrize("gate,host_net,policy,want,err", [
    (False, False, "ClusterFirst", net.POD_DNS_CLUSTER, False),
    (False, True, "ClusterFirstWithHostNet", net.POD_DNS_CLUSTER, False),
    (False, False, "ClusterFirstWithHostNet", net.POD_DNS_CLUSTER, False),
    (False, False, "Default", net.POD_DNS_HOST, False),
    (False, True, "Default", net.POD_DNS_HOST, False),
    (False, True, "ClusterFirst", net.POD_DNS_HOST, False),
    (True, False, "None", net.POD_DNS_NONE, False),
    (False, False, "None", None, True),
    (False, False, "invalidPolicy", None, True),
])
def test_get_pod_dns_type(feature_gate, gate, host_net, policy, want, err):
    feature_gate.set(f"CustomPodDNS={str(gate).lower()}")
    typ, e = net.get_pod_dns_type({"metadata": {}, "spec": {"dnsPolicy": policy, "hostNetwork": host_net}})
    assert bool(e) == err
    if not err:
        assert typ == want


def pods4():
    pods = [{"metadata": {"name": f"pod{i}", "uid": str(10000 + i)}, "spec": {"hostNetwork": True}} for i in range(4)]
    pods[0]["spec"]["dnsPolicy"] = "ClusterFirstWithHostNet"
    pods[1]["spec"]["dnsPolicy"] = "ClusterFirst"
    pods[2]["spec"]["dnsPolicy"] = "ClusterFirst"
    pods[2]["spec"]["hostNetwork"] = False
    pods[3]["spec"]["dnsPolicy"] = "Default"
    return pods


def test_get_pod_dns(tmp_path):
    cluster_ns = "203.0.113.1"
    c, _ = configurer([cluster_ns], "kubernetes.io", "")
    out = [c.pod_dns(p) for p in pods4()]
    assert out[0][0] == [cluster_ns] and out[0][1][0] == ".svc.kubernetes.io"
    assert out[1][0] == ["127.0.0.1"] and out[1][1] == ["."]           # no resolv.conf: localhost, "."
    assert out[2][0] == [cluster_ns] and out[2][1][0] == ".svc.kubernetes.io"
    assert out[3][0] == ["127.0.0.1"] and out[3][1] == ["."]
    rc = tmp_path / "resolv.conf"
    rc.write_text("nameserver 192.0.2.53\nsearch a.example b.example c.example d.example\n")
    c, _ = configurer([cluster_ns], "kubernetes.io", str(rc))
    out = [c.pod_dns(p) for p in pods4()]
    assert out[0][0] == [cluster_ns]
    exp = min(len(out[1][1]) + 3, 6)
    assert len(out[0][1]) == exp and out[0][1][0] == ".svc.kubernetes.io"
    assert out[2][0] == [cluster_ns] and len(out[2][1]) == exp
    assert out[1][0] == ["192.0.2.53"]


def test_ipv6_node_without_resolv_conf_uses_ipv6_loopback():
    c, _ = configurer([], "kubernetes.io", "")
    c.node_ip = "fd00::1"
    assert c.pod_dns({"metadata": {"name": "p"}, "spec": {"dnsPolicy": "Default"}})[:2] == (["::1"], ["."])


def test_missing_cluster_dns_falls_back_with_events():
    c, events = configurer([], "kubernetes.io", "")
    ns, search, _ = c.pod_dns({"metadata": {"name": "p", "namespace": "d", "uid": "u"}, "spec": {"dnsPolicy": "ClusterFirst"}})
    assert (ns, search) == (["127.0.0.1"], ["."])
    assert [e[1] for e in events] == ["MissingClusterDNS", "MissingClusterDNS"]


def test_get_pod_dns_custom(feature_gate):
    cluster_ns = "203.0.113.1"
    c, _ = configurer([cluster_ns], "kubernetes.io", "")
    pod = {"metadata": {"name": "test_pod", "namespace": "testNS"}, "spec": {"dnsPolicy": "ClusterFirst"}}
    cluster_first = c.pod_dns(pod)
    pod["spec"]["dnsPolicy"] = "None"
    # gate disabled: None falls back to ClusterFirst
    feature_gate.set("CustomPodDNS=false")
    assert c.pod_dns(pod) == cluster_first
    feature_gate.set("CustomPodDNS=true")
    assert c.pod_dns(pod) == ([], [], [])
    pod["spec"]["dnsConfig"] = {"nameservers": ["10.0.0.10"], "searches": ["my.domain", "second.domain"],
                                "options": [{"name": "ndots", "value": "3"}, {"name": "debug"}]}
    ns, search, opts = c.pod_dns(pod)
    assert ns == ["10.0.0.10"] and search == ["my.domain", "second.domain"] and sorted(opts) == ["debug", "ndots:3"]


def test_check_limits_for_resolv_conf(tmp_path):
    rc = tmp_path / "resolv.conf"
    rc.write_text("search " + " ".join(f"d{i}.example" for i in range(4)) + "\n")
    c, events = configurer([], "cluster.local", str(rc))
    c.check_limits_for_resolv_conf()
    assert events and "more than 3 domains" in events[0][2]
    events.clear()
    c, events = configurer([], "", str(rc))
    c.check_limits_for_resolv_conf()
    assert events == []
    c, events = configurer([], "", str(tmp_path / "missing"))
    c.check_limits_for_resolv_conf()
    assert events[0][1] == "CheckLimitsForResolvConf"


def _spec(**kw):
    return {"containers": [{"name": "c", "image": "busybox"}], "restartPolicy": "Always", **kw}


@pytest.mark.parametrize("gate,spec,want", [
    (False, _spec(dnsPolicy="None", dnsConfig={"nameservers": ["1.1.1.1"]}), ["can not use 'None'", "Forbidden"]),
    (False, _spec(dnsPolicy="ClusterFirst"), []),
    (True, _spec(dnsPolicy="None"), ["must provide `dnsConfig`"]),
    (True, _spec(dnsPolicy="None", dnsConfig={}), ["must provide at least one DNS nameserver"]),
    (True, _spec(dnsPolicy="None", dnsConfig={"nameservers": ["1.1.1.1"]}), []),
    (True, _spec(dnsPolicy="ClusterFirst", dnsConfig={"nameservers": ["1.1.1.1", "2.2.2.2", "3.3.3.3", "4.4.4.4"]}),
     ["must not have more than 3 nameservers"]),
    (True, _spec(dnsPolicy="ClusterFirst", dnsConfig={"nameservers": ["not-an-ip"]}), ["must be valid IP address"]),
    (True, _spec(dnsPolicy="ClusterFirst", dnsConfig={"searches": [f"s{i}" for i in range(7)]}),
     ["must not have more than 6 search paths"]),
    (True, _spec(dnsPolicy="ClusterFirst", dnsConfig={"searches": ["Bad_Domain"]}), ["DNS-1123 subdomain"]),
    (True, _spec(dnsPolicy="ClusterFirst", dnsConfig={"options": [{"value": "1"}]}), ["must not be empty"]),
    (True, _spec(dnsPolicy="bogus"), ["Unsupported value"]),
])
def test_validate_pod_dns(feature_gate, gate, spec, want):
    from kubernetes_amd.api.validation import validate_pod_spec
    feature_gate.set(f"CustomPodDNS={str(gate).lower()}")
    errs = [str(e) for e in validate_pod_spec(spec, "spec") if "dns" in str(e).lower()]
    for w in want:
        assert any(w in e for e in errs), (w, errs)
    if not want:
        assert errs == []


# -- pkg/kubelet/kubelet_pods_test.go: hosts files and hostnames ------------------------------------
HEADER = ("127.0.0.1\tlocalhost\n::1\tlocalhost ip6-localhost ip6-loopback\nfe00::0\tip6-localnet\n"
          "fe00::0\tip6-mcastprefix\nfe00::1\tip6-allnodes\nfe00::2\tip6-allrouters\n")
ALIASES1 = [{"ip": "123.45.67.89", "hostnames": ["foo", "bar", "baz"]}]
ALIASES2 = ALIASES1 + [{"ip": "456.78.90.123", "hostnames": ["park", "doo", "boo"]}]
ALIAS_TEXT1 = "\n# Entries added by HostAliases.\n123.45.67.89\tfoo\n123.45.67.89\tbar\n123.45.67.89\tbaz\n"
ALIAS_TEXT2 = ALIAS_TEXT1 + "456.78.90.123\tpark\n456.78.90.123\tdoo\n456.78.90.123\tboo\n"


@pytest.mark.parametrize("raw,aliases,want_tail", [
    ("# hosts file for testing.\n" + HEADER + "123.45.67.89\tsome.domain\n", [], ""),
    ("# another hosts file for testing.\n" + HEADER + "12.34.56.78\tanother.domain\n", [], ""),
    ("# hosts file for testing.\n" + HEADER + "123.45.67.89\tsome.domain\n", ALIASES1, ALIAS_TEXT1),
    ("# another hosts file for testing.\n" + HEADER + "12.34.56.78\tanother.domain\n", ALIASES2, ALIAS_TEXT2),
])
def test_node_hosts_file_content(tmp_path, raw, aliases, want_tail):
    f = tmp_path / "hosts"
    f.write_text(raw)
    assert net.node_hosts_file_content(str(f), aliases) == raw + want_tail


@pytest.mark.parametrize("ip,host,domain,aliases,entry,tail", [
    ("123.45.67.89", "podFoo", "", [], "123.45.67.89\tpodFoo\n", ""),
    ("203.0.113.1", "podFoo", "domainFoo", [], "203.0.113.1\tpodFoo.domainFoo\tpodFoo\n", ""),
    ("203.0.113.1", "podFoo", "domainFoo", ALIASES1, "203.0.113.1\tpodFoo.domainFoo\tpodFoo\n", ALIAS_TEXT1),
    ("203.0.113.1", "podFoo", "domainFoo", ALIASES2, "203.0.113.1\tpodFoo.domainFoo\tpodFoo\n", ALIAS_TEXT2),
])
def test_managed_hosts_file_content(ip, host, domain, aliases, entry, tail):
    assert net.managed_hosts_file_content(ip, host, domain, aliases) == \
        "# Kubernetes-managed hosts file.\n" + HEADER + entry + tail


@pytest.mark.parametrize("inp,out", [
    ("test.pod.hostname", "test.pod.hostname"),
    ("1234567." * 9, "1234567." * 7 + "1234567"),
    ("1234567." * 7 + "123456.1234567.", "1234567." * 7 + "123456"),
    ("1234567." * 7 + "123456-1234567.", "1234567." * 7 + "123456"),
])
def test_truncate_pod_hostname(inp, out):
    assert net.truncate_pod_hostname("test-pod", inp) == out


def test_generate_pod_hostname_and_domain():
    p = {"metadata": {"name": "web-0", "namespace": "ml"}, "spec": {"hostname": "w0", "subdomain": "workers"}}
    assert net.generate_pod_hostname_and_domain(p, "cluster.local") == ("w0", "workers.ml.svc.cluster.local")
    assert net.generate_pod_hostname_and_domain({"metadata": {"name": "x"}, "spec": {}}, "c") == ("x", "")
    with pytest.raises(ValueError, match="not a valid DNS label"):
        net.generate_pod_hostname_and_domain({"metadata": {"name": "x"}, "spec": {"hostname": "Bad_Name"}}, "c")


def test_host_network_pod_gets_node_hosts_plus_aliases(tmp_path, monkeypatch):
    node_hosts = tmp_path / "node-hosts"
    node_hosts.write_text("127.0.0.1\tlocalhost\n10.0.0.5\tnode-a\n")
    monkeypatch.setattr(net, "ETC_HOSTS_PATH", str(node_hosts))
    d = net.DNSConfigurer([], "cluster.local", "")
    pod = {"metadata": {"name": "h", "namespace": "d"}, "spec": {"hostNetwork": True, "hostAliases": ALIASES1}}
    mounts = d.write_pod_files(str(tmp_path / "pod"), pod, "10.0.0.5", hosts_only=True)
    assert mounts[0]["containerPath"] == "/etc/hosts"
    assert (tmp_path / "pod" / "etc-hosts").read_text() == node_hosts.read_text() + ALIAS_TEXT1


# -- pkg/kubelet/kubelet_network_test.go TestNodeIPParam -------------------------------------------
@pytest.mark.parametrize("ip,msg", [
    ("", "must be a valid IP address"), ("127.0.0.1", "loopback"), ("::1", "loopback"),
    ("224.0.0.1", "multicast"), ("ff00::1", "multicast"), ("169.254.0.1", "link-local"),
    ("fe80::0202:b3ff:fe1e:8329", "link-local"), ("0.0.0.0", "all zeros"), ("::", "all zeros"),
    ("1.2.3.4", "not found in the host's network interfaces"),
])
def test_node_ip_param_rejected(ip, msg):
    with pytest.raises(ValueError, match=msg):
        net.validate_node_ip(ip, host_addrs={"10.0.0.5", "fd00::2"})


def test_node_ip_param_host_addresses_accepted():
    usable = [a for a in net.host_ip_addresses() if not a.startswith(("127.", "::1", "fe80"))]
    for a in usable:
        net.validate_node_ip(a)
    net.validate_node_ip("10.0.0.5", host_addrs={"10.0.0.5"})
