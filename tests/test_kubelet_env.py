"""Container environment and `$(VAR)` expansion.

Reference: `third_party/forked/golang/expansion/expand_test.go` (TestMapping, TestMappingDual:
the full doExpansionTest table, with one and with two mapping contexts) and
`pkg/kubelet/kubelet_pods.go` makeEnvironmentVariables (envFrom prefixes, invalid keys skipped,
`$(VAR)` against earlier entries and the service variables, service variables never overriding).
"""
import base64

import pytest

from kubernetes_amd.kubelet.kubelet import expand

CTX = {"VAR_A": "A", "VAR_B": "B", "VAR_C": "C", "VAR_REF": "$(VAR_A)", "VAR_EMPTY": ""}
CTX1 = {"VAR_A": "A", "VAR_EMPTY": ""}
CTX2 = {"VAR_B": "B", "VAR_C": "C", "VAR_REF": "$(VAR_A)"}

CASES = [
    ("$(VAR_A)", "A"), ("$(VAR_A)-$(VAR_A)", "A-A"), ("$(VAR_A)-1", "A-1"), ("___$(VAR_B)___", "___B___"),
    ("___$(VAR_C)", "___C"), ("$(VAR_A)_$(VAR_B)_$(VAR_C)", "A_B_C"), ("$$(VAR_B)_$(VAR_A)", "$(VAR_B)_A"),
    ("$$(VAR_A)_$$(VAR_B)", "$(VAR_A)_$(VAR_B)"), ("f000-$$VAR_A", "f000-$VAR_A"),
    ("foo\\$(VAR_C)bar", "foo\\Cbar"), ("foo\\\\$(VAR_C)bar", "foo\\\\Cbar"),
    ("foo\\\\\\\\$(VAR_A)bar", "foo\\\\\\\\Abar"), ("$(VAR_A$(VAR_B))", "$(VAR_A$(VAR_B))"),
    ("$(VAR_A$(VAR_B)", "$(VAR_A$(VAR_B)"), ("$(VAR_REF)", "$(VAR_A)"),
    ("%%$(VAR_REF)--$(VAR_REF)%%", "%%$(VAR_A)--$(VAR_A)%%"), ("foo$(VAR_EMPTY)bar", "foobar"),
    ("foo$(VAR_Awhoops!", "foo$(VAR_Awhoops!"), ("f00__(VAR_A)__", "f00__(VAR_A)__"), ("$?_boo_$!", "$?_boo_$!"),
    ("$VAR_A", "$VAR_A"), ("$(VAR_DNE)", "$(VAR_DNE)"), ("$$$$$$(BIG_MONEY)", "$$$(BIG_MONEY)"),
    ("$$$$$$(VAR_A)", "$$$(VAR_A)"), ("$$$$$$$(GOOD_ODDS)", "$$$$(GOOD_ODDS)"), ("$$$$$$$(VAR_A)", "$$$A"),
    ("$VAR_A)", "$VAR_A)"), ("${VAR_A}", "${VAR_A}"), ("$(VAR_B)_______$(A", "B_______$(A"),
    ("$(VAR_C)_______$(", "C_______$("), ("$(VAR_A)foobarzab$", "Afoobarzab$"), ("foo-\\$(VAR_A", "foo-\\$(VAR_A"),
    ("--$($($($($--", "--$($($($($--"), ("$($($($($--foo$(", "$($($($($--foo$("), ("foo0--$($($($(", "foo0--$($($($("),
    ("$(foo$$var)", "$(foo$$var)"), ("\n", "\n"),
]


@pytest.mark.parametrize("inp,want", CASES, ids=[repr(c[0]) for c in CASES])
def test_mapping(inp, want):
    assert expand(inp, CTX) == want


@pytest.mark.parametrize("inp,want", CASES, ids=[repr(c[0]) for c in CASES])
def test_mapping_dual(inp, want):
    assert expand(inp, CTX1, CTX2) == want


def test_make_environment_variables(run, tmp_path):
    from kubernetes_amd.kubelet.volumes import VolumeManager

    class FakeClient:
        objs = {("configmaps", "ns", "cm"): {"data": {"A": "1", "B": "2", "1bad": "x", "ok.dotted": "3"}},
                ("secrets", "ns", "sec"): {"data": {"S": base64.b64encode(b"s3cr3t").decode()}}}

        async def get(self, resource, name, namespace=None):
            return self.objs[(resource, namespace, name)]

    vm = VolumeManager.__new__(VolumeManager)
    vm.client = FakeClient()
    vm.host_ip = "10.0.0.1"
    vm.allocatable = {}

    async def _get(resource, ns, name, optional=None):
        return FakeClient.objs.get((resource, ns, name))
    vm._get = _get
    pod = {"metadata": {"name": "p", "namespace": "ns", "uid": "u"}, "spec": {}}
    ctr = {"name": "c", "envFrom": [{"configMapRef": {"name": "cm"}, "prefix": "P_"}, {"secretRef": {"name": "sec"}}],
           "env": [{"name": "X", "value": "$(P_A)-$(SVC_HOST)-$(MISSING)"}, {"name": "SVC_PORT", "value": "override"}]}
    base = [{"name": "SVC_HOST", "value": "10.1.1.1"}, {"name": "SVC_PORT", "value": "80"}]

    async def main():
        return await vm.env_for(pod, ctr, "node", "1.2.3.4", base_env=base)
    env = {e["name"]: e["value"] for e in run(main())}
    assert env["P_A"] == "1" and env["P_B"] == "2" and env["S"] == "s3cr3t" and env["P_ok.dotted"] == "3"
    assert "P_1bad" in env             # prefixed, the key becomes a valid name
    assert env["X"] == "1-10.1.1.1-$(MISSING)"
    assert env["SVC_PORT"] == "override" and env["SVC_HOST"] == "10.1.1.1"
    ctr2 = {"name": "c", "envFrom": [{"configMapRef": {"name": "cm"}}]}

    async def main2():
        return await vm.env_for(pod, ctr2)
    env2 = {e["name"]: e["value"] for e in run(main2())}
    assert "1bad" not in env2 and env2["A"] == "1"     # an invalid name is skipped, not fatal


def test_from_services():
    """envvars_test.go TestFromServices: the docker-link style variables, IPv6 bracketed in URLs,
    headless / IP-less services skipped."""
    from kubernetes_amd.kubelet.envvars import from_services

    def svc(name, ip, *ports):
        return {"metadata": {"name": name}, "spec": {"clusterIP": ip, "ports": [
            dict({"port": p, "protocol": proto}, **({"name": n} if n else {})) for n, p, proto in ports]}}
    services = [svc("foo-bar", "1.2.3.4", (None, 8080, "TCP")),
                svc("abc-123", "5.6.7.8", ("u-d-p", 8081, "UDP"), ("t-c-p", 8081, "TCP")),
                svc("q-u-u-x", "9.8.7.6", (None, 8082, "TCP"), ("8083", 8083, "TCP")),
                svc("svrc-clusterip-none", "None", (None, 8082, "TCP")),
                svc("svrc-clusterip-empty", "", (None, 8082, "TCP")),
                svc("super-ipv6", "2001:DB8::", ("u-d-p", 8084, "UDP"), ("t-c-p", 8084, "TCP"))]
    got = [(e["name"], e["value"]) for e in from_services(services)]
    want = [
        ("FOO_BAR_SERVICE_HOST", "1.2.3.4"), ("FOO_BAR_SERVICE_PORT", "8080"), ("FOO_BAR_PORT", "tcp://1.2.3.4:8080"),
        ("FOO_BAR_PORT_8080_TCP", "tcp://1.2.3.4:8080"), ("FOO_BAR_PORT_8080_TCP_PROTO", "tcp"),
        ("FOO_BAR_PORT_8080_TCP_PORT", "8080"), ("FOO_BAR_PORT_8080_TCP_ADDR", "1.2.3.4"),
        ("ABC_123_SERVICE_HOST", "5.6.7.8"), ("ABC_123_SERVICE_PORT", "8081"), ("ABC_123_SERVICE_PORT_U_D_P", "8081"),
        ("ABC_123_SERVICE_PORT_T_C_P", "8081"), ("ABC_123_PORT", "udp://5.6.7.8:8081"),
        ("ABC_123_PORT_8081_UDP", "udp://5.6.7.8:8081"), ("ABC_123_PORT_8081_UDP_PROTO", "udp"),
        ("ABC_123_PORT_8081_UDP_PORT", "8081"), ("ABC_123_PORT_8081_UDP_ADDR", "5.6.7.8"),
        ("ABC_123_PORT_8081_TCP", "tcp://5.6.7.8:8081"), ("ABC_123_PORT_8081_TCP_PROTO", "tcp"),
        ("ABC_123_PORT_8081_TCP_PORT", "8081"), ("ABC_123_PORT_8081_TCP_ADDR", "5.6.7.8"),
        ("Q_U_U_X_SERVICE_HOST", "9.8.7.6"), ("Q_U_U_X_SERVICE_PORT", "8082"), ("Q_U_U_X_SERVICE_PORT_8083", "8083"),
        ("Q_U_U_X_PORT", "tcp://9.8.7.6:8082"), ("Q_U_U_X_PORT_8082_TCP", "tcp://9.8.7.6:8082"),
        ("Q_U_U_X_PORT_8082_TCP_PROTO", "tcp"), ("Q_U_U_X_PORT_8082_TCP_PORT", "8082"),
        ("Q_U_U_X_PORT_8082_TCP_ADDR", "9.8.7.6"), ("Q_U_U_X_PORT_8083_TCP", "tcp://9.8.7.6:8083"),
        ("Q_U_U_X_PORT_8083_TCP_PROTO", "tcp"), ("Q_U_U_X_PORT_8083_TCP_PORT", "8083"),
        ("Q_U_U_X_PORT_8083_TCP_ADDR", "9.8.7.6"),
        ("SUPER_IPV6_SERVICE_HOST", "2001:DB8::"), ("SUPER_IPV6_SERVICE_PORT", "8084"),
        ("SUPER_IPV6_SERVICE_PORT_U_D_P", "8084"), ("SUPER_IPV6_SERVICE_PORT_T_C_P", "8084"),
        ("SUPER_IPV6_PORT", "udp://[2001:DB8::]:8084"), ("SUPER_IPV6_PORT_8084_UDP", "udp://[2001:DB8::]:8084"),
        ("SUPER_IPV6_PORT_8084_UDP_PROTO", "udp"), ("SUPER_IPV6_PORT_8084_UDP_PORT", "8084"),
        ("SUPER_IPV6_PORT_8084_UDP_ADDR", "2001:DB8::"), ("SUPER_IPV6_PORT_8084_TCP", "tcp://[2001:DB8::]:8084"),
        ("SUPER_IPV6_PORT_8084_TCP_PROTO", "tcp"), ("SUPER_IPV6_PORT_8084_TCP_PORT", "8084"),
        ("SUPER_IPV6_PORT_8084_TCP_ADDR", "2001:DB8::"),
    ]
    assert got == want


# -- pkg/kubelet/kubelet_pods_test.go TestMakeEnvironmentVariables: the service cases -------------
def _svc(name, ns, ip, port):
    return {"metadata": {"name": name, "namespace": ns}, "spec": {"clusterIP": ip, "ports": [{"protocol": "TCP",
                                                                                              "port": port}]}}


MEV_SERVICES = [_svc("kubernetes", "default", "1.2.3.1", 8081), _svc("test", "test1", "1.2.3.3", 8083),
                _svc("kubernetes", "test2", "1.2.3.4", 8084), _svc("test", "test2", "1.2.3.5", 8085),
                _svc("test", "test2", "None", 8085), _svc("test", "test2", "", 8085),
                _svc("kubernetes", "kubernetes", "1.2.3.6", 8086), _svc("not-special", "kubernetes", "1.2.3.8", 8088),
                _svc("not-special", "kubernetes", "None", 8088), _svc("not-special", "kubernetes", "", 8088)]


def _svc_vars(prefix, ip, port):
    return {f"{prefix}_SERVICE_HOST": ip, f"{prefix}_SERVICE_PORT": str(port), f"{prefix}_PORT": f"tcp://{ip}:{port}",
            f"{prefix}_PORT_{port}_TCP": f"tcp://{ip}:{port}", f"{prefix}_PORT_{port}_TCP_PROTO": "tcp",
            f"{prefix}_PORT_{port}_TCP_PORT": str(port), f"{prefix}_PORT_{port}_TCP_ADDR": ip}


@pytest.mark.parametrize("ns,master_ns,want", [
    ("test1", "default", {**_svc_vars("TEST", "1.2.3.3", 8083), **_svc_vars("KUBERNETES", "1.2.3.1", 8081)}),
    # master service in pod ns: the namespace's own "kubernetes" wins over the master one
    ("test2", "kubernetes", {**_svc_vars("TEST", "1.2.3.5", 8085), **_svc_vars("KUBERNETES", "1.2.3.4", 8084)}),
    # pod in master service ns: every service there, with the master kubernetes service
    ("kubernetes", "kubernetes", {**_svc_vars("NOT_SPECIAL", "1.2.3.8", 8088), **_svc_vars("KUBERNETES", "1.2.3.6", 8086)}),
    ("downward-api", "nothing", {}),
])
def test_make_environment_variables_services(ns, master_ns, want):
    from kubernetes_amd.kubelet.envvars import service_env
    got = {e["name"]: e["value"] for e in service_env(MEV_SERVICES, ns, master_ns)}
    assert got == want


def test_make_environment_variables_missing_keys_and_invalid_names(run):
    """configmapkeyref / secretkeyref with missing keys (optional or not), envFrom with invalid
    key names reported by an InvalidEnvironmentVariableNames event."""
    import base64

    from kubernetes_amd.kubelet.volumes import VolumeError, VolumeManager

    class FakeClient:
        objs = {("configmaps", "ns", "cm"): {"data": {"REAL": "1", "1bad": "x", "also bad": "y"}},
                ("secrets", "ns", "sec"): {"data": {"S": base64.b64encode(b"s3").decode()}}}

        async def get(self, kind, name, ns=None, **kw):
            from kubernetes_amd.client.rest import APIStatusError
            o = self.objs.get((kind, ns, name))
            if o is None:
                raise APIStatusError(404, {"reason": "NotFound", "message": f"{kind} {name} not found"})
            return o

    events = []
    vm = VolumeManager(FakeClient(), "/tmp/unused")
    vm.recorder = lambda obj, t, r, m: events.append((t, r, m))
    pod = {"metadata": {"name": "p", "namespace": "ns"}, "spec": {}}

    async def main():
        env = await vm.env_for(pod, {"envFrom": [{"configMapRef": {"name": "cm"}}]})
        assert env == [{"name": "REAL", "value": "1"}]
        assert events == [("Warning", "InvalidEnvironmentVariableNames",
                           "Keys [1bad, also bad] from the EnvFrom configMap ns/cm were skipped since they are "
                           "considered invalid environment variable names.")]
        optional = {"env": [{"name": "A", "valueFrom": {"configMapKeyRef": {"name": "cm", "key": "nope", "optional": True}}},
                            {"name": "B", "valueFrom": {"secretKeyRef": {"name": "sec", "key": "nope", "optional": True}}},
                            {"name": "C", "valueFrom": {"configMapKeyRef": {"name": "gone", "key": "k", "optional": True}}}]}
        assert await vm.env_for(pod, optional) == []
        with pytest.raises(VolumeError, match="Couldn't find key nope in ConfigMap ns/cm"):
            await vm.env_for(pod, {"env": [{"name": "A", "valueFrom": {"configMapKeyRef": {"name": "cm", "key": "nope"}}}]})
        with pytest.raises(VolumeError, match="Couldn't find key nope in Secret ns/sec"):
            await vm.env_for(pod, {"env": [{"name": "A", "valueFrom": {"secretKeyRef": {"name": "sec", "key": "nope"}}}]})
    run(main())
