"""PodSecurityPolicy providers and plugin: ported tables.

Reference: `pkg/security/podsecuritypolicy/provider_test.go` (TestValidatePodSecurityContextFailures
:174, TestValidateContainerSecurityContextFailures :405, TestValidatePodSecurityContextSuccess
:548, TestCreate*SecurityContextNonmutating, TestGenerateContainerSecurityContextReadOnlyRootFS,
TestValidateAllowPrivilegeEscalation) and `plugin/pkg/admission/security/podsecuritypolicy/
admission_test.go` (TestAdmitPreferNonmutating, TestPolicyAuthorization, TestAdmitCaps, ...).
Pods are v1 dicts, so the reference's `SecurityContext.HostNetwork` is `spec.hostNetwork`.
"""
import copy

import pytest

from kubernetes_amd.apiserver.admission import CREATE, UPDATE, AdmissionError, Attributes
from kubernetes_amd.apiserver.admission.psp import Provider, ProviderError, has_path_prefix
from kubernetes_amd.apiserver.admission.security import PodSecurityPolicy
from kubernetes_amd.apiserver.auth import User


def default_psp(name="psp-sa", annotations=None, **spec):
    base = {"runAsUser": {"rule": "RunAsAny"}, "seLinux": {"rule": "RunAsAny"}, "fsGroup": {"rule": "RunAsAny"},
            "supplementalGroups": {"rule": "RunAsAny"}, "allowPrivilegeEscalation": True}
    base.update(spec)
    return {"metadata": {"name": name, "annotations": dict(annotations or {})}, "spec": base}


def default_pod(annotations=None, **spec):
    base = {"securityContext": {}, "containers": [{"name": "defaultContainerName",
                                                   "securityContext": {"privileged": False}}]}
    base.update(spec)
    return {"metadata": {"annotations": dict(annotations or {})}, "spec": base}


def with_ctr_sc(pod, **sc):
    pod["spec"]["containers"][0]["securityContext"].update(sc)
    return pod


def flex_psp(allow_all_flex, allow_all_volumes):
    return default_psp(allowedFlexVolumes=[] if allow_all_flex else [{"driver": "example/foo"},
                                                                     {"driver": "example/bar"}],
                       volumes=["*" if allow_all_volumes else "flexVolume"])


FLEX_BAD = default_pod(volumes=[{"name": "flex-volume", "flexVolume": {"driver": "example/unknown"}}])
FLEX_OK = default_pod(volumes=[{"name": "flex-volume", "flexVolume": {"driver": "example/bar"}}])
SUP_PSP = default_psp(supplementalGroups={"rule": "MustRunAs", "ranges": [{"min": 1, "max": 1}]})
FS_PSP = default_psp(fsGroup={"rule": "MustRunAs", "ranges": [{"min": 1, "max": 1}]})
SEL_PSP = default_psp(seLinux={"rule": "MustRunAs", "seLinuxOptions": {"level": "foo"}})

POD_FAILURES = [
    ("failHostNetwork", default_pod(hostNetwork=True), default_psp(), "Host network is not allowed to be used"),
    ("failHostPID", default_pod(hostPID=True), default_psp(), "Host PID is not allowed to be used"),
    ("failHostIPC", default_pod(hostIPC=True), default_psp(), "Host IPC is not allowed to be used"),
    ("failSupplementalGroupOutOfRange", default_pod(securityContext={"supplementalGroups": [999]}), SUP_PSP,
     "999 is not an allowed group"),
    ("failSupplementalGroupEmpty", default_pod(), SUP_PSP, "unable to validate empty groups against required ranges"),
    ("failFSGroupOutOfRange", default_pod(securityContext={"fsGroup": 999}), FS_PSP, "999 is not an allowed group"),
    ("failFSGroupEmpty", default_pod(), FS_PSP, "unable to validate empty groups against required ranges"),
    ("failNilSELinux", default_pod(), SEL_PSP, "seLinuxOptions: Required"),
    ("failInvalidSELinux", default_pod(securityContext={"seLinuxOptions": {"level": "bar"}}), SEL_PSP,
     "seLinuxOptions.level: Invalid value"),
    ("failHostDirPSP", default_pod(volumes=[{"name": "bad volume", "hostPath": {}}]), default_psp(),
     "hostPath volumes are not allowed to be used"),
    ("failHostPathDirPSP", default_pod(volumes=[{"name": "bad volume", "hostPath": {"path": "/fail"}}]),
     default_psp(volumes=["hostPath"], allowedHostPaths=[{"pathPrefix": "/foo/bar"}]), "is not allowed to be used"),
    ("failSafeSysctlFooPod with failNoSysctlAllowedSCC",
     default_pod({"security.alpha.kubernetes.io/sysctls": "foo=1"}),
     default_psp(annotations={"security.alpha.kubernetes.io/sysctls": ""}), "sysctls are not allowed"),
    ("failUnsafeSysctlFooPod with failNoSysctlAllowedSCC",
     default_pod({"security.alpha.kubernetes.io/unsafe-sysctls": "foo=1"}),
     default_psp(annotations={"security.alpha.kubernetes.io/sysctls": ""}), "sysctls are not allowed"),
    ("failSafeSysctlFooPod with failOtherSysctlsAllowedSCC",
     default_pod({"security.alpha.kubernetes.io/sysctls": "foo=1"}),
     default_psp(annotations={"security.alpha.kubernetes.io/sysctls": "bar,abc"}), 'sysctl "foo" is not allowed'),
    ("failUnsafeSysctlFooPod with failOtherSysctlsAllowedSCC",
     default_pod({"security.alpha.kubernetes.io/unsafe-sysctls": "foo=1"}),
     default_psp(annotations={"security.alpha.kubernetes.io/sysctls": "bar,abc"}), 'sysctl "foo" is not allowed'),
    ("failInvalidSeccomp", default_pod({"seccomp.security.alpha.kubernetes.io/pod": "foo"}), default_psp(),
     "Forbidden: seccomp may not be set"),
    ("disallowed flexVolume when flex volumes are allowed", FLEX_BAD, flex_psp(False, False),
     "Flexvolume driver is not allowed to be used"),
    ("disallowed flexVolume when all volumes are allowed", FLEX_BAD, flex_psp(False, True),
     "Flexvolume driver is not allowed to be used"),
]


@pytest.mark.parametrize("name,pod,psp,expected", POD_FAILURES, ids=[c[0] for c in POD_FAILURES])
def test_validate_pod_security_context_failures(name, pod, psp, expected):
    errs = Provider(psp).validate_pod_security_context(pod)
    assert errs and expected in errs[0], errs


CTR = "defaultContainerName"
APPARMOR_PSP = default_psp(annotations={"apparmor.security.beta.kubernetes.io/allowedProfileNames": "runtime/default"})
CONTAINER_FAILURES = [
    ("failUserPSP", with_ctr_sc(default_pod(), runAsUser=1),
     default_psp(runAsUser={"rule": "MustRunAs", "ranges": [{"min": 999, "max": 999}]}), "runAsUser: Invalid value"),
    ("failSELinuxPSP", with_ctr_sc(default_pod(), seLinuxOptions={"level": "bar"}), SEL_PSP,
     "seLinuxOptions.level: Invalid value"),
    ("failNilAppArmor", default_pod(), APPARMOR_PSP, "AppArmor profile must be set"),
    ("failInvalidAppArmor", default_pod({f"container.apparmor.security.beta.kubernetes.io/{CTR}": "localhost/foo"}),
     APPARMOR_PSP, 'localhost/foo is not an allowed profile. Allowed values: "runtime/default"'),
    ("failPrivPSP", with_ctr_sc(default_pod(), privileged=True), default_psp(), "Privileged containers are not allowed"),
    ("failCapsPSP", with_ctr_sc(default_pod(), capabilities={"add": ["foo"]}), default_psp(),
     "capability may not be added"),
    ("failHostPortPSP", default_pod(containers=[{"name": CTR, "securityContext": {"privileged": False},
                                                 "ports": [{"hostPort": 1}]}]), default_psp(),
     "Host port 1 is not allowed to be used. Allowed ports: []"),
    ("failReadOnlyRootFS - nil", default_pod(), default_psp(readOnlyRootFilesystem=True),
     "ReadOnlyRootFilesystem may not be nil and must be set to true"),
    ("failReadOnlyRootFS - false", with_ctr_sc(default_pod(), readOnlyRootFilesystem=False),
     default_psp(readOnlyRootFilesystem=True), "ReadOnlyRootFilesystem must be set to true"),
    ("failSeccompContainerAnnotation", default_pod({f"container.seccomp.security.alpha.kubernetes.io/{CTR}": "foo"}),
     default_psp(), "Forbidden: seccomp may not be set"),
    ("failSeccompContainerPodAnnotation", default_pod({"seccomp.security.alpha.kubernetes.io/pod": "foo"}),
     default_psp(), "Forbidden: seccomp may not be set"),
]


@pytest.mark.parametrize("name,pod,psp,expected", CONTAINER_FAILURES, ids=[c[0] for c in CONTAINER_FAILURES])
def test_validate_container_security_context_failures(name, pod, psp, expected):
    errs = Provider(psp).validate_container_security_context(pod, pod["spec"]["containers"][0], "")
    assert errs and expected in errs[0], errs


SEL_FULL = {"user": "user", "role": "role", "type": "type", "level": "level"}
HOSTPATH_OK = default_pod(volumes=[{"name": "good volume", "hostPath": {"path": "/foo/bar/baz"}}])
POD_SUCCESSES = [
    ("hostNetwork", default_pod(hostNetwork=True), default_psp(hostNetwork=True)),
    ("hostPID", default_pod(hostPID=True), default_psp(hostPID=True)),
    ("hostIPC", default_pod(hostIPC=True), default_psp(hostIPC=True)),
    ("supplemental group", default_pod(securityContext={"supplementalGroups": [3]}),
     default_psp(supplementalGroups={"rule": "MustRunAs", "ranges": [{"min": 1, "max": 5}]})),
    ("fs group", default_pod(securityContext={"fsGroup": 3}),
     default_psp(fsGroup={"rule": "MustRunAs", "ranges": [{"min": 1, "max": 5}]})),
    ("selinux", default_pod(securityContext={"seLinuxOptions": dict(SEL_FULL)}),
     default_psp(seLinux={"rule": "MustRunAs", "seLinuxOptions": dict(SEL_FULL)})),
    ("sysctl specific profile with safe sysctl", default_pod({"security.alpha.kubernetes.io/sysctls": "foo=1"}),
     default_psp(annotations={"security.alpha.kubernetes.io/sysctls": "foo"})),
    ("sysctl specific profile with unsafe sysctl",
     default_pod({"security.alpha.kubernetes.io/unsafe-sysctls": "foo=1"}),
     default_psp(annotations={"security.alpha.kubernetes.io/sysctls": "foo"})),
    ("empty profile with safe sysctl", default_pod({"security.alpha.kubernetes.io/sysctls": "foo=1"}), default_psp()),
    ("hostDir allowed directory", HOSTPATH_OK,
     default_psp(volumes=["hostPath"], allowedHostPaths=[{"pathPrefix": "/foo/bar"}])),
    ("hostDir all volumes allowed", HOSTPATH_OK,
     default_psp(volumes=["*"], allowedHostPaths=[{"pathPrefix": "/foo/bar"}])),
    ("seccomp", default_pod({"seccomp.security.alpha.kubernetes.io/pod": "foo"}),
     default_psp(annotations={"seccomp.security.alpha.kubernetes.io/allowedProfileNames": "foo"})),
    ("flex whitelist, all volumes", FLEX_OK, flex_psp(False, True)),
    ("flex empty whitelist, all volumes", FLEX_OK, flex_psp(True, True)),
    ("flex whitelist, only flex", FLEX_OK, flex_psp(False, False)),
    ("flex empty whitelist, only flex", FLEX_OK, flex_psp(True, False)),
]


@pytest.mark.parametrize("name,pod,psp", POD_SUCCESSES, ids=[c[0] for c in POD_SUCCESSES])
def test_validate_pod_security_context_success(name, pod, psp):
    assert Provider(psp).validate_pod_security_context(pod) == []


def test_host_path_prefix_is_segment_aware():
    assert has_path_prefix("/foo/bar/baz", "/foo/bar") and has_path_prefix("/foo/bar", "/foo/bar/")
    assert not has_path_prefix("/foo/barbaz", "/foo/bar") and not has_path_prefix("/fo", "/foo")


def test_create_security_context_nonmutating():
    """Defaulting works on copies: the pod and the policy are unchanged."""
    psp = default_psp(runAsUser={"rule": "MustRunAs", "ranges": [{"min": 1, "max": 1}]},
                      seLinux={"rule": "MustRunAs", "seLinuxOptions": {"level": "s0"}},
                      fsGroup={"rule": "MustRunAs", "ranges": [{"min": 1, "max": 1}]},
                      defaultAddCapabilities=["foo"], requiredDropCapabilities=["bar"],
                      readOnlyRootFilesystem=True,
                      annotations={"seccomp.security.alpha.kubernetes.io/defaultProfileName": "docker/default"})
    pod = default_pod()
    before_pod, before_psp = copy.deepcopy(pod), copy.deepcopy(psp)
    prov = Provider(psp)
    psc, anns = prov.create_pod_security_context(pod)
    sc, _ = prov.create_container_security_context(pod, pod["spec"]["containers"][0])
    assert pod == before_pod and psp == before_psp
    assert psc["fsGroup"] == 1 and psc["seLinuxOptions"] == {"level": "s0"}
    assert anns["seccomp.security.alpha.kubernetes.io/pod"] == "docker/default"
    assert sc["runAsUser"] == 1 and sc["capabilities"] == {"add": ["foo"], "drop": ["bar"]}
    assert sc["readOnlyRootFilesystem"] is True


@pytest.mark.parametrize("psp_ro,pod_ro,want", [(False, None, None), (False, True, True), (False, False, False),
                                                (True, None, True), (True, True, True), (True, False, False)])
def test_generate_read_only_root_fs(psp_ro, pod_ro, want):
    pod = default_pod()
    if pod_ro is not None:
        with_ctr_sc(pod, readOnlyRootFilesystem=pod_ro)
    sc, _ = Provider(default_psp(readOnlyRootFilesystem=psp_ro)).create_container_security_context(
        pod, pod["spec"]["containers"][0])
    assert sc.get("readOnlyRootFilesystem") == want


@pytest.mark.parametrize("pod_ape,psp_ape,default_ape,want_err,want_value", [
    (None, True, None, False, None), (None, False, None, False, False), (True, False, None, True, True),
    (False, False, None, False, False), (None, True, True, False, True), (None, True, False, False, False),
    (None, False, False, False, False)])
def test_allow_privilege_escalation(pod_ape, psp_ape, default_ape, want_err, want_value):
    """TestValidateAllowPrivilegeEscalation / TestValidateDefaultAllowPrivilegeEscalation."""
    spec = {"allowPrivilegeEscalation": psp_ape}
    if default_ape is not None:
        spec["defaultAllowPrivilegeEscalation"] = default_ape
    prov = Provider(default_psp(**spec))
    pod = default_pod()
    if pod_ape is not None:
        with_ctr_sc(pod, allowPrivilegeEscalation=pod_ape)
    prov.assign(pod)
    errs = prov.validate_container_security_context(pod, pod["spec"]["containers"][0], "")
    assert bool(errs) == want_err, errs
    assert pod["spec"]["containers"][0]["securityContext"].get("allowPrivilegeEscalation") == want_value


@pytest.mark.parametrize("spec", [{"runAsUser": {"rule": "MustRunAs"}}, {"runAsUser": {"rule": "Bogus"}},
                                  {"seLinux": {"rule": "MustRunAs"}}, {"fsGroup": {"rule": "MustRunAs"}},
                                  {"supplementalGroups": {"rule": "Nope"}}])
def test_invalid_policies_make_no_provider(spec):
    with pytest.raises(ProviderError):
        Provider(default_psp(**spec))


def test_capabilities_generate_and_validate():
    """TestAdmitCaps essentials: default adds, required drops, allowed and `*`."""
    prov = Provider(default_psp(defaultAddCapabilities=["foo"], requiredDropCapabilities=["bar"],
                                allowedCapabilities=["baz"]))
    pod = with_ctr_sc(default_pod(), capabilities={"add": ["baz"], "drop": ["foo"]})
    assert prov.assign(pod) == []
    # the container dropped a default add: it stays dropped, the required drop is added
    assert pod["spec"]["containers"][0]["securityContext"]["capabilities"] == {"add": ["baz"], "drop": ["bar", "foo"]}
    bad = with_ctr_sc(default_pod(), capabilities={"add": ["qux"]})
    assert any("capability may not be added" in e for e in prov.assign(bad))
    assert Provider(default_psp(allowedCapabilities=["*"])).assign(
        with_ctr_sc(default_pod(), capabilities={"add": ["anything"]})) == []


# -- the admission plugin ------------------------------------------------------------------------

class _Authz:
    """Allows `use` of a policy for the listed (user, policy) pairs."""

    def __init__(self, grants):
        self.grants = grants

    def authorize(self, a):
        ok = a.verb == "use" and a.resource == "podsecuritypolicies" and (a.user.name, a.name) in self.grants
        return ok, ""


class _Server:
    def __init__(self, policies, grants=None):
        self.policies = policies
        self.authz = _Authz(grants) if grants is not None else None

    def list_objects(self, resource, namespace=None):
        return list(self.policies) if resource == "podsecuritypolicies" else []


def _pod(name="p", **ctr_sc):
    return {"metadata": {"name": name, "namespace": "ns"},
            "spec": {"containers": [{"name": "c", "image": "x", **({"securityContext": ctr_sc} if ctr_sc else {})}]}}


def _admit(plugin, pod, user="alice", op=CREATE, old=None):
    a = Attributes(op, "pods", "", "ns", pod["metadata"]["name"], pod, old, User(user))
    if op == CREATE:
        plugin.admit(a)
    plugin.validate(a)
    return pod


def test_admit_prefers_nonmutating_policy():
    """TestAdmitPreferNonmutating: an earlier mutating policy loses to a later one that accepts as-is."""
    mutating = default_psp("mutating1", runAsUser={"rule": "MustRunAs", "ranges": [{"min": 1000, "max": 1000}]})
    plain = default_psp("privileged")
    pl = PodSecurityPolicy(_Server([mutating, plain]))
    pod = _admit(pl, _pod())
    assert pod["metadata"]["annotations"]["kubernetes.io/psp"] == "privileged"
    assert "securityContext" not in pod["spec"]["containers"][0]
    # only the mutating policy available: it defaults the UID
    pl = PodSecurityPolicy(_Server([mutating]))
    pod = _admit(pl, _pod())
    assert pod["spec"]["containers"][0]["securityContext"]["runAsUser"] == 1000
    assert pod["metadata"]["annotations"]["kubernetes.io/psp"] == "mutating1"


def test_validate_phase_refuses_later_mutations():
    """Validate (no mutation allowed) catches a change made after PSP admit, e.g. a later plugin."""
    pl = PodSecurityPolicy(_Server([default_psp("restricted")]))
    pod = _pod()
    a = Attributes(CREATE, "pods", "", "ns", "p", pod, None, User("alice"))
    pl.admit(a)
    pod["spec"]["containers"][0]["securityContext"] = {"privileged": True}
    with pytest.raises(AdmissionError, match="Privileged containers are not allowed"):
        pl.validate(a)


def test_policy_authorization():
    """TestPolicyAuthorization: the user or the pod's service account must be allowed to `use` it."""
    policies = [default_psp("policy")]
    with pytest.raises(AdmissionError, match=r"unable to validate against any pod security policy: \[\]"):
        _admit(PodSecurityPolicy(_Server(policies, grants=set())), _pod())
    _admit(PodSecurityPolicy(_Server(policies, grants={("alice", "policy")})), _pod())
    sa_pod = _pod()
    sa_pod["spec"]["serviceAccountName"] = "builder"
    _admit(PodSecurityPolicy(_Server(policies, grants={("system:serviceaccount:ns:builder", "policy")})), sa_pod)


def test_policy_authorization_errors_only_from_usable_policies():
    """TestPolicyAuthorizationErrors: errors of policies the user may not use are not reported."""
    policies = [default_psp("visible"), default_psp("hidden", hostNetwork=False)]
    pl = PodSecurityPolicy(_Server(policies, grants={("alice", "visible")}))
    pod = _pod(privileged=True)
    with pytest.raises(AdmissionError) as e:
        _admit(pl, pod)
    assert "provider visible" in str(e.value) and "provider hidden" not in str(e.value)


def test_fail_on_no_policies_and_gc_updates():
    with pytest.raises(AdmissionError, match="no providers available"):
        _admit(PodSecurityPolicy(_Server([])), _pod())
    _admit(PodSecurityPolicy(_Server([]), {"failOnNoPolicies": False}), _pod())
    # an update that only changes ownerReferences / finalizers is not re-validated
    pl = PodSecurityPolicy(_Server([default_psp("restricted")]))
    old = _pod(privileged=True)
    new = copy.deepcopy(old)
    new["metadata"]["finalizers"] = ["x"]
    _admit(pl, new, op=UPDATE, old=old)
    changed = copy.deepcopy(old)
    changed["metadata"]["labels"] = {"a": "b"}
    with pytest.raises(AdmissionError):
        _admit(pl, changed, op=UPDATE, old=old)
