"""PodSecurityPolicy strategy tables ported from `pkg/security/podsecuritypolicy/user/*_test.go`,
`group/*_test.go`, `selinux/*_test.go` and `capabilities/mustrunas_test.go`."""
import pytest

from kubernetes_amd.apiserver.admission.psp import ProviderError, _Capabilities, _Group, _SELinux, _User


# -- user ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("opts,ok", [(None, True), ({"rule": "MustRunAs"}, False),
                                     ({"rule": "MustRunAs", "ranges": [{"min": 1, "max": 1}]}, True)])
def test_user_new_must_run_as(opts, ok):
    if ok:
        _User(opts)
    else:
        with pytest.raises(ProviderError):
            _User(opts)


def test_user_must_run_as_generate_and_validate():
    s = _User({"rule": "MustRunAs", "ranges": [{"min": 1, "max": 1}, {"min": 10, "max": 20}]})
    assert s.generate() == 1
    assert s.validate("sc", None, 15) == []
    e = s.validate("sc", None, None)
    assert len(e) == 1 and "runAsUser: Required" in e[0]
    e = s.validate("sc", None, 21)
    assert len(e) == 1 and "runAsUser: Invalid" in e[0]


def test_user_run_as_any():
    s = _User({"rule": "RunAsAny"})
    assert s.generate() is None
    assert s.validate("sc", None, None) == [] and s.validate("sc", False, 0) == []


@pytest.mark.parametrize("non_root,uid,err", [
    (None, 0, True), (None, 1, False), (False, None, True), (True, 1, False), (None, None, True)])
def test_user_non_root_validate(non_root, uid, err):
    s = _User({"rule": "MustRunAsNonRoot"})
    assert s.generate() is None
    assert bool(s.validate("sc", non_root, uid)) == err


# -- group --------------------------------------------------------------------------------------
@pytest.mark.parametrize("ranges,ok", [([], False), ([{"min": 1, "max": 1}], True)])
def test_group_must_run_as_options(ranges, ok):
    if ok:
        _Group({"rule": "MustRunAs", "ranges": ranges}, "fsGroup")
    else:
        with pytest.raises(ProviderError):
            _Group({"rule": "MustRunAs", "ranges": ranges}, "fsGroup")


@pytest.mark.parametrize("ranges,want", [
    ([{"min": 1, "max": 2}], 1), ([{"min": 1, "max": 1}], 1), ([{"min": 1, "max": 2}, {"min": 3, "max": 4}], 1)])
def test_group_must_run_as_generate(ranges, want):
    s = _Group({"rule": "MustRunAs", "ranges": ranges}, "supplementalGroups")
    assert s.generate() == [want] and s.generate_single() == want


@pytest.mark.parametrize("groups,ok", [
    (None, False), ([], False), ([5], False), ([2], True), ([1], True), ([3], True), ([4], True)])
def test_group_must_run_as_validate(groups, ok):
    s = _Group({"rule": "MustRunAs", "ranges": [{"min": 1, "max": 3}, {"min": 4, "max": 4}]}, "fsGroup")
    assert (s.validate(groups) == []) == ok


def test_group_run_as_any():
    s = _Group({"rule": "RunAsAny"}, "fsGroup")
    assert s.generate() is None and s.generate_single() is None
    assert s.validate(None) == [] and s.validate([0, 65535]) == []


# -- selinux ------------------------------------------------------------------------------------
OPTS = {"user": "user", "role": "role", "type": "type", "level": "level"}


def test_selinux_must_run_as_options():
    with pytest.raises(ProviderError):
        _SELinux({"rule": "MustRunAs"})
    _SELinux({"rule": "MustRunAs", "seLinuxOptions": dict(OPTS)})


def test_selinux_must_run_as_generate():
    assert _SELinux({"rule": "MustRunAs", "seLinuxOptions": dict(OPTS)}).generate() == OPTS


@pytest.mark.parametrize("field,msg", [("role", "role: Invalid value"), ("user", "user: Invalid value"),
                                       ("level", "level: Invalid value"), ("type", "type: Invalid value"),
                                       (None, "")])
def test_selinux_must_run_as_validate(field, msg):
    s = _SELinux({"rule": "MustRunAs", "seLinuxOptions": dict(OPTS)})
    se = dict(OPTS)
    if field:
        se[field] = "invalid"
    errs = s.validate("sc.seLinuxOptions", se)
    if msg:
        assert len(errs) == 1 and msg in errs[0]
    else:
        assert errs == []


def test_selinux_run_as_any():
    s = _SELinux({"rule": "RunAsAny"})
    assert s.generate() is None and s.validate("sc", None) == [] and s.validate("sc", {"user": "x"}) == []


# -- capabilities -------------------------------------------------------------------------------
def _c(caps):
    return {"securityContext": {"capabilities": caps}} if caps is not None else {}


@pytest.mark.parametrize("default_add,caps,want", [
    ([], None, None),
    ([], {}, {}),
    (["foo"], None, {"add": ["foo"]}),
    (["foo"], {"add": ["foo"]}, {"add": ["foo"]}),
    (["foo", "bar", "baz"], {"add": ["foo"]}, {"add": ["bar", "baz", "foo"]}),
    (["foo"], {"add": ["bar"]}, {"add": ["bar", "foo"]}),
    (["foo", "bar"], {"add": ["foo", "foo", "bar", "baz"]}, {"add": ["foo", "foo", "bar", "baz"]}),   # no mutation
    (["foo", "bar"], {"add": ["foo", "baz"]}, {"add": ["bar", "baz", "foo"]}),
    (["foo"], {"add": ["FOO"]}, {"add": ["FOO", "foo"]}),
])
def test_capabilities_generate_adds(default_add, caps, want):
    assert _Capabilities(default_add, None, None).generate(_c(caps)) == want


@pytest.mark.parametrize("default_add,required_drop,caps,want", [
    ([], [], None, None),
    ([], [], {}, {}),
    ([], ["foo"], None, {"drop": ["foo"]}),
    ([], ["baz"], {"drop": ["foo", "bar"]}, {"drop": ["bar", "baz", "foo"]}),
    ([], ["baz"], {"drop": ["foo", "bar", "baz"]}, {"drop": ["foo", "bar", "baz"]}),
    (["foo"], [], {"drop": ["foo"]}, {"drop": ["foo"]}),
    (["foo"], [], {"drop": ["bar"]}, {"add": ["foo"], "drop": ["bar"]}),
    (["foo", "bar", "baz"], ["abc"], {"drop": ["foo"]}, {"add": ["bar", "baz"], "drop": ["abc", "foo"]}),
    ([], ["baz", "foo"], {"drop": ["bar", "foo"]}, {"drop": ["bar", "baz", "foo"]}),
    ([], ["bar"], {"drop": ["BAR"]}, {"drop": ["BAR", "bar"]}),
])
def test_capabilities_generate_drops(default_add, required_drop, caps, want):
    assert _Capabilities(default_add, required_drop, None).generate(_c(caps)) == want


@pytest.mark.parametrize("default_add,allowed,caps,ok", [
    ([], [], None, True),
    ([], ["foo"], None, True),
    (["foo"], [], None, False),
    (["foo"], [], {"add": ["foo"]}, True),
    (["foo"], [], {"add": ["bar"]}, False),
    ([], ["foo"], {"add": ["foo"]}, True),
    ([], ["*"], {"add": ["foo"]}, True),
    ([], ["foo"], {"add": ["bar"]}, False),
    (["foo"], ["bar"], {"add": ["foo"]}, True),
    (["foo"], ["bar"], {"add": ["bar"]}, True),
    (["foo"], ["bar"], {"add": ["baz"]}, False),
    (["foo"], [], {"add": ["FOO"]}, False),
])
def test_capabilities_validate_adds(default_add, allowed, caps, ok):
    assert (_Capabilities(default_add, None, allowed).validate("sc", caps) == []) == ok


@pytest.mark.parametrize("required_drop,caps,ok", [
    ([], None, True), (["foo"], None, False), (["foo"], {"drop": ["foo"]}, True), (["foo"], {"drop": ["bar"]}, False),
    (["foo"], {"drop": ["FOO"]}, False)])
def test_capabilities_validate_drops(required_drop, caps, ok):
    assert (_Capabilities(None, required_drop, None).validate("sc", caps) == []) == ok
