"""Pod status generation and normalization ported from `pkg/kubelet/status/generate_test.go`
(TestGeneratePodReadyCondition, TestGeneratePodInitializedCondition) and
`pkg/kubelet/status/status_manager_test.go` (TestStatusEquality,
TestStatusNormalizationEnforcesMaxBytes), plus the kubelet's conditions on a running pod."""
import random

import pytest

from kubernetes_amd.kubelet.podstatus import (
    CONTAINERS_NOT_INITIALIZED, CONTAINERS_NOT_READY, MAX_POD_TERMINATION_MESSAGE_LOG_LENGTH, POD_COMPLETED,
    UNKNOWN_CONTAINER_STATUSES, generate_pod_initialized_condition, generate_pod_ready_condition, normalize_status,
    sort_init_container_statuses)


def ready(name):
    return {"name": name, "ready": True}


def not_ready(name):
    return {"name": name, "ready": False}


def spec(*names, init=()):
    return {"containers": [{"name": n} for n in names], "initContainers": [{"name": n} for n in init]}


def rc(ok, reason="", message=""):
    c = {"type": "Ready", "status": "True" if ok else "False"}
    if reason:
        c["reason"] = reason
    if message:
        c["message"] = message
    return c


READY_CASES = [
    (None, None, "Running", rc(False, UNKNOWN_CONTAINER_STATUSES)),
    ({}, [], "Running", rc(True)),
    (spec("1234"), [], "Running", rc(False, CONTAINERS_NOT_READY, "containers with unknown status: [1234]")),
    (spec("1234", "5678"), [ready("1234"), ready("5678")], "Running", rc(True)),
    (spec("1234", "5678"), [ready("1234")], "Running",
     rc(False, CONTAINERS_NOT_READY, "containers with unknown status: [5678]")),
    (spec("1234", "5678"), [ready("1234"), not_ready("5678")], "Running",
     rc(False, CONTAINERS_NOT_READY, "containers with unready status: [5678]")),
    (spec("1234"), [not_ready("1234")], "Succeeded", rc(False, POD_COMPLETED)),
    # both kinds at once, joined like the reference
    (spec("a", "b", "c"), [not_ready("a")], "Running",
     rc(False, CONTAINERS_NOT_READY, "containers with unknown status: [b c], containers with unready status: [a]")),
]


@pytest.mark.parametrize("sp,statuses,phase,want", READY_CASES)
def test_generate_pod_ready_condition(sp, statuses, phase, want):
    assert generate_pod_ready_condition(sp, statuses, phase) == want


TWO = spec(init=("1234", "5678"))
ONE = spec(init=("1234",))
INIT_CASES = [
    (TWO, None, "Running", "False", UNKNOWN_CONTAINER_STATUSES),
    ({}, [], "Running", "True", ""),
    (ONE, [], "Running", "False", CONTAINERS_NOT_INITIALIZED),
    (TWO, [ready("1234"), ready("5678")], "Running", "True", ""),
    (TWO, [ready("1234")], "Running", "False", CONTAINERS_NOT_INITIALIZED),
    (TWO, [ready("1234"), not_ready("5678")], "Running", "False", CONTAINERS_NOT_INITIALIZED),
    (ONE, [ready("1234")], "Succeeded", "True", POD_COMPLETED),
]


@pytest.mark.parametrize("sp,statuses,phase,status,reason", INIT_CASES)
def test_generate_pod_initialized_condition(sp, statuses, phase, status, reason):
    c = generate_pod_initialized_condition(sp, statuses, phase)
    assert c["type"] == "Initialized"
    assert (c["status"], c.get("reason", "")) == (status, reason)


def test_initialized_message_names_incomplete_containers():
    c = generate_pod_initialized_condition(TWO, [not_ready("1234")], "Pending")
    assert c["message"] == "containers with unknown status: [5678], containers with incomplete status: [1234]"


def test_status_equality_ignores_container_order():
    pod = {"spec": {}}
    statuses = [{"name": f"container{i}"} for i in range(10)]
    new = normalize_status(pod, {"containerStatuses": list(statuses)})
    rnd = random.Random(7)
    for _ in range(10):
        shuffled = list(statuses)
        rnd.shuffle(shuffled)
        assert normalize_status(pod, {"containerStatuses": shuffled}) == new


def test_status_normalization_enforces_max_bytes():
    pod = {"spec": {}}
    statuses = [{"name": f"container{i}", "lastState": {"terminated": {"message": "abcdefgh" * (24 + i % 3)}}}
                for i in range(48)]
    status = {"initContainerStatuses": statuses[:24], "containerStatuses": statuses[24:]}
    result = normalize_status(pod, status)
    count = 0
    for s in result["initContainerStatuses"]:
        n = len(s["lastState"]["terminated"]["message"])
        assert 192 <= n <= 256
        count += n
    assert count <= MAX_POD_TERMINATION_MESSAGE_LOG_LENGTH


def test_normalization_splits_budget_over_spec_containers():
    pod = {"spec": {"containers": [{"name": "a"}, {"name": "b"}], "initContainers": [{"name": "i"}]}}
    st = {"containerStatuses": [{"name": "b", "state": {"terminated": {"message": "x" * 9000}}},
                                {"name": "a", "state": {"running": {}}}],
          "initContainerStatuses": [{"name": "i", "state": {"terminated": {"message": "y" * 10}}}]}
    normalize_status(pod, st)
    assert [s["name"] for s in st["containerStatuses"]] == ["a", "b"]
    assert len(st["containerStatuses"][1]["state"]["terminated"]["message"]) == MAX_POD_TERMINATION_MESSAGE_LOG_LENGTH // 3
    assert st["initContainerStatuses"][0]["state"]["terminated"]["message"] == "y" * 10


def test_sort_init_container_statuses_follows_spec():
    pod = {"spec": {"initContainers": [{"name": n} for n in ("first", "second", "third")]}}
    st = [{"name": "third"}, {"name": "extra"}, {"name": "first"}, {"name": "second"}]
    sort_init_container_statuses(pod, st)
    assert [s["name"] for s in st] == ["first", "second", "third", "extra"]


# -- pkg/kubelet/container/helpers_test.go -------------------------------------------------------
from types import SimpleNamespace  # noqa: E402

from kubernetes_amd.kubelet.kubelet import expand_container_command_and_args, should_container_be_restarted  # noqa: E402
from kubernetes_amd.kubelet.runtime.base import CREATED, EXITED, RUNNING, UNKNOWN  # noqa: E402


def test_should_container_be_restarted():
    # statuses latest first; FindContainerStatusByName takes the first match
    statuses = [("alive", RUNNING, 0), ("succeed", EXITED, 0), ("failed", EXITED, 1), ("alive", EXITED, 2),
                ("unknown", UNKNOWN, 0), ("failed", EXITED, 3), ("created", CREATED, 0)]

    def latest(name):
        for n, state, code in statuses:
            if n == name:
                return SimpleNamespace(state=state, exit_code=code)
        return None

    expected = {"no-history": (True, True, True), "alive": (False, False, False), "succeed": (False, False, True),
                "failed": (False, True, True), "unknown": (True, True, True), "created": (True, True, True)}
    for name, want in expected.items():
        got = tuple(should_container_be_restarted(p, latest(name)) for p in ("Never", "OnFailure", "Always"))
        assert got == want, name


EXPAND_CASES = [
    ("none", {}, [], None, None),
    ("command expanded", {"command": ["foo", "$(VAR_TEST)", "$(VAR_TEST2)"]},
     [("VAR_TEST", "zoo"), ("VAR_TEST2", "boo")], ["foo", "zoo", "boo"], None),
    ("args expanded", {"args": ["zap", "$(VAR_TEST)", "$(VAR_TEST2)"]},
     [("VAR_TEST", "hap"), ("VAR_TEST2", "trap")], None, ["zap", "hap", "trap"]),
    ("both expanded", {"command": ["$(VAR_TEST2)--$(VAR_TEST)", "foo", "$(VAR_TEST3)"],
                       "args": ["foo", "$(VAR_TEST)", "$(VAR_TEST2)"]},
     [("VAR_TEST", "zoo"), ("VAR_TEST2", "boo"), ("VAR_TEST3", "roo")], ["boo--zoo", "foo", "roo"],
     ["foo", "zoo", "boo"]),
    ("later variable wins, unknown kept, $$ escapes", {"command": ["$(A)", "$(MISSING)", "$$(A)"]},
     [("A", "1"), ("A", "2")], ["2", "$(MISSING)", "$(A)"], None),
]


@pytest.mark.parametrize("name,c,envs,cmd,args", EXPAND_CASES, ids=[x[0] for x in EXPAND_CASES])
def test_expand_container_command_and_args(name, c, envs, cmd, args):
    got = expand_container_command_and_args(c, [{"name": n, "value": v} for n, v in envs])
    assert got == (cmd, args)


# -- pkg/kubelet/kuberuntime/security_context_test.go TestVerifyRunAsNonRoot ---------------------
from kubernetes_amd.kubelet.kubelet import image_user, verify_run_as_non_root  # noqa: E402


@pytest.mark.parametrize("non_root,run_as,image_uid,fail", [
    (None, None, 0, False),          # no SecurityContext
    (None, 0, 0, False),             # RunAsNonRoot not set
    (False, None, 0, False),         # RunAsNonRoot false, image user root
    (False, 0, 123, False),          # RunAsNonRoot false, RunAsUser root
    (True, 0, 123, True),            # RunAsUser root with RunAsNonRoot
    (True, None, 0, True),           # image user root with RunAsNonRoot
    (True, None, 123, False),
    (True, 1000, 0, False),
])
def test_verify_run_as_non_root(non_root, run_as, image_uid, fail):
    assert bool(verify_run_as_non_root(non_root, run_as, image_uid)) == fail


def test_image_user_and_non_numeric_name():
    assert image_user({}) == (0, "") and image_user(None) == (0, "")
    assert image_user({"User": "123"}) == (123, "") and image_user({"User": "123:456"}) == (123, "")
    assert image_user({"User": "nobody"}) == (None, "nobody")
    assert "non-numeric user (nobody)" in verify_run_as_non_root(True, None, None, "nobody")
