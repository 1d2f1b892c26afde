"""Container GC selection ported from `pkg/kubelet/kuberuntime/kuberuntime_gc_test.go`
(TestContainerGC): evict units per (pod, container), min age on createdAt, per-unit and overall
limits, deleted and terminated pods."""
import time

import pytest

from kubernetes_amd.kubelet.kubelet import containers_to_evict
from kubernetes_amd.kubelet.runtime.base import EXITED, RUNNING

NOW = time.time()
HOUR = 3600.0


def gc(pod, name, attempt, created, state=EXITED):
    return (pod, name, attempt, created, state)


DEFAULT = {"min_age": HOUR, "max_per_pod_container": 2, "max_containers": 6}

CASES = [
    ("all containers should be removed when max container limit is 0",
     [gc("foo", "bar", 0, 0)], {"min_age": 60, "max_per_pod_container": 1, "max_containers": 0}, [], False),
    ("max containers should be complied when no max per pod container limit is set",
     [gc("foo", "bar", i, i) for i in (4, 3, 2, 1, 0)],
     {"min_age": 60, "max_per_pod_container": -1, "max_containers": 4}, [0, 1, 2, 3], False),
    ("no containers should be removed if both max container and per pod container limits are not set",
     [gc("foo", "bar", i, i) for i in (2, 1, 0)],
     {"min_age": 60, "max_per_pod_container": -1, "max_containers": -1}, [0, 1, 2], False),
    ("recently started containers should not be removed",
     [gc("foo", "bar", i, NOW) for i in (2, 1, 0)], None, [0, 1, 2], False),
    ("oldest containers should be removed when per pod container limit exceeded",
     [gc("foo", "bar", i, i) for i in (2, 1, 0)], None, [0, 1], False),
    ("running containers should not be removed",
     [gc("foo", "bar", 2, 2), gc("foo", "bar", 1, 1), gc("foo", "bar", 0, 0, RUNNING)], None, [0, 1, 2], False),
    ("no containers should be removed when limits are not exceeded",
     [gc("foo", "bar", 1, 1), gc("foo", "bar", 0, 0)], None, [0, 1], False),
    ("max container count should apply per (UID, container) pair",
     [gc(p, n, i, i) for p, n in (("foo", "bar"), ("foo1", "baz"), ("foo2", "bar")) for i in (2, 1, 0)],
     None, [0, 1, 3, 4, 6, 7], False),
    ("max limit should apply and try to keep from every pod",
     [gc(f"foo{k or ''}", f"bar{k or ''}", i, i) for k in range(5) for i in (1, 0)], None, [0, 2, 4, 6, 8], False),
    ("oldest pods should be removed if limit exceeded",
     [gc("foo", "bar", 2, 2), gc("foo", "bar", 1, 1), gc("foo1", "bar1", 2, 2), gc("foo1", "bar1", 1, 1),
      gc("foo2", "bar2", 1, 1), gc("foo3", "bar3", 0, 0), gc("foo4", "bar4", 1, 1), gc("foo5", "bar5", 0, 0),
      gc("foo6", "bar6", 2, 2), gc("foo7", "bar7", 1, 1)], None, [0, 2, 4, 6, 8, 9], False),
    ("all non-running containers should be removed when evictTerminatedPods is set",
     [gc("foo", "bar", 2, 2), gc("foo", "bar", 1, 1), gc("foo1", "bar1", 2, 2), gc("foo1", "bar1", 1, 1),
      gc("running", "bar2", 1, 1), gc("foo3", "bar3", 0, 0, RUNNING)], None, [4, 5], True),
    ("containers for deleted pods should be removed",
     [gc("foo", "bar", 1, 1), gc("foo", "bar", 0, 0), gc("deleted", "bar1", 2, NOW), gc("deleted", "bar1", 1, 1),
      gc("deleted", "bar1", 0, 0)], None, [0, 1, 2], False),
]


@pytest.mark.parametrize("desc,templates,policy,remain,evict_terminated", CASES, ids=[c[0] for c in CASES])
def test_container_gc(desc, templates, policy, remain, evict_terminated):
    recs = [(f"c{i}", f"uid-{pod}", name, created, state)
            for i, (pod, name, attempt, created, state) in enumerate(templates)]
    removed = containers_to_evict(recs, policy or DEFAULT, NOW, lambda uid: uid == "uid-deleted",
                                  lambda uid: uid != "uid-running", evict_terminated)
    left = sorted(int(cid[1:]) for cid, *_ in recs if cid not in removed)
    assert left == remain
    assert len(set(removed)) == len(removed)


def test_orphans_are_their_own_units_and_respect_min_age():
    recs = [("a", "", "x", 0, EXITED), ("b", "", "x", NOW, EXITED), ("c", "", "y", 0, RUNNING)]
    assert containers_to_evict(recs, {"min_age": 60}, NOW, lambda uid: True, lambda uid: False) == ["a"]


def test_sources_not_ready_keeps_deleted_pods_units():
    recs = [("a", "uid-gone", "x", 0, EXITED)]
    pol = {"min_age": 0, "max_per_pod_container": 1, "max_containers": -1}
    assert containers_to_evict(recs, pol, NOW, lambda uid: True, lambda uid: True, all_sources_ready=False) == []
