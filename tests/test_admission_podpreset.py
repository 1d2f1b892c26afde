"""PodPreset: ported tables.

Reference: `plugin/pkg/admission/podpreset/admission_test.go` — TestMergeEnv, TestMergeEnvFrom,
TestMergeVolumeMounts, TestMergeVolumes (the merge functions), and the admit cases: a preset in
another namespace or with a non-matching selector does nothing, a conflict leaves the pod
unchanged (and admitted), a matching preset applies volumes / env / envFrom and the annotation,
mirror pods and opted-out pods are skipped.
"""
import copy

import pytest

from kubernetes_amd.apiserver.admission import CREATE, Attributes
from kubernetes_amd.apiserver.admission.security import (PodPreset, PresetConflict, merge_env, merge_env_from,
                                                         merge_volume_mounts, merge_volumes)


def pp(name="hello", ns="namespace", rv="1", selector=None, **spec):
    spec["selector"] = selector or {"matchExpressions": [{"key": "security", "operator": "In", "values": ["S2"]}]}
    return {"metadata": {"name": name, "namespace": ns, "resourceVersion": rv}, "spec": spec}


def E(name, value):
    return {"name": name, "value": value}


def CM(name, prefix=None):
    out = {"configMapRef": {"name": name}}
    if prefix:
        out["prefix"] = prefix
    return out


def VM(name, path):
    return {"name": name, "mountPath": path}


def ED(name):
    return {"name": name, "emptyDir": {}}


@pytest.mark.parametrize("orig,mod,result", [
    (None, [E("abc", "value2"), E("ABC", "value3")], [E("abc", "value2"), E("ABC", "value3")]),
    ([E("abcd", "value2"), E("hello", "value3")], [E("abc", "value2"), E("ABC", "value3")],
     [E("abcd", "value2"), E("hello", "value3"), E("abc", "value2"), E("ABC", "value3")]),
    ([E("abc", "value3")], [E("abc", "value2"), E("ABC", "value3")], None),
    ([E("abc", "value2"), E("hello", "value3")], [E("abc", "value2"), E("ABC", "value3")],
     [E("abc", "value2"), E("hello", "value3"), E("ABC", "value3")]),
], ids=["empty original", "good merge", "conflict", "one is exact same"])
def test_merge_env(orig, mod, result):
    if result is None:
        with pytest.raises(PresetConflict, match="conflict on abc"):
            merge_env(orig, [pp(env=mod)])
    else:
        assert merge_env(orig, [pp(env=mod)]) == result


@pytest.mark.parametrize("orig,mod,result", [
    (None, [CM("abc"), CM("abc", "pre_")], [CM("abc"), CM("abc", "pre_")]),
    ([CM("thing")], [CM("abc"), CM("abc", "pre_")], [CM("thing"), CM("abc"), CM("abc", "pre_")]),
], ids=["empty original", "good merge"])
def test_merge_env_from(orig, mod, result):
    assert merge_env_from(orig, [pp(envFrom=mod)]) == result


@pytest.mark.parametrize("orig,mod,result", [
    (None, [VM("simply-mounted-volume", "/opt/")], [VM("simply-mounted-volume", "/opt/")]),
    ([VM("etc-volume", "/etc/")], [VM("simply-mounted-volume", "/opt/")],
     [VM("etc-volume", "/etc/"), VM("simply-mounted-volume", "/opt/")]),
    ([VM("etc-volume", "/etc/")], [VM("simply-mounted-volume", "/opt/"), VM("etc-volume", "/things/")], None),
    ([VM("etc-volume", "/etc/")], [VM("simply-mounted-volume", "/opt/"), VM("things-volume", "/etc/")], None),
    ([VM("etc-volume", "/etc/")], [VM("simply-mounted-volume", "/opt/"), VM("etc-volume", "/etc/")],
     [VM("etc-volume", "/etc/"), VM("simply-mounted-volume", "/opt/")]),
], ids=["empty original", "good merge", "conflict", "conflict on mount path", "one is exact same"])
def test_merge_volume_mounts(orig, mod, result):
    if result is None:
        with pytest.raises(PresetConflict):
            merge_volume_mounts(orig, [pp(volumeMounts=mod)])
    else:
        assert merge_volume_mounts(orig, [pp(volumeMounts=mod)]) == result


@pytest.mark.parametrize("orig,mod,result", [
    (None, [ED("vol"), ED("vol2")], [ED("vol"), ED("vol2")]),
    ([ED("vol3"), ED("vol4")], [ED("vol"), ED("vol2")], [ED("vol3"), ED("vol4"), ED("vol"), ED("vol2")]),
    ([ED("vol3"), ED("vol4")], [{"name": "vol3", "hostPath": {"path": "/etc/apparmor.d"}}, ED("vol2")], None),
    ([ED("vol3"), ED("vol4")], [ED("vol3"), ED("vol2")], [ED("vol3"), ED("vol4"), ED("vol2")]),
], ids=["empty original", "good merge", "conflict", "one is exact same"])
def test_merge_volumes(orig, mod, result):
    if result is None:
        with pytest.raises(PresetConflict):
            merge_volumes(orig, [pp(volumes=mod)])
    else:
        assert merge_volumes(orig, [pp(volumes=mod)]) == result


def test_merge_conflict_between_presets():
    with pytest.raises(PresetConflict):
        merge_env([], [pp("a", env=[E("X", "1")]), pp("b", env=[E("X", "2")])])


class _Server:
    def __init__(self, presets):
        self.presets = presets

    def list_objects(self, resource, namespace=None):
        assert resource == "podpresets"
        return [p for p in self.presets if p["metadata"]["namespace"] == namespace]


def _pod(env=None, labels=None, annotations=None, ns="namespace"):
    md = {"name": "mypod", "namespace": ns, "labels": labels if labels is not None else {"security": "S2"}}
    if annotations:
        md["annotations"] = annotations
    return {"metadata": md, "spec": {"containers": [{"name": "container", "image": "x",
                                                     "env": env or [E("abc", "value2"), E("ABCD", "value3")]}]}}


FULL = dict(volumes=[ED("vol")], env=[E("abcd", "value"), E("ABC", "value")], envFrom=[CM("abc"), CM("abc", "pre_")])


def _admit(pod, *presets, ns="namespace"):
    PodPreset(_Server(list(presets))).admit(Attributes(CREATE, "pods", "", ns, "", pod))


@pytest.mark.parametrize("case,pod,preset", [
    ("conflict with different namespace", _pod(env=[E("abc", "value2"), E("ABC", "value3")]),
     pp(ns="different", **FULL)),
    ("non-matching labels", _pod(labels={"security": "S3"}), pp(**FULL)),
    ("conflict", _pod(env=[E("abc", "value2"), E("ABC", "value3")]), pp(**FULL)),
    ("mirror pod", _pod(annotations={"kubernetes.io/config.mirror": "mirror"}), pp(**FULL)),
    ("exclusion", _pod(annotations={"podpreset.admission.kubernetes.io/exclude": "true"}), pp(**FULL)),
    ("empty pod namespace", _pod(ns=""), pp(ns="different", **FULL)),
])
def test_admit_leaves_pod_unchanged(case, pod, preset):
    orig = copy.deepcopy(pod)
    _admit(pod, preset, ns=pod["metadata"]["namespace"])
    assert pod == orig, case


def test_admit_applies_matching_preset():
    pod = _pod()
    _admit(pod, pp(**FULL))
    c = pod["spec"]["containers"][0]
    assert c["env"] == [E("abc", "value2"), E("ABCD", "value3"), E("abcd", "value"), E("ABC", "value")]
    assert c["envFrom"] == [CM("abc"), CM("abc", "pre_")]
    assert pod["spec"]["volumes"] == [ED("vol")]
    assert pod["metadata"]["annotations"] == {"podpreset.admission.kubernetes.io/podpreset-hello": "1"}


def test_admit_is_all_or_nothing_across_presets():
    """One conflicting preset keeps the others from being applied too (safeToApplyPodPresetsOnPod)."""
    pod = _pod()
    orig = copy.deepcopy(pod)
    _admit(pod, pp("a", env=[E("NEW", "1")]), pp("b", env=[E("abc", "other")]))
    assert pod == orig
