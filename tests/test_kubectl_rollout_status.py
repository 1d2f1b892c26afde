"""`kubectl rollout status` viewers ported from `pkg/kubectl/rollout_status_test.go`
(TestDeploymentStatusViewerStatus, TestDaemonSetStatusViewerStatus,
TestStatefulSetStatusViewerStatus, TestDaemonSetStatusViewerStatusWithWrongUpdateStrategyType)."""
import pytest

from kubernetes_amd.kubectl.cli import rollout_status


def dep(gen, replicas, observed, total, updated, available):
    return {"kind": "Deployment", "metadata": {"name": "foo", "namespace": "bar", "generation": gen},
            "spec": {"replicas": replicas},
            "status": {"observedGeneration": observed, "replicas": total, "updatedReplicas": updated,
                       "availableReplicas": available}}


@pytest.mark.parametrize("d,msg,done", [
    (dep(0, 1, 1, 1, 0, 1), "Waiting for rollout to finish: 0 out of 1 new replicas have been updated...", False),
    (dep(1, 1, 1, 2, 1, 2), "Waiting for rollout to finish: 1 old replicas are pending termination...", False),
    (dep(1, 2, 1, 2, 2, 1), "Waiting for rollout to finish: 1 of 2 updated replicas are available...", False),
    (dep(1, 2, 1, 2, 2, 2), 'deployment "foo" successfully rolled out', True),
    (dep(2, 2, 1, 2, 2, 2), "Waiting for deployment spec update to be observed...", False),
])
def test_deployment_status_viewer(d, msg, done):
    assert rollout_status(d) == (msg, done)


def test_deployment_revision_mismatch_is_an_error():
    d = dep(1, 1, 1, 1, 1, 1)
    d["metadata"]["annotations"] = {"deployment.kubernetes.io/revision": "2"}
    assert rollout_status(d, 2)[1] is True
    with pytest.raises(SystemExit, match=r"desired revision \(3\) is different from the running revision \(2\)"):
        rollout_status(d, 3)


def ds(gen, observed, updated, desired, available, strategy="RollingUpdate"):
    return {"kind": "DaemonSet", "metadata": {"name": "foo", "generation": gen},
            "spec": {"updateStrategy": {"type": strategy}},
            "status": {"observedGeneration": observed, "updatedNumberScheduled": updated,
                       "desiredNumberScheduled": desired, "numberAvailable": available}}


@pytest.mark.parametrize("d,msg,done", [
    (ds(0, 1, 0, 1, 0), "Waiting for rollout to finish: 0 out of 1 new pods have been updated...", False),
    (ds(1, 1, 2, 2, 1), "Waiting for rollout to finish: 1 of 2 updated pods are available...", False),
    (ds(1, 1, 2, 2, 2), 'daemon set "foo" successfully rolled out', True),
    (ds(2, 1, 2, 2, 2), "Waiting for daemon set spec update to be observed...", False),
])
def test_daemon_set_status_viewer(d, msg, done):
    assert rollout_status(d) == (msg, done)


def test_daemon_set_wrong_update_strategy():
    with pytest.raises(SystemExit, match="Status is available only for RollingUpdate strategy type"):
        rollout_status(ds(1, 1, 1, 1, 1, strategy="OnDelete"))


def sts(gen, observed, replicas, ready, current, updated, strategy, cur_rev="", upd_rev=""):
    st = {"replicas": replicas, "readyReplicas": ready, "currentReplicas": current, "updatedReplicas": updated,
          "currentRevision": cur_rev, "updateRevision": upd_rev}
    if observed is not None:
        st["observedGeneration"] = observed
    return {"kind": "StatefulSet", "metadata": {"name": "foo", "generation": gen},
            "spec": {"replicas": 3, "updateStrategy": strategy}, "status": st}


RU = {"type": "RollingUpdate"}


@pytest.mark.parametrize("s,msg,done", [
    (sts(2, 1, 3, 3, 3, 0, RU), "Waiting for statefulset spec update to be observed...", False),
    (sts(1, None, 3, 3, 3, 0, RU), "Waiting for statefulset spec update to be observed...", False),
    (sts(1, 2, 3, 2, 3, 0, RU), "Waiting for 1 pods to be ready...", False),
    (sts(1, 2, 3, 3, 3, 1, {"type": "RollingUpdate", "rollingUpdate": {"partition": 2}}),
     "partitioned roll out complete: 1 new pods have been updated...", True),
    (sts(1, 2, 3, 3, 3, 0, {"type": "RollingUpdate", "rollingUpdate": {"partition": 2}}),
     "Waiting for partitioned roll out to finish: 0 out of 1 new pods have been updated...", False),
    (sts(1, 2, 3, 3, 3, 3, RU, "foo", "bar"), "waiting for statefulset rolling update to complete 3 pods at revision bar...",
     False),
    (sts(1, 2, 3, 3, 3, 3, RU, "foo", "foo"), "statefulset rolling update complete 3 pods at revision foo...", True),
])
def test_stateful_set_status_viewer(s, msg, done):
    assert rollout_status(s) == (msg, done)


def test_stateful_set_on_delete_is_an_error():
    with pytest.raises(SystemExit, match="OnDelete updateStrategy does not have a Status"):
        rollout_status(sts(1, 1, 0, 1, 0, 0, {"type": "OnDelete"}))
