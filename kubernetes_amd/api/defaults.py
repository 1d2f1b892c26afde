"""API defaulting for the workload and policy groups (the `SetDefaults_*` functions the
reference's scheme runs on every decoded object, before validation).

Parity (reference paths):
  * pod template / pod spec: `pkg/apis/core/v1/defaults.go` (restartPolicy Always, dnsPolicy
    ClusterFirst, terminationGracePeriodSeconds 30, schedulerName default-scheduler, container
    terminationMessagePath/Policy, port protocol TCP, probe periods/thresholds, volume source
    defaults) — the fork's ER limits→requests copy lives in `core.set_defaults_pod`.
    imagePullPolicy is left unset (the kubelet's image manager treats unset as IfNotPresent:
    this cluster has no registry to re-pull `:latest` from);
  * ReplicationController: `pkg/apis/core/v1/defaults.go` SetDefaults_ReplicationController
    (selector and labels from the template, replicas 1);
  * Deployment / ReplicaSet / DaemonSet / StatefulSet: `pkg/apis/extensions/v1beta1/defaults.go`,
    `pkg/apis/apps/v1beta2/defaults.go` (replicas 1, RollingUpdate 25%/25%, revisionHistoryLimit,
    progressDeadlineSeconds 600, DaemonSet OnDelete→RollingUpdate maxUnavailable 1, StatefulSet
    OrderedReady + RollingUpdate partition 0; the pre-apps/v1 selector default from template
    labels is kept for clients that omit it);
  * Job / CronJob: `pkg/apis/batch/v1/defaults.go` (completions/parallelism 1, backoffLimit 6),
    `pkg/apis/batch/v1beta1/defaults.go` (concurrencyPolicy Allow, suspend false, history 3/1);
  * HorizontalPodAutoscaler: `pkg/apis/autoscaling/v1/defaults.go` (minReplicas 1);
  * Service / Secret / PV / PVC small defaults.
"""
from __future__ import annotations

from . import core


def _default(d, k, v):
    if d.get(k) is None:
        d[k] = v


def _probe(p):
    if not p:
        return
    _default(p, "timeoutSeconds", 1)
    _default(p, "periodSeconds", 10)
    _default(p, "successThreshold", 1)
    _default(p, "failureThreshold", 3)
    hg = p.get("httpGet")
    if hg:
        _default(hg, "path", "/")
        _default(hg, "scheme", "HTTP")


def _container(c):
    _default(c, "terminationMessagePath", "/dev/termination-log")
    _default(c, "terminationMessagePolicy", "File")
    for p in c.get("ports") or ():
        _default(p, "protocol", "TCP")
    _probe(c.get("livenessProbe"))
    _probe(c.get("readinessProbe"))


def pod_spec(spec):
    if spec is None:
        return
    _default(spec, "restartPolicy", "Always")
    _default(spec, "dnsPolicy", "ClusterFirst")
    _default(spec, "terminationGracePeriodSeconds", 30)
    _default(spec, "schedulerName", "default-scheduler")
    _default(spec, "securityContext", {})
    for c in list(spec.get("containers") or ()) + list(spec.get("initContainers") or ()):
        if isinstance(c, dict):
            _container(c)
    for v in spec.get("volumes") or ():
        if not isinstance(v, dict):
            continue
        for src in ("secret", "configMap", "downwardAPI", "projected"):
            if isinstance(v.get(src), dict):
                _default(v[src], "defaultMode", 0o644)
        if isinstance(v.get("hostPath"), dict):
            _default(v["hostPath"], "type", "")


def _template(spec):
    t = spec.get("template")
    if isinstance(t, dict):
        pod_spec(t.setdefault("spec", {}))
    return t


def _selector_from_template(spec):
    """extensions/v1beta1 / apps/v1beta1 SetDefaults: a missing selector is the template's labels."""
    t = spec.get("template")
    labels = ((t or {}).get("metadata") or {}).get("labels") if isinstance(t, dict) else None
    if spec.get("selector") is None and labels:
        spec["selector"] = {"matchLabels": dict(labels)}


def _labels_from_template(obj):
    t = (obj.get("spec") or {}).get("template")
    labels = ((t or {}).get("metadata") or {}).get("labels") if isinstance(t, dict) else None
    md = obj.setdefault("metadata", {})
    if not md.get("labels") and labels:
        md["labels"] = dict(labels)


def deployment(obj):
    spec = obj.setdefault("spec", {})
    _template(spec)
    _selector_from_template(spec)
    _labels_from_template(obj)
    _default(spec, "replicas", 1)
    st = spec.setdefault("strategy", {})
    _default(st, "type", "RollingUpdate")
    if st["type"] == "RollingUpdate":
        ru = st.setdefault("rollingUpdate", {})
        _default(ru, "maxUnavailable", "25%")
        _default(ru, "maxSurge", "25%")
    _default(spec, "revisionHistoryLimit", 10)
    _default(spec, "progressDeadlineSeconds", 600)


def replicaset(obj):
    spec = obj.setdefault("spec", {})
    _template(spec)
    _selector_from_template(spec)
    _labels_from_template(obj)
    _default(spec, "replicas", 1)


def daemonset(obj):
    spec = obj.setdefault("spec", {})
    _template(spec)
    _selector_from_template(spec)
    _labels_from_template(obj)
    us = spec.setdefault("updateStrategy", {})
    _default(us, "type", "RollingUpdate")
    if us["type"] == "RollingUpdate":
        _default(us.setdefault("rollingUpdate", {}), "maxUnavailable", 1)
    _default(spec, "revisionHistoryLimit", 10)


def statefulset(obj):
    spec = obj.setdefault("spec", {})
    _template(spec)
    _selector_from_template(spec)
    _labels_from_template(obj)
    _default(spec, "replicas", 1)
    _default(spec, "podManagementPolicy", "OrderedReady")
    us = spec.setdefault("updateStrategy", {})
    _default(us, "type", "RollingUpdate")
    if us["type"] == "RollingUpdate":
        _default(us.setdefault("rollingUpdate", {}), "partition", 0)
    _default(spec, "revisionHistoryLimit", 10)


def replicationcontroller(obj):
    spec = obj.setdefault("spec", {})
    t = _template(spec)
    labels = ((t or {}).get("metadata") or {}).get("labels") if isinstance(t, dict) else None
    if not spec.get("selector") and labels:
        spec["selector"] = dict(labels)
    _labels_from_template(obj)
    _default(spec, "replicas", 1)


def job_spec(spec):
    _template(spec)
    if spec.get("completions") is None and spec.get("parallelism") is None:
        spec["completions"] = 1
        spec["parallelism"] = 1
    _default(spec, "parallelism", 1)
    _default(spec, "backoffLimit", 6)


def job(obj):
    spec = obj.setdefault("spec", {})
    job_spec(spec)
    _labels_from_template(obj)


def cronjob(obj):
    spec = obj.setdefault("spec", {})
    _default(spec, "concurrencyPolicy", "Allow")
    _default(spec, "suspend", False)
    _default(spec, "successfulJobsHistoryLimit", 3)
    _default(spec, "failedJobsHistoryLimit", 1)
    jt = spec.get("jobTemplate")
    if isinstance(jt, dict):
        job_spec(jt.setdefault("spec", {}))


def hpa(obj):
    _default(obj.setdefault("spec", {}), "minReplicas", 1)


def podtemplate(obj):
    t = obj.get("template")
    if isinstance(t, dict):
        pod_spec(t.setdefault("spec", {}))


def secret(obj):
    _default(obj, "type", "Opaque")


def persistentvolume(obj):
    spec = obj.setdefault("spec", {})
    _default(spec, "persistentVolumeReclaimPolicy", "Retain")
    st = obj.setdefault("status", {})
    _default(st, "phase", "Pending")


def persistentvolumeclaim(obj):
    _default(obj.setdefault("status", {}), "phase", "Pending")


def networkpolicy(obj):
    spec = obj.setdefault("spec", {})
    for rule in list(spec.get("ingress") or ()) + list(spec.get("egress") or ()):
        for p in (rule or {}).get("ports") or ():
            _default(p, "protocol", "TCP")


def pod(obj):
    pod_spec(obj.setdefault("spec", {}))


BY_KIND = {
    "Pod": pod, "Deployment": deployment, "ReplicaSet": replicaset, "DaemonSet": daemonset, "StatefulSet": statefulset,
    "ReplicationController": replicationcontroller, "Job": job, "CronJob": cronjob,
    "HorizontalPodAutoscaler": hpa, "PodTemplate": podtemplate, "Secret": secret,
    "PersistentVolume": persistentvolume, "PersistentVolumeClaim": persistentvolumeclaim,
    "NetworkPolicy": networkpolicy,
}


def apply(kind, obj):
    """Default `obj` of `kind` in place (no-op for kinds without defaults)."""
    fn = BY_KIND.get(kind)
    if fn is not None and isinstance(obj, dict):
        fn(obj)
    return obj


__all__ = ["apply", "pod_spec", "core"]
