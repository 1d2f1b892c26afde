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
  * Service (sessionAffinity None / ClientIP timeout, type ClusterIP, port protocol and
    targetPort, externalTrafficPolicy), Endpoints, Namespace status, Node externalID and
    allocatable, LimitRangeItem defaults from max/min, volume sources (emptyDir when none,
    iscsi/rbd/azureDisk), field refs, lifecycle httpGet: `pkg/apis/core/v1/defaults.go`;
  * StorageClass, webhook configurations (failurePolicy Ignore, empty namespaceSelector),
    RBAC binding apiGroups, CSR usages, PodSecurityPolicy allowPrivilegeEscalation: their
    groups' `defaults.go`;
  * Secret / PV / PVC small defaults.
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
    for e in c.get("env") or ():
        fr = ((e or {}).get("valueFrom") or {}).get("fieldRef")
        if isinstance(fr, dict):
            _default(fr, "apiVersion", "v1")                  # SetDefaults_ObjectFieldSelector
    for h in ((c.get("lifecycle") or {}).get("postStart"), (c.get("lifecycle") or {}).get("preStop")):
        if isinstance(h, dict) and isinstance(h.get("httpGet"), dict):
            _default(h["httpGet"], "path", "/")               # SetDefaults_HTTPGetAction
            _default(h["httpGet"], "scheme", "HTTP")
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
        if not any(k != "name" and isinstance(val, dict) for k, val in v.items()):
            v["emptyDir"] = {}                                  # SetDefaults_Volume
        if isinstance(v.get("iscsi"), dict):
            _default(v["iscsi"], "iscsiInterface", "default")
        if isinstance(v.get("rbd"), dict):
            for k, d in (("pool", "rbd"), ("user", "admin"), ("keyring", "/etc/ceph/keyring")):
                _default(v["rbd"], k, d)
        if isinstance(v.get("azureDisk"), dict):
            for k, d in (("cachingMode", "ReadWrite"), ("kind", "Shared"), ("fsType", "ext4"), ("readOnly", False)):
                _default(v["azureDisk"], k, d)
        for item in (v.get("downwardAPI") or {}).get("items") or () if isinstance(v.get("downwardAPI"), dict) else ():
            if isinstance(item.get("fieldRef"), dict):
                _default(item["fieldRef"], "apiVersion", "v1")


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


def service(obj):
    """SetDefaults_Service (core/v1/defaults.go:94-130)."""
    spec = obj.setdefault("spec", {})
    _default(spec, "sessionAffinity", "None")
    if spec["sessionAffinity"] == "None":
        spec.pop("sessionAffinityConfig", None)
    elif spec["sessionAffinity"] == "ClientIP":
        cfg = spec.get("sessionAffinityConfig") or {}
        if (cfg.get("clientIP") or {}).get("timeoutSeconds") is None:
            spec["sessionAffinityConfig"] = {"clientIP": {"timeoutSeconds": 10800}}   # 3 hours
    _default(spec, "type", "ClusterIP")
    for p in spec.get("ports") or ():
        if not isinstance(p, dict):
            continue
        _default(p, "protocol", "TCP")
        if p.get("targetPort") in (None, 0, "") and p.get("port") is not None:
            p["targetPort"] = p["port"]
    if spec["type"] in ("NodePort", "LoadBalancer"):
        _default(spec, "externalTrafficPolicy", "Cluster")


def endpoints(obj):
    """SetDefaults_Endpoints: port protocol TCP."""
    for ss in obj.get("subsets") or ():
        for p in (ss or {}).get("ports") or ():
            _default(p, "protocol", "TCP")


def namespace(obj):
    """SetDefaults_NamespaceStatus: phase Active."""
    _default(obj.setdefault("status", {}), "phase", "Active")


def node(obj):
    """SetDefaults_Node (externalID = name) and SetDefaults_NodeStatus (allocatable = capacity)."""
    spec = obj.setdefault("spec", {})
    if not spec.get("externalID") and (obj.get("metadata") or {}).get("name"):
        spec["externalID"] = obj["metadata"]["name"]
    st = obj.get("status")
    if isinstance(st, dict) and st.get("allocatable") is None and st.get("capacity") is not None:
        st["allocatable"] = dict(st["capacity"])


def limitrange(obj):
    """SetDefaults_LimitRangeItem: for Container items, default <- max, defaultRequest <- default,
    then defaultRequest <- min, key by key where unset."""
    for item in (obj.get("spec") or {}).get("limits") or ():
        if item.get("type") != "Container":
            continue
        dflt = item.setdefault("default", {}) if item.get("default") is None else item["default"]
        dreq = item.setdefault("defaultRequest", {}) if item.get("defaultRequest") is None else item["defaultRequest"]
        for k, v in (item.get("max") or {}).items():
            dflt.setdefault(k, v)
        for k, v in dflt.items():
            dreq.setdefault(k, v)
        for k, v in (item.get("min") or {}).items():
            dreq.setdefault(k, v)


def storageclass(obj):
    """storage/v1 SetDefaults_StorageClass: reclaimPolicy Delete, volumeBindingMode Immediate."""
    _default(obj, "reclaimPolicy", "Delete")
    _default(obj, "volumeBindingMode", "Immediate")


def webhook_configuration(obj):
    """admissionregistration/v1beta1 SetDefaults_Webhook: failurePolicy Ignore, an empty
    (match-everything) namespaceSelector."""
    for w in obj.get("webhooks") or ():
        if isinstance(w, dict):
            _default(w, "failurePolicy", "Ignore")
            _default(w, "namespaceSelector", {})


def _rbac_subjects(obj):
    """rbac/v1 SetDefaults_Subject: User / Group subjects get apiGroup rbac.authorization.k8s.io;
    SetDefaults_(Cluster)RoleBinding: roleRef apiGroup likewise."""
    rr = obj.get("roleRef")
    if isinstance(rr, dict) and not rr.get("apiGroup"):
        rr["apiGroup"] = "rbac.authorization.k8s.io"
    for sub in obj.get("subjects") or ():
        if isinstance(sub, dict) and not sub.get("apiGroup") and sub.get("kind") in ("User", "Group"):
            sub["apiGroup"] = "rbac.authorization.k8s.io"


def csr(obj):
    """certificates/v1beta1 SetDefaults_CertificateSigningRequestSpec: usages."""
    spec = obj.setdefault("spec", {})
    if not spec.get("usages"):
        spec["usages"] = ["digital signature", "key encipherment"]


def psp(obj):
    """extensions/v1beta1 SetDefaults_PodSecurityPolicySpec: allowPrivilegeEscalation true."""
    _default(obj.setdefault("spec", {}), "allowPrivilegeEscalation", True)



BY_KIND = {
    "Pod": pod, "Deployment": deployment, "ReplicaSet": replicaset, "DaemonSet": daemonset, "StatefulSet": statefulset,
    "ReplicationController": replicationcontroller, "Job": job, "CronJob": cronjob,
    "HorizontalPodAutoscaler": hpa, "PodTemplate": podtemplate, "Secret": secret,
    "PersistentVolume": persistentvolume, "PersistentVolumeClaim": persistentvolumeclaim,
    "NetworkPolicy": networkpolicy, "Service": service, "Endpoints": endpoints, "Namespace": namespace,
    "Node": node, "LimitRange": limitrange, "StorageClass": storageclass,
    "MutatingWebhookConfiguration": webhook_configuration, "ValidatingWebhookConfiguration": webhook_configuration,
    "RoleBinding": _rbac_subjects, "ClusterRoleBinding": _rbac_subjects,
    "CertificateSigningRequest": csr, "PodSecurityPolicy": psp,
}


def apply(kind, obj):
    """Default `obj` of `kind` in place (no-op for kinds without defaults)."""
    fn = BY_KIND.get(kind)
    if fn is not None and isinstance(obj, dict):
        fn(obj)
    return obj


__all__ = ["apply", "pod_spec", "core"]