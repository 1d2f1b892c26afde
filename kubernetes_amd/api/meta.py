"""ObjectMeta helpers, resource registry and time formatting.

Objects are plain JSON-shaped dicts in the external (v1) wire form — the same shape
`kubectl` reads and writes (reference: `staging/src/k8s.io/apimachinery/pkg/apis/meta/v1/types.go`).
There is deliberately no separate "internal" hub version: the reference converts
internal<->v1 on every request (`pkg/apis/core/v1/zz_generated.conversion.go`); we keep one
representation and save that work on the hot path.
"""
from __future__ import annotations

import copy
import datetime as _dt
import os
import time
from dataclasses import dataclass


def new_uid() -> str:
    """A random (version 4) UUID string."""
    b = bytearray(os.urandom(16))
    b[6] = (b[6] & 0x0F) | 0x40
    b[8] = (b[8] & 0x3F) | 0x80
    h = b.hex()
    return f"{h[:8]}-{h[8:12]}-{h[12:16]}-{h[16:20]}-{h[20:]}"


_NOW = [-1, ""]        # (second, its RFC 3339 text): every write stamps the current second


def now_rfc3339(t: float | None = None) -> str:
    """metav1.Time JSON form (second precision, UTC, 'Z')."""
    s = int(time.time() if t is None else t)
    if s == _NOW[0]:
        return _NOW[1]
    text = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(s))
    if t is None:
        _NOW[0], _NOW[1] = s, text
    return text


def now_rfc3339_micro(t: float | None = None) -> str:
    """metav1.MicroTime JSON form."""
    t = time.time() if t is None else t
    return _dt.datetime.fromtimestamp(t, _dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def parse_rfc3339(s: str | None) -> float | None:
    if not s:
        return None
    s = s.replace("Z", "+00:00")
    return _dt.datetime.fromisoformat(s).timestamp()


@dataclass(frozen=True)
class ResourceInfo:
    group: str
    version: str
    kind: str
    plural: str
    namespaced: bool
    short: tuple = ()

    @property
    def group_version(self) -> str:
        return f"{self.group}/{self.version}" if self.group else self.version

    @property
    def list_kind(self) -> str:
        return self.kind + "List"

    @property
    def group_resource(self) -> str:
        return f"{self.plural}.{self.group}" if self.group else self.plural


# Resources served by the API server (subset of `pkg/master/master.go:369-404` install set,
# grown as controllers land).
RESOURCES = [
    ResourceInfo("", "v1", "Pod", "pods", True, ("po",)),
    ResourceInfo("", "v1", "Node", "nodes", False, ("no",)),
    ResourceInfo("", "v1", "Namespace", "namespaces", False, ("ns",)),
    ResourceInfo("", "v1", "Event", "events", True, ("ev",)),
    ResourceInfo("", "v1", "Service", "services", True, ("svc",)),
    ResourceInfo("", "v1", "Endpoints", "endpoints", True, ("ep",)),
    ResourceInfo("", "v1", "ConfigMap", "configmaps", True, ("cm",)),
    ResourceInfo("", "v1", "Secret", "secrets", True, ()),
    ResourceInfo("", "v1", "ServiceAccount", "serviceaccounts", True, ("sa",)),
    ResourceInfo("", "v1", "ResourceQuota", "resourcequotas", True, ("quota",)),
    ResourceInfo("", "v1", "LimitRange", "limitranges", True, ("limits",)),
    ResourceInfo("", "v1", "ReplicationController", "replicationcontrollers", True, ("rc",)),
    ResourceInfo("", "v1", "PersistentVolume", "persistentvolumes", False, ("pv",)),
    ResourceInfo("", "v1", "PersistentVolumeClaim", "persistentvolumeclaims", True, ("pvc",)),
    ResourceInfo("", "v1", "PodTemplate", "podtemplates", True, ()),
    ResourceInfo("apps", "v1", "ReplicaSet", "replicasets", True, ("rs",)),
    ResourceInfo("apps", "v1", "Deployment", "deployments", True, ("deploy",)),
    ResourceInfo("apps", "v1", "DaemonSet", "daemonsets", True, ("ds",)),
    ResourceInfo("apps", "v1", "StatefulSet", "statefulsets", True, ("sts",)),
    ResourceInfo("apps", "v1", "ControllerRevision", "controllerrevisions", True, ()),
    ResourceInfo("batch", "v1", "Job", "jobs", True, ()),
    ResourceInfo("batch", "v1beta1", "CronJob", "cronjobs", True, ("cj",)),
    ResourceInfo("policy", "v1beta1", "PodDisruptionBudget", "poddisruptionbudgets", True, ("pdb",)),
    ResourceInfo("scheduling.k8s.io", "v1alpha1", "PriorityClass", "priorityclasses", False, ("pc",)),
    ResourceInfo("coordination.k8s.io", "v1", "Lease", "leases", True, ()),
    ResourceInfo("rbac.authorization.k8s.io", "v1", "Role", "roles", True, ()),
    ResourceInfo("rbac.authorization.k8s.io", "v1", "RoleBinding", "rolebindings", True, ()),
    ResourceInfo("rbac.authorization.k8s.io", "v1", "ClusterRole", "clusterroles", False, ()),
    ResourceInfo("rbac.authorization.k8s.io", "v1", "ClusterRoleBinding", "clusterrolebindings", False, ()),
    ResourceInfo("autoscaling", "v1", "HorizontalPodAutoscaler", "horizontalpodautoscalers", True, ("hpa",)),
    ResourceInfo("storage.k8s.io", "v1", "StorageClass", "storageclasses", False, ("sc",)),
    ResourceInfo("apiextensions.k8s.io", "v1beta1", "CustomResourceDefinition", "customresourcedefinitions", False, ("crd",)),
    ResourceInfo("admissionregistration.k8s.io", "v1beta1", "MutatingWebhookConfiguration",
                 "mutatingwebhookconfigurations", False, ()),
    ResourceInfo("admissionregistration.k8s.io", "v1beta1", "ValidatingWebhookConfiguration",
                 "validatingwebhookconfigurations", False, ()),
    ResourceInfo("apiregistration.k8s.io", "v1beta1", "APIService", "apiservices", False, ()),
    ResourceInfo("admissionregistration.k8s.io", "v1alpha1", "InitializerConfiguration",
                 "initializerconfigurations", False, ()),
    ResourceInfo("certificates.k8s.io", "v1beta1", "CertificateSigningRequest", "certificatesigningrequests", False, ("csr",)),
    ResourceInfo("networking.k8s.io", "v1", "NetworkPolicy", "networkpolicies", True, ("netpol",)),
    ResourceInfo("extensions", "v1beta1", "Ingress", "ingresses", True, ("ing",)),
    ResourceInfo("policy", "v1beta1", "PodSecurityPolicy", "podsecuritypolicies", False, ("psp",)),
    ResourceInfo("settings.k8s.io", "v1alpha1", "PodPreset", "podpresets", True, ()),
    ResourceInfo("storage.k8s.io", "v1beta1", "VolumeAttachment", "volumeattachments", False, ()),
    # virtual (create-only, never stored): answered from the authenticator / authorizer
    ResourceInfo("authentication.k8s.io", "v1", "TokenReview", "tokenreviews", False, ()),
    ResourceInfo("authorization.k8s.io", "v1", "SubjectAccessReview", "subjectaccessreviews", False, ()),
    ResourceInfo("authorization.k8s.io", "v1", "SelfSubjectAccessReview", "selfsubjectaccessreviews", False, ()),
    ResourceInfo("authorization.k8s.io", "v1", "LocalSubjectAccessReview", "localsubjectaccessreviews", True, ()),
]
BUILTIN = tuple(RESOURCES)          # the compiled-in resources (RESOURCES also gains CRDs)

VIRTUAL = {"tokenreviews", "subjectaccessreviews", "selfsubjectaccessreviews", "localsubjectaccessreviews"}

BY_PLURAL = {r.plural: r for r in RESOURCES}
BY_KIND = {r.kind: r for r in RESOURCES}

# Additional group/versions a resource is served under (`pkg/master/master.go` installs the
# same storage under every enabled version: e.g. Deployments under apps/v1, apps/v1beta2,
# apps/v1beta1 and extensions/v1beta1). Objects are stored once, in the canonical version;
# responses carry the requested apiVersion.
_ALIAS_TABLE = {
    ("extensions", "v1beta1"): ("deployments", "daemonsets", "replicasets", "podsecuritypolicies", "networkpolicies"),
    ("apps", "v1beta1"): ("deployments", "statefulsets", "controllerrevisions"),
    ("apps", "v1beta2"): ("deployments", "daemonsets", "replicasets", "statefulsets", "controllerrevisions"),
    ("batch", "v2alpha1"): ("cronjobs",),
    ("autoscaling", "v2beta1"): ("horizontalpodautoscalers",),
    ("rbac.authorization.k8s.io", "v1beta1"): ("roles", "rolebindings", "clusterroles", "clusterrolebindings"),
    ("rbac.authorization.k8s.io", "v1alpha1"): ("roles", "rolebindings", "clusterroles", "clusterrolebindings"),
    ("storage.k8s.io", "v1beta1"): ("storageclasses",),
    ("authentication.k8s.io", "v1beta1"): ("tokenreviews",),
    ("authorization.k8s.io", "v1beta1"): ("subjectaccessreviews", "selfsubjectaccessreviews", "localsubjectaccessreviews"),
    ("events.k8s.io", "v1beta1"): ("events",),
}
ALIASES = {(g, v, p): p for (g, v), ps in _ALIAS_TABLE.items() for p in ps}


def served_versions():
    """{group: {version, ...}} over canonical resources and aliases."""
    out = {}
    for r in RESOURCES:
        out.setdefault(r.group, set()).add(r.version)
    for (g, v, _p) in ALIASES:
        out.setdefault(g, set()).add(v)
    return out


def version_priority(v: str):
    """Kubernetes version ordering (`apimachinery/pkg/version/helpers.go`): GA > beta > alpha,
    higher major first, higher minor first — as a sort key (largest = most preferred)."""
    import re
    mt = re.fullmatch(r"v(\d+)(?:(alpha|beta)(\d+))?", v)
    if not mt:
        return (-1, 0, 0, v)
    major, kind, minor = int(mt.group(1)), mt.group(2), int(mt.group(3) or 0)
    return ({None: 2, "beta": 1, "alpha": 0}[kind], major, minor, v)


def lookup(name: str) -> ResourceInfo | None:
    """Resolve plural / singular / kind / short name (kubectl RESTMapper behaviour)."""
    n = name.lower()
    for r in RESOURCES:
        if n in (r.plural, r.kind.lower(), r.plural.rstrip("s")) or n in r.short:
            return r
    for r in RESOURCES:
        if n == r.group_resource:
            return r
    return None


def register(ri: ResourceInfo):
    """Add a resource (CRDs)."""
    if ri.plural not in BY_PLURAL:
        RESOURCES.append(ri)
    else:
        RESOURCES[:] = [r for r in RESOURCES if r.plural != ri.plural] + [ri]
    BY_PLURAL[ri.plural] = ri
    BY_KIND[ri.kind] = ri


def unregister(ri: ResourceInfo):
    if BY_PLURAL.get(ri.plural) == ri:
        del BY_PLURAL[ri.plural]
        RESOURCES[:] = [r for r in RESOURCES if r != ri]
    if BY_KIND.get(ri.kind) == ri:
        del BY_KIND[ri.kind]


def key_for(ri: ResourceInfo, namespace: str | None, name: str) -> str:
    """etcd key layout `/registry/<resource>/<ns>/<name>` (`pkg/kubeapiserver/options/storage_versions.go:29`)."""
    res = ri.plural if not ri.group or ri.group in ("apps", "batch", "policy", "") else ri.group_resource
    if ri.namespaced:
        return f"/registry/{res}/{namespace}/{name}"
    return f"/registry/{res}/{name}"


def prefix_for(ri: ResourceInfo, namespace: str | None = None) -> str:
    res = ri.plural if not ri.group or ri.group in ("apps", "batch", "policy", "") else ri.group_resource
    if ri.namespaced and namespace:
        return f"/registry/{res}/{namespace}/"
    return f"/registry/{res}/"


def meta(obj) -> dict:
    m = obj.get("metadata")
    if m is None:
        m = obj["metadata"] = {}
    return m


def name_of(obj) -> str:
    return (obj.get("metadata") or {}).get("name", "")


def namespace_of(obj) -> str:
    return (obj.get("metadata") or {}).get("namespace", "")


def uid_of(obj) -> str:
    return (obj.get("metadata") or {}).get("uid", "")


def rv_of(obj) -> int:
    v = (obj.get("metadata") or {}).get("resourceVersion")
    return int(v) if v else 0


def ns_name(obj) -> str:
    m = obj.get("metadata") or {}
    ns = m.get("namespace")
    return f"{ns}/{m.get('name', '')}" if ns else m.get("name", "")


def deepcopy(obj):
    return copy.deepcopy(obj)


def fast_copy(obj):
    """Deep copy of JSON-shaped data, ~5x faster than copy.deepcopy."""
    t = type(obj)
    if t is dict:
        return {k: fast_copy(v) for k, v in obj.items()}
    if t is list:
        return [fast_copy(v) for v in obj]
    return obj


def owner_reference(owner, controller=True, block=True) -> dict:
    ri = BY_KIND[owner["kind"]]
    return {
        "apiVersion": ri.group_version,
        "kind": owner["kind"],
        "name": name_of(owner),
        "uid": uid_of(owner),
        "controller": controller,
        "blockOwnerDeletion": block,
    }


def controller_of(obj) -> dict | None:
    for ref in (obj.get("metadata") or {}).get("ownerReferences") or []:
        if ref.get("controller"):
            return ref
    return None


def status_obj(code: int, reason: str, message: str, details=None) -> dict:
    """metav1.Status error body."""
    s = {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure",
         "message": message, "reason": reason, "code": code}
    if details:
        s["details"] = details
    return s
