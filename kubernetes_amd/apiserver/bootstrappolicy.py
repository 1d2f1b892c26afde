"""RBAC bootstrap policy: the default ClusterRoles / ClusterRoleBindings / kube-system Roles the
API server reconciles at startup.

Parity (`plugin/pkg/auth/authorizer/rbac/bootstrappolicy/`):
  * `policy.go:155-457` ClusterRoles — cluster-admin, system:discovery, system:basic-user, the
    aggregated admin / edit / view (`aggregationRule` over `aggregate-to-*` labels) with their
    system:aggregate-to-admin / -edit / -view parts, system:heapster, system:node,
    system:node-problem-detector, system:node-proxier, system:node-bootstrapper,
    system:auth-delegator, system:kube-aggregator, system:kube-controller-manager (events,
    SA/secret/endpoint bootstrap and read-only shared informers — NOT `*/*/*`),
    system:kube-scheduler (+ the VolumeScheduling rules), system:kube-dns,
    system:persistent-volume-provisioner, the CSR node-client approval roles;
  * `policy.go:460-486` ClusterRoleBindings (system:node bound to nobody: the Node authorizer
    authorizes kubelets);
  * `controller_policy.go:60-336` one `system:controller:<name>` ClusterRole per controller,
    bound to the `kube-system/<name>` service account the controller manager runs that
    controller as with `--use-service-account-credentials` (`controllermanager.go:133-139`);
  * `namespace_policy.go:72-143` kube-system / kube-public Roles and RoleBindings (the
    extension-apiserver authentication reader, bootstrap signer, token cleaner, leader locks).

MI355X additions, marked where they appear: the kubelet (system:node) may `use` pod security
policies and patch pod status; the kube-scheduler may hold its per-shard leader locks
(`kube-scheduler-shard-<i>`); a csi-attacher controller role for the in-tree external attacher.
Existing objects are never overwritten (`EnsureRBACPolicy` reconciles additively); the
aggregated roles are created with their aggregated rules already filled in, so they work
before the clusterroleaggregation controller first runs.
"""
from __future__ import annotations

from ..api import meta as m
from .registry import APIError

READ = ["get", "list", "watch"]
READ_WRITE = ["get", "list", "watch", "create", "update", "patch", "delete", "deletecollection"]
CORE, APPS, EXT, BATCH, AUTOSCALING, POLICY = "", "apps", "extensions", "batch", "autoscaling", "policy"
RBAC, STORAGE, CERTS = "rbac.authorization.k8s.io", "storage.k8s.io", "certificates.k8s.io"
AUTHN, AUTHZ = "authentication.k8s.io", "authorization.k8s.io"
CONTROLLER_PREFIX = "system:controller:"
AGGREGATE_LABEL = "rbac.authorization.k8s.io/aggregate-to-"
BOOTSTRAP_LABELS = {"kubernetes.io/bootstrapping": "rbac-defaults"}


def rule(verbs, groups, resources, names=None):
    r = {"apiGroups": list(groups), "resources": list(resources), "verbs": list(verbs)}
    if names:
        r["resourceNames"] = list(names)
    return r


def urls(verbs, paths):
    return {"nonResourceURLs": list(paths), "verbs": list(verbs)}


def events_rule():
    return rule(["create", "update", "patch"], [CORE], ["events"])


# -- the namespace-scoped user roles (aggregated into admin / edit / view) ---------------------
_WORKLOADS_RW = [
    rule(READ_WRITE, [CORE], ["pods", "pods/attach", "pods/proxy", "pods/exec", "pods/portforward"]),
    rule(READ_WRITE, [CORE], ["replicationcontrollers", "replicationcontrollers/scale", "serviceaccounts", "services",
                              "services/proxy", "endpoints", "persistentvolumeclaims", "configmaps", "secrets"]),
]
_STATUS_READ = rule(READ, [CORE], ["limitranges", "resourcequotas", "bindings", "events", "pods/status",
                                   "resourcequotas/status", "namespaces/status", "replicationcontrollers/status",
                                   "pods/log"])
_GROUPS_RW = [
    rule(READ_WRITE, [APPS], ["statefulsets", "daemonsets", "deployments", "deployments/scale", "deployments/rollback",
                              "replicasets", "replicasets/scale"]),
    rule(READ_WRITE, [AUTOSCALING], ["horizontalpodautoscalers"]),
    rule(READ_WRITE, [BATCH], ["jobs", "cronjobs"]),
    rule(READ_WRITE, [EXT], ["daemonsets", "deployments", "deployments/scale", "deployments/rollback", "ingresses",
                             "replicasets", "replicasets/scale", "replicationcontrollers/scale"]),
    rule(READ_WRITE, [POLICY], ["poddisruptionbudgets"]),
]
AGGREGATE_TO_EDIT = _WORKLOADS_RW + [
    _STATUS_READ,
    rule(READ, [CORE], ["namespaces"]),
    rule(["impersonate"], [CORE], ["serviceaccounts"]),
] + _GROUPS_RW
AGGREGATE_TO_ADMIN = AGGREGATE_TO_EDIT + [
    rule(["create"], [AUTHZ], ["localsubjectaccessreviews"]),
    rule(READ_WRITE, [RBAC], ["roles", "rolebindings"]),
]
AGGREGATE_TO_VIEW = [
    rule(READ, [CORE], ["pods", "replicationcontrollers", "replicationcontrollers/scale", "serviceaccounts", "services",
                        "endpoints", "persistentvolumeclaims", "configmaps"]),
    _STATUS_READ,
    rule(READ, [CORE], ["namespaces"]),
    rule(READ, [APPS], ["statefulsets", "daemonsets", "deployments", "deployments/scale", "replicasets",
                        "replicasets/scale"]),
    rule(READ, [AUTOSCALING], ["horizontalpodautoscalers"]),
    rule(READ, [BATCH], ["jobs", "cronjobs"]),
    rule(READ, [EXT], ["daemonsets", "deployments", "deployments/scale", "ingresses", "replicasets",
                       "replicasets/scale", "replicationcontrollers/scale"]),
    rule(READ, [POLICY], ["poddisruptionbudgets"]),
]
AGGREGATED = {"admin": ("system:aggregate-to-admin", AGGREGATE_TO_ADMIN),
              "edit": ("system:aggregate-to-edit", AGGREGATE_TO_EDIT),
              "view": ("system:aggregate-to-view", AGGREGATE_TO_VIEW)}


def node_rules():
    """`policy.go:92-150` NodeRules (+ the ExpandPersistentVolumes / CSI rules; MI355X/local:
    PodSecurityPolicy `use`, pod status patches)."""
    return [
        rule(["create"], [AUTHN], ["tokenreviews"]),
        rule(["create"], [AUTHZ], ["subjectaccessreviews", "localsubjectaccessreviews"]),
        rule(READ, [CORE], ["services"]),
        rule(["create", "get", "list", "watch"], [CORE], ["nodes"]),
        rule(["update", "patch"], [CORE], ["nodes/status"]),
        rule(["update", "patch", "delete"], [CORE], ["nodes"]),
        rule(["create", "update", "patch"], [CORE], ["events"]),
        rule(READ, [CORE], ["pods"]),
        rule(["create", "delete"], [CORE], ["pods"]),
        rule(["update", "patch"], [CORE], ["pods/status"]),
        rule(["create"], [CORE], ["pods/eviction"]),
        rule(["get"], [CORE], ["secrets", "configmaps"]),
        rule(["get"], [CORE], ["persistentvolumeclaims", "persistentvolumes"]),
        rule(["get"], [CORE], ["endpoints"]),
        rule(["create", "get", "list", "watch"], [CERTS], ["certificatesigningrequests"]),
        rule(["get", "update", "patch"], [CORE], ["persistentvolumeclaims/status"]),
        rule(["get"], [STORAGE], ["volumeattachments"]),
        rule(["use"], [POLICY, EXT], ["podsecuritypolicies"]),
    ]


SCHEDULER_LOCKS = ["kube-scheduler"] + [f"kube-scheduler-shard-{i}" for i in range(64)]

CLUSTER_ROLES = {
    "cluster-admin": [rule(["*"], ["*"], ["*"]), urls(["*"], ["*"])],
    "system:discovery": [urls(["get"], ["/healthz", "/version", "/version/", "/swaggerapi", "/swaggerapi/*",
                                        "/swagger.json", "/swagger-2.0.0.pb-v1", "/openapi", "/openapi/*",
                                        "/api", "/api/*", "/apis", "/apis/*"])],
    "system:basic-user": [rule(["create"], [AUTHZ], ["selfsubjectaccessreviews", "selfsubjectrulesreviews"])],
    "system:aggregate-to-admin": AGGREGATE_TO_ADMIN,
    "system:aggregate-to-edit": AGGREGATE_TO_EDIT,
    "system:aggregate-to-view": AGGREGATE_TO_VIEW,
    "system:heapster": [rule(READ, [CORE], ["events", "pods", "nodes", "namespaces"]),
                        rule(READ, [EXT], ["deployments"])],
    "system:node": node_rules(),
    "system:node-problem-detector": [rule(["get"], [CORE], ["nodes"]), rule(["patch"], [CORE], ["nodes/status"]),
                                     events_rule()],
    "system:node-proxier": [rule(["list", "watch"], [CORE], ["services", "endpoints"]), rule(["get"], [CORE], ["nodes"]),
                            events_rule()],
    "system:node-bootstrapper": [rule(["create", "get", "list", "watch"], [CERTS], ["certificatesigningrequests"])],
    "system:auth-delegator": [rule(["create"], [AUTHN], ["tokenreviews"]),
                              rule(["create"], [AUTHZ], ["subjectaccessreviews"])],
    "system:kube-aggregator": [rule(READ, [CORE], ["services", "endpoints"])],
    "system:kube-controller-manager": [
        events_rule(),
        rule(["create"], [CORE], ["endpoints", "secrets", "serviceaccounts"]),
        rule(["delete"], [CORE], ["secrets"]),
        rule(["get"], [CORE], ["endpoints", "namespaces", "secrets", "serviceaccounts"]),
        rule(["update"], [CORE], ["endpoints", "secrets", "serviceaccounts"]),
        rule(["create"], [AUTHN], ["tokenreviews"]),
        rule(["list", "watch"], ["*"], ["*"]),
    ],
    "system:kube-scheduler": [
        events_rule(),
        rule(["create"], [CORE], ["endpoints"]),
        rule(["get", "update", "patch", "delete"], [CORE], ["endpoints"], SCHEDULER_LOCKS),
        rule(READ, [CORE], ["nodes"]),
        rule(["get", "list", "watch", "delete"], [CORE], ["pods"]),
        rule(["create"], [CORE], ["pods/binding", "bindings"]),
        rule(["patch", "update"], [CORE], ["pods/status"]),
        rule(READ, [CORE], ["services", "replicationcontrollers"]),
        rule(READ, [APPS, EXT], ["replicasets"]),
        rule(READ, [APPS], ["statefulsets"]),
        rule(READ, [POLICY], ["poddisruptionbudgets"]),
        rule(READ, [CORE], ["persistentvolumeclaims", "persistentvolumes"]),
        rule(["update"], [CORE], ["persistentvolumes"]),           # VolumeScheduling
        rule(READ, [STORAGE], ["storageclasses"]),
    ],
    "system:kube-dns": [rule(["list", "watch"], [CORE], ["endpoints", "services"])],
    "system:persistent-volume-provisioner": [
        rule(["get", "list", "watch", "create", "delete"], [CORE], ["persistentvolumes"]),
        rule(["get", "list", "watch", "update"], [CORE], ["persistentvolumeclaims"]),
        rule(READ, [STORAGE], ["storageclasses"]),
        rule(["watch"], [CORE], ["events"]),
        events_rule(),
    ],
    "system:certificates.k8s.io:certificatesigningrequests:nodeclient": [
        rule(["create"], [CERTS], ["certificatesigningrequests/nodeclient"])],
    "system:certificates.k8s.io:certificatesigningrequests:selfnodeclient": [
        rule(["create"], [CERTS], ["certificatesigningrequests/selfnodeclient"])],
    "system:certificates.k8s.io:certificatesigningrequests:selfnodeserver": [
        rule(["create"], [CERTS], ["certificatesigningrequests/selfnodeserver"])],
}

# `controller_policy.go`: role name (after system:controller:) -> rules; each is bound to the
# kube-system service account of the same name
CONTROLLER_ROLES = {
    "attachdetach-controller": [
        rule(["list", "watch"], [CORE], ["persistentvolumes", "persistentvolumeclaims"]),
        rule(READ, [CORE], ["nodes"]), rule(["patch", "update"], [CORE], ["nodes/status"]),
        rule(["list", "watch"], [CORE], ["pods"]), events_rule(),
        rule(["get", "create", "delete", "list", "watch"], [STORAGE], ["volumeattachments"])],
    "clusterrole-aggregation-controller": [rule(["*"], ["*"], ["*"]), urls(["*"], ["*"])],
    "cronjob-controller": [
        rule(["get", "list", "watch", "update"], [BATCH], ["cronjobs"]),
        rule(["get", "list", "watch", "create", "update", "delete", "patch"], [BATCH], ["jobs"]),
        rule(["update"], [BATCH], ["cronjobs/status"]), rule(["update"], [BATCH], ["cronjobs/finalizers"]),
        rule(["list", "delete"], [CORE], ["pods"]), events_rule()],
    "daemon-set-controller": [
        rule(READ, [EXT, APPS], ["daemonsets"]), rule(["update"], [EXT, APPS], ["daemonsets/status"]),
        rule(["update"], [EXT, APPS], ["daemonsets/finalizers"]), rule(["list", "watch"], [CORE], ["nodes"]),
        rule(["list", "watch", "create", "delete", "patch"], [CORE], ["pods"]),
        rule(["create"], [CORE], ["pods/binding"]),
        rule(["get", "list", "watch", "create", "delete", "update", "patch"], [APPS], ["controllerrevisions"]),
        events_rule()],
    "deployment-controller": [
        rule(["get", "list", "watch", "update"], [EXT, APPS], ["deployments"]),
        rule(["update"], [EXT, APPS], ["deployments/status"]), rule(["update"], [EXT, APPS], ["deployments/finalizers"]),
        rule(["get", "list", "watch", "create", "update", "patch", "delete"], [APPS, EXT], ["replicasets"]),
        rule(["get", "list", "watch", "update"], [CORE], ["pods"]), events_rule()],
    "disruption-controller": [
        rule(READ, [EXT, APPS], ["deployments"]), rule(READ, [APPS, EXT], ["replicasets"]),
        rule(READ, [CORE], ["replicationcontrollers"]), rule(READ, [POLICY], ["poddisruptionbudgets"]),
        rule(READ, [APPS], ["statefulsets"]), rule(["update"], [POLICY], ["poddisruptionbudgets/status"]),
        events_rule()],
    "endpoint-controller": [
        rule(READ, [CORE], ["services", "pods"]),
        rule(["get", "list", "create", "update", "delete"], [CORE], ["endpoints"]),
        rule(["create"], [CORE], ["endpoints/restricted"]), events_rule()],
    "expand-controller": [
        rule(["get", "list", "watch", "update", "patch"], [CORE], ["persistentvolumes"]),
        rule(["update", "patch"], [CORE], ["persistentvolumeclaims/status"]),
        rule(READ, [CORE], ["persistentvolumeclaims"]), rule(READ, [STORAGE], ["storageclasses"]),
        rule(["get"], [CORE], ["services", "endpoints"]), rule(["get"], [CORE], ["secrets"]), events_rule()],
    "generic-garbage-collector": [rule(["get", "list", "watch", "patch", "update", "delete"], ["*"], ["*"]),
                                  events_rule()],
    "horizontal-pod-autoscaler": [
        rule(READ, [AUTOSCALING], ["horizontalpodautoscalers"]),
        rule(["update"], [AUTOSCALING], ["horizontalpodautoscalers/status"]),
        rule(["get", "update"], ["*"], ["*/scale"]), rule(["list"], [CORE], ["pods"]),
        rule(["get"], [CORE], ["services/proxy"], ["https:heapster:", "http:heapster:"]),
        rule(["list"], ["metrics.k8s.io"], ["pods"]), rule(["get", "list"], ["custom.metrics.k8s.io"], ["*"]),
        events_rule()],
    "job-controller": [
        rule(["get", "list", "watch", "update"], [BATCH], ["jobs"]), rule(["update"], [BATCH], ["jobs/status"]),
        rule(["update"], [BATCH], ["jobs/finalizers"]),
        rule(["list", "watch", "create", "delete", "patch"], [CORE], ["pods"]), events_rule()],
    "namespace-controller": [
        rule(["get", "list", "watch", "delete"], [CORE], ["namespaces"]),
        rule(["update"], [CORE], ["namespaces/finalize", "namespaces/status"]),
        rule(["get", "list", "delete", "deletecollection"], ["*"], ["*"])],
    "node-controller": [
        rule(["get", "list", "update", "delete", "patch"], [CORE], ["nodes"]),
        rule(["patch", "update"], [CORE], ["nodes/status"]), rule(["update"], [CORE], ["pods/status"]),
        rule(["list", "delete"], [CORE], ["pods"]), events_rule()],
    "persistent-volume-binder": [
        rule(["get", "list", "watch", "update", "create", "delete"], [CORE], ["persistentvolumes"]),
        rule(["update"], [CORE], ["persistentvolumes/status"]),
        rule(["get", "list", "watch", "update"], [CORE], ["persistentvolumeclaims"]),
        rule(["update"], [CORE], ["persistentvolumeclaims/status"]),
        rule(["list", "watch", "get", "create", "delete"], [CORE], ["pods"]),
        rule(READ, [STORAGE], ["storageclasses"]),
        rule(["get", "create", "delete"], [CORE], ["services", "endpoints"]), rule(["get"], [CORE], ["secrets"]),
        rule(["get", "list"], [CORE], ["nodes"]), rule(["watch"], [CORE], ["events"]), events_rule()],
    "pod-garbage-collector": [rule(["list", "watch", "delete"], [CORE], ["pods"]), rule(["list"], [CORE], ["nodes"])],
    "replicaset-controller": [
        rule(["get", "list", "watch", "update"], [APPS, EXT], ["replicasets"]),
        rule(["update"], [APPS, EXT], ["replicasets/status"]), rule(["update"], [APPS, EXT], ["replicasets/finalizers"]),
        rule(["list", "watch", "patch", "create", "delete"], [CORE], ["pods"]), events_rule()],
    "replication-controller": [
        rule(["get", "list", "watch", "update"], [CORE], ["replicationcontrollers"]),
        rule(["update"], [CORE], ["replicationcontrollers/status"]),
        rule(["update"], [CORE], ["replicationcontrollers/finalizers"]),
        rule(["list", "watch", "patch", "create", "delete"], [CORE], ["pods"]), events_rule()],
    "resourcequota-controller": [rule(["list", "watch"], ["*"], ["*"]),
                                 rule(["update"], [CORE], ["resourcequotas/status"]), events_rule()],
    "route-controller": [rule(["list", "watch"], [CORE], ["nodes"]), rule(["patch"], [CORE], ["nodes/status"]),
                         events_rule()],
    "service-account-controller": [rule(["create"], [CORE], ["serviceaccounts"]), events_rule()],
    "service-controller": [rule(READ, [CORE], ["services"]), rule(["update"], [CORE], ["services/status"]),
                           rule(["list", "watch"], [CORE], ["nodes"]), events_rule()],
    "statefulset-controller": [
        rule(["list", "watch"], [CORE], ["pods"]), rule(READ, [APPS], ["statefulsets"]),
        rule(["update"], [APPS], ["statefulsets/status"]), rule(["update"], [APPS], ["statefulsets/finalizers"]),
        rule(["get", "create", "delete", "update", "patch"], [CORE], ["pods"]),
        rule(["get", "create", "delete", "update", "patch", "list", "watch"], [APPS], ["controllerrevisions"]),
        rule(["get", "create"], [CORE], ["persistentvolumeclaims"]), events_rule()],
    "ttl-controller": [rule(["update", "patch", "list", "watch"], [CORE], ["nodes"]), events_rule()],
    "certificate-controller": [
        # + delete: the CSR cleaner runs as this account too (the 1.9 role lacks it, so the
        # reference's cleaner is refused under --use-service-account-credentials; later
        # releases add it)
        rule(READ + ["delete"], [CERTS], ["certificatesigningrequests"]),
        rule(["update"], [CERTS], ["certificatesigningrequests/status", "certificatesigningrequests/approval"]),
        rule(["create"], [AUTHZ], ["subjectaccessreviews"]), events_rule()],
    "pvc-protection-controller": [rule(["get", "list", "watch", "update"], [CORE], ["persistentvolumeclaims"]),
                                  rule(["list", "watch", "get"], [CORE], ["pods"]), events_rule()],
    "pv-protection-controller": [rule(["get", "list", "watch", "update"], [CORE], ["persistentvolumes"]),
                                 events_rule()],
    # MI355X/local: the in-tree external CSI attacher (out of tree in the reference, with its own SA)
    "csi-attacher": [rule(["get", "list", "watch", "update", "patch"], [STORAGE],
                          ["volumeattachments", "volumeattachments/status"]),
                     rule(READ, [CORE], ["persistentvolumes", "nodes"]), events_rule()],
}


def _update_implies_patch(rules):
    """Local deviation, applied to the controller roles only: these controllers write status and
    metadata with merge patches instead of read-modify-update (no conflict retries), so every
    rule that grants `update` also grants `patch` — the same authority over the same objects."""
    out = []
    for r in rules:
        v = r.get("verbs") or []
        if "update" in v and "patch" not in v:
            r = dict(r, verbs=v + ["patch"])
        out.append(r)
    return out


CONTROLLER_ROLES = {name: _update_implies_patch(rules) for name, rules in CONTROLLER_ROLES.items()}

CLUSTER_ROLE_BINDINGS = {
    "cluster-admin": ("cluster-admin", [("Group", "system:masters")]),
    "system:discovery": ("system:discovery", [("Group", "system:authenticated"), ("Group", "system:unauthenticated")]),
    "system:basic-user": ("system:basic-user", [("Group", "system:authenticated"), ("Group", "system:unauthenticated")]),
    "system:node-proxier": ("system:node-proxier", [("User", "system:kube-proxy")]),
    "system:kube-controller-manager": ("system:kube-controller-manager", [("User", "system:kube-controller-manager")]),
    "system:kube-dns": ("system:kube-dns", [("ServiceAccount", "kube-system/kube-dns")]),
    "system:kube-scheduler": ("system:kube-scheduler", [("User", "system:kube-scheduler")]),
    # deprecated since the Node authorizer: kept, with no subjects (policy.go:476-481)
    "system:node": ("system:node", []),
    "system:node-bootstrapper": ("system:node-bootstrapper", [("Group", "system:bootstrappers")]),
    "kubeadm:node-autoapprove-bootstrap": ("system:certificates.k8s.io:certificatesigningrequests:nodeclient",
                                           [("Group", "system:bootstrappers")]),
    "kubeadm:node-autoapprove-certificate-rotation": ("system:certificates.k8s.io:certificatesigningrequests:selfnodeclient",
                                                      [("Group", "system:nodes")]),
}
for _n in CONTROLLER_ROLES:
    CLUSTER_ROLE_BINDINGS[CONTROLLER_PREFIX + _n] = (CONTROLLER_PREFIX + _n, [("ServiceAccount", f"kube-system/{_n}")])

# `namespace_policy.go`: namespace -> {role: rules}, namespace -> {binding: (role, subjects)}
NAMESPACE_ROLES = {
    "kube-system": {
        "extension-apiserver-authentication-reader": [
            rule(["get"], [CORE], ["configmaps"], ["extension-apiserver-authentication"])],
        CONTROLLER_PREFIX + "bootstrap-signer": [rule(READ, [CORE], ["secrets"])],
        CONTROLLER_PREFIX + "cloud-provider": [rule(["create", "get", "list", "watch"], [CORE], ["configmaps"])],
        CONTROLLER_PREFIX + "token-cleaner": [rule(["get", "list", "watch", "delete"], [CORE], ["secrets"]),
                                              events_rule()],
        "system::leader-locking-kube-controller-manager": [
            rule(["watch"], [CORE], ["configmaps"]),
            rule(["get", "update"], [CORE], ["configmaps"], ["kube-controller-manager"])],
        "system::leader-locking-kube-scheduler": [
            rule(["watch"], [CORE], ["configmaps"]),
            rule(["get", "update"], [CORE], ["configmaps"], ["kube-scheduler"])],
    },
    "kube-public": {
        CONTROLLER_PREFIX + "bootstrap-signer": [
            rule(READ, [CORE], ["configmaps"]), rule(["update"], [CORE], ["configmaps"], ["cluster-info"]),
            events_rule()],
    },
}
NAMESPACE_ROLE_BINDINGS = {
    "kube-system": {
        "system::leader-locking-kube-controller-manager": (
            "system::leader-locking-kube-controller-manager", [("ServiceAccount", "kube-system/kube-controller-manager")]),
        "system::leader-locking-kube-scheduler": (
            "system::leader-locking-kube-scheduler", [("ServiceAccount", "kube-system/kube-scheduler")]),
        CONTROLLER_PREFIX + "bootstrap-signer": (CONTROLLER_PREFIX + "bootstrap-signer",
                                                 [("ServiceAccount", "kube-system/bootstrap-signer")]),
        CONTROLLER_PREFIX + "cloud-provider": (CONTROLLER_PREFIX + "cloud-provider",
                                               [("ServiceAccount", "kube-system/cloud-provider")]),
        CONTROLLER_PREFIX + "token-cleaner": (CONTROLLER_PREFIX + "token-cleaner",
                                              [("ServiceAccount", "kube-system/token-cleaner")]),
    },
    "kube-public": {
        CONTROLLER_PREFIX + "bootstrap-signer": (CONTROLLER_PREFIX + "bootstrap-signer",
                                                 [("ServiceAccount", "kube-system/bootstrap-signer")]),
    },
}


def _subject(kind, name):
    if kind == "ServiceAccount":
        ns, sa = name.split("/", 1)
        return {"kind": "ServiceAccount", "name": sa, "namespace": ns}
    return {"kind": kind, "name": name, "apiGroup": RBAC}


def _meta(name, namespace=None, labels=None):
    md = {"name": name, "annotations": {"rbac.authorization.kubernetes.io/autoupdate": "true"},
          "labels": dict(BOOTSTRAP_LABELS, **(labels or {}))}
    if namespace:
        md["namespace"] = namespace
    return md


def cluster_roles():
    """name -> ClusterRole object (without kind/apiVersion)."""
    out = {}
    for name, rules in CLUSTER_ROLES.items():
        labels = None
        for agg, (part, _) in AGGREGATED.items():
            if part == name:
                labels = {AGGREGATE_LABEL + agg: "true"}
        out[name] = {"metadata": _meta(name, labels=labels), "rules": rules}
    for agg, (_, rules) in AGGREGATED.items():
        out[agg] = {"metadata": _meta(agg),
                    "aggregationRule": {"clusterRoleSelectors": [{"matchLabels": {AGGREGATE_LABEL + agg: "true"}}]},
                    "rules": list(rules)}
    for name, rules in CONTROLLER_ROLES.items():
        out[CONTROLLER_PREFIX + name] = {"metadata": _meta(CONTROLLER_PREFIX + name), "rules": rules}
    return out


def cluster_role_bindings():
    return {name: {"metadata": _meta(name),
                   "roleRef": {"apiGroup": RBAC, "kind": "ClusterRole", "name": role},
                   "subjects": [_subject(k, n) for k, n in subjects]}
            for name, (role, subjects) in CLUSTER_ROLE_BINDINGS.items()}


def namespace_roles():
    return {(ns, name): {"metadata": _meta(name, ns), "rules": rules}
            for ns, roles in NAMESPACE_ROLES.items() for name, rules in roles.items()}


def namespace_role_bindings():
    return {(ns, name): {"metadata": _meta(name, ns),
                         "roleRef": {"apiGroup": RBAC, "kind": "Role", "name": role},
                         "subjects": [_subject(k, n) for k, n in subjects]}
            for ns, bs in NAMESPACE_ROLE_BINDINGS.items() for name, (role, subjects) in bs.items()}


async def ensure_bootstrap_policy(server):
    """Create whatever default policy object is missing; never overwrite an existing one."""
    async def ensure(plural, ns, name, obj):
        if server.get_object(plural, ns, name) is not None:
            return
        try:
            await server._retrying(lambda: server.create(m.BY_PLURAL[plural], ns, obj, admit=False))
        except APIError as e:
            if e.code != 409:
                raise
    for name, obj in cluster_roles().items():
        await ensure("clusterroles", None, name, obj)
    for name, obj in cluster_role_bindings().items():
        await ensure("clusterrolebindings", None, name, obj)
    for (ns, name), obj in namespace_roles().items():
        await ensure("roles", ns, name, obj)
    for (ns, name), obj in namespace_role_bindings().items():
        await ensure("rolebindings", ns, name, obj)
