"""RBAC bootstrap policy: the default ClusterRoles / ClusterRoleBindings created at startup.

Parity: `plugin/pkg/auth/authorizer/rbac/bootstrappolicy/policy.go` (cluster-admin, admin, edit,
view, system:basic-user, system:discovery, system:node, system:node-bootstrapper,
system:kube-scheduler, system:kube-controller-manager, system:kube-proxy, the CSR node-client
approval roles) and `controller_policy.go`; bindings from `ClusterRoleBindings()`
(cluster-admin -> system:masters, discovery/basic-user -> system:authenticated +
system:unauthenticated, kube-scheduler / controller-manager / kube-proxy users, node-bootstrapper
-> system:bootstrappers). MI355X addition: `view` / `edit` cover the device-plugin era objects and
`system:node` may read PodSecurityPolicies and patch its own GPU capacity status.
Existing objects are never overwritten (`EnsureRBACPolicy` reconciles additively).
"""
from __future__ import annotations

from ..api import meta as m
from .registry import APIError

READ = ["get", "list", "watch"]
WRITE = ["create", "delete", "deletecollection", "patch", "update"]
CORE_WORKLOADS = ["pods", "pods/attach", "pods/exec", "pods/portforward", "pods/proxy", "replicationcontrollers",
                  "replicationcontrollers/scale", "services", "services/proxy", "endpoints", "persistentvolumeclaims",
                  "configmaps", "secrets", "serviceaccounts"]


def _r(groups, resources, verbs, **kw):
    r = {"apiGroups": groups, "resources": resources, "verbs": verbs}
    r.update(kw)
    return r


ROLES = {
    "cluster-admin": [_r(["*"], ["*"], ["*"]), {"nonResourceURLs": ["*"], "verbs": ["*"]}],
    "admin": [_r([""], CORE_WORKLOADS, READ + WRITE), _r(["apps", "extensions"], ["*"], READ + WRITE),
              _r(["batch"], ["jobs", "cronjobs"], READ + WRITE), _r(["autoscaling"], ["horizontalpodautoscalers"], READ + WRITE),
              _r(["policy"], ["poddisruptionbudgets"], READ + WRITE),
              _r(["rbac.authorization.k8s.io"], ["roles", "rolebindings"], READ + WRITE),
              _r([""], ["events", "pods/log", "pods/status", "namespaces", "resourcequotas", "limitranges"], READ),
              _r(["authorization.k8s.io"], ["localsubjectaccessreviews"], ["create"])],
    "edit": [_r([""], CORE_WORKLOADS, READ + WRITE), _r(["apps", "extensions"], ["*"], READ + WRITE),
             _r(["batch"], ["jobs", "cronjobs"], READ + WRITE), _r(["autoscaling"], ["horizontalpodautoscalers"], READ + WRITE),
             _r(["policy"], ["poddisruptionbudgets"], READ + WRITE),
             _r([""], ["events", "pods/log", "pods/status", "namespaces", "resourcequotas", "limitranges"], READ)],
    "view": [_r([""], ["pods", "replicationcontrollers", "services", "endpoints", "persistentvolumeclaims", "configmaps",
                       "serviceaccounts", "events", "pods/log", "pods/status", "namespaces", "resourcequotas", "limitranges"], READ),
             _r(["apps", "extensions", "batch", "autoscaling", "policy"], ["*"], READ)],
    "system:basic-user": [_r(["authorization.k8s.io"], ["selfsubjectaccessreviews", "selfsubjectrulesreviews"], ["create"])],
    "system:discovery": [{"nonResourceURLs": ["/healthz", "/version", "/version/", "/api", "/api/*", "/apis", "/apis/*",
                                              "/openapi", "/openapi/*", "/swagger.json", "/swaggerapi", "/swaggerapi/*"],
                          "verbs": ["get"]}],
    "system:node": [_r([""], ["nodes", "nodes/status"], READ + ["create", "update", "patch", "delete"]),
                    _r([""], ["pods"], READ + ["create", "delete"]), _r([""], ["pods/status"], ["update", "patch"]),
                    _r([""], ["events"], ["create", "patch", "update"]),
                    _r([""], ["services", "endpoints"], READ),
                    _r([""], ["secrets", "configmaps", "persistentvolumeclaims", "persistentvolumes"], ["get"]),
                    _r(["certificates.k8s.io"], ["certificatesigningrequests"], ["create", "get", "list", "watch"]),
                    _r(["authentication.k8s.io"], ["tokenreviews"], ["create"]),
                    _r(["authorization.k8s.io"], ["subjectaccessreviews", "localsubjectaccessreviews"], ["create"]),
                    _r(["policy"], ["podsecuritypolicies"], ["use"])],
    "system:node-bootstrapper": [_r(["certificates.k8s.io"], ["certificatesigningrequests"], ["create", "get", "list", "watch"])],
    "system:certificates.k8s.io:certificatesigningrequests:nodeclient": [
        _r(["certificates.k8s.io"], ["certificatesigningrequests/nodeclient"], ["create"])],
    "system:certificates.k8s.io:certificatesigningrequests:selfnodeclient": [
        _r(["certificates.k8s.io"], ["certificatesigningrequests/selfnodeclient"], ["create"])],
    "system:kube-scheduler": [_r([""], ["events"], ["create", "patch", "update"]),
                              _r([""], ["endpoints"], ["create", "get", "update"]),
                              _r([""], ["nodes", "pods", "services", "replicationcontrollers", "persistentvolumes",
                                        "persistentvolumeclaims"], READ),
                              _r([""], ["pods/binding", "bindings"], ["create"]), _r([""], ["pods/status"], ["patch", "update"]),
                              _r([""], ["pods"], ["delete"]),
                              _r(["apps", "extensions", "policy"], ["*"], READ)],
    "system:kube-controller-manager": [_r(["*"], ["*"], ["*"])],
    "system:node-proxier": [_r([""], ["services", "endpoints"], READ), _r([""], ["nodes"], ["get"]),
                            _r([""], ["events"], ["create", "patch", "update"])],
}

BINDINGS = {
    "cluster-admin": ("cluster-admin", [("Group", "system:masters")]),
    "system:discovery": ("system:discovery", [("Group", "system:authenticated"), ("Group", "system:unauthenticated")]),
    "system:basic-user": ("system:basic-user", [("Group", "system:authenticated"), ("Group", "system:unauthenticated")]),
    "system:kube-scheduler": ("system:kube-scheduler", [("User", "system:kube-scheduler")]),
    "system:kube-controller-manager": ("system:kube-controller-manager", [("User", "system:kube-controller-manager")]),
    "system:node-proxier": ("system:node-proxier", [("User", "system:kube-proxy")]),
    "system:node-bootstrapper": ("system:node-bootstrapper", [("Group", "system:bootstrappers")]),
    "kubeadm:node-autoapprove-bootstrap": ("system:certificates.k8s.io:certificatesigningrequests:nodeclient",
                                           [("Group", "system:bootstrappers")]),
    "kubeadm:node-autoapprove-certificate-rotation": ("system:certificates.k8s.io:certificatesigningrequests:selfnodeclient",
                                                      [("Group", "system:nodes")]),
}


async def ensure_bootstrap_policy(server):
    cr, crb = m.BY_PLURAL["clusterroles"], m.BY_PLURAL["clusterrolebindings"]
    ann = {"rbac.authorization.kubernetes.io/autoupdate": "true"}
    for name, rules in ROLES.items():
        if server.get_object("clusterroles", None, name) is None:
            obj = {"metadata": {"name": name, "annotations": dict(ann),
                                "labels": {"kubernetes.io/bootstrapping": "rbac-defaults"}}, "rules": rules}
            try:
                await server._retrying(lambda obj=obj: server.create(cr, None, obj, admit=False))
            except APIError as e:
                if e.code != 409:
                    raise
    for name, (role, subjects) in BINDINGS.items():
        if server.get_object("clusterrolebindings", None, name) is None:
            obj = {"metadata": {"name": name, "annotations": dict(ann),
                                "labels": {"kubernetes.io/bootstrapping": "rbac-defaults"}},
                   "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": role},
                   "subjects": [{"kind": k, "name": n, **({"apiGroup": "rbac.authorization.k8s.io"})} for k, n in subjects]}
            try:
                await server._retrying(lambda obj=obj: server.create(crb, None, obj, admit=False))
            except APIError as e:
                if e.code != 409:
                    raise
