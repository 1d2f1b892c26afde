"""Built-in admission plugins.

  * ResourceV2 — the fork's device-request normaliser
    (`plugin/pkg/admission/resourcev2/admission.go:32-118`), keyed to `amd.com/gpu` and
    configurable (the reference hard-codes `nvidia.com/gpu` at :64,79).
  * ResourceQuota — also counts pod-level ExtendedResources, closing the reference's gap
    where GPU quota went unenforced after ResourceV2 stripped container limits
    (`pkg/quota/evaluator/core/pods.go:299-335`).
  * LimitRanger — `limitranger.py`.
  * NamespaceLifecycle, ServiceAccount, DefaultTolerationSeconds, Priority,
    ExtendedResourceToleration, NodeRestriction, AlwaysPullImages, AlwaysAdmit, AlwaysDeny,
    PodNodeSelector — per `plugin/pkg/admission/*`.
"""
from __future__ import annotations

import os

from ... import quota
from ...utils.features import DefaultFeatureGate
from ...api import core
from ...api import meta as m
from ...api.meta import new_uid
from ...api.quantity import Quantity, parse_quantity
from . import CREATE, DELETE, UPDATE, AdmissionError, Attributes, Plugin, register

SYSTEM_NAMESPACES = ("default", "kube-system", "kube-public")


@register
class ResourceV2(Plugin):
    name = "ResourceV2"
    operations = (CREATE, UPDATE)

    def __init__(self, server=None, config=None):
        super().__init__(server, config)
        names = (config or {}).get("resourceNames") or os.environ.get("KAMD_RESOURCEV2_NAMES", core.AMD_GPU)
        self.names = set(names.split(",")) if isinstance(names, str) else set(names)

    def admit(self, a: Attributes):
        if a.subresource or a.resource != "pods":
            return
        pod = a.obj
        if not isinstance(pod, dict) or pod.get("kind", "Pod") != "Pod":
            raise AdmissionError(f"expected Pod but got {type(pod).__name__}", 400, "BadRequest")
        spec = pod.setdefault("spec", {})
        ers = spec.get("extendedResources")
        if ers is None:
            ers = []
        changed = False
        for key in ("initContainers", "containers"):
            for c in spec.get(key) or ():
                res = c.get("resources") or {}
                limits = res.get("limits") or {}
                for rname in [r for r in limits if r in self.names]:
                    val = limits[rname]
                    name = new_uid()
                    c["extendedResourceRequests"] = [name]
                    ers.append({"name": name,
                                "resources": {"limits": {rname: val}, "requests": {rname: val}},
                                "affinity": {}})
                    limits.pop(rname, None)
                    (res.get("requests") or {}).pop(rname, None)
                    changed = True
        if changed:
            spec["extendedResources"] = ers


@register
class NamespaceLifecycle(Plugin):
    name = "NamespaceLifecycle"

    def validate(self, a: Attributes):
        if a.resource == "namespaces":
            if a.operation == DELETE and a.name in SYSTEM_NAMESPACES:
                raise AdmissionError(f"namespace {a.name} is immutable (system namespace)")
            return
        if not a.namespace or a.operation != CREATE:
            return
        if a.resource in ("events", "subjectaccessreviews", "tokenreviews"):
            return
        ns = self.server.get_object("namespaces", None, a.namespace) if self.server else None
        if ns is None:
            if a.namespace in SYSTEM_NAMESPACES:
                return
            raise AdmissionError(f"namespaces \"{a.namespace}\" not found", 404, "NotFound")
        if (ns.get("status") or {}).get("phase") == "Terminating" or (ns.get("metadata") or {}).get("deletionTimestamp"):
            raise AdmissionError(f"unable to create new content in namespace {a.namespace} because it is being terminated")


@register
class NamespaceExists(Plugin):
    """`plugin/pkg/admission/namespace/exists`: create, update and delete of namespaced objects
    are refused (404) unless the namespace exists."""
    name = "NamespaceExists"
    operations = (CREATE, UPDATE, DELETE)

    def validate(self, a: Attributes):
        if not a.namespace or a.resource == "namespaces" or not self.server:
            return
        if self.server.get_object("namespaces", None, a.namespace) is None:
            raise AdmissionError(f"namespaces \"{a.namespace}\" not found", 404, "NotFound")


@register
class NamespaceAutoProvision(Plugin):
    """`plugin/pkg/admission/namespace/autoprovision`: creating an object in a namespace that
    does not exist creates the namespace first (AlreadyExists from a racing request is fine;
    any other failure is 403)."""
    name = "NamespaceAutoProvision"
    operations = (CREATE,)

    async def prepare(self, a: Attributes):
        if not a.namespace or a.resource == "namespaces" or not self.server:
            return
        if self.server.get_object("namespaces", None, a.namespace) is not None:
            return
        from ...api import meta as _m
        try:
            await self.server.create(_m.BY_PLURAL["namespaces"], None,
                                     {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": a.namespace}},
                                     user=a.user)
        except Exception as e:       # noqa: BLE001 - APIError from the server
            if getattr(e, "code", None) != 409:
                raise AdmissionError(f"{a.resource} \"{a.name}\" is forbidden: {e}", 403, "Forbidden")


@register
class MutatingAdmissionWebhook(Plugin):
    """`staging/src/k8s.io/apiserver/pkg/admission/plugin/webhook/mutating`: enables calling
    the MutatingWebhookConfiguration hooks (dispatched by `extensions.WebhookDispatcher`)."""
    name = "MutatingAdmissionWebhook"


@register
class ValidatingAdmissionWebhook(Plugin):
    """`.../admission/plugin/webhook/validating`: enables the ValidatingWebhookConfiguration
    hooks."""
    name = "ValidatingAdmissionWebhook"


SA_MOUNT_PATH = "/var/run/secrets/kubernetes.io/serviceaccount"
ENFORCE_MOUNTABLE_SECRETS = "kubernetes.io/enforce-mountable-secrets"
MIRROR_POD_ANNOTATION = "kubernetes.io/config.mirror"


def _parse_bool(v) -> bool:
    """strconv.ParseBool (an unparsable value is false)."""
    return str(v) in ("1", "t", "T", "TRUE", "true", "True")


@register
class ServiceAccount(Plugin):
    """`plugin/pkg/admission/serviceaccount/admission.go`:
      * the pod runs as `default` unless it names an account (:158-161);
      * unless `automountServiceAccountToken` is false on the pod or, when the pod does not say,
        on the account (:245-256), the account's first referenced API token secret is a volume
        mounted read-only at /var/run/secrets/kubernetes.io/serviceaccount in every container
        and init container that has nothing mounted there (:402-490);
      * a pod without `imagePullSecrets` gets the account's (:175-178);
      * an account annotated `kubernetes.io/enforce-mountable-secrets: "true"` limits the pod to
        the secrets it references — secret volumes, `secretKeyRef` env of containers and init
        containers, and image pull secrets against the account's `imagePullSecrets`
        (:220-224, :258-271, :352-400);
      * mirror pods are not mutated and may reference neither an account nor a secret
        (:151-156, :198-212).
    The reference rejects the pod until the account (`DeniesInvalidServiceAccount`) and its
    token (`RequireAPIToken`, a 504 ServerTimeout) exist; here both are plugin config
    (`requireServiceAccount`, `requireAPIToken`, default off): by default a pod whose account
    or token does not exist yet is admitted without the mount and without the account's pull
    secrets, so a cluster without the service-account and token controllers (no
    --service-account-private-key-file) still runs pods."""
    name = "ServiceAccount"
    operations = (CREATE,)

    def __init__(self, server=None, config=None):
        super().__init__(server, config)
        self.require_account = bool(self.config.get("requireServiceAccount", False))
        self.require_token = bool(self.config.get("requireAPIToken", False))

    def _forbid(self, a, msg):
        md = a.obj.get("metadata") or {}
        return AdmissionError(f'pods "{md.get("name") or md.get("generateName", "")}" is forbidden: {msg}')

    def _account(self, namespace, name):
        try:
            return self.server.get_object("serviceaccounts", namespace, name)
        except RuntimeError:
            return None

    def admit(self, a):
        if a.resource != "pods" or a.subresource or not isinstance(a.obj, dict):
            return
        if ((a.obj.get("metadata") or {}).get("annotations") or {}).get(MIRROR_POD_ANNOTATION) is not None:
            return                                   # mirror pods are only validated
        spec = a.obj.setdefault("spec", {})
        if not spec.get("serviceAccountName"):
            spec["serviceAccountName"] = "default"
        if not self.server:
            return
        sa = self._account(a.namespace, spec["serviceAccountName"])
        if sa is None:
            if self.require_account:
                raise self._forbid(a, f"error looking up service account {a.namespace}/{spec['serviceAccountName']}: "
                                      f"serviceaccount \"{spec['serviceAccountName']}\" not found")
            return
        automount = spec.get("automountServiceAccountToken")
        if automount is None:
            automount = sa.get("automountServiceAccountToken")
        if automount is not False:
            self._mount_token(a, sa, spec)
        if not spec.get("imagePullSecrets") and sa.get("imagePullSecrets"):
            spec["imagePullSecrets"] = [dict(r) for r in sa["imagePullSecrets"]]

    def _mount_token(self, a, sa, spec):
        token = None
        for ref in sa.get("secrets") or ():
            try:
                sec = self.server.get_object("secrets", a.namespace, ref.get("name", ""))
            except RuntimeError:
                return
            if sec is not None and sec.get("type") == "kubernetes.io/service-account-token":
                token = sec["metadata"]["name"]
                break
        if token is None:
            if self.require_token:
                raise AdmissionError(f"No API token found for service account \"{sa['metadata']['name']}\", retry after "
                                     "the token is automatically created and added to the service account",
                                     504, "ServerTimeout")
            return
        vols = spec.get("volumes") or []
        vol = next((v["name"] for v in vols if (v.get("secret") or {}).get("secretName") == token), None)
        has_volume = vol is not None
        if vol is None:
            vol = token
            if any(v.get("name") == vol for v in vols):
                vol = f"{token}-{new_uid()[:5]}"     # names.SimpleNameGenerator
        needs = False
        for c in (spec.get("initContainers") or []) + (spec.get("containers") or []):
            mounts = c.setdefault("volumeMounts", [])
            if not any(m.get("mountPath") == SA_MOUNT_PATH for m in mounts):
                mounts.append({"name": vol, "readOnly": True, "mountPath": SA_MOUNT_PATH})
                needs = True
        if needs and not has_volume:
            # written as defaulting would leave it (admission runs after defaulting): an update
            # of the pod then carries the same volume and is not refused as a spec change
            vols.append({"name": vol, "secret": {"secretName": token, "defaultMode": 0o644}})
            spec["volumes"] = vols

    def validate(self, a):
        if a.resource != "pods" or a.subresource or not isinstance(a.obj, dict):
            return
        md = a.obj.get("metadata") or {}
        spec = a.obj.get("spec") or {}
        if (md.get("annotations") or {}).get(MIRROR_POD_ANNOTATION) is not None:
            if spec.get("serviceAccountName"):
                raise AdmissionError(f'pods "{md.get("name", "")}" is forbidden: a mirror pod may not reference '
                                     "service accounts")
            if core.pod_secret_names(a.obj):
                raise AdmissionError(f'pods "{md.get("name", "")}" is forbidden: a mirror pod may not reference secrets')
            return
        if not self.server or not spec.get("serviceAccountName"):
            return
        sa = self._account(a.namespace, spec["serviceAccountName"])
        if sa is None or not _parse_bool((sa["metadata"].get("annotations") or {}).get(ENFORCE_MOUNTABLE_SECRETS)):
            return
        err = limit_secret_references(sa, a.obj)
        if err:
            raise AdmissionError(f'pods "{md.get("name") or md.get("generateName", "")}" is forbidden: {err}')


def limit_secret_references(sa, pod):
    """serviceaccount/admission.go:352-400 — the first secret reference the account does not
    allow, as the reference's error message, or None."""
    spec = pod.get("spec") or {}
    mountable = {s.get("name") for s in sa.get("secrets") or ()}
    sa_name = sa["metadata"]["name"]
    for v in spec.get("volumes") or ():
        src = v.get("secret")
        if src is None:
            continue
        if src.get("secretName") not in mountable:
            return (f'volume with secret.secretName="{src.get("secretName", "")}" is not allowed because service '
                    f"account {sa_name} does not reference that secret")
    for kind, ctrs in (("init container", spec.get("initContainers")), ("container", spec.get("containers"))):
        for c in ctrs or ():
            for env in c.get("env") or ():
                ref = (env.get("valueFrom") or {}).get("secretKeyRef")
                if ref is not None and ref.get("name") not in mountable:
                    return (f'{kind} {c.get("name", "")} with envVar {env.get("name", "")} referencing '
                            f'secret.secretName="{ref.get("name", "")}" is not allowed because service account '
                            f"{sa_name} does not reference that secret")
    pull = {s.get("name") for s in sa.get("imagePullSecrets") or ()}
    for i, ref in enumerate(spec.get("imagePullSecrets") or ()):
        if ref.get("name") not in pull:
            return (f'imagePullSecrets[{i}].name="{ref.get("name", "")}" is not allowed because service account '
                    f"{sa_name} does not reference that imagePullSecret")
    return None


def add_or_update_toleration(spec, tol) -> bool:
    """`helper.AddOrUpdateTolerationInPod`: replace the toleration matching `tol` (same key,
    operator, value, effect — `Toleration.MatchToleration`) or append it."""
    key = lambda t: (t.get("key", ""), t.get("operator", "Equal") or "Equal", t.get("value", ""), t.get("effect", ""))  # noqa: E731
    out, updated = [], False
    for t in spec.get("tolerations") or ():
        if key(t) == key(tol):
            if t == tol:
                return False
            out.append(dict(tol))
            updated = True
        else:
            out.append(t)
    if not updated:
        out.append(dict(tol))
    spec["tolerations"] = out
    return True


@register
class DefaultTolerationSeconds(Plugin):
    """`plugin/pkg/admission/defaulttolerationseconds/admission.go`: a pod that does not tolerate
    `node.kubernetes.io/not-ready:NoExecute` (resp. `unreachable`) — a toleration with that key
    or an empty key, and effect NoExecute or empty — gets one with tolerationSeconds 300
    (plugin config `defaultNotReadyTolerationSeconds` / `defaultUnreachableTolerationSeconds`,
    the reference's --default-*-toleration-seconds flags). Create and update of pods proper."""
    name = "DefaultTolerationSeconds"
    operations = (CREATE, UPDATE)
    NOT_READY, UNREACHABLE = "node.kubernetes.io/not-ready", "node.kubernetes.io/unreachable"

    def __init__(self, server=None, config=None):
        super().__init__(server, config)
        self.seconds = {self.NOT_READY: int(self.config.get("defaultNotReadyTolerationSeconds", 300)),
                        self.UNREACHABLE: int(self.config.get("defaultUnreachableTolerationSeconds", 300))}

    def admit(self, a):
        if a.resource != "pods" or a.subresource or not isinstance(a.obj, dict):
            return
        spec = a.obj.setdefault("spec", {})
        tols = spec.get("tolerations") or []
        for k in (self.NOT_READY, self.UNREACHABLE):
            if any(t.get("key", "") in (k, "") and t.get("effect", "") in ("NoExecute", "") for t in tols):
                continue
            add_or_update_toleration(spec, {"key": k, "operator": "Exists", "effect": "NoExecute",
                                            "tolerationSeconds": self.seconds[k]})


@register
class ExtendedResourceToleration(Plugin):
    """Pods requesting an extended resource tolerate the taint named after it
    (`plugin/pkg/admission/extendedresourcetoleration/admission.go:55-94`): for every extended
    resource in a (init) container's requests, `{key: <name>, operator: Exists, effect:
    NoSchedule}` is added or updated with `AddOrUpdateTolerationInPod`. GPU-aware: the pod-level
    `spec.extendedResources` entries count too, since ResourceV2 (earlier in the chain) moves
    `amd.com/gpu` out of the container resources."""
    name = "ExtendedResourceToleration"
    operations = (CREATE, UPDATE)

    def admit(self, a):
        if a.resource != "pods" or a.subresource:
            return
        spec = a.obj.setdefault("spec", {})
        names = set()
        for c in (spec.get("containers") or []) + (spec.get("initContainers") or []):
            for k in core.container_requests(c):
                if core.is_extended_resource_name(k):
                    names.add(k)
        for per in spec.get("extendedResources") or ():
            try:
                names.add(core.pod_extended_resource_name(per))
            except ValueError:
                pass
        for n in sorted(names):     # sets.String.List(): stable sorted order (admission.go:84-91)
            add_or_update_toleration(spec, {"key": n, "operator": "Exists", "effect": "NoSchedule"})


SYSTEM_CRITICAL_PRIORITY = 2 * 1000000000                  # scheduling.SystemCriticalPriority
SYSTEM_PRIORITY_CLASSES = {"system-cluster-critical": SYSTEM_CRITICAL_PRIORITY,
                           "system-node-critical": SYSTEM_CRITICAL_PRIORITY + 1000}
HIGHEST_USER_DEFINABLE_PRIORITY = 1000000000


@register
class Priority(Plugin):
    """`plugin/pkg/admission/priority/admission.go`:
      * pods (create, PodPriority gate): a client may not set `spec.priority` itself; it is
        resolved from `priorityClassName` — the system classes first, then user classes ("no
        PriorityClass with name X was found" otherwise) — or, without a class name, from the
        globalDefault class, else 0 (:147-185);
      * PriorityClasses (create / update): the value may not exceed 1e9, the system class names
        are reserved, and at most one class is the globalDefault (:187-215)."""
    name = "Priority"
    operations = (CREATE, UPDATE, DELETE)

    def _classes(self):
        return self.server.list_objects("priorityclasses") if self.server else []

    def admit(self, a):
        if a.subresource or a.resource != "pods" or a.operation != CREATE or not isinstance(a.obj, dict):
            return
        spec = a.obj.setdefault("spec", {})
        if spec.get("priority") is not None:
            raise AdmissionError(f'pods "{(a.obj.get("metadata") or {}).get("name", "")}" is forbidden: the integer '
                                 "value of priority must not be provided in pod spec. Priority admission controller "
                                 "populates the value from the given PriorityClass name")
        if not DefaultFeatureGate("PodPriority"):
            return
        pcn = spec.get("priorityClassName")
        if not pcn:
            default = next((pc for pc in self._classes() if pc.get("globalDefault")), None)
            spec["priority"] = int(default.get("value", 0)) if default else 0
            return
        if pcn in SYSTEM_PRIORITY_CLASSES:
            spec["priority"] = SYSTEM_PRIORITY_CLASSES[pcn]
            return
        pc = self.server.get_object("priorityclasses", None, pcn) if self.server else None
        if pc is None:
            raise AdmissionError(f'pods "{(a.obj.get("metadata") or {}).get("name", "")}" is forbidden: no '
                                 f"PriorityClass with name {pcn} was found")
        spec["priority"] = int(pc.get("value", 0))

    def validate(self, a):
        if a.subresource or a.resource != "priorityclasses" or a.operation not in (CREATE, UPDATE):
            return
        pc = a.obj or {}
        name = (pc.get("metadata") or {}).get("name", "")

        def forbid(msg):
            return AdmissionError(f'priorityclasses.scheduling.k8s.io "{name}" is forbidden: {msg}')
        if int(pc.get("value", 0) or 0) > HIGHEST_USER_DEFINABLE_PRIORITY:
            raise forbid(f"maximum allowed value of a user defined priority is {HIGHEST_USER_DEFINABLE_PRIORITY}")
        if name in SYSTEM_PRIORITY_CLASSES:
            raise forbid(f"the name of the priority class is a reserved name for system use only: {name}")
        if pc.get("globalDefault"):
            other = next((c for c in self._classes() if c.get("globalDefault")), None)
            if other is not None and (a.operation == CREATE or other["metadata"]["name"] != name):
                raise forbid(f"PriorityClass {other['metadata']['name']} is already marked as default. "
                             "Only one default can exist")


def node_identity(user):
    """`pkg/auth/nodeidentifier/default.go`: (node name, True) for a user named
    `system:node:<name>` in the `system:nodes` group, else ("", False)."""
    if user is None or not user.name.startswith("system:node:") or "system:nodes" not in (user.groups or ()):
        return "", False
    return user.name[len("system:node:"):], True


def pod_configmap_names(pod) -> list[str]:
    """`VisitPodConfigmapNames` (pkg/api/pod/util.go): envFrom / configMapKeyRef, configMap and
    projected configMap volumes."""
    spec = pod.get("spec") or {}
    out = []
    for c in (spec.get("initContainers") or []) + (spec.get("containers") or []):
        out += [ef["configMapRef"].get("name", "") for ef in c.get("envFrom") or () if ef.get("configMapRef") is not None]
        out += [e["valueFrom"]["configMapKeyRef"].get("name", "") for e in c.get("env") or ()
                if (e.get("valueFrom") or {}).get("configMapKeyRef") is not None]
    for v in spec.get("volumes") or ():
        if v.get("configMap") is not None:
            out.append(v["configMap"].get("name", ""))
        for src in (v.get("projected") or {}).get("sources") or ():
            if src.get("configMap") is not None:
                out.append(src["configMap"].get("name", ""))
    return out


@register
class NodeRestriction(Plugin):
    """`plugin/pkg/admission/noderestriction/admission.go`: a kubelet (`system:node:<name>`,
    group `system:nodes`) may
      * create only mirror pods bound to itself that reference no service account, secret,
        configmap or persistent volume claim (:133-172), and delete only pods bound to itself
        (:174-191); no other pod write, and no pod subresource but status / eviction (:104-115);
      * update the status of, and evict, only pods bound to itself (:198-254);
      * create and modify only its own Node, never setting a new `spec.configSource` (:300-342);
      * update only `status.capacity` / `status.conditions` of PVCs, with the
        ExpandPersistentVolumes gate (:256-298).
    Requests from a node identity whose node name is empty are refused (:99-102)."""
    name = "NodeRestriction"
    operations = (CREATE, UPDATE, DELETE)

    def validate(self, a):
        node, is_node = node_identity(a.user)
        if not is_node:
            return
        if not node:
            raise self._forbid(a, f"could not determine node from user {a.user.name!r}")
        if a.resource == "pods":
            if a.subresource == "":
                self._pod(node, a)
            elif a.subresource == "status":
                if a.operation != UPDATE:
                    raise self._forbid(a, f"unexpected operation {a.operation!r}")
                if ((a.old or {}).get("spec") or {}).get("nodeName") != node:
                    raise self._forbid(a, f"node {node!r} can only update pod status for pods with spec.nodeName set "
                                          "to itself")
            elif a.subresource == "eviction":
                self._eviction(node, a)
            else:
                raise self._forbid(a, f"unexpected pod subresource {a.subresource!r}")
        elif a.resource == "nodes":
            self._node(node, a)
        elif a.resource == "persistentvolumeclaims":
            if a.subresource != "status":
                raise self._forbid(a, "may only update PVC status")
            self._pvc_status(node, a)

    @staticmethod
    def _forbid(a, msg):
        return AdmissionError(f'{a.resource} "{a.name or ""}" is forbidden: {msg}')

    def _pod(self, node, a):
        if a.operation == CREATE:
            pod = a.obj or {}
            md, spec = pod.get("metadata") or {}, pod.get("spec") or {}
            if MIRROR_POD_ANNOTATION not in (md.get("annotations") or {}):
                raise self._forbid(a, f"pod does not have \"{MIRROR_POD_ANNOTATION}\" annotation, node \"{node}\" "
                                      "can only create mirror pods")
            if spec.get("nodeName") != node:
                raise self._forbid(a, f"node {node!r} can only create pods with spec.nodeName set to itself")
            if spec.get("serviceAccountName"):
                raise self._forbid(a, f"node {node!r} can not create pods that reference a service account")
            if core.pod_secret_names(pod):
                raise self._forbid(a, f"node {node!r} can not create pods that reference secrets")
            if pod_configmap_names(pod):
                raise self._forbid(a, f"node {node!r} can not create pods that reference configmaps")
            if any(v.get("persistentVolumeClaim") is not None for v in spec.get("volumes") or ()):
                raise self._forbid(a, f"node {node!r} can not create pods that reference persistentvolumeclaims")
        elif a.operation == DELETE:
            if ((a.old or {}).get("spec") or {}).get("nodeName") != node:
                raise self._forbid(a, f"node {node!r} can only delete pods with spec.nodeName set to itself")
        else:
            raise self._forbid(a, f"unexpected operation {a.operation!r}")

    def _eviction(self, node, a):
        if a.operation != CREATE:
            raise self._forbid(a, f"unexpected operation {a.operation}")
        pod = a.old
        if pod is None and self.server is not None:
            name = a.name or ((a.obj or {}).get("metadata") or {}).get("name")
            if not name:
                raise self._forbid(a, "could not determine pod from request data")
            pod = self.server.get_object("pods", a.namespace, name)
        if pod is None:
            raise AdmissionError(f'pods "{a.name}" not found', 404, "NotFound")
        if (pod.get("spec") or {}).get("nodeName") != node:
            raise self._forbid(a, f"node {node} can only evict pods with spec.nodeName set to itself")

    def _node(self, node, a):
        requested = a.name
        if a.operation == CREATE:
            if ((a.obj or {}).get("spec") or {}).get("configSource") is not None:
                raise self._forbid(a, "cannot create with non-nil configSource")
            requested = requested or ((a.obj or {}).get("metadata") or {}).get("name")
        if requested != node:
            raise self._forbid(a, f"node {node!r} cannot modify node {requested!r}")
        if a.operation == UPDATE:
            new = ((a.obj or {}).get("spec") or {}).get("configSource")
            if new is not None and new != ((a.old or {}).get("spec") or {}).get("configSource"):
                raise self._forbid(a, "cannot update configSource to a new non-nil configSource")

    def _pvc_status(self, node, a):
        if a.operation != UPDATE:
            raise self._forbid(a, f"unexpected operation {a.operation!r}")
        if not DefaultFeatureGate("ExpandPersistentVolumes"):
            raise self._forbid(a, f"node {node!r} may not update persistentvolumeclaim metadata")

        def strip(o):
            o = dict(o or {})
            o["metadata"] = {k: v for k, v in (o.get("metadata") or {}).items() if k != "resourceVersion"}
            o["status"] = {k: v for k, v in (o.get("status") or {}).items() if k not in ("capacity", "conditions")}
            return o
        if strip(a.old) != strip(a.obj):
            raise self._forbid(a, f"node {node!r} may not update fields other than status.capacity and status.conditions")


@register
class AlwaysPullImages(Plugin):
    """`plugin/pkg/admission/alwayspullimages/admission.go`: every container and init container
    of a created or updated pod pulls Always (a node's cached image is not trusted across
    tenants); validation refuses any other policy that a later mutating step put back."""
    name = "AlwaysPullImages"
    operations = (CREATE, UPDATE)

    def admit(self, a):
        if a.resource != "pods" or a.subresource or not isinstance(a.obj, dict):
            return
        spec = a.obj.get("spec") or {}
        for c in (spec.get("initContainers") or []) + (spec.get("containers") or []):
            c["imagePullPolicy"] = "Always"

    def validate(self, a):
        if a.resource != "pods" or a.subresource or not isinstance(a.obj, dict):
            return
        spec = a.obj.get("spec") or {}
        for kind in ("initContainers", "containers"):
            for i, c in enumerate(spec.get(kind) or ()):
                if c.get("imagePullPolicy") != "Always":
                    raise AdmissionError(f'pods "{(a.obj.get("metadata") or {}).get("name", "")}" is forbidden: '
                                         f"spec.{kind}[{i}].imagePullPolicy: Unsupported value: "
                                         f"\"{c.get('imagePullPolicy', '')}\": supported values: \"Always\"")


def selector_to_labels_map(text) -> dict:
    """`labels.ConvertSelectorToLabelsMap`: "k1=v1,k2=v2" (`==` accepted) -> {k: v}; an
    unparsable term is an error."""
    out = {}
    for term in (text or "").split(","):
        term = term.strip()
        if not term:
            continue
        k, sep, v = term.partition("==") if "==" in term else term.partition("=")
        k, v = k.strip(), v.strip()
        if not sep or not k or "!" in k:
            raise ValueError(f"invalid selector: {term!r}")
        out[k] = v
    return out


def labels_conflict(a: dict, b: dict) -> bool:
    """`labels.Conflicts`: a key both sets have, with different values."""
    return any(k in b and b[k] != v for k, v in a.items())


@register
class PodNodeSelector(Plugin):
    """`plugin/pkg/admission/podnodeselector/admission.go`: the namespace's node selector —
    the `scheduler.alpha.kubernetes.io/node-selector` annotation, else the plugin config's
    `clusterDefaultNodeSelector` — is merged into the pod's `nodeSelector` (the pod's own
    labels win, a conflicting value is refused), and the result must stay within the
    namespace's whitelist from the plugin config (`podNodeSelectorPluginConfig: {<namespace>:
    "k=v,..."}`). Create and update of pods proper; subresources are ignored."""
    name = "PodNodeSelector"
    operations = (CREATE, UPDATE)
    ANN = "scheduler.alpha.kubernetes.io/node-selector"

    def __init__(self, server=None, config=None):
        super().__init__(server, config)
        cfg = self.config
        self.cluster = dict(cfg.get("podNodeSelectorPluginConfig") or cfg.get("PodNodeSelectorPluginConfig") or
                            {k: v for k, v in cfg.items() if isinstance(v, str)})

    def _ignore(self, a):
        return a.resource != "pods" or a.subresource or not isinstance(a.obj, dict)

    def _namespace_selector(self, a):
        ns = self.server.get_object("namespaces", None, a.namespace) if self.server else None
        if ns is None:
            if self.server is not None and a.namespace not in SYSTEM_NAMESPACES:
                raise AdmissionError(f"namespace {a.namespace} does not exist", 404, "NotFound")
            ns = {"metadata": {"name": a.namespace}}
        ann = (ns.get("metadata") or {}).get("annotations") or {}
        try:
            if self.ANN in ann:
                return selector_to_labels_map(ann[self.ANN])
            return selector_to_labels_map(self.cluster.get("clusterDefaultNodeSelector", ""))
        except ValueError as e:
            raise AdmissionError(str(e), 500, "InternalError")

    def _forbid(self, a, msg):
        return AdmissionError(f'pods "{(a.obj.get("metadata") or {}).get("name", "")}" is forbidden: {msg}')

    def admit(self, a):
        if self._ignore(a):
            return
        if a.operation == UPDATE and a.old is not None and \
                not ((a.old.get("metadata") or {}).get("initializers") or {}).get("pending"):
            return                  # the node selector of an initialized pod is immutable (:101-108)
        nsel = self._namespace_selector(a)
        spec = a.obj.setdefault("spec", {})
        pod_sel = spec.get("nodeSelector") or {}
        if labels_conflict(nsel, pod_sel):
            raise self._forbid(a, "pod node label selector conflicts with its namespace node label selector")
        if nsel:
            spec["nodeSelector"] = {**nsel, **pod_sel}

    def validate(self, a):
        if self._ignore(a):
            return
        nsel = self._namespace_selector(a)
        pod_sel = (a.obj.get("spec") or {}).get("nodeSelector") or {}
        if labels_conflict(nsel, pod_sel):
            raise self._forbid(a, "pod node label selector conflicts with its namespace node label selector")
        try:
            white = selector_to_labels_map(self.cluster.get(a.namespace, ""))
        except ValueError as e:
            raise AdmissionError(str(e), 500, "InternalError")
        # labels.AreLabelsInWhiteList: an empty whitelist allows everything
        if white and any(white.get(k) != v for k, v in pod_sel.items()):
            raise self._forbid(a, "pod node label selector labels conflict with its namespace whitelist")


@register
class DefaultStorageClass(Plugin):
    """`plugin/pkg/admission/storageclass/setdefault/admission.go`: a claim without a class gets
    the StorageClass annotated `storageclass.kubernetes.io/is-default-class=true` (error if several)."""
    name = "DefaultStorageClass"
    operations = (CREATE,)
    ANN = ("storageclass.kubernetes.io/is-default-class", "storageclass.beta.kubernetes.io/is-default-class")

    def admit(self, a):
        if a.resource != "persistentvolumeclaims" or a.subresource:
            return
        spec = a.obj.setdefault("spec", {})
        if "storageClassName" in spec or (a.obj.get("metadata", {}).get("annotations") or {}).get(
                "volume.beta.kubernetes.io/storage-class") is not None:
            return
        defaults = [sc for sc in self.server.list_objects("storageclasses")
                    if any((sc["metadata"].get("annotations") or {}).get(k) == "true" for k in self.ANN)]
        if len(defaults) > 1:
            raise AdmissionError(f"{len(defaults)} default StorageClasses were found", 403)
        if defaults:
            spec["storageClassName"] = defaults[0]["metadata"]["name"]


def _storage(pvc):
    from ...api.quantity import parse_quantity
    v = (((pvc or {}).get("spec") or {}).get("resources") or {}).get("requests", {}).get("storage")
    return parse_quantity(str(v)).value if v is not None else 0


@register
class PersistentVolumeClaimResize(Plugin):
    """`plugin/pkg/admission/persistentvolume/resize/admission.go`: a claim may only grow, only
    when bound, only when its StorageClass sets `allowVolumeExpansion: true`, and only when the
    bound volume's type can be expanded (here: hostPath volumes from the built-in provisioner,
    local and CSI volumes)."""
    name = "PersistentVolumeClaimResize"
    operations = (UPDATE,)
    EXPANDABLE = ("hostPath", "local", "csi")

    def validate(self, a):
        if a.resource != "persistentvolumeclaims" or a.subresource or a.old is None:
            return
        new, old = _storage(a.obj), _storage(a.old)
        if new <= old:
            if new < old:
                raise AdmissionError("spec.resources.requests.storage: field can not be less than previous value", 403)
            return
        if ((a.old.get("status") or {}).get("phase") != "Bound") or not (a.old.get("spec") or {}).get("volumeName"):
            raise AdmissionError("Only bound persistent volume claims can be expanded", 403)
        cls = (a.old.get("spec") or {}).get("storageClassName") or ""
        sc = self.server.get_object("storageclasses", None, cls) if cls else None
        if not sc or not sc.get("allowVolumeExpansion"):
            raise AdmissionError("only dynamically provisioned pvc can be resized and the storageclass that provisions "
                                 "the pvc must support resize", 403)
        pv = self.server.get_object("persistentvolumes", None, a.old["spec"]["volumeName"])
        if pv is None or not any(k in (pv.get("spec") or {}) for k in self.EXPANDABLE):
            raise AdmissionError("volume plugin does not support resize", 403)


def _rule_matches(rule, group, version, resource):
    def ok(vals, v):
        return not vals or "*" in vals or v in vals
    return ok(rule.get("apiGroups"), group) and ok(rule.get("apiVersions"), version) and ok(rule.get("resources"), resource)


@register
class Initializers(Plugin):
    """`staging/src/k8s.io/apiserver/pkg/admission/plugin/initialization/initialization.go`
    (alpha): on CREATE, the initializers of every `InitializerConfiguration` whose rules match
    the resource are written to `metadata.initializers.pending`; the object stays hidden from
    list/watch (unless `includeUninitialized=true`) until each initializer controller removes
    its own entry — the head of the list — by UPDATE. An emptied list is dropped, which makes
    the object visible (watchers see it ADDED)."""
    name = "Initializers"
    operations = (CREATE, UPDATE)

    def admit(self, a):
        if a.subresource or a.resource in ("initializerconfigurations", "events"):
            return
        md = a.obj.setdefault("metadata", {})
        if a.operation == CREATE:
            if md.get("initializers") is not None:
                return                    # explicitly set by the creator
            from ...api import meta as m
            ri = m.BY_PLURAL.get(a.resource)
            group, version = (ri.group, ri.version) if ri else ("", "v1")
            pending = []
            for cfg in self.server.list_objects("initializerconfigurations"):
                for init in cfg.get("initializers") or ():
                    if any(_rule_matches(r, group, version, a.resource) for r in init.get("rules") or ()):
                        if init["name"] not in [p["name"] for p in pending]:
                            pending.append({"name": init["name"]})
            if pending:
                md["initializers"] = {"pending": pending}
            return
        ini = md.get("initializers")
        if ini is not None and not ini.get("pending") and not ini.get("result"):
            md.pop("initializers", None)

    def validate(self, a):
        if a.operation != UPDATE or a.old is None or a.subresource:
            return
        old = ((a.old.get("metadata") or {}).get("initializers") or {}).get("pending") or []
        new = ((a.obj.get("metadata") or {}).get("initializers") or {}).get("pending") or []
        if not old:
            if new:
                raise AdmissionError("initializers may not be added to an initialized object", 403)
            return
        if new and [p["name"] for p in new] != [p["name"] for p in old] and \
                [p["name"] for p in new] != [p["name"] for p in old[1:]]:
            raise AdmissionError("initializers may only be removed from the front of metadata.initializers.pending", 403)


@register
class AlwaysAdmit(Plugin):
    name = "AlwaysAdmit"


@register
class AlwaysDeny(Plugin):
    name = "AlwaysDeny"

    def validate(self, a):
        raise AdmissionError("admission control is denying all modifications")


_POD_EVALUATOR = quota.PodEvaluator()


def pod_usage(pod) -> dict[str, Quantity]:
    """Quota usage of a pod (`quota.PodEvaluator.usage`), including the fork's pod-level
    extended resources."""
    return _POD_EVALUATOR.usage(pod)


@register
class ResourceQuota(Plugin):
    """`plugin/pkg/admission/resourcequota` (`controller.go` checkRequest / checkQuotas):

      * the evaluator for the request's group/resource decides whether the operation can
        change usage at all (pods / object counts: CREATE; services: CREATE and UPDATE);
      * every quota in the namespace that names a matching resource and whose scopes all match
        is "interesting": its per-kind constraints must hold (pods must state cpu/memory when
        those are quota'd) and it must already carry usage for every hard name ("status unknown
        for quota" until the controller has counted);
      * the request's usage (on UPDATE, the non-negative delta over the old object) is added to
        status.used, masked to each quota's hard names, and must stay within hard;
      * the new status.used is written back with the quota's resourceVersion — concurrent
        admissions therefore serialise on the quota object — and quotas whose write conflicted
        are re-read and re-checked (3 retries), exactly as the reference's evaluator loop;
      * `limitedResources` (plugin config) names resources that may only be consumed when some
        quota covers them ("insufficient quota to consume").

    The check runs in `charge()`, the chain's asynchronous last step before the object is
    committed, because the status write is an API round trip."""
    name = "ResourceQuota"
    operations = (CREATE, UPDATE)
    RETRIES = 3

    def __init__(self, server=None, config=None):
        super().__init__(server, config)
        self.registry = quota.Registry()
        self.limited = list((self.config or {}).get("limitedResources") or ())

    @staticmethod
    def _group(plural):
        ri = m.BY_PLURAL.get(plural)
        return ri.group if ri is not None else ""

    def _limited_names(self, group, resource, usage):
        """`limitedByDefault`: consumed names matching a configured limitedResources entry."""
        out = set()
        for lr in self.limited:
            if lr.get("resource") != resource or (lr.get("apiGroup") or "") != group:
                continue
            for k, v in usage.items():
                if quota.qty(v) > quota.ZERO and any(mc in k for mc in lr.get("matchContains") or ()):
                    out.add(k)
        return out

    def check_request(self, quotas, ev, a, group):
        """Returns the quotas with status.used as it would be if the request were admitted."""
        obj = a.obj
        limited = set()
        if any(lr.get("resource") == a.resource and (lr.get("apiGroup") or "") == group for lr in self.limited):
            limited = self._limited_names(group, a.resource, ev.usage(obj))
        interesting, restricted = [], set()
        for i, q in enumerate(quotas):
            if not ev.matches(q, obj):
                continue
            st = q.get("status") or {}
            hard = st.get("hard") or {}
            names = ev.matching_resources(list(hard))
            msg = ev.constraints(names, obj)
            if msg:
                raise AdmissionError(f"failed quota: {m.name_of(q)}: {msg}")
            used = st.get("used") or {}
            if any(k not in used for k in hard):
                raise AdmissionError(f"status unknown for quota: {m.name_of(q)}")
            interesting.append(i)
            restricted.update(names)
        uncovered = limited - restricted
        if uncovered:
            raise AdmissionError(f"insufficient quota to consume: {','.join(sorted(uncovered))}")
        if not interesting:
            return quotas
        delta = ev.usage(obj)
        neg = quota.is_negative(delta)
        if neg:
            raise AdmissionError(f"quota usage is negative for resource(s): {','.join(neg)}")
        if a.operation == UPDATE:
            if a.old is None:
                raise AdmissionError("unable to get previous usage since prior version of object was not found")
            if (a.old.get("metadata") or {}).get("resourceVersion"):
                delta = quota.subtract_non_negative(delta, ev.usage(a.old))
        if quota.is_zero(delta):
            return quotas
        out = list(quotas)
        for i in interesting:
            q = quotas[i]
            st = q.get("status") or {}
            hard = st.get("hard") or {}
            requested = quota.mask(delta, hard)
            new_used = quota.add(st.get("used") or {}, requested)
            ok, exceeded = quota.less_than_or_equal(quota.mask(new_used, requested), hard)
            if not ok:
                raise AdmissionError(
                    f"exceeded quota: {m.name_of(q)}, requested: {quota.pretty(quota.mask(requested, exceeded))}, "
                    f"used: {quota.pretty(quota.mask(st.get('used') or {}, exceeded))}, "
                    f"limited: {quota.pretty(quota.mask(hard, exceeded))}")
            nq = dict(q, status=dict(st, used=quota.to_strings(new_used)))
            out[i] = nq
        return out

    async def charge(self, a):
        if a.subresource or self.server is None or not a.namespace:
            return
        group = self._group(a.resource)
        ev = self.registry.get(group, a.resource)
        if not ev.handles(a.operation):
            return
        quotas = await self.server.quota_objects(a.namespace)
        if not quotas and not self.limited:
            return
        for attempt in range(self.RETRIES + 1):
            new = self.check_request(quotas, ev, a, group)
            failed = []
            for old, nq in zip(quotas, new):
                if nq is old:
                    continue
                try:
                    await self.server.write_quota_status(nq)
                except Exception as e:   # noqa: BLE001 - a conflicting writer: re-read and re-check
                    if getattr(e, "code", None) != 409:
                        raise
                    failed.append(m.name_of(nq))
            if not failed:
                return
            if attempt == self.RETRIES:
                raise AdmissionError(f"Operation cannot be fulfilled on resourcequotas \"{failed[0]}\": "
                                     "the object has been modified; please apply your changes to the latest version "
                                     "and try again", 409, "Conflict")
            quotas = [q for q in await self.server.quota_objects(a.namespace, fresh=True) if m.name_of(q) in failed]
