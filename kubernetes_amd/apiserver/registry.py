"""Per-resource REST strategies (create/update/status/delete semantics).

Parity:
  * generic `Store` CRUD: `staging/src/k8s.io/apiserver/pkg/registry/generic/registry/store.go:262-1153`
  * pod strategy + graceful delete: `pkg/registry/core/pod/strategy.go`
  * **BindingREST with devices** (fork F6): `pkg/registry/core/pod/storage/storage.go:139-210`
    — one atomic update sets `spec.nodeName`, merges annotations, writes
    `spec.extendedResources[i].assigned` from `target.extendedResourceBinding[name]` and
    sets `PodScheduled=True`. Added checks: the binding must cover
    every requested ER with exactly the requested count, and a device may not be bound
    to two live pods on the same node.
"""
from __future__ import annotations

import random
import time

from ..api import core, validation, validation_ext
from ..api.meta import new_uid, now_rfc3339
from ..api.quantity import parse_quantity


class APIError(Exception):
    def __init__(self, code, reason, message, details=None):
        super().__init__(message)
        self.code, self.reason, self.message, self.details = code, reason, message, details


def not_found(ri, name):
    return APIError(404, "NotFound", f'{ri.group_resource} "{name}" not found',
                    {"name": name, "group": ri.group, "kind": ri.plural})


def already_exists(ri, name):
    return APIError(409, "AlreadyExists", f'{ri.group_resource} "{name}" already exists',
                    {"name": name, "group": ri.group, "kind": ri.plural})


def conflict(ri, name, msg):
    return APIError(409, "Conflict", f'Operation cannot be fulfilled on {ri.group_resource} "{name}": {msg}',
                    {"name": name, "group": ri.group, "kind": ri.plural})


def invalid(ri, name, errs):
    return APIError(422, "Invalid", f'{ri.kind} "{name}" is invalid: ' + "; ".join(str(e) for e in errs),
                    {"name": name, "group": ri.group, "kind": ri.kind,
                     "causes": [{"reason": "FieldValue" + e.type.replace(" ", ""), "message": e.detail, "field": e.field} for e in errs]})


def bad_request(msg):
    return APIError(400, "BadRequest", msg)


_GEN_CHARS = "bcdfghjklmnpqrstvwxz2456789"


def generate_name(base):
    return base + "".join(random.choice(_GEN_CHARS) for _ in range(5))


# per-kind create validation: core kinds (api/validation.py) and every other served kind
# (api/validation_ext.py)
_VALIDATORS = {**validation.VALIDATORS, **validation_ext.VALIDATORS}


class Strategy:
    """Default strategy: spec+status updated together, no status subresource."""
    has_status = True      # exposes /status; main updates ignore status changes
    bump_generation = True
    generation_on_annotations = False

    def __init__(self, ri):
        self.ri = ri

    def prepare_create(self, obj):
        pass

    def prepare_update(self, new, old):
        if self.has_status and "status" in old:
            new["status"] = old["status"]

    def prepare_status_update(self, new, old):
        for k in list(new.keys()):
            if k not in ("status", "metadata", "kind", "apiVersion"):
                new.pop(k)
        for k, v in old.items():
            if k not in ("status", "metadata"):
                new[k] = v
        # status updates may not touch labels etc. except through main resource
        nm, om = new.get("metadata", {}), old.get("metadata", {})
        for k in ("labels", "annotations", "finalizers", "ownerReferences", "deletionTimestamp",
                  "deletionGracePeriodSeconds"):
            if k in om:
                nm[k] = om[k]
            else:
                nm.pop(k, None)

    def validate(self, obj):
        fn = _VALIDATORS.get(self.ri.kind)
        return fn(obj) if fn else validation.validate_generic(obj, self.ri.namespaced)

    def validate_update(self, new, old):
        return self.validate(new) + validation_ext.validate_update(self.ri.kind, new, old)

    _PHASES = {"Pending", "Running", "Succeeded", "Failed", "Unknown", "Active", "Terminating", "",
               "Available", "Bound", "Released", "Lost"}   # pods, namespaces, PVs / PVCs

    def validate_status(self, obj):
        errs = validation.validate_object_meta(obj, self.ri.namespaced)
        st = obj.get("status")
        if st is not None and not isinstance(st, dict):
            errs.append(validation.invalid("status", "must be an object"))
        elif st and st.get("phase", "") not in self._PHASES:
            errs.append(validation.not_supported("status.phase", st.get("phase")))
        return errs

    def graceful_seconds(self, obj, opts) -> int:
        """0 = delete immediately."""
        return 0

    def export(self, obj):
        """`?export=true` without `exact`: strip cluster-specific state (the reference falls back
        to PrepareForCreate when a kind has no ExportStrategy)."""
        self.prepare_create(obj)


class PodStrategy(Strategy):
    def prepare_create(self, pod):
        core.set_defaults_pod(pod)
        pod["status"] = {"phase": core.POD_PENDING, "qosClass": qos_class(pod)}

    def prepare_update(self, new, old):
        super().prepare_update(new, old)
        # scheduler-owned fields are only written through pods/binding
        os_ = old.get("spec") or {}
        ns = new["spec"] = dict(new.get("spec") or {})   # never mutate structure shared with the cache
        if os_.get("nodeName"):
            ns["nodeName"] = os_["nodeName"]
        if os_.get("extendedResources") and ns.get("extendedResources"):
            amap = {r.get("name"): r.get("assigned") for r in os_["extendedResources"]}
            ers = []
            for r in ns["extendedResources"]:
                if amap.get(r.get("name")) and r.get("assigned") != amap[r["name"]]:
                    r = dict(r, assigned=amap[r["name"]])
                ers.append(r)
            ns["extendedResources"] = ers

    def prepare_status_update(self, new, old):
        """`podStatusStrategy.PrepareForUpdate` (pkg/registry/core/pod/strategy.go:184-193): the
        spec, deletion timestamp and owner references stay the old ones; the rest of the
        metadata may change — the scheduler writes its `NominatedNodeName` annotation this way
        (factory.go:1271-1287)."""
        nm = dict(new.get("metadata") or {})
        super().prepare_status_update(new, old)
        md = new["metadata"] = dict(new.get("metadata") or {})
        for k in ("labels", "annotations"):
            if k in nm:
                if nm[k] is None:
                    md.pop(k, None)
                else:
                    md[k] = nm[k]

    def validate_update(self, new, old):
        # `ValidatePodUpdate`: images, activeDeadlineSeconds and tolerations only
        return validation.validate_pod_update(new, old) + validation.validate_object_meta_update(new, old)

    def export(self, pod):
        self.prepare_create(pod)
        spec = pod.get("spec") or {}
        spec.pop("nodeName", None)                      # where it ran, and which devices, is cluster state
        for er in spec.get("extendedResources") or ():
            er.pop("assigned", None)

    def graceful_seconds(self, pod, opts):
        spec = pod.get("spec") or {}
        if not spec.get("nodeName") or core.pod_is_terminal(pod):
            return 0
        g = (opts or {}).get("gracePeriodSeconds")
        if g is None:
            g = spec.get("terminationGracePeriodSeconds", 30)
        return max(int(g), 0)


class NodeStrategy(Strategy):
    bump_generation = False

    def prepare_create(self, node):
        node.setdefault("spec", {})
        node.setdefault("status", {})


class NamespaceStrategy(Strategy):
    def prepare_create(self, ns):
        ns.setdefault("spec", {}).setdefault("finalizers", ["kubernetes"])
        ns["status"] = {"phase": "Active"}


class NoStatusStrategy(Strategy):
    has_status = False


class SecretStrategy(NoStatusStrategy):
    def export(self, secret):
        """Service-account token secrets are minted per cluster: exported without their data."""
        ann = (secret.get("metadata") or {}).get("annotations") or {}
        if secret.get("type") == "kubernetes.io/service-account-token" or ann.get("kubernetes.io/service-account.uid"):
            secret.pop("data", None)
            ann.pop("kubernetes.io/service-account.uid", None)


class WorkloadStrategy(Strategy):
    """Kinds whose status only controllers write: a client's status is dropped on create
    (`PrepareForCreate`: `Status = {}` in pkg/registry/{apps,extensions,batch,autoscaling,policy,
    networking}/*/strategy.go) and kept from the stored object on a main-resource update."""
    initial_status: dict = {}

    def prepare_create(self, obj):
        obj["status"] = dict(self.initial_status)


class VolumeStrategy(WorkloadStrategy):
    """PV / PVC: status reset on create, phase Pending until the binder moves it
    (`pkg/registry/core/persistentvolume{,claim}/strategy.go` + SetDefaults)."""
    initial_status = {"phase": "Pending"}


class JobStrategy(WorkloadStrategy):
    """`pkg/registry/batch/job/strategy.go`: unless `spec.manualSelector` is true the selector is
    generated — `controller-uid=<uid>` is added to the selector and `controller-uid` + `job-name`
    to the template's labels (`generateSelector`), and validation then requires exactly that
    (`validateGeneratedSelector`)."""

    def prepare_create(self, job):
        super().prepare_create(job)
        spec = job.setdefault("spec", {})
        if spec.get("manualSelector"):
            return
        md = job["metadata"]
        uid = md.get("uid", "")
        sel = spec["selector"] = dict(spec.get("selector") or {})
        ml = sel["matchLabels"] = dict(sel.get("matchLabels") or {})
        ml.setdefault("controller-uid", uid)
        tpl = spec["template"] = dict(spec.get("template") or {})
        tmd = tpl["metadata"] = dict(tpl.get("metadata") or {})
        labels = tmd["labels"] = dict(tmd.get("labels") or {})
        labels.setdefault("controller-uid", uid)
        labels.setdefault("job-name", md.get("name", ""))

    def validate(self, job):
        errs = super().validate(job)
        spec = job.get("spec") or {}
        if spec.get("manualSelector"):
            return errs
        uid = job["metadata"].get("uid", "")
        labels = ((spec.get("template") or {}).get("metadata") or {}).get("labels") or {}
        if labels.get("controller-uid") != uid:
            errs.append(validation.invalid("spec.template.metadata.labels", "`selector` does not match template `labels`"))
        if ((spec.get("selector") or {}).get("matchLabels") or {}).get("controller-uid") != uid:
            errs.append(validation.invalid("spec.selector", "`selector` not auto-generated"))
        return errs


class DeploymentStrategy(WorkloadStrategy):
    """`pkg/registry/extensions/deployment/strategy.go` PrepareForUpdate: a change of the spec or
    of the annotations (rollback records there) bumps metadata.generation."""
    generation_on_annotations = True


_QOS_RESOURCES = ("cpu", "memory")


def _qos_resource(name) -> bool:
    """isSupportedQoSComputeResource: cpu, memory and hugepages-<size>."""
    return name in _QOS_RESOURCES or name.startswith("hugepages-")


def qos_class(pod) -> str:
    """`qos.GetPodQOS` (pkg/apis/core/v1/helper/qos/qos.go): positive cpu/memory requests and
    limits are summed over the app containers; BestEffort without any, Guaranteed when every
    container limits both and the summed requests equal the summed limits for each resource
    (requests left unset by the client were defaulted to the limits), else Burstable. Other
    resources (GPUs) never affect the class; hugepages are summed like cpu/memory, and a container
    limiting hugepages as well counts 3 limited resources against the 2 the rule expects, so it is
    Burstable, as in the reference."""
    requests, limits, guaranteed = {}, {}, True
    for c in (pod.get("spec") or {}).get("containers") or ():
        res = c.get("resources") or {}
        for k, v in (res.get("requests") or {}).items():
            if _qos_resource(k):
                qv = parse_quantity(str(v))
                if qv.value > 0:
                    requests[k] = requests[k] + qv if k in requests else qv
        found = 0
        for k, v in (res.get("limits") or {}).items():
            if _qos_resource(k):
                qv = parse_quantity(str(v))
                if qv.value > 0:
                    found += 1
                    limits[k] = limits[k] + qv if k in limits else qv
        if found != len(_QOS_RESOURCES):
            guaranteed = False
    if not requests and not limits:
        return "BestEffort"
    if guaranteed:
        for k, req in requests.items():
            if k not in limits or limits[k] != req:
                guaranteed = False
                break
    if guaranteed and len(requests) == len(limits):
        return "Guaranteed"
    return "Burstable"


class ServiceStrategy(Strategy):
    """`pkg/registry/core/service/strategy.go`: status subresource (load balancer ingress);
    allocation lives in `service_alloc` (done by the API server before validation)."""

    def prepare_create(self, svc):
        svc["status"] = {"loadBalancer": {}}

    def prepare_update(self, new, old):
        super().prepare_update(new, old)
        ns, os_ = new.setdefault("spec", {}), old.get("spec") or {}
        if not ns.get("clusterIP") and os_.get("clusterIP") and ns.get("type", "ClusterIP") != "ExternalName":
            ns["clusterIP"] = os_["clusterIP"]
        if ns.get("type", "ClusterIP") in ("NodePort", "LoadBalancer"):
            old_np = {(p.get("port"), p.get("protocol", "TCP")): p.get("nodePort") for p in os_.get("ports") or ()}
            for p in ns.get("ports") or ():
                if not p.get("nodePort") and old_np.get((p.get("port"), p.get("protocol", "TCP"))):
                    p["nodePort"] = old_np[(p.get("port"), p.get("protocol", "TCP"))]

    def export(self, svc):
        """`svcStrategy.Export`: drop the allocated cluster IP (unless headless) and node ports."""
        spec = svc.get("spec") or {}
        if spec.get("clusterIP") and spec["clusterIP"] != "None":
            spec.pop("clusterIP")
        if spec.get("type") == "NodePort":
            for p in spec.get("ports") or ():
                p.pop("nodePort", None)

    def validate(self, obj):
        from .service_alloc import validate_service
        return validate_service(obj)

    def validate_update(self, new, old):
        from .service_alloc import validate_service_update
        return validate_service_update(new, old)


STRATEGIES = {"pods": PodStrategy, "services": ServiceStrategy, "nodes": NodeStrategy, "namespaces": NamespaceStrategy,
              "events": NoStatusStrategy, "configmaps": NoStatusStrategy, "secrets": SecretStrategy,
              "serviceaccounts": NoStatusStrategy, "endpoints": NoStatusStrategy,
              "limitranges": NoStatusStrategy, "priorityclasses": NoStatusStrategy,
              "leases": NoStatusStrategy, "roles": NoStatusStrategy, "rolebindings": NoStatusStrategy,
              "clusterroles": NoStatusStrategy, "clusterrolebindings": NoStatusStrategy,
              "controllerrevisions": NoStatusStrategy, "storageclasses": NoStatusStrategy,
              "mutatingwebhookconfigurations": NoStatusStrategy, "validatingwebhookconfigurations": NoStatusStrategy,
              "networkpolicies": NoStatusStrategy, "podsecuritypolicies": NoStatusStrategy,
              "podpresets": NoStatusStrategy,
              "deployments": DeploymentStrategy, "replicasets": WorkloadStrategy, "statefulsets": WorkloadStrategy,
              "daemonsets": WorkloadStrategy, "replicationcontrollers": WorkloadStrategy, "jobs": JobStrategy,
              "cronjobs": WorkloadStrategy, "horizontalpodautoscalers": WorkloadStrategy,
              "poddisruptionbudgets": WorkloadStrategy, "ingresses": WorkloadStrategy,
              "persistentvolumes": VolumeStrategy, "persistentvolumeclaims": VolumeStrategy}


def export_object(strat, obj, exact=False):
    """`genericregistry.Store.Export` + `exportObjectMeta`."""
    from ..api.meta import fast_copy
    out = fast_copy(obj)
    md = out.setdefault("metadata", {})
    for k in ("uid", "creationTimestamp", "deletionTimestamp", "resourceVersion", "selfLink"):
        md.pop(k, None)
    if not exact:
        md.pop("namespace", None)
        if md.get("generateName"):
            md.pop("name", None)
        strat.export(out)
    return out


def strategy_for(ri):
    return STRATEGIES.get(ri.plural, Strategy)(ri)


def init_object_meta(obj, ri, namespace):
    m = obj.setdefault("metadata", {})
    if not m.get("name") and m.get("generateName"):
        m["name"] = generate_name(m["generateName"])
    if ri.namespaced:
        if m.get("namespace") and namespace and m["namespace"] != namespace:
            raise bad_request("the namespace of the provided object does not match the namespace sent on the request")
        m["namespace"] = namespace or m.get("namespace") or "default"
    else:
        m.pop("namespace", None)
    m["uid"] = new_uid()
    m["creationTimestamp"] = now_rfc3339()
    m.pop("deletionTimestamp", None)
    m.pop("deletionGracePeriodSeconds", None)
    if ri.plural not in ("nodes", "events", "namespaces"):
        m["generation"] = 1
    obj["kind"] = ri.kind
    obj["apiVersion"] = ri.group_version


def apply_binding(pod, binding) -> None:
    """Fork `setPodHostAndAnnotations` + `assignPod` (storage.go:155-210), mutating `pod`."""
    target = binding.get("target") or {}
    node = target.get("name", "")
    if not node:
        raise bad_request("Binding target name is required")
    spec = pod.setdefault("spec", {})
    meta = pod.setdefault("metadata", {})
    if meta.get("deletionTimestamp"):
        raise APIError(409, "Conflict", f"pod {meta.get('name')} is being deleted, cannot be assigned to a host")
    if spec.get("nodeName"):
        raise APIError(409, "Conflict", f"pod {meta.get('name')} is already assigned to node \"{spec['nodeName']}\"")
    spec["nodeName"] = node
    ann = (binding.get("metadata") or {}).get("annotations")
    if ann:
        meta.setdefault("annotations", {}).update(ann)
    erb = target.get("extendedResourceBinding") or {}
    for per in spec.get("extendedResources") or ():
        got = erb.get(per.get("name"))
        if got is None:
            raise bad_request(f"binding does not assign extended resource {per.get('name')}")
        ids = list(got.get("resources") or [])
        want = core.pod_extended_resource_count(per)
        if len(ids) != want or len(set(ids)) != len(ids):
            raise bad_request(f"extended resource {per.get('name')}: binding assigns {len(ids)} distinct devices, pod requests {want}")
        per["assigned"] = ids
    st = pod.setdefault("status", {})
    core.set_condition(st, {"type": core.COND_POD_SCHEDULED, "status": "True",
                            "lastProbeTime": None, "lastTransitionTime": now_rfc3339()})


def deletion_stamp(grace: int):
    return now_rfc3339(time.time() + grace)
