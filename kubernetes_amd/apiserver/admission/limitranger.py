"""LimitRanger admission: LimitRange defaults and min / max / maxLimitRequestRatio.

Parity: `plugin/pkg/admission/limitranger/admission.go`
  * defaults (`defaultContainerResourceRequirements` / `mergeContainerResources` /
    `mergePodResourceRequirements`, :203-281): every Container item's `default` (limits) and
    `defaultRequest` (requests) fill what a container — init containers included — leaves
    unset, and the pod is annotated `kubernetes.io/limit-ranger: LimitRanger plugin set: ...`;
  * constraints (`minConstraint` / `maxConstraint` / `maxRequestConstraint` /
    `limitRequestRatioConstraint`, :298-374) for the Container type (each container and init
    container), the Pod type (sum over containers, then max with every init container,
    :545-592) and the PersistentVolumeClaim type (requests.storage only, :464-486), with the
    reference's error strings, aggregated per LimitRange like `utilerrors.NewAggregate`;
  * the reference compares at milli precision (`requestLimitEnforcedValues`, :284-295).

GPU-aware: after ResourceV2 moves `amd.com/gpu` out of container limits into
`spec.extendedResources`, the constraints still see it — a container's requests/limits
include the pod-level entries it names in `extendedResourceRequests`, so
`LimitRange{max: {amd.com/gpu: 2}}` refuses a 4-GPU container (Container type) or pod (Pod type).
Defaults run before ResourceV2 in the mutating chain (as in `hack/local-up-cluster.sh:424`), so a
defaulted `amd.com/gpu` limit is converted like one the user wrote.

Deliberate difference: defaults are applied on CREATE only. The 1.9 plugin also mutates on
UPDATE, which makes any later update of a pod that predates a LimitRange fail pod-spec
immutability (upstream later stopped handling pod updates); constraints are still enforced on
UPDATE, as `TestLimitRangerAdmitPod` expects.
"""
from __future__ import annotations

from ...api.quantity import Quantity, parse_quantity
from . import CREATE, UPDATE, AdmissionError, Plugin, register

LIMIT_RANGER_ANNOTATION = "kubernetes.io/limit-ranger"
CONTAINER, POD, PVC = "Container", "Pod", "PersistentVolumeClaim"


def _q(v) -> Quantity:
    return v if isinstance(v, Quantity) else parse_quantity(str(v))


def _milli(q: Quantity) -> int:
    return q.milli_value()


# -- defaults ------------------------------------------------------------------------------------

def default_container_requirements(limit_range) -> tuple[dict, dict]:
    """(requests, limits) defaults from the LimitRange's Container items (:203-222)."""
    req, lim = {}, {}
    for item in (limit_range.get("spec") or {}).get("limits") or ():
        if item.get("type") == CONTAINER:
            req.update(item.get("defaultRequest") or {})
            lim.update(item.get("default") or {})
    return req, lim


def merge_container_resources(container, defaults, prefix, notes):
    dreq, dlim = defaults
    res = container.get("resources") or {}
    limits = dict(res.get("limits") or {})
    requests = dict(res.get("requests") or {})
    set_lim = sorted(k for k in dlim if k not in limits)
    set_req = sorted(k for k in dreq if k not in requests)
    for k in set_lim:
        limits[k] = dlim[k]
    for k in set_req:
        requests[k] = dreq[k]
    if set_lim or set_req:
        res = dict(res)
        res["limits"], res["requests"] = limits, requests
        container["resources"] = res
    if set_req:
        notes.append(f"{', '.join(set_req)} request for {prefix} {container.get('name', '')}")
    if set_lim:
        notes.append(f"{', '.join(set_lim)} limit for {prefix} {container.get('name', '')}")
    return notes


def merge_pod_resource_requirements(pod, defaults):
    """:263-281 — containers, then init containers; one annotation lists what was set."""
    notes: list[str] = []
    spec = pod.setdefault("spec", {})
    for c in spec.get("containers") or ():
        merge_container_resources(c, defaults, "container", notes)
    for c in spec.get("initContainers") or ():
        merge_container_resources(c, defaults, "init container", notes)
    if notes:
        md = pod.setdefault("metadata", {})
        md["annotations"] = dict(md.get("annotations") or {},
                                 **{LIMIT_RANGER_ANNOTATION: "LimitRanger plugin set: " + "; ".join(notes)})


def pod_mutate_limit(limit_range, pod):
    merge_pod_resource_requirements(pod, default_container_requirements(limit_range))


# -- constraints ---------------------------------------------------------------------------------

def min_constraint(kind, rname, enforced, request, limit):
    enf = _q(enforced)
    if rname not in request:
        return f"minimum {rname} usage per {kind} is {enf}.  No request is specified."
    req = _q(request[rname])
    if _milli(req) < _milli(enf):
        return f"minimum {rname} usage per {kind} is {enf}, but request is {req}."
    if rname in limit and _milli(_q(limit[rname])) < _milli(enf):
        return f"minimum {rname} usage per {kind} is {enf}, but limit is {_q(limit[rname])}."
    return None


def max_request_constraint(kind, rname, enforced, request):
    enf = _q(enforced)
    if rname not in request:
        return f"maximum {rname} usage per {kind} is {enf}.  No request is specified."
    req = _q(request[rname])
    if _milli(req) > _milli(enf):
        return f"maximum {rname} usage per {kind} is {enf}, but request is {req}."
    return None


def max_constraint(kind, rname, enforced, request, limit):
    enf = _q(enforced)
    if rname not in limit:
        return f"maximum {rname} usage per {kind} is {enf}.  No limit is specified."
    lim = _q(limit[rname])
    if _milli(lim) > _milli(enf):
        return f"maximum {rname} usage per {kind} is {enf}, but limit is {lim}."
    if rname in request and _milli(_q(request[rname])) > _milli(enf):
        return f"maximum {rname} usage per {kind} is {enf}, but request is {_q(request[rname])}."
    return None


def limit_request_ratio_constraint(kind, rname, enforced, request, limit):
    enf = _q(enforced)
    req = _milli(_q(request[rname])) if rname in request else 0
    lim = _milli(_q(limit[rname])) if rname in limit else 0
    if req == 0:
        return (f"{rname} max limit to request ratio per {kind} is {enf}, but no request is specified or "
                f"request is 0.")
    if lim == 0:
        return f"{rname} max limit to request ratio per {kind} is {enf}, but no limit is specified or limit is 0."
    ratio = lim / req
    if ratio * 1000 > _milli(enf):
        return f"{rname} max limit to request ratio per {kind} is {enf}, but provided ratio is {ratio:f}."
    return None


def _container_resources(container, ers):
    """(requests, limits) of a container as Quantity maps, its pod-level extended resources
    (ResourceV2, the `amd.com/gpu` it asked for) included."""
    res = container.get("resources") or {}
    req = {k: _q(v) for k, v in (res.get("requests") or {}).items()}
    lim = {k: _q(v) for k, v in (res.get("limits") or {}).items()}
    for name in container.get("extendedResourceRequests") or ():
        per = ers.get(name)
        if per is None:
            continue
        r = per.get("resources") or {}
        for k, v in (r.get("requests") or {}).items():
            req[k] = req.get(k, Quantity(0)) + _q(v)
        for k, v in (r.get("limits") or {}).items():
            lim[k] = lim.get(k, Quantity(0)) + _q(v)
    return req, lim


def _sum(lists):
    """:378-413 — a key missing from any input is omitted from the sum."""
    keys = set()
    for d in lists:
        keys.update(d)
    out = {}
    for k in keys:
        if all(k in d for d in lists):
            total = Quantity(0)
            for d in lists:
                total = total + d[k]
            out[k] = total
    return out


def _check_item(kind, item, requests, limits, errs):
    for k, v in (item.get("min") or {}).items():
        e = min_constraint(kind, k, v, requests, limits)
        if e:
            errs.append(e)
    for k, v in (item.get("max") or {}).items():
        e = max_constraint(kind, k, v, requests, limits)
        if e:
            errs.append(e)
    for k, v in (item.get("maxLimitRequestRatio") or {}).items():
        e = limit_request_ratio_constraint(kind, k, v, requests, limits)
        if e:
            errs.append(e)


def pod_validate_limit(limit_range, pod) -> list[str]:
    """:499-595."""
    spec = pod.get("spec") or {}
    ers = {per.get("name"): per for per in spec.get("extendedResources") or ()}
    ctrs = [_container_resources(c, ers) for c in spec.get("containers") or ()]
    inits = [_container_resources(c, ers) for c in spec.get("initContainers") or ()]
    errs: list[str] = []
    for item in (limit_range.get("spec") or {}).get("limits") or ():
        kind = item.get("type")
        if kind == CONTAINER:
            for req, lim in ctrs + inits:
                _check_item(kind, item, req, lim, errs)
        elif kind == POD:
            preq = _sum([r for r, _ in ctrs])
            plim = _sum([l for _, l in ctrs])
            for req, lim in inits:          # max(sum of containers, any init container)
                for k, v in req.items():
                    if k not in preq or v > preq[k]:
                        preq[k] = v
                for k, v in lim.items():
                    if k not in plim or v > plim[k]:
                        plim[k] = v
            _check_item(kind, item, preq, plim, errs)
    return errs


def pvc_validate_limit(limit_range, pvc) -> list[str]:
    """:464-486 — requests only: limits are not user input for claims."""
    requests = ((pvc.get("spec") or {}).get("resources") or {}).get("requests") or {}
    errs: list[str] = []
    for item in (limit_range.get("spec") or {}).get("limits") or ():
        if item.get("type") != PVC:
            continue
        for k, v in (item.get("min") or {}).items():
            e = min_constraint(PVC, k, v, requests, {})
            if e:
                errs.append(e)
        for k, v in (item.get("max") or {}).items():
            e = max_request_constraint(PVC, k, v, requests)
            if e:
                errs.append(e)
    return errs


def aggregate(errs):
    """utilerrors.NewAggregate(...).Error()."""
    return errs[0] if len(errs) == 1 else "[" + ", ".join(errs) + "]"


@register
class LimitRanger(Plugin):
    name = "LimitRanger"
    operations = (CREATE, UPDATE)

    def _limit_ranges(self, a):
        if a.subresource or a.resource not in ("pods", "persistentvolumeclaims") or not self.server:
            return ()
        if not isinstance(a.obj, dict):
            return ()
        return self.server.list_objects("limitranges", a.namespace) or ()

    def admit(self, a):
        if a.operation != CREATE or a.resource != "pods":
            return
        for lr in self._limit_ranges(a):
            pod_mutate_limit(lr, a.obj)

    def validate(self, a):
        for lr in self._limit_ranges(a):
            errs = pod_validate_limit(lr, a.obj) if a.resource == "pods" else pvc_validate_limit(lr, a.obj)
            if errs:
                md = a.obj.get("metadata") or {}
                name = md.get("name") or md.get("generateName") or "Unknown"
                raise AdmissionError(f'{a.resource} "{name}" is forbidden: {aggregate(errs)}')


__all__ = ["LimitRanger", "LIMIT_RANGER_ANNOTATION", "pod_mutate_limit", "pod_validate_limit", "pvc_validate_limit",
           "default_container_requirements", "merge_pod_resource_requirements"]
