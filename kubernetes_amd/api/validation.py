"""Object validation (the subset of `pkg/apis/core/validation/validation.go` the served
resources need), including the fork's ResourceV2 rules:

  * `ValidateExtendedResources`  (validation.go:2950-2991): names unique & non-empty,
    exactly one limit and one request, equal, selector parses.
  * `validateContainersExtendedResources` (validation.go:2457-2483): references exist and
    are not shared. The reference only checks `containers` (call site :2883-2888); we also
    check `initContainers`.
"""
from __future__ import annotations

import re

from . import core
from .labels import SelectorError, is_qualified_name, is_valid_label_value
from .quantity import QuantityError, parse_quantity

DNS1123_LABEL = re.compile(r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?$")
DNS1123_SUBDOMAIN = re.compile(r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*$")


class FieldError:
    __slots__ = ("type", "field", "detail")

    def __init__(self, type_, field, detail):
        self.type, self.field, self.detail = type_, field, detail

    def __str__(self):
        return f"{self.field}: {self.type}: {self.detail}" if self.detail != "" else f"{self.field}: {self.type}"

    __repr__ = __str__


def invalid(field, detail):
    return FieldError("Invalid value", field, detail)


def required(field, detail="Required value"):
    return FieldError("Required value", field, detail)


def duplicate(field, detail):
    return FieldError("Duplicate value", field, detail)


def not_supported(field, detail):
    return FieldError("Unsupported value", field, detail)


def is_dns1123_label(s):
    return bool(s) and len(s) <= 63 and bool(DNS1123_LABEL.match(s))


def is_dns1123_subdomain(s):
    return bool(s) and len(s) <= 253 and bool(DNS1123_SUBDOMAIN.match(s))


def validate_object_meta(obj, namespaced: bool, name_fn=is_dns1123_subdomain, path="metadata"):
    errs = []
    m = obj.get("metadata") or {}
    name = m.get("name")
    if not name and not m.get("generateName"):
        errs.append(required(f"{path}.name", "name or generateName is required"))
    elif name and not name_fn(name):
        errs.append(invalid(f"{path}.name", f"{name!r}: a DNS-1123 subdomain must consist of lower case alphanumeric characters, '-' or '.'"))
    ns = m.get("namespace")
    if namespaced:
        if not ns:
            errs.append(required(f"{path}.namespace"))
        elif not is_dns1123_label(ns):
            errs.append(invalid(f"{path}.namespace", ns))
    elif ns:
        errs.append(FieldError("Forbidden", f"{path}.namespace", "not allowed on this type"))
    for k, v in (m.get("labels") or {}).items():
        if not is_qualified_name(k):
            errs.append(invalid(f"{path}.labels", f"invalid label key {k!r}"))
        if not isinstance(v, str) or not is_valid_label_value(v):
            errs.append(invalid(f"{path}.labels", f"invalid label value {v!r}"))
    for k in (m.get("annotations") or {}):
        if not is_qualified_name(k.lower()):
            errs.append(invalid(f"{path}.annotations", f"invalid annotation key {k!r}"))
    return errs


def _validate_resource_list(rl, path):
    errs = []
    for k, v in (rl or {}).items():
        if not is_qualified_name(k) and k not in core.BASIC_RESOURCES:
            errs.append(invalid(f"{path}[{k}]", "must be a standard resource type or fully qualified"))
        try:
            qv = parse_quantity(str(v))
        except QuantityError:
            errs.append(invalid(f"{path}[{k}]", f"{v!r}: quantities must match the regular expression"))
            continue
        if qv.value < 0:
            errs.append(invalid(f"{path}[{k}]", "must be greater than or equal to 0"))
        if core.is_extended_resource_name(k) and qv.value.denominator != 1:
            errs.append(invalid(f"{path}[{k}]", "must be an integer"))
    return errs


def _validate_resources(res, path):
    errs = []
    lim = res.get("limits") or {}
    req = res.get("requests") or {}
    errs += _validate_resource_list(lim, f"{path}.limits")
    errs += _validate_resource_list(req, f"{path}.requests")
    if errs:
        return errs
    for k, v in req.items():
        if k in lim and parse_quantity(str(v)) > parse_quantity(str(lim[k])):
            errs.append(invalid(f"{path}.requests[{k}]", "must be less than or equal to limit"))
        if core.is_extended_resource_name(k) and k in lim and parse_quantity(str(v)) != parse_quantity(str(lim[k])):
            errs.append(invalid(f"{path}.requests[{k}]", "must be equal to limit for extended resources"))
    return errs


def validate_extended_resources(ers, path="spec.extendedResources"):
    """Fork `ValidateExtendedResources`: returns (name -> ref count map, errors)."""
    collection: dict[str, int] = {}
    errs = []
    for i, r in enumerate(ers or ()):
        p = f"{path}[{i}]"
        name = r.get("name", "")
        if not name:
            errs.append(invalid(p, "Extended resource name can't be empty"))
        if name in collection:
            errs.append(invalid(p, "Extended resource name should be unique"))
        collection[name] = 0
        res = r.get("resources") or {}
        lim = res.get("limits") or {}
        req = res.get("requests") or {}
        if len(lim) != 1:
            errs.append(invalid(f"{p}.resources.limits", "unexpected limits length != 1"))
        if len(req) != 1:
            errs.append(invalid(f"{p}.resources.requests", "unexpected requests length != 1"))
        for rn, lv in lim.items():
            rv = req.get(rn)
            try:
                if rv is None or parse_quantity(str(rv)) != parse_quantity(str(lv)):
                    errs.append(invalid(f"{p}.resources", "Invalid Requests, Limits and Requests should be equal"))
                elif parse_quantity(str(lv)).value <= 0 or parse_quantity(str(lv)).value.denominator != 1:
                    errs.append(invalid(f"{p}.resources", "device count must be a positive integer"))
            except QuantityError as e:
                errs.append(invalid(f"{p}.resources", str(e)))
        aff = (r.get("affinity") or {}).get("required")
        if aff:
            try:
                core.extended_requirements_as_selector(aff)
            except SelectorError as e:
                errs.append(invalid(f"{p}.affinity", str(e)))
    return collection, errs


def validate_containers_extended_resources(containers, names, path):
    errs = []
    for ci, c in enumerate(containers or ()):
        for v in c.get("extendedResourceRequests") or ():
            if v not in names:
                errs.append(invalid(f"{path}[{ci}].extendedResourceRequests", "Reference to unknown extended resource"))
                continue
            if names[v] != 0:
                errs.append(invalid(f"{path}[{ci}].extendedResourceRequests",
                                    "Multiple reference to extended resource (sharing is not allowed)"))
                continue
            names[v] += 1
    return errs


_RESTART = ("Always", "OnFailure", "Never")
_PULL = ("Always", "IfNotPresent", "Never")


def _validate_container_list(cs, path, require):
    errs = []
    if not cs:
        if require:
            errs.append(required(path))
        return errs
    seen = set()
    for i, c in enumerate(cs):
        p = f"{path}[{i}]"
        name = c.get("name", "")
        if not is_dns1123_label(name):
            errs.append(invalid(f"{p}.name", f"{name!r} must be a DNS-1123 label"))
        if name in seen:
            errs.append(duplicate(f"{p}.name", name))
        seen.add(name)
        if not c.get("image"):
            errs.append(required(f"{p}.image"))
        pp = c.get("imagePullPolicy")
        if pp and pp not in _PULL:
            errs.append(not_supported(f"{p}.imagePullPolicy", pp))
        errs += _validate_resources(c.get("resources") or {}, f"{p}.resources")
        for j, port in enumerate(c.get("ports") or ()):
            cp = port.get("containerPort")
            if not isinstance(cp, int) or not 0 < cp < 65536:
                errs.append(invalid(f"{p}.ports[{j}].containerPort", cp))
        for j, e in enumerate(c.get("env") or ()):
            if not e.get("name"):
                errs.append(required(f"{p}.env[{j}].name"))
    return errs


def validate_pod_spec(spec, path="spec"):
    errs = []
    errs += _validate_container_list(spec.get("containers"), f"{path}.containers", True)
    errs += _validate_container_list(spec.get("initContainers"), f"{path}.initContainers", False)
    names = {c.get("name") for c in spec.get("containers") or ()}
    for c in spec.get("initContainers") or ():
        if c.get("name") in names:
            errs.append(duplicate(f"{path}.initContainers", c.get("name")))
    rp = spec.get("restartPolicy")
    if rp and rp not in _RESTART:
        errs.append(not_supported(f"{path}.restartPolicy", rp))
    names_ref, er_errs = validate_extended_resources(spec.get("extendedResources"), f"{path}.extendedResources")
    errs += er_errs
    errs += validate_containers_extended_resources(spec.get("containers"), names_ref, f"{path}.containers")
    errs += validate_containers_extended_resources(spec.get("initContainers"), names_ref, f"{path}.initContainers")
    for k, v in (spec.get("nodeSelector") or {}).items():
        if not is_qualified_name(k):
            errs.append(invalid(f"{path}.nodeSelector", k))
    vols = set()
    for i, v in enumerate(spec.get("volumes") or ()):
        n = v.get("name", "")
        if not is_dns1123_label(n):
            errs.append(invalid(f"{path}.volumes[{i}].name", n))
        if n in vols:
            errs.append(duplicate(f"{path}.volumes[{i}].name", n))
        vols.add(n)
    tgp = spec.get("terminationGracePeriodSeconds")
    if tgp is not None and (not isinstance(tgp, int) or tgp < 0):
        errs.append(invalid(f"{path}.terminationGracePeriodSeconds", tgp))
    return errs


def validate_pod(pod):
    return validate_object_meta(pod, True) + validate_pod_spec(pod.get("spec") or {})


def validate_pod_update(new, old):
    """Pod spec is immutable except for image / activeDeadlineSeconds / tolerations
    (validation.go `ValidatePodUpdate`). The scheduler-owned fields nodeName and
    extendedResources[].assigned may only be set through pods/binding."""
    errs = validate_pod(new)
    ns, os_ = new.get("spec") or {}, old.get("spec") or {}
    if ns.get("nodeName", "") != os_.get("nodeName", ""):
        errs.append(FieldError("Forbidden", "spec.nodeName", "may only be set through pods/binding"))
    na = [r.get("assigned") for r in ns.get("extendedResources") or ()]
    oa = [r.get("assigned") for r in os_.get("extendedResources") or ()]
    if na != oa:
        errs.append(FieldError("Forbidden", "spec.extendedResources.assigned", "may only be set through pods/binding"))
    return errs


def validate_node(node):
    errs = validate_object_meta(node, False)
    st = node.get("status") or {}
    for rname, dom in (st.get("extendedResources") or {}).items():
        for did, dev in ((dom or {}).get("resources") or {}).items():
            if dev.get("health") not in (None, "", core.HEALTHY, core.UNHEALTHY):
                errs.append(invalid(f"status.extendedResources[{rname}].resources[{did}].health", dev.get("health")))
    for t in (node.get("spec") or {}).get("taints") or ():
        if t.get("effect") not in (core.TAINT_NO_SCHEDULE, core.TAINT_PREFER_NO_SCHEDULE, core.TAINT_NO_EXECUTE):
            errs.append(not_supported("spec.taints.effect", t.get("effect")))
    return errs


def validate_namespace(ns):
    return validate_object_meta(ns, False, is_dns1123_label)


def validate_generic(obj, namespaced):
    return validate_object_meta(obj, namespaced)


def is_path_segment_name(s):
    """`path.IsValidPathSegmentName` — RBAC object names may contain ':' (system:node ...)."""
    return bool(s) and s not in (".", "..") and "/" not in s and "%" not in s


def _rbac(namespaced):
    return lambda obj: validate_object_meta(obj, namespaced, is_path_segment_name)


VALIDATORS = {
    "Pod": validate_pod,
    "Node": validate_node,
    "Namespace": validate_namespace,
    "Role": _rbac(True),
    "RoleBinding": _rbac(True),
    "ClusterRole": _rbac(False),
    "ClusterRoleBinding": _rbac(False),
}
