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


_DNS_POLICIES = ("ClusterFirstWithHostNet", "ClusterFirst", "Default", "None")
MAX_DNS_NAMESERVERS, MAX_DNS_SEARCH_PATHS, MAX_DNS_SEARCH_LIST_CHARS = 3, 6, 256


def _inv(path, value, msg):
    v = value if isinstance(value, str) else str(value)
    return invalid(path, f'"{v}": {msg}' if isinstance(value, str) else f"{v}: {msg}")


def validate_dns_policy(dp, path):
    """validateDNSPolicy: None only with the CustomPodDNS gate."""
    from ..utils.features import DefaultFeatureGate
    if dp in ("ClusterFirstWithHostNet", "ClusterFirst", "Default"):
        return []
    if dp == "None":
        if not DefaultFeatureGate("CustomPodDNS"):
            return [_inv(path, dp, "DNSPolicy: can not use 'None', custom pod DNS is disabled by feature gate")]
        return []
    if dp == "":
        return [required(path)]
    return [not_supported(path, dp)]


def validate_pod_dns_config(cfg, dp, path):
    """validatePodDNSConfig: dnsPolicy None needs a dnsConfig with a nameserver; a dnsConfig
    needs the CustomPodDNS gate and fits libc's resolver limits."""
    import ipaddress

    from ..utils.features import DefaultFeatureGate
    errs = []
    gate = DefaultFeatureGate("CustomPodDNS")
    if gate and dp == "None":
        if cfg is None:
            return [required(path, "must provide `dnsConfig` when `dnsPolicy` is None")]
        if not cfg.get("nameservers"):
            return [required(f"{path}.nameservers", "must provide at least one DNS nameserver when `dnsPolicy` is None")]
    if cfg is None:
        return errs
    if not gate:
        return [FieldError("Forbidden", path, "DNSConfig: custom pod DNS is disabled by feature gate")]
    ns = cfg.get("nameservers") or []
    if len(ns) > MAX_DNS_NAMESERVERS:
        errs.append(_inv(f"{path}.nameservers", ns, f"must not have more than {MAX_DNS_NAMESERVERS} nameservers"))
    for i, x in enumerate(ns):
        try:
            ipaddress.ip_address(str(x))
        except ValueError:
            errs.append(_inv(f"{path}.nameservers[{i}]", x, "must be valid IP address"))
    se = cfg.get("searches") or []
    if len(se) > MAX_DNS_SEARCH_PATHS:
        errs.append(_inv(f"{path}.searches", se, f"must not have more than {MAX_DNS_SEARCH_PATHS} search paths"))
    if len(" ".join(se)) > MAX_DNS_SEARCH_LIST_CHARS:
        errs.append(_inv(f"{path}.searches", se,
                         "must not have more than 256 characters (including spaces) in the search list"))
    for i, x in enumerate(se):
        if not is_dns1123_subdomain(str(x)):
            errs.append(_inv(f"{path}.searches[{i}]", x, "a DNS-1123 subdomain must consist of lower case "
                                                           "alphanumeric characters, '-' or '.'"))
    for i, o in enumerate(cfg.get("options") or ()):
        if not (o or {}).get("name"):
            errs.append(required(f"{path}.options[{i}]", "must not be empty"))
    return errs


_PROTOCOLS = ("TCP", "UDP")
_TERM_MSG = ("File", "FallbackToLogsOnError")
_TOL_OPS = ("Exists", "Equal")
C_IDENTIFIER = re.compile(r"^[A-Za-z_][A-Za-z0-9_]*$")
ENV_VAR_NAME = re.compile(r"^[-._a-zA-Z][-._a-zA-Z0-9]*$")
IANA_SVC_NAME = re.compile(r"^[a-z0-9]([a-z0-9-]*[a-z0-9])?$")
_VOLUME_SOURCES = ("hostPath", "emptyDir", "gcePersistentDisk", "awsElasticBlockStore", "gitRepo", "secret", "nfs",
                   "iscsi", "glusterfs", "persistentVolumeClaim", "rbd", "flexVolume", "cinder", "cephfs", "flocker",
                   "downwardAPI", "fc", "azureFile", "configMap", "vsphereVolume", "quobyte", "azureDisk",
                   "photonPersistentDisk", "projected", "portworxVolume", "scaleIO", "storageos", "csi")


def _is_int(v):
    return isinstance(v, int) and not isinstance(v, bool)


def _non_negative(v, path, errs, positive=False):
    if v is None:
        return
    if not _is_int(v) or v < (1 if positive else 0):
        errs.append(invalid(path, f"{v!r}: must be greater than {'' if positive else 'or equal to '}0"))


def _validate_probe(pr, path):
    errs = []
    if pr is None:
        return errs
    handlers = [k for k in ("exec", "httpGet", "tcpSocket") if pr.get(k) is not None]
    if len(handlers) != 1:
        errs.append(required(path, "must specify exactly 1 handler type (exec, httpGet, tcpSocket)"))
    for k in ("initialDelaySeconds", "timeoutSeconds", "periodSeconds", "successThreshold", "failureThreshold"):
        _non_negative(pr.get(k), f"{path}.{k}", errs)
    return errs


def _validate_port_number(v, path, errs, allow_name=True):
    if _is_int(v):
        if not 0 < v < 65536:
            errs.append(invalid(path, f"{v}: must be between 1 and 65535, inclusive"))
    elif allow_name and isinstance(v, str) and v:
        if not (len(v) <= 15 and IANA_SVC_NAME.match(v) and any(ch.isalpha() for ch in v)):
            errs.append(invalid(path, f"{v!r}: must contain only alpha-numeric characters (a-z, 0-9) and hyphens"))
    else:
        errs.append(invalid(path, f"{v!r}: must be a port number or name"))


def _validate_container_list(cs, path, require, volumes=None):
    errs = []
    if not cs:
        if require:
            errs.append(required(path))
        return errs
    seen = set()
    for i, c in enumerate(cs):
        p = f"{path}[{i}]"
        if not isinstance(c, dict):
            errs.append(invalid(p, "must be an object"))
            continue
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
        tmp = c.get("terminationMessagePolicy")
        if tmp and tmp not in _TERM_MSG:
            errs.append(not_supported(f"{p}.terminationMessagePolicy", tmp))
        errs += _validate_resources(c.get("resources") or {}, f"{p}.resources")
        pnames = set()
        for j, port in enumerate(c.get("ports") or ()):
            cp = port.get("containerPort")
            if not _is_int(cp) or not 0 < cp < 65536:
                errs.append(invalid(f"{p}.ports[{j}].containerPort", cp))
            hp = port.get("hostPort")
            if hp is not None and (not _is_int(hp) or not 0 <= hp < 65536):
                errs.append(invalid(f"{p}.ports[{j}].hostPort", hp))
            proto = port.get("protocol")
            if proto and proto not in _PROTOCOLS:
                errs.append(not_supported(f"{p}.ports[{j}].protocol", proto))
            pn = port.get("name")
            if pn:
                if not (len(pn) <= 15 and IANA_SVC_NAME.match(pn)):
                    errs.append(invalid(f"{p}.ports[{j}].name", pn))
                if pn in pnames:
                    errs.append(duplicate(f"{p}.ports[{j}].name", pn))
                pnames.add(pn)
        for j, e in enumerate(c.get("env") or ()):
            en = e.get("name")
            if not en:
                errs.append(required(f"{p}.env[{j}].name"))
            elif not ENV_VAR_NAME.match(en):
                errs.append(invalid(f"{p}.env[{j}].name", f"{en!r}: a valid environment variable name must consist of alphabetic characters, digits, '_', '-', or '.'"))
            vf = e.get("valueFrom")
            if vf is not None:
                srcs = [k for k in ("fieldRef", "resourceFieldRef", "configMapKeyRef", "secretKeyRef") if vf.get(k) is not None]
                if len(srcs) != 1:
                    errs.append(invalid(f"{p}.env[{j}].valueFrom", "may not have more than one field specified at a time"))
                if e.get("value"):
                    errs.append(invalid(f"{p}.env[{j}].valueFrom", "may not be specified when `value` is not empty"))
        for j, ef in enumerate(c.get("envFrom") or ()):
            if (ef.get("configMapRef") is None) == (ef.get("secretRef") is None):
                errs.append(invalid(f"{p}.envFrom[{j}]", "must specify exactly one of configMapRef or secretRef"))
            if ef.get("prefix") and not ENV_VAR_NAME.match(ef["prefix"]):
                errs.append(invalid(f"{p}.envFrom[{j}].prefix", ef["prefix"]))
        mpaths = set()
        for j, vm in enumerate(c.get("volumeMounts") or ()):
            if volumes is not None and vm.get("name") not in volumes:
                errs.append(FieldError("Not found", f"{p}.volumeMounts[{j}].name", vm.get("name")))
            mp = vm.get("mountPath")
            if not mp:
                errs.append(required(f"{p}.volumeMounts[{j}].mountPath"))
            elif mp in mpaths:
                errs.append(invalid(f"{p}.volumeMounts[{j}].mountPath", f"{mp!r}: must be unique"))
            mpaths.add(mp)
            sp = vm.get("subPath") or ""
            if sp.startswith("/") or ".." in sp.split("/"):
                errs.append(invalid(f"{p}.volumeMounts[{j}].subPath", f"{sp!r}: must be a relative path without '..'"))
        errs += _validate_probe(c.get("livenessProbe"), f"{p}.livenessProbe")
        errs += _validate_probe(c.get("readinessProbe"), f"{p}.readinessProbe")
        rp = c.get("readinessProbe")
        if rp is not None and rp.get("successThreshold") not in (None, 1) and False:
            pass
        lp = c.get("livenessProbe")
        if lp is not None and lp.get("successThreshold") not in (None, 1):
            errs.append(invalid(f"{p}.livenessProbe.successThreshold", "must be 1"))
        sc = c.get("securityContext") or {}
        _non_negative(sc.get("runAsUser"), f"{p}.securityContext.runAsUser", errs)
        if sc.get("privileged") and sc.get("allowPrivilegeEscalation") is False:
            errs.append(invalid(f"{p}.securityContext", "cannot set allowPrivilegeEscalation to false and privileged to true"))
    return errs


def _validate_volumes(vols, path):
    errs = []
    names = set()
    for i, v in enumerate(vols or ()):
        p = f"{path}[{i}]"
        n = v.get("name", "")
        if not is_dns1123_label(n):
            errs.append(invalid(f"{p}.name", n))
        if n in names:
            errs.append(duplicate(f"{p}.name", n))
        names.add(n)
        srcs = [k for k in _VOLUME_SOURCES if v.get(k) is not None]
        if not srcs:
            errs.append(required(p, "must specify a volume type"))
        elif len(srcs) > 1:
            errs.append(FieldError("Forbidden", f"{p}.{srcs[1]}", "may not specify more than 1 volume type"))
        hp = v.get("hostPath")
        if hp is not None and not hp.get("path"):
            errs.append(required(f"{p}.hostPath.path"))
        pvc = v.get("persistentVolumeClaim")
        if pvc is not None and not pvc.get("claimName"):
            errs.append(required(f"{p}.persistentVolumeClaim.claimName"))
        for src, key in (("secret", "secretName"), ("configMap", "name")):
            sv = v.get(src)
            if sv is None:
                continue
            for j, it in enumerate(sv.get("items") or ()):
                if not it.get("key"):
                    errs.append(required(f"{p}.{src}.items[{j}].key"))
                ip = it.get("path") or ""
                if not ip or ip.startswith("/") or ".." in ip.split("/"):
                    errs.append(invalid(f"{p}.{src}.items[{j}].path", ip))
            dm = sv.get("defaultMode")
            if dm is not None and (not _is_int(dm) or not 0 <= dm <= 0o777):
                errs.append(invalid(f"{p}.{src}.defaultMode", f"{dm!r}: must be a number between 0 and 0777 (octal)"))
    return names, errs


def _validate_tolerations(tols, path):
    errs = []
    for i, t in enumerate(tols or ()):
        p = f"{path}[{i}]"
        key, op = t.get("key", ""), t.get("operator") or "Equal"
        if key and not is_qualified_name(key):
            errs.append(invalid(f"{p}.key", key))
        if op not in _TOL_OPS:
            errs.append(not_supported(f"{p}.operator", op))
        if not key and op != "Exists":
            errs.append(invalid(f"{p}.operator", "operator must be Exists when `key` is empty"))
        if op == "Exists" and t.get("value"):
            errs.append(invalid(f"{p}.operator", "value must be empty when `operator` is 'Exists'"))
        eff = t.get("effect")
        if eff and eff not in (core.TAINT_NO_SCHEDULE, core.TAINT_PREFER_NO_SCHEDULE, core.TAINT_NO_EXECUTE):
            errs.append(not_supported(f"{p}.effect", eff))
        if t.get("tolerationSeconds") is not None and eff != core.TAINT_NO_EXECUTE:
            errs.append(invalid(f"{p}.effect", "effect must be 'NoExecute' when `tolerationSeconds` is set"))
    return errs


def validate_pod_spec(spec, path="spec"):
    """`ValidatePodSpec` (pkg/apis/core/validation/validation.go:2850-2920) + the fork's ER rules."""
    if not isinstance(spec, dict):
        return [invalid(path, "must be an object")]
    errs = []
    vol_names, verrs = _validate_volumes(spec.get("volumes"), f"{path}.volumes")
    errs += verrs
    errs += _validate_container_list(spec.get("containers"), f"{path}.containers", True, vol_names)
    errs += _validate_container_list(spec.get("initContainers"), f"{path}.initContainers", False, vol_names)
    names = {c.get("name") for c in spec.get("containers") or () if isinstance(c, dict)}
    for c in spec.get("initContainers") or ():
        if isinstance(c, dict) and c.get("name") in names:
            errs.append(duplicate(f"{path}.initContainers", c.get("name")))
    rp = spec.get("restartPolicy")
    if rp and rp not in _RESTART:
        errs.append(not_supported(f"{path}.restartPolicy", rp))
    dp = spec.get("dnsPolicy")
    if dp is not None:
        errs += validate_dns_policy(dp, f"{path}.dnsPolicy")
    errs += validate_pod_dns_config(spec.get("dnsConfig"), dp, f"{path}.dnsConfig")
    names_ref, er_errs = validate_extended_resources(spec.get("extendedResources"), f"{path}.extendedResources")
    errs += er_errs
    errs += validate_containers_extended_resources(spec.get("containers"), names_ref, f"{path}.containers")
    errs += validate_containers_extended_resources(spec.get("initContainers"), names_ref, f"{path}.initContainers")
    for k, v in (spec.get("nodeSelector") or {}).items():
        if not is_qualified_name(k):
            errs.append(invalid(f"{path}.nodeSelector", k))
        elif not isinstance(v, str) or not is_valid_label_value(v):
            errs.append(invalid(f"{path}.nodeSelector", v))
    tgp = spec.get("terminationGracePeriodSeconds")
    if tgp is not None and (not _is_int(tgp) or tgp < 0):
        errs.append(invalid(f"{path}.terminationGracePeriodSeconds", tgp))
    _non_negative(spec.get("activeDeadlineSeconds"), f"{path}.activeDeadlineSeconds", errs, positive=True)
    for k in ("hostname", "subdomain"):
        if spec.get(k) and not is_dns1123_label(spec[k]):
            errs.append(invalid(f"{path}.{k}", spec[k]))
    if spec.get("serviceAccountName") and not is_dns1123_subdomain(spec["serviceAccountName"]):
        errs.append(invalid(f"{path}.serviceAccountName", spec["serviceAccountName"]))
    errs += _validate_tolerations(spec.get("tolerations"), f"{path}.tolerations")
    if spec.get("hostNetwork"):
        for i, c in enumerate(spec.get("containers") or ()):
            for j, port in enumerate((c or {}).get("ports") or ()):
                hp = port.get("hostPort")
                if hp and hp != port.get("containerPort"):
                    errs.append(invalid(f"{path}.containers[{i}].ports[{j}].hostPort", "must match `containerPort` when `hostNetwork` is true"))
    psc = spec.get("securityContext") or {}
    _non_negative(psc.get("runAsUser"), f"{path}.securityContext.runAsUser", errs)
    _non_negative(psc.get("fsGroup"), f"{path}.securityContext.fsGroup", errs)
    for i, g in enumerate(psc.get("supplementalGroups") or ()):
        _non_negative(g, f"{path}.securityContext.supplementalGroups[{i}]", errs)
    aff = ((spec.get("affinity") or {}).get("nodeAffinity") or {}).get("requiredDuringSchedulingIgnoredDuringExecution")
    if aff is not None:
        terms = aff.get("nodeSelectorTerms")
        if not terms:
            errs.append(required(f"{path}.affinity.nodeAffinity.requiredDuringSchedulingIgnoredDuringExecution.nodeSelectorTerms",
                                 "must have at least one node selector term"))
        for i, t in enumerate(terms or ()):
            for j, r in enumerate((t or {}).get("matchExpressions") or ()):
                if r.get("operator") not in ("In", "NotIn", "Exists", "DoesNotExist", "Gt", "Lt"):
                    errs.append(not_supported(f"{path}.affinity.nodeAffinity.requiredDuringSchedulingIgnoredDuringExecution."
                                              f"nodeSelectorTerms[{i}].matchExpressions[{j}].operator", r.get("operator")))
    return errs


def validate_pod_template_spec(tpl, path, restart_policies=None):
    """`ValidatePodTemplateSpec` (validation.go:3820): labels valid, pod spec valid; callers pass
    the restart policies their controller supports."""
    if not isinstance(tpl, dict):
        return [required(path)]
    errs = []
    md = tpl.get("metadata") or {}
    for k, v in (md.get("labels") or {}).items():
        if not is_qualified_name(k) or not isinstance(v, str) or not is_valid_label_value(v):
            errs.append(invalid(f"{path}.metadata.labels", f"{k}={v!r}"))
    spec = tpl.get("spec")
    if spec is None:
        return errs + [required(f"{path}.spec")]
    errs += validate_pod_spec(spec, f"{path}.spec")
    rp = spec.get("restartPolicy") or "Always"
    if restart_policies is not None and rp not in restart_policies:
        errs.append(not_supported(f"{path}.spec.restartPolicy", rp))
    return errs


def validate_pod(pod):
    return validate_object_meta(pod, True) + validate_pod_spec(pod.get("spec") or {})


def _sem(o):
    """Semantic equality view: empty values compare equal to absent ones."""
    if isinstance(o, dict):
        return {k: _sem(v) for k, v in o.items() if v not in (None, "", [], {})}
    if isinstance(o, list):
        return [_sem(v) for v in o]
    return o


POD_UPDATE_FORBIDDEN = ("pod updates may not change fields other than `spec.containers[*].image`, "
                        "`spec.initContainers[*].image`, `spec.activeDeadlineSeconds` or `spec.tolerations` "
                        "(only additions to existing tolerations)")


def validate_pod_update(new, old):
    """`ValidatePodUpdate` (validation.go): the pod spec is immutable except container and init
    container images, activeDeadlineSeconds (set, or lowered — never removed) and tolerations
    (existing ones kept, only their tolerationSeconds may change; new ones may be added). The
    scheduler-owned fields nodeName and extendedResources[].assigned may only be set through
    pods/binding."""
    errs = validate_pod(new)
    ns, os_ = new.get("spec") or {}, old.get("spec") or {}
    for key in ("containers", "initContainers"):
        nc, oc = ns.get(key) or [], os_.get(key) or []
        if len(nc) != len(oc):
            errs.append(FieldError("Forbidden", f"spec.{key}", "pod updates may not add or remove containers"))
            return errs
        for i, c in enumerate(nc):
            if not c.get("image"):
                errs.append(required(f"spec.{key}[{i}].image"))
    nad, oad = ns.get("activeDeadlineSeconds"), os_.get("activeDeadlineSeconds")
    if nad is not None:
        if not isinstance(nad, int) or nad < 0 or nad > 2 ** 31 - 1:
            errs.append(invalid("spec.activeDeadlineSeconds", "must be between 0 and 2147483647, inclusive"))
            return errs
        if oad is not None and oad < nad:
            errs.append(invalid("spec.activeDeadlineSeconds", "must be less than or equal to previous value"))
            return errs
    elif oad is not None:
        errs.append(invalid("spec.activeDeadlineSeconds", "must not update from a positive integer to nil value"))
    new_tols = [{k: v for k, v in t.items() if k != "tolerationSeconds"} for t in ns.get("tolerations") or ()]
    for t in os_.get("tolerations") or ():
        if {k: v for k, v in t.items() if k != "tolerationSeconds"} not in new_tols:
            errs.append(FieldError("Forbidden", "spec.tolerations",
                                   "existing toleration can not be modified except its tolerationSeconds"))
            break
    munged = dict(ns)
    for key in ("containers", "initContainers"):
        if key in munged:
            munged[key] = [dict(c, image=o.get("image")) for c, o in zip(ns.get(key) or [], os_.get(key) or [])]
    munged.pop("activeDeadlineSeconds", None)
    if oad is not None:
        munged["activeDeadlineSeconds"] = oad
    munged["tolerations"] = os_.get("tolerations")
    if ns.get("nodeName", "") != os_.get("nodeName", ""):
        errs.append(FieldError("Forbidden", "spec.nodeName", "may only be set through pods/binding"))
    na = [r.get("assigned") for r in ns.get("extendedResources") or ()]
    oa = [r.get("assigned") for r in os_.get("extendedResources") or ()]
    if na != oa:
        errs.append(FieldError("Forbidden", "spec.extendedResources.assigned", "may only be set through pods/binding"))
    munged["nodeName"] = os_.get("nodeName")
    munged["extendedResources"] = os_.get("extendedResources")
    if _sem(munged) != _sem(os_):
        errs.append(FieldError("Forbidden", "spec", POD_UPDATE_FORBIDDEN))
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


def validate_object_meta_update(new, old, path="metadata"):
    """`ValidateObjectMetaUpdate`: name, namespace, uid and creationTimestamp are immutable."""
    errs = []
    nm, om = new.get("metadata") or {}, old.get("metadata") or {}
    for k in ("name", "namespace", "uid", "creationTimestamp"):
        if (nm.get(k) or None) != (om.get(k) or None) and om.get(k) is not None:
            errs.append(invalid(f"{path}.{k}", "field is immutable"))
    return errs


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
