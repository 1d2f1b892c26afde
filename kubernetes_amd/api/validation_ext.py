"""Validation of every served kind beyond pods / nodes / namespaces / services.

Each validator returns a list of `FieldError`s (the API server answers 422 Invalid with their
field paths); `UPDATE_VALIDATORS` adds the update-only rules (immutable fields). Parity
(reference `/root/reference` paths):
  * core: `pkg/apis/core/validation/validation.go` — ValidateReplicationController(Spec)
    :3781-3830, ValidatePodTemplate(Spec) :3820, ValidateConfigMap :4376, ValidateSecret,
    ValidateEndpoints, ValidateLimitRange, ValidateResourceQuota, ValidateServiceAccount,
    ValidatePersistentVolume(Claim), ValidateEvent;
  * apps / extensions: `pkg/apis/extensions/validation/validation.go` — ValidateDeploymentSpec
    :268, ValidateDeployment :365, ValidateReplicaSetSpec, ValidateDaemonSetSpec, ValidateIngress;
    `pkg/apis/apps/validation/validation.go` — ValidateStatefulSetSpec, ValidateControllerRevision;
  * batch: `pkg/apis/batch/validation/validation.go` — validateJobSpec / ValidateJob :78-150,
    ValidateCronJob;
  * autoscaling, policy (PDB, PSP), rbac, storage, networking, scheduling, settings,
    certificates, admissionregistration, apiregistration: the matching
    `pkg/apis/<group>/validation/validation.go`.
"""
from __future__ import annotations

import ipaddress
import re

from . import core
from .labels import LABEL_SELECTOR_OPS, SelectorError, is_qualified_name, is_valid_label_value, label_selector_as_selector
from .quantity import QuantityError, parse_quantity
from .validation import (FieldError, _is_int, _non_negative, _validate_resource_list, duplicate, invalid,
                         is_dns1123_label, is_dns1123_subdomain, is_path_segment_name, not_supported, required,
                         validate_object_meta, validate_object_meta_update, validate_pod_template_spec)

CONFIG_MAP_KEY = re.compile(r"^[-._a-zA-Z0-9]+$")
MAX_SECRET_SIZE = 1024 * 1024


def forbidden(field, detail):
    return FieldError("Forbidden", field, detail)


# ---------------------------------------------------------------------------------------------
# shared pieces
def validate_label_selector(sel, path):
    """`ValidateLabelSelector` (apimachinery meta/v1/validation)."""
    errs = []
    if sel is None:
        return errs
    for k, v in (sel.get("matchLabels") or {}).items():
        if not is_qualified_name(k):
            errs.append(invalid(f"{path}.matchLabels", f"invalid label key {k!r}"))
        if not isinstance(v, str) or not is_valid_label_value(v):
            errs.append(invalid(f"{path}.matchLabels", f"invalid label value {v!r}"))
    for i, e in enumerate(sel.get("matchExpressions") or ()):
        p = f"{path}.matchExpressions[{i}]"
        op = e.get("operator")
        if op not in LABEL_SELECTOR_OPS:
            errs.append(invalid(f"{p}.operator", f"{op!r} is not a valid pod selector operator"))
            continue
        if op in ("In", "NotIn") and not e.get("values"):
            errs.append(required(f"{p}.values", "must be specified when `operator` is 'In' or 'NotIn'"))
        if op in ("Exists", "DoesNotExist") and e.get("values"):
            errs.append(forbidden(f"{p}.values", "may not be specified when `operator` is 'Exists' or 'DoesNotExist'"))
        if not is_qualified_name(e.get("key", "")):
            errs.append(invalid(f"{p}.key", e.get("key")))
    return errs


def _selector_matches_template(sel, tpl, path):
    """The selector is non-empty and the template's labels satisfy it."""
    if sel is None:
        return [required(f"{path}.selector")]
    if not (sel.get("matchLabels") or sel.get("matchExpressions")):
        return [invalid(f"{path}.selector", "empty selector is invalid for deployment")]
    errs = validate_label_selector(sel, f"{path}.selector")
    if errs:
        return errs
    labels = ((tpl or {}).get("metadata") or {}).get("labels") or {}
    try:
        if not label_selector_as_selector(sel).matches(labels):
            errs.append(invalid(f"{path}.template.metadata.labels", f"{labels}: `selector` does not match template `labels`"))
    except SelectorError as e:
        errs.append(invalid(f"{path}.selector", str(e)))
    return errs


def _int_or_percent(v, path, errs, allow_zero=True):
    """An IntOrString that must be a non-negative int or a percentage 0..100%."""
    if _is_int(v):
        if v < 0 or (not allow_zero and v == 0):
            errs.append(invalid(path, f"{v}: must be greater than {'or equal to ' if allow_zero else ''}0"))
        return v
    if isinstance(v, str):
        m = re.fullmatch(r"(\d+)%", v)
        if not m:
            errs.append(invalid(path, f"{v!r}: must be an integer or percentage (e.g '5%')"))
            return None
        pct = int(m.group(1))
        if pct > 100:
            errs.append(invalid(path, f"{v!r}: must not be greater than 100%"))
        return pct if pct else 0
    if v is not None:
        errs.append(invalid(path, f"{v!r}: must be an integer or percentage"))
    return None


def _replicas(spec, path, errs):
    _non_negative(spec.get("replicas"), f"{path}.replicas", errs)
    _non_negative(spec.get("minReadySeconds"), f"{path}.minReadySeconds", errs)


def _meta(obj, namespaced=True, name_fn=is_dns1123_subdomain):
    return validate_object_meta(obj, namespaced, name_fn)


# ---------------------------------------------------------------------------------------------
# core group
def validate_replication_controller(rc):
    errs = _meta(rc)
    spec = rc.get("spec") or {}
    _replicas(spec, "spec", errs)
    sel = spec.get("selector") or {}
    if not sel:
        errs.append(required("spec.selector"))
    tpl = spec.get("template")
    if tpl is None:
        errs.append(required("spec.template"))
    else:
        labels = (tpl.get("metadata") or {}).get("labels") or {}
        if sel and any(labels.get(k) != v for k, v in sel.items()):
            errs.append(invalid("spec.template.metadata.labels", f"{labels}: `selector` does not match template `labels`"))
        errs += validate_pod_template_spec(tpl, "spec.template", ("Always",))
    return errs


def validate_pod_template(pt):
    return _meta(pt) + validate_pod_template_spec(pt.get("template"), "template")


def _config_map_key(k):
    return bool(k) and len(k) <= 253 and k not in (".", "..") and not k.startswith("..") and bool(CONFIG_MAP_KEY.match(k))


def validate_config_map(cm):
    errs = _meta(cm)
    size = 0
    data, binary = cm.get("data") or {}, cm.get("binaryData") or {}
    for field, d in (("data", data), ("binaryData", binary)):
        if not isinstance(d, dict):
            errs.append(invalid(field, "must be a map"))
            continue
        for k, v in d.items():
            if not _config_map_key(k):
                errs.append(invalid(f"{field}[{k}]", f"{k!r}: a valid config key must consist of alphanumeric characters, '-', '_' or '.'"))
            if not isinstance(v, str):
                errs.append(invalid(f"{field}[{k}]", "must be a string"))
            else:
                size += len(v)
    for k in set(data) & set(binary):
        errs.append(duplicate(f"binaryData[{k}]", "key is also present in data"))
    if size > MAX_SECRET_SIZE:
        errs.append(FieldError("Too long", "data", f"must have at most {MAX_SECRET_SIZE} bytes"))
    return errs


_SECRET_REQUIRED = {"kubernetes.io/dockercfg": (".dockercfg",), "kubernetes.io/dockerconfigjson": (".dockerconfigjson",),
                    "kubernetes.io/ssh-auth": ("ssh-privatekey",), "kubernetes.io/tls": ("tls.crt", "tls.key")}


def validate_secret(sec):
    errs = _meta(sec)
    size = 0
    data = sec.get("data") or {}
    for field, d in (("data", data), ("stringData", sec.get("stringData") or {})):
        for k, v in d.items():
            if not _config_map_key(k):
                errs.append(invalid(f"{field}[{k}]", f"{k!r}: a valid config key must consist of alphanumeric characters, '-', '_' or '.'"))
            size += len(v or "")
    if size > MAX_SECRET_SIZE:
        errs.append(FieldError("Too long", "data", f"must have at most {MAX_SECRET_SIZE} bytes"))
    t = sec.get("type") or "Opaque"
    keys = set(data) | set(sec.get("stringData") or {})
    for k in _SECRET_REQUIRED.get(t, ()):
        if k not in keys:
            errs.append(required(f"data[{k}]"))
    if t == "kubernetes.io/service-account-token":
        if not (sec.get("metadata") or {}).get("annotations", {}).get("kubernetes.io/service-account.name"):
            errs.append(required("metadata.annotations[kubernetes.io/service-account.name]"))
    if t == "kubernetes.io/basic-auth" and not ({"username", "password"} & keys):
        errs.append(required("data[username]", "must have at least one of username or password"))
    return errs


def validate_secret_update(new, old):
    errs = []
    if (new.get("type") or "Opaque") != (old.get("type") or "Opaque"):
        errs.append(invalid("type", "field is immutable"))
    return errs


def _ip(v):
    try:
        ipaddress.ip_address(v)
        return True
    except (ValueError, TypeError):
        return False


def _cidr(v):
    try:
        ipaddress.ip_network(v, strict=False)
        return "/" in v
    except (ValueError, TypeError):
        return False


def validate_endpoints(ep):
    errs = _meta(ep)
    for i, ss in enumerate(ep.get("subsets") or ()):
        p = f"subsets[{i}]"
        if not ss.get("addresses") and not ss.get("notReadyAddresses"):
            errs.append(required(p, "must specify `addresses` or `notReadyAddresses`"))
        for key in ("addresses", "notReadyAddresses"):
            for j, a in enumerate(ss.get(key) or ()):
                if not _ip(a.get("ip")):
                    errs.append(invalid(f"{p}.{key}[{j}].ip", a.get("ip")))
                if a.get("hostname") and not is_dns1123_label(a["hostname"]):
                    errs.append(invalid(f"{p}.{key}[{j}].hostname", a["hostname"]))
        if not ss.get("ports"):
            errs.append(required(f"{p}.ports"))
        for j, port in enumerate(ss.get("ports") or ()):
            pn = port.get("port")
            if not _is_int(pn) or not 0 < pn < 65536:
                errs.append(invalid(f"{p}.ports[{j}].port", pn))
            if port.get("protocol") and port["protocol"] not in ("TCP", "UDP"):
                errs.append(not_supported(f"{p}.ports[{j}].protocol", port["protocol"]))
            if len(ss.get("ports") or ()) > 1 and not port.get("name"):
                errs.append(required(f"{p}.ports[{j}].name"))
    return errs


def validate_limit_range(lr):
    errs = _meta(lr)
    seen = set()
    for i, item in enumerate((lr.get("spec") or {}).get("limits") or ()):
        p = f"spec.limits[{i}]"
        t = item.get("type")
        if t not in ("Pod", "Container", "PersistentVolumeClaim"):
            errs.append(not_supported(f"{p}.type", t))
        if t in seen:
            errs.append(duplicate(f"{p}.type", t))
        seen.add(t)
        q = {}
        for k in ("max", "min", "default", "defaultRequest", "maxLimitRequestRatio"):
            errs += _validate_resource_list(item.get(k) or {}, f"{p}.{k}")
            try:
                q[k] = {r: parse_quantity(str(v)) for r, v in (item.get(k) or {}).items()}
            except QuantityError:
                q[k] = {}
        if t == "Pod" and (item.get("default") or item.get("defaultRequest")):
            errs.append(forbidden(f"{p}.default", "may not be specified when `type` is 'Pod'"))
        for r, mn in q["min"].items():
            if r in q["max"] and mn > q["max"][r]:
                errs.append(invalid(f"{p}.min[{r}]", f"min value {mn} is greater than max value {q['max'][r]}"))
            for k in ("default", "defaultRequest"):
                if r in q[k] and q[k][r] < mn:
                    errs.append(invalid(f"{p}.{k}[{r}]", f"min value {mn} is greater than {k} value {q[k][r]}"))
        for r, mx in q["max"].items():
            for k in ("default", "defaultRequest"):
                if r in q[k] and q[k][r] > mx:
                    errs.append(invalid(f"{p}.{k}[{r}]", f"{k} value {q[k][r]} is greater than max value {mx}"))
        for r, dr in q["defaultRequest"].items():
            if r in q["default"] and dr > q["default"][r]:
                errs.append(invalid(f"{p}.defaultRequest[{r}]", f"default request value {dr} is greater than default limit value {q['default'][r]}"))
        for r, ratio in q["maxLimitRequestRatio"].items():
            if ratio < 1:
                errs.append(invalid(f"{p}.maxLimitRequestRatio[{r}]", "ratio must be greater than or equal to 1"))
    return errs


_QUOTA_SCOPES = ("Terminating", "NotTerminating", "BestEffort", "NotBestEffort")


_STANDARD_QUOTA_RESOURCES = frozenset((
    "cpu", "memory", "ephemeral-storage", "requests.cpu", "requests.memory", "requests.storage",
    "requests.ephemeral-storage", "limits.cpu", "limits.memory", "limits.ephemeral-storage", "pods", "resourcequotas",
    "services", "replicationcontrollers", "secrets", "persistentvolumeclaims", "configmaps", "services.nodeports",
    "services.loadbalancers"))
_POD_COMPUTE_QUOTA = frozenset(("cpu", "memory", "limits.cpu", "limits.memory", "requests.cpu", "requests.memory"))


def _quota_scope_valid_for(scope, resource):
    """`helper.IsResourceQuotaScopeValidForResource` (the fork's pod extended resources are
    pod-tracked too, so the compute scopes accept them)."""
    if scope == "BestEffort":
        return resource == "pods"
    if scope in ("Terminating", "NotTerminating", "NotBestEffort"):
        return resource == "pods" or resource in _POD_COMPUTE_QUOTA or (
            "/" in resource and not resource.startswith("count/") and ".storageclass.storage.k8s.io/" not in resource)
    return True


def validate_resource_quota(rq):
    """`ValidateResourceQuota`: hard names are standard quota resources, hugepages or fully
    qualified (`count/<resource>[.<group>]`, `<class>.storageclass.storage.k8s.io/...`, extended
    resources); quantities are non-negative; scopes are standard, not contradictory, and every
    hard name is one the scopes can track."""
    errs = _meta(rq)
    spec = rq.get("spec") or {}
    hard = spec.get("hard") or {}
    for k, v in hard.items():
        if "/" not in k:
            if not (k in _STANDARD_QUOTA_RESOURCES or k.startswith(("hugepages-", "requests.hugepages-"))):
                errs.append(invalid(f"spec.hard[{k}]", "must be a standard resource for quota"))
        elif not is_qualified_name(k):
            errs.append(invalid(f"spec.hard[{k}]", "must be a standard resource for quota"))
        try:
            if parse_quantity(str(v)).value < 0:
                errs.append(invalid(f"spec.hard[{k}]", "must be greater than or equal to 0"))
        except QuantityError:
            errs.append(invalid(f"spec.hard[{k}]", v))
    scopes = spec.get("scopes") or ()
    for i, sc in enumerate(scopes):
        if sc not in _QUOTA_SCOPES:
            errs.append(not_supported(f"spec.scopes[{i}]", sc))
            continue
        for k in hard:
            if not _quota_scope_valid_for(sc, k):
                errs.append(invalid("spec.scopes", f"unsupported scope applied to resource {k}"))
    for a, b in (("Terminating", "NotTerminating"), ("BestEffort", "NotBestEffort")):
        if a in scopes and b in scopes:
            errs.append(invalid("spec.scopes", f"conflicting scopes {a} and {b}"))
    return errs


def validate_resource_quota_update(new, old):
    """`ValidateResourceQuotaUpdate`: scopes are immutable."""
    if sorted((new.get("spec") or {}).get("scopes") or ()) != sorted((old.get("spec") or {}).get("scopes") or ()):
        return [invalid("spec.scopes", "field is immutable")]
    return []


def validate_service_account(sa):
    errs = _meta(sa)
    for i, s in enumerate(sa.get("secrets") or ()):
        if s.get("name") and not is_dns1123_subdomain(s["name"]):
            errs.append(invalid(f"secrets[{i}].name", s["name"]))
    return errs


_ACCESS_MODES = ("ReadWriteOnce", "ReadOnlyMany", "ReadWriteMany")
_PV_SOURCES = ("gcePersistentDisk", "awsElasticBlockStore", "hostPath", "glusterfs", "nfs", "rbd", "iscsi", "cinder",
               "cephfs", "fc", "flocker", "flexVolume", "azureFile", "vsphereVolume", "quobyte", "azureDisk",
               "photonPersistentDisk", "portworxVolume", "scaleIO", "local", "storageos", "csi")


def validate_persistent_volume(pv):
    errs = _meta(pv, namespaced=False)
    spec = pv.get("spec") or {}
    modes = spec.get("accessModes") or ()
    if not modes:
        errs.append(required("spec.accessModes"))
    for m in modes:
        if m not in _ACCESS_MODES:
            errs.append(not_supported("spec.accessModes", m))
    cap = spec.get("capacity") or {}
    if "storage" not in cap or len(cap) != 1:
        errs.append(required("spec.capacity", "must specify exactly one resource: storage"))
    errs += _validate_resource_list(cap, "spec.capacity")
    srcs = [k for k in _PV_SOURCES if spec.get(k) is not None]
    if not srcs:
        errs.append(required("spec", "must specify a volume type"))
    elif len(srcs) > 1:
        errs.append(forbidden(f"spec.{srcs[1]}", "may not specify more than 1 volume type"))
    rp = spec.get("persistentVolumeReclaimPolicy")
    if rp and rp not in ("Retain", "Recycle", "Delete"):
        errs.append(not_supported("spec.persistentVolumeReclaimPolicy", rp))
    if spec.get("storageClassName") and not is_dns1123_subdomain(spec["storageClassName"]):
        errs.append(invalid("spec.storageClassName", spec["storageClassName"]))
    return errs


def validate_persistent_volume_claim(pvc):
    errs = _meta(pvc)
    spec = pvc.get("spec") or {}
    modes = spec.get("accessModes") or ()
    if not modes:
        errs.append(required("spec.accessModes", "at least 1 access mode is required"))
    for m in modes:
        if m not in _ACCESS_MODES:
            errs.append(not_supported("spec.accessModes", m))
    req = ((spec.get("resources") or {}).get("requests") or {})
    if "storage" not in req:
        errs.append(required("spec.resources[storage]"))
    else:
        try:
            if parse_quantity(str(req["storage"])).value <= 0:
                errs.append(invalid("spec.resources[storage]", "must be greater than zero"))
        except QuantityError:
            errs.append(invalid("spec.resources[storage]", req["storage"]))
    errs += validate_label_selector(spec.get("selector"), "spec.selector")
    return errs


def validate_persistent_volume_claim_update(new, old):
    """Bound claims: only the storage request may change (grow: ExpandPersistentVolumes)."""
    errs = []
    ns, os_ = dict(new.get("spec") or {}), dict(old.get("spec") or {})
    if os_.get("volumeName"):
        nr = ((ns.pop("resources", None) or {}).get("requests") or {}).get("storage")
        orr = ((os_.pop("resources", None) or {}).get("requests") or {}).get("storage")
        if ns != os_:
            errs.append(forbidden("spec", "is immutable after creation except resources.requests for bound claims"))
        try:
            if nr is not None and orr is not None and parse_quantity(str(nr)) < parse_quantity(str(orr)):
                errs.append(forbidden("spec.resources.requests.storage", "field can not be less than previous value"))
        except QuantityError:
            pass
    return errs


def validate_event(ev):
    errs = _meta(ev)
    io = ev.get("involvedObject") or {}
    ns = (ev.get("metadata") or {}).get("namespace")
    if io.get("namespace") and ns and io["namespace"] != ns:
        errs.append(invalid("involvedObject.namespace", "does not match event.namespace"))
    for k in ("type",):
        if ev.get(k) and ev[k] not in ("Normal", "Warning"):
            errs.append(not_supported(k, ev[k]))
    return errs


# ---------------------------------------------------------------------------------------------
# apps / extensions
def _rolling(ru, path, errs, surge=True):
    mu = _int_or_percent((ru or {}).get("maxUnavailable"), f"{path}.maxUnavailable", errs)
    if surge:
        ms = _int_or_percent((ru or {}).get("maxSurge"), f"{path}.maxSurge", errs)
        if mu == 0 and ms == 0:
            errs.append(invalid(f"{path}.maxUnavailable", "may not be 0 when `maxSurge` is 0"))


def validate_deployment(d):
    errs = _meta(d)
    spec = d.get("spec") or {}
    _replicas(spec, "spec", errs)
    errs += _selector_matches_template(spec.get("selector"), spec.get("template"), "spec")
    errs += validate_pod_template_spec(spec.get("template"), "spec.template", ("Always",))
    st = spec.get("strategy") or {}
    t = st.get("type") or "RollingUpdate"
    if t not in ("Recreate", "RollingUpdate"):
        errs.append(not_supported("spec.strategy.type", t))
    if t == "Recreate" and st.get("rollingUpdate") is not None:
        errs.append(forbidden("spec.strategy.rollingUpdate", "may not be specified when strategy `type` is 'Recreate'"))
    if t == "RollingUpdate":
        _rolling(st.get("rollingUpdate"), "spec.strategy.rollingUpdate", errs)
    _non_negative(spec.get("revisionHistoryLimit"), "spec.revisionHistoryLimit", errs)
    pds = spec.get("progressDeadlineSeconds")
    if pds is not None:
        _non_negative(pds, "spec.progressDeadlineSeconds", errs)
        if _is_int(pds) and pds <= (spec.get("minReadySeconds") or 0):
            errs.append(invalid("spec.progressDeadlineSeconds", "must be greater than minReadySeconds"))
    rb = spec.get("rollbackTo")
    if rb is not None:
        _non_negative(rb.get("revision"), "spec.rollbackTo.revision", errs)
    return errs


def _selector_immutable(new, old, path="spec.selector"):
    if (new.get("spec") or {}).get("selector") != (old.get("spec") or {}).get("selector"):
        return [invalid(path, "field is immutable")]
    return []


def validate_replica_set(rs):
    errs = _meta(rs)
    spec = rs.get("spec") or {}
    _replicas(spec, "spec", errs)
    errs += _selector_matches_template(spec.get("selector"), spec.get("template"), "spec")
    errs += validate_pod_template_spec(spec.get("template"), "spec.template", ("Always",))
    return errs


def validate_daemon_set(ds):
    errs = _meta(ds)
    spec = ds.get("spec") or {}
    _non_negative(spec.get("minReadySeconds"), "spec.minReadySeconds", errs)
    errs += _selector_matches_template(spec.get("selector"), spec.get("template"), "spec")
    errs += validate_pod_template_spec(spec.get("template"), "spec.template", ("Always",))
    us = spec.get("updateStrategy") or {}
    t = us.get("type") or "RollingUpdate"
    if t not in ("OnDelete", "RollingUpdate"):
        errs.append(not_supported("spec.updateStrategy.type", t))
    if t == "RollingUpdate":
        mu = _int_or_percent((us.get("rollingUpdate") or {}).get("maxUnavailable", 1),
                             "spec.updateStrategy.rollingUpdate.maxUnavailable", errs)
        if mu == 0:
            errs.append(invalid("spec.updateStrategy.rollingUpdate.maxUnavailable", "cannot be 0"))
    _non_negative(spec.get("revisionHistoryLimit"), "spec.revisionHistoryLimit", errs)
    return errs


def validate_stateful_set(ss):
    errs = _meta(ss, name_fn=is_dns1123_label)
    spec = ss.get("spec") or {}
    _non_negative(spec.get("replicas"), "spec.replicas", errs)
    pmp = spec.get("podManagementPolicy") or "OrderedReady"
    if pmp not in ("OrderedReady", "Parallel"):
        errs.append(not_supported("spec.podManagementPolicy", pmp))
    us = spec.get("updateStrategy") or {}
    t = us.get("type") or "RollingUpdate"
    if t not in ("OnDelete", "RollingUpdate"):
        errs.append(not_supported("spec.updateStrategy.type", t))
    if t == "OnDelete" and us.get("rollingUpdate") is not None:
        errs.append(invalid("spec.updateStrategy.rollingUpdate", "only allowed for updateStrategy 'RollingUpdate'"))
    if t == "RollingUpdate":
        _non_negative((us.get("rollingUpdate") or {}).get("partition"), "spec.updateStrategy.rollingUpdate.partition", errs)
    errs += _selector_matches_template(spec.get("selector"), spec.get("template"), "spec")
    # the pod spec is checked as the controller will create it: with one persistentVolumeClaim
    # volume per claim template (`updateStorage`), so mounts of claim templates resolve. The
    # reference skips pod-spec validation here for exactly that reason (apps/validation.go:55-58,
    # whose TODO asks for this union check instead)
    errs += validate_pod_template_spec(_with_claim_volumes(spec), "spec.template", ("Always",))
    if ((spec.get("template") or {}).get("spec") or {}).get("activeDeadlineSeconds") is not None:
        errs.append(forbidden("spec.template.spec.activeDeadlineSeconds", "activeDeadlineSeconds in StatefulSet is not Supported"))
    _non_negative(spec.get("revisionHistoryLimit"), "spec.revisionHistoryLimit", errs)
    for i, vct in enumerate(spec.get("volumeClaimTemplates") or ()):
        p = f"spec.volumeClaimTemplates[{i}]"
        md = vct.get("metadata") or {}
        if not is_dns1123_label(md.get("name", "")):
            errs.append(invalid(f"{p}.metadata.name", md.get("name")))
    return errs


def _with_claim_volumes(spec):
    tmpl = spec.get("template")
    claims = [(c.get("metadata") or {}).get("name") for c in spec.get("volumeClaimTemplates") or ()
              if isinstance(c, dict)]
    if not isinstance(tmpl, dict) or not claims:
        return tmpl
    pspec = dict(tmpl.get("spec") or {})
    vols = [{"name": n, "persistentVolumeClaim": {"claimName": f"{n}-validation-0"}} for n in claims if n]
    pspec["volumes"] = vols + [v for v in pspec.get("volumes") or () if v.get("name") not in claims]
    return dict(tmpl, spec=pspec)


def validate_stateful_set_update(new, old):
    """Only replicas, template and updateStrategy may change (apps/validation.go ValidateStatefulSetUpdate)."""
    ns, os_ = dict(new.get("spec") or {}), dict(old.get("spec") or {})
    for k in ("replicas", "template", "updateStrategy"):
        ns.pop(k, None)
        os_.pop(k, None)
    if ns != os_:
        return [forbidden("spec", "updates to statefulset spec for fields other than 'replicas', 'template', and "
                                  "'updateStrategy' are forbidden")]
    return []


def validate_controller_revision(cr):
    errs = _meta(cr)
    if cr.get("data") is None:
        errs.append(required("data"))
    _non_negative(cr.get("revision"), "revision", errs)
    return errs


def validate_controller_revision_update(new, old):
    if new.get("data") != old.get("data"):
        return [invalid("data", "field is immutable")]
    return []


def validate_ingress(ing):
    errs = _meta(ing)
    spec = ing.get("spec") or {}

    def backend(b, path):
        out = []
        if not b:
            return out
        if not is_dns1123_label(b.get("serviceName", "")):
            out.append(invalid(f"{path}.serviceName", b.get("serviceName")))
        sp = b.get("servicePort")
        if sp is None:
            out.append(required(f"{path}.servicePort"))
        elif _is_int(sp):
            if not 0 < sp < 65536:
                out.append(invalid(f"{path}.servicePort", sp))
        elif not (isinstance(sp, str) and is_dns1123_label(sp)):
            out.append(invalid(f"{path}.servicePort", sp))
        return out
    errs += backend(spec.get("backend"), "spec.backend")
    if not spec.get("backend") and not spec.get("rules"):
        errs.append(invalid("spec", "either `backend` or `rules` must be specified"))
    for i, r in enumerate(spec.get("rules") or ()):
        host = r.get("host")
        if host:
            if _ip(host):
                errs.append(invalid(f"spec.rules[{i}].host", "must be a DNS name, not an IP address"))
            elif not is_dns1123_subdomain(host.replace("*.", "", 1)):
                errs.append(invalid(f"spec.rules[{i}].host", host))
        http = r.get("http")
        if http is not None:
            if not http.get("paths"):
                errs.append(required(f"spec.rules[{i}].http.paths"))
            for j, pth in enumerate(http.get("paths") or ()):
                if pth.get("path") and not pth["path"].startswith("/"):
                    errs.append(invalid(f"spec.rules[{i}].http.paths[{j}].path", "must be an absolute path"))
                errs += backend(pth.get("backend"), f"spec.rules[{i}].http.paths[{j}].backend")
    for i, t in enumerate(spec.get("tls") or ()):
        for j, h in enumerate(t.get("hosts") or ()):
            if not is_dns1123_subdomain(h.replace("*.", "", 1)):
                errs.append(invalid(f"spec.tls[{i}].hosts[{j}]", h))
    return errs


# ---------------------------------------------------------------------------------------------
# batch
def _validate_job_spec(spec, path, generated_selector=True):
    errs = []
    for k in ("parallelism", "completions", "backoffLimit"):
        _non_negative(spec.get(k), f"{path}.{k}", errs)
    _non_negative(spec.get("activeDeadlineSeconds"), f"{path}.activeDeadlineSeconds", errs, positive=True)
    tpl = spec.get("template")
    if spec.get("selector") is not None:
        errs += _selector_matches_template(spec.get("selector"), tpl, path)
    errs += validate_pod_template_spec(tpl, f"{path}.template", ("OnFailure", "Never"))
    return errs


def validate_job(job):
    return _meta(job) + _validate_job_spec(job.get("spec") or {}, "spec")


def validate_job_update(new, old):
    errs = []
    ns, os_ = new.get("spec") or {}, old.get("spec") or {}
    for k in ("completions", "selector", "template"):
        if ns.get(k) != os_.get(k):
            errs.append(invalid(f"spec.{k}", "field is immutable"))
    return errs


_CRON_FIELD = re.compile(r"^(\*|\?|[0-9A-Za-z]+(-[0-9A-Za-z]+)?)(/[0-9]+)?$")
_CRON_RANGES = ((0, 59), (0, 23), (1, 31), (1, 12), (0, 7))
_MONTHS = {m: i + 1 for i, m in enumerate("jan feb mar apr may jun jul aug sep oct nov dec".split())}
_DAYS = {d: i for i, d in enumerate("sun mon tue wed thu fri sat".split())}


def valid_cron(expr):
    """Standard 5-field cron (robfig/cron ParseStandard, as `ValidateCronJob` uses) or @every/@hourly..."""
    if not isinstance(expr, str) or not expr.strip():
        return False
    e = expr.strip()
    if e.startswith("@"):
        return e in ("@yearly", "@annually", "@monthly", "@weekly", "@daily", "@midnight", "@hourly") or \
            bool(re.fullmatch(r"@every (\d+(\.\d+)?(ns|us|ms|s|m|h))+", e))
    fields = e.split()
    if len(fields) != 5:
        return False
    for f, (lo, hi), names in zip(fields, _CRON_RANGES, (None, None, None, _MONTHS, _DAYS)):
        for part in f.split(","):
            if not _CRON_FIELD.match(part):
                return False
            rng = part.split("/")[0]
            if rng in ("*", "?"):
                continue
            for x in rng.split("-"):
                v = names.get(x.lower()) if names and not x.isdigit() else (int(x) if x.isdigit() else None)
                if v is None or not lo <= v <= hi:
                    return False
    return True


def validate_cron_job(cj):
    errs = _meta(cj)
    name = (cj.get("metadata") or {}).get("name") or ""
    if len(name) > 52:
        errs.append(invalid("metadata.name", "must be no more than 52 characters"))
    spec = cj.get("spec") or {}
    if not spec.get("schedule"):
        errs.append(required("spec.schedule"))
    elif not valid_cron(spec["schedule"]):
        errs.append(invalid("spec.schedule", f"{spec['schedule']!r}: not a valid cron schedule"))
    cp = spec.get("concurrencyPolicy") or "Allow"
    if cp not in ("Allow", "Forbid", "Replace"):
        errs.append(not_supported("spec.concurrencyPolicy", cp))
    for k in ("startingDeadlineSeconds", "successfulJobsHistoryLimit", "failedJobsHistoryLimit"):
        _non_negative(spec.get(k), f"spec.{k}", errs)
    jt = spec.get("jobTemplate")
    if jt is None:
        errs.append(required("spec.jobTemplate"))
    else:
        errs += _validate_job_spec(jt.get("spec") or {}, "spec.jobTemplate.spec")
    return errs


# ---------------------------------------------------------------------------------------------
# autoscaling
def validate_hpa(hpa):
    errs = _meta(hpa)
    spec = hpa.get("spec") or {}
    ref = spec.get("scaleTargetRef") or {}
    if not ref.get("kind"):
        errs.append(required("spec.scaleTargetRef.kind"))
    if not ref.get("name"):
        errs.append(required("spec.scaleTargetRef.name"))
    mn, mx = spec.get("minReplicas"), spec.get("maxReplicas")
    if mn is not None and (not _is_int(mn) or mn < 1):
        errs.append(invalid("spec.minReplicas", f"{mn!r}: must be greater than 0"))
    if not _is_int(mx) or mx < 1:
        errs.append(invalid("spec.maxReplicas", f"{mx!r}: must be greater than 0"))
    elif _is_int(mn) and mx < mn:
        errs.append(invalid("spec.maxReplicas", "must be greater than or equal to `minReplicas`"))
    t = spec.get("targetCPUUtilizationPercentage")
    if t is not None and (not _is_int(t) or t < 1):
        errs.append(invalid("spec.targetCPUUtilizationPercentage", f"{t!r}: must be greater than 0"))
    for i, m in enumerate(spec.get("metrics") or ()):
        mt = m.get("type")
        if mt not in ("Object", "Pods", "Resource", "External"):
            errs.append(not_supported(f"spec.metrics[{i}].type", mt))
    return errs


# ---------------------------------------------------------------------------------------------
# policy
def validate_pdb(pdb):
    errs = _meta(pdb)
    spec = pdb.get("spec") or {}
    if spec.get("minAvailable") is not None and spec.get("maxUnavailable") is not None:
        errs.append(invalid("spec", "minAvailable and maxUnavailable cannot be both set"))
    for k in ("minAvailable", "maxUnavailable"):
        if spec.get(k) is not None:
            _int_or_percent(spec[k], f"spec.{k}", errs)
    errs += validate_label_selector(spec.get("selector"), "spec.selector")
    return errs


def validate_pdb_update(new, old):
    if (new.get("spec") or {}) != (old.get("spec") or {}):
        return [forbidden("spec", "updates to poddisruptionbudget spec are forbidden.")]
    return []


_PSP_VOLUMES = {"*", "azureFile", "azureDisk", "flexVolume", "flocker", "hostPath", "emptyDir", "gcePersistentDisk",
                "awsElasticBlockStore", "gitRepo", "secret", "nfs", "iscsi", "glusterfs", "persistentVolumeClaim",
                "rbd", "cinder", "cephfs", "downwardAPI", "fc", "configMap", "vsphereVolume", "quobyte",
                "photonPersistentDisk", "projected", "portworxVolume", "scaleIO", "storageos", "csi", "none"}


def _id_ranges(rule, path, rules_ok, errs, need_ranges=("MustRunAs",)):
    r = (rule or {}).get("rule")
    if r not in rules_ok:
        errs.append(not_supported(f"{path}.rule", r))
    if r in need_ranges and not (rule or {}).get("ranges"):
        errs.append(invalid(f"{path}.ranges", "must provide at least one range"))
    for i, rg in enumerate((rule or {}).get("ranges") or ()):
        mn, mx = rg.get("min"), rg.get("max")
        if not _is_int(mn) or not _is_int(mx) or mn < 0 or mx < mn:
            errs.append(invalid(f"{path}.ranges[{i}]", "min must be >= 0 and <= max"))


def validate_psp(psp):
    errs = _meta(psp, namespaced=False)
    spec = psp.get("spec") or {}
    _id_ranges(spec.get("runAsUser"), "spec.runAsUser", ("MustRunAs", "MustRunAsNonRoot", "RunAsAny"), errs)
    _id_ranges(spec.get("supplementalGroups"), "spec.supplementalGroups", ("MustRunAs", "RunAsAny"), errs)
    _id_ranges(spec.get("fsGroup"), "spec.fsGroup", ("MustRunAs", "RunAsAny"), errs)
    se = (spec.get("seLinux") or {}).get("rule")
    if se not in ("MustRunAs", "RunAsAny"):
        errs.append(not_supported("spec.seLinux.rule", se))
    for i, v in enumerate(spec.get("volumes") or ()):
        if v not in _PSP_VOLUMES:
            errs.append(not_supported(f"spec.volumes[{i}]", v))
    add = set(spec.get("defaultAddCapabilities") or ()) | set(spec.get("allowedCapabilities") or ())
    for c in set(spec.get("requiredDropCapabilities") or ()) & add:
        errs.append(invalid("spec.defaultAddCapabilities", f"capability {c!r} is also in requiredDropCapabilities"))
    for i, hp in enumerate(spec.get("hostPorts") or ()):
        mn, mx = hp.get("min"), hp.get("max")
        if not _is_int(mn) or not _is_int(mx) or not 0 <= mn <= mx <= 65535:
            errs.append(invalid(f"spec.hostPorts[{i}]", "min/max must be 0-65535 and min <= max"))
    return errs


# ---------------------------------------------------------------------------------------------
# rbac
RBAC_GROUP = "rbac.authorization.k8s.io"


def _policy_rules(rules, path, cluster):
    errs = []
    for i, r in enumerate(rules or ()):
        p = f"{path}[{i}]"
        if not r.get("verbs"):
            errs.append(required(f"{p}.verbs", "verbs must contain at least one value"))
        nru = r.get("nonResourceURLs") or ()
        if nru:
            if not cluster:
                errs.append(invalid(f"{p}.nonResourceURLs", "namespaced rules cannot apply to non-resource URLs"))
            if r.get("apiGroups") or r.get("resources"):
                errs.append(invalid(f"{p}.nonResourceURLs", "rules cannot apply to both regular resources and non-resource URLs"))
            continue
        if r.get("apiGroups") is None or not isinstance(r.get("apiGroups"), list) or len(r.get("apiGroups")) == 0:
            errs.append(required(f"{p}.apiGroups", "resource rules must supply at least one api group"))
        if not r.get("resources"):
            errs.append(required(f"{p}.resources", "resource rules must supply at least one resource"))
    return errs


def validate_role(role, cluster=False):
    errs = validate_object_meta(role, not cluster, is_path_segment_name)
    errs += _policy_rules(role.get("rules"), "rules", cluster)
    return errs


def _subjects(subs, path, cluster):
    errs = []
    for i, s in enumerate(subs or ()):
        p = f"{path}[{i}]"
        kind = s.get("kind")
        if not s.get("name"):
            errs.append(required(f"{p}.name"))
        if kind == "ServiceAccount":
            if s.get("apiGroup"):
                errs.append(not_supported(f"{p}.apiGroup", s["apiGroup"]))
            if cluster and not s.get("namespace"):
                errs.append(required(f"{p}.namespace"))
            if s.get("name") and not is_dns1123_subdomain(s["name"]):
                errs.append(invalid(f"{p}.name", s["name"]))
        elif kind in ("User", "Group"):
            if s.get("apiGroup", RBAC_GROUP) != RBAC_GROUP:
                errs.append(not_supported(f"{p}.apiGroup", s.get("apiGroup")))
        else:
            errs.append(not_supported(f"{p}.kind", kind))
    return errs


def validate_role_binding(rb, cluster=False):
    errs = validate_object_meta(rb, not cluster, is_path_segment_name)
    ref = rb.get("roleRef") or {}
    if ref.get("apiGroup") != RBAC_GROUP:
        errs.append(not_supported("roleRef.apiGroup", ref.get("apiGroup")))
    kinds = ("ClusterRole",) if cluster else ("Role", "ClusterRole")
    if ref.get("kind") not in kinds:
        errs.append(not_supported("roleRef.kind", ref.get("kind")))
    if not ref.get("name"):
        errs.append(required("roleRef.name"))
    elif not is_path_segment_name(ref["name"]):
        errs.append(invalid("roleRef.name", ref["name"]))
    errs += _subjects(rb.get("subjects"), "subjects", cluster)
    return errs


def validate_role_binding_update(new, old):
    if new.get("roleRef") != old.get("roleRef"):
        return [invalid("roleRef", "cannot change roleRef")]
    return []


# ---------------------------------------------------------------------------------------------
# storage / scheduling / settings / certificates / networking / admission / aggregation
def validate_storage_class(sc):
    errs = _meta(sc, namespaced=False)
    prov = sc.get("provisioner") or ""
    if not prov:
        errs.append(required("provisioner"))
    elif not is_qualified_name(prov.lower()) and not re.fullmatch(r"[a-z0-9]([-a-z0-9.]*[a-z0-9])?(/[-a-z0-9A-Z_.]+)?", prov):
        errs.append(invalid("provisioner", prov))
    params = sc.get("parameters") or {}
    if len(params) > 512:
        errs.append(FieldError("Too many", "parameters", "must have at most 512 parameters"))
    if sum(len(k) + len(str(v)) for k, v in params.items()) > 256 * 1024:
        errs.append(FieldError("Too long", "parameters", "must have at most 262144 bytes"))
    rp = sc.get("reclaimPolicy")
    if rp and rp not in ("Delete", "Retain"):
        errs.append(not_supported("reclaimPolicy", rp))
    vbm = sc.get("volumeBindingMode")
    if vbm and vbm not in ("Immediate", "WaitForFirstConsumer"):
        errs.append(not_supported("volumeBindingMode", vbm))
    return errs


def validate_storage_class_update(new, old):
    errs = []
    for k in ("provisioner", "parameters", "reclaimPolicy"):
        if new.get(k) != old.get(k):
            errs.append(forbidden(k, "updates to " + k + " are forbidden."))
    return errs


def validate_volume_attachment(va):
    errs = _meta(va, namespaced=False)
    spec = va.get("spec") or {}
    if not spec.get("attacher"):
        errs.append(required("spec.attacher"))
    if not spec.get("nodeName"):
        errs.append(required("spec.nodeName"))
    if not (spec.get("source") or {}).get("persistentVolumeName"):
        errs.append(required("spec.source.persistentVolumeName"))
    return errs


HIGHEST_USER_PRIORITY = 1_000_000_000


def validate_priority_class(pc):
    errs = _meta(pc, namespaced=False)
    name = (pc.get("metadata") or {}).get("name") or ""
    v = pc.get("value")
    if not _is_int(v):
        errs.append(required("value"))
    elif not name.startswith("system-") and v > HIGHEST_USER_PRIORITY:
        errs.append(forbidden("value", f"maximum allowed value of a user defined priority is {HIGHEST_USER_PRIORITY}"))
    return errs


def validate_priority_class_update(new, old):
    if new.get("value") != old.get("value"):
        return [forbidden("value", "may not be changed in an update.")]
    return []


def validate_pod_preset(pp):
    errs = _meta(pp)
    spec = pp.get("spec") or {}
    errs += validate_label_selector(spec.get("selector"), "spec.selector")
    if not (spec.get("env") or spec.get("envFrom") or spec.get("volumes") or spec.get("volumeMounts")):
        errs.append(required("spec", "must specify at least one of env, envFrom, volumes or volumeMounts"))
    return errs


def validate_csr(csr):
    errs = _meta(csr, namespaced=False)
    req = (csr.get("spec") or {}).get("request")
    if not req:
        errs.append(required("spec.request"))
    else:
        import base64
        try:
            pem = base64.b64decode(req, validate=True)
        except (ValueError, TypeError):
            pem = b""
        if b"BEGIN CERTIFICATE REQUEST" not in pem:
            errs.append(invalid("spec.request", "PEM block type must be CERTIFICATE REQUEST"))
    for i, u in enumerate((csr.get("spec") or {}).get("usages") or ()):
        if not isinstance(u, str) or not u:
            errs.append(invalid(f"spec.usages[{i}]", u))
    return errs


def _np_port(p, path, errs):
    proto = p.get("protocol")
    if proto and proto not in ("TCP", "UDP"):
        errs.append(not_supported(f"{path}.protocol", proto))
    port = p.get("port")
    if port is not None:
        if _is_int(port):
            if not 0 < port < 65536:
                errs.append(invalid(f"{path}.port", port))
        elif not (isinstance(port, str) and re.fullmatch(r"[a-z0-9]([a-z0-9-]*[a-z0-9])?", port) and len(port) <= 15):
            errs.append(invalid(f"{path}.port", port))


def _np_peer(peer, path, errs):
    kinds = [k for k in ("podSelector", "namespaceSelector", "ipBlock") if peer.get(k) is not None]
    if len(kinds) != 1:
        errs.append(forbidden(path, "must specify exactly one of podSelector, namespaceSelector or ipBlock"))
    for k in ("podSelector", "namespaceSelector"):
        if peer.get(k) is not None:
            errs.extend(validate_label_selector(peer[k], f"{path}.{k}"))
    ib = peer.get("ipBlock")
    if ib is not None:
        cidr = ib.get("cidr")
        if not _cidr(cidr or ""):
            errs.append(invalid(f"{path}.ipBlock.cidr", cidr))
        else:
            net = ipaddress.ip_network(cidr, strict=False)
            for j, ex in enumerate(ib.get("except") or ()):
                if not _cidr(ex or ""):
                    errs.append(invalid(f"{path}.ipBlock.except[{j}]", ex))
                elif not ipaddress.ip_network(ex, strict=False).subnet_of(net):
                    errs.append(invalid(f"{path}.ipBlock.except[{j}]", "must be a strict subset of `cidr`"))


def validate_network_policy(np_):
    errs = _meta(np_)
    spec = np_.get("spec") or {}
    if "podSelector" not in spec:
        errs.append(required("spec.podSelector"))
    errs += validate_label_selector(spec.get("podSelector"), "spec.podSelector")
    for key, peers in (("ingress", "from"), ("egress", "to")):
        for i, rule in enumerate(spec.get(key) or ()):
            for j, p in enumerate((rule or {}).get("ports") or ()):
                _np_port(p, f"spec.{key}[{i}].ports[{j}]", errs)
            for j, peer in enumerate((rule or {}).get(peers) or ()):
                _np_peer(peer, f"spec.{key}[{i}].{peers}[{j}]", errs)
    for i, t in enumerate(spec.get("policyTypes") or ()):
        if t not in ("Ingress", "Egress"):
            errs.append(not_supported(f"spec.policyTypes[{i}]", t))
    return errs


_OPS = ("*", "CREATE", "UPDATE", "DELETE", "CONNECT")


def _webhook_config(wc, mutating):
    errs = _meta(wc, namespaced=False)
    names = set()
    for i, w in enumerate(wc.get("webhooks") or ()):
        p = f"webhooks[{i}]"
        n = w.get("name", "")
        if len(n.split(".")) < 3 or not is_dns1123_subdomain(n):
            errs.append(invalid(f"{p}.name", f"{n!r}: should be a domain with at least three segments separated by dots"))
        if n in names:
            errs.append(duplicate(f"{p}.name", n))
        names.add(n)
        for j, r in enumerate(w.get("rules") or ()):
            for op in r.get("operations") or ():
                if op not in _OPS:
                    errs.append(not_supported(f"{p}.rules[{j}].operations", op))
            if not r.get("apiGroups") or not r.get("apiVersions") or not r.get("resources"):
                errs.append(required(f"{p}.rules[{j}]", "apiGroups, apiVersions and resources are required"))
        fp = w.get("failurePolicy")
        if fp and fp not in ("Ignore", "Fail"):
            errs.append(not_supported(f"{p}.failurePolicy", fp))
        cc = w.get("clientConfig") or {}
        if (cc.get("url") is None) == (cc.get("service") is None):
            errs.append(required(f"{p}.clientConfig", "exactly one of url or service is required"))
        url = cc.get("url")
        if url is not None and not str(url).startswith("https://") and not _loopback_http(str(url)):
            # deviation: plain http is accepted for a loopback webhook (in-process tests, node-local
            # sidecars); anything that leaves the host must be https as in the reference
            errs.append(invalid(f"{p}.clientConfig.url", "'https' is the only allowed URL scheme"))
        svc = cc.get("service")
        if svc is not None and (not svc.get("name") or not svc.get("namespace")):
            errs.append(required(f"{p}.clientConfig.service", "service name and namespace are required"))
    return errs


def _loopback_http(url):
    from urllib.parse import urlparse
    u = urlparse(url)
    return u.scheme == "http" and u.hostname in ("127.0.0.1", "localhost", "::1")


def validate_initializer_configuration(ic):
    errs = _meta(ic, namespaced=False)
    for i, it in enumerate(ic.get("initializers") or ()):
        n = it.get("name", "")
        if len(n.split(".")) < 3 or not is_dns1123_subdomain(n):
            errs.append(invalid(f"initializers[{i}].name", f"{n!r}: should be a domain with at least three segments separated by dots"))
        for j, r in enumerate(it.get("rules") or ()):
            if not r.get("apiGroups") or not r.get("apiVersions") or not r.get("resources"):
                errs.append(required(f"initializers[{i}].rules[{j}]", "apiGroups, apiVersions and resources are required"))
    return errs


def validate_apiservice(a):
    errs = validate_object_meta(a, False, lambda n: bool(n))
    spec = a.get("spec") or {}
    name = (a.get("metadata") or {}).get("name") or ""
    group, version = spec.get("group", ""), spec.get("version", "")
    if not version:
        errs.append(required("spec.version"))
    elif name != f"{version}.{group}".rstrip(".") and name != f"{version}.{group}":
        errs.append(invalid("metadata.name", f"must be spec.version+\".\"+spec.group: {version}.{group}"))
    gpm, vp = spec.get("groupPriorityMinimum"), spec.get("versionPriority")
    if not _is_int(gpm) or not 0 < gpm <= 20000:
        errs.append(invalid("spec.groupPriorityMinimum", f"{gpm!r}: must be positive and less than 20000"))
    if not _is_int(vp) or not 0 < vp <= 1000:
        errs.append(invalid("spec.versionPriority", f"{vp!r}: must be positive and less than 1000"))
    if spec.get("service") is not None:
        if spec.get("insecureSkipTLSVerify") and spec.get("caBundle"):
            errs.append(invalid("spec.insecureSkipTLSVerify", "may not be true if caBundle is present"))
    return errs


def validate_lease(lease):
    errs = _meta(lease)
    spec = lease.get("spec") or {}
    _non_negative(spec.get("leaseDurationSeconds"), "spec.leaseDurationSeconds", errs, positive=True)
    _non_negative(spec.get("leaseTransitions"), "spec.leaseTransitions", errs)
    return errs


VALIDATORS = {
    "ReplicationController": validate_replication_controller, "PodTemplate": validate_pod_template,
    "ConfigMap": validate_config_map, "Secret": validate_secret, "Endpoints": validate_endpoints,
    "LimitRange": validate_limit_range, "ResourceQuota": validate_resource_quota,
    "ServiceAccount": validate_service_account, "PersistentVolume": validate_persistent_volume,
    "PersistentVolumeClaim": validate_persistent_volume_claim, "Event": validate_event,
    "Deployment": validate_deployment, "ReplicaSet": validate_replica_set, "DaemonSet": validate_daemon_set,
    "StatefulSet": validate_stateful_set, "ControllerRevision": validate_controller_revision,
    "Ingress": validate_ingress, "Job": validate_job, "CronJob": validate_cron_job,
    "HorizontalPodAutoscaler": validate_hpa, "PodDisruptionBudget": validate_pdb, "PodSecurityPolicy": validate_psp,
    "Role": lambda o: validate_role(o, False), "ClusterRole": lambda o: validate_role(o, True),
    "RoleBinding": lambda o: validate_role_binding(o, False),
    "ClusterRoleBinding": lambda o: validate_role_binding(o, True),
    "StorageClass": validate_storage_class, "VolumeAttachment": validate_volume_attachment,
    "PriorityClass": validate_priority_class, "PodPreset": validate_pod_preset,
    "CertificateSigningRequest": validate_csr, "NetworkPolicy": validate_network_policy,
    "MutatingWebhookConfiguration": lambda o: _webhook_config(o, True),
    "ValidatingWebhookConfiguration": lambda o: _webhook_config(o, False),
    "InitializerConfiguration": validate_initializer_configuration, "APIService": validate_apiservice,
    "Lease": validate_lease,
}

def validate_node_update(new, old):
    """`ValidateNodeUpdate`: podCIDR and providerID may only go from "" to a value; status
    addresses are unique."""
    errs = []
    ns, os_ = new.get("spec") or {}, old.get("spec") or {}
    for k in ("podCIDR", "providerID"):
        if os_.get(k) and ns.get(k) != os_.get(k):
            errs.append(FieldError("Forbidden", f"spec.{k}", f"node updates may not change {k} except from \"\" to valid"))
    seen = set()
    for i, a in enumerate((new.get("status") or {}).get("addresses") or ()):
        key = (a.get("type"), a.get("address"))
        if key in seen:
            errs.append(duplicate(f"status.addresses[{i}]", a))
        seen.add(key)
    return errs


_PV_NOT_SOURCE = {"capacity", "accessModes", "claimRef", "persistentVolumeReclaimPolicy", "storageClassName",
                  "mountOptions", "volumeMode", "nodeAffinity"}


def validate_persistent_volume_update(new, old):
    """`ValidatePersistentVolumeUpdate`: the volume source (hostPath, nfs, csi, local, ...) is
    immutable after creation."""
    ns, os_ = new.get("spec") or {}, old.get("spec") or {}
    src = lambda sp: {k: v for k, v in sp.items() if k not in _PV_NOT_SOURCE}  # noqa: E731
    if src(ns) != src(os_):
        return [FieldError("Forbidden", "spec.persistentvolumesource", "is immutable after creation")]
    return []


UPDATE_VALIDATORS = {
    "Secret": validate_secret_update,
    "PersistentVolumeClaim": validate_persistent_volume_claim_update,
    "Deployment": _selector_immutable, "ReplicaSet": _selector_immutable, "DaemonSet": _selector_immutable,
    "StatefulSet": validate_stateful_set_update, "ControllerRevision": validate_controller_revision_update,
    "Job": validate_job_update, "PodDisruptionBudget": validate_pdb_update,
    "RoleBinding": validate_role_binding_update, "ClusterRoleBinding": validate_role_binding_update,
    "StorageClass": validate_storage_class_update, "PriorityClass": validate_priority_class_update,
    "ResourceQuota": validate_resource_quota_update,
    "Node": validate_node_update, "PersistentVolume": validate_persistent_volume_update,
}


def validate_update(kind, new, old):
    """Update-only rules: object meta identity + the kind's immutable fields."""
    fn = UPDATE_VALIDATORS.get(kind)
    return validate_object_meta_update(new, old) + (fn(new, old) if fn else [])


__all__ = ["VALIDATORS", "UPDATE_VALIDATORS", "validate_update", "valid_cron", "validate_label_selector", "core"]
