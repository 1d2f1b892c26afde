"""Resource quota: usage evaluators and resource-list arithmetic, shared by the ResourceQuota
admission plugin and the resource quota controller.

Parity:
  * `pkg/quota/resources.go` — Add / SubtractWithNonNegativeResult / Mask / LessThanOrEqual /
    IsZero / IsNegative / Equals / Max over resource lists (here: dicts name -> Quantity);
  * `pkg/quota/generic/evaluator.go` — `count/<resource>[.<group>]` object-count names,
    `Matches` (the quota names at least one matching resource AND every scope matches),
    `CalculateUsageStats` (zero-filled per tracked resource);
  * `pkg/quota/evaluator/core/{pods,services,persistent_volume_claims,registry}.go` — the pod
    evaluator (compute requests/limits, hugepages, QuotaPod terminal/grace rules, the
    Terminating / NotTerminating / BestEffort / NotBestEffort scopes, the "must specify"
    constraint when cpu/memory are quota'd), services (services, nodeports, loadbalancers),
    PVCs (claims, requests.storage, per-storage-class names) and the legacy object counts
    (configmaps, secrets, replicationcontrollers, resourcequotas).

Fork extension: the pod evaluator also charges extended resources — container requests for
`amd.com/gpu`-style names (as `requests.<name>` and `<name>`) and the pod-level
`spec.extendedResources` counts the fork's scheduler allocates — so a namespace can be held to a
GPU budget. The reference 1.9 pod evaluator ignores extended resources (`pods.go:43-63`).
"""
from __future__ import annotations

import time

from ..api import core
from ..api.meta import parse_rfc3339
from ..api.quantity import Quantity, parse_quantity

ZERO = Quantity(0)


# ---------------------------------------------------------------- resource list arithmetic
def qty(v) -> Quantity:
    return v if isinstance(v, Quantity) else parse_quantity(str(v))


def add(a: dict, b: dict) -> dict:
    out = {k: qty(v) for k, v in a.items()}
    for k, v in b.items():
        out[k] = out[k] + qty(v) if k in out else qty(v)
    return out


def subtract_non_negative(a: dict, b: dict) -> dict:
    """`SubtractWithNonNegativeResult`: a - b per name, floored at zero."""
    out = {}
    for k, v in a.items():
        d = qty(v) - b[k] if k in b else qty(v)
        out[k] = d if d > ZERO else Quantity(0)
    return out


def max_(a: dict, b: dict) -> dict:
    out = {k: qty(v) for k, v in a.items()}
    for k, v in b.items():
        v = qty(v)
        if k not in out or v > out[k]:
            out[k] = v
    return out


def mask(a: dict, names) -> dict:
    names = set(names)
    return {k: v for k, v in a.items() if k in names}


def less_than_or_equal(a: dict, b: dict):
    """(all of a <= b for names present in b, [names exceeding])."""
    exceeded = sorted(k for k, v in a.items() if k in b and qty(v) > qty(b[k]))
    return not exceeded, exceeded


def is_zero(a: dict) -> bool:
    return all(qty(v).is_zero() for v in a.values())


def is_negative(a: dict) -> list:
    return sorted(k for k, v in a.items() if qty(v) < ZERO)


def equals(a: dict, b: dict) -> bool:
    return set(a) == set(b) and all(qty(a[k]) == qty(b[k]) for k in a)


def to_strings(a: dict) -> dict:
    return {k: str(qty(v)) for k, v in a.items()}


def pretty(a: dict) -> str:
    return ",".join(f"{k}={qty(a[k])}" for k in sorted(a))


def object_count_name(resource: str, group: str = "") -> str:
    """`generic.ObjectCountQuotaResourceNameFor`."""
    return f"count/{resource}" if not group else f"count/{resource}.{group}"


# ---------------------------------------------------------------- evaluators
CREATE, UPDATE = "CREATE", "UPDATE"


class Evaluator:
    """`quota.Evaluator`: which quota resource names an object kind charges, and how much."""
    resource = ""
    group = ""
    operations = (CREATE,)

    def handles(self, operation: str) -> bool:
        return operation in self.operations

    def matching_resources(self, names) -> list:
        raise NotImplementedError

    def matches_scope(self, scope: str, obj) -> bool:
        return False          # generic.MatchesNoScopeFunc

    def matches(self, quota_obj, obj) -> bool:
        hard = (quota_obj.get("status") or {}).get("hard") or {}
        if not self.matching_resources(list(hard)):
            return False
        return all(self.matches_scope(s, obj) for s in (quota_obj.get("spec") or {}).get("scopes") or ())

    def constraints(self, required, obj):
        return None

    def usage(self, obj) -> dict:
        raise NotImplementedError

    def usage_stats(self, objs, resources, scopes) -> dict:
        """`generic.CalculateUsageStats`: every tracked resource zero-filled, then the usage of
        the objects matching all scopes summed (masked to the tracked set)."""
        used = {r: Quantity(0) for r in resources}
        for o in objs:
            if all(self.matches_scope(s, o) for s in scopes):
                used = add(used, mask(self.usage(o), resources))
        return used


class ObjectCountEvaluator(Evaluator):
    """`generic.NewObjectCountEvaluator`: one per object created; `alias` is the legacy name
    (`configmaps`, `secrets`, ...) the reference keeps alongside `count/<resource>`."""

    def __init__(self, resource, group="", alias=""):
        self.resource, self.group, self.alias = resource, group, alias
        self.names = [object_count_name(resource, group)] + ([alias] if alias else [])

    def matching_resources(self, names):
        return [n for n in names if n in self.names]

    def usage(self, obj):
        return {n: Quantity(1) for n in self.names}


POD_RESOURCES = ("count/pods", "cpu", "memory", "ephemeral-storage", "requests.cpu", "requests.memory",
                 "requests.ephemeral-storage", "limits.cpu", "limits.memory", "limits.ephemeral-storage", "pods")
POD_RESOURCE_PREFIXES = ("hugepages-", "requests.hugepages-")
VALIDATION_SET = frozenset(("cpu", "memory", "requests.cpu", "requests.memory", "limits.cpu", "limits.memory"))
SCOPES = ("Terminating", "NotTerminating", "BestEffort", "NotBestEffort")


def _is_extended(name: str) -> bool:
    """An extended-resource quota name (`amd.com/gpu`, `requests.amd.com/gpu`) — not an object
    count or a per-storage-class name, which also carry a '/'."""
    if name.startswith("count/") or ".storageclass.storage.k8s.io/" in name:
        return False
    return core.is_extended_resource_name(name[len("requests."):] if name.startswith("requests.") else name)


def compute_usage(requests: dict, limits: dict) -> dict:
    """`podComputeUsageHelper` (+ the fork's extended resources)."""
    out = {"pods": Quantity(1)}
    for base in ("cpu", "memory", "ephemeral-storage"):
        if base in requests:
            out[base] = out["requests." + base] = qty(requests[base])
        if base in limits:
            out["limits." + base] = qty(limits[base])
    for k, v in requests.items():
        if k.startswith("hugepages-") or core.is_extended_resource_name(k):
            out[k] = out["requests." + k] = qty(v)
    for k, v in limits.items():
        if k.startswith("hugepages-"):
            out["limits." + k] = qty(v)
    return out


def _container_resources(c):
    """(requests, limits) as stored: the API server's defaulter has already copied limits into
    absent requests (`SetDefaults_Pod`), so the evaluator reads both as they are."""
    res = c.get("resources") or {}
    return dict(res.get("requests") or {}), dict(res.get("limits") or {})


def quota_pod(pod, now=None) -> bool:
    """`QuotaPod`: terminal pods, and pods past their deletion grace, stop being charged."""
    if core.pod_is_terminal(pod):
        return False
    md = pod.get("metadata") or {}
    if md.get("deletionTimestamp") and md.get("deletionGracePeriodSeconds") is not None:
        t = parse_rfc3339(md["deletionTimestamp"])
        if t is not None and (now if now is not None else time.time()) > t + int(md["deletionGracePeriodSeconds"]):
            return False
    return True


def is_best_effort(pod) -> bool:
    """`qos.GetPodQOS(pod) == BestEffort`: no container asks for (or limits) cpu or memory."""
    spec = pod.get("spec") or {}
    for c in list(spec.get("containers") or ()) + list(spec.get("initContainers") or ()):
        req, lim = _container_resources(c)
        for k in ("cpu", "memory"):
            if (k in req and not qty(req[k]).is_zero()) or (k in lim and not qty(lim[k]).is_zero()):
                return False
    return True


def is_terminating(pod) -> bool:
    ads = (pod.get("spec") or {}).get("activeDeadlineSeconds")
    return ads is not None and int(ads) >= 0


class PodEvaluator(Evaluator):
    resource = "pods"

    def __init__(self, clock=time.time):
        self.clock = clock

    def handles(self, operation):
        return operation == CREATE

    def matching_resources(self, names):
        return [n for n in names if n in POD_RESOURCES or n.startswith(POD_RESOURCE_PREFIXES) or _is_extended(n)]

    def matches_scope(self, scope, pod):
        if scope == "Terminating":
            return is_terminating(pod)
        if scope == "NotTerminating":
            return not is_terminating(pod)
        if scope == "BestEffort":
            return is_best_effort(pod)
        if scope == "NotBestEffort":
            return not is_best_effort(pod)
        return False

    def constraints(self, required, pod):
        """BACKWARD COMPATIBILITY REQUIREMENT (pods.go): when cpu or memory is quota'd, every
        container must state it explicitly."""
        req_set = set(required) & VALIDATION_SET
        if not req_set:
            return None
        spec = pod.get("spec") or {}
        missing = set()
        for c in list(spec.get("containers") or ()) + list(spec.get("initContainers") or ()):
            res = c.get("resources") or {}
            have = set(compute_usage(res.get("requests") or {}, res.get("limits") or {}))
            missing |= req_set - have
        return f"must specify {','.join(sorted(missing))}" if missing else None

    def usage(self, pod):
        out = {"count/pods": Quantity(1)}
        if not quota_pod(pod, self.clock()):
            return out
        spec = pod.get("spec") or {}
        requests, limits = {}, {}
        for c in spec.get("containers") or ():
            r, lim = _container_resources(c)
            requests, limits = add(requests, r), add(limits, lim)
        for c in spec.get("initContainers") or ():
            r, lim = _container_resources(c)
            requests, limits = max_(requests, r), max_(limits, lim)
        out = add(out, compute_usage(requests, limits))
        for per in spec.get("extendedResources") or ():
            try:
                rn = core.pod_extended_resource_name(per)
                n = Quantity(core.pod_extended_resource_count(per))
            except (ValueError, KeyError):
                continue
            out = add(out, {"requests." + rn: n, rn: n})
        return out


class ServiceEvaluator(Evaluator):
    resource = "services"
    operations = (CREATE, UPDATE)
    NAMES = ("count/services", "services", "services.nodeports", "services.loadbalancers")

    def matching_resources(self, names):
        return [n for n in names if n in self.NAMES]

    def usage(self, svc):
        spec = svc.get("spec") or {}
        ports = len(spec.get("ports") or ())
        out = {"count/services": Quantity(1), "services": Quantity(1),
               "services.loadbalancers": Quantity(0), "services.nodeports": Quantity(0)}
        typ = spec.get("type")
        if typ == "NodePort":
            out["services.nodeports"] = Quantity(ports)
        elif typ == "LoadBalancer":
            out["services.nodeports"] = Quantity(ports)
            out["services.loadbalancers"] = Quantity(1)
        return out


STORAGE_CLASS_SUFFIX = ".storageclass.storage.k8s.io/"


def pvc_class(pvc) -> str:
    """`helper.GetPersistentVolumeClaimClass`: the beta annotation wins over spec."""
    ann = (pvc.get("metadata") or {}).get("annotations") or {}
    if "volume.beta.kubernetes.io/storage-class" in ann:
        return ann["volume.beta.kubernetes.io/storage-class"]
    return (pvc.get("spec") or {}).get("storageClassName") or ""


class PVCEvaluator(Evaluator):
    resource = "persistentvolumeclaims"
    NAMES = ("count/persistentvolumeclaims", "persistentvolumeclaims", "requests.storage")

    def matching_resources(self, names):
        return [n for n in names if n in self.NAMES or n.endswith(STORAGE_CLASS_SUFFIX + "persistentvolumeclaims")
                or n.endswith(STORAGE_CLASS_SUFFIX + "requests.storage")]

    def usage(self, pvc):
        out = {"persistentvolumeclaims": Quantity(1), "count/persistentvolumeclaims": Quantity(1)}
        cls = pvc_class(pvc)
        if cls:
            out[cls + STORAGE_CLASS_SUFFIX + "persistentvolumeclaims"] = Quantity(1)
        req = (((pvc.get("spec") or {}).get("resources") or {}).get("requests") or {}).get("storage")
        if req is not None:
            out["requests.storage"] = qty(req)
            if cls:
                out[cls + STORAGE_CLASS_SUFFIX + "requests.storage"] = qty(req)
        return out


LEGACY_COUNTS = {"configmaps": "configmaps", "resourcequotas": "resourcequotas",
                 "replicationcontrollers": "replicationcontrollers", "secrets": "secrets"}


class Registry:
    """`generic.Registry` + `core.NewEvaluators`: the static evaluators, and object-count
    evaluators created on demand for any other (group, resource)."""

    def __init__(self, clock=time.time):
        self.evaluators = {("", "pods"): PodEvaluator(clock), ("", "services"): ServiceEvaluator(),
                           ("", "persistentvolumeclaims"): PVCEvaluator()}
        for r, alias in LEGACY_COUNTS.items():
            self.evaluators[("", r)] = ObjectCountEvaluator(r, "", alias)

    def get(self, group: str, resource: str, create=True):
        ev = self.evaluators.get((group, resource))
        if ev is None and create:
            ev = self.evaluators[(group, resource)] = ObjectCountEvaluator(resource, group)
        return ev

    def for_name(self, name: str):
        """The evaluator that tracks a quota resource name (for the controller's recount):
        `count/<resource>[.<group>]` resolves to that resource's evaluator."""
        for ev in self.evaluators.values():
            if ev.matching_resources([name]):
                return ev
        if name.startswith("count/"):
            res, _, group = name[len("count/"):].partition(".")
            return self.get(group, res)
        return None


def calculate_usage(namespace_objects, scopes, hard: dict, registry: Registry) -> dict:
    """`quota.CalculateUsage`: for each evaluator covering some hard name, its usage stats over
    `namespace_objects(group, resource)`; the result covers exactly the names some evaluator
    tracks (the caller masks to hard)."""
    names = list(hard)
    used: dict = {}
    seen = set()
    for n in names:
        ev = registry.for_name(n)
        if ev is None or id(ev) in seen:
            continue
        seen.add(id(ev))
        tracked = ev.matching_resources(names)
        if not tracked:
            continue
        # a scoped quota only counts kinds that know the scope (pods)
        if scopes and not isinstance(ev, PodEvaluator):
            continue
        used.update(ev.usage_stats(namespace_objects(ev.group, ev.resource), tracked, scopes))
    return used
