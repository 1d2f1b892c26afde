"""Eviction manager: node pressure conditions, pressure-aware admission, node-level reclaim and
pod eviction.

Parity: `pkg/kubelet/eviction/eviction_manager.go` and `helpers.go`:

  * signals (`helpers.go:67-90`): memory.available and allocatableMemory.available (memory,
    MemoryPressure); nodefs.available, nodefs.inodesFree, imagefs.available,
    imagefs.inodesFree (the disk resources, DiskPressure);
  * `ParseThresholdConfig` (:101): hard (`--eviction-hard`) and soft (`--eviction-soft`, each
    needing a `--eviction-soft-grace-period`) statements `signal<quantity|percent` (positive
    values only), `--eviction-minimum-reclaim` per signal, and the allocatable threshold
    (allocatableMemory.available<0, min-reclaim 0) when `--enforce-node-allocatable` has `pods`;
  * `synchronize` (:213): thresholds met now, plus the ones met last pass that their minimum
    reclaim has not yet resolved; first-observed times; node conditions kept for
    `--eviction-pressure-transition-period` after the last observation; thresholds whose grace
    period has passed; only thresholds with fresh stats act. Then: an `EvictionThresholdMet`
    event, node-level reclaim first (terminated containers, then unused images, for the disk
    resources) — if that resolves every met threshold no pod is evicted; otherwise the active
    pods are ranked and ONE is evicted (critical static pods skipped): phase Failed, reason
    Evicted, message `The node was low on resource: <resource>.`, grace 0 for a hard threshold
    and `--eviction-max-pod-grace-period` for a soft one (`killPodFunc` override);
  * ranking (`rankMemoryPressure` / `rankDiskPressureFunc`): pods without stats first, then
    pods whose usage exceeds their requests, then lower priority (with the PodPriority gate),
    then the largest usage above requests;
  * `Admit` (:119): with no pressure everything; critical pods always; under MemoryPressure
    only, non-BestEffort pods; otherwise `The node was low on resource: [<conditions>].`;
  * local storage (`localStorageEviction`, LocalStorageCapacityIsolation gate): emptyDir over
    its sizeLimit, pod or container ephemeral-storage over its limit.

Signals come from `signals_fn()` -> {signal: (available, capacity)} so hollow nodes and tests
inject them; the default observes the host (psutil, statvfs of the kubelet root). Per-pod usage
comes from `stats_fn(pod)` -> {"memory": bytes, "disk": bytes, "inodes": n, "volumes":
{name: bytes}, "containers": {name: bytes}} or None (no stats).
"""
from __future__ import annotations

import inspect
import logging
import os
import time

from ..api.quantity import parse_quantity
from ..utils.features import DefaultFeatureGate
from . import qos

log = logging.getLogger("kubelet.eviction")

REASON = "Evicted"
MESSAGE = "The node was low on resource: {}."

MEMORY, NODEFS, NODEFS_INODES, IMAGEFS, IMAGEFS_INODES = "memory", "nodefs", "nodefsInodes", "imagefs", "imagefsInodes"
# signal -> (starved resource, node condition)
SIGNALS = {
    "memory.available": (MEMORY, "MemoryPressure"),
    "allocatableMemory.available": (MEMORY, "MemoryPressure"),
    "nodefs.available": (NODEFS, "DiskPressure"),
    "nodefs.inodesFree": (NODEFS_INODES, "DiskPressure"),
    "imagefs.available": (IMAGEFS, "DiskPressure"),
    "imagefs.inodesFree": (IMAGEFS_INODES, "DiskPressure"),
}
# compatibility views
SIGNAL_RESOURCE = {s: r for s, (r, _c) in SIGNALS.items()}
SIGNAL_CONDITION = {s: c for s, (_r, c) in SIGNALS.items()}
RESOURCE_CLAIM_TO_SIGNAL = {NODEFS: ["nodefs.available"], IMAGEFS: ["imagefs.available"],
                            NODEFS_INODES: ["nodefs.inodesFree"], IMAGEFS_INODES: ["imagefs.inodesFree"]}
# `resourceToRankFunc` (no dedicated image fs): which usage a disk resource ranks by
RANK_USAGE = {MEMORY: "memory", NODEFS: "disk", IMAGEFS: "disk", NODEFS_INODES: "inodes", IMAGEFS_INODES: "inodes"}


class Threshold:
    """`evictionapi.Threshold`: `grace` 0 = hard (evicts at once); a soft threshold acts only
    after it has been met for `grace` seconds. Values: `value` (bytes / inodes) or `percent`
    (0-100 of capacity). `min_reclaim`: ("value", n) | ("percent", p) | None."""

    def __init__(self, signal, value=None, percent=None, grace=0.0, min_reclaim=None):
        self.signal, self.value, self.percent = signal, value, percent
        self.grace = float(grace or 0.0)
        self.min_reclaim = min_reclaim

    @property
    def hard(self):
        return self.grace == 0

    def key(self):
        """`hasThreshold` identity: signal, operator, value and grace period."""
        return (self.signal, self.value, self.percent, self.grace)

    def limit(self, capacity):
        return self.value if self.value is not None else capacity * self.percent / 100.0

    def met(self, available, capacity, reclaiming=False):
        """`thresholdsMet`: available < threshold (+ minimum reclaim when enforcing it)."""
        limit = self.limit(capacity)
        if reclaiming and self.min_reclaim:
            kind, v = self.min_reclaim
            limit += v if kind == "value" else capacity * v / 100.0
        return available < limit

    def __repr__(self):
        return f"{self.signal}<{self.value if self.value is not None else f'{self.percent:g}%'}"


def parse_duration(v: str) -> float:
    """Go duration subset: 1m30s, 90s, 2h, 500ms."""
    import re
    total, pos = 0.0, 0
    units = {"h": 3600, "m": 60, "s": 1, "ms": 1e-3}
    for m in re.finditer(r"(\d+(?:\.\d+)?)(ms|h|m|s)", v):
        if m.start() != pos:
            break
        total += float(m.group(1)) * units[m.group(2)]
        pos = m.end()
    if pos != len(v) or not v:
        raise ValueError(f"invalid duration {v!r}")
    return total


def _valid(signal):
    if signal not in SIGNALS:
        raise ValueError(f"unsupported eviction signal {signal}")


def _statements(spec, sep):
    """'a<b,c<d' (sep '<') or 'a=b,c=d' (sep '=') or a dict -> {signal: value}."""
    if isinstance(spec, dict):
        return dict(spec)
    out = {}
    for part in (spec or "").split(","):
        part = part.strip()
        if not part:
            continue
        if sep not in part:
            raise ValueError(f"invalid eviction entry {part!r}")
        k, v = part.split(sep, 1)
        out[k.strip()] = v.strip()
    return out


def _percent(v):
    try:
        return float(v.rstrip("%"))
    except ValueError:
        raise ValueError(f"invalid percentage {v!r}") from None


def parse_threshold_statement(signal, val):
    """`parseThresholdStatement`: a positive quantity or a positive percentage."""
    _valid(signal)
    if val.endswith("%"):
        p = _percent(val)
        if p <= 0:
            raise ValueError(f"eviction percentage threshold {signal} must be positive: {val}")
        return Threshold(signal, percent=p)
    q = parse_quantity(val)
    if q.value <= 0:
        raise ValueError(f"eviction threshold {signal} must be positive: {val}")
    return Threshold(signal, value=int(q.int_value()))


def parse_grace_periods(spec):
    out = {}
    for sig, v in _statements(spec, "=").items():
        _valid(sig)
        if v.startswith("-"):
            raise ValueError(f"invalid eviction grace period specified: {v}, must be a positive value")
        out[sig] = parse_duration(v)
    return out


def parse_minimum_reclaims(spec):
    out = {}
    for sig, v in _statements(spec, "=").items():
        _valid(sig)
        if v.endswith("%"):
            p = _percent(v)
            if p <= 0:
                raise ValueError(f"eviction percentage minimum reclaim {sig} must be positive: {v}")
            out[sig] = ("percent", p)
            continue
        q = parse_quantity(v)
        if q.value < 0:
            raise ValueError(f"negative eviction minimum reclaim specified for {sig}")
        out[sig] = ("value", int(q.int_value()))
    return out


def parse_threshold_config(allocatable_config=(), hard="", soft="", soft_grace="", min_reclaim=""):
    """`ParseThresholdConfig`."""
    out = []
    if "pods" in (allocatable_config or ()):
        out.append(Threshold("allocatableMemory.available", value=0, min_reclaim=("value", 0)))
    out += [parse_threshold_statement(s, v) for s, v in _statements(hard, "<").items()]
    softs = [parse_threshold_statement(s, v) for s, v in _statements(soft, "<").items()]
    graces = parse_grace_periods(soft_grace)
    for t in softs:
        if t.signal not in graces:
            raise ValueError(f"grace period must be specified for the soft eviction threshold {t.signal}")
        t.grace = graces[t.signal]
    out += softs
    reclaims = parse_minimum_reclaims(min_reclaim)
    for t in out:
        if t.signal in reclaims:
            t.min_reclaim = reclaims[t.signal]
    return out


def parse_thresholds(spec: str, min_reclaim: str = ""):
    """Hard thresholds (`--eviction-hard`) with their minimum reclaims."""
    return parse_threshold_config((), spec, "", "", min_reclaim)


def parse_soft_thresholds(spec: str, grace_periods: str, min_reclaim: str = ""):
    """Soft thresholds (`--eviction-soft` + `--eviction-soft-grace-period`)."""
    return parse_threshold_config((), "", spec, grace_periods, min_reclaim)


def host_signals(root="/"):
    """memory.available from the host, nodefs.{available,inodesFree} from statvfs of the kubelet
    root; with no dedicated image fs the imagefs signals observe the same file system."""
    out = {}
    try:
        import psutil
        vm = psutil.virtual_memory()
        out["memory.available"] = (vm.available, vm.total)
    except Exception:      # noqa: BLE001 - no psutil: no memory signal
        pass
    try:
        st = os.statvfs(root if os.path.exists(root) else "/")
        out["nodefs.available"] = out["imagefs.available"] = (st.f_bavail * st.f_frsize, st.f_blocks * st.f_frsize)
        if st.f_files:
            out["nodefs.inodesFree"] = out["imagefs.inodesFree"] = (st.f_favail, st.f_files)
    except OSError:
        pass
    return out


def _q(v):
    return parse_quantity(str(v)).int_value() if v is not None else 0


def pod_request(pod, resource):
    """`podRequest`: sum over containers, or the largest init container if that is more;
    ephemeral storage only with LocalStorageCapacityIsolation."""
    if resource == "disk" and not DefaultFeatureGate("LocalStorageCapacityIsolation"):
        return 0
    key = "memory" if resource == "memory" else "ephemeral-storage"
    if resource == "inodes":
        return 0
    spec = pod.get("spec") or {}
    total = sum(_q(((c.get("resources") or {}).get("requests") or {}).get(key)) for c in spec.get("containers") or ())
    init = max((_q(((c.get("resources") or {}).get("requests") or {}).get(key)) for c in spec.get("initContainers") or ()),
               default=0)
    return max(total, init)


def _cmp_bool(a, b):
    """`cmpBool`: true sorts first."""
    if a == b:
        return 0
    return -1 if not b else 1


def rank(pods, resource, stats_fn):
    """`rankMemoryPressure` / `rankDiskPressureFunc`: orderedBy(exceedRequests, priority,
    usage above requests) — a stable sort, most evictable first."""
    import functools
    usage_key = RANK_USAGE[resource]
    prio_on = DefaultFeatureGate("PodPriority")

    def usage(p):
        s = stats_fn(p)
        return None if s is None else int(s.get(usage_key, 0) or 0)

    cache = {id(p): usage(p) for p in pods}

    def cmp(p1, p2):
        u1, u2 = cache[id(p1)], cache[id(p2)]
        if u1 is None or u2 is None:
            return _cmp_bool(u1 is None, u2 is None)
        r1, r2 = pod_request(p1, usage_key), pod_request(p2, usage_key)
        c = _cmp_bool(u1 > r1, u2 > r2)
        if c:
            return c
        if prio_on:
            a = int((p1.get("spec") or {}).get("priority") or 0)
            b = int((p2.get("spec") or {}).get("priority") or 0)
            if a != b:
                return -1 if a < b else 1
        d1, d2 = u1 - r1, u2 - r2
        return (d2 > d1) - (d2 < d1)
    return sorted(pods, key=functools.cmp_to_key(cmp))


def is_static(pod):
    src = ((pod.get("metadata") or {}).get("annotations") or {}).get("kubernetes.io/config.source")
    return bool(src) and src != "api"


def critical(pod):
    return DefaultFeatureGate("ExperimentalCriticalPodAnnotation") and qos.is_critical_pod(pod)


class EvictionManager:
    """`thresholds` may mix hard and soft ones; `max_pod_grace` is
    --eviction-max-pod-grace-period (the kill grace of a soft eviction). `reclaim_fns`:
    {resource: [callable -> bytes freed (may be async)]} node-level reclaim (container GC, image
    GC); `recorder(obj_or_None, type, reason, message)` receives node events (obj None = node)."""

    def __init__(self, thresholds, signals_fn=None, usage_fn=None, pressure_transition_period=0.0, max_pod_grace=0,
                 clock=time.monotonic, stats_fn=None, reclaim_fns=None, recorder=None):
        self.thresholds = list(thresholds)
        self.signals_fn = signals_fn or host_signals
        if stats_fn is None:
            # the older single-number usage hook: memory (and disk) usage in bytes
            ufn = usage_fn or (lambda pod: 0)
            stats_fn = (lambda pod: {"memory": ufn(pod), "disk": ufn(pod), "inodes": 0})
        self.stats_fn = stats_fn
        self.usage_fn = usage_fn
        self.transition = pressure_transition_period
        self.max_pod_grace = max_pod_grace
        self.clock = clock
        self.reclaim_fns = reclaim_fns or {}
        self.recorder = recorder
        self.node_conditions: list = []
        self.conditions: dict[str, float] = {}     # condition -> last observed (nodeConditionsLastObservedAt)
        self.first_observed: dict = {}             # threshold key -> first time met
        self.thresholds_met: list = []             # thresholds that passed their grace last pass
        self.last_observation: dict = {}

    # -- observation ------------------------------------------------------------------------
    def _met(self, thresholds, obs, enforce_min_reclaim):
        return [t for t in thresholds if t.signal in obs and t.met(*obs[t.signal], reclaiming=enforce_min_reclaim)]

    def observe(self, obs=None):
        """One `synchronize` bookkeeping pass -> the thresholds whose grace period has passed
        (hard ones: immediately), hard first. Node conditions follow every met threshold
        (soft ones before their grace period too) for the transition period."""
        obs = self.signals_fn() if obs is None else obs
        now = self.clock()
        met = self._met(self.thresholds, obs, False)
        if self.thresholds_met:
            keys = {t.key() for t in met}
            met += [t for t in self._met(self.thresholds_met, obs, True) if t.key() not in keys]
        self.first_observed = {t.key(): self.first_observed.get(t.key(), now) for t in met}
        for t in met:
            self.conditions[SIGNAL_CONDITION[t.signal]] = now
        for c, at in list(self.conditions.items()):
            if now - at >= self.transition and not any(SIGNAL_CONDITION[t.signal] == c for t in met):
                del self.conditions[c]
        self.node_conditions = sorted(self.conditions)
        ripe = [t for t in met if now - self.first_observed[t.key()] >= t.grace]
        self.thresholds_met = ripe
        self.last_observation = obs
        return sorted(ripe, key=lambda t: not t.hard)

    def hard_memory_bytes(self):
        """The memory.available hard threshold in bytes (percent thresholds count as 0 here:
        node allocatable needs an absolute value)."""
        return sum(int(t.value or 0) for t in self.thresholds if t.signal == "memory.available" and t.hard)

    def has(self, condition):
        return condition in self.conditions

    def admit(self, pod):
        """`Admit` -> None, or (reason, message) when the pod must be rejected."""
        if not self.conditions:
            return None
        if critical(pod):
            return None
        if "MemoryPressure" in self.conditions and qos.pod_qos(pod) != qos.BEST_EFFORT:
            return None
        return REASON, MESSAGE.format("[" + " ".join(sorted(self.conditions)) + "]")     # Go's %v of a slice

    # -- eviction ------------------------------------------------------------------------
    def rank(self, pods, signal):
        return rank(pods, SIGNAL_RESOURCE[signal], self.stats_fn)

    @staticmethod
    def _starved(thresholds):
        """`getStarvedResources` sorted `byEvictionPriority` (memory first)."""
        res = [SIGNAL_RESOURCE[t.signal] for t in thresholds]
        return sorted(res, key=lambda r: r != MEMORY)

    def _plan(self, ripe):
        resource = self._starved(ripe)[0]
        soft = not any(t.hard for t in ripe if SIGNAL_RESOURCE[t.signal] == resource)
        return resource, soft

    def _pick(self, pods, resource, soft):
        for p in rank(pods, resource, self.stats_fn):
            if critical(p) and is_static(p):
                continue
            grace = int(self.max_pod_grace) if soft else 0
            return p, MESSAGE.format(resource), grace
        return None, None, 0

    def select_victim(self, pods):
        victim, msg, _grace = self.select_victim_with_grace(pods)
        return victim, msg

    def select_victim_with_grace(self, pods):
        """A synchronous pass without node-level reclaim -> (pod, message, grace) or
        (None, None, 0)."""
        ripe = self.observe()
        if not ripe or not pods:
            return None, None, 0
        resource, soft = self._plan(ripe)
        return self._pick(pods, resource, soft)

    async def _reclaim(self, resource, obs):
        """`reclaimNodeLevelResources`: run the resource's reclaim functions in order, adding
        what they free to its signals; True once no met threshold remains (min reclaim
        enforced)."""
        for fn in self.reclaim_fns.get(resource, ()):
            try:
                freed = fn()
                if inspect.isawaitable(freed):
                    freed = await freed
            except Exception as e:      # noqa: BLE001 - the reference logs and goes on
                log.warning("eviction manager: node-level reclaim for %s failed: %s", resource, e)
                freed = 0
            for sig in RESOURCE_CLAIM_TO_SIGNAL.get(resource, ()):
                if sig in obs:
                    avail, cap = obs[sig]
                    obs[sig] = (avail + int(freed or 0), cap)
            if not self._met(self.thresholds_met, obs, True):
                return True
        return False

    def local_storage_violation(self, pod):
        """`localStorageEviction` (LocalStorageCapacityIsolation) -> message or None."""
        if not DefaultFeatureGate("LocalStorageCapacityIsolation"):
            return None
        s = self.stats_fn(pod)
        if not s:
            return None
        spec = pod.get("spec") or {}
        vols = s.get("volumes") or {}
        for v in spec.get("volumes") or ():
            lim = (v.get("emptyDir") or {}).get("sizeLimit") if "emptyDir" in v else None
            if lim is not None and _q(lim) > 0 and vols.get(v.get("name"), 0) > _q(lim):
                return f"emptyDir usage exceeds the limit {lim!r}"
        limits = [((c.get("resources") or {}).get("limits") or {}).get("ephemeral-storage") for c in spec.get("containers") or ()]
        if any(lim is not None for lim in limits):
            total = sum(_q(lim) for lim in limits)
            if s.get("disk", 0) > total:
                return f"pod ephemeral local storage usage exceeds the total limit of containers {total}"
        used = s.get("containers") or {}
        for c in spec.get("containers") or ():
            lim = ((c.get("resources") or {}).get("limits") or {}).get("ephemeral-storage")
            if lim is not None and _q(lim) and used.get(c.get("name"), 0) > _q(lim):
                return f"container's ephemeral local storage usage exceeds the limit {lim!r}"
        return None

    async def synchronize(self, pods):
        """`synchronize` -> (pod, message, grace, event message) or (None, None, 0, None)."""
        if not self.thresholds:
            return None, None, 0, None
        obs = dict(self.signals_fn())
        ripe = self.observe(obs)
        for p in pods:
            why = self.local_storage_violation(p)
            if why is not None and not (critical(p) and is_static(p)):
                return p, MESSAGE.format("ephemeral-storage"), 0, why
        if not ripe:
            return None, None, 0, None
        resource, soft = self._plan(ripe)
        if self.recorder is not None:
            self.recorder(None, "Warning", "EvictionThresholdMet", f"Attempting to reclaim {resource}")
        if await self._reclaim(resource, obs):
            return None, None, 0, None
        if not pods:
            return None, None, 0, None
        victim, msg, grace = self._pick(pods, resource, soft)
        return victim, msg, grace, msg
