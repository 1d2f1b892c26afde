"""Eviction manager: node pressure conditions, pressure-aware admission, pod eviction.

Parity: `pkg/kubelet/eviction/eviction_manager.go:151-214` (`synchronize`: observe signals,
compare with thresholds, update node conditions, evict at most one pod per pass),
`helpers.go` (threshold parsing `memory.available<100Mi`, `nodefs.available<10%`, soft thresholds
with grace periods, minimum reclaim, the max pod grace period of a soft eviction; ranking:
pods whose usage exceeds requests first by QoS — BestEffort, Burstable, Guaranteed — then by
priority, then by usage), `admit` (MemoryPressure rejects BestEffort pods, DiskPressure rejects
all) and the evicted pod status (phase Failed, reason Evicted).

Signals come from `signals_fn()` so hollow nodes and tests can inject them; the default
observes the host (psutil.virtual_memory, statvfs of the kubelet root).
"""
from __future__ import annotations

import logging
import os
import time

from ..api.quantity import parse_quantity

log = logging.getLogger("kubelet.eviction")

SIGNAL_RESOURCE = {"memory.available": "memory", "nodefs.available": "ephemeral-storage"}
SIGNAL_CONDITION = {"memory.available": "MemoryPressure", "nodefs.available": "DiskPressure"}
QOS_RANK = {"BestEffort": 0, "Burstable": 1, "Guaranteed": 2}


class Threshold:
    """`evictionapi.Threshold`: a hard threshold (grace None) evicts at once; a soft one only
    after it has been met for `grace` seconds. `min_reclaim` (bytes or percent of capacity):
    once met, the threshold stays met until that much more than the threshold is available."""

    def __init__(self, signal, value=None, percent=None, grace=None, min_reclaim=None):
        self.signal, self.value, self.percent = signal, value, percent
        self.grace = grace
        self.min_reclaim = min_reclaim      # ("value", bytes) | ("percent", p) | None

    def limit(self, capacity):
        return self.value if self.value is not None else capacity * self.percent / 100.0

    def met(self, available, capacity, reclaiming=False):
        limit = self.limit(capacity)
        if reclaiming and self.min_reclaim:
            kind, v = self.min_reclaim
            limit += v if kind == "value" else capacity * v / 100.0
        return available < limit

    @property
    def hard(self):
        return self.grace is None

    def __repr__(self):
        return f"{self.signal}<{self.value if self.value is not None else str(self.percent) + '%'}"


def _parse_map(spec, sep="="):
    out = {}
    for part in (spec or "").split(","):
        part = part.strip()
        if part:
            if sep not in part:
                raise ValueError(f"invalid entry {part!r}")
            k, v = part.split(sep, 1)
            if k not in SIGNAL_CONDITION:
                raise ValueError(f"unsupported eviction signal {k!r}")
            out[k] = v
    return out


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


def parse_soft_thresholds(spec: str, grace_periods: str, min_reclaim: str = ""):
    """--eviction-soft + --eviction-soft-grace-period (required for every soft signal, as the
    reference's ParseThresholdConfig demands) + --eviction-minimum-reclaim."""
    graces = {k: parse_duration(v) for k, v in _parse_map(grace_periods).items()}
    out = parse_thresholds(spec, min_reclaim)
    for t in out:
        if t.signal not in graces:
            raise ValueError(f"grace period must be specified for the soft eviction threshold {t!r}")
        t.grace = graces[t.signal]
    return out


def parse_thresholds(spec: str, min_reclaim: str = ""):
    reclaim = {}
    for sig, v in _parse_map(min_reclaim).items():
        reclaim[sig] = ("percent", float(v[:-1])) if v.endswith("%") else ("value", int(parse_quantity(v).int_value()))
    out = []
    for part in (spec or "").split(","):
        part = part.strip()
        if not part:
            continue
        if "<" not in part:
            raise ValueError(f"invalid eviction threshold {part!r}")
        sig, val = part.split("<", 1)
        if sig not in SIGNAL_CONDITION:
            raise ValueError(f"unsupported eviction signal {sig!r}")
        if val.endswith("%"):
            out.append(Threshold(sig, percent=float(val[:-1]), min_reclaim=reclaim.get(sig)))
        else:
            out.append(Threshold(sig, value=int(parse_quantity(val).int_value()), min_reclaim=reclaim.get(sig)))
    return out


def host_signals(root="/"):
    out = {}
    try:
        import psutil
        vm = psutil.virtual_memory()
        out["memory.available"] = (vm.available, vm.total)
    except Exception:
        pass
    try:
        st = os.statvfs(root if os.path.exists(root) else "/")
        out["nodefs.available"] = (st.f_bavail * st.f_frsize, st.f_blocks * st.f_frsize)
    except OSError:
        pass
    return out


class EvictionManager:
    """`thresholds` may mix hard and soft ones (`parse_soft_thresholds`); `max_pod_grace` is
    --eviction-max-pod-grace-period, the termination grace a soft eviction grants at most."""

    def __init__(self, thresholds, signals_fn=None, usage_fn=None, pressure_transition_period=0.0, max_pod_grace=0,
                 clock=time.monotonic):
        self.thresholds = list(thresholds)
        self.signals_fn = signals_fn or host_signals
        self.usage_fn = usage_fn or (lambda pod: 0)
        self.transition = pressure_transition_period
        self.max_pod_grace = max_pod_grace
        self.clock = clock
        self.conditions: dict[str, float] = {}     # condition -> last time observed
        self.last_observation = {}
        self._first_met: dict[int, float] = {}     # id(threshold) -> first time met (thresholdsFirstObservedAt)
        self._reclaiming: set[int] = set()         # thresholds met last pass (minimum reclaim applies)

    def observe(self):
        """-> thresholds whose grace period has passed (hard ones: immediately). Node conditions
        follow every met threshold, soft ones before their grace period too."""
        sig = self.signals_fn()
        self.last_observation = sig
        now = self.clock()
        met, ripe = [], []
        for t in self.thresholds:
            if t.signal in sig and t.met(*sig[t.signal], reclaiming=id(t) in self._reclaiming):
                met.append(t)
                self.conditions[SIGNAL_CONDITION[t.signal]] = now
                first = self._first_met.setdefault(id(t), now)
                if t.hard or now - first >= t.grace:
                    ripe.append(t)
            else:
                self._first_met.pop(id(t), None)
        self._reclaiming = {id(t) for t in met}
        # a condition stays set for the transition period after the last observation
        for c, ts in list(self.conditions.items()):
            if now - ts > self.transition and not any(SIGNAL_CONDITION[t.signal] == c for t in met):
                del self.conditions[c]
        # hard thresholds first: they decide the (zero) grace of this pass's eviction
        return sorted(ripe, key=lambda t: not t.hard)

    def hard_memory_bytes(self):
        """The memory.available hard threshold in bytes (percent thresholds count as 0 here:
        node allocatable needs an absolute value)."""
        return sum(int(getattr(t, "value", 0) or 0) for t in self.thresholds
                   if getattr(t, "signal", "") == "memory.available" and t.hard)

    def has(self, condition):
        return condition in self.conditions

    def admit(self, pod):
        """Returns (reason, message) if the pod must be rejected under node pressure."""
        if self.has("DiskPressure"):
            return "Evicted", "The node was low on resource: [DiskPressure]."
        if self.has("MemoryPressure") and ((pod.get("status") or {}).get("qosClass") or "BestEffort") == "BestEffort":
            return "Evicted", "The node was low on resource: [MemoryPressure]."
        return None

    def rank(self, pods, signal):
        res = SIGNAL_RESOURCE[signal]

        def requests(p):
            tot = 0
            for c in (p.get("spec") or {}).get("containers") or ():
                q = ((c.get("resources") or {}).get("requests") or {}).get(res)
                if q:
                    tot += parse_quantity(str(q)).int_value()
            return tot

        def key(p):
            usage = self.usage_fn(p)
            exceeds = usage > requests(p)
            qos = QOS_RANK.get((p.get("status") or {}).get("qosClass") or "BestEffort", 0)
            prio = int((p.get("spec") or {}).get("priority") or 0)
            return (not exceeds, qos, prio, -usage)
        return sorted(pods, key=key)

    def select_victim(self, pods):
        """At most one pod to evict this pass (eviction_manager.go: one per synchronize)."""
        victim, msg, _grace = self.select_victim_with_grace(pods)
        return victim, msg

    def select_victim_with_grace(self, pods):
        """-> (pod, message, termination grace seconds): 0 for a hard threshold, for a soft one
        the pod's own grace capped at --eviction-max-pod-grace-period."""
        met = self.observe()
        if not met or not pods:
            return None, None, 0
        t = met[0]
        victim = self.rank(pods, t.signal)[0]
        grace = 0
        if not t.hard:
            own = int((victim.get("spec") or {}).get("terminationGracePeriodSeconds", 30))
            grace = min(own, int(self.max_pod_grace)) if self.max_pod_grace > 0 else own
        return victim, f"The node was low on resource: {SIGNAL_RESOURCE[t.signal]}. Threshold {t!r} met.", grace
