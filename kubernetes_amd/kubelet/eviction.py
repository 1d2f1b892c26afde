"""Eviction manager: node pressure conditions, pressure-aware admission, pod eviction.

Parity: `pkg/kubelet/eviction/eviction_manager.go:151-214` (`synchronize`: observe signals,
compare with thresholds, update node conditions, evict at most one pod per pass),
`helpers.go` (threshold parsing `memory.available<100Mi`, `nodefs.available<10%`; ranking:
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
    def __init__(self, signal, value=None, percent=None):
        self.signal, self.value, self.percent = signal, value, percent

    def met(self, available, capacity):
        limit = self.value if self.value is not None else capacity * self.percent / 100.0
        return available < limit

    def __repr__(self):
        return f"{self.signal}<{self.value if self.value is not None else str(self.percent) + '%'}"


def parse_thresholds(spec: str):
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
            out.append(Threshold(sig, percent=float(val[:-1])))
        else:
            out.append(Threshold(sig, value=int(parse_quantity(val).int_value())))
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
    def __init__(self, thresholds, signals_fn=None, usage_fn=None, pressure_transition_period=0.0):
        self.thresholds = thresholds
        self.signals_fn = signals_fn or host_signals
        self.usage_fn = usage_fn or (lambda pod: 0)
        self.transition = pressure_transition_period
        self.conditions: dict[str, float] = {}     # condition -> last time observed
        self.last_observation = {}

    def observe(self):
        sig = self.signals_fn()
        self.last_observation = sig
        now = time.monotonic()
        met = []
        for t in self.thresholds:
            if t.signal in sig and t.met(*sig[t.signal]):
                met.append(t)
                self.conditions[SIGNAL_CONDITION[t.signal]] = now
        # a condition stays set for the transition period after the last observation
        for c, ts in list(self.conditions.items()):
            if now - ts > self.transition and not any(SIGNAL_CONDITION[t.signal] == c for t in met):
                del self.conditions[c]
        return met

    def hard_memory_bytes(self):
        """The memory.available hard threshold in bytes (percent thresholds count as 0 here:
        node allocatable needs an absolute value)."""
        return sum(int(getattr(t, "value", 0) or 0) for t in self.thresholds
                   if getattr(t, "signal", "") == "memory.available")

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
        met = self.observe()
        if not met or not pods:
            return None, None
        t = met[0]
        ranked = self.rank(pods, t.signal)
        return ranked[0], f"The node was low on resource: {SIGNAL_RESOURCE[t.signal]}. Threshold {t!r} met."
