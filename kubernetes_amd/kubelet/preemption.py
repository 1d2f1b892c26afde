"""Critical-pod admission preemption (`pkg/kubelet/preemption/preemption.go`).

When a critical pod (`qos.is_critical_pod`: a kube-system pod with the critical-pod annotation,
or a system priority — e.g. the amd.com/gpu device-plugin DaemonSet) is rejected by the kubelet's
admission only for lack of cpu / memory / pod slots, the kubelet evicts running non-critical pods
to make room instead of failing the critical one:

  * candidates are grouped by QoS class; the set is chosen so Guaranteed pods go only if
    evicting every BestEffort and Burstable pod would not be enough, then Burstable pods only if
    BestEffort ones are not enough, then BestEffort pods;
  * inside a class, pods are picked greedily by *distance* to the remaining shortfall — the sum
    over short resources of (uncovered fraction)², each resource weighted equally whatever its
    magnitude — ties going to the pod with the smaller request (amd.com/gpu, then memory, cpu);
  * victims are killed and marked Failed/`Preempting` with a Warning event before the critical
    pod is admitted.
"""
from __future__ import annotations

from ..api import core
from .qos import BEST_EFFORT, BURSTABLE, GUARANTEED, is_critical_pod, pod_qos

PREEMPT_REASON = "Preempting"
PREEMPT_MESSAGE = "Preempted in order to admit critical pod"
RESOURCE_REASONS = {"OutOfcpu": "cpu", "OutOfmemory": "memory", "OutOfpods": "pods"}
SMALLER_ORDER = (core.AMD_GPU, "memory", "cpu")


def request_of(pod, resource) -> int:
    """`resource.GetResourceRequest`: cpu in millicores, memory/extended in units, pods = 1."""
    if resource == "pods":
        return 1
    q = core.pod_requests(pod).get(resource)
    if q is None:
        return 0
    return q.milli_value() if resource == "cpu" else q.value


def remaining(reqs: dict, pods) -> dict:
    out = {}
    for r, need in reqs.items():
        left = need - sum(request_of(p, r) for p in pods)
        if left > 0:
            out[r] = left
    return out


def distance(reqs: dict, pod) -> float:
    return sum((max(0, need - request_of(pod, r)) / need) ** 2 for r, need in reqs.items())


def _smaller(a, b) -> bool:
    for r in SMALLER_ORDER:
        x, y = request_of(a, r), request_of(b, r)
        if x != y:
            return x < y
    return True


def _by_distance(pods, reqs):
    pods = list(pods)
    chosen = []
    while reqs:
        if not pods:
            raise ValueError(f"no set of running pods found to reclaim resources: {reqs}")
        best = 0
        best_d = distance(reqs, pods[0])
        for i in range(1, len(pods)):
            d = distance(reqs, pods[i])
            if d < best_d or (d == best_d and _smaller(pods[i], pods[best])):
                best, best_d = i, d
        victim = pods.pop(best)
        chosen.append(victim)
        reqs = remaining(reqs, [victim])
    return chosen


def pods_to_preempt(active_pods, reqs: dict):
    """The victims for a shortfall `reqs` ({resource: amount}); raises ValueError if even
    evicting every non-critical pod would not cover it."""
    classes = {BEST_EFFORT: [], BURSTABLE: [], GUARANTEED: []}
    for p in active_pods:
        if not is_critical_pod(p):
            classes.setdefault(pod_qos(p), []).append(p)
    be, bu, gu = classes[BEST_EFFORT], classes[BURSTABLE], classes[GUARANTEED]
    if remaining(reqs, be + bu + gu):
        raise ValueError(f"no set of running pods found to reclaim resources: {remaining(reqs, be + bu + gu)}")
    g = _by_distance(gu, remaining(reqs, be + bu))
    b = _by_distance(bu, remaining(reqs, be + g))
    e = _by_distance(be, remaining(reqs, b + g))
    return e + b + g


class CriticalPodAdmissionHandler:
    """`HandleAdmissionFailure`: returns True when victims were evicted and the pod can be
    re-admitted. `kill(pod, status)` stops a victim and writes its Failed status."""

    def __init__(self, active_pods, kill, recorder=None):
        self.active_pods = active_pods
        self.kill = kill
        self.recorder = recorder

    async def handle_admission_failure(self, pod, shortfall: dict) -> bool:
        if not is_critical_pod(pod) or not shortfall:
            return False
        others = [p for p in self.active_pods() if p["metadata"]["uid"] != pod["metadata"]["uid"]]
        victims = pods_to_preempt(others, shortfall)
        for v in victims:
            if self.recorder is not None:
                self.recorder.event(v, "Warning", PREEMPT_REASON, PREEMPT_MESSAGE)
            await self.kill(v, {"phase": core.POD_FAILED, "reason": PREEMPT_REASON, "message": PREEMPT_MESSAGE})
        return True
