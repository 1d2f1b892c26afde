"""Pod QoS classes, OOM score adjustment and critical pods (`pkg/kubelet/qos`, `pkg/kubelet/types`).

  * `pod_qos(pod)`          — `qos.GetPodQOS` (Guaranteed / Burstable / BestEffort), the same rule
                              the API server uses to fill `status.qosClass`;
  * `oom_score_adj(...)`    — `qos.GetContainerOOMScoreAdjust` (`pkg/kubelet/qos/policy.go`):
                              Guaranteed -998, BestEffort 1000, Burstable
                              `1000 - 1000*memoryRequest/memoryCapacity` clamped to [2, 999] so a
                              Burstable container is never killed after a Guaranteed one and
                              always after BestEffort; the pause container -998;
  * `is_critical_pod(pod)`  — `kubetypes.IsCriticalPod` (`pkg/kubelet/types/pod_update.go`): the
                              `scheduler.alpha.kubernetes.io/critical-pod` annotation in
                              kube-system, or a system priority (>= 2e9, priority admission).
"""
from __future__ import annotations

from ..api.quantity import parse_quantity

GUARANTEED, BURSTABLE, BEST_EFFORT = "Guaranteed", "Burstable", "BestEffort"
CRITICAL_POD_ANNOTATION = "scheduler.alpha.kubernetes.io/critical-pod"
SYSTEM_CRITICAL_PRIORITY = 2_000_000_000

PAUSE_OOM_SCORE_ADJ = -998
GUARANTEED_OOM_SCORE_ADJ = -998
BESTEFFORT_OOM_SCORE_ADJ = 1000
KUBELET_OOM_SCORE_ADJ = -999


def pod_qos(pod) -> str:
    st = (pod.get("status") or {}).get("qosClass")
    if st:
        return st
    from ..apiserver.registry import qos_class
    return qos_class(pod)


def is_critical_pod(pod) -> bool:
    md = pod.get("metadata") or {}
    # IsCritical: kube-system only, and the annotation's value must be empty
    if md.get("namespace") == "kube-system" and (md.get("annotations") or {}).get(CRITICAL_POD_ANNOTATION) == "":
        return True
    prio = (pod.get("spec") or {}).get("priority")
    return prio is not None and int(prio) >= SYSTEM_CRITICAL_PRIORITY


def _mem_request(container) -> int:
    """`Requests.Memory().Value()`: the (defaulted) request only, 0 when unset."""
    r = ((container.get("resources") or {}).get("requests") or {}).get("memory")
    return parse_quantity(str(r)).value if r is not None else 0


def oom_score_adj(pod, container, memory_capacity_bytes: int) -> int:
    """`GetContainerOOMScoreAdjust` (pkg/kubelet/qos/policy.go:43): by QoS class only, so a
    critical pod's containers score like any other pod of their class."""
    q = pod_qos(pod)
    if q == GUARANTEED:
        return GUARANTEED_OOM_SCORE_ADJ
    if q == BEST_EFFORT:
        return BESTEFFORT_OOM_SCORE_ADJ
    if memory_capacity_bytes <= 0:
        return 999
    adj = 1000 - (1000 * _mem_request(container)) // memory_capacity_bytes
    floor = 1000 + GUARANTEED_OOM_SCORE_ADJ      # 2: a Guaranteed pod at 100% memory scores ~2 too
    if adj < floor:
        return floor
    return BESTEFFORT_OOM_SCORE_ADJ - 1 if adj == BESTEFFORT_OOM_SCORE_ADJ else adj
