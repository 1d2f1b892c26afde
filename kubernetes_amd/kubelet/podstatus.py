"""Pod status helpers of the kubelet status manager.

  * `generate_pod_ready_condition` / `generate_pod_initialized_condition` —
    `pkg/kubelet/status/generate.go:36,91`: the Ready condition from the app containers'
    `ready` flags (PodCompleted once the pod succeeded, UnknownContainerStatuses without
    statuses, otherwise ContainersNotReady naming unknown and unready containers), the
    Initialized condition from the init containers' (an init container is ready once it
    exited 0, `prober_manager.go:212`).
  * `normalize_status` — `status_manager.go:565` normalizeStatus: terminated messages are cut to
    an equal share of `MAX_POD_TERMINATION_MESSAGE_LOG_LENGTH` per container; app container
    statuses are sorted by name and init container statuses into spec order, so their order
    never makes two statuses differ.
"""
from __future__ import annotations

UNKNOWN_CONTAINER_STATUSES = "UnknownContainerStatuses"
POD_COMPLETED = "PodCompleted"
CONTAINERS_NOT_READY = "ContainersNotReady"
CONTAINERS_NOT_INITIALIZED = "ContainersNotInitialized"

MAX_CONTAINER_TERMINATION_MESSAGE_LENGTH = 1024 * 4      # kubecontainer.MaxContainerTerminationMessageLength
MAX_POD_TERMINATION_MESSAGE_LOG_LENGTH = 1024 * 12      # kubecontainer.MaxPodTerminationMessageLogLength


def _go_list(names) -> str:
    return "[" + " ".join(names) + "]"


def _classify(containers, statuses):
    by_name = {s.get("name"): s for s in statuses}
    unknown, unready = [], []
    for c in containers or ():
        s = by_name.get(c["name"])
        if s is None:
            unknown.append(c["name"])
        elif not s.get("ready"):
            unready.append(c["name"])
    return unknown, unready


def _cond(ctype, ok, reason=None, message=None):
    c = {"type": ctype, "status": "True" if ok else "False"}
    if reason:
        c["reason"] = reason
    if message:
        c["message"] = message
    return c


def generate_pod_ready_condition(spec, statuses, phase) -> dict:
    if statuses is None:
        return _cond("Ready", False, UNKNOWN_CONTAINER_STATUSES)
    unknown, unready = _classify((spec or {}).get("containers"), statuses)
    if phase == "Succeeded" and not unknown:
        return _cond("Ready", False, POD_COMPLETED)
    msgs = []
    if unknown:
        msgs.append(f"containers with unknown status: {_go_list(unknown)}")
    if unready:
        msgs.append(f"containers with unready status: {_go_list(unready)}")
    if msgs:
        return _cond("Ready", False, CONTAINERS_NOT_READY, ", ".join(msgs))
    return _cond("Ready", True)


def generate_pod_initialized_condition(spec, statuses, phase) -> dict:
    spec = spec or {}
    if statuses is None and spec.get("initContainers"):
        return _cond("Initialized", False, UNKNOWN_CONTAINER_STATUSES)
    unknown, unready = _classify(spec.get("initContainers"), statuses or ())
    if phase == "Succeeded" and not unknown:
        return _cond("Initialized", True, POD_COMPLETED)
    msgs = []
    if unknown:
        msgs.append(f"containers with unknown status: {_go_list(unknown)}")
    if unready:
        msgs.append(f"containers with incomplete status: {_go_list(unready)}")
    if msgs:
        return _cond("Initialized", False, CONTAINERS_NOT_INITIALIZED, ", ".join(msgs))
    return _cond("Initialized", True)


def normalize_status(pod, status) -> dict:
    """In place; returns `status`."""
    spec = pod.get("spec") or {}
    per = MAX_POD_TERMINATION_MESSAGE_LOG_LENGTH
    n = len(spec.get("containers") or ()) + len(spec.get("initContainers") or ())
    if n > 0:
        per //= n

    def cut(state):
        t = (state or {}).get("terminated")
        if t and t.get("message") and len(t["message"]) > per:
            t["message"] = t["message"][:per]

    for key in ("containerStatuses", "initContainerStatuses"):
        for cs in status.get(key) or ():
            cut(cs.get("state"))
            cut(cs.get("lastState"))
    if status.get("containerStatuses"):
        status["containerStatuses"].sort(key=lambda s: s.get("name", ""))
    if status.get("initContainerStatuses"):
        sort_init_container_statuses(pod, status["initContainerStatuses"])
    return status


def sort_init_container_statuses(pod, statuses):
    """`kubetypes.SortInitContainerStatuses`: into the spec's init-container order (statuses of
    names not in the spec stay behind, in their relative order after the swaps)."""
    cur = 0
    for c in (pod.get("spec") or {}).get("initContainers") or ():
        for j in range(cur, len(statuses)):
            if statuses[j].get("name") == c["name"]:
                statuses[cur], statuses[j] = statuses[j], statuses[cur]
                cur += 1
                break
