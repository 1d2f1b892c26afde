"""Kubelet runtime state behind the node's Ready condition (`pkg/kubelet/runtime.go`,
`Kubelet.updateRuntimeUp` in `pkg/kubelet/kubelet.go:2102`, `setNodeReadyCondition` in
`pkg/kubelet/kubelet_node_status.go:738`).

  * `RuntimeState` keeps the time of the last successful runtime sanity check, an internal
    error, named health checks and the network error (initially "network state unknown").
    `runtime_errors()` reports "container runtime is down" once the last check is older than
    the threshold (`maxWaitForContainerRuntime`, 30 s), the internal error and each failing
    health check ("<name> is not healthy: <err>").
  * `update_runtime_up(state, status, now)` applies one runtime `Status()` result: an error or
    None changes nothing (the check goes stale); NetworkReady false or missing sets the
    network error; RuntimeReady false or missing stops before the sync time is refreshed.
  * `ready_condition(errors)` is the (status, reason, message) of NodeReady.
"""
from __future__ import annotations

import time

RUNTIME_READY, NETWORK_READY = "RuntimeReady", "NetworkReady"
MAX_WAIT_FOR_CONTAINER_RUNTIME = 30.0


class RuntimeState:
    def __init__(self, threshold: float = MAX_WAIT_FOR_CONTAINER_RUNTIME, clock=time.time):
        self.threshold = threshold
        self.clock = clock
        self.last_sync = 0.0
        self.internal_error: str | None = None
        self.network_error: str | None = "network state unknown"
        self.health_checks: list = []          # (name, fn() -> (ok, err))

    def set_runtime_sync(self, t):
        self.last_sync = t

    def set_internal_error(self, err):
        self.internal_error = None if err is None else str(err)

    def set_network_state(self, err):
        self.network_error = None if err is None else str(err)

    def add_health_check(self, name, fn):
        self.health_checks.append((name, fn))

    def runtime_errors(self) -> list:
        out = []
        if not self.last_sync + self.threshold > self.clock():
            out.append("container runtime is down")
        if self.internal_error:
            out.append(self.internal_error)
        for name, fn in self.health_checks:
            ok, err = fn()
            if not ok:
                out.append(f"{name} is not healthy: {err}")
        return out

    def network_errors(self) -> list:
        return [self.network_error] if self.network_error else []


def _cond_str(name, cond):
    if cond is None:
        return "<nil>"
    ok, reason, msg = cond
    return f"{name}={'true' if ok else 'false'} reason:{reason} message:{msg}"


def update_runtime_up(state: RuntimeState, status, now=None, error=None) -> bool:
    """`status`: {type: (ok, reason, message)} from the runtime's Status(), or None. Returns
    whether the runtime sync time was refreshed."""
    if error is not None or status is None:
        return False
    net = status.get(NETWORK_READY)
    if net is None or not net[0]:
        state.set_network_state(f"runtime network not ready: {_cond_str(NETWORK_READY, net)}")
    else:
        state.set_network_state(None)
    rt = status.get(RUNTIME_READY)
    if rt is None or not rt[0]:
        return False
    state.set_runtime_sync(state.clock() if now is None else now)
    return True


def ready_condition(errors) -> tuple:
    if not errors:
        return "True", "KubeletReady", "kubelet is posting ready status"
    return "False", "KubeletNotReady", ",".join(errors)
