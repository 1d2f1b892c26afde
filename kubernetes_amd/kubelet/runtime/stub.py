"""Stub runtime — fake sandboxes/containers for kubemark hollow nodes and the density bench.

Parity: kubemark's hollow kubelet drives a fake docker client (`cmd/kubemark/hollow-node.go:114-137`,
`pkg/kubelet/dockershim/libdocker/fake_client.go`, `EnableSleep`): containers "run" without
processes. Added for MI355X: an optional GPU *payload* — when a container was given AMD GPU
device nodes by the device plugin, `payload(opts)` is invoked at container start (e.g. the HIP
vector_add kernel on the rank's real MI355X, `ops.hip_kernels.Payload`) and a failing payload
makes the container exit with code 1, like a real GPU container crashing at start.

Containers may declare a run time with the annotation `kubemark.amd.com/run-seconds` (or a
`["sleep", N]` command); otherwise they run until stopped.

Stopping honours the grace period the kubelet passes (the pod's deletion grace /
terminationGracePeriodSeconds, `kuberuntime_container.go:574-599`): a container whose pod
carries `kubemark.amd.com/stop-seconds: S` keeps running for S seconds after the stop signal —
a workload draining on SIGTERM — and exits 0 then; when S reaches the grace period it is killed
at the grace period (137), like a workload that ignores SIGTERM. Without the annotation the stop
is immediate, as with kubemark's fake docker.
"""
from __future__ import annotations

import asyncio
import inspect
import itertools
import time

from .base import CREATED, EXITED, RUNNING, ContainerStatus, Runtime, RunContainerOptions

RUN_SECONDS = "kubemark.amd.com/run-seconds"
STOP_SECONDS = "kubemark.amd.com/stop-seconds"


class StubRuntime(Runtime):
    name = "stub"

    def __init__(self, payload=None, start_latency=0.0):
        super().__init__()
        self._ids = itertools.count(1)
        self.sandboxes: dict[str, dict] = {}
        self.containers: dict[str, ContainerStatus] = {}
        self.meta: dict[str, dict] = {}
        self.payload = payload
        self.start_latency = start_latency
        self.payload_runs = 0
        self.payload_failures = 0
        self._timers = {}
        self.exec_codes: dict[tuple, int] = {}

    async def run_pod_sandbox(self, pod, annotations):
        sid = f"sb-{next(self._ids)}"
        self.sandboxes[sid] = {"pod_uid": pod["metadata"]["uid"], "annotations": dict(annotations or {}),
                               "state": "SANDBOX_READY", "created": time.time()}
        return sid

    async def stop_pod_sandbox(self, sid):
        sb = self.sandboxes.get(sid)
        if sb:
            sb["state"] = "SANDBOX_NOTREADY"
            for cid, m in list(self.meta.items()):
                if m["sandbox"] == sid:
                    await self.stop_container(cid, 0)

    async def remove_pod_sandbox(self, sid):
        for cid, m in list(self.meta.items()):
            if m["sandbox"] == sid:
                await self.remove_container(cid)
        self.sandboxes.pop(sid, None)

    async def create_container(self, sid, pod, container, opts: RunContainerOptions):
        cid = f"stub://{next(self._ids)}"
        self.containers[cid] = ContainerStatus(cid, container["name"], CREATED, image=container.get("image", ""))
        run_s = None
        ann = (pod["metadata"].get("annotations") or {}).get(RUN_SECONDS)
        cmd = container.get("command") or []
        if ann is not None:
            run_s = float(ann)
        elif len(cmd) == 2 and cmd[0] == "sleep":
            run_s = float(cmd[1])
        stop_s = float((pod["metadata"].get("annotations") or {}).get(STOP_SECONDS) or 0)
        self.meta[cid] = {"sandbox": sid, "pod_uid": pod["metadata"]["uid"], "opts": opts, "run_s": run_s,
                          "container": container, "stop_s": stop_s,
                          "exec_code": (pod["metadata"].get("annotations") or {}).get("kubemark.amd.com/exec-exit-code", 0)}
        return cid

    async def start_container(self, cid):
        st = self.containers[cid]
        m = self.meta[cid]
        if self.start_latency:
            await asyncio.sleep(self.start_latency)
        st.state = RUNNING
        st.started_at = time.time()
        opts = m["opts"]
        if self.payload is not None and any("/dev/dri/" in d.get("pathOnHost", "") for d in opts.devices):
            self.payload_runs += 1
            ok = False
            try:
                res = self.payload(opts)
                if inspect.isawaitable(res):     # e.g. kubemark.payload.PayloadClient (another process)
                    res = await res
                ok = bool(res)
            except Exception as e:  # payload crash = container crash
                st.message = str(e)
            if not ok:
                self.payload_failures += 1
                self._exit(cid, 1, "Error")
                return
        if m["run_s"] is not None:
            loop = asyncio.get_event_loop()
            self._timers[cid] = loop.call_later(max(0.0, m["run_s"]), self._exit, cid, 0, "Completed")

    def _exit(self, cid, code, reason):
        st = self.containers.get(cid)
        if st is None or st.state == EXITED:
            return
        self._timers.pop(cid, None)
        st.state = EXITED
        st.exit_code = code
        st.reason = reason
        st.finished_at = time.time()
        self._fire_exit(self.meta[cid]["pod_uid"], cid)

    async def stop_container(self, cid, timeout):
        st = self.containers.get(cid)
        m = self.meta.get(cid) or {}
        stop_s = m.get("stop_s") or 0.0
        if st is not None and st.state != EXITED and timeout > 0 and stop_s > 0:
            # SIGTERM sent: the workload drains for stop_s, or is SIGKILLed at the grace period
            await asyncio.sleep(min(stop_s, timeout))
            killed = stop_s >= timeout
        else:
            killed = timeout == 0
        h = self._timers.pop(cid, None)
        if h:
            h.cancel()
        if st is not None and st.state != EXITED:
            st.state = EXITED
            st.exit_code = 137 if killed else 0
            st.reason = "Killed" if killed else "Completed"
            st.finished_at = time.time()

    async def remove_container(self, cid):
        await self.stop_container(cid, 0)
        self.containers.pop(cid, None)
        self.meta.pop(cid, None)

    def container_status(self, cid):
        return self.containers.get(cid)

    async def exec_sync(self, cid, cmd, timeout):
        """Fake exec: exit code from `exec_codes[(pod uid, container)]`, else the pod annotation
        `kubemark.amd.com/exec-exit-code`, else 0 (lets tests flip probe results)."""
        st, m = self.containers.get(cid), self.meta.get(cid)
        if st is None or st.state != RUNNING:
            return 126, b"container is not running"
        key = (m["pod_uid"], st.name)
        if key in self.exec_codes:
            return self.exec_codes[key], b""
        return int(m.get("exec_code", 0)), b""

    def list_containers(self):
        return list(self.containers.values())

    async def pod_states(self):
        out: dict = {}
        for sid, sb in self.sandboxes.items():
            out.setdefault(sb["pod_uid"], {"sandboxes": [], "containers": []})["sandboxes"].append(
                (sid, sb["state"] == "SANDBOX_READY", None))
        for cid, m in self.meta.items():
            st = self.containers.get(cid)
            if st is not None:
                out.setdefault(m["pod_uid"], {"sandboxes": [], "containers": []})["containers"].append(
                    (st.name, cid, getattr(m["opts"], "attempt", 0), st.created_at, m["sandbox"]))
        return out

    async def container_logs(self, cid, tail=None):
        st = self.containers.get(cid)
        return b"" if st is None else f"stub container {st.name} ({st.state})\n".encode()
