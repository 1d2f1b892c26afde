"""Container runtime interface used by the kubelet (the CRI's RuntimeService, in-process).

Parity: CRI `RuntimeService` (`pkg/kubelet/apis/cri/v1alpha1/runtime/api.proto:17-104`:
RunPodSandbox / StopPodSandbox / RemovePodSandbox / CreateContainer / StartContainer /
StopContainer / RemoveContainer / ContainerStatus / ListContainers) and
`kubecontainer.RunContainerOptions` (envs, devices, mounts, annotations from the device
manager, `pkg/kubelet/container/runtime.go`).
"""
from __future__ import annotations

import asyncio
import time
from dataclasses import dataclass, field

CREATED, RUNNING, EXITED, UNKNOWN = "CONTAINER_CREATED", "CONTAINER_RUNNING", "CONTAINER_EXITED", "CONTAINER_UNKNOWN"


@dataclass
class RunContainerOptions:
    envs: list = field(default_factory=list)          # [{"name","value"}]
    devices: list = field(default_factory=list)       # [{"pathOnHost","pathInContainer","permissions"}]
    mounts: list = field(default_factory=list)        # [{"containerPath","hostPath","readOnly"}]
    annotations: list = field(default_factory=list)   # [{"name","value"}]
    oom_score_adj: int | None = None                  # qos.oom_score_adj (CRI LinuxContainerResources)
    cgroup_parent: str | None = None                  # pod cgroup directory (cgroups.CgroupManager)
    attempt: int = 0                                  # restart count (CRI ContainerMetadata.attempt)
    run_as_user: int | None = None                    # securityContext.runAsUser (CRI LinuxContainerSecurityContext)
    run_as_group: int | None = None                   # securityContext.runAsGroup: the primary group
    supplemental_groups: list = field(default_factory=list)   # pod fsGroup + supplementalGroups
    privileged: bool = False                          # securityContext.privileged: host /dev, all caps
    cap_add: list = field(default_factory=list)       # securityContext.capabilities.add ("NET_ADMIN", ...)
    cap_drop: list = field(default_factory=list)
    readonly_rootfs: bool = False                     # securityContext.readOnlyRootFilesystem

    @classmethod
    def from_device_opts(cls, d):
        return cls(list(d.get("envs") or []), list(d.get("devices") or []), list(d.get("mounts") or []),
                   list(d.get("annotations") or []))

    def env_dict(self):
        return {e["name"]: e["value"] for e in self.envs}


@dataclass
class ContainerStatus:
    id: str
    name: str
    state: str = CREATED
    created_at: float = field(default_factory=time.time)
    started_at: float = 0.0
    finished_at: float = 0.0
    exit_code: int = 0
    reason: str = ""
    message: str = ""
    image: str = ""
    log_path: str = ""


class RuntimeError_(Exception):
    pass


class Runtime:
    """Base class. `on_exit(cb)` registers cb(pod_uid, container_id) for event-driven PLEG."""
    name = "base"

    def __init__(self):
        self._exit_cbs = []

    def on_exit(self, cb):
        self._exit_cbs.append(cb)

    def _fire_exit(self, pod_uid, cid):
        for cb in self._exit_cbs:
            cb(pod_uid, cid)

    async def version(self):
        return {"runtimeName": self.name, "runtimeVersion": "1.0", "runtimeApiVersion": "v1alpha1"}

    async def run_pod_sandbox(self, pod, annotations: dict) -> str:
        raise NotImplementedError

    async def stop_pod_sandbox(self, sandbox_id: str):
        raise NotImplementedError

    async def remove_pod_sandbox(self, sandbox_id: str):
        raise NotImplementedError

    async def create_container(self, sandbox_id: str, pod, container, opts: RunContainerOptions) -> str:
        raise NotImplementedError

    async def start_container(self, cid: str):
        raise NotImplementedError

    async def stop_container(self, cid: str, timeout: float):
        raise NotImplementedError

    async def remove_container(self, cid: str):
        raise NotImplementedError

    def container_status(self, cid: str) -> ContainerStatus | None:
        raise NotImplementedError

    async def container_logs(self, cid: str, tail: int | None = None) -> bytes:
        return b""

    async def exec_sync(self, cid: str, cmd: list, timeout: float) -> tuple:
        """CRI ExecSync: run cmd in the container's context; returns (exit code, output bytes)."""
        raise NotImplementedError(f"{self.name} runtime does not support exec")

    async def exec_interactive(self, cid: str, cmd: list, stdin, stdout, stderr, tty: bool, resize) -> int:
        """Streaming exec (`ExecInContainer`, `pkg/kubelet/server/remotecommand/exec.go:33`):
        stdin / resize are async iterators of bytes / (width, height) or None; stdout / stderr
        async callables or None. This default runs the command to completion through exec_sync
        (no stdin) and sends its combined output at the end; runtimes with real processes
        stream."""
        rc, out = await self.exec_sync(cid, cmd, 300)
        sink = stdout or stderr
        if sink is not None and out:
            await sink(out if isinstance(out, bytes) else str(out).encode())
        return rc

    async def attach(self, cid: str, stdin, stdout, stderr, tty: bool, resize) -> int:
        """Attach to a running container (`pkg/kubelet/server/remotecommand/attach.go`): the
        output it writes from now on, until it exits. This default follows container_logs."""
        sent = len(await self.container_logs(cid))
        sink = stdout or stderr
        while True:
            st = self.container_status(cid)
            data = await self.container_logs(cid)
            if sink is not None and len(data) > sent:
                await sink(data[sent:])
            sent = max(sent, len(data))
            if st is None or st.state != RUNNING:
                return 0 if st is None else int(st.exit_code or 0)
            await asyncio.sleep(0.1)

    def list_containers(self):
        return []

    def container_pids(self) -> dict:
        """{container id: host pid of its root process} for running containers (GPU process
        attribution in the summary API). Runtimes without host processes return {}."""
        return {}

    def isolation_status(self) -> dict | None:
        """Whether the runtime enforces a container's device view (mount namespace + private /dev
        + device cgroup): {"enforced": bool, "reason": str, "message": str}. None = not applicable
        (containers are not real processes, e.g. the kubemark stub runtime)."""
        return None

    async def pod_states(self) -> dict:
        """What survives a kubelet restart (kuberuntime `GetPods`): pod uid -> {"sandboxes":
        [(sandbox id, ready, ip or None)], "containers": [(container name, id, attempt, created_at,
        sandbox id)]}.
        The restarted kubelet adopts them instead of starting the pod again. Runtimes whose state
        does not outlive the kubelet return {}."""
        return {}
