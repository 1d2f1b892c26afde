"""Kubelet-side CRI client: the kubelet's Runtime interface implemented over gRPC, plus a
generic PLEG relist and the remote image service.

Parity: `pkg/kubelet/remote/remote_runtime.go:82-177` (RunPodSandbox, CreateContainer, ...
each with a per-call timeout), `remote_image.go` (ListImages/ImageStatus/PullImage/RemoveImage/
ImageFsInfo), `pkg/kubelet/kuberuntime/kuberuntime_sandbox.go:35-93` +
`kuberuntime_container.go:88-209` (sandbox / container configs: metadata, labels
`io.kubernetes.pod.*`, annotations incl. the device plugin's pod annotations, devices, mounts,
envs, log path) and `pkg/kubelet/pleg/generic.go:182-260` (relist every period, diff container
states, emit ContainerDied → the kubelet re-syncs the pod).

The kubelet reads container status synchronously (`container_status(cid)`), so this client keeps
a status cache refreshed by its own calls and by the relist; a RUNNING→EXITED transition seen by
the relist fires the runtime exit callbacks, exactly the events PLEG feeds the sync loop.
"""
from __future__ import annotations

import asyncio
import json
import logging
import time

import grpc

from ..deviceplugin.api import _Stub
from ..utils import grpclite
from ..kubelet.sysctl import SysctlAdmitHandler
from ..kubelet.runtime.base import CREATED, EXITED, RUNNING, UNKNOWN, ContainerStatus, Runtime, RuntimeError_
from . import api as A
from . import labels as L

log = logging.getLogger("cri.remote")

_STATES = {A.CONTAINER_CREATED: CREATED, A.CONTAINER_RUNNING: RUNNING, A.CONTAINER_EXITED: EXITED,
           A.CONTAINER_UNKNOWN: UNKNOWN}


_RPC_ERRORS = (grpc.aio.AioRpcError, grpclite.RpcError)


def _target(endpoint):
    if endpoint.startswith("unix://"):
        return endpoint
    if endpoint.startswith("/"):
        return "unix://" + endpoint
    return endpoint


class RemoteRuntime(Runtime):
    name = "remote"

    def __init__(self, endpoint: str, timeout: float = 10.0, relist_period: float = 1.0, transport: str = "lite"):
        super().__init__()
        self.endpoint = endpoint
        # "lite": gRPC over HTTP/2 on the kubelet's loop (utils/grpclite.py), the kubelet's
        # 1-s relist and every pod's sandbox/container calls; "grpc": grpc.aio
        self.transport = transport
        self.timeout = timeout
        self.relist_period = relist_period
        self.channel = None
        self.rs = None
        self.images = None
        self.cache: dict[str, ContainerStatus] = {}
        self.pod_of: dict[str, str] = {}       # cid -> pod uid
        self._relist_task = None
        self.relists = 0
        self.runtime_name = "remote"
        self._isolation = None

    def isolation_status(self):
        return self._isolation

    async def connect(self):
        if self.channel is None:
            self.channel = (grpclite.Channel(_target(self.endpoint)) if self.transport == "lite"
                            else grpc.aio.insecure_channel(_target(self.endpoint)))
            self.rs = _Stub(self.channel, A.RUNTIME_SERVICE, A.RUNTIME_METHODS)
            self.images = RemoteImageService(_Stub(self.channel, A.IMAGE_SERVICE, A.IMAGE_METHODS), self.timeout)
            v = await self.rs.Version(A.MSG["VersionRequest"](version="0.1.0"), timeout=self.timeout)
            self.runtime_name = v.runtime_name
            st = await self.rs.Status(A.MSG["StatusRequest"](), timeout=self.timeout)
            for c in st.status.conditions:
                if c.type == A.DEVICE_ISOLATION_CONDITION:
                    # the tier rides at the head of the message ("tier landlock (...)")
                    tier = c.message.split()[1] if c.message.startswith("tier ") else \
                        ("none" if not c.status else "namespaces")
                    self._isolation = {"enforced": c.status, "reason": c.reason, "message": c.message,
                                       "tier": tier.rstrip(":")}
            if self.relist_period and self._relist_task is None:
                self._relist_task = asyncio.ensure_future(self._relist_loop())
        return self

    async def close(self):
        if self._relist_task is not None:
            self._relist_task.cancel()
            self._relist_task = None
        if self.channel is not None:
            await self.channel.close()
            self.channel = None

    async def _call(self, name, req):
        if self.channel is None:
            await self.connect()
        try:
            return await getattr(self.rs, name)(req, timeout=self.timeout)
        except _RPC_ERRORS as e:
            raise RuntimeError_(f"{name}: {e.details() or e.code().name}") from None

    # ---------------------------------------------------------------- Runtime interface
    async def version(self):
        v = await self._call("Version", A.MSG["VersionRequest"](version="0.1.0"))
        return {"runtimeName": v.runtime_name, "runtimeVersion": v.runtime_version,
                "runtimeApiVersion": v.runtime_api_version}

    def _pod_labels(self, pod):
        return L.new_pod_labels(pod)

    def _sandbox_config(self, pod, annotations):
        md = pod["metadata"]
        ann = L.new_pod_annotations(pod)
        ann.update(annotations or {})
        ann[A.POD_SPEC_ANNOTATION] = json.dumps(pod, separators=(",", ":"))
        ports = [A.MSG["PortMapping"](protocol=A.UDP if p.get("protocol") == "UDP" else A.TCP,
                                      container_port=int(p.get("containerPort") or 0), host_port=int(p.get("hostPort") or 0))
                 for c in (pod.get("spec") or {}).get("containers") or () for p in c.get("ports") or () if p.get("hostPort")]
        return A.MSG["PodSandboxConfig"](
            metadata=A.MSG["PodSandboxMetadata"](name=md.get("name", ""), uid=md.get("uid", ""),
                                                 namespace=md.get("namespace", ""), attempt=0),
            hostname=(pod.get("spec") or {}).get("hostname") or md.get("name", ""),
            log_directory=f"/var/log/pods/{md.get('uid', '')}", port_mappings=ports,
            labels=self._pod_labels(pod), annotations=ann,
            linux=A.MSG["LinuxPodSandboxConfig"](sysctls=SysctlAdmitHandler.pod_sysctls(pod)))

    async def run_pod_sandbox(self, pod, annotations):
        r = await self._call("RunPodSandbox", A.MSG["RunPodSandboxRequest"](config=self._sandbox_config(pod, annotations)))
        return r.pod_sandbox_id

    async def stop_pod_sandbox(self, sid):
        await self._call("StopPodSandbox", A.MSG["StopPodSandboxRequest"](pod_sandbox_id=sid))
        now = time.time()
        for cid, st in self.cache.items():
            if getattr(st, "_sandbox", None) == sid and st.state != EXITED:
                st.state, st.finished_at = EXITED, now

    async def remove_pod_sandbox(self, sid):
        await self._call("RemovePodSandbox", A.MSG["RemovePodSandboxRequest"](pod_sandbox_id=sid))
        for cid in [c for c, st in self.cache.items() if getattr(st, "_sandbox", None) == sid]:
            self.cache.pop(cid, None)
            self.pod_of.pop(cid, None)

    async def create_container(self, sid, pod, container, opts):
        md = pod["metadata"]
        envs = [A.MSG["KeyValue"](key=e["name"], value=str(e["value"])) for e in container.get("env") or () if "value" in e]
        envs += [A.MSG["KeyValue"](key=e["name"], value=str(e["value"])) for e in opts.envs]
        ann = L.new_container_annotations(container, pod, int(opts.attempt or 0), opts.annotations)
        ann[A.CONTAINER_SPEC_ANNOTATION] = json.dumps(container, separators=(",", ":"))
        if opts.cgroup_parent:
            ann[A.CGROUP_PARENT_ANNOTATION] = opts.cgroup_parent
        if opts.run_as_group is not None:
            ann[A.RUN_AS_GROUP_ANNOTATION] = str(int(opts.run_as_group))
        labels = L.new_container_labels(container, pod)
        cfg = A.MSG["ContainerConfig"](
            metadata=A.MSG["ContainerMetadata"](name=container["name"], attempt=int(opts.attempt or 0)),
            image=A.MSG["ImageSpec"](image=container.get("image", "")),
            command=list(container.get("command") or []), args=list(container.get("args") or []),
            working_dir=container.get("workingDir") or "", envs=envs,
            mounts=[A.MSG["Mount"](container_path=m.get("containerPath", ""), host_path=m.get("hostPath", ""),
                                   readonly=bool(m.get("readOnly"))) for m in opts.mounts],
            devices=[A.MSG["Device"](container_path=d.get("pathInContainer", ""), host_path=d.get("pathOnHost", ""),
                                     permissions=d.get("permissions", "rwm")) for d in opts.devices],
            labels=labels, annotations=ann, log_path=L.container_log_path(container["name"], opts.attempt or 0),
            linux=A.MSG["LinuxContainerConfig"](
                resources=A.MSG["LinuxContainerResources"](oom_score_adj=opts.oom_score_adj or 0),
                security_context=A.MSG["LinuxContainerSecurityContext"](
                    # securityContext.runAsUser; the pod's fsGroup + supplementalGroups as supplemental groups
                    run_as_user=(A.MSG["Int64Value"](value=opts.run_as_user) if opts.run_as_user is not None else None),
                    supplemental_groups=list(opts.supplemental_groups), privileged=bool(opts.privileged),
                    readonly_rootfs=bool(opts.readonly_rootfs),
                    capabilities=(A.MSG["Capability"](add_capabilities=list(opts.cap_add), drop_capabilities=list(opts.cap_drop))
                                  if opts.cap_add or opts.cap_drop else None))))
        r = await self._call("CreateContainer", A.MSG["CreateContainerRequest"](
            pod_sandbox_id=sid, config=cfg, sandbox_config=self._sandbox_config(pod, {})))
        st = ContainerStatus(r.container_id, container["name"], CREATED, image=container.get("image", ""))
        st._sandbox = sid
        self.cache[r.container_id] = st
        self.pod_of[r.container_id] = md.get("uid", "")
        return r.container_id

    async def start_container(self, cid):
        await self._call("StartContainer", A.MSG["StartContainerRequest"](container_id=cid))
        await self._refresh(cid)

    async def stop_container(self, cid, timeout):
        await self._call("StopContainer", A.MSG["StopContainerRequest"](container_id=cid, timeout=int(timeout)))
        await self._refresh(cid)

    async def remove_container(self, cid):
        await self._call("RemoveContainer", A.MSG["RemoveContainerRequest"](container_id=cid))
        self.cache.pop(cid, None)
        self.pod_of.pop(cid, None)

    def container_status(self, cid):
        return self.cache.get(cid)

    async def _refresh(self, cid):
        try:
            r = await self.rs.ContainerStatus(A.MSG["ContainerStatusRequest"](container_id=cid), timeout=self.timeout)
        except _RPC_ERRORS:
            return None
        return self._apply(r.status)

    def _apply(self, s):
        st = self.cache.get(s.id)
        if st is None:
            return None
        prev = st.state
        st.state = _STATES.get(s.state, UNKNOWN)
        st.created_at = s.created_at / 1e9 if s.created_at else st.created_at
        st.started_at = s.started_at / 1e9 if s.started_at else st.started_at
        st.finished_at = s.finished_at / 1e9 if s.finished_at else st.finished_at
        st.exit_code, st.reason, st.message = s.exit_code, s.reason, s.message
        st.log_path = s.log_path or st.log_path
        if prev != EXITED and st.state == EXITED:
            self._fire_exit(self.pod_of.get(s.id, ""), s.id)
        return st

    async def relist(self):
        """One PLEG relist: ListContainers, then ContainerStatus for every container whose
        state changed since the last relist."""
        self.relists += 1
        r = await self._call("ListContainers", A.MSG["ListContainersRequest"]())
        for c in r.containers:
            st = self.cache.get(c.id)
            if st is not None and _STATES.get(c.state, UNKNOWN) != st.state:
                await self._refresh(c.id)

    async def _relist_loop(self):
        while True:
            await asyncio.sleep(self.relist_period)
            try:
                await self.relist()
            except asyncio.CancelledError:
                raise
            except Exception as e:   # runtime down: keep trying (PLEG Healthy() turns false)
                log.debug("relist failed: %s", e)

    async def exec_sync(self, cid, cmd, timeout):
        r = await self._call("ExecSync", A.MSG["ExecSyncRequest"](container_id=cid, cmd=list(cmd), timeout=int(max(1, timeout))))
        return r.exit_code, bytes(r.stdout) + bytes(r.stderr)

    async def exec_url(self, cid, cmd, tty=False, stdin=False, stdout=True, stderr=None):
        r = await self._call("Exec", A.MSG["ExecRequest"](container_id=cid, cmd=list(cmd), tty=tty, stdin=stdin,
                                                         stdout=stdout, stderr=(not tty) if stderr is None else stderr))
        return r.url

    async def attach_url(self, cid, tty=False, stdin=False, stdout=True, stderr=None):
        r = await self._call("Attach", A.MSG["AttachRequest"](container_id=cid, tty=tty, stdin=stdin, stdout=stdout,
                                                             stderr=(not tty) if stderr is None else stderr))
        return r.url

    async def port_forward_url(self, sid, ports):
        r = await self._call("PortForward", A.MSG["PortForwardRequest"](pod_sandbox_id=sid, port=list(ports)))
        return r.url

    def list_containers(self):
        return list(self.cache.values())

    async def pod_states(self):
        """ListPodSandbox + ListContainers of the runtime, grouped by the pod-uid label; every
        listed container enters this client's status cache (so the restarted kubelet's PLEG
        tracks the adopted containers too)."""
        out: dict = {}
        sbs = await self._call("ListPodSandbox", A.MSG["ListPodSandboxRequest"]())
        for sb in sbs.items:
            uid = sb.labels.get(A.POD_UID, "") or sb.metadata.uid
            ip = None
            try:
                st = await self._call("PodSandboxStatus", A.MSG["PodSandboxStatusRequest"](pod_sandbox_id=sb.id))
                ip = st.status.network.ip or None
            except Exception:  # noqa: BLE001 - the sandbox may be going away
                pass
            out.setdefault(uid, {"sandboxes": [], "containers": []})["sandboxes"].append(
                (sb.id, sb.state == A.SANDBOX_READY, ip))
        cs = await self._call("ListContainers", A.MSG["ListContainersRequest"]())
        for c in cs.containers:
            uid = c.labels.get(A.POD_UID, "")
            name = c.labels.get(A.CONTAINER_NAME, "") or c.metadata.name
            if c.id not in self.cache:
                st = ContainerStatus(c.id, name, _STATES.get(c.state, UNKNOWN), image=c.image.image)
                st._sandbox = c.pod_sandbox_id
                self.cache[c.id] = st
                self.pod_of[c.id] = uid
                await self._refresh(c.id)
            out.setdefault(uid, {"sandboxes": [], "containers": []})["containers"].append(
                (name, c.id, c.metadata.attempt, c.created_at / 1e9 if c.created_at else 0.0, c.pod_sandbox_id))
        return out

    def log_path(self, cid):
        st = self.cache.get(cid)
        return (st.log_path or None) if st is not None else None

    async def container_logs(self, cid, tail=None):
        st = self.cache.get(cid)
        if st is None or not st.log_path:
            return b""
        try:
            with open(st.log_path, "rb") as f:
                data = f.read()
        except OSError:
            return b""
        if tail:
            data = b"\n".join(data.splitlines()[-tail:]) + b"\n"
        return data

    async def status(self):
        r = await self._call("Status", A.MSG["StatusRequest"]())
        return {c.type: c.status for c in r.status.conditions}

    async def container_stats(self):
        r = await self._call("ListContainerStats", A.MSG["ListContainerStatsRequest"]())
        return {s.attributes.id: {"cpu_ns": s.cpu.usage_core_nano_seconds.value,
                                  "working_set_bytes": s.memory.working_set_bytes.value} for s in r.stats}


class RemoteImageService:
    def __init__(self, stub, timeout):
        self.stub = stub
        self.timeout = timeout

    async def _call(self, name, req):
        try:
            return await getattr(self.stub, name)(req, timeout=self.timeout)
        except _RPC_ERRORS as e:
            raise RuntimeError_(f"{name}: {e.details() or e.code().name}") from None

    async def pull_image(self, image, auth=None):
        req = A.MSG["PullImageRequest"](image=A.MSG["ImageSpec"](image=image))
        if auth is not None:
            req.auth.CopyFrom(A.MSG["AuthConfig"](username=auth.username, password=auth.password,
                                                  identity_token=auth.identity_token,
                                                  registry_token=auth.registry_token))
        return (await self._call("PullImage", req)).image_ref

    async def image_status(self, image):
        r = await self._call("ImageStatus", A.MSG["ImageStatusRequest"](image=A.MSG["ImageSpec"](image=image)))
        if not r.HasField("image"):
            return None
        return {"id": r.image.id, "repoTags": list(r.image.repo_tags), "repoDigests": list(r.image.repo_digests),
                "size": r.image.size}

    async def list_images(self):
        r = await self._call("ListImages", A.MSG["ListImagesRequest"]())
        return [{"id": i.id, "repoTags": list(i.repo_tags), "size": i.size} for i in r.images]

    async def remove_image(self, image):
        await self._call("RemoveImage", A.MSG["RemoveImageRequest"](image=A.MSG["ImageSpec"](image=image)))

    async def image_fs_info(self):
        r = await self._call("ImageFsInfo", A.MSG["ImageFsInfoRequest"]())
        fs = r.image_filesystems[0] if r.image_filesystems else None
        return {"usedBytes": fs.used_bytes.value if fs else 0, "inodesUsed": fs.inodes_used.value if fs else 0}
