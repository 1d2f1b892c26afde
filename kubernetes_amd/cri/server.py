"""CRI gRPC server: RuntimeService + ImageService over a unix socket, backed by an in-process
runtime (process / stub), plus the streaming server that Exec / Attach / PortForward URLs
point at.

Parity: the dockershim's CRI endpoint (`pkg/kubelet/dockershim/remote/docker_server.go`,
`docker_service.go`), sandbox + container bookkeeping with labels/annotations and filters
(`docker_sandbox.go:78`, `docker_container.go:88-400`), `ExecSync` (`exec.go`), the streaming
server (`pkg/kubelet/server/streaming/server.go`: GetExec/GetAttach/GetPortForward hand out
single-use token URLs), image service (`docker_image.go`), `Status` runtime/network
conditions (`docker_service.go:Status`).

Streaming protocols: WebSocket with the Kubernetes channel sub-protocols (`channel.k8s.io`,
`v4.channel.k8s.io`, base64 variants; `cri/remotecommand.py`) on every token URL, and a framed
fallback for clients without WebSocket:
  exec/attach  GET /exec/<token>  -> chunked body of frames: 1 byte stream id (1 stdout,
               2 stderr, 3 exit status as ASCII) + payload
  portforward  GET /portforward/<token>?port=N with `Connection: Upgrade`, `Upgrade: tcp`
               -> `101 Switching Protocols`, then the connection is a raw byte tunnel to
               the container port (pods share the host network namespace in this runtime).
"""
from __future__ import annotations

import asyncio
import hashlib
import json
import logging
import os
import secrets
import time

import grpc

from ..deviceplugin.api import generic_handler
from ..utils import grpclite
from ..kubelet.runtime.base import EXITED, RUNNING, RunContainerOptions, RuntimeError_
from ..utils.websocket import is_websocket_request
from . import api as A

log = logging.getLogger("cri.server")

STUB_IMAGE_SIZE = 4 << 20


def _ns(t):
    return int((t or 0) * 1e9)


class ImageStore:
    """Local image store. `resolver(image) -> size or None` decides what can be "pulled"
    (there is no registry access: the process runtime resolves well-known images to built
    native binaries; the stub runtime accepts any image like kubemark's fake docker)."""

    def __init__(self, resolver):
        self.resolver = resolver
        self.images: dict[str, dict] = {}     # id -> {id, repo_tags, size}
        self.by_tag: dict[str, str] = {}      # normalized tag -> id

    @staticmethod
    def normalize(ref):
        ref = ref.split("@")[0]
        last = ref.rsplit("/", 1)[-1]
        return ref if ":" in last else ref + ":latest"

    def _find(self, ref):
        iid = self.by_tag.get(self.normalize(ref)) or (ref if ref in self.images else None)
        return self.images.get(iid) if iid else None

    def pull(self, ref):
        img = self._find(ref)
        if img is not None:
            return img["id"]
        size = self.resolver(ref)
        if size is None:
            raise LookupError(f"pull access denied for {ref}: image not found (no registry access)")
        tag = self.normalize(ref)
        iid = "sha256:" + hashlib.sha256(tag.encode()).hexdigest()
        self.images[iid] = {"id": iid, "repo_tags": [tag], "size": int(size)}
        self.by_tag[tag] = iid
        return iid

    def status(self, ref):
        return self._find(ref)

    def remove(self, ref):
        img = self._find(ref)
        if img is not None:
            self.images.pop(img["id"], None)
            for t in img["repo_tags"]:
                self.by_tag.pop(t, None)

    def used_bytes(self):
        return sum(i["size"] for i in self.images.values())


def LocalImageService(store: ImageStore):
    """The CRI image-service API over built-in images only (in-process runtimes without an OCI
    store); see `images.service.ImageService`."""
    from ..images.service import ImageService
    return ImageService(builtins=store)


def process_image_resolver(ref):
    from ..kubelet.runtime.process import builtin_argv
    base = ImageStore.normalize(ref).rsplit(":", 1)[0]
    argv = builtin_argv(base)
    if not argv:
        return None
    try:
        return os.path.getsize(argv[0])
    except OSError:
        return None


def stub_image_resolver(ref):
    return STUB_IMAGE_SIZE


def host_image_resolver(ref):
    """Process runtime: well-known images resolve to built binaries; any other image runs its
    command on the host root filesystem, which acts as an always-present image of size 0."""
    size = process_image_resolver(ref)
    return 0 if size is None else size


class StreamingServer:
    """Single-use token URLs for exec / attach / port-forward (streaming/server.go)."""

    TOKEN_TTL = 60.0

    def __init__(self, runtime, host="127.0.0.1"):
        self.runtime = runtime
        self.host = host
        self.port = None
        self.server = None
        self.tokens: dict[str, tuple] = {}

    async def start(self):
        self.server = await asyncio.start_server(self._conn, self.host, 0)
        self.port = self.server.sockets[0].getsockname()[1]
        return self

    async def stop(self):
        if self.server is not None:
            self.server.close()
            await self.server.wait_closed()

    def url(self, kind, req):
        tok = secrets.token_urlsafe(12)
        self.tokens[tok] = (kind, req, time.monotonic())
        return f"http://{self.host}:{self.port}/{kind}/{tok}"

    def _take(self, tok):
        t = self.tokens.pop(tok, None)
        if t is None or time.monotonic() - t[2] > self.TOKEN_TTL:
            return None
        return t

    async def _conn(self, reader, writer):
        try:
            head = await reader.readuntil(b"\r\n\r\n")
            line = head.split(b"\r\n", 1)[0].decode()
            _, target, _ = line.split(" ", 2)
            path, _, qs = target.partition("?")
            q = dict(p.split("=", 1) for p in qs.split("&") if "=" in p)
            parts = path.strip("/").split("/")
            t = self._take(parts[1]) if len(parts) == 2 else None
            if t is None or t[0] != parts[0]:
                writer.write(b"HTTP/1.1 404 Not Found\r\nContent-Length: 0\r\n\r\n")
                return
            kind, req, _ = t
            headers = {}
            for ln in head.decode("latin-1").split("\r\n")[1:]:
                k, _, v = ln.partition(":")
                k = k.strip().lower()
                if k:
                    headers[k] = headers[k] + ", " + v.strip() if k in headers else v.strip()
            from .remotecommand import is_spdy_request
            if is_websocket_request(headers):
                await self._websocket(kind, req, q, headers, reader, writer)
            elif is_spdy_request(headers):
                await self._spdy(kind, req, headers, reader, writer)
            elif kind in ("exec", "attach"):
                await self._exec(kind, req, writer)
            elif kind == "portforward":
                await self._portforward(req, int(q.get("port") or (req.port[0] if req.port else 0)), reader, writer)
        except (asyncio.IncompleteReadError, ConnectionError, ValueError):
            pass
        finally:
            try:
                writer.close()
            except Exception:
                pass

    async def _websocket(self, kind, req, q, headers, reader, writer):
        """The Kubernetes WebSocket channel protocols on a token URL (`cri/remotecommand.py`);
        stream options come from the CRI request the token was issued for."""
        from . import remotecommand as rcm
        if kind == "portforward":
            ports = [int(p) for p in (q.get("ports") or q.get("port") or "").split(",") if p] or list(req.port)
            conn = await rcm.accept_raw(reader, writer, headers, rcm.PORTFORWARD_PROTOCOLS)
            if conn is not None:
                await rcm.serve_portforward(conn, ports, lambda port: asyncio.open_connection("127.0.0.1", port))
            return
        conn = await rcm.accept_raw(reader, writer, headers, rcm.EXEC_PROTOCOLS)
        if conn is None:
            return
        opts = rcm.Options(bool(req.stdin), bool(req.stdout), bool(req.stderr), bool(req.tty))
        rt, cid = self.runtime, req.container_id
        if kind == "exec":
            cmd = list(req.cmd)

            async def run(stdin, stdout, stderr, tty, resize):
                return await rt.exec_interactive(cid, cmd, stdin, stdout, stderr, tty, resize)
        else:
            async def run(stdin, stdout, stderr, tty, resize):
                return await rt.attach(cid, stdin, stdout, stderr, tty, resize)
        await rcm.serve_exec(conn, opts, run)

    async def _spdy(self, kind, req, headers, reader, writer):
        from . import remotecommand as rcm
        if kind == "portforward":
            if await rcm.accept_raw_spdy(writer, headers, (rcm.SPDY_PORTFORWARD_PROTOCOL,)) is not None:
                await rcm.serve_spdy_portforward(reader, writer, lambda port: asyncio.open_connection("127.0.0.1", port))
            return
        proto = await rcm.accept_raw_spdy(writer, headers, rcm.SPDY_EXEC_PROTOCOLS)
        if proto is None:
            return
        opts = rcm.Options(bool(req.stdin), bool(req.stdout), bool(req.stderr), bool(req.tty))
        rt, cid = self.runtime, req.container_id
        if kind == "exec":
            cmd = list(req.cmd)

            async def run(stdin, stdout, stderr, tty, resize):
                return await rt.exec_interactive(cid, cmd, stdin, stdout, stderr, tty, resize)
        else:
            async def run(stdin, stdout, stderr, tty, resize):
                return await rt.attach(cid, stdin, stdout, stderr, tty, resize)
        await rcm.serve_spdy_exec(reader, writer, proto or "channel.k8s.io", opts, run)

    async def _exec(self, kind, req, writer):
        writer.write(b"HTTP/1.1 200 OK\r\nContent-Type: application/vnd.kamd.stream\r\nTransfer-Encoding: chunked\r\n\r\n")

        def frame(ch, data):
            payload = bytes([ch]) + data
            writer.write(b"%x\r\n%s\r\n" % (len(payload), payload))
        if kind == "exec":
            rc, out = await self.runtime.exec_sync(req.container_id, list(req.cmd), 300)
        else:
            rc, out = 0, await self.runtime.container_logs(req.container_id)
        if out:
            frame(1, out if isinstance(out, bytes) else str(out).encode())
        frame(3, str(rc).encode())
        writer.write(b"0\r\n\r\n")
        await writer.drain()

    async def _portforward(self, req, port, reader, writer):
        try:
            ur, uw = await asyncio.open_connection("127.0.0.1", port)
        except OSError as e:
            msg = f"unable to do port forwarding: {e}".encode()
            writer.write(b"HTTP/1.1 502 Bad Gateway\r\nContent-Length: %d\r\n\r\n%s" % (len(msg), msg))
            return
        writer.write(b"HTTP/1.1 101 Switching Protocols\r\nConnection: Upgrade\r\nUpgrade: tcp\r\n\r\n")
        await writer.drain()
        await splice(reader, writer, ur, uw)


async def splice(r1, w1, r2, w2):
    async def pipe(r, w):
        try:
            while True:
                d = await r.read(65536)
                if not d:
                    break
                w.write(d)
                await w.drain()
        except (ConnectionError, asyncio.CancelledError):
            pass
        finally:
            try:
                w.write_eof()
            except (OSError, RuntimeError, AttributeError):
                pass
    await asyncio.gather(pipe(r1, w2), pipe(r2, w1))
    for w in (w1, w2):
        try:
            w.close()
        except Exception:
            pass


def _ck_key(sid):
    return sid.replace("://", "_").replace("/", "_")


def _pairs(d):
    return {k: v for k, v in (d or {}).items()}


class CRIServer:
    """Serves RuntimeService + ImageService for `runtime` on `socket_path`."""

    def __init__(self, runtime, socket_path, image_resolver=None, checkpoint_dir=None, transport="lite"):
        self.rt = runtime
        self.path = socket_path
        self.transport = transport
        self.checkpoints = None
        if checkpoint_dir:
            from ..utils.checkpoint import CheckpointManager
            self.checkpoints = CheckpointManager(checkpoint_dir)
        # the runtime's own image service (OCI store + registry) when it has one, else built-ins
        from ..images.service import ImageService
        svc = getattr(runtime, "images", None)
        self.images = svc if isinstance(svc, ImageService) else ImageService(builtins=ImageStore(
            image_resolver or (stub_image_resolver if runtime.name == "stub" else host_image_resolver)))
        self.sandboxes: dict[str, dict] = {}
        self.cmeta: dict[str, dict] = {}
        self.streaming = StreamingServer(runtime)
        self.server = None
        self.pod_cidr = ""

    def _restore_checkpoints(self):
        """Sandboxes checkpointed by a previous run come back NOTREADY (their processes are gone),
        so the kubelet sees them, tears their network down and removes them
        (`docker_sandbox.go` ListPodSandbox over checkpoints)."""
        if self.checkpoints is None:
            return
        for sid, ck in self.checkpoints.load_all():
            if sid in self.sandboxes:
                continue
            md = A.MSG["PodSandboxMetadata"](name=ck.get("name", ""), namespace=ck.get("namespace", ""),
                                             uid=ck.get("uid", ""), attempt=0)
            self.sandboxes[sid] = {"pod": {"metadata": {"name": ck.get("name"), "namespace": ck.get("namespace"),
                                                        "uid": ck.get("uid")}, "spec": {}},
                                   "metadata": md, "labels": ck.get("labels") or {}, "annotations": {},
                                   "created": ck.get("created", 0.0), "state": A.SANDBOX_NOTREADY,
                                   "ip": (ck.get("data") or {}).get("ip", ""), "restored": True}

    async def start(self):
        if os.path.exists(self.path):
            os.unlink(self.path)
        self._restore_checkpoints()
        if hasattr(self.rt, "start"):
            await self.rt.start()          # watch the containers re-adopted after a restart
        await self.streaming.start()
        if self.transport == "grpc":
            self.server = grpc.aio.server()
            self.server.add_generic_rpc_handlers((generic_handler(A.RUNTIME_SERVICE, A.RUNTIME_METHODS, self),
                                                  generic_handler(A.IMAGE_SERVICE, A.IMAGE_METHODS, self)))
        else:       # utils/grpclite.py: same wire protocol, served on the event loop
            self.server = grpclite.Server()
            self.server.add_service(A.RUNTIME_SERVICE, A.RUNTIME_METHODS, self)
            self.server.add_service(A.IMAGE_SERVICE, A.IMAGE_METHODS, self)
        self.server.add_insecure_port("unix://" + self.path)
        await self.server.start()
        return self

    async def stop(self):
        if self.server is not None:
            await self.server.stop(0)
        await self.streaming.stop()

    # ---------------------------------------------------------------- runtime service
    async def Version(self, req, ctx):
        v = await self.rt.version()
        return A.MSG["VersionResponse"](version="0.1.0", runtime_name=f"kamd-{v['runtimeName']}",
                                        runtime_version=v.get("runtimeVersion", "1.0"), runtime_api_version="v1alpha1")

    async def RunPodSandbox(self, req, ctx):
        c = req.config
        ann = _pairs(c.annotations)
        spec = ann.pop(A.POD_SPEC_ANNOTATION, None)
        pod = json.loads(spec) if spec else {
            "metadata": {"name": c.metadata.name, "namespace": c.metadata.namespace, "uid": c.metadata.uid,
                         "labels": _pairs(c.labels)}, "spec": {}}
        sid = await self.rt.run_pod_sandbox(pod, ann)
        self.sandboxes[sid] = {"pod": pod, "metadata": c.metadata, "labels": _pairs(c.labels), "annotations": ann,
                               "created": time.time(), "state": A.SANDBOX_READY, "ip": ann.get("kubernetes-amd.io/pod-ip", "")}
        if self.checkpoints is not None:
            ports = [{"protocol": pm.protocol, "container_port": pm.container_port, "host_port": pm.host_port}
                     for pm in c.port_mappings]
            self.checkpoints.create(_ck_key(sid), {
                "version": "v1", "name": c.metadata.name, "namespace": c.metadata.namespace, "uid": c.metadata.uid,
                "labels": _pairs(c.labels), "created": self.sandboxes[sid]["created"],
                "data": {"port_mappings": ports, "host_network": bool((pod.get("spec") or {}).get("hostNetwork")),
                         "ip": self.sandboxes[sid]["ip"]}})
        return A.MSG["RunPodSandboxResponse"](pod_sandbox_id=sid)

    def _sandbox(self, sid, ctx=None):
        sb = self.sandboxes.get(sid)
        if sb is None:
            raise KeyError(f"sandbox {sid} not found")
        return sb

    async def StopPodSandbox(self, req, ctx):
        sb = self.sandboxes.get(req.pod_sandbox_id)
        if sb is not None and not sb.get("restored"):
            await self.rt.stop_pod_sandbox(req.pod_sandbox_id)
            sb["state"] = A.SANDBOX_NOTREADY
        return A.MSG["StopPodSandboxResponse"]()

    async def RemovePodSandbox(self, req, ctx):
        if self.checkpoints is not None:
            self.checkpoints.remove(_ck_key(req.pod_sandbox_id))
        if req.pod_sandbox_id in self.sandboxes:
            if not self.sandboxes[req.pod_sandbox_id].get("restored"):
                await self.rt.remove_pod_sandbox(req.pod_sandbox_id)
            self.sandboxes.pop(req.pod_sandbox_id, None)
            for cid in [k for k, m in self.cmeta.items() if m["sandbox"] == req.pod_sandbox_id]:
                self.cmeta.pop(cid, None)
        return A.MSG["RemovePodSandboxResponse"]()

    def _sb_status(self, sid, sb):
        return A.MSG["PodSandboxStatus"](id=sid, metadata=sb["metadata"], state=sb["state"], created_at=_ns(sb["created"]),
                                         network=A.MSG["PodSandboxNetworkStatus"](ip=sb["ip"]),
                                         labels=sb["labels"], annotations=sb["annotations"])

    async def PodSandboxStatus(self, req, ctx):
        sb = self.sandboxes.get(req.pod_sandbox_id)
        if sb is None:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, f"sandbox {req.pod_sandbox_id} not found")
        return A.MSG["PodSandboxStatusResponse"](status=self._sb_status(req.pod_sandbox_id, sb))

    async def ListPodSandbox(self, req, ctx):
        flt = req.filter if req.HasField("filter") else None
        items = []
        for sid, sb in self.sandboxes.items():
            if flt is not None:
                if flt.id and flt.id != sid:
                    continue
                if flt.HasField("state") and flt.state.state != sb["state"]:
                    continue
                if any(sb["labels"].get(k) != v for k, v in flt.label_selector.items()):
                    continue
            items.append(A.MSG["PodSandbox"](id=sid, metadata=sb["metadata"], state=sb["state"], created_at=_ns(sb["created"]),
                                             labels=sb["labels"], annotations=sb["annotations"]))
        return A.MSG["ListPodSandboxResponse"](items=items)

    async def CreateContainer(self, req, ctx):
        sb = self.sandboxes.get(req.pod_sandbox_id)
        if sb is None:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, f"sandbox {req.pod_sandbox_id} not found")
        c = req.config
        ann = _pairs(c.annotations)
        cspec = ann.pop(A.CONTAINER_SPEC_ANNOTATION, None)
        container = json.loads(cspec) if cspec else {
            "name": c.metadata.name, "image": c.image.image, "command": list(c.command), "args": list(c.args),
            "workingDir": c.working_dir or None}
        devices = [{"pathOnHost": d.host_path, "pathInContainer": d.container_path, "permissions": d.permissions}
                   for d in c.devices]
        mounts = [{"containerPath": m.container_path, "hostPath": m.host_path, "readOnly": m.readonly} for m in c.mounts]
        if cspec:
            # the container spec carries its own env; the rest came from the device manager / volumes
            own = {e["name"] for e in container.get("env") or () if "value" in e}
            envs = [{"name": kv.key, "value": kv.value} for kv in c.envs if kv.key not in own]
        else:
            container["env"] = [{"name": kv.key, "value": kv.value} for kv in c.envs]
            envs = []
        res = c.linux.resources if c.HasField("linux") else None
        sc = c.linux.security_context if c.HasField("linux") and c.linux.HasField("security_context") else None
        opts = RunContainerOptions(envs=envs, devices=devices, mounts=mounts,
                                   annotations=[{"name": k, "value": v} for k, v in ann.items()],
                                   oom_score_adj=(res.oom_score_adj if res is not None and res.oom_score_adj else None),
                                   cgroup_parent=ann.get(A.CGROUP_PARENT_ANNOTATION),
                                   run_as_user=(sc.run_as_user.value if sc is not None and sc.HasField("run_as_user") else None),
                                   run_as_group=(int(ann[A.RUN_AS_GROUP_ANNOTATION]) if A.RUN_AS_GROUP_ANNOTATION in ann else None),
                                   supplemental_groups=list(sc.supplemental_groups) if sc is not None else [],
                                   privileged=bool(sc is not None and sc.privileged),
                                   cap_add=list(sc.capabilities.add_capabilities) if sc is not None and sc.HasField("capabilities") else [],
                                   cap_drop=list(sc.capabilities.drop_capabilities) if sc is not None and sc.HasField("capabilities") else [],
                                   readonly_rootfs=bool(sc is not None and sc.readonly_rootfs))
        try:
            cid = await self.rt.create_container(req.pod_sandbox_id, sb["pod"], container, opts)
        except (FileNotFoundError, OSError, ValueError) as e:
            await ctx.abort(grpc.StatusCode.UNKNOWN, str(e))
        self.cmeta[cid] = {"sandbox": req.pod_sandbox_id, "metadata": c.metadata, "image": c.image.image,
                           "labels": _pairs(c.labels), "annotations": ann, "created": time.time()}
        return A.MSG["CreateContainerResponse"](container_id=cid)

    async def StartContainer(self, req, ctx):
        try:
            await self.rt.start_container(req.container_id)
        except KeyError:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, f"container {req.container_id} not found")
        except OSError as e:
            await ctx.abort(grpc.StatusCode.UNKNOWN, f"failed to start container: {e}")
        return A.MSG["StartContainerResponse"]()

    async def StopContainer(self, req, ctx):
        await self.rt.stop_container(req.container_id, float(req.timeout))
        return A.MSG["StopContainerResponse"]()

    async def RemoveContainer(self, req, ctx):
        await self.rt.remove_container(req.container_id)
        self.cmeta.pop(req.container_id, None)
        return A.MSG["RemoveContainerResponse"]()

    def _state(self, st):
        return {"CONTAINER_CREATED": A.CONTAINER_CREATED, "CONTAINER_RUNNING": A.CONTAINER_RUNNING,
                "CONTAINER_EXITED": A.CONTAINER_EXITED}.get(st.state, A.CONTAINER_UNKNOWN)

    async def ListContainers(self, req, ctx):
        flt = req.filter if req.HasField("filter") else None
        out = []
        for st in self.rt.list_containers():
            m = self.cmeta.get(st.id)
            if m is None:
                continue
            state = self._state(st)
            if flt is not None:
                if flt.id and flt.id != st.id:
                    continue
                if flt.pod_sandbox_id and flt.pod_sandbox_id != m["sandbox"]:
                    continue
                if flt.HasField("state") and flt.state.state != state:
                    continue
                if any(m["labels"].get(k) != v for k, v in flt.label_selector.items()):
                    continue
            out.append(A.MSG["Container"](id=st.id, pod_sandbox_id=m["sandbox"], metadata=m["metadata"],
                                          image=A.MSG["ImageSpec"](image=m["image"]), image_ref=m["image"], state=state,
                                          created_at=_ns(m["created"]), labels=m["labels"], annotations=m["annotations"]))
        return A.MSG["ListContainersResponse"](containers=out)

    async def ContainerStatus(self, req, ctx):
        st = self.rt.container_status(req.container_id)
        m = self.cmeta.get(req.container_id)
        if st is None or m is None:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, f"container {req.container_id} not found")
        s = A.MSG["ContainerStatus"](id=st.id, metadata=m["metadata"], state=self._state(st), created_at=_ns(st.created_at),
                                     started_at=_ns(st.started_at), finished_at=_ns(st.finished_at), exit_code=st.exit_code,
                                     image=A.MSG["ImageSpec"](image=m["image"]), image_ref=m["image"], reason=st.reason,
                                     message=st.message, labels=m["labels"], annotations=m["annotations"],
                                     log_path=st.log_path or "")
        return A.MSG["ContainerStatusResponse"](status=s)

    async def UpdateContainerResources(self, req, ctx):
        return A.MSG["UpdateContainerResourcesResponse"]()

    async def ExecSync(self, req, ctx):
        rc, out = await self.rt.exec_sync(req.container_id, list(req.cmd), float(req.timeout or 60))
        return A.MSG["ExecSyncResponse"](stdout=out if isinstance(out, bytes) else str(out).encode(), exit_code=rc)

    async def Exec(self, req, ctx):
        return A.MSG["ExecResponse"](url=self.streaming.url("exec", req))

    async def Attach(self, req, ctx):
        return A.MSG["AttachResponse"](url=self.streaming.url("attach", req))

    async def PortForward(self, req, ctx):
        return A.MSG["PortForwardResponse"](url=self.streaming.url("portforward", req))

    def _stats(self, cid):
        m = self.cmeta.get(cid) or {}
        now = time.time_ns()
        cpu = mem = 0
        pid = None
        meta = getattr(self.rt, "meta", {}).get(cid) or {}
        proc = meta.get("proc")
        if proc is not None and getattr(proc, "returncode", 0) is None:
            pid = proc.pid
        if pid:
            try:
                with open(f"/proc/{pid}/stat") as f:
                    fields = f.read().rsplit(")", 1)[1].split()
                cpu = (int(fields[11]) + int(fields[12])) * (1_000_000_000 // os.sysconf("SC_CLK_TCK"))
                with open(f"/proc/{pid}/statm") as f:
                    mem = int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE")
            except (OSError, IndexError, ValueError):
                pass
        return A.MSG["ContainerStats"](
            attributes=A.MSG["ContainerAttributes"](id=cid, metadata=m.get("metadata"), labels=m.get("labels") or {},
                                                    annotations=m.get("annotations") or {}),
            cpu=A.MSG["CpuUsage"](timestamp=now, usage_core_nano_seconds=A.MSG["UInt64Value"](value=cpu)),
            memory=A.MSG["MemoryUsage"](timestamp=now, working_set_bytes=A.MSG["UInt64Value"](value=mem)))

    async def ContainerStats(self, req, ctx):
        return A.MSG["ContainerStatsResponse"](stats=self._stats(req.container_id))

    async def ListContainerStats(self, req, ctx):
        flt = req.filter if req.HasField("filter") else None
        out = []
        for cid, m in self.cmeta.items():
            if flt is not None and ((flt.id and flt.id != cid) or (flt.pod_sandbox_id and flt.pod_sandbox_id != m["sandbox"])):
                continue
            out.append(self._stats(cid))
        return A.MSG["ListContainerStatsResponse"](stats=out)

    async def UpdateRuntimeConfig(self, req, ctx):
        self.pod_cidr = req.runtime_config.network_config.pod_cidr
        return A.MSG["UpdateRuntimeConfigResponse"]()

    async def Status(self, req, ctx):
        conds = [A.MSG["RuntimeCondition"](type="RuntimeReady", status=True),
                 A.MSG["RuntimeCondition"](type="NetworkReady", status=True)]
        iso = self.rt.isolation_status()
        if iso is not None:
            # not a CRI v1alpha1 condition: how the kubelet learns whether the runtime enforces
            # the device view it asked for (node condition IsolationUnavailable)
            conds.append(A.MSG["RuntimeCondition"](type=A.DEVICE_ISOLATION_CONDITION, status=bool(iso["enforced"]),
                                                   reason=iso["reason"], message=iso["message"]))
        return A.MSG["StatusResponse"](status=A.MSG["RuntimeStatus"](conditions=conds))

    # ---------------------------------------------------------------- image service
    def _image(self, img):
        return A.MSG["Image"](id=img["id"], repo_tags=img.get("repoTags") or [], repo_digests=img.get("repoDigests") or [],
                              size=img.get("size", 0))

    async def ListImages(self, req, ctx):
        ref = req.filter.image.image if req.HasField("filter") else ""
        imgs = await self.images.list_images()
        if ref:
            want = await self.images.image_status(ref)
            imgs = [i for i in imgs if want is not None and i["id"] == want["id"]]
        return A.MSG["ListImagesResponse"](images=[self._image(i) for i in imgs])

    async def ImageStatus(self, req, ctx):
        img = await self.images.image_status(req.image.image)
        return A.MSG["ImageStatusResponse"](image=self._image(img)) if img else A.MSG["ImageStatusResponse"]()

    async def PullImage(self, req, ctx):
        from ..images.registry import Auth, RegistryError
        auth = None
        if req.HasField("auth"):
            a = req.auth
            auth = Auth(a.username, a.password, a.auth, a.identity_token, a.registry_token)
        try:
            return A.MSG["PullImageResponse"](image_ref=await self.images.pull_image(req.image.image, auth))
        except (LookupError, RegistryError, RuntimeError_, OSError, ValueError) as e:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, str(e))

    async def RemoveImage(self, req, ctx):
        await self.images.remove_image(req.image.image)
        return A.MSG["RemoveImageResponse"]()

    async def ImageFsInfo(self, req, ctx):
        info = await self.images.image_fs_info()
        fs = A.MSG["FilesystemUsage"](timestamp=time.time_ns(), storage_id=A.MSG["StorageIdentifier"](uuid="kamd-images"),
                                      used_bytes=A.MSG["UInt64Value"](value=info["usedBytes"]),
                                      inodes_used=A.MSG["UInt64Value"](value=info["inodesUsed"]))
        return A.MSG["ImageFsInfoResponse"](image_filesystems=[fs])


def container_is_running(st):
    return st is not None and st.state == RUNNING


def container_is_exited(st):
    return st is not None and st.state == EXITED
