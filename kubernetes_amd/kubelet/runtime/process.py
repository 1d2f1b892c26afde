"""Process runtime — runs containers as host child processes (no docker/containerd in this image).

  * sandbox  = the native `pause` binary (native/pause/pause.cc) in its own session, holding the
               pod's lifetime like the pause container of a docker sandbox;
  * container = `command + args` as a child process in its own process group, stdout/stderr to
               `<root>/containers/<id>/log`; an OCI `config.json` with the injected GPU devices
               is written into the container bundle (`runtime/oci.py`) for audit/OCI runtimes;
  * images   = a local image map (`IMAGES`) resolves well-known images to built executables,
               e.g. `kubernetes-amd/hip-vector-add` → native/bin/hip-vector-add;
  * GPUs     = without device namespaces the runtime narrows HIP enumeration itself:
               `AMD_VISIBLE_DEVICES` from the device plugin becomes `HIP_VISIBLE_DEVICES`.
Exit is observed by awaiting the child (event-driven PLEG), like a CRI event stream.

Restart survival (docker keeps containers when the kubelet restarts): every sandbox and
container writes `state.json` next to its files (pid + kernel start time, pod uid, name, CRI
attempt, exit code once known). A runtime constructed on the same root re-adopts the processes
that are still alive (same pid AND start time, so a recycled pid is never adopted) and watches
them with a pidfd; their exit code is unknowable (not our children) and reads as 255
"ExitCodeUnknown". `pod_states()` hands them to the restarted kubelet.
"""
from __future__ import annotations

import asyncio
import itertools
import json
import os
import shutil
import signal
import time

from ...native import BIN_DIR
from . import oci
from .base import CREATED, EXITED, RUNNING, ContainerStatus, Runtime, RunContainerOptions

UNKNOWN_EXIT = 255


def _start_ticks(pid):
    """Kernel start time of pid (clock ticks since boot, /proc/<pid>/stat field 22) or None."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            data = f.read()
        return int(data[data.rindex(")") + 2:].split()[19])
    except (OSError, ValueError, IndexError):
        return None


class _AdoptedProcess:
    """A process started by an earlier runtime instance (not our child): asyncio.Process-like
    pid / returncode / wait / terminate / kill, exit observed through a pidfd."""

    def __init__(self, pid, ticks):
        self.pid, self.ticks = pid, ticks
        self.returncode = None if _start_ticks(pid) == ticks else UNKNOWN_EXIT
        self._done = None

    async def wait(self):
        if self.returncode is not None:
            return self.returncode
        loop = asyncio.get_running_loop()
        if self._done is None:
            self._done = loop.create_future()
            try:
                fd = os.pidfd_open(self.pid)
            except (OSError, AttributeError):
                fd = None
            if fd is not None:
                def ready():
                    loop.remove_reader(fd)
                    os.close(fd)
                    self.returncode = UNKNOWN_EXIT
                    if not self._done.done():
                        self._done.set_result(None)
                loop.add_reader(fd, ready)
            else:
                async def poll():
                    while _start_ticks(self.pid) == self.ticks:
                        await asyncio.sleep(0.2)
                    self.returncode = UNKNOWN_EXIT
                    self._done.set_result(None)
                spawn(poll())
        await asyncio.shield(self._done)
        return self.returncode

    def terminate(self):
        os.kill(self.pid, signal.SIGTERM)

    def kill(self):
        os.kill(self.pid, signal.SIGKILL)


def _write_state(d, state):
    tmp = os.path.join(d, "state.json.tmp")
    with open(tmp, "w") as f:
        json.dump(state, f, separators=(",", ":"))
    os.replace(tmp, os.path.join(d, "state.json"))


def _read_state(d):
    try:
        with open(os.path.join(d, "state.json")) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None
from ...utils.tasks import spawn

IMAGES = {
    "kubernetes-amd/hip-vector-add": [os.path.join(BIN_DIR, "hip-vector-add")],
    "kubernetes-amd/xgmi-probe": [os.path.join(BIN_DIR, "xgmi-probe")],
    "kubernetes-amd/pause": [os.path.join(BIN_DIR, "pause")],
    "busybox": ["/bin/sh"],
}


def resolve_command(container):
    cmd = list(container.get("command") or [])
    args = list(container.get("args") or [])
    if not cmd:
        img = (container.get("image") or "").split("@")[0]
        base = img.rsplit(":", 1)[0] if ":" in img.split("/")[-1] else img
        cmd = list(IMAGES.get(base, []))
        if not cmd:
            raise FileNotFoundError(f"image {img!r} has no local entrypoint and no command was given")
    return cmd + args


CONTAINER_INIT = os.path.join(BIN_DIR, "container-init")


def _init_argv(argv, env, cpus, oom_adj, cgroup, uid=None, gid=None):
    """Prefix argv with the native container-init helper (native/pause/container_init.cc), which
    applies the cpuset, OOM score and cgroup and then execs the entrypoint — so the spawn needs
    no Python pre-exec hook and can use vfork (a hook forces a full fork of the kubelet: ~3 ms
    of kubelet CPU per container instead of ~0.5 ms). The entrypoint is resolved here so a
    missing binary is still a StartError rather than exit 127 of the helper."""
    exe = argv[0]
    if os.sep not in exe:
        found = shutil.which(exe, path=env.get("PATH", os.defpath))
        if found is None:
            raise FileNotFoundError(2, "No such file or directory", exe)
    elif not os.access(exe, os.X_OK):
        raise FileNotFoundError(2, "No such file or directory", exe)
    pre = [CONTAINER_INIT]
    if cpus:
        pre += ["-c", ",".join(str(c) for c in sorted(cpus))]
    if oom_adj is not None:
        pre += ["-o", str(int(oom_adj))]
    if cgroup:
        pre += ["-g", cgroup]
    if gid is not None:
        pre += ["-G", str(int(gid))]
    if uid is not None:
        pre += ["-u", str(int(uid))]
    return pre + ["--"] + list(argv)


def _child_setup(cpus, oom_adj, cgroup):
    """Fallback when container-init is not built: runs in the forked child before exec — cpuset
    pinning, the kubelet's OOM score adjustment, pod cgroup membership. Failures are ignored
    (an unprivileged kubelet can raise but not lower oom_score_adj, and may not own a cgroup
    subtree)."""
    def pre():
        if cpus:
            os.sched_setaffinity(0, cpus)
        if oom_adj is not None:
            try:
                with open("/proc/self/oom_score_adj", "w") as f:
                    f.write(str(oom_adj))
            except OSError:
                pass
        if cgroup:
            try:
                with open(os.path.join(cgroup, "cgroup.procs"), "w") as f:
                    f.write("0")            # "0" = the writing process itself
            except OSError:
                pass
    return pre


class ProcessRuntime(Runtime):
    name = "process"
    shares_host_network = True     # containers are host processes: pod IP = node address

    def __init__(self, root_dir: str, inherit_env: bool = True):
        super().__init__()
        self.root = os.path.abspath(root_dir)
        os.makedirs(os.path.join(self.root, "containers"), exist_ok=True)
        os.makedirs(os.path.join(self.root, "sandboxes"), exist_ok=True)
        self.sandboxes: dict[str, dict] = {}
        self.containers: dict[str, ContainerStatus] = {}
        self.meta: dict[str, dict] = {}
        self.inherit_env = inherit_env
        self._ids = itertools.count(self._load_state() + 1)

    def _load_state(self) -> int:
        """Re-adopt sandboxes/containers an earlier runtime instance on this root left running
        (or exited with a recorded code). Returns the highest id in use."""
        top = 0
        sdir = os.path.join(self.root, "sandboxes")
        for sid in sorted(os.listdir(sdir)):
            st = _read_state(os.path.join(sdir, sid))
            try:
                top = max(top, int(sid[2:].split("-", 1)[0]))
            except ValueError:
                pass
            if not st:
                continue
            self.sandboxes[sid] = {"proc": _AdoptedProcess(st["pid"], st.get("ticks")), "dir": os.path.join(sdir, sid),
                                   "pod_uid": st["pod_uid"], "annotations": st.get("annotations") or {}}
        cdir = os.path.join(self.root, "containers")
        for name in sorted(os.listdir(cdir)):
            d = os.path.join(cdir, name)
            st = _read_state(d)
            try:
                top = max(top, int(name.split("-", 1)[0]))
            except ValueError:
                pass
            if not st or st.get("sandbox") not in self.sandboxes:
                continue
            cid = st["id"]
            cs = ContainerStatus(cid, st["name"], CREATED, image=st.get("image", ""), log_path=os.path.join(d, "log"))
            cs.created_at = st.get("created_at", cs.created_at)
            cs.started_at = st.get("started_at", 0.0)
            proc = None
            if "exit_code" in st:
                cs.state, cs.exit_code, cs.reason = EXITED, st["exit_code"], st.get("reason", "")
                cs.finished_at = st.get("finished_at", 0.0)
            elif st.get("pid"):
                proc = _AdoptedProcess(st["pid"], st.get("ticks"))
                if proc.returncode is None:
                    cs.state = RUNNING
                else:
                    cs.state, cs.exit_code, cs.reason = EXITED, UNKNOWN_EXIT, "ExitCodeUnknown"
                    cs.finished_at = time.time()
            self.containers[cid] = cs
            self.meta[cid] = {"sandbox": st["sandbox"], "pod_uid": st["pod_uid"], "argv": st.get("argv") or [],
                              "env": st.get("env") or {}, "cwd": st.get("cwd"), "proc": proc, "dir": d, "spec": None,
                              "oom_score_adj": None, "cgroup": None, "attempt": st.get("attempt", 0),
                              "adopted": proc is not None and proc.returncode is None}
        return top

    def _container_state(self, cid, **extra):
        m, cs = self.meta.get(cid), self.containers.get(cid)
        if m is None or cs is None:
            return
        proc = m.get("proc")
        st = {"id": cid, "name": cs.name, "pod_uid": m["pod_uid"], "sandbox": m["sandbox"], "attempt": m.get("attempt", 0),
              "image": cs.image, "created_at": cs.created_at, "started_at": cs.started_at, "argv": m["argv"],
              "env": m["env"], "cwd": m["cwd"]}
        if proc is not None:
            st["pid"], st["ticks"] = proc.pid, _start_ticks(proc.pid)
        st.update(extra)
        try:
            _write_state(m["dir"], st)
        except OSError:
            pass

    async def run_pod_sandbox(self, pod, annotations):
        sid = f"sb{next(self._ids)}-{pod['metadata']['uid'][:8]}"
        d = os.path.join(self.root, "sandboxes", sid)
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "annotations.json"), "w") as f:
            json.dump(annotations or {}, f)
        proc = await asyncio.create_subprocess_exec(os.path.join(BIN_DIR, "pause"), start_new_session=True,
                                                    stdout=asyncio.subprocess.DEVNULL, stderr=asyncio.subprocess.DEVNULL)
        self.sandboxes[sid] = {"proc": proc, "dir": d, "pod_uid": pod["metadata"]["uid"], "annotations": annotations}
        _write_state(d, {"pod_uid": pod["metadata"]["uid"], "pid": proc.pid, "ticks": _start_ticks(proc.pid),
                         "annotations": annotations or {}})
        return sid

    async def stop_pod_sandbox(self, sid):
        sb = self.sandboxes.get(sid)
        if not sb:
            return
        for cid, m in list(self.meta.items()):
            if m["sandbox"] == sid:
                await self.stop_container(cid, 2)
        p = sb["proc"]
        if p.returncode is None:
            try:
                p.terminate()
                await asyncio.wait_for(p.wait(), 5)
            except (ProcessLookupError, asyncio.TimeoutError):
                try:
                    p.kill()
                except ProcessLookupError:
                    pass

    async def remove_pod_sandbox(self, sid):
        await self.stop_pod_sandbox(sid)
        for cid, m in list(self.meta.items()):
            if m["sandbox"] == sid:
                await self.remove_container(cid)
        sb = self.sandboxes.pop(sid, None)
        if sb is not None:
            try:
                os.unlink(os.path.join(sb["dir"], "state.json"))
            except OSError:
                pass

    async def create_container(self, sid, pod, container, opts: RunContainerOptions):
        cid = f"process://{next(self._ids)}-{container['name']}"
        d = os.path.join(self.root, "containers", cid.split("://", 1)[1])
        os.makedirs(d, exist_ok=True)
        argv = resolve_command(container)
        env = dict(os.environ) if self.inherit_env else {"PATH": os.environ.get("PATH", "/usr/bin:/bin")}
        for e in container.get("env") or ():
            if "value" in e:
                env[e["name"]] = str(e["value"])
        dev_env = opts.env_dict()
        env.update(dev_env)
        env.pop("ROCR_VISIBLE_DEVICES", None)
        env.pop("CUDA_VISIBLE_DEVICES", None)
        if "AMD_VISIBLE_DEVICES" in dev_env:
            env["HIP_VISIBLE_DEVICES"] = dev_env["AMD_VISIBLE_DEVICES"]
        else:
            env["HIP_VISIBLE_DEVICES"] = "-1"   # a container without allocated GPUs sees none
        sb = self.sandboxes.get(sid) or {}
        spec = oci.build_spec(pod, dict(container, command=argv, args=[]), opts,
                              sandbox_pid=getattr(sb.get("proc"), "pid", None))
        with open(os.path.join(d, "config.json"), "w") as f:
            json.dump(spec, f, separators=(",", ":"))
        st = ContainerStatus(cid, container["name"], CREATED, image=container.get("image", ""),
                             log_path=os.path.join(d, "log"))
        self.containers[cid] = st
        self.meta[cid] = {"sandbox": sid, "pod_uid": pod["metadata"]["uid"], "argv": argv, "env": env,
                          "cwd": container.get("workingDir") or None, "proc": None, "dir": d, "spec": spec,
                          "oom_score_adj": opts.oom_score_adj, "cgroup": opts.cgroup_parent,
                          "attempt": opts.attempt, "run_as_user": opts.run_as_user, "run_as_group": opts.run_as_group}
        return cid

    @staticmethod
    def _gpu_pod(opts):
        return any("/dev/dri/" in x.get("pathOnHost", "") for x in opts.devices)

    async def start_container(self, cid):
        m = self.meta[cid]
        st = self.containers[cid]
        log = open(st.log_path, "ab")
        cpus = None
        if m["env"].get("KAMD_CPUSET") and hasattr(os, "sched_setaffinity"):
            # cpu manager's cpuset (cgroup cpuset.cpus in a real runtime): pin before exec
            from ..cpumanager import parse_cpulist
            cpus = set(parse_cpulist(m["env"]["KAMD_CPUSET"])) & set(os.sched_getaffinity(0)) or None
        pre = None
        argv = m["argv"]
        try:
            identity = m.get("run_as_user") is not None or m.get("run_as_group") is not None
            if identity and not os.access(CONTAINER_INIT, os.X_OK):
                raise OSError(1, "runAsUser needs the container-init helper (python -m kubernetes_amd.native.build)")
            if cpus or m.get("oom_score_adj") is not None or m.get("cgroup") or identity:
                if os.access(CONTAINER_INIT, os.X_OK):
                    argv = _init_argv(argv, m["env"], cpus, m.get("oom_score_adj"), m.get("cgroup"),
                                      m.get("run_as_user"), m.get("run_as_group"))
                else:
                    pre = _child_setup(cpus, m.get("oom_score_adj"), m.get("cgroup"))
            proc = await asyncio.create_subprocess_exec(*argv, env=m["env"], cwd=m["cwd"], stdout=log,
                                                        stderr=asyncio.subprocess.STDOUT, start_new_session=True,
                                                        preexec_fn=pre)
        except OSError as e:
            log.close()
            st.state = EXITED
            st.exit_code = 128
            st.reason = "StartError"
            st.message = str(e)
            st.finished_at = time.time()
            raise
        log.close()
        m["proc"] = proc
        st.state = RUNNING
        st.started_at = time.time()
        self._container_state(cid)
        spawn(self._wait(cid, proc))

    async def pod_states(self):
        """Sandboxes/containers of this runtime, including the ones re-adopted from state.json
        after a restart (their exits are watched from here on)."""
        for cid, m in self.meta.items():
            if m.pop("adopted", False):
                spawn(self._wait(cid, m["proc"]))
        out: dict = {}
        for sid, sb in self.sandboxes.items():
            alive = sb["proc"].returncode is None
            out.setdefault(sb["pod_uid"], {"sandboxes": [], "containers": []})["sandboxes"].append((sid, alive, None))
        for cid, m in self.meta.items():
            st = self.containers.get(cid)
            if st is not None:
                out.setdefault(m["pod_uid"], {"sandboxes": [], "containers": []})["containers"].append(
                    (st.name, cid, m.get("attempt", 0), st.created_at, m["sandbox"]))
        return out

    async def _wait(self, cid, proc):
        code = await proc.wait()
        st = self.containers.get(cid)
        if st is None:
            return
        if st.state != EXITED:
            st.state = EXITED
            st.exit_code = code if code >= 0 else 128 - code
            st.reason = ("Completed" if code == 0 else "Error") if code != UNKNOWN_EXIT or \
                not isinstance(proc, _AdoptedProcess) else "ExitCodeUnknown"
            st.finished_at = time.time()
        self._container_state(cid, exit_code=st.exit_code, reason=st.reason, finished_at=st.finished_at)
        self._fire_exit(self.meta[cid]["pod_uid"], cid)

    async def stop_container(self, cid, timeout):
        m = self.meta.get(cid)
        if not m or m["proc"] is None or m["proc"].returncode is not None:
            st = self.containers.get(cid)
            if st is not None and st.state != EXITED:
                st.state = EXITED
                st.finished_at = time.time()
            return
        proc = m["proc"]
        try:
            os.killpg(proc.pid, signal.SIGTERM)
            await asyncio.wait_for(proc.wait(), max(timeout, 0.01))
        except (ProcessLookupError, PermissionError):
            pass
        except asyncio.TimeoutError:
            try:
                os.killpg(proc.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            await proc.wait()
        st = self.containers[cid]
        if st.state != EXITED:
            st.state = EXITED
            st.exit_code = 143
            st.reason = "Killed"
            st.finished_at = time.time()

    async def remove_container(self, cid):
        await self.stop_container(cid, 0)
        self.containers.pop(cid, None)
        m = self.meta.pop(cid, None)
        if m is not None:
            try:
                os.unlink(os.path.join(m["dir"], "state.json"))
            except OSError:
                pass

    def container_status(self, cid):
        return self.containers.get(cid)

    async def exec_sync(self, cid, cmd, timeout):
        m = self.meta.get(cid)
        st = self.containers.get(cid)
        if m is None or st is None or st.state != RUNNING:
            return 126, b"container is not running"
        try:
            proc = await asyncio.create_subprocess_exec(*cmd, env=m["env"], cwd=m["cwd"], stdout=asyncio.subprocess.PIPE,
                                                        stderr=asyncio.subprocess.STDOUT, start_new_session=True)
        except OSError as e:
            return 127, str(e).encode()
        try:
            out, _ = await asyncio.wait_for(proc.communicate(), timeout)
        except asyncio.TimeoutError:
            try:
                os.killpg(proc.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            await proc.wait()
            return 124, b"timeout"
        return proc.returncode, out

    def list_containers(self):
        return list(self.containers.values())

    async def container_logs(self, cid, tail=None):
        st = self.containers.get(cid)
        if st is None or not os.path.exists(st.log_path):
            return b""
        with open(st.log_path, "rb") as f:
            data = f.read()
        if tail:
            data = b"\n".join(data.splitlines()[-tail:]) + b"\n"
        return data
