"""Process runtime — runs containers as host child processes (no docker/containerd in this image).

  * sandbox  = the native `pause` binary (native/pause/pause.cc), holding the pod's lifetime like
               the pause container of a docker sandbox; with isolation it also holds the pod's
               shared ipc + uts (and, unprivileged, user) namespaces that its containers join;
  * container = `command + args`, stdout/stderr to `<root>/containers/<id>/log`, described by an
               OCI bundle (`config.json`, `runtime/oci.py`) holding the injected GPU devices;
  * isolation = when the host allows it (`kamd-runc features`), the bundle is EXECUTED by the
               native OCI executor `kamd-runc` (native/runc/kamd_runc.cc): private mount / pid /
               ipc / uts namespaces, a tmpfs `/dev` holding only the default nodes plus the
               allocated `/dev/kfd` + `/dev/dri/renderD<minor>`, and a cgroup device filter
               (v2 BPF or v1 devices.allow) — a pod cannot reach a render node it was not given,
               whatever HIP_VISIBLE_DEVICES says. Where namespaces are not allowed (an
               unprivileged kubelet on a host without user namespaces) the runtime says so
               and uses the next tier when the kernel has it: Landlock — kamd-runc runs the
               container without namespaces but restricts it (no_new_privs + a Landlock ruleset)
               so that under /dev/dri only the allocated render node(s) can be opened (EACCES for
               the others). Only when neither tier works does the runtime say so
               (`isolation_status()` → node condition IsolationUnavailable) and fall back to
               narrowing HIP enumeration with HIP_VISIBLE_DEVICES; `isolation="required"` refuses
               device containers instead;
  * images   = a local image map (`IMAGES`) resolves well-known images to built executables,
               e.g. `kubernetes-amd/hip-vector-add` → native/bin/hip-vector-add.
Exit is observed by awaiting the child (event-driven PLEG), like a CRI event stream.

Restart survival (docker keeps containers when the kubelet restarts): every sandbox and
container writes `state.json` next to its files (pid + kernel start time, pod uid, name, CRI
attempt, exit code once known). A runtime constructed on the same root re-adopts the processes
that are still alive (same pid AND start time, so a recycled pid is never adopted) and watches
them with a pidfd from `start()`; their exit code is unknowable (not our children) and reads as
255 "ExitCodeUnknown". `pod_states()` hands them to the restarted kubelet.
"""
from __future__ import annotations

import asyncio
import itertools
import json
import os
import shutil
import signal
import subprocess
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
    # the e2e image of `test/e2e/common/docker_containers.go`: an ENTRYPOINT and a CMD
    "kubernetes-amd/entrypoint-tester": ["/bin/echo", "entrypoint"],
}
# image CMD (default arguments), used only when the container sets neither command nor args
IMAGE_CMD = {
    "kubernetes-amd/entrypoint-tester": ["default", "arguments"],
    # the busybox image has no ENTRYPOINT and CMD ["sh"]: `args: [sh, -c, ...]` replaces the CMD
    "busybox": ["/bin/sh"],
}


def builtin_argv(base):
    """The executable a built-in image runs (its ENTRYPOINT, else its CMD); None if not built in."""
    return IMAGES.get(base) or IMAGE_CMD.get(base)


def resolve_command(container):
    """ENTRYPOINT/CMD semantics (`pkg/kubelet/kuberuntime` + docker): `command` replaces the
    image's entrypoint AND drops its CMD; `args` alone replaces the CMD; neither runs both."""
    cmd = list(container.get("command") or [])
    args = list(container.get("args") or [])
    if not cmd:
        img = (container.get("image") or "").split("@")[0]
        base = img.rsplit(":", 1)[0] if ":" in img.split("/")[-1] else img
        if base not in IMAGES and base not in IMAGE_CMD:
            raise FileNotFoundError(f"image {img!r} has no local entrypoint and no command was given")
        cmd = list(IMAGES.get(base, []))
        if not args:
            args = list(IMAGE_CMD.get(base, []))
    if not cmd + args:
        raise FileNotFoundError("the container has neither a command nor arguments")
    return cmd + args


CONTAINER_INIT = os.path.join(BIN_DIR, "container-init")
KAMD_RUNC = os.path.join(BIN_DIR, "kamd-runc")
_FEATURES: dict = {}


def runc_features(cgroup_dir=None) -> dict:
    """`kamd-runc features`: which isolation primitives this host grants (cached per cgroup)."""
    key = cgroup_dir or ""
    if key not in _FEATURES:
        if not os.access(KAMD_RUNC, os.X_OK):
            _FEATURES[key] = {"isolation": False, "namespace_error": "kamd-runc is not built"}
        else:
            try:
                r = subprocess.run([KAMD_RUNC, "features"] + (["--cgroup", cgroup_dir] if cgroup_dir else []),
                                   capture_output=True, text=True, timeout=20)
                _FEATURES[key] = json.loads(r.stdout)
            except (OSError, ValueError, subprocess.SubprocessError) as e:
                _FEATURES[key] = {"isolation": False, "namespace_error": f"kamd-runc features: {e}"}
    return _FEATURES[key]


def _init_argv(argv, env, cpus, oom_adj, cgroup, uid=None, gid=None, groups=()):
    """Prefix argv with the native container-init helper (native/pause/container_init.cc), which
    applies the cpuset, OOM score, cgroup and identity and then execs the entrypoint — so the
    spawn needs no Python pre-exec hook and can use vfork (a hook forces a full fork of the
    kubelet: ~3 ms of kubelet CPU per container instead of ~0.5 ms). The entrypoint is resolved
    here so a missing binary is still a StartError rather than exit 127 of the helper."""
    _check_entrypoint(argv, env)
    pre = [CONTAINER_INIT]
    if cpus:
        pre += ["-c", ",".join(str(c) for c in sorted(cpus))]
    if oom_adj is not None:
        pre += ["-o", str(int(oom_adj))]
    if cgroup:
        pre += ["-g", cgroup]
    if groups:
        pre += ["-S", ",".join(str(int(g)) for g in groups)]
    if gid is not None:
        pre += ["-G", str(int(gid))]
    if uid is not None:
        pre += ["-u", str(int(uid))]
    return pre + ["--"] + list(argv)


def _check_entrypoint(argv, env):
    exe = argv[0]
    if os.sep not in exe:
        if shutil.which(exe, path=env.get("PATH", os.defpath)) is None:
            raise FileNotFoundError(2, "No such file or directory", exe)
    elif not os.access(exe, os.X_OK):
        raise FileNotFoundError(2, "No such file or directory", exe)


async def _spawn_runc(bundle, stdout, timeout=30.0, stdin=None):
    """Start `kamd-runc run` on a bundle; returns (process, container init pid, isolation report)
    once the container's namespaces, /dev and identity are set up (the ready pipe), or raises
    OSError with kamd-runc's diagnostics if the setup failed."""
    loop = asyncio.get_running_loop()
    r, w = os.pipe()
    try:
        proc = await asyncio.create_subprocess_exec(KAMD_RUNC, "run", "--bundle", bundle, "--ready-fd", str(w),
                                                    pass_fds=(w,), stdout=stdout, stderr=asyncio.subprocess.STDOUT,
                                                    stdin=stdin if stdin is not None else asyncio.subprocess.DEVNULL,
                                                    start_new_session=True)
    finally:
        os.close(w)
    reader = asyncio.StreamReader()
    transport, _ = await loop.connect_read_pipe(lambda: asyncio.StreamReaderProtocol(reader), os.fdopen(r, "rb", 0))
    try:
        line = await asyncio.wait_for(reader.readline(), timeout)
    except asyncio.TimeoutError:
        line = b""
    finally:
        transport.close()
    if not line:
        try:
            code = await asyncio.wait_for(proc.wait(), 5)
        except asyncio.TimeoutError:
            proc.kill()
            code = await proc.wait()
        raise OSError(126, f"kamd-runc failed to set up the container (exit {code})")
    pid, _, report = line.decode().strip().partition(" ")
    return proc, int(pid), json.loads(report or "{}")


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

    def __init__(self, root_dir: str, inherit_env: bool = True, isolation: str | None = None, images=None,
                 tier: str | None = None, landlock_dir: str = "/dev/dri"):
        super().__init__()
        # an images.service.ImageService: OCI images (pulled or imported) run on an overlay of
        # their unpacked layers; without one, images resolve to built binaries / the host root
        if images is not None:
            self.images = images
        self.root = os.path.abspath(root_dir)
        os.makedirs(os.path.join(self.root, "containers"), exist_ok=True)
        os.makedirs(os.path.join(self.root, "sandboxes"), exist_ok=True)
        self.sandboxes: dict[str, dict] = {}
        self.containers: dict[str, ContainerStatus] = {}
        self.meta: dict[str, dict] = {}
        self.inherit_env = inherit_env
        # "auto": isolate when the host allows it; "required": refuse device containers when it
        # does not; "off": host processes narrowed by HIP_VISIBLE_DEVICES only
        self.isolation = isolation or os.environ.get("KAMD_ISOLATION", "auto")
        if self.isolation not in ("auto", "required", "off"):
            raise ValueError(f"isolation must be auto, required or off, not {self.isolation!r}")
        self.features = runc_features() if self.isolation != "off" else {}
        self.isolated = bool(self.features.get("isolation"))
        # enforcement tier: "namespaces" (private /dev + device cgroup), "landlock" (no
        # namespaces; /dev/dri opens limited to the allocation) or "none". KAMD_ISOLATION_TIER /
        # `tier` pins one (tests rehearse the unprivileged tier on a host that has namespaces).
        want = tier or os.environ.get("KAMD_ISOLATION_TIER", "auto")
        has_ll = int(self.features.get("landlock") or 0) > 0 and os.access(KAMD_RUNC, os.X_OK)
        if self.isolation == "off":
            self.tier = "none"
        elif want == "auto":
            self.tier = "namespaces" if self.isolated else ("landlock" if has_ll else "none")
        elif want == "landlock":
            if not has_ll:
                raise ValueError("isolation tier landlock requested, but " +
                                 (self.features.get("landlock_error") or "kamd-runc reports no Landlock support"))
            self.tier = "landlock"
        elif want in ("namespaces", "none"):
            if want == "namespaces" and not self.isolated:
                raise ValueError("isolation tier namespaces requested, but " +
                                 (self.features.get("namespace_error") or "namespaces are unavailable"))
            self.tier = want
        else:
            raise ValueError(f"isolation tier must be auto, namespaces, landlock or none, not {want!r}")
        self.isolated = self.tier == "namespaces"
        self.landlocked = self.tier == "landlock"
        self.landlock_dir = landlock_dir
        self._started = False
        self._ids = itertools.count(self._load_state() + 1)

    def isolation_status(self):
        if self.isolation == "off":
            return {"enforced": False, "tier": "none", "reason": "IsolationDisabled",
                    "message": "container isolation is off: GPU enumeration is narrowed by HIP_VISIBLE_DEVICES only"}
        f = self.features
        if self.isolated:
            dc = f.get("device_cgroup", "none")
            return {"enforced": True, "tier": "namespaces", "reason": "DeviceIsolationEnforced",
                    "message": f"tier namespaces: mount/pid/ipc/uts namespaces"
                               f"{' in a user namespace' if f.get('user_ns') else ''}, "
                               f"private /dev with only the allocated device nodes, device cgroup: {dc}"}
        if self.landlocked:
            return {"enforced": True, "tier": "landlock", "reason": "DeviceIsolationEnforced",
                    "message": f"tier landlock (ABI {f.get('landlock')}): no container namespaces here ("
                               + (f.get("namespace_error") or "unavailable") + f"), but each container opens "
                               f"only its allocated nodes under {self.landlock_dir} (Landlock ruleset under "
                               f"no_new_privs; the others are refused, reported EPERM by the preloaded errno "
                               f"shim so ROCr skips them as under a device cgroup)"}
        return {"enforced": False, "tier": "none", "reason": "IsolationUnavailable",
                "message": "no mount namespace for containers (" + (f.get("namespace_error") or "unknown") +
                           ") and no Landlock (" + (f.get("landlock_error") or "unknown") +
                           "): a pod can open any /dev/dri/renderD* of the host; GPU enumeration is narrowed by "
                           "HIP_VISIBLE_DEVICES only"}

    async def start(self):
        """Watch the processes re-adopted from state.json (exit of an adopted container is then
        reported even when nobody calls pod_states(), e.g. behind kamd-cri)."""
        if self._started:
            return
        self._started = True
        for cid, m in self.meta.items():
            if m.pop("adopted", False):
                spawn(self._wait(cid, m["proc"]))
        for sb in self.sandboxes.values():
            if isinstance(sb["proc"], _AdoptedProcess) and sb["proc"].returncode is None:
                spawn(sb["proc"].wait())

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
                                   "pod_uid": st["pod_uid"], "annotations": st.get("annotations") or {},
                                   "init_pid": st.get("init_pid"), "user_ns": st.get("user_ns", False)}
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
                              "init_pid": st.get("init_pid"), "isolated": st.get("isolated", False),
                              "user": st.get("user"), "landlock": st.get("landlock"),
                              "adopted": proc is not None and proc.returncode is None}
        return top

    def _container_state(self, cid, **extra):
        m, cs = self.meta.get(cid), self.containers.get(cid)
        if m is None or cs is None:
            return
        proc = m.get("proc")
        st = {"id": cid, "name": cs.name, "pod_uid": m["pod_uid"], "sandbox": m["sandbox"], "attempt": m.get("attempt", 0),
              "image": cs.image, "created_at": cs.created_at, "started_at": cs.started_at, "argv": m["argv"],
              "env": m["env"], "cwd": m["cwd"], "isolated": m.get("isolated", False)}
        if m.get("init_pid"):
            st["init_pid"], st["user"] = m["init_pid"], m.get("user")
        if m.get("landlock"):
            st["landlock"] = m["landlock"]
        if proc is not None:
            st["pid"], st["ticks"] = proc.pid, _start_ticks(proc.pid)
        st.update(extra)
        try:
            _write_state(m["dir"], st)
        except OSError:
            pass

    async def run_pod_sandbox(self, pod, annotations):
        await self.start()
        sid = f"sb{next(self._ids)}-{pod['metadata']['uid'][:8]}"
        d = os.path.join(self.root, "sandboxes", sid)
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "annotations.json"), "w") as f:
            json.dump(annotations or {}, f)
        pause = os.path.join(BIN_DIR, "pause")
        init_pid, user_ns = None, False
        if self.isolated:
            with open(os.path.join(d, "config.json"), "w") as f:
                json.dump(oci.sandbox_spec(pod, pause), f, separators=(",", ":"))
            with open(os.path.join(d, "log"), "ab") as log:
                proc, init_pid, report = await _spawn_runc(d, log)
            user_ns = bool(report.get("user_ns"))
        else:
            proc = await asyncio.create_subprocess_exec(pause, start_new_session=True,
                                                        stdout=asyncio.subprocess.DEVNULL, stderr=asyncio.subprocess.DEVNULL)
        self.sandboxes[sid] = {"proc": proc, "dir": d, "pod_uid": pod["metadata"]["uid"], "annotations": annotations,
                               "init_pid": init_pid, "user_ns": user_ns}
        _write_state(d, {"pod_uid": pod["metadata"]["uid"], "pid": proc.pid, "ticks": _start_ticks(proc.pid),
                         "annotations": annotations or {}, "init_pid": init_pid, "user_ns": user_ns})
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
        leaf = cid.split("://", 1)[1]
        d = os.path.join(self.root, "containers", leaf)
        os.makedirs(d, exist_ok=True)
        image = container.get("image") or ""
        svc = getattr(self, "images", None)
        cfg = svc.image_config(image) if svc is not None and hasattr(svc, "image_config") else None
        image_root = None
        if cfg is not None:
            from ...images.service import command_for, env_for, user_for
            argv = command_for(container, cfg)
            if not argv:
                raise OSError(2, f"image {image!r} has no entrypoint and the container gives no command")
            image_root = svc.rootfs(image)
            own = {e["name"]: str(e["value"]) for e in container.get("env") or () if "value" in e}
            env = env_for(cfg, own)
            env.setdefault("PATH", "/usr/local/sbin:/usr/local/bin:/usr/sbin:/usr/bin:/sbin:/bin")
            if opts.run_as_user is None:
                ug = user_for(cfg, image_root)
                if ug is not None:
                    import dataclasses
                    opts = dataclasses.replace(opts, run_as_user=ug[0],
                                               run_as_group=opts.run_as_group if opts.run_as_group is not None else ug[1])
            if not container.get("workingDir") and cfg.get("WorkingDir") and self.isolated:
                container = dict(container, workingDir=cfg["WorkingDir"])
        else:
            argv = resolve_command(container)
            env = dict(os.environ) if self.inherit_env else {"PATH": os.environ.get("PATH", "/usr/bin:/bin")}
            for e in container.get("env") or ():
                if "value" in e:
                    env[e["name"]] = str(e["value"])
        dev_env = opts.env_dict()
        env.update(dev_env)
        env.pop("ROCR_VISIBLE_DEVICES", None)
        env.pop("CUDA_VISIBLE_DEVICES", None)
        env.pop("HIP_VISIBLE_DEVICES", None)
        if opts.devices and self.tier == "none" and self.isolation == "required":
            raise OSError(1, "IsolationUnavailable: the runtime cannot give this container a private /dev "
                             f"({self.isolation_status()['message']})")
        if self.tier == "none":
            # no enforcement: narrow HIP enumeration to the allocation; a container without
            # allocated GPUs sees none. (In the enforced tiers a container can open only its own
            # render nodes, so HIP's default enumeration is already right.)
            env["HIP_VISIBLE_DEVICES"] = dev_env.get("AMD_VISIBLE_DEVICES", "-1")
        sb = self.sandboxes.get(sid) or {}
        cgroup = os.path.join(opts.cgroup_parent, f"ctr-{leaf}") if opts.cgroup_parent else None
        cpus = None
        if env.get("KAMD_CPUSET") and hasattr(os, "sched_setaffinity"):
            # cpu manager's cpuset (cgroup cpuset.cpus in a real runtime): pinned before exec
            from ..cpumanager import parse_cpulist
            cpus = set(parse_cpulist(env["KAMD_CPUSET"])) & set(os.sched_getaffinity(0)) or None
        ns_paths = {}
        if self.isolated and sb.get("init_pid"):
            ns_paths = {t: f"/proc/{sb['init_pid']}/ns/{t}" for t in ("ipc", "uts")}
            if sb.get("user_ns"):
                ns_paths["user"] = f"/proc/{sb['init_pid']}/ns/user"
        rootfs, overlay = "/", None
        if image_root is not None and self.isolated:
            # copy-on-write root: the image's unpacked layers under this container's upper dir,
            # mounted by kamd-runc inside the container's mount namespace
            overlay = {k: os.path.join(d, k) for k in ("rootfs", "upper", "work")}
            for p in overlay.values():
                os.makedirs(p, exist_ok=True)
            rootfs = overlay["rootfs"]
        spec = oci.build_spec(pod, dict(container, command=argv, args=[]), opts, rootfs=rootfs,
                              sandbox_pid=getattr(sb.get("proc"), "pid", None),
                              env=env if (self.isolated or self.landlocked) else None, cgroups_path=cgroup,
                              ns_paths=ns_paths, host_network=self.shares_host_network,
                              cpus=",".join(str(c) for c in sorted(cpus)) if cpus else None)
        landlock = None
        if self.landlocked:
            # no namespaces at all: kamd-runc restricts the process itself before exec
            spec["linux"]["namespaces"] = []
            spec["annotations"].update({"kamd.io/isolation-tier": "landlock", "kamd.io/landlock-dir": self.landlock_dir})
            nodes = [d.get("kamd.io/host-path") or d["path"] for d in spec["linux"]["devices"]]
            landlock = self.landlock_dir + ":" + ",".join(nodes)
        if overlay is not None:
            spec["annotations"].update({"kamd.io/rootfs-lower": image_root, "kamd.io/rootfs-upper": overlay["upper"],
                                        "kamd.io/rootfs-work": overlay["work"]})
        with open(os.path.join(d, "config.json"), "w") as f:
            json.dump(spec, f, separators=(",", ":"))
        stdin_fifo = None
        if container.get("stdin"):
            # `stdin: true`: the container reads a FIFO that attach writes into; the runtime holds
            # a write end so the process sees no EOF before an attach (stdinOnce: after the first)
            stdin_fifo = os.path.join(d, "stdin")
            if not os.path.exists(stdin_fifo):
                os.mkfifo(stdin_fifo, 0o600)
        st = ContainerStatus(cid, container["name"], CREATED, image=container.get("image", ""),
                             log_path=os.path.join(d, "log"))
        self.containers[cid] = st
        self.meta[cid] = {"sandbox": sid, "pod_uid": pod["metadata"]["uid"], "argv": argv, "env": env,
                          "cwd": container.get("workingDir") or None, "proc": None, "dir": d, "spec": spec,
                          "oom_score_adj": opts.oom_score_adj, "cgroup": cgroup, "cpus": cpus,
                          "attempt": opts.attempt, "run_as_user": opts.run_as_user, "run_as_group": opts.run_as_group,
                          "groups": list(opts.supplemental_groups), "isolated": self.isolated or self.landlocked,
                          "landlock": landlock,
                          "stdin_fifo": stdin_fifo, "stdin_once": bool(container.get("stdinOnce")), "stdin_w": None,
                          "image_rootfs": overlay is not None,
                          "user": f"{spec['process']['user']['uid']}:{spec['process']['user']['gid']}"}
        return cid

    @staticmethod
    def _gpu_pod(opts):
        return any("/dev/dri/" in x.get("pathOnHost", "") for x in opts.devices)

    async def start_container(self, cid):
        m = self.meta[cid]
        st = self.containers[cid]
        log = open(st.log_path, "ab")
        rfd = None
        try:
            if m.get("stdin_fifo"):
                rfd = os.open(m["stdin_fifo"], os.O_RDONLY | os.O_NONBLOCK)
                m["stdin_w"] = os.open(m["stdin_fifo"], os.O_WRONLY | os.O_NONBLOCK)
                os.set_blocking(rfd, True)
            if m.get("isolated"):
                if not m.get("image_rootfs"):      # (an image's entrypoint lives in its own root)
                    _check_entrypoint(m["argv"], m["env"])
                proc, m["init_pid"], m["isolation"] = await _spawn_runc(m["dir"], log, stdin=rfd)
            else:
                proc = await self._start_host_process(m, log, stdin=rfd)
        except OSError as e:
            if rfd is not None:
                os.close(rfd)
            log.close()
            st.state = EXITED
            st.exit_code = 128
            st.reason = "StartError"
            st.message = str(e)
            st.finished_at = time.time()
            raise
        log.close()
        if rfd is not None:
            os.close(rfd)
        m["proc"] = proc
        st.state = RUNNING
        st.started_at = time.time()
        self._container_state(cid)
        spawn(self._wait(cid, proc))

    async def _start_host_process(self, m, log, stdin=None):
        cpus = m.get("cpus")
        pre = None
        argv = m["argv"]
        identity = m.get("run_as_user") is not None or m.get("run_as_group") is not None or m.get("groups")
        if identity and not os.access(CONTAINER_INIT, os.X_OK):
            raise OSError(1, "runAsUser needs the container-init helper (python -m kubernetes_amd.native.build)")
        if cpus or m.get("oom_score_adj") is not None or m.get("cgroup") or identity:
            if os.access(CONTAINER_INIT, os.X_OK):
                argv = _init_argv(argv, m["env"], cpus, m.get("oom_score_adj"), m.get("cgroup"),
                                  m.get("run_as_user"), m.get("run_as_group"), m.get("groups") or ())
            else:
                pre = _child_setup(cpus, m.get("oom_score_adj"), m.get("cgroup"))
        return await asyncio.create_subprocess_exec(*argv, env=m["env"], cwd=m["cwd"], stdout=log,
                                                    stderr=asyncio.subprocess.STDOUT, start_new_session=True,
                                                    stdin=stdin if stdin is not None else asyncio.subprocess.DEVNULL,
                                                    preexec_fn=pre)

    async def pod_states(self):
        """Sandboxes/containers of this runtime, including the ones re-adopted from state.json
        after a restart (their exits are watched from `start()` on)."""
        await self.start()
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
        if cid in self.meta:
            self._close_stdin(self.meta[cid])
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

    def container_pids(self):
        return {cid: m["proc"].pid for cid, m in self.meta.items()
                if m.get("proc") is not None and m["proc"].returncode is None}

    async def kill_all(self):
        """Kill every container and sandbox process group of this runtime (cluster teardown)."""
        procs = [m["proc"] for m in self.meta.values() if m.get("proc") is not None] + \
            [sb["proc"] for sb in self.sandboxes.values()]
        for p in procs:
            if p.returncode is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass
        for p in procs:
            try:
                await asyncio.wait_for(p.wait(), 5)
            except (asyncio.TimeoutError, ProcessLookupError):
                pass

    def container_status(self, cid):
        return self.containers.get(cid)

    async def exec_sync(self, cid, cmd, timeout):
        m = self.meta.get(cid)
        st = self.containers.get(cid)
        if m is None or st is None or st.state != RUNNING:
            return 126, b"container is not running"
        argv, cwd = self._exec_argv(m, cmd)
        try:
            proc = await asyncio.create_subprocess_exec(*argv, env=m["env"], cwd=cwd, stdout=asyncio.subprocess.PIPE,
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

    @staticmethod
    def _exec_argv(m, cmd):
        argv, cwd = list(cmd), m["cwd"]
        if m.get("init_pid"):
            # into the container's namespaces (its /dev view, pid namespace) as its user
            argv = [KAMD_RUNC, "exec", "--pid", str(m["init_pid"]), "--cwd", cwd or "/"] + \
                (["--user", m["user"]] if m.get("user") else []) + \
                (["--landlock", m["landlock"]] if m.get("landlock") else []) + ["--"] + argv
            cwd = None
        return argv, cwd

    async def exec_interactive(self, cid, cmd, stdin, stdout, stderr, tty, resize):
        """A streamed exec: pipes, or a pseudo-terminal (controlling tty of the new session,
        resized by TIOCSWINSZ) when tty is set."""
        m = self.meta.get(cid)
        st = self.containers.get(cid)
        if m is None or st is None or st.state != RUNNING:
            raise OSError(f"container {cid} is not running")
        argv, cwd = self._exec_argv(m, cmd)
        if tty:
            return await self._exec_tty(argv, cwd, m["env"], stdin, stdout or stderr, resize)
        pipe, null = asyncio.subprocess.PIPE, asyncio.subprocess.DEVNULL
        proc = await asyncio.create_subprocess_exec(
            *argv, env=m["env"], cwd=cwd, stdin=pipe if stdin is not None else null,
            stdout=pipe if stdout is not None else null, stderr=pipe if stderr is not None else null,
            start_new_session=True)

        async def pump_out(stream, sink):
            while True:
                d = await stream.read(65536)
                if not d:
                    return
                await sink(d)

        async def pump_in():
            try:
                async for d in stdin:
                    proc.stdin.write(d)
                    await proc.stdin.drain()
            except (ConnectionError, BrokenPipeError):
                pass
            finally:
                proc.stdin.close()
        tasks = [asyncio.ensure_future(pump_in())] if stdin is not None else []
        outs = [pump_out(s, k) for s, k in ((proc.stdout, stdout), (proc.stderr, stderr)) if k is not None]
        try:
            await asyncio.gather(*outs)
            return await proc.wait()
        finally:
            for t in tasks:
                t.cancel()
            if proc.returncode is None:
                try:
                    os.killpg(proc.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                await proc.wait()

    async def _exec_tty(self, argv, cwd, env, stdin, sink, resize):
        import fcntl
        import pty
        import struct
        import termios
        master, slave = pty.openpty()

        def ctty():
            fcntl.ioctl(0, termios.TIOCSCTTY, 0)
        try:
            proc = await asyncio.create_subprocess_exec(*argv, env=env, cwd=cwd, stdin=slave, stdout=slave,
                                                        stderr=slave, start_new_session=True, preexec_fn=ctty)
        finally:
            os.close(slave)
        loop = asyncio.get_running_loop()
        os.set_blocking(master, False)
        done = loop.create_future()
        chunks: asyncio.Queue = asyncio.Queue()

        def readable():
            try:
                d = os.read(master, 65536)
            except BlockingIOError:
                return
            except OSError:          # EIO: every slave end is closed (the session ended)
                d = b""
            if not d:
                loop.remove_reader(master)
                if not done.done():
                    done.set_result(None)
            chunks.put_nowait(d)
        loop.add_reader(master, readable)

        async def pump_out():
            while True:
                d = await chunks.get()
                if not d:
                    return
                if sink is not None:
                    await sink(d)

        async def pump_in():
            async for d in stdin:
                while d:
                    try:
                        n = os.write(master, d)
                    except BlockingIOError:
                        await asyncio.sleep(0.01)
                        continue
                    d = d[n:]

        async def pump_resize():
            async for w, h in resize:
                fcntl.ioctl(master, termios.TIOCSWINSZ, struct.pack("HHHH", h, w, 0, 0))
        tasks = []
        if stdin is not None:
            tasks.append(asyncio.ensure_future(pump_in()))
        if resize is not None:
            tasks.append(asyncio.ensure_future(pump_resize()))
        out_task = asyncio.ensure_future(pump_out())
        tasks.append(out_task)
        try:
            rc = await proc.wait()
            # the rest of the output: until EIO, or briefly if a background child keeps the tty
            await asyncio.wait([out_task], timeout=2.0)
            return rc
        finally:
            for t in tasks:
                t.cancel()
            loop.remove_reader(master)
            os.close(master)
            if proc.returncode is None:
                try:
                    os.killpg(proc.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                await proc.wait()

    def _close_stdin(self, m):
        fd, m["stdin_w"] = m.get("stdin_w"), None
        if fd is not None:
            try:
                os.close(fd)
            except OSError:
                pass

    async def _pump_stdin(self, m, stdin):
        """Attach's stdin into the container's FIFO; stdinOnce closes it when the stream ends."""
        try:
            async for data in stdin:
                fd = m.get("stdin_w")
                if fd is None:
                    break
                view = memoryview(data)
                while view:
                    try:
                        n = os.write(fd, view)
                        view = view[n:]
                    except BlockingIOError:
                        await asyncio.sleep(0.01)
                    except OSError:          # the container closed its stdin / exited
                        return
        finally:
            if m.get("stdin_once"):
                self._close_stdin(m)

    async def attach(self, cid, stdin, stdout, stderr, tty, resize):
        """Follow the container's output file from its current end until the container exits;
        with `stdin: true` the attach's input goes to the container's stdin FIFO."""
        st = self.containers.get(cid)
        if st is None:
            raise OSError(f"container {cid} not found")
        m = self.meta.get(cid) or {}
        pump = None
        if stdin is not None and m.get("stdin_w") is not None:
            pump = asyncio.ensure_future(self._pump_stdin(m, stdin))
        sink = stdout or stderr
        pos = os.path.getsize(st.log_path) if os.path.exists(st.log_path) else 0
        while True:
            st = self.containers.get(cid)
            running = st is not None and st.state == RUNNING
            if st is not None and os.path.exists(st.log_path):
                with open(st.log_path, "rb") as f:
                    f.seek(pos)
                    data = f.read()
                if data:
                    pos += len(data)
                    if sink is not None:
                        await sink(data)
            if not running:
                if pump is not None:
                    pump.cancel()
                return 0 if st is None else int(st.exit_code or 0)
            await asyncio.sleep(0.05)

    def list_containers(self):
        return list(self.containers.values())

    def log_path(self, cid):
        st = self.containers.get(cid)
        return st.log_path if st is not None else None

    async def container_logs(self, cid, tail=None):
        st = self.containers.get(cid)
        if st is None or not os.path.exists(st.log_path):
            return b""
        with open(st.log_path, "rb") as f:
            data = f.read()
        if tail:
            data = b"\n".join(data.splitlines()[-tail:]) + b"\n"
        return data
