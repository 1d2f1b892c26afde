"""OCI runtime-spec generation with AMD GPU device injection.

The reference delegated GPU injection to nvidia-container-runtime, selected per container by
dockershim hooks (`pkg/kubelet/dockershim/docker_hooks.go:139-160`), and docker put the
device plugin's DeviceSpecs into `HostConfig.Resources.Devices`
(`pkg/kubelet/dockershim/docker_container.go:164-172`). On MI355X nothing vendor-specific is
needed at the runtime level: the kubelet writes the device plugin's `DeviceSpec`s straight into
the bundle — `/dev/kfd` + `/dev/dri/renderD<minor>` as `linux.devices`, matching cgroup allow
rules (DRM char major 226; kfd's dynamic major) after a deny-all — plus the ROCm userspace as
read-only mounts. Device numbers come from the native helper (`native/oci/oci_devices.cc`, stat()
of each host node). The process runtime executes this spec with `kamd-runc`
(`native/runc/kamd_runc.cc`): private mount/pid/ipc/uts namespaces, a tmpfs `/dev` holding only
these nodes, and a cgroup device filter.
"""
from __future__ import annotations

import os

from ...native.oci import oci_devices
from .base import RunContainerOptions

DEFAULT_CAPS = ["CAP_CHOWN", "CAP_DAC_OVERRIDE", "CAP_FSETID", "CAP_FOWNER", "CAP_MKNOD", "CAP_NET_RAW",
                "CAP_SETGID", "CAP_SETUID", "CAP_SETFCAP", "CAP_SETPCAP", "CAP_NET_BIND_SERVICE",
                "CAP_SYS_CHROOT", "CAP_KILL", "CAP_AUDIT_WRITE"]
ALL_CAPS = ["CAP_CHOWN", "CAP_DAC_OVERRIDE", "CAP_DAC_READ_SEARCH", "CAP_FOWNER", "CAP_FSETID", "CAP_KILL",
            "CAP_SETGID", "CAP_SETUID", "CAP_SETPCAP", "CAP_LINUX_IMMUTABLE", "CAP_NET_BIND_SERVICE",
            "CAP_NET_BROADCAST", "CAP_NET_ADMIN", "CAP_NET_RAW", "CAP_IPC_LOCK", "CAP_IPC_OWNER", "CAP_SYS_MODULE",
            "CAP_SYS_RAWIO", "CAP_SYS_CHROOT", "CAP_SYS_PTRACE", "CAP_SYS_PACCT", "CAP_SYS_ADMIN", "CAP_SYS_BOOT",
            "CAP_SYS_NICE", "CAP_SYS_RESOURCE", "CAP_SYS_TIME", "CAP_SYS_TTY_CONFIG", "CAP_MKNOD", "CAP_LEASE",
            "CAP_AUDIT_WRITE", "CAP_AUDIT_CONTROL", "CAP_SETFCAP", "CAP_MAC_OVERRIDE", "CAP_MAC_ADMIN",
            "CAP_SYSLOG", "CAP_WAKE_ALARM", "CAP_BLOCK_SUSPEND", "CAP_AUDIT_READ"]
# runc / docker defaults (OCI runtime-spec config-linux.md "maskedPaths" / "readonlyPaths")
MASKED_PATHS = ["/proc/acpi", "/proc/kcore", "/proc/keys", "/proc/latency_stats", "/proc/timer_list",
                "/proc/timer_stats", "/proc/sched_debug", "/proc/scsi", "/sys/firmware"]
READONLY_PATHS = ["/proc/asound", "/proc/bus", "/proc/fs", "/proc/irq", "/proc/sys", "/proc/sysrq-trigger"]


def _cap(name):
    name = name.upper()
    return name if name.startswith("CAP_") else "CAP_" + name


def capability_set(opts: RunContainerOptions):
    """securityContext.capabilities over the default set (`kuberuntime/security_context.go`
    → docker's `TweakCapabilities`): "ALL" in add/drop means every capability."""
    if opts.privileged:
        return list(ALL_CAPS)
    drop = {_cap(c) for c in opts.cap_drop}
    caps = [] if "CAP_ALL" in drop else [c for c in DEFAULT_CAPS if c not in drop]
    for c in opts.cap_add:
        c = _cap(c)
        for x in (ALL_CAPS if c == "CAP_ALL" else [c]):
            if x not in caps:
                caps.append(x)
    return caps


def build_spec(pod, container, opts: RunContainerOptions, rootfs="rootfs", hostname=None, sandbox_pid=None,
               env=None, cgroups_path=None, ns_paths=None, host_network=False, cpus=None) -> dict:
    """`env`: the container's complete environment (dict) when the caller resolved it (the
    process runtime does); `ns_paths`: {"ipc"|"uts"|"user"|"network": path} namespaces to join
    (the pod sandbox's); `host_network`: no network namespace (the process runtime's pods use
    the node's)."""
    if env is not None:
        env_list = [f"{k}={v}" for k, v in env.items()]
    else:
        env_list = ["PATH=/usr/local/sbin:/usr/local/bin:/usr/sbin:/usr/bin:/sbin:/bin"]
        for e in container.get("env") or ():
            if "value" in e:
                env_list.append(f"{e['name']}={e['value']}")
        for e in opts.envs:
            env_list.append(f"{e['name']}={e['value']}")
    args = list(container.get("command") or []) + list(container.get("args") or [])
    mounts = [{"destination": "/proc", "type": "proc", "source": "proc", "options": ["nosuid", "noexec", "nodev"]}]
    if not opts.privileged:
        mounts += [
            {"destination": "/dev", "type": "tmpfs", "source": "tmpfs", "options": ["nosuid", "strictatime", "mode=755", "size=65536k"]},
            {"destination": "/dev/pts", "type": "devpts", "source": "devpts",
             "options": ["nosuid", "noexec", "newinstance", "ptmxmode=0666", "mode=0620"]},
            {"destination": "/dev/shm", "type": "tmpfs", "source": "shm", "options": ["nosuid", "noexec", "nodev", "mode=1777", "size=65536k"]},
        ]
    mounts.append({"destination": "/sys", "type": "sysfs", "source": "sysfs", "options": ["nosuid", "noexec", "nodev", "ro"]})
    for mt in opts.mounts:
        o = ["rbind", "ro" if mt.get("readOnly") else "rw"]
        mounts.append({"destination": mt["containerPath"], "type": "bind", "source": mt["hostPath"], "options": o})
    present = [d for d in opts.devices if os.path.exists(d["pathOnHost"])]
    missing = [d["pathOnHost"] for d in opts.devices if not os.path.exists(d["pathOnHost"])]
    devs, allow = [], [{"allow": False, "access": "rwm"}]
    if present:
        info = oci_devices([d["pathOnHost"] for d in present])
        for d, di, rule in zip(present, info["devices"], info["allow"]):
            di = dict(di)
            di["path"] = d["pathInContainer"]
            if d["pathOnHost"] != d["pathInContainer"]:
                di["kamd.io/host-path"] = d["pathOnHost"]
            devs.append(di)
            rule["access"] = _access(d.get("permissions"))
            allow.append(rule)
    if opts.privileged:
        devs, allow = [], [{"allow": True, "access": "rwm"}]
    annotations = {a["name"]: a["value"] for a in opts.annotations}
    if missing:
        annotations["amd.com/missing-device-nodes"] = ",".join(missing)
    user = {"uid": opts.run_as_user if opts.run_as_user is not None else os.geteuid(),
            "gid": opts.run_as_group if opts.run_as_group is not None else os.getegid()}
    if opts.supplemental_groups:
        user["additionalGids"] = list(opts.supplemental_groups)
    caps = capability_set(opts)
    process = {"terminal": False, "user": user, "args": args or ["/pause"], "env": env_list,
               "cwd": container.get("workingDir") or "/",
               "capabilities": {k: caps for k in ("bounding", "effective", "permitted")},
               "noNewPrivileges": not opts.privileged}
    if opts.oom_score_adj is not None:
        process["oomScoreAdj"] = int(opts.oom_score_adj)
    ns_paths = ns_paths or {}
    namespaces = []
    for t in ("user", "pid", "ipc", "uts", "mount"):
        if t in ns_paths:
            namespaces.append({"type": t, "path": ns_paths[t]})
        elif t != "user":
            namespaces.append({"type": t})
    if not host_network:
        net = ns_paths.get("network") or (f"/proc/{sandbox_pid}/ns/net" if sandbox_pid else None)
        namespaces.append({"type": "network", "path": net} if net else {"type": "network"})
    linux = {"devices": devs, "resources": {"devices": allow}, "namespaces": namespaces}
    if not opts.privileged:
        linux["maskedPaths"] = list(MASKED_PATHS)
        linux["readonlyPaths"] = list(READONLY_PATHS)
    if cgroups_path:
        linux["cgroupsPath"] = cgroups_path
    cpus = cpus or annotations.get("io.kubernetes.cpuset")   # cpu manager (static policy) exclusive cpus
    if cpus:
        linux["resources"]["cpu"] = {"cpus": cpus}
    spec = {
        "ociVersion": "1.0.2",
        "process": process,
        "root": {"path": rootfs, "readonly": bool(opts.readonly_rootfs)},
        "hostname": hostname or pod["metadata"]["name"],
        "mounts": mounts,
        "annotations": annotations,
        "linux": linux,
    }
    return spec


def sandbox_spec(pod, pause_path, user_ns=False) -> dict:
    """The pod sandbox: `pause` holding the pod's shared ipc + uts namespaces (and, for an
    unprivileged runtime, the pod's user namespace), which every container of the pod joins —
    the pause container of a docker sandbox (`pkg/kubelet/dockershim/docker_sandbox.go:78`)."""
    ns = [{"type": "ipc"}, {"type": "uts"}] + ([{"type": "user"}] if user_ns else [])
    return {"ociVersion": "1.0.2",
            "process": {"args": [pause_path], "env": ["PATH=/usr/bin:/bin"], "cwd": "/",
                        "user": {"uid": os.geteuid(), "gid": os.getegid()},
                        "capabilities": {"bounding": []}, "noNewPrivileges": True},
            "root": {"path": "/"}, "hostname": pod["metadata"]["name"][:63], "mounts": [],
            "linux": {"namespaces": ns}}


def _access(perm):
    perm = perm or "rw"
    return "".join(c for c in "rwm" if c in perm) or "rw"
