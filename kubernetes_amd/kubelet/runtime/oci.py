"""OCI runtime-spec generation with AMD GPU device injection.

The reference delegated GPU injection to nvidia-container-runtime, selected per container by
dockershim hooks (`pkg/kubelet/dockershim/docker_hooks.go:139-160`). On MI355X nothing
vendor-specific is needed at the runtime level: the kubelet writes the device plugin's
`DeviceSpec`s straight into the bundle — `/dev/kfd` + `/dev/dri/renderD<minor>` as
`linux.devices`, matching cgroup allow rules (DRM char major 226; kfd's dynamic major) — plus
the ROCm userspace as read-only mounts. Device numbers come from the native helper
(`native/oci/oci_devices.cc`, stat() of each host node).
"""
from __future__ import annotations

import os

from ...native.oci import oci_devices
from .base import RunContainerOptions

DEFAULT_CAPS = ["CAP_CHOWN", "CAP_DAC_OVERRIDE", "CAP_FSETID", "CAP_FOWNER", "CAP_MKNOD", "CAP_NET_RAW",
                "CAP_SETGID", "CAP_SETUID", "CAP_SETFCAP", "CAP_SETPCAP", "CAP_NET_BIND_SERVICE",
                "CAP_SYS_CHROOT", "CAP_KILL", "CAP_AUDIT_WRITE"]


def build_spec(pod, container, opts: RunContainerOptions, rootfs="rootfs", hostname=None, sandbox_pid=None) -> dict:
    env = ["PATH=/usr/local/sbin:/usr/local/bin:/usr/sbin:/usr/bin:/sbin:/bin"]
    for e in container.get("env") or ():
        if "value" in e:
            env.append(f"{e['name']}={e['value']}")
    for e in opts.envs:
        env.append(f"{e['name']}={e['value']}")
    args = list(container.get("command") or []) + list(container.get("args") or [])
    mounts = [
        {"destination": "/proc", "type": "proc", "source": "proc"},
        {"destination": "/dev", "type": "tmpfs", "source": "tmpfs", "options": ["nosuid", "strictatime", "mode=755", "size=65536k"]},
        {"destination": "/sys", "type": "sysfs", "source": "sysfs", "options": ["nosuid", "noexec", "nodev", "ro"]},
    ]
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
            devs.append(di)
            rule["access"] = _access(d.get("permissions"))
            allow.append(rule)
    annotations = {a["name"]: a["value"] for a in opts.annotations}
    if missing:
        annotations["amd.com/missing-device-nodes"] = ",".join(missing)
    spec = {
        "ociVersion": "1.0.2",
        "process": {"terminal": False, "user": {"uid": 0, "gid": 0}, "args": args or ["/pause"], "env": env,
                    "cwd": container.get("workingDir") or "/",
                    "capabilities": {k: DEFAULT_CAPS for k in ("bounding", "effective", "permitted")},
                    "noNewPrivileges": True},
        "root": {"path": rootfs, "readonly": False},
        "hostname": hostname or pod["metadata"]["name"],
        "mounts": mounts,
        "annotations": annotations,
        "linux": {"devices": devs, "resources": {"devices": allow},
                  "namespaces": [{"type": t} for t in ("pid", "ipc", "uts", "mount")] +
                                ([{"type": "network", "path": f"/proc/{sandbox_pid}/ns/net"}] if sandbox_pid else [{"type": "network"}])},
    }
    if "io.kubernetes.cpuset" in annotations:   # cpu manager (static policy) exclusive cpus
        spec["linux"]["resources"]["cpu"] = {"cpus": annotations["io.kubernetes.cpuset"]}
    return spec


def _access(perm):
    perm = perm or "rw"
    return "".join(c for c in "rwm" if c in perm) or "rw"
