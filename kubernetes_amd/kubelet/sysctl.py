"""Pod sysctls admission (`pkg/kubelet/sysctl/whitelist.go`, Kubernetes 1.9 alpha API).

Sysctls are requested through two pod annotations of comma-separated `name=value` pairs:
`security.alpha.kubernetes.io/sysctls` (safe ones) and
`security.alpha.kubernetes.io/unsafe-sysctls`. A pod is admitted only if
  * every safe sysctl is on the safe whitelist (kernel.shm_rmid_forced,
    net.ipv4.ip_local_port_range, net.ipv4.tcp_syncookies);
  * every unsafe sysctl matches `--experimental-allowed-unsafe-sysctls` (exact names or
    `prefix*` patterns);
  * every sysctl is namespaced (kernel.shm*, kernel.msg*, kernel.sem, fs.mqueue.*, net.*), and
    not in a namespace the pod shares with the host (net.* with hostNetwork; the IPC group with
    hostIPC).
Otherwise the pod is rejected with reason `SysctlForbidden`. The accepted sysctls go to the
sandbox (CRI `LinuxPodSandboxConfig.sysctls`).
"""
from __future__ import annotations

SAFE_ANNOTATION = "security.alpha.kubernetes.io/sysctls"
UNSAFE_ANNOTATION = "security.alpha.kubernetes.io/unsafe-sysctls"
SAFE_SYSCTLS = ("kernel.shm_rmid_forced", "net.ipv4.ip_local_port_range", "net.ipv4.tcp_syncookies")
REASON = "SysctlForbidden"

# namespaced sysctl groups (`pkg/kubelet/sysctl/namespace.go`)
_IPC = ("kernel.shmall", "kernel.shmmax", "kernel.shmmni", "kernel.shm_rmid_forced", "kernel.msgmax",
        "kernel.msgmnb", "kernel.msgmni", "kernel.sem")
_IPC_PREFIX = ("fs.mqueue.",)
_NET_PREFIX = ("net.",)


def parse(annotation_value: str | None) -> dict:
    out = {}
    for kv in (annotation_value or "").split(","):
        kv = kv.strip()
        if not kv:
            continue
        k, sep, v = kv.partition("=")
        if not sep or not k:
            raise ValueError(f"sysctl {kv!r} not of the format sysctl_name=value")
        out[k.strip()] = v.strip()
    return out


def namespace_of(name: str) -> str | None:
    if name in _IPC or name.startswith(_IPC_PREFIX):
        return "ipc"
    if name.startswith(_NET_PREFIX):
        return "net"
    return None


class Whitelist:
    def __init__(self, patterns, annotation):
        self.exact, self.prefixes = set(), []
        for p in patterns:
            if p.endswith("*"):
                base = p[:-1]
                if namespace_of(base + "x") is None and not base.startswith(("kernel.shm", "kernel.msg")):
                    raise ValueError(f"sysctl pattern {p!r} is not known to be namespaced")
                self.prefixes.append(base)
            else:
                if namespace_of(p) is None:
                    raise ValueError(f"sysctl {p!r} is not known to be namespaced")
                self.exact.add(p)
        self.annotation = annotation

    def allowed(self, name) -> bool:
        return name in self.exact or any(name.startswith(p) for p in self.prefixes)

    def validate(self, pod) -> str | None:
        md = pod.get("metadata") or {}
        spec = pod.get("spec") or {}
        try:
            sysctls = parse((md.get("annotations") or {}).get(self.annotation))
        except ValueError as e:
            return str(e)
        for name in sysctls:
            ns = namespace_of(name)
            if ns is None:
                return f"sysctl {name!r} is not known to be namespaced"
            if ns == "net" and spec.get("hostNetwork"):
                return f"sysctl {name!r} not allowed with host net enabled"
            if ns == "ipc" and spec.get("hostIPC"):
                return f"sysctl {name!r} not allowed with host ipc enabled"
            if not self.allowed(name):
                return f"{self.annotation} {name!r} not whitelisted"
        return None


class SysctlAdmitHandler:
    """Kubelet admit handler: the safe whitelist, plus the operator's unsafe patterns."""

    def __init__(self, allowed_unsafe=()):
        self.safe = Whitelist(SAFE_SYSCTLS, SAFE_ANNOTATION)
        self.unsafe = Whitelist(list(allowed_unsafe), UNSAFE_ANNOTATION)

    def admit(self, pod):
        for wl in (self.safe, self.unsafe):
            msg = wl.validate(pod)
            if msg:
                return REASON, msg
        return None

    @staticmethod
    def pod_sysctls(pod) -> dict:
        ann = (pod.get("metadata") or {}).get("annotations") or {}
        out = {}
        for key in (SAFE_ANNOTATION, UNSAFE_ANNOTATION):
            try:
                out.update(parse(ann.get(key)))
            except ValueError:
                pass
        return out
