"""IPVS proxier: virtual servers for every service address, real servers for every endpoint.

Parity: `pkg/proxy/ipvs/proxier.go` (1.9, alpha): for each service port a virtual server on
the cluster IP (address bound to the dummy interface `kube-ipvs0`), one per external IP /
load-balancer ingress, and one per node IP for node ports; scheduler `--ipvs-scheduler`
(default `rr`); ClientIP affinity = IPVS persistence with the affinity timeout; real servers =
ready endpoints with weight 1, masquerade forwarding; the sync diffs desired vs current state
(add / update / delete virtual and real servers, unbind addresses no longer used:
`syncService`, `syncEndpoint`, `cleanLegacyService`). Masquerading of off-cluster traffic
stays in iptables (KUBE-POSTROUTING / KUBE-MARK-MASQ), like the reference.

`FakeIPVS` is the kernel-state double (the reference's `ipvs/testing/fake.go`); `ExecIPVS`
applies `ipvsadm -R` batches when `ipvsadm` is installed.
"""
from __future__ import annotations

import shutil
import subprocess
import time
from dataclasses import dataclass, field

from .config import ProxyState

DUMMY_DEV = "kube-ipvs0"


@dataclass(frozen=True)
class VSKey:
    address: str
    port: int
    protocol: str     # TCP / UDP


@dataclass
class VirtualServer:
    key: VSKey
    scheduler: str = "rr"
    persistent_timeout: int = 0
    reals: dict = field(default_factory=dict)   # "ip:port" -> weight


class FakeIPVS:
    def __init__(self):
        self.services: dict[VSKey, VirtualServer] = {}
        self.bound: set = set()
        self.ops = []

    def apply(self, ops):
        for op in ops:
            self.ops.append(op)
            kind = op[0]
            if kind == "add-vs" or kind == "edit-vs":
                vs = op[1]
                cur = self.services.get(vs.key)
                reals = cur.reals if cur else {}
                self.services[vs.key] = VirtualServer(vs.key, vs.scheduler, vs.persistent_timeout, dict(reals))
            elif kind == "del-vs":
                self.services.pop(op[1], None)
            elif kind == "add-rs":
                self.services[op[1]].reals[op[2]] = op[3]
            elif kind == "del-rs":
                self.services[op[1]].reals.pop(op[2], None)
            elif kind == "bind":
                self.bound.add(op[1])
            elif kind == "unbind":
                self.bound.discard(op[1])


def _flag(proto):
    return "-u" if proto == "UDP" else "-t"


class ExecIPVS(FakeIPVS):
    def __init__(self):
        super().__init__()
        self.ipvsadm = shutil.which("ipvsadm")
        self.ip = shutil.which("ip")
        if not self.ipvsadm:
            raise FileNotFoundError("ipvsadm not found")

    def apply(self, ops):
        lines = []
        for op in ops:
            kind = op[0]
            if kind in ("add-vs", "edit-vs"):
                vs = op[1]
                a = f"{'-A' if kind == 'add-vs' else '-E'} {_flag(vs.key.protocol)} {vs.key.address}:{vs.key.port} -s {vs.scheduler}"
                if vs.persistent_timeout:
                    a += f" -p {vs.persistent_timeout}"
                lines.append(a)
            elif kind == "del-vs":
                lines.append(f"-D {_flag(op[1].protocol)} {op[1].address}:{op[1].port}")
            elif kind == "add-rs":
                lines.append(f"-a {_flag(op[1].protocol)} {op[1].address}:{op[1].port} -r {op[2]} -m -w {op[3]}")
            elif kind == "del-rs":
                lines.append(f"-d {_flag(op[1].protocol)} {op[1].address}:{op[1].port} -r {op[2]}")
            elif kind in ("bind", "unbind") and self.ip:
                subprocess.run([self.ip, "addr", "add" if kind == "bind" else "del", f"{op[1]}/32", "dev", DUMMY_DEV],
                               check=False, capture_output=True)
        if lines:
            subprocess.run([self.ipvsadm, "-R"], input=("\n".join(lines) + "\n").encode(), check=True)
        super().apply(ops)


class IPVSProxier:
    def __init__(self, state: ProxyState, ipvs=None, scheduler="rr", node_ips=("127.0.0.1",), min_sync_period=0.0):
        self.state = state
        self.ipvs = ipvs or FakeIPVS()
        self.scheduler = scheduler
        self.node_ips = list(node_ips)
        self.min_sync_period = min_sync_period
        self.last_sync = 0.0
        self.syncs = 0
        self.last_ops = []

    def desired(self):
        want: dict[VSKey, VirtualServer] = {}
        bind = set()
        for spn, info in self.state.services.items():
            pt = info.sticky_seconds if info.session_affinity == "ClientIP" else 0
            reals = {e.endpoint: 1 for e in self.state.endpoints.get(spn) or ()}
            local_reals = {e.endpoint: 1 for e in self.state.endpoints.get(spn) or () if e.is_local}
            addrs = [(info.cluster_ip, info.port, reals)]
            bind.add(info.cluster_ip)
            for ip in info.external_ips + info.load_balancer_ips:
                addrs.append((ip, info.port, local_reals if info.only_local else reals))
                bind.add(ip)
            if info.node_port:
                for nip in self.node_ips:
                    addrs.append((nip, info.node_port, local_reals if info.only_local else reals))
            for ip, port, rs in addrs:
                k = VSKey(ip, port, info.protocol)
                want[k] = VirtualServer(k, self.scheduler, pt, dict(rs))
        return want, bind

    def sync(self, force=False):
        now = time.monotonic()
        if not force and now - self.last_sync < self.min_sync_period:
            return False
        want, bind = self.desired()
        cur = self.ipvs.services
        ops = []
        for a in sorted(bind - self.ipvs.bound):
            ops.append(("bind", a))
        for k, vs in want.items():
            c = cur.get(k)
            if c is None:
                ops.append(("add-vs", vs))
                ops += [("add-rs", k, r, w) for r, w in sorted(vs.reals.items())]
                continue
            if (c.scheduler, c.persistent_timeout) != (vs.scheduler, vs.persistent_timeout):
                ops.append(("edit-vs", vs))
            ops += [("add-rs", k, r, w) for r, w in sorted(vs.reals.items()) if c.reals.get(r) != w]
            ops += [("del-rs", k, r) for r in sorted(c.reals) if r not in vs.reals]
        for k in sorted(set(cur) - set(want), key=lambda k: (k.address, k.port, k.protocol)):
            ops.append(("del-vs", k))
        node_ips = set(self.node_ips)
        for a in sorted(self.ipvs.bound - bind - node_ips):
            ops.append(("unbind", a))
        self.ipvs.apply(ops)
        self.last_ops = ops
        self.last_sync = now
        self.syncs += 1
        return True
