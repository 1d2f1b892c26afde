"""iptables proxier: renders the whole ruleset as one `iptables-restore` transaction.

Parity with `pkg/proxy/iptables/proxier.go`:
  * chain names: `KUBE-SVC-` / `KUBE-SEP-` / `KUBE-FW-` / `KUBE-XLB-` + the first 16 chars of
    base32(sha256(servicePortName + protocol [+ endpoint])) (`:907-945`);
  * top-level chains KUBE-SERVICES, KUBE-NODEPORTS, KUBE-POSTROUTING, KUBE-MARK-MASQ,
    KUBE-MARK-DROP (nat) and KUBE-SERVICES, KUBE-FORWARD (filter), masquerade mark 0x4000
    (`--iptables-masquerade-bit` 14);
  * per service port: cluster-IP capture (with `! -s clusterCIDR` masquerade or
    masquerade-all), external IPs, load-balancer ingress via KUBE-FW, node ports via
    KUBE-NODEPORTS, REJECT in filter when there are no endpoints (`:1160-1440`);
  * endpoints: ClientIP affinity with `-m recent --rcheck --seconds T --reap`, random balancing
    `-m statistic --mode random --probability 1/(n-i)` with 10 decimals, hairpin masquerade and
    DNAT per endpoint chain, `externalTrafficPolicy: Local` XLB chains over local endpoints only
    (`:1444-1592`);
  * stale chains are flushed and deleted (`:1594-1608`), the NODEPORTS jump is last (`:1610-1616`);
  * syncs are rate limited by `min_sync_period` and forced every `sync_period`.
Execution is pluggable: `FakeIptables` (kubemark's hollow proxy) records the last restore
payload; `ExecIptables` pipes it into `iptables-restore --noflush --counters` when present.
"""
from __future__ import annotations

import base64
import hashlib
import shutil
import subprocess
import time

from .config import ProxyState

KUBE_SERVICES, KUBE_NODEPORTS, KUBE_POSTROUTING = "KUBE-SERVICES", "KUBE-NODEPORTS", "KUBE-POSTROUTING"
KUBE_MARK_MASQ, KUBE_MARK_DROP, KUBE_FORWARD = "KUBE-MARK-MASQ", "KUBE-MARK-DROP", "KUBE-FORWARD"


def _hash(s):
    return base64.b32encode(hashlib.sha256(s.encode()).digest()).decode()[:16]


def svc_chain(spn, proto):
    return "KUBE-SVC-" + _hash(str(spn) + proto.lower())


def fw_chain(spn, proto):
    return "KUBE-FW-" + _hash(str(spn) + proto.lower())


def xlb_chain(spn, proto):
    return "KUBE-XLB-" + _hash(str(spn) + proto.lower())


def sep_chain(spn, proto, endpoint):
    return "KUBE-SEP-" + _hash(str(spn) + proto.lower() + endpoint)


def probability(n):
    return "%0.10f" % (1.0 / n)


def _cidr(ip):
    return ip if "/" in ip else ip + "/32"


class FakeIptables:
    def __init__(self):
        self.restores = []
        self.last = ""

    def restore_all(self, data: str):
        self.last = data
        self.restores.append(data)

    def save(self):
        return self.last


class ExecIptables:
    def __init__(self, binary="iptables-restore"):
        self.binary = shutil.which(binary)
        if not self.binary:
            raise FileNotFoundError(f"{binary} not found")

    def restore_all(self, data: str):
        subprocess.run([self.binary, "--noflush", "--counters"], input=data.encode(), check=True)


class IptablesProxier:
    def __init__(self, state: ProxyState, iptables=None, cluster_cidr="", masquerade_all=False, masquerade_bit=14,
                 min_sync_period=0.0, node_ips=("127.0.0.1",), recorder=None):
        self.state = state
        self.iptables = iptables or FakeIptables()
        self.cluster_cidr = cluster_cidr
        self.masquerade_all = masquerade_all
        self.mark = "0x%08x/0x%08x" % (1 << masquerade_bit, 1 << masquerade_bit)
        self.min_sync_period = min_sync_period
        self.node_ips = list(node_ips)
        self.last_sync = 0.0
        self.syncs = 0
        self.rules = 0
        self._prev_nat_chains: set = set()

    def sync(self, force=False):
        now = time.monotonic()
        if not force and now - self.last_sync < self.min_sync_period:
            return False
        data = self.render()
        self.iptables.restore_all(data)
        self.last_sync = now
        self.syncs += 1
        return True

    def render(self) -> str:
        st = self.state
        filter_chains = [KUBE_SERVICES, KUBE_FORWARD]
        nat_chains = [KUBE_SERVICES, KUBE_NODEPORTS, KUBE_POSTROUTING, KUBE_MARK_MASQ, KUBE_MARK_DROP]
        filter_rules, nat_rules = [], []
        nat_rules.append(f'-A {KUBE_POSTROUTING} -m comment --comment "kubernetes service traffic requiring SNAT" '
                         f"-m mark --mark {self.mark} -j MASQUERADE")
        nat_rules.append(f"-A {KUBE_MARK_MASQ} -j MARK --set-xmark {self.mark}")
        nat_rules.append(f"-A {KUBE_MARK_DROP} -j MARK --set-xmark 0x00008000/0x00008000")
        for spn in sorted(st.services, key=str):
            info = st.services[spn]
            proto = info.protocol.lower()
            name = str(spn)
            eps = st.endpoints.get(spn) or []
            svc = svc_chain(spn, proto)
            has_eps = bool(eps)
            if has_eps:
                nat_chains.append(svc)
            xlb = xlb_chain(spn, proto)
            if info.only_local:
                nat_chains.append(xlb)
            base = (f'-A {KUBE_SERVICES} -m comment --comment "{name} cluster IP" -m {proto} -p {proto} '
                    f"-d {_cidr(info.cluster_ip)} --dport {info.port}")
            if has_eps:
                if self.masquerade_all:
                    nat_rules.append(f"{base} -j {KUBE_MARK_MASQ}")
                elif self.cluster_cidr:
                    nat_rules.append(f"{base} ! -s {self.cluster_cidr} -j {KUBE_MARK_MASQ}")
                nat_rules.append(f"{base} -j {svc}")
            else:
                filter_rules.append(f'-A {KUBE_SERVICES} -m comment --comment "{name} has no endpoints" -m {proto} '
                                    f"-p {proto} -d {_cidr(info.cluster_ip)} --dport {info.port} -j REJECT")
            for ext in info.external_ips:
                eb = (f'-A {KUBE_SERVICES} -m comment --comment "{name} external IP" -m {proto} -p {proto} '
                      f"-d {_cidr(ext)} --dport {info.port}")
                if has_eps:
                    nat_rules.append(f"{eb} -j {KUBE_MARK_MASQ}")
                    nat_rules.append(f"{eb} -m physdev ! --physdev-is-in -m addrtype ! --src-type LOCAL -j {svc}")
                    nat_rules.append(f"{eb} -m addrtype --dst-type LOCAL -j {svc}")
                else:
                    filter_rules.append(f'-A {KUBE_SERVICES} -m comment --comment "{name} has no endpoints" -m {proto} '
                                        f"-p {proto} -d {_cidr(ext)} --dport {info.port} -j REJECT")
            if has_eps and info.load_balancer_ips:
                fw = fw_chain(spn, proto)
                nat_chains.append(fw)
                target = xlb if info.only_local else svc
                for lb in info.load_balancer_ips:
                    nat_rules.append(f'-A {KUBE_SERVICES} -m comment --comment "{name} loadbalancer IP" -m {proto} '
                                     f"-p {proto} -d {_cidr(lb)} --dport {info.port} -j {fw}")
                    if not info.load_balancer_source_ranges:
                        if not info.only_local:
                            nat_rules.append(f'-A {fw} -m comment --comment "{name} loadbalancer IP" -j {KUBE_MARK_MASQ}')
                        nat_rules.append(f'-A {fw} -m comment --comment "{name} loadbalancer IP" -j {target}')
                    else:
                        for src in info.load_balancer_source_ranges:
                            nat_rules.append(f'-A {fw} -m comment --comment "{name} loadbalancer IP" -s {src} -j {target}')
                    nat_rules.append(f'-A {fw} -m comment --comment "{name} loadbalancer IP" -j {KUBE_MARK_DROP}')
            if info.node_port:
                nb = f'-A {KUBE_NODEPORTS} -m comment --comment "{name}" -m {proto} -p {proto} --dport {info.node_port}'
                if has_eps:
                    if info.only_local:
                        nat_rules.append(f"{nb} -s 127.0.0.0/8 -j {KUBE_MARK_MASQ}")
                        nat_rules.append(f"{nb} -j {xlb}")
                    else:
                        nat_rules.append(f"{nb} -j {KUBE_MARK_MASQ}")
                        nat_rules.append(f"{nb} -j {svc}")
                else:
                    filter_rules.append(f'-A {KUBE_SERVICES} -m comment --comment "{name} has no endpoints" '
                                        f"-m addrtype --dst-type LOCAL -m {proto} -p {proto} --dport {info.node_port} -j REJECT")
            if not has_eps:
                continue
            seps = [sep_chain(spn, proto, e.endpoint) for e in eps]
            nat_chains.extend(seps)
            if info.session_affinity == "ClientIP":
                for c in seps:
                    nat_rules.append(f"-A {svc} -m comment --comment {name} -m recent --name {c} --rcheck "
                                     f"--seconds {info.sticky_seconds} --reap -j {c}")
            n = len(seps)
            for i, (e, c) in enumerate(zip(eps, seps)):
                r = f"-A {svc} -m comment --comment {name}"
                if i < n - 1:
                    r += f" -m statistic --mode random --probability {probability(n - i)}"
                nat_rules.append(f"{r} -j {c}")
                pre = f"-A {c} -m comment --comment {name}"
                nat_rules.append(f"{pre} -s {_cidr(e.ip)} -j {KUBE_MARK_MASQ}")
                rec = f" -m recent --name {c} --set" if info.session_affinity == "ClientIP" else ""
                nat_rules.append(f"{pre}{rec} -m {proto} -p {proto} -j DNAT --to-destination {e.endpoint}")
            if info.only_local:
                local = [(e, c) for e, c in zip(eps, seps) if e.is_local]
                if self.cluster_cidr:
                    nat_rules.append(f'-A {xlb} -m comment --comment "Redirect pods trying to reach external loadbalancer VIP '
                                     f'to clusterIP" -s {self.cluster_cidr} -j {svc}')
                if not local:
                    nat_rules.append(f'-A {xlb} -m comment --comment "{name} has no local endpoints" -j {KUBE_MARK_DROP}')
                else:
                    if info.session_affinity == "ClientIP":
                        for _, c in local:
                            nat_rules.append(f"-A {xlb} -m comment --comment {name} -m recent --name {c} --rcheck "
                                             f"--seconds {info.sticky_seconds} --reap -j {c}")
                    m = len(local)
                    for i, (_, c) in enumerate(local):
                        r = f'-A {xlb} -m comment --comment "Balancing rule {i} for {name}"'
                        if i < m - 1:
                            r += f" -m statistic --mode random --probability {probability(m - i)}"
                        nat_rules.append(f"{r} -j {c}")
        nat_rules.append(f'-A {KUBE_SERVICES} -m comment --comment "kubernetes service nodeports; NOTE: this must be the '
                         f'last rule in this chain" -m addrtype --dst-type LOCAL -j {KUBE_NODEPORTS}')
        filter_rules.append(f'-A {KUBE_FORWARD} -m comment --comment "kubernetes forwarding rules" -m mark --mark {self.mark} -j ACCEPT')
        if self.cluster_cidr:
            filter_rules.append(f'-A {KUBE_FORWARD} -s {self.cluster_cidr} -m comment --comment "kubernetes forwarding conntrack '
                                f'pod source rule" -m conntrack --ctstate RELATED,ESTABLISHED -j ACCEPT')
            filter_rules.append(f'-A {KUBE_FORWARD} -m comment --comment "kubernetes forwarding conntrack pod destination rule" '
                                f"-d {self.cluster_cidr} -m conntrack --ctstate RELATED,ESTABLISHED -j ACCEPT")
        # chains of services / endpoints that went away: flush (chain line) and delete (-X)
        active = set(nat_chains)
        stale = sorted(c for c in self._prev_nat_chains - active
                       if c.startswith(("KUBE-SVC-", "KUBE-SEP-", "KUBE-FW-", "KUBE-XLB-")))
        self._prev_nat_chains = active
        nat_chains += stale
        nat_rules += [f"-X {c}" for c in stale]
        self.rules = len(nat_rules) + len(filter_rules)
        out = ["*filter"] + [f":{c} - [0:0]" for c in filter_chains] + filter_rules + ["COMMIT", "*nat"]
        seen = set()
        for c in nat_chains:
            if c not in seen:
                seen.add(c)
                out.append(f":{c} - [0:0]")
        out += nat_rules + ["COMMIT", ""]
        return "\n".join(out)
