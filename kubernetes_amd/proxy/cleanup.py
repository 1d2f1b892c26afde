"""kube-proxy host state outside the service rules: `--cleanup` and the conntrack table.

Parity:
* `pkg/proxy/iptables/proxier.go` CleanupLeftovers (+ ipvs / userspace): remove every jump into
  a KUBE-* chain from the built-in chains, then flush and delete the KUBE-* chains, in the nat
  and filter tables. Done as one `iptables-save` -> filtered -> `iptables-restore` per table so
  no half-cleaned state is ever visible; IPVS: `ipvsadm --clear` and the kube-ipvs0 dummy device;
* `cmd/kube-proxy/app/conntrack.go` + `server.go`: nf_conntrack_max = max(per-core x CPUs, min)
  (and the hash table at max/4), the established-TCP timeout, written under /proc (a `root`
  prefix makes it testable).
"""
from __future__ import annotations

import logging
import os
import shutil
import subprocess

log = logging.getLogger("kube-proxy")
BUILTIN = {"PREROUTING", "INPUT", "FORWARD", "OUTPUT", "POSTROUTING"}


def strip_kube_rules(save_text: str) -> str:
    """An `iptables-save` dump without KUBE-* chains and without rules that jump into them."""
    out = []
    for line in save_text.splitlines():
        s = line.strip()
        if s.startswith(":KUBE-"):
            continue                                     # chain declaration
        if s.startswith("-A "):
            parts = s.split()
            chain = parts[1] if len(parts) > 1 else ""
            if chain.startswith("KUBE-"):
                continue                                 # a rule inside a KUBE chain
            if "-j" in parts and parts.index("-j") + 1 < len(parts) and parts[parts.index("-j") + 1].startswith("KUBE-"):
                continue                                 # a jump into one
            if "-g" in parts and parts.index("-g") + 1 < len(parts) and parts[parts.index("-g") + 1].startswith("KUBE-"):
                continue
        out.append(line)
    return "\n".join(out) + "\n"


def cleanup_iptables(run=subprocess.run) -> bool:
    save, restore = shutil.which("iptables-save"), shutil.which("iptables-restore")
    if not save or not restore:
        log.warning("iptables-save/iptables-restore not found: nothing to clean")
        return False
    for table in ("nat", "filter"):
        dump = run([save, "-t", table], capture_output=True, text=True, check=True).stdout
        run([restore], input=strip_kube_rules(dump), text=True, check=True)
    return True


def cleanup_ipvs(run=subprocess.run) -> bool:
    ipvsadm, ip = shutil.which("ipvsadm"), shutil.which("ip")
    ok = False
    if ipvsadm:
        run([ipvsadm, "--clear"], check=False)
        ok = True
    if ip:
        run([ip, "link", "del", "kube-ipvs0"], check=False, capture_output=True)
    return ok


def conntrack_max(per_core: int, minimum: int, cpus: int | None = None) -> int:
    if per_core <= 0:
        return 0
    return max(per_core * (cpus or os.cpu_count() or 1), minimum)


def set_conntrack(max_entries: int, tcp_established_timeout: int, root="/") -> list[str]:
    """Write the conntrack tunables; -> the settings that could not be written (logged)."""
    failed = []
    writes = []
    if max_entries > 0:
        writes += [("proc/sys/net/netfilter/nf_conntrack_max", max_entries),
                   ("sys/module/nf_conntrack/parameters/hashsize", max(1, max_entries // 4))]
    if tcp_established_timeout > 0:
        writes.append(("proc/sys/net/netfilter/nf_conntrack_tcp_timeout_established", tcp_established_timeout))
    for rel, v in writes:
        path = os.path.join(root, rel)
        try:
            with open(path) as f:
                if int(f.read().strip() or 0) >= v and "hashsize" in rel:
                    continue                             # never shrink the hash table
        except (OSError, ValueError):
            pass
        try:
            with open(path, "w") as f:
                f.write(str(v))
        except OSError as e:
            log.warning("conntrack: could not set %s=%s: %s", rel, v, e)
            failed.append(rel)
    return failed
