"""CPU manager with the static policy, aligned to the NUMA nodes of the pod's GPUs.

Parity: `pkg/kubelet/cm/cpumanager` — `policy_static.go:86-196` (shared pool = all CPUs minus
the reserved ones; a container of a Guaranteed pod with an integer CPU request gets exclusive
CPUs removed from the shared pool, returned on removal), `cpu_assignment.go:149`
(`takeByTopology`: whole sockets first, then whole physical cores, then single threads, from
the least-allocated socket), `state/state_file.go` (JSON checkpoint {policyName,
defaultCpuSet, entries}) and `topology/topology.go` (CPU → core / socket from sysfs).

MI355X addition: an 8-GPU node has GPUs on both sockets (amd.com/numa attribute from AMD SMI);
a GPU pod's exclusive CPUs are taken first from the NUMA nodes of the GPUs it was bound to, so
host threads feeding a GPU do not cross the socket interconnect.
"""
from __future__ import annotations

import glob
import json
import os
from dataclasses import dataclass


def parse_cpulist(s: str) -> list[int]:
    out = []
    for part in (s or "").strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def format_cpulist(cpus) -> str:
    cpus = sorted(set(cpus))
    out, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)


@dataclass(frozen=True)
class CPUInfo:
    cpu: int
    core: int      # globally unique physical core id
    socket: int
    numa: int


class CPUTopology:
    def __init__(self, cpus: list[CPUInfo]):
        self.cpus = {c.cpu: c for c in cpus}

    @classmethod
    def synthetic(cls, sockets=2, cores_per_socket=8, threads_per_core=2):
        out = []
        n = sockets * cores_per_socket
        for t in range(threads_per_core):
            for s in range(sockets):
                for k in range(cores_per_socket):
                    core = s * cores_per_socket + k
                    out.append(CPUInfo(t * n + core, core, s, s))
        return cls(out)

    @classmethod
    def discover(cls, sysfs="/sys/devices/system"):
        numa_of = {}
        for nd in glob.glob(os.path.join(sysfs, "node", "node[0-9]*")):
            try:
                with open(os.path.join(nd, "cpulist")) as f:
                    for c in parse_cpulist(f.read()):
                        numa_of[c] = int(os.path.basename(nd)[4:])
            except OSError:
                pass
        out = []
        allowed = set(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
        for cd in glob.glob(os.path.join(sysfs, "cpu", "cpu[0-9]*")):
            cpu = int(os.path.basename(cd)[3:])
            if allowed is not None and cpu not in allowed:
                continue
            try:
                with open(os.path.join(cd, "topology", "physical_package_id")) as f:
                    sock = int(f.read())
                with open(os.path.join(cd, "topology", "core_id")) as f:
                    core = int(f.read())
            except OSError:
                sock, core = 0, cpu
            out.append(CPUInfo(cpu, sock * 100000 + core, sock, numa_of.get(cpu, sock)))
        return cls(out or [CPUInfo(0, 0, 0, 0)])

    def cores(self, cpus):
        d = {}
        for c in cpus:
            d.setdefault(self.cpus[c].core, []).append(c)
        return d


def take_by_topology(topo: CPUTopology, available: set, n: int, prefer_numa=()):
    """`cpu_assignment.go:149` takeByTopology (topology-aware best fit), with the reference's
    `cpuAccumulator` orderings read lexicographically:

      1. whole free sockets, ascending id, while at least a socket's worth is still needed;
      2. whole free cores while at least a core's worth is needed — sockets with fewer free
         cores first (best fit), then by id;
      3. single threads, ordering cores by: most CPUs already taken by this request on the
         core's socket, fewest free CPUs on the socket, fewest free CPUs on the core (fill
         partially used cores before splitting whole ones), socket id, core id.

    MI355X addition: with `prefer_numa` (the NUMA nodes of the pod's GPUs) the CPUs are taken
    from those nodes when they can hold all n."""
    if n > len(available):
        raise ValueError("not enough cpus available to satisfy request")
    if n <= 0:
        return []
    pool = set(available)
    if prefer_numa:
        pref = {c for c in available if topo.cpus[c].numa in set(prefer_numa)}
        if len(pref) >= n:
            pool = pref
    socket_cpus, core_cpus = {}, {}
    for c in topo.cpus.values():
        socket_cpus.setdefault(c.socket, set()).add(c.cpu)
        core_cpus.setdefault(c.core, set()).add(c.cpu)
    per_socket = max(len(v) for v in socket_cpus.values())
    per_core = max(len(v) for v in core_cpus.values())
    free = set(pool)
    result: set = set()

    def take(cpus):
        nonlocal n
        result.update(cpus)
        free.difference_update(cpus)
        n -= len(cpus)

    def free_in(group):
        return group & free

    # 1) whole sockets
    for s in sorted(socket_cpus):
        if n >= per_socket and free_in(socket_cpus[s]) == socket_cpus[s] and len(socket_cpus[s]) == per_socket:
            take(socket_cpus[s])
            if n <= 0:
                return sorted(result)
    # 2) whole cores, best-fit sockets first
    if n >= per_core:
        def free_cores(s):
            return [k for k, v in core_cpus.items() if topo.cpus[next(iter(v))].socket == s
                    and len(v) == per_core and free_in(v) == v]
        for s in sorted({topo.cpus[c].socket for c in free}, key=lambda s: (len(free_cores(s)), s)):
            for k in sorted(free_cores(s)):
                if n >= per_core and free_in(core_cpus[k]) == core_cpus[k]:
                    take(core_cpus[k])
                    if n <= 0:
                        return sorted(result)
    # 3) single threads
    cores = sorted({topo.cpus[c].core for c in free}, key=lambda k: (
        -len(socket_cpus[topo.cpus[next(iter(core_cpus[k]))].socket] & result),
        len(free_in(socket_cpus[topo.cpus[next(iter(core_cpus[k]))].socket])),
        len(free_in(core_cpus[k])),
        topo.cpus[next(iter(core_cpus[k]))].socket, k))
    for k in cores:
        for c in sorted(free_in(core_cpus[k])):
            if n > 0:
                take({c})
        if n <= 0:
            return sorted(result)
    raise ValueError("failed to allocate cpus")


class StaticPolicy:
    name = "static"

    def __init__(self, topo: CPUTopology, reserved: int = 1, state_file: str | None = None):
        self.topo = topo
        all_cpus = sorted(topo.cpus)
        # reserved CPUs: taken by topology from the lowest socket like the reference
        self.reserved = set(take_by_topology(topo, set(all_cpus), min(reserved, len(all_cpus)))) if reserved else set()
        self.default = set(all_cpus) - self.reserved
        self.assignments: dict[str, list[int]] = {}      # "<pod uid>/<container>" -> cpus
        self.state_file = state_file
        self._load()

    # -- checkpoint ---------------------------------------------------------
    def _load(self):
        if not self.state_file or not os.path.exists(self.state_file):
            return
        try:
            with open(self.state_file) as f:
                st = json.load(f)
        except (OSError, ValueError):
            return
        if st.get("policyName") != self.name:
            return
        self.assignments = {k: parse_cpulist(v) for k, v in (st.get("entries") or {}).items()}
        used = {c for v in self.assignments.values() for c in v}
        self.default = (set(self.topo.cpus) - self.reserved) - used

    def _save(self):
        if not self.state_file:
            return
        tmp = self.state_file + ".tmp"
        os.makedirs(os.path.dirname(self.state_file) or ".", exist_ok=True)
        with open(tmp, "w") as f:
            json.dump({"policyName": self.name, "defaultCpuSet": format_cpulist(self.default),
                       "entries": {k: format_cpulist(v) for k, v in self.assignments.items()}}, f)
        os.replace(tmp, self.state_file)

    # -- policy -------------------------------------------------------------
    @staticmethod
    def guaranteed_cpus(pod, container) -> int:
        """Exclusive CPU count for a Guaranteed pod's container with an integer CPU request."""
        if ((pod.get("status") or {}).get("qosClass")) != "Guaranteed":
            return 0
        from ..api.quantity import parse_quantity
        res = container.get("resources") or {}
        q = (res.get("requests") or {}).get("cpu") or (res.get("limits") or {}).get("cpu")
        if q is None:
            return 0
        v = parse_quantity(str(q)).value
        return int(v) if v.denominator == 1 and v > 0 else 0

    def allocate(self, pod, container, prefer_numa=()):
        """Returns the container's cpuset (exclusive, or the shared pool)."""
        key = f"{pod['metadata']['uid']}/{container['name']}"
        if key in self.assignments:
            return self.assignments[key]
        n = self.guaranteed_cpus(pod, container)
        if n == 0:
            return sorted(self.default)
        cpus = take_by_topology(self.topo, self.default, n, prefer_numa)
        self.default -= set(cpus)
        self.assignments[key] = cpus
        self._save()
        return cpus

    def release_pod(self, uid):
        changed = False
        for key in [k for k in self.assignments if k.startswith(uid + "/")]:
            self.default |= set(self.assignments.pop(key))
            changed = True
        if changed:
            self._save()

    def shared_pool(self):
        return sorted(self.default)
