"""Pod and QoS cgroups (`pkg/kubelet/cm`: `qos_container_manager_linux.go`,
`pod_container_manager_linux.go`, `helpers_linux.go`, `node_container_manager.go`).

Hierarchy under the kubelet's cgroup root (cgroup v2 file names):

    <root>/kubepods/                      node allocatable: cpu.weight, memory.max
    <root>/kubepods/pod<uid>/             Guaranteed pods
    <root>/kubepods/burstable/            cpu.weight = Σ Burstable pods' cpu requests
    <root>/kubepods/burstable/pod<uid>/
    <root>/kubepods/besteffort/           cpu.weight of the minimum 2 shares
    <root>/kubepods/besteffort/pod<uid>/

A pod cgroup carries `ResourceConfigForPod`: cpu shares from the summed cpu requests (min 2),
a cpu quota only when every container has a cpu limit (period 100 ms, min 1 ms), and a memory
limit only when every container has one; BestEffort pods get the minimum shares. Shares are
written as cgroup v2 weights (`1 + (shares-2)*9999/262142`, the runc conversion). Each container
runs in its own leaf `<pod>/ctr-<id>/` created by the runtime (container-init / kamd-runc): cgroup
v2's no-internal-process rule forbids processes in the pod cgroup once it delegates cpu and memory
to its children, so the pod cgroup never holds a process itself.

`root` can be a real delegated cgroup v2 directory (the kubelet then enables the cpu and
memory controllers for its children) or any directory (tests, or hosts where the kubelet may not
manage cgroups: the files are written as a record of the intended limits).
"""
from __future__ import annotations

import logging
import os
import shutil

from ..api import core
from ..api.quantity import parse_quantity
from .qos import BEST_EFFORT, BURSTABLE, GUARANTEED, pod_qos

log = logging.getLogger("kubelet.cgroups")

MIN_SHARES, MAX_SHARES, SHARES_PER_CPU = 2, 262144, 1024
QUOTA_PERIOD_US, MIN_QUOTA_US = 100_000, 1000


def milli_cpu_to_shares(milli: int) -> int:
    if milli == 0:
        return MIN_SHARES
    return max(MIN_SHARES, min(MAX_SHARES, milli * SHARES_PER_CPU // 1000))


def milli_cpu_to_quota(milli: int, period=QUOTA_PERIOD_US) -> int:
    if milli == 0:
        return 0
    return max(MIN_QUOTA_US, milli * period // 1000)


def shares_to_weight(shares: int) -> int:
    return 1 + ((max(MIN_SHARES, shares) - 2) * 9999) // 262142


def _limits(c):
    return (c.get("resources") or {}).get("limits") or {}


def resource_config_for_pod(pod) -> dict:
    """{"cpu_shares", "cpu_quota" (µs or None), "memory_limit" (bytes or None)}."""
    spec = pod.get("spec") or {}
    conts = list(spec.get("containers") or ())
    req = core.pod_requests(pod)
    cpu_req = req["cpu"].milli_value() if "cpu" in req else 0
    cpu_lim = mem_lim = 0
    all_cpu = all_mem = bool(conts)
    for c in conts:
        lim = _limits(c)
        if "cpu" in lim:
            cpu_lim += parse_quantity(str(lim["cpu"])).milli_value()
        else:
            all_cpu = False
        if "memory" in lim:
            mem_lim += parse_quantity(str(lim["memory"])).value
        else:
            all_mem = False
    # an init container's limit can exceed the sum of the app containers'
    for c in spec.get("initContainers") or ():
        lim = _limits(c)
        if "cpu" in lim:
            cpu_lim = max(cpu_lim, parse_quantity(str(lim["cpu"])).milli_value())
        if "memory" in lim:
            mem_lim = max(mem_lim, parse_quantity(str(lim["memory"])).value)
    q = pod_qos(pod)
    if q == BEST_EFFORT:
        return {"cpu_shares": MIN_SHARES, "cpu_quota": None, "memory_limit": None}
    cfg = {"cpu_shares": milli_cpu_to_shares(cpu_req), "cpu_quota": None, "memory_limit": None}
    if q == GUARANTEED or all_cpu:
        cfg["cpu_quota"] = milli_cpu_to_quota(cpu_lim)
    if q == GUARANTEED or all_mem:
        cfg["memory_limit"] = mem_lim
    return cfg


class CgroupManager:
    def __init__(self, root, node_allocatable=None, cpu_cfs_quota=True):
        self.root = os.path.abspath(root)
        self.cpu_cfs_quota = cpu_cfs_quota        # False: cpu limits are not enforced (no cpu.max)
        self.kubepods = os.path.join(self.root, "kubepods")
        self.node_allocatable = node_allocatable or {}      # {"cpu": milli, "memory": bytes}
        self.pods: dict[str, tuple] = {}                     # uid -> (qos, path, pod)
        self.real = os.path.exists(os.path.join(self.root, "cgroup.controllers"))

    # -- files ---------------------------------------------------------------
    def _write(self, d, name, value):
        p = os.path.join(d, name)
        try:
            if self.real and not os.path.exists(p) and name not in ("cgroup.procs", "cgroup.subtree_control"):
                return False                                 # controller not enabled here
            with open(p, "w") as f:
                f.write(str(value))
            return True
        except OSError as e:
            log.debug("cgroup write %s=%s failed: %s", p, value, e)
            return False

    def _mkdir(self, d):
        os.makedirs(d, exist_ok=True)
        if self.real:
            # delegate cpu + memory to children (cgroup v2: a parent enables controllers)
            self._write(os.path.dirname(d), "cgroup.subtree_control", "+cpu +memory")
            self._write(d, "cgroup.subtree_control", "+cpu +memory")

    def _apply(self, d, shares, quota=None, mem=None):
        self._write(d, "cpu.weight", shares_to_weight(shares))
        self._write(d, "cpu.max", f"{quota} {QUOTA_PERIOD_US}" if quota else f"max {QUOTA_PERIOD_US}")
        self._write(d, "memory.max", str(mem) if mem else "max")

    # -- QoS level -----------------------------------------------------------
    def start(self):
        """`qosContainerManager.Start` + node allocatable enforcement on kubepods."""
        for d in (self.kubepods, self.qos_dir(BURSTABLE), self.qos_dir(BEST_EFFORT)):
            self._mkdir(d)
        cpu = self.node_allocatable.get("cpu", 0)
        self._apply(self.kubepods, milli_cpu_to_shares(cpu) if cpu else MAX_SHARES, None,
                    self.node_allocatable.get("memory") or None)
        self._apply(self.qos_dir(BEST_EFFORT), MIN_SHARES)
        self.update_qos()
        return self

    def qos_dir(self, qos):
        return self.kubepods if qos == GUARANTEED else os.path.join(self.kubepods, qos.lower())

    def update_qos(self):
        """`UpdateCgroups`: the Burstable cgroup's shares follow its pods' cpu requests."""
        milli = 0
        for q, _, pod in self.pods.values():
            if q == BURSTABLE:
                r = core.pod_requests(pod)
                milli += r["cpu"].milli_value() if "cpu" in r else 0
        self._write(self.qos_dir(BURSTABLE), "cpu.weight", shares_to_weight(milli_cpu_to_shares(milli)))

    # -- pod level -----------------------------------------------------------
    def pod_dir(self, pod):
        uid = pod["metadata"]["uid"]
        ent = self.pods.get(uid)
        return ent[1] if ent else os.path.join(self.qos_dir(pod_qos(pod)), f"pod{uid}")

    def ensure_pod(self, pod):
        uid = pod["metadata"]["uid"]
        q = pod_qos(pod)
        d = os.path.join(self.qos_dir(q), f"pod{uid}")
        if uid not in self.pods:
            self._mkdir(d)
            cfg = resource_config_for_pod(pod)
            self._apply(d, cfg["cpu_shares"], cfg["cpu_quota"] if self.cpu_cfs_quota else None, cfg["memory_limit"])
            self.pods[uid] = (q, d, pod)
            if q == BURSTABLE:
                self.update_qos()
        return d

    def add_process(self, pod_uid, pid) -> bool:
        ent = self.pods.get(pod_uid)
        return bool(ent) and self._write(ent[1], "cgroup.procs", pid)

    def destroy_pod(self, pod_uid):
        ent = self.pods.pop(pod_uid, None)
        if not ent:
            return
        q, d, _ = ent
        if self.real:
            # container cgroups (leaves the runtime created under the pod) go first
            try:
                for name in os.listdir(d):
                    if name.startswith("ctr-") and os.path.isdir(os.path.join(d, name)):
                        try:
                            os.rmdir(os.path.join(d, name))
                        except OSError as e:
                            log.warning("removing container cgroup %s/%s: %s", d, name, e)
            except OSError:
                pass
            try:
                os.rmdir(d)          # a cgroup directory is removed with rmdir once empty
            except OSError as e:
                log.warning("removing pod cgroup %s: %s", d, e)
        else:
            shutil.rmtree(d, ignore_errors=True)
        if q == BURSTABLE:
            self.update_qos()

    def read(self, d, name):
        try:
            with open(os.path.join(d, name)) as f:
                return f.read().strip()
        except OSError:
            return None
