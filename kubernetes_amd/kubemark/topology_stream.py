"""Mixed-size GPU pod stream on real MI355X node shapes: can the allocator keep multi-GPU pods
placeable while 1-GPU pods churn?

A discrete-event simulation (simulated seconds, seeded) drives the REAL scheduler —
`GenericScheduler` with the default predicates/priorities, `SchedulerCache` device accounting
and the topology allocator — the way scheduler_perf drives it without kubelets
(`test/integration/scheduler_perf`). Nodes carry the device list the real `amd.com/gpu` plugin
publishes for an 8×MI355X UBB (fake AMD SMI fixture through `gpu_attributes` /
`xgmi_peer_map`): one fully connected 8-package xGMI hive, 2 NUMA nodes of 4 packages (`spx`),
or the same packages in CPX mode, 8 compute partitions each, 64 devices per node (`cpx`).

Stream: 1-device pods arrive as a Poisson process and hold their device for an exponential
lifetime; 2- and 4-GPU pods (`cpx`: 8- and 16-partition pods, one and two packages) with
`amd.com/xgmi-policy: required` arrive among them. Pending pods are retried, in priority then
arrival order, whenever a pod ends (MoveAllToActiveQueue on a delete). Offered load is set to
~85 % of the cluster's devices so placement quality decides whether multi-GPU pods wait.

Reported per shape, for the multi-device pods:
  * `wait_p50_s` / `wait_p99_s` — arrival → placement (simulated seconds);
  * `frag_wait_s_per_multi_pod` — seconds a multi-device pod waited, on average, while the
    cluster held enough free devices for it (the capacity existed, fragmented across nodes), and
    `frag_blocked_fraction`, that time's share of all their waiting (`frag_blocked_attempt_
    fraction`: the same by failed scheduling attempts);
  * `node_frag_blocked_fraction` — failed attempts while some single node had enough free
    devices (fragmentation inside a node: no valid set there);
  * `numa_fit_fraction` (spx) — placed sets inside one NUMA node;
    `min_packages_fraction` (cpx) — placed sets on the fewest packages possible.
The same stream is replayed with the reference's placement — default 1.9 priorities (spreading
LeastRequested/BalancedAllocation, no device bin-packing) and first-N device choice in device
order (`plugin/pkg/scheduler/core/extended_resources.go:42-183`) — as `reference_*`.

    python -m kubernetes_amd.kubemark.topology_stream --nodes 16 --pods 4000
"""
from __future__ import annotations

import argparse
import heapq
import json
import random
import time

from ..api import core
from ..deviceplugin.amdgpu import gpu_attributes, xgmi_peer_map
from ..native import amdsmi
from ..scheduler import priorities as PR
from ..scheduler.cache import PodInfo, SchedulerCache
from ..scheduler.generic import FitError, GenericScheduler
from ..scheduler.topology import POLICY_ANNOTATION, REQUIRED
from .density import pct

SHAPES = {
    # name: (compute partition, per-pod device counts of the multi-device stream, share of
    # arrivals that are multi-device)
    "spx": ("SPX", (2, 4), 0.12),
    "cpx": ("CPX", (8, 16), 0.06),
}

_DEVICES: dict = {}


def node_devices(partition="SPX"):
    """{device id: device} of one 8×MI355X node, as the amd.com/gpu plugin publishes it."""
    got = _DEVICES.get(partition)
    if got is None:
        smi = amdsmi.SMI(fixture=amdsmi.fixture_file(8, hives=1, partition=partition))
        gpus = smi.gpus()
        peers = xgmi_peer_map(smi, gpus)
        got = {}
        for g in gpus:
            did = g.device_id_str
            got[did] = {"id": did, "health": core.HEALTHY,
                        "attributes": gpu_attributes(g, smi.metrics(g.index), peers.get(g.index))}
        _DEVICES[partition] = got
    return got


def make_node(name, partition="SPX"):
    return {"metadata": {"name": name, "labels": {"kubernetes.io/hostname": name}}, "spec": {},
            "status": {"allocatable": {"cpu": "192", "memory": "3Ti", "pods": "512"},
                       "conditions": [{"type": "Ready", "status": "True"}],
                       "extendedResources": {core.AMD_GPU: {"resources": node_devices(partition)}}}}


def make_pod(name, n, required):
    ann = {POLICY_ANNOTATION: REQUIRED} if required else {}
    return {"metadata": {"name": name, "namespace": "topo", "uid": name, "annotations": ann},
            "spec": {"containers": [{"name": "c", "image": "x", "extendedResourceRequests": ["er"],
                                     "resources": {"requests": {"cpu": "1", "memory": "8Gi"}}}],
                     "extendedResources": [{"name": "er", "resources": {"limits": {core.AMD_GPU: str(n)},
                                                                         "requests": {core.AMD_GPU: str(n)}}}]}}


def _first_n_allocate(reqs, er, policy=None):
    """The reference allocator: the first N free devices that match, in device order, no
    topology (extended_resources.go:42-183; map order made deterministic)."""
    binding = {}
    for r in reqs:
        free = sorted(((i, d) for devs in (er.hive_free.get(r.rname) or {}).values() for i, d in devs.items()),
                      key=lambda x: int((x[1].get("attributes") or {}).get(core.ATTR_INDEX, 0)))
        if len(free) < r.count:
            return None, 0, f"Insufficient {r.rname}"
        binding[r.name] = {"resources": [i for i, _ in free[:r.count]]}
    return binding, 5.0, ""


def _stream(capacity, n_pods, sizes, multi_share, seed, load):
    """[(arrival time, pod name, devices, lifetime)] offering `load` × `capacity` devices."""
    rng = random.Random(seed)
    mean_life = 60.0                                       # 1-device pods; multi-device pods live 2x
    work = (1 - multi_share) * mean_life + multi_share * 2 * mean_life * sum(sizes) / len(sizes)
    rate = load * capacity / work                          # Little's law: busy devices = rate x device-seconds
    t, out = 0.0, []
    for i in range(n_pods):
        t += rng.expovariate(rate)
        if rng.random() < multi_share:
            n = rng.choice(sizes)
            life = rng.expovariate(1.0 / (mean_life * 2))
        else:
            n = 1
            life = rng.expovariate(1.0 / mean_life)
        out.append((t, f"p{i}", n, life))
    return out


def run_shape(shape="spx", n_nodes=16, n_pods=4000, seed=1, load=0.9, reference=False):
    partition, sizes, share = SHAPES[shape]
    names = [f"n{i:03d}" for i in range(n_nodes)]
    cache = SchedulerCache()
    for name in names:
        cache.add_node(make_node(name, partition))
    if reference:
        prios = {k: v for k, v in PR.DEFAULT_PRIORITIES.items()
                 if k not in ("XGMITopologyPriority", "GPUBinPackingPriority")}
        gs = GenericScheduler(cache, priorities=prios, equivalence_cache=False)
        import kubernetes_amd.scheduler.generic as G
        orig = (G.allocate, G.feasible, G.fast_path)
        G.allocate, G.fast_path = _first_n_allocate, (lambda reqs: False)
    else:
        gs = GenericScheduler(cache, equivalence_cache=False)
    per_node = len(node_devices(partition))
    total = n_nodes * per_node
    events = []                                   # (time, seq, kind, payload)
    seq = 0
    for t, name, n, life in _stream(total, n_pods, sizes, share, seed, load):
        events.append((t, seq, "arrive", (name, n, life)))
        seq += 1
    heapq.heapify(events)
    pending: list = []                            # (arrival, name, devices, lifetime), FIFO
    placed_multi, waits, fails, frag, node_frag = 0, [], 0, 0, 0
    topo_good = 0
    running = {}
    busy_area, last_t, t_end = 0.0, 0.0, 0.0
    wait_area = frag_area = 0.0
    # utilization over the steady part: after two lifetimes of ramp-up, until the last arrival
    arrivals = [e[0] for e in events]
    win0, win1 = min(120.0, max(arrivals) / 4), max(arrivals)
    wall0 = time.perf_counter()
    attempts = 0

    def free_total():
        return sum(ni.er.free_count(core.AMD_GPU) for ni in cache.node_list())

    def try_place(name, n, life, arrived, now):
        nonlocal seq, placed_multi, fails, frag, node_frag, topo_good, attempts
        pod = make_pod(name, n, n > 1)
        pi = PodInfo(pod)
        attempts += 1
        try:
            host, binding = gs.schedule(pod, pi)
        except FitError:
            if n > 1:
                fails += 1
                if free_total() >= n:
                    frag += 1
                if any(ni.er.free_count(core.AMD_GPU) >= n for ni in cache.node_list()):
                    node_frag += 1
            return False
        ids = binding["er"]["resources"]
        pod["spec"]["nodeName"] = host
        pod["spec"]["extendedResources"][0]["assigned"] = list(ids)
        cache.add_pod(pod)
        running[name] = pod
        heapq.heappush(events, (now + life, seq, "end", name))
        seq += 1
        if n > 1:
            placed_multi += 1
            waits.append(now - arrived)
            devs = cache.nodes[host].er.allocatable[core.AMD_GPU]
            attrs = [devs[i].get("attributes") or {} for i in ids]
            if shape == "spx":
                topo_good += len({a.get(core.ATTR_NUMA) for a in attrs}) == 1
            else:
                topo_good += len({a.get(core.ATTR_SOCKET) for a in attrs}) == -(-n // 8)
        return True

    try:
        while events:
            now, _, kind, payload = heapq.heappop(events)
            lo, hi = max(last_t, win0), min(now, win1)
            free = free_total()
            if hi > lo:
                busy_area += (total - free) * (hi - lo)
            # waiting multi-device pods: all waiting time, and the part of it during which the
            # cluster held enough free devices (the capacity existed but was fragmented)
            for ent in pending:
                if ent[2] > 1:
                    wait_area += now - last_t
                    if free >= ent[2]:
                        frag_area += now - last_t
            last_t = now
            if kind == "arrive":
                name, n, life = payload
                if not try_place(name, n, life, now, now):
                    pending.append((now, name, n, life))
            else:
                cache.remove_pod(running.pop(payload))
                if pending:
                    pending.sort()
                    keep = []
                    for ent in pending:
                        arrived, name, n, life = ent
                        if not try_place(name, n, life, arrived, now):
                            keep.append(ent)
                    pending = keep
            t_end = now
    finally:
        if reference:
            G.allocate, G.feasible, G.fast_path = orig
    multi_total = placed_multi + sum(1 for e in pending if e[2] > 1)
    out = {"nodes": n_nodes, "devices_per_node": per_node, "pods": n_pods, "multi_pods": multi_total,
           "multi_sizes": list(sizes), "offered_load": load,
           "utilization": round(busy_area / max(1e-9, (win1 - win0) * total), 3),
           "wait_p50_s": round(pct(waits, 0.5), 2), "wait_p99_s": round(pct(waits, 0.99), 2),
           "never_placed": sum(1 for e in pending if e[2] > 1),
           "failed_attempts": fails,
           "frag_blocked_attempt_fraction": round(frag / max(1, fails), 4),
           "node_frag_blocked_fraction": round(node_frag / max(1, fails), 4),
           "frag_wait_s_per_multi_pod": round(frag_area / max(1, multi_total), 2),
           "frag_blocked_fraction": round(frag_area / wait_area, 4) if wait_area else 0.0,
           "schedule_attempts": attempts, "wall_s": round(time.perf_counter() - wall0, 2)}
    key = "numa_fit_fraction" if shape == "spx" else "min_packages_fraction"
    out[key] = round(topo_good / max(1, placed_multi), 4)
    return out


def run(n_nodes=16, n_pods=4000, seed=1, load=0.85, shapes=("spx", "cpx"), reference=True):
    """Every shape gets `n_pods` arrivals; CPX nodes expose 8x the devices, so the CPX cluster
    has a quarter of the nodes (the stream then spans a comparable number of pod lifetimes)."""
    res = {}
    for s in shapes:
        nodes = n_nodes if s == "spx" else max(2, n_nodes // 4)
        r = run_shape(s, nodes, n_pods, seed, load)
        if reference:
            ref = run_shape(s, nodes, n_pods, seed, load, reference=True)
            for k in ("wait_p50_s", "wait_p99_s", "frag_blocked_fraction", "frag_wait_s_per_multi_pod",
                      "frag_blocked_attempt_fraction", "node_frag_blocked_fraction",
                      "numa_fit_fraction", "min_packages_fraction", "never_placed", "utilization"):
                if k in ref:
                    r["reference_" + k] = ref[k]
        res[s] = r
    return res


def main(argv=None):
    ap = argparse.ArgumentParser("topology-stream")
    ap.add_argument("--nodes", type=int, default=16)
    ap.add_argument("--pods", type=int, default=4000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--load", type=float, default=0.85)
    ap.add_argument("--shapes", default="spx,cpx")
    ap.add_argument("--no-reference", action="store_true")
    a = ap.parse_args(argv)
    print(json.dumps(run(a.nodes, a.pods, a.seed, a.load, tuple(a.shapes.split(",")), not a.no_reference)))


if __name__ == "__main__":
    main()
