#!/usr/bin/env python3
"""Flagship benchmark: GPU pods/sec + pod-startup latency, kubemark density on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Setup (BASELINE.json: "GPU pods/sec scheduled + p50 pod-startup latency, 8xMI355X kubemark density"):
  * rank 0 starts the control plane as separate processes — kube-apiserver (embedded MVCC
    store) and kube-scheduler — before anything touches the GPU;
  * every rank (one per GPU) hosts `--nodes-per-rank` kubemark hollow nodes, each a real kubelet
    with the real DeviceManager and an amd.com/gpu device plugin over gRPC advertising 8 MI355X
    (fake AMD SMI fixture, one xGMI hive), and a stub container runtime whose GPU containers run
    a real HIP vector_add payload on the rank's own MI355X at container start;
  * every rank generates load for its share: `8 x nodes-per-rank` single-GPU pods per step
    (weak scaling: per-GPU work is fixed), created through the API (ResourceV2 admission),
    scheduled with device IDs, admitted by the kubelet, started, observed Running on a watch,
    then deleted (graceful; kubelet finalizes) and observed gone — one step = one full
    saturation/churn cycle of the rank's share of the cluster.
`value` = total pods / wall time over all ranks (max over ranks). Startup latency percentiles
are over every pod of the timed steps. Data: synthetic pods, stub containers.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "GPU pods/sec scheduled + p50 pod-startup latency, 8×MI355X kubemark density"
BASELINE_DENSITY_PODS_PER_S = 8.0        # test/e2e/scalability/density.go:55-57 (MinPodsPerSecondThroughput)
BASELINE_SCHED_WARN_PODS_PER_S = 100.0   # test/integration/scheduler_perf/scheduler_test.go:35-36


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _xgmi4_summary(allstats):
    from kubernetes_amd.kubemark.density import pct
    xs = [s["xgmi4"] for s in allstats if "xgmi4" in s]
    if not xs:
        return {}
    lat = [x for s in xs for x in s["lat"]]
    return {"xgmi4_pods_per_s": round(sum(s["pods"] for s in xs) / max(max(s["t"] for s in xs), 1e-9), 2),
            "xgmi4_p50_startup_ms": round(pct(lat, 0.5) * 1000, 2),
            "xgmi4_single_hive_fraction": round(sum(s["single_hive"] for s in xs) / max(1, sum(s["total"] for s in xs)), 4),
            # every pair of the 4 packages has a direct up xGMI link (amd.com/xgmi-peers)
            "xgmi4_fully_linked_fraction": round(sum(s["linked"] for s in xs) / max(1, sum(s["total"] for s in xs)), 4)}


def _interval_summary(allstats):
    """scheduler_perf's throughput definition (`test/integration/scheduler_perf/scheduler_test.go:131-182`):
    the count sampled once per second over the whole job, reported as the average and the WORST
    full 1-s interval — for scheduled pods (bound) and for pods observed Running. Only full
    intervals inside the timed region count."""
    from kubernetes_amd.kubemark.density import interval_rates
    start = min(s["t_start"] for s in allstats)
    end = max(s["t_end"] for s in allstats)
    out = {"timed_region_s": round(end - start, 3), "full_1s_intervals": int(end - start)}
    for key, name in (("scheduled_at", "sched"), ("running_at", "running")):
        avg, worst = interval_rates([x for s in allstats for x in s[key]], 1.0, start, end)
        out[f"{name}_rate_avg_pods_per_s"] = round(avg, 1)
        out[f"{name}_rate_worst_1s_pods_per_s"] = round(worst, 1) if worst is not None else None
    return out


def _linked(peers, node, ids):
    got = [peers.get((node, i)) for i in ids]
    if any(g is None for g in got):
        return False
    return all(a[0] == b[0] or ((a[1] >> b[0]) & 1 and (b[1] >> a[0]) & 1) for x, a in enumerate(got) for b in got[x + 1:])


def cpu_budget():
    """CPUs this job may use: affinity mask capped by the cgroup v2 quota. KAMD_BENCH_CPUS
    overrides it (rehearsing the whole-node control-plane shape on a smaller machine)."""
    if os.environ.get("KAMD_BENCH_CPUS"):
        return int(os.environ["KAMD_BENCH_CPUS"])
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return n


# Per-pod host CPU of each control-plane component at the N=1 headline rate, measured on the
# MI355X box (`cpu_ms_per_pod`): round 5 profiles/r5_gpu/bench_r5{b,c}*.json — API server
# 0.61-0.63 ms, scheduler 0.29-0.33 ms, hollow kubelets 0.50-0.53 ms per pod at 4613-4864 pods/s;
# round 6 profiles/r6_gpu/bench_r6a.json — 0.627 / 0.321 / 0.557 ms at 4614 pods/s. A whole node sizes each component for the load of `world` ranks at that
# rate so that at linear weak scaling every process is at most 70 % busy with HEADROOM to spare
# (ceilings at 70 % busy >= 1.3x the linear rate: profiles/r5_gpu/whole_node_ceiling.md),
# instead of a fixed-size control plane.
N1_RATE_PODS_PER_S = 4700.0
CPU_MS_PER_POD = {"apiserver": 0.63, "scheduler": 0.32, "hollow": 0.56}
TARGET_UTIL = 0.7
HEADROOM = 1.3


def demand(component, world):
    """Processes `component` needs so that `world` ranks at HEADROOM x the N=1 rate keep it
    <= 70 % busy."""
    import math
    return max(1, math.ceil(world * N1_RATE_PODS_PER_S * HEADROOM * CPU_MS_PER_POD[component] / 1000.0 / TARGET_UTIL))


def control_plane_shape(world, workers=0, shards=0):
    """API server workers and scheduler shards for `world` ranks (0 = auto).

    Small boxes (< 64 CPUs, e.g. the 16-CPU MI355X CI lease) keep the measured shapes
    (profiles/r2_partitioned: n1_shapes, scale_r2d; profiles/r2_density_clients/worker_sweep):
    N=1 w=3 s=2 (2594-2611 pods/s; w=2 2363-2389, w=4 2380-2462), N=4 w=4 s=4 (3184 vs w=4 s=2
    2727). A whole 8-GPU node (>= 64 CPUs) is sized from the per-pod CPU of each component
    (`demand`): at N=8 that is 44 API workers and 23 scheduler shards — ceilings at 70 % busy of
    ~49.7 k and ~50.3 k pods/s against the 37.6 k that linear weak scaling needs (the round-3 caps
    of 16 / 8 capped it at ~14 k) — scaled down together with the hollow-node processes when the
    CPU budget is smaller (`cpus - ranks - store threads`). Pods and events are not cached by the
    API workers (the store's fan-out serves their watches) and scheduler shards only see their
    own unassigned pods and their own nodes' pods, so adding processes does not add per-pod work."""
    cpus = cpu_budget()
    spare = cpus - world - 1
    big = cpus >= 64
    if big:
        want_w, want_s = demand("apiserver", world), demand("scheduler", world)
        want_h = demand("hollow", world)
        budget = max(4, spare - 2)                         # 2: the store's commit + fan-out threads
        scale = min(1.0, budget / float(want_w + want_s + want_h))
        if workers <= 0:
            workers = max(3, int(want_w * scale))
        if shards <= 0:
            shards = max(2, int(want_s * scale))
        return workers, shards
    if workers <= 0:
        if spare < 3:
            workers = 1
        else:
            workers = 3 if world == 1 else 2 if world < 4 else 4
    if shards <= 0:
        if spare < 3:
            shards = 1
        else:
            shards = 2 if world < 4 else 4
    return workers, shards


def hollow_procs_for(world, nodes_per_rank, workers, shards, want=0):
    """Hollow-node processes per rank (0 = auto): kubemark runs one process per hollow node;
    here the rank's nodes are spread over several processes so kubelet work uses several cores,
    bounded by the CPUs left after ranks and the control plane."""
    if want > 0:
        return max(1, min(want, nodes_per_rank))
    cpus = cpu_budget()
    spare = cpus - workers - shards - 1
    if cpus >= 64:
        # a whole node: the hollow kubelets' share of the per-pod demand model, per rank
        # (5 processes per rank at 0.51 ms per pod with headroom), but at least 6 — hollow kubelets wait on
        # the control plane, and 6 beat 4 per rank in interleaved box runs at both API shapes
        # (profiles/r4_gpu/sweep: w4 s3 h6 3982-4062 vs h4 3537-3828 pods/s) — within the CPUs left
        per_rank = max(6, -(-demand("hollow", world) // world))
        return max(1, min(nodes_per_rank, per_rank, max(2, (spare - world) // max(1, world))))
    # hollow kubelets are mostly waiting on the control plane: mild oversubscription pays
    # (profiles/r2_hollow_procs, r2_scale: N=4 on 16 CPUs 1868 -> 2578 pods/s with 2 per rank;
    # N=1 on the 16-CPU box: 6 processes 2601-2693 vs 4 processes 2583-2590 pods/s)
    cap = 6 if world == 1 else 4
    return max(1, min(nodes_per_rank, cap, max(2, spare // max(1, world))))


def spawn_hollow_procs(args, url, rank, nprocs, tmp, payload_socket):
    """Start the rank's hollow nodes in `nprocs` child processes (none touches the GPU: GPU
    payloads go to the rank's PayloadServer)."""
    env = dict(os.environ)
    env["PYTHONPATH"] = HERE + os.pathsep + env.get("PYTHONPATH", "")
    base, extra = divmod(args.nodes_per_rank, nprocs)
    procs = []
    for j in range(nprocs):
        n = base + (1 if j < extra else 0)
        if n == 0:
            continue
        cmd = [sys.executable, "-m", "kubernetes_amd.cmd.hollow_node", "--master", url, "--count", str(n),
               "--name-prefix", f"r{rank}p{j}", "--gpus-per-node", str(args.gpus_per_node),
               "--hives", str(args.hives), "--links-down", args.links_down]
        if payload_socket:
            cmd += ["--payload-socket", payload_socket]
        if args.no_events:
            cmd.append("--no-events")
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.DEVNULL,
                                      stderr=open(os.path.join(tmp, f"hollow-r{rank}p{j}.log"), "w")))
    return procs


def spawn_control_plane(tmp, args):
    env = dict(os.environ)
    env["PYTHONPATH"] = HERE + os.pathsep + env.get("PYTHONPATH", "")
    env.pop("HIP_VISIBLE_DEVICES", None)
    pf = os.path.join(tmp, "apiserver.port")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    workers, shards = control_plane_shape(world, args.apiserver_workers, args.scheduler_shards)
    args.apiserver_workers, args.scheduler_shards = workers, shards
    api = subprocess.Popen([sys.executable, "-m", "kubernetes_amd.cmd.apiserver", "--port", "0", "--port-file", pf,
                            "--storage-engine", args.storage_engine, "--workers", str(workers)],
                           env=env, stdout=subprocess.DEVNULL, stderr=open(os.path.join(tmp, "apiserver.log"), "w"))
    t = time.time()
    while not os.path.exists(pf):
        if api.poll() is not None:
            raise RuntimeError("apiserver exited: " + open(os.path.join(tmp, "apiserver.log")).read()[-2000:])
        if time.time() - t > 120:
            raise TimeoutError("apiserver did not start")
        time.sleep(0.05)
    url = f"http://127.0.0.1:{open(pf).read().strip()}"
    sched = subprocess.Popen([sys.executable, "-m", "kubernetes_amd.cmd.scheduler", "--master", url,
                              "--percentage-of-nodes-to-score", str(args.percentage_of_nodes_to_score),
                              "--shards", str(shards)]
                             + (["--no-events"] if args.no_events else []),
                             env=env, stdout=subprocess.DEVNULL, stderr=open(os.path.join(tmp, "scheduler.log"), "w"))
    return url, [api, sched]


class Dist:
    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.torch = None
        self.cuda = False
        self.backend = None
        self.dist = None

    def init(self):
        import torch
        self.torch = torch
        # KAMD_BENCH_FORCE_CPU=1: rehearse N ranks with gloo and no GPU payload (e.g. 8 ranks on
        # a 1-GPU box) — measures the control plane's scaling only
        self.cuda = torch.cuda.is_available() and not os.environ.get("KAMD_BENCH_FORCE_CPU")
        if self.cuda:
            torch.cuda.set_device(self.local_rank)
        # KAMD_BENCH_FORCE_PG=1 (under a launcher): a process group even for one rank, so a
        # one-GPU box exercises the RCCL init, device binding and barrier path of N > 1
        if self.world > 1 or (os.environ.get("KAMD_BENCH_FORCE_PG") and "MASTER_ADDR" in os.environ):
            import torch.distributed as dist
            self.backend = "nccl" if self.cuda else "gloo"   # "nccl" is RCCL on ROCm
            if self.cuda:
                # bind the process group to this rank's GPU: barriers also run on executor
                # threads, whose current device would otherwise be GPU 0 for every rank
                dist.init_process_group(self.backend, device_id=torch.device("cuda", self.local_rank))
            else:
                dist.init_process_group(self.backend)
            self.dist = dist

    def _bind_thread(self):
        # the current GPU is per thread: object collectives and barriers also run on executor
        # threads, where it would be GPU 0 for every rank (a rank's RCCL communicator is on its
        # own GPU)
        if self.cuda:
            self.torch.cuda.set_device(self.local_rank)

    def broadcast(self, obj):
        if self.dist is None:
            return obj
        self._bind_thread()
        lst = [obj]
        self.dist.broadcast_object_list(lst, src=0)
        return lst[0]

    def barrier(self):
        self._bind_thread()
        if self.dist is not None:
            if self.cuda:
                self.dist.barrier(device_ids=[self.local_rank])
            else:
                self.dist.barrier()
        if self.cuda:
            self.torch.cuda.synchronize()

    def allgather(self, obj):
        if self.dist is None:       # one rank without a process group (KAMD_BENCH_FORCE_PG makes one)
            return [obj]
        self._bind_thread()
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out


def _cp_cpu(procs):
    """CPU seconds (user+sys) used so far by the control-plane processes, by component."""
    out = {}
    if not procs:
        return out
    import psutil
    for name, pid in procs:
        try:
            ps = [psutil.Process(pid)]
            ps += ps[0].children(recursive=True)
        except psutil.NoSuchProcess:
            continue
        for p in ps:
            try:
                t = p.cpu_times()
                comp = "store" if p.name() == "kamd-etcd" else name
            except psutil.NoSuchProcess:
                continue
            out[comp] = out.get(comp, 0.0) + t.user + t.system
    return out


async def rank_main(args, d: Dist, url, cp_procs=()):
    from kubernetes_amd.client.rest import Client
    from kubernetes_amd.kubemark.density import DensityRunner, pct
    from kubernetes_amd.cmd.hollow_node import parse_links
    from kubernetes_amd.kubemark.hollow import HollowCluster

    loop = asyncio.get_running_loop()

    async def abarrier():
        await loop.run_in_executor(None, d.barrier)

    payload = None
    payload_fn = None
    if d.cuda and args.payload != "off":
        from kubernetes_amd.ops.hip_kernels import Payload
        payload = Payload(d.local_rank)
        payload_fn = lambda opts: payload.run()  # noqa: E731
    hollow, hprocs, psrv = None, [], None
    if args.hollow_procs > 1:
        from kubernetes_amd.kubemark.payload import PayloadServer
        sock = None
        if payload is not None:
            sock = os.path.join(tempfile.mkdtemp(prefix="kamd-pl-"), "payload.sock")
            psrv = await PayloadServer(payload.run, sock).start()
        hprocs = spawn_hollow_procs(args, url, d.rank, args.hollow_procs, tempfile.mkdtemp(prefix="kamd-hollow-"), sock)
    else:
        hollow = HollowCluster(url, args.nodes_per_rank, prefix=f"r{d.rank}", gpus=args.gpus_per_node,
                               hives=args.hives, payload=payload_fn, emit_events=not args.no_events,
                               links_down=parse_links(args.links_down))
        await hollow.start()
        await hollow.wait_registered()
    # wait until every rank's nodes are visible with their GPUs
    c = Client(url)
    want_nodes = d.world * args.nodes_per_rank
    t = time.time()
    while True:
        nodes = (await c.list("nodes"))["items"]
        ok = [n for n in nodes if int((n["status"].get("capacity") or {}).get("amd.com/gpu", "0")) == args.gpus_per_node]
        if len(ok) >= want_nodes:
            break
        if time.time() - t > 120:
            raise TimeoutError(f"only {len(ok)}/{want_nodes} GPU nodes ready")
        dead = [p.args for p in hprocs if p.poll() is not None]
        if dead:
            raise RuntimeError(f"hollow-node process exited: {dead[0]}")
        await asyncio.sleep(0.05)
    await c.close()
    pods_per_step = args.pods_per_rank or args.nodes_per_rank * args.gpus_per_node // args.gpus_per_pod
    runner = DensityRunner(url, d.rank, pods_per_step=pods_per_step, gpus_per_pod=args.gpus_per_pod,
                           client_procs=args.client_procs, workdir=tempfile.mkdtemp(prefix="kamd-dc-"))
    await runner.start()
    from kubernetes_amd.cmd._common import tune_gc
    tune_gc()        # same GC settings as the control-plane components
    await abarrier()
    for w in range(args.warmup):
        await runner.step(f"w{w}", timeout=args.step_timeout)
        await abarrier()
    results = []
    await abarrier()
    hollow_pids = [("hollow", p.pid) for p in hprocs]
    # request-issuing helpers are load generator CPU, reported beside the rank's own
    hollow_pids += [("density_clients", p.pid) for p in (runner.pool.procs if runner.pool else ())]
    cp0 = _cp_cpu(list(cp_procs) + hollow_pids)
    load0 = os.getloadavg()
    my0 = time.process_time()
    t_start = time.monotonic()
    t0 = time.perf_counter()
    for k in range(args.steps):
        results.append(await runner.step(k, timeout=args.step_timeout))
        # lock-step ranks by default: measured on the 16-CPU box, free-running ranks were not
        # faster (N=4: 3154 vs 3917 pods/s, profiles/r2_fanout_thread/) — their phases collide
        if not args.no_step_barrier and k + 1 < args.steps:
            await abarrier()
    await abarrier()
    elapsed = time.perf_counter() - t0
    my_cpu = time.process_time() - my0
    cp1 = _cp_cpu(list(cp_procs) + hollow_pids)
    load1 = os.getloadavg()
    lat = [x for r in results for x in r["latencies"]]
    t_end = time.monotonic()
    stats = {"elapsed": elapsed, "lat": lat, "pods": sum(r["pods"] for r in results),
             # CLOCK_MONOTONIC is host-wide: the ranks' timelines merge into the cluster's
             "t_start": t_start, "t_end": t_end,
             "scheduled_at": [x for r in results for x in r["scheduled_at"]],
             "running_at": [x for r in results for x in r["running_at"]],
             "to_running": [r["to_running_s"] for r in results], "cycle": [r["cycle_s"] for r in results],
             "phases": {k: [r[k] for r in results] for k in ("create_s", "to_running_s", "delete_issued_s", "cycle_s")},
             "api_lat": {v: [x for r in results for x in r["api_latencies"][v]] for v in ("create", "delete")},
             "payload_runs": (psrv.runs if psrv else sum(getattr(k.runtime, "payload_runs", 0) for k in hollow.nodes)
                              if hollow or psrv else 0),
             "payload_failures": (psrv.failures if psrv else sum(getattr(k.runtime, "payload_failures", 0) for k in hollow.nodes)
                                  if hollow or psrv else 0),
             "cpu_s": my_cpu,
             "loadavg": {"before": [round(x, 2) for x in load0], "after": [round(x, 2) for x in load1]},
             "cp_cpu_s": {k: cp1.get(k, 0.0) - cp0.get(k, 0.0) for k in cp1}}
    await runner.stop()
    # secondary workload (outside the timed region, not part of `value`): 4-GPU pods that must
    # land on one fully connected xGMI hive (BASELINE: "4-GPU xGMI-hive workload")
    if args.xgmi4_steps and args.gpus_per_node >= 4:
        await abarrier()
        r4 = DensityRunner(url, d.rank, namespace="density-xgmi4",
                           pods_per_step=args.nodes_per_rank * args.gpus_per_node // 4, gpus_per_pod=4,
                           annotations={"amd.com/xgmi-policy": "required"})
        await r4.start()
        x_lat, x_pods, x_t = [], 0, 0.0
        c = Client(url)
        hive, peers = {}, {}
        for n in (await c.list("nodes"))["items"]:
            for rn, dom in ((n.get("status") or {}).get("extendedResources") or {}).items():
                for i, dev in ((dom or {}).get("resources") or {}).items():
                    a = dev.get("attributes") or {}
                    hive[(n["metadata"]["name"], i)] = a.get("amd.com/xgmi-hive", "")
                    if "amd.com/xgmi-peers" in a:
                        peers[(n["metadata"]["name"], i)] = (int(a["amd.com/xgmi-node"]), int(a["amd.com/xgmi-peers"], 16))
        await c.close()
        single = total = linked = 0
        for k in range(args.xgmi4_steps):
            await abarrier()
            r = await r4.step(f"x{k}", timeout=args.step_timeout)
            x_lat += r["latencies"]
            x_pods += r["pods"]
            x_t += r["cycle_s"]
            for name in r["names"]:
                node, ids = r4.assigned.get(name, (None, []))
                total += 1
                single += len(ids) == 4 and len({hive.get((node, i)) for i in ids}) == 1
                linked += len(ids) == 4 and _linked(peers, node, ids)
        await r4.stop()
        stats["xgmi4"] = {"lat": x_lat, "pods": x_pods, "t": x_t, "single_hive": single, "total": total,
                          "linked": linked}
    allstats = await loop.run_in_executor(None, d.allgather, stats)
    # keep serving other ranks' pods until everyone is done
    await abarrier()
    if hollow is not None:
        await hollow.stop()
    for p in hprocs:
        p.terminate()
    for p in hprocs:
        try:
            await loop.run_in_executor(None, p.wait, 10)
        except subprocess.TimeoutExpired:
            p.kill()
    if psrv is not None:
        await psrv.stop()
    if payload is not None:
        payload.close()
    return allstats


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """Run this script as `n` ranks under torch.distributed.run in a child process; its rank 0
    prints the JSON line to our stdout (inherited). Returns the launcher's exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    log("bench.py: launching", " ".join(cmd[1:]))
    p = subprocess.Popen(cmd, env=env)
    try:
        return p.wait()
    except KeyboardInterrupt:
        p.terminate()
        return p.wait()


def raise_fd_limit():
    """The whole-node control plane holds a socket per watch (hundreds of hollow kubelets per
    rank, scheduler shards, API workers): lift the soft RLIMIT_NOFILE to the hard limit for this
    process and every component it starts."""
    import resource
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    want = hard if hard != resource.RLIM_INFINITY else 1 << 20
    if soft < want:
        try:
            resource.setrlimit(resource.RLIMIT_NOFILE, (want, hard))
        except (ValueError, OSError):
            pass


def main():
    raise_fd_limit()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks = GPUs (default: WORLD_SIZE, else 1); without a launcher N > 1 starts "
                         "torch.distributed.run as a child process")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    # 100 hollow nodes x 8 GPUs per rank (scheduler_perf's 100-node cluster): 800 single-GPU pods
    # per step, so --steps 20 times >= 5 s of full churn and the worst 1-s interval is measured
    ap.add_argument("--nodes-per-rank", type=int, default=100)
    ap.add_argument("--gpus-per-node", type=int, default=8)
    ap.add_argument("--hives", type=int, default=2,
                    help="xGMI hives per hollow node (2 x 4 GPUs: the 4-GPU workload can land across hives)")
    ap.add_argument("--links-down", default="",
                    help="failed xGMI links in every hollow node's fake packages, e.g. '2-5' (pairwise-topology variant)")
    ap.add_argument("--gpus-per-pod", type=int, default=1)
    ap.add_argument("--pods-per-rank", type=int, default=0)
    ap.add_argument("--percentage-of-nodes-to-score", type=int, default=100)
    ap.add_argument("--payload", default="auto", choices=["auto", "on", "off"])
    ap.add_argument("--storage-engine", default="native", choices=["native", "python"])
    ap.add_argument("--no-events", action="store_true")
    ap.add_argument("--apiserver-workers", type=int, default=0,
                    help="API server processes over one native store (0 = auto from the CPU budget)")
    ap.add_argument("--xgmi4-steps", type=int, default=2,
                    help="untimed secondary steps of 4-GPU xGMI-hive pods (0 = skip)")
    ap.add_argument("--topology-pods", type=int, default=4000,
                    help="untimed secondary: mixed 1/2/4-GPU pod stream through the real scheduler on the real "
                         "8xMI355X node shape and its CPX variant (kubemark.topology_stream; 0 = skip)")
    ap.add_argument("--step-timeout", type=float, default=120.0, help="fail (with diagnostics) if a step stalls")
    ap.add_argument("--client-procs", type=int, default=0,
                    help="helper processes per rank that issue the density creates/deletes (0 = the rank itself)")
    ap.add_argument("--no-step-barrier", action="store_true",
                    help="ranks run their timed steps independently (barriers only around the timed region)")
    ap.add_argument("--scheduler-shards", type=int, default=0,
                    help="parallel scheduler shard processes (0 = auto from the CPU budget)")
    ap.add_argument("--hollow-procs", type=int, default=0,
                    help="hollow-node processes per rank (0 = auto from the CPU budget; 1 = in the rank process)")
    args = ap.parse_args()
    launched = "WORLD_SIZE" in os.environ
    if args.gpus is None:
        args.gpus = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if not launched and args.gpus > 1:
        # --gpus is authoritative: without a launcher, start one rank per GPU under
        # torch.distributed.run as a CHILD process (nothing here has touched the GPU yet, and an
        # exec after GPU init is not allowed on the pool), relay its output, exit with its code
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        log(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
        sys.exit(2)
    if not os.environ.get("KAMD_BENCH_FORCE_CPU"):
        import torch   # device_count() does not initialise HIP on this image
        ndev = torch.cuda.device_count()
        if ndev and ndev < world:
            log(f"bench.py: {world} ranks need {world} GPUs, only {ndev} visible")
            sys.exit(2)
    d = Dist()
    tmp = tempfile.mkdtemp(prefix="kamd-bench-")
    procs = []
    url = None
    try:
        if d.rank == 0:
            url, procs = spawn_control_plane(tmp, args)   # before any GPU init
        d.init()
        url, d.broadcast_done_workers, d.shards = d.broadcast((url, args.apiserver_workers, args.scheduler_shards))
        args.hollow_procs = hollow_procs_for(d.world, args.nodes_per_rank, d.broadcast_done_workers, d.shards,
                                             args.hollow_procs)
        cp = [("apiserver", procs[0].pid), ("scheduler", procs[1].pid)] if procs else []
        if os.environ.get("KAMD_PROFILE_DIR"):
            import cProfile
            pr = cProfile.Profile()
            pr.enable()
            allstats = asyncio.run(rank_main(args, d, url, cp))
            pr.disable()
            pr.dump_stats(os.path.join(os.environ["KAMD_PROFILE_DIR"], f"rank{d.rank}.prof"))
        else:
            allstats = asyncio.run(rank_main(args, d, url, cp))
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
    if d.rank != 0:
        return
    from kubernetes_amd.kubemark.density import pct
    elapsed = max(s["elapsed"] for s in allstats)
    pods = sum(s["pods"] for s in allstats)
    lat = [x for s in allstats for x in s["lat"]]
    value = pods / elapsed
    n = d.world
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "pods/s", "n_gpus": n, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1000, 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": round(value / BASELINE_DENSITY_PODS_PER_S, 2),
        # an orchestrator has no compute dtype; the only GPU arithmetic is the fp32 vector_add payload
        "dtype": "fp32",
        "data": "synthetic GPU-requesting pods, stub containers (HIP vector_add payload on the rank's MI355X)"
        if any(s["payload_runs"] for s in allstats) else "synthetic GPU-requesting pods, stub containers",
        "config": {"model": "kubemark-density/8xMI355X-hollow-nodes/1-GPU-pods", "global_batch": pods // args.steps,
                   "seq_len": None, "parallelism": f"ranks{n}", "hollow_nodes": n * args.nodes_per_rank,
                   "gpus_per_node": args.gpus_per_node, "xgmi_hives_per_node": args.hives,
                   "advertised_gpus": n * args.nodes_per_rank * args.gpus_per_node,
                   "gpus_per_pod": args.gpus_per_pod, "apiserver_workers": d.broadcast_done_workers,
                   "scheduler_shards": d.shards, "hollow_procs_per_rank": args.hollow_procs,
                   "world_size": n, "backend": d.backend,
                   "topology": f"synthetic fake-AMD-SMI fixture: {args.hives} xGMI hive(s) x "
                               f"{args.gpus_per_node // max(1, args.hives)} GPUs per hollow node"
                               + (" (a real 8xMI355X node is one fully connected 8-GPU hive)" if args.hives > 1 else "")},
        "p50_startup_ms": round(pct(lat, 0.50) * 1000, 2), "p90_startup_ms": round(pct(lat, 0.90) * 1000, 2),
        "p99_startup_ms": round(pct(lat, 0.99) * 1000, 2),
        "to_running_s_per_step": [round(max(s["to_running"][k] for s in allstats), 4) for k in range(args.steps)],
        "step_ms_max": round(1000 * max(max(s["cycle"]) for s in allstats), 2),
        # mean over steps of the slowest rank: pods created / all Running / deletes issued / all gone
        "step_phases_ms": {k: round(1000 * sum(max(s["phases"][k][i] for s in allstats) for i in range(args.steps))
                                    / max(1, args.steps), 2)
                           for k in ("create_s", "to_running_s", "delete_issued_s", "cycle_s")},
        # client-observed API call latency under load (reference SLO: non-list p99 <= 1 s,
        # test/e2e/framework/metrics_util.go:52-59)
        "api_call_ms": {v: {q: round(pct([x for s in allstats for x in s["api_lat"][v]], p) * 1000, 2)
                            for q, p in (("p50", 0.5), ("p99", 0.99))} for v in ("create", "delete")},
        **_interval_summary(allstats),
        "vs_scheduler_perf_warn_threshold": round(value / BASELINE_SCHED_WARN_PODS_PER_S, 2),
        "payload_runs": sum(s["payload_runs"] for s in allstats),
        "payload_failures": sum(s["payload_failures"] for s in allstats),
        **_xgmi4_summary(allstats),
        # where the host CPU goes (timed region): ms of CPU per pod, by component
        "cpu_ms_per_pod": {k: round(v * 1000 / max(pods, 1), 3) for k, v in
                           dict(sum_ranks=sum(s["cpu_s"] for s in allstats),
                                **{c: sum(s["cp_cpu_s"].get(c, 0.0) for s in allstats)
                                   for c in ("apiserver", "scheduler", "store", "hollow", "density_clients")}).items()},
    }
    # host contention context for `value` (the lease shares its host): 1/5/15-min load averages
    # around the timed region and the CPUs this job may use
    out["host"] = {"cpus": cpu_budget(), "loadavg_before": allstats[0]["loadavg"]["before"],
                   "loadavg_after": allstats[0]["loadavg"]["after"]}
    if args.topology_pods:
        # secondary, after the timed region and not part of `value`: fragmentation / NUMA fit /
        # multi-GPU wait on the real node shape (one 8-package hive) and CPX, against the
        # reference's spreading + first-N placement on the same seeded stream
        from kubernetes_amd.kubemark import topology_stream
        t = time.perf_counter()
        out["topology_stream"] = topology_stream.run(16, args.topology_pods)
        out["topology_stream"]["wall_s"] = round(time.perf_counter() - t, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
