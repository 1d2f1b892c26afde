"""bench.py contract (the driver's headline measurement): one JSON line with the metric, value
(whole-job pods/s), steps/warmup, weak scaling, config — for N=1 in one process and for N=2
ranks under torch.distributed.run (gloo on CPU here; RCCL on MI355X), with hollow nodes both
in the rank process and in child processes."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, out[-3000:]
    return json.loads(lines[0])


def _check(d, n, steps, warmup):
    assert d["metric"].startswith("GPU pods/sec scheduled") and d["unit"] == "pods/s"
    assert d["n_gpus"] == n and d["steps"] == steps and d["warmup"] == warmup
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["value"] > 0
    assert d["config"]["model"] == "kubemark-density/8xMI355X-hollow-nodes/1-GPU-pods"
    assert d["config"]["hollow_nodes"] == n * d["config"]["hollow_nodes"] // n
    assert abs(d["vs_baseline"] - d["value"] / 8.0) <= 0.01
    assert d["p50_startup_ms"] > 0 and d["payload_failures"] == 0


def test_bench_single_rank_hollow_processes():
    env = dict(os.environ, KAMD_BENCH_FORCE_CPU="1")
    r = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--nodes-per-rank", "2",
                        "--hollow-procs", "2", "--xgmi4-steps", "1"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    _check(d, 1, 2, 1)
    assert d["config"]["hollow_procs_per_rank"] == 2 and d["config"]["global_batch"] == 16
    assert d["xgmi4_single_hive_fraction"] == 1.0


def test_bench_two_ranks_gloo():
    env = dict(os.environ, KAMD_BENCH_FORCE_CPU="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29731", "bench.py", "--gpus", "2",
                        "--steps", "2", "--warmup", "1", "--nodes-per-rank", "2", "--xgmi4-steps", "0"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    _check(d, 2, 2, 1)
    assert d["config"]["parallelism"] == "ranks2" and d["config"]["hollow_nodes"] == 4
    assert d["config"]["global_batch"] == 32                 # weak scaling: 2 ranks x 2 nodes x 8 GPUs


def test_bench_gpus_flag_launches_ranks_without_a_launcher():
    """--gpus N is authoritative: `python bench.py --gpus 2` (no torch.distributed.run) starts
    the two ranks itself as a child launcher and reports n_gpus 2."""
    env = dict(os.environ, KAMD_BENCH_FORCE_CPU="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--nodes-per-rank", "2", "--xgmi4-steps", "0"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    _check(d, 2, 2, 1)
    assert d["config"]["parallelism"] == "ranks2" and d["config"]["world_size"] == 2
    assert d["config"]["backend"] == "gloo" and d["dtype"] == "fp32"
    assert "synthetic" in d["config"]["topology"]


def test_bench_gpus_mismatch_fails():
    env = dict(os.environ, KAMD_BENCH_FORCE_CPU="1", WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--steps", "1", "--warmup", "0"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr, r.stderr[-2000:]


def test_bench_eight_ranks_whole_node_shape():
    """The N=8 path the driver runs on a whole MI355X node, rehearsed with gloo on CPU: 8 ranks
    under torch.distributed.run with the >= 64-CPU control-plane shape (KAMD_BENCH_CPUS=64:
    the demand model scaled to that budget — 21 API server workers, 11 scheduler shards) and
    small per-rank work."""
    env = dict(os.environ, KAMD_BENCH_FORCE_CPU="1", KAMD_BENCH_CPUS="64")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", "29747", "bench.py", "--gpus", "8",
                        "--steps", "2", "--warmup", "1", "--nodes-per-rank", "1", "--xgmi4-steps", "0"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    _check(d, 8, 2, 1)
    assert d["config"]["parallelism"] == "ranks8" and d["config"]["hollow_nodes"] == 8
    assert d["config"]["global_batch"] == 64
    assert d["config"]["apiserver_workers"] == 21 and d["config"]["scheduler_shards"] == 11


def test_payload_server_batches_starts(run, tmp_path):
    """Hollow-node processes ask the rank's PayloadServer for GPU payload runs: starts issued
    together are answered as one batch (run_batch), failures are reported per start."""
    import asyncio
    from kubernetes_amd.kubemark.payload import PayloadClient, PayloadServer

    class Fake:
        def __init__(self):
            self.calls = []

        def run(self):
            return True

        def run_batch(self, k):
            self.calls.append(k)
            base = sum(self.calls) - k
            return [(base + i) % 5 != 4 for i in range(k)]    # every 5th start fails

    async def main():
        f = Fake()
        srv = await PayloadServer(f.run, str(tmp_path / "p.sock")).start()
        cl = PayloadClient(str(tmp_path / "p.sock"))
        oks = await asyncio.gather(*(cl() for _ in range(10)))
        assert oks.count(False) == 2 and srv.runs == 10 and srv.failures == 2
        assert len(f.calls) < 10                         # coalesced into batches
        # a plain callable works too (one run per start)
        srv2 = await PayloadServer(lambda: True, str(tmp_path / "q.sock")).start()
        cl2 = PayloadClient(str(tmp_path / "q.sock"))
        assert await asyncio.gather(*(cl2() for _ in range(4))) == [True] * 4
        for c in (cl, cl2):
            await c.close()
        for s in (srv, srv2):
            await s.stop()
    run(main())


def test_control_plane_shape_grows_with_ranks_on_a_big_node(monkeypatch):
    """Whole node: each component sized for world x the N=1 rate from its measured per-pod CPU
    so that at 70 % busy its ceiling (processes / ms per pod) is >= 1.3x linear weak scaling
    (profiles/r5_gpu/whole_node_ceiling.md)."""
    import bench
    monkeypatch.setattr(bench, "cpu_budget", lambda: 192)
    assert bench.control_plane_shape(1) == (6, 3)
    assert bench.control_plane_shape(4) == (22, 12)
    w, s = bench.control_plane_shape(8)
    assert (w, s) == (44, 23)
    need = 8 * bench.N1_RATE_PODS_PER_S * 1.3
    assert w / bench.CPU_MS_PER_POD["apiserver"] * 1000 * 0.7 >= need
    assert s / bench.CPU_MS_PER_POD["scheduler"] * 1000 * 0.7 >= need
    h = bench.hollow_procs_for(8, 100, w, s)
    assert 8 * h / bench.CPU_MS_PER_POD["hollow"] * 1000 * 0.7 >= need
    assert 8 + w + s + 8 * h + 2 <= 192
    monkeypatch.setattr(bench, "cpu_budget", lambda: 64)
    w, s = bench.control_plane_shape(8)
    assert 8 + w + s + 8 * bench.hollow_procs_for(8, 100, w, s) + 2 <= 64 + 8   # scaled to the budget
    monkeypatch.setattr(bench, "cpu_budget", lambda: 16)
    assert bench.control_plane_shape(1) == (3, 2) and bench.control_plane_shape(4) == (4, 4)


def test_store_bench_small():
    """kamd-etcd under the density write + watch pattern: every event reaches its watchers."""
    from kubernetes_amd.kubemark.store_bench import run
    r = run(writers=2, pods=400, nodes=8, all_watches=1, fan_threads=2, inflight=16, shards=2)
    # node watch: bind, Running, delete; shard watch: create, bind (leaves); namespace observer
    # and the whole-prefix watch: all 4
    assert r["pods"] == 400 and r["events_delivered"] == r["events_expected"] == 400 * (3 + 2 + 4 + 4), r
    assert r["pods_per_s"] > 0 and set(r["store_cpu_ms_per_pod"]) >= {"store", "fan0", "fan1"}


def test_hollow_procs_per_rank(monkeypatch):
    import bench
    monkeypatch.setattr(bench, "cpu_budget", lambda: 192)
    assert bench.hollow_procs_for(8, 100, 32, 18) == 6       # a whole node: demand model, at least 6
    assert bench.hollow_procs_for(8, 4, 32, 18) == 4         # never more than the rank's nodes
    monkeypatch.setattr(bench, "cpu_budget", lambda: 64)
    assert bench.hollow_procs_for(8, 100, 16, 9) == 3        # bounded by the spare CPUs
    monkeypatch.setattr(bench, "cpu_budget", lambda: 16)
    assert bench.hollow_procs_for(1, 8, 3, 2) == 6 and bench.hollow_procs_for(2, 8, 2, 2) == 4
    assert bench.hollow_procs_for(1, 8, 3, 2, want=3) == 3
