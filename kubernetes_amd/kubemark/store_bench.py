"""Capacity of the shared native store (`kamd-etcd`) under the density workload's write and
watch pattern, without the Python API server in front of it.

P writer processes run pod lifecycles against the store the way API server workers commit them
(create, bind to a node, Running status, delete with a tombstone: 4 transactions and 4 watch
events per pod, values framed with the index header the fan-out matches on). Meanwhile the
store's fan-out serves the density run's watches, each drained by a reader thread: one per hollow
kubelet (`spec.nodeName=<node>`), one per scheduler shard (unassigned pods of its shard,
`?kamdShard=i/n`), one density observer per writer (its namespace) and optionally A unfiltered
whole-prefix watches. Reported: pods/s, and the store's CPU per pod split by thread (the store thread commits
and answers writers, the fan-out threads match and write watch streams) — 1 / (busiest thread's
CPU per pod) is the store's ceiling in pods/s.

    python -m kubernetes_amd.kubemark.store_bench --writers 8 --pods 40000 --shards 8 --fan-threads 1 2
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time

from ..storage import wire
from ..storage.remote import FanoutClient, RemoteStore, StoreServer

_FRAME = b"\x00KH"


def _value(name, ns, node, phase, rv_pad=1200):
    fields = {"metadata.name": name, "metadata.namespace": ns, "spec.nodeName": node, "status.phase": phase}
    hdr = json.dumps([fields, {"app": "density"}], separators=(",", ":")).encode()
    obj = {"metadata": {"name": name, "namespace": ns, "labels": {"app": "density"}},
           "spec": {"nodeName": node, "containers": [{"name": "c", "image": "x"}], "pad": "x" * rv_pad},
           "status": {"phase": phase}}
    return _FRAME + len(hdr).to_bytes(4, "little") + hdr + json.dumps(obj, separators=(",", ":")).encode()


async def _writer_main(addr, wid, pods, nodes, inflight):
    st = await RemoteStore(addr).connect()
    ns = f"bench-{wid}"
    sem = asyncio.Semaphore(inflight)

    async def one(i):
        async with sem:
            name = f"p{i}"
            key = f"/registry/pods/{ns}/{name}"
            node = f"node-{(wid * 7919 + i) % nodes}"
            r = await st.txn([(wire.CMP_ABSENT, key, 0, None)], [(wire.OP_PUT, key, _value(name, ns, "", "Pending"))])
            for nd, ph in ((node, "Pending"), (node, "Running")):
                r = await st.txn([(wire.CMP_MOD_REV, key, r.rev, None)], [(wire.OP_PUT, key, _value(name, ns, nd, ph))])
            await st.txn([(wire.CMP_MOD_REV, key, r.rev, None)],
                         [(wire.OP_DELETE_TOMBSTONE, key, _value(name, ns, node, "Running"), b"\x00rv\x00")])
    await asyncio.gather(*(one(i) for i in range(pods)))
    await st.close()


def _writer_cli(argv):
    """`--writer ADDR WID PODS NODES INFLIGHT`: one writer process (a fresh interpreter, not a
    fork of a process that already runs reader / asyncio / gRPC threads). Prints its elapsed
    seconds as JSON on success."""
    addr, wid, pods, nodes, inflight = argv[0], *map(int, argv[1:5])
    t0 = time.perf_counter()
    asyncio.run(_writer_main(addr, wid, pods, nodes, inflight))
    print(json.dumps({"elapsed": time.perf_counter() - t0}), flush=True)


def _spawn_writers(addr, writers, per, nodes, inflight, timeout):
    here = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, PYTHONPATH=here + os.pathsep + os.environ.get("PYTHONPATH", ""))
    ps = [subprocess.Popen([sys.executable, "-m", "kubernetes_amd.kubemark.store_bench", "--writer", str(addr),
                            str(w), str(per), str(nodes), str(inflight)],
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, start_new_session=True)
          for w in range(writers)]
    deadline = time.time() + timeout
    errors = []
    for w, p in enumerate(ps):
        try:
            out, err = p.communicate(timeout=max(0.1, deadline - time.time()))
            if p.returncode != 0:
                errors.append(f"writer {w}: exit {p.returncode}: {err.decode()[-500:]}")
        except subprocess.TimeoutExpired:
            errors.append(f"writer {w}: no result after {timeout}s")
    for p in ps:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()
    return errors


_EVENT = b'{"type":"'


def _drain(sock, counter, stop):
    sock.settimeout(0.2)
    tail = b""
    while not stop.is_set():
        try:
            b = sock.recv(1 << 20)
        except socket.timeout:
            continue
        except OSError:
            return
        if not b:
            return
        data = tail + b
        counter[0] += data.count(_EVENT)          # one per watch event
        tail = data[-(len(_EVENT) - 1):]          # a marker split across reads is counted once
        counter[1] += len(b)


def _thread_cpu(pid):
    """{thread name: cpu seconds} of a process, from /proc (the store names no threads, so the
    first TID is the store thread and the rest are fan-out threads, in creation order)."""
    out = {}
    tids = sorted(int(t) for t in os.listdir(f"/proc/{pid}/task"))
    tick = os.sysconf("SC_CLK_TCK")
    for k, tid in enumerate(tids):
        with open(f"/proc/{pid}/task/{tid}/stat") as f:
            parts = f.read().rsplit(")", 1)[1].split()
        out["store" if k == 0 else f"fan{k - 1}"] = (int(parts[11]) + int(parts[12])) / tick
    return out


def run(writers=4, pods=20000, nodes=64, all_watches=0, fan_threads=1, inflight=64, shards=4, timeout=600.0):
    srv = StoreServer(fan_threads=fan_threads)
    addr = srv.start()
    fc = FanoutClient.for_store(addr)
    stop = threading.Event()
    readers, counters, socks = [], [], []
    from ..api.sharding import SHARD_OFFSET_LABEL
    specs = [[(FanoutClient.FIELD, "=", "spec.nodeName", [f"node-{n}"])] for n in range(nodes)]
    specs += [[(FanoutClient.FIELD, "=", "spec.nodeName", [""]), (FanoutClient.LABEL, "shard", SHARD_OFFSET_LABEL, [shards, i])]
              for i in range(shards)]
    specs += [[(FanoutClient.FIELD, "=", "metadata.namespace", [f"bench-{w}"])] for w in range(writers)]
    specs += [[] for _ in range(all_watches)]
    for reqs in specs:
        a, b = socket.socketpair()
        fc.handoff(a.fileno(), fc.encode("/registry/pods/", False, 0, 0, reqs))
        a.close()
        c = [0, 0]
        t = threading.Thread(target=_drain, args=(b, c, stop), daemon=True)
        t.start()
        readers.append(t)
        counters.append(c)
        socks.append(b)
    time.sleep(0.3)
    cpu0 = _thread_cpu(srv.proc.pid)
    per = pods // writers
    t0 = time.perf_counter()
    errors = _spawn_writers(addr, writers, per, nodes, inflight, timeout)
    elapsed = time.perf_counter() - t0
    if errors:
        stop.set()
        srv.stop()
        raise RuntimeError(f"store bench writers failed: {errors}")
    # per pod: its node's watch sees bind (ADDED), Running, delete; its shard's watch the create
    # (ADDED) and the bind (DELETED: no longer unassigned); its namespace observer and every
    # whole-prefix watch all 4 events
    want = (pods // writers) * writers * (3 + (2 if shards else 0) + 4 + 4 * all_watches)
    deadline = time.time() + 10
    while sum(c[0] for c in counters) < want and time.time() < deadline:
        time.sleep(0.05)   # let the fan-out finish writing
    cpu1 = _thread_cpu(srv.proc.pid)
    stop.set()
    for s in socks:
        s.close()
    srv.stop()
    total = per * writers
    cpu = {k: cpu1.get(k, 0.0) - cpu0.get(k, 0.0) for k in cpu1}
    per_pod_ms = {k: round(v / total * 1e3, 4) for k, v in cpu.items()}
    busiest = max(per_pod_ms.values()) if per_pod_ms else 0.0
    return {"pods": total, "elapsed_s": round(elapsed, 3), "pods_per_s": round(total / elapsed, 1),
            "events_delivered": sum(c[0] for c in counters), "bytes_delivered": sum(c[1] for c in counters),
            "events_expected": want, "watches": len(specs), "fan_threads": fan_threads, "writers": writers,
            "store_cpu_ms_per_pod": per_pod_ms,
            "ceiling_pods_per_s": round(1e3 / busiest, 0) if busiest else None}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if argv and argv[0] == "--writer":
        return _writer_cli(argv[1:])
    ap = argparse.ArgumentParser("store-bench")
    ap.add_argument("--writers", type=int, default=4)
    ap.add_argument("--pods", type=int, default=20000)
    ap.add_argument("--nodes", type=int, default=64)
    ap.add_argument("--all-watches", type=int, default=0)
    ap.add_argument("--shards", type=int, default=4)
    ap.add_argument("--fan-threads", type=int, nargs="+", default=[1])
    ap.add_argument("--inflight", type=int, default=64)
    a = ap.parse_args(argv)
    for ft in a.fan_threads:
        print(json.dumps(run(a.writers, a.pods, a.nodes, a.all_watches, ft, a.inflight, a.shards)), flush=True)


if __name__ == "__main__":
    main()
