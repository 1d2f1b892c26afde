"""CPU per device-plugin RPC: grpc.aio vs utils/grpclite, client and server in one process (the
kubemark hollow-node layout: the fake AMD GPU plugin and the kubelet share a loop).

    python -m kubernetes_amd.kubemark.rpc_bench [--calls 4000]

Prints one JSON line per (server, client) transport pair: process CPU (all threads, so
grpc-core's poller thread counts) per AdmitPod round trip, sequential and 50 in flight.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import tempfile
import time

import grpc

from ..deviceplugin import api
from ..deviceplugin.server import DevicePluginServer, device
from ..utils import grpclite


async def measure(server_t, client_t, calls):
    d = tempfile.mkdtemp(prefix="rpcbench-")
    sock = os.path.join(d, "p.sock")
    srv = await DevicePluginServer("amd.com/gpu", sock, [device("g0")], transport=server_t).start()
    ch = grpclite.Channel("unix://" + sock) if client_t == "lite" else grpc.aio.insecure_channel("unix://" + sock)
    stub = api.device_plugin_stub(ch)
    req = api.DP["AdmitPodRequest"](pod_name="density-pod")
    req.containers["c"].name = "c"
    req.containers["c"].devices.extend(["g0"])
    try:
        for _ in range(200):
            await stub.AdmitPod(req, timeout=10)
        t0, w0 = time.process_time(), time.perf_counter()
        for _ in range(calls):
            await stub.AdmitPod(req, timeout=10)
        seq_cpu, seq_wall = (time.process_time() - t0) / calls, (time.perf_counter() - w0) / calls
        t0 = time.process_time()
        for _ in range(calls // 50):
            await asyncio.gather(*[stub.AdmitPod(req, timeout=10) for _ in range(50)])
        conc_cpu = (time.process_time() - t0) / (calls // 50 * 50)
    finally:
        await ch.close()
        await srv.stop()
        os.rmdir(d) if not os.listdir(d) else None
    return {"server": server_t, "client": client_t, "cpu_us_per_call_sequential": round(seq_cpu * 1e6, 1),
            "wall_us_per_call_sequential": round(seq_wall * 1e6, 1),
            "cpu_us_per_call_50_in_flight": round(conc_cpu * 1e6, 1)}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--calls", type=int, default=4000)
    a = ap.parse_args(argv)
    for s, c in (("grpc", "grpc"), ("lite", "lite"), ("grpc", "lite"), ("lite", "grpc")):
        print(json.dumps(asyncio.run(measure(s, c, a.calls))), flush=True)


if __name__ == "__main__":
    main()
