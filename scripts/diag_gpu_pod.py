"""GPU-box diagnostic for a real-GPU pod stuck before it runs: one LocalCluster node on the real
AMD SMI with the process runtime, one hip-vector-add pod; after at most 40 s the pod status, the
kubelet/runtime DEBUG log and every small file of the runtime's container/sandbox dirs (OCI
config, isolation report, state, logs) are written under gpurun_out/diag/."""
import asyncio
import json
import logging
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "gpurun_out", "diag")


async def main():
    from kubernetes_amd.api import core
    from kubernetes_amd.cluster import LocalCluster
    os.makedirs(OUT, exist_ok=True)
    logging.basicConfig(level=logging.DEBUG, filename=os.path.join(OUT, "debug.log"),
                        format="%(asctime)s %(levelname).1s %(name)s] %(message)s")
    report = {}
    async with LocalCluster(nodes=1, gpus_per_node=8, runtime="process", real_gpus=True) as cl:
        rt = cl.nodes[0].runtime
        report["isolation"] = rt.isolation_status()
        await cl.client.create("pods", {"metadata": {"name": "vector-add", "namespace": "default"},
                                        "spec": {"restartPolicy": "Never", "containers": [
                                            {"name": "c", "image": "kubernetes-amd/hip-vector-add",
                                             "resources": {"limits": {core.AMD_GPU: "1"}}}]}})
        for i in range(80):
            p = await cl.client.get("pods", "vector-add", "default")
            if (p.get("status") or {}).get("phase") in ("Succeeded", "Failed"):
                break
            await asyncio.sleep(0.5)
            if i % 10 == 0:
                print("waiting", i, (p.get("status") or {}).get("phase"), flush=True)
        report["pod_status"] = p.get("status")
        report["files"] = {}
        for base, _, files in os.walk(rt.root):
            for fn in files:
                path = os.path.join(base, fn)
                try:
                    if os.path.getsize(path) < 64 << 10:
                        report["files"][os.path.relpath(path, rt.root)] = open(path, errors="replace").read()[-4000:]
                except OSError as e:
                    report["files"][path] = str(e)
    with open(os.path.join(OUT, "report.json"), "w") as f:
        json.dump(report, f, indent=1, default=str)
    print(json.dumps(report.get("pod_status"), default=str)[:2000])


if __name__ == "__main__":
    asyncio.run(main())
