"""GPU e2e smoke: one real MI355X pod through the whole stack (BASELINE configs 1-3).

API server → ResourceV2 admission → scheduler (device-ID binding) → kubelet admission via the
DeviceManager → real amd.com/gpu plugin on AMD SMI (InitContainer: /dev/kfd + renderD) → process
runtime runs `hip-vector-add` (gfx950 kernel) on the allocated GPU → pod Succeeded,
log says "Test PASSED" (the reference's cuda-vector-add e2e check,
test/e2e/scheduling/nvidia-gpus.go:51-113).

The pod's own view is checked, not only the bundle: HIP inside the pod enumerates exactly the
allocated GPU(s). With enforced isolation (kamd-runc: private /dev) the pod's /dev/dri holds
only its render node and HIP_VISIBLE_DEVICES is unset; on a node that cannot isolate (an
unprivileged kubelet without user namespaces, e.g. the GPU CI box) the node must carry
IsolationUnavailable=True and the runtime narrows HIP with HIP_VISIBLE_DEVICES instead.
"""
from __future__ import annotations

import asyncio
import json
import os
import re

from ..api import core
from ..cluster import LocalCluster


async def gpu_pod_e2e(timeout=120, cri=False):
    """cri=True: the kubelet drives the pod through the CRI gRPC socket (RemoteRuntime + PLEG
    relist) of a kamd-cri server backed by the process runtime — the dockershim topology."""
    srv = rt_remote = None
    async with LocalCluster(nodes=0 if cri else 1, gpus_per_node=8, runtime="process", real_gpus=True) as cl:
        if cri:
            import tempfile
            from ..cri.remote import RemoteRuntime
            from ..cri.server import CRIServer
            from ..kubelet.runtime.process import ProcessRuntime
            d = tempfile.mkdtemp(prefix="kamd-cri-")
            backend = ProcessRuntime(os.path.join(d, "rt"))
            srv = await CRIServer(backend, os.path.join(d, "cri.sock")).start()
            rt_remote = await RemoteRuntime(os.path.join(d, "cri.sock"), relist_period=0.1).connect()
            await cl.add_node("mi355x-cri", runtime=rt_remote)
            await cl.wait_nodes_ready()
        node = await cl.client.get("nodes", cl.nodes[0].name)
        cap = int(node["status"]["capacity"].get(core.AMD_GPU, "0"))
        assert cap >= 1, node["status"]
        pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "vector-add", "namespace": "default"},
               "spec": {"restartPolicy": "Never",
                        "containers": [{"name": "vector-add", "image": "kubernetes-amd/hip-vector-add",
                                        "resources": {"limits": {core.AMD_GPU: "1"}}}]}}
        await cl.client.create("pods", pod)
        p = await cl.wait_pod("vector-add", phase="Succeeded", timeout=timeout)
        rt = srv.rt if cri else cl.nodes[0].runtime
        cs = rt.list_containers()[0]
        logs = open(cs.log_path).read()
        spec = json.load(open(os.path.join(os.path.dirname(cs.log_path), "config.json")))
        paths = [d["path"] for d in spec["linux"]["devices"]]
        result = {"node_capacity": cap, "assigned": p["spec"]["extendedResources"][0]["assigned"],
                  "devices": paths, "allow": spec["linux"]["resources"]["devices"], "log": logs,
                  "attributes": node["status"]["extendedResources"][core.AMD_GPU]["resources"][
                      p["spec"]["extendedResources"][0]["assigned"][0]]["attributes"]}
        assert "Test PASSED" in logs, logs
        assert "/dev/kfd" in paths and any(x.startswith("/dev/dri/renderD") for x in paths), paths
        m = re.search(r"(\d+) visible device", logs)
        result["hip_visible_devices_in_pod"] = int(m.group(1)) if m else None
        assert result["hip_visible_devices_in_pod"] == 1, logs
        # what the pod's process sees of /dev and its environment
        view = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "dev-view", "namespace": "default"},
                "spec": {"restartPolicy": "Never",
                         "containers": [{"name": "v", "image": "busybox",
                                         "command": ["/bin/sh", "-c", "echo DRI=$(ls /dev/dri | tr '\\n' ' '); "
                                                     "echo HIP=${HIP_VISIBLE_DEVICES-unset}"],
                                         "resources": {"limits": {core.AMD_GPU: "1"}}}]}}
        await cl.client.create("pods", view)
        pv = await cl.wait_pod("dev-view", phase="Succeeded", timeout=timeout)
        vcs = [c for c in rt.list_containers() if c.name == "v"][0]
        vlog = open(vcs.log_path).read()
        node = await cl.client.get("nodes", cl.nodes[0].name)
        cond = {c["type"]: c for c in node["status"]["conditions"]}.get("IsolationUnavailable")
        iso = rt.isolation_status()
        result["isolation"] = iso
        result["dev_view"] = vlog.strip()
        assert cond is not None and cond["status"] == ("False" if iso["enforced"] else "True"), cond
        minor = node["status"]["extendedResources"][core.AMD_GPU]["resources"][
            pv["spec"]["extendedResources"][0]["assigned"][0]]["attributes"].get(core.ATTR_RENDER_MINOR)
        dri = vlog.split("DRI=", 1)[1].split("\n", 1)[0].split()
        if iso["enforced"]:
            assert dri == [f"renderD{minor}"], vlog
            assert "HIP=unset" in vlog, vlog
        else:
            assert "HIP=unset" not in vlog and "HIP=-1" not in vlog, vlog
        if cri:
            await rt_remote.close()
            await srv.stop()
            result["runtime"] = rt_remote.runtime_name
        return result


def run_gpu_pod_smoke():
    r = asyncio.run(gpu_pod_e2e())
    print(json.dumps({k: v for k, v in r.items() if k != "allow"}, indent=1))
    return r
