"""GPU e2e smoke: one real MI355X pod through the whole stack (BASELINE configs 1-3).

API server → ResourceV2 admission → scheduler (device-ID binding) → kubelet admission via the
DeviceManager → real amd.com/gpu plugin on AMD SMI (InitContainer: /dev/kfd + renderD) → process
runtime runs `hip-vector-add` (gfx950 kernel) on the allocated GPU → pod Succeeded,
log says "Test PASSED" (the reference's cuda-vector-add e2e check,
test/e2e/scheduling/nvidia-gpus.go:51-113).

The pod's own view is checked, not only the bundle: HIP inside the pod enumerates exactly the
allocated GPU(s). Which enforcement tier is in force is decided by the node's own
`kamd-runc features` output and reported:
  * namespaces — private /dev: the pod's /dev/dri holds only its render node;
  * landlock   — no namespaces (an unprivileged kubelet without user namespaces, e.g. the GPU CI
                 box): /dev/dri lists everything, but the pod can open only its allocated node;
                 every node the kubelet itself can open but did not allocate must be denied
                 (reported EPERM through kamd-runc's errno shim, so ROCr skips sibling GPUs
                 instead of failing hsa_init on Landlock's EACCES: `landlock_errno_shim`);
  * none       — the node carries IsolationUnavailable=True and HIP is narrowed with
                 HIP_VISIBLE_DEVICES only.
In the enforced tiers HIP_VISIBLE_DEVICES stays unset.
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
                                                     "for n in /dev/dri/*; do if [ -c \"$n\" ]; then "
                                                     "if (exec 3<>\"$n\") 2>/dev/null; then echo \"OPEN $n\"; "
                                                     "else echo \"DENIED $n\"; fi; fi; done; "
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
        mine = f"/dev/dri/renderD{minor}"
        opened = {ln.split()[1] for ln in vlog.splitlines() if ln.startswith("OPEN ")}
        denied = {ln.split()[1] for ln in vlog.splitlines() if ln.startswith("DENIED ")}
        # what the kubelet itself may open: a node the pod is denied only proves confinement if
        # the same user could open it outside the pod
        host_openable = set()
        for n in sorted(os.listdir("/dev/dri")) if os.path.isdir("/dev/dri") else ():
            p = os.path.join("/dev/dri", n)
            try:
                os.close(os.open(p, os.O_RDWR))
                host_openable.add(p)
            except OSError:
                pass
        result["tier"] = iso.get("tier")
        # Landlock tier: kamd-runc preloads the errno shim so a denied sibling node reads EPERM
        # (device-cgroup semantics, skipped by ROCr's thunk) instead of Landlock's EACCES (fatal
        # to hsa_init); the container's isolation report says whether it was in force
        rep_path = os.path.join(os.path.dirname(vcs.log_path), "isolation.json")
        if os.path.exists(rep_path):
            rep = json.load(open(rep_path))
            result["landlock_errno_shim"] = rep.get("devshim")
        result["pod_opened"], result["pod_denied"] = sorted(opened), sorted(denied)
        result["host_openable"] = sorted(host_openable)
        result["confinement_demonstrated"] = bool(iso["enforced"] and (host_openable - {mine}) and
                                                  (host_openable - {mine}) <= denied)
        if iso["enforced"]:
            assert "HIP=unset" in vlog, vlog
            assert mine in opened or iso.get("tier") == "namespaces" and dri == [f"renderD{minor}"], vlog
            if iso.get("tier") == "namespaces":
                assert dri == [f"renderD{minor}"], vlog
            else:
                # Landlock: every node this user could open that is not the pod's is denied
                assert not (opened - {mine}), vlog
                assert (host_openable - {mine}) <= denied, (vlog, host_openable)
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
