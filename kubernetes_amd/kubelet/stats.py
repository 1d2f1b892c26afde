"""Kubelet summary API (`/stats/summary`) with per-container accelerator stats.

Parity: `pkg/kubelet/apis/stats/v1alpha1/types.go:121-122,213-234` (`ContainerStats.Accelerators`:
make, model, id, memoryTotal, memoryUsed, dutyCycle) filled in the reference by cAdvisor's NVML
collector (`vendor/github.com/google/cadvisor/accelerators/nvidia.go:172-222`, devices cgroup
char major 195). Here the container -> GPU mapping comes from the allocation record itself
(`spec.extendedResources[].assigned`), and the numbers from AMD SMI through the native shim.
"""
from __future__ import annotations

import time

from ..api import core
from ..api.meta import now_rfc3339


def _gpu_index(dm):
    """device ID -> (attributes) from the device manager's capacity map."""
    cap, _ = dm.get_capacity()
    return (cap.get(core.AMD_GPU) or {}).get("resources") or {}


def accelerator_stats(kubelet, ids):
    devs = _gpu_index(kubelet.dm)
    smi = None
    h = getattr(kubelet.dm, "handler", None)
    out = []
    for i in ids:
        d = devs.get(i)
        if d is None:
            continue
        attrs = d.get("attributes") or {}
        entry = {"make": "amd", "model": attrs.get(core.ATTR_PRODUCT, ""), "id": i,
                 "memoryTotal": int(attrs.get(core.ATTR_MEMORY, "0")) << 20, "memoryUsed": 0, "dutyCycle": 0}
        try:
            from ..native import amdsmi
            if smi is None:
                smi = getattr(kubelet, "smi", None)
            if smi is not None:
                m = smi.metrics(int(attrs.get(core.ATTR_INDEX, "0")))
                entry["memoryUsed"] = m.vram_used_bytes
                entry["dutyCycle"] = m.gfx_activity
                entry["powerWatts"] = m.power_w
                entry["temperatureC"] = m.temp_hotspot_c
            del amdsmi
        except Exception:
            pass
        out.append(entry)
    del h
    return out


def summary(kubelet):
    now = now_rfc3339()
    pods = []
    for st in kubelet.pods.values():
        pod = st.pod
        md = pod["metadata"]
        containers = []
        for c in (pod.get("spec") or {}).get("containers") or ():
            ids = core.pod_extended_resource_assigned(core.AMD_GPU, c, pod) if c.get("extendedResourceRequests") else []
            cs = {"name": c["name"], "startTime": st.start_time, "cpu": {"time": now}, "memory": {"time": now}}
            acc = accelerator_stats(kubelet, ids)
            if acc:
                cs["accelerators"] = acc
            containers.append(cs)
        pods.append({"podRef": {"name": md["name"], "namespace": md.get("namespace", ""), "uid": md["uid"]},
                     "startTime": st.start_time, "containers": containers})
    return {"node": {"nodeName": kubelet.node_name, "startTime": now, "cpu": {"time": now}, "memory": {"time": now},
                     "systemContainers": [{"name": "kubelet", "startTime": now}]},
            "pods": pods, "time": time.time()}
