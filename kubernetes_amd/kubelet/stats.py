"""Kubelet summary API (`/stats/summary`) with per-container accelerator stats.

Parity: `pkg/kubelet/apis/stats/v1alpha1/types.go:121-122,213-234` (`ContainerStats.Accelerators`:
make, model, id, memoryTotal, memoryUsed, dutyCycle) filled in the reference by cAdvisor's NVML
collector (`vendor/github.com/google/cadvisor/accelerators/nvidia.go:172-222`, devices cgroup
char major 195), which reports the DEVICE's memory use for every container holding it. Here:
  * the container -> GPU mapping comes from the allocation record itself
    (`spec.extendedResources[].assigned`);
  * memory is attributed PER CONTAINER, from the container's own processes: the DRM fdinfo
    of every open render node (`/proc/<pid>/fdinfo/<fd>`: drm-pdev, drm-client-id,
    drm-resident-vram — amdgpu accounts KFD/HIP allocations to the render-node file whose VM
    they share), summed over the container's process tree and deduplicated by client id. This
    works inside pid namespaces, where AMD SMI's process list (`amdsmi_get_gpu_process_list`)
    reports host pids the kubelet cannot see; that list is the fallback when fdinfo carries no
    memory keys (older kernels) and the pids are the kubelet's own. Two pods sharing a GPU
    (compute partitions, or a multi-tenant device) are therefore not both charged the whole
    device. `memoryUsed` is the container's own VRAM, `deviceMemoryUsed` the device's;
    `dutyCycle` is the container's share of the gfx engine over the last sampling interval when
    its processes report engine time, else the device's activity.
"""
from __future__ import annotations

import logging
import time

from ..api import core
from ..api.meta import now_rfc3339

log = logging.getLogger("kubelet.stats")


def _gpu_index(dm):
    """device ID -> (attributes) from the device manager's capacity map."""
    cap, _ = dm.get_capacity()
    return (cap.get(core.AMD_GPU) or {}).get("resources") or {}


def _ppid(pid):
    try:
        with open(f"/proc/{pid}/stat") as f:
            return int(f.read().rsplit(")", 1)[1].split()[1])
    except (OSError, ValueError, IndexError):
        return 0


def _descendants(root):
    """root and every process below it (/proc/<pid>/task/<tid>/children)."""
    import os
    out, todo = [], [root]
    while todo and len(out) < 4096:
        pid = todo.pop()
        out.append(pid)
        try:
            for tid in os.listdir(f"/proc/{pid}/task"):
                try:
                    with open(f"/proc/{pid}/task/{tid}/children") as f:
                        todo.extend(int(x) for x in f.read().split())
                except (OSError, ValueError):
                    pass
        except OSError:
            pass
    return out


def _drm_fdinfo(pid):
    """[(pdev, client id, resident VRAM bytes, gfx engine ns)] of the render nodes pid has open."""
    import os
    out = []
    try:
        fds = os.listdir(f"/proc/{pid}/fd")
    except OSError:
        return out
    for fd in fds:
        try:
            if not os.readlink(f"/proc/{pid}/fd/{fd}").startswith("/dev/dri/"):
                continue
            with open(f"/proc/{pid}/fdinfo/{fd}") as f:
                info = f.read()
        except OSError:
            continue
        kv = {}
        for line in info.splitlines():
            k, _, v = line.partition(":")
            kv[k.strip()] = v.strip()
        if "drm-pdev" not in kv:
            continue
        vram = kv.get("drm-resident-vram") or kv.get("drm-memory-vram")
        if vram is None:
            continue
        n, _, unit = vram.partition(" ")
        mult = {"KiB": 1 << 10, "MiB": 1 << 20, "GiB": 1 << 30}.get(unit.strip(), 1)
        gfx = kv.get("drm-engine-gfx", "0").split()[0]
        try:
            out.append((kv["drm-pdev"], kv.get("drm-client-id", f"{pid}/{fd}"), int(n) * mult, int(gfx)))
        except ValueError:
            continue
    return out


def gpu_process_usage(kubelet):
    """{container id: {device BDF: (vram bytes, gfx engine ns)}} — each GPU client charged to the
    container whose root process is its ancestor."""
    pids_fn = getattr(kubelet.runtime, "container_pids", None)
    if pids_fn is None:
        return {}
    roots = pids_fn()
    if not roots:
        return {}
    out: dict = {}
    for cid, root in roots.items():
        seen = set()
        for pid in _descendants(root):
            for pdev, client, vram, gfx in _drm_fdinfo(pid):
                if (pdev, client) in seen:
                    continue
                seen.add((pdev, client))
                v, g = out.setdefault(cid, {}).get(pdev, (0, 0))
                out[cid][pdev] = (v + vram, g + gfx)
    smi = getattr(kubelet, "smi", None)
    if smi is None:
        return out
    # AMD SMI's process list: its pids are the host's, usable when the kubelet shares the pid
    # namespace (and the only source without DRM fdinfo memory keys)
    from ..native.amdsmi import SMIError
    by_root = {pid: cid for cid, pid in roots.items()}
    for i in range(smi.count()):
        try:
            procs = smi.processes(i)
            bdf = smi.gpu(i).bdf if procs else ""
        except SMIError as e:
            log.warning("AMD SMI process list of GPU %d: %s", i, e)
            continue
        for p in procs:
            pid, depth = p.pid, 0
            while pid > 1 and pid not in by_root and depth < 64:
                pid, depth = _ppid(pid), depth + 1
            cid = by_root.get(pid)
            if cid is None or bdf in out.get(cid, {}):
                continue        # fdinfo already accounted this container on this device
            per = out.setdefault(cid, {})
            v, g = per.get(("smi", bdf), (0, 0))
            per[("smi", bdf)] = (v + p.vram_bytes, g + p.gfx_ns)
    for per in out.values():
        for k in [k for k in per if isinstance(k, tuple)]:
            per[k[1]] = per.pop(k)
    return out


def accelerator_stats(kubelet, ids, usage=None, cid=None, now=None):
    """ContainerStats.Accelerators for the device IDs a container holds. `usage`: the result of
    gpu_process_usage() for this summary (per-container VRAM / engine time)."""
    devs = _gpu_index(kubelet.dm)
    smi = getattr(kubelet, "smi", None)
    mine = (usage or {}).get(cid, {}) if cid else {}
    samples = kubelet.__dict__.setdefault("_gfx_samples", {})
    out = []
    for i in ids:
        d = devs.get(i)
        if d is None:
            continue
        attrs = d.get("attributes") or {}
        idx = int(attrs.get(core.ATTR_INDEX, "0"))
        bdf = attrs.get(core.ATTR_BDF, "")
        entry = {"make": "amd", "model": attrs.get(core.ATTR_PRODUCT, ""), "id": i,
                 "memoryTotal": int(attrs.get(core.ATTR_MEMORY, "0")) << 20, "memoryUsed": 0, "dutyCycle": 0}
        if smi is not None:
            from ..native.amdsmi import SMIError
            try:
                m = smi.metrics(idx)
            except SMIError as e:
                log.warning("AMD SMI metrics of GPU %d: %s", idx, e)
                m = None
            if m is not None:
                entry["deviceMemoryUsed"] = m.vram_used_bytes
                entry["dutyCycle"] = m.gfx_activity
                entry["powerWatts"] = m.power_w
                entry["temperatureC"] = m.temp_hotspot_c
        if bdf in mine:
            vram, gfx = mine[bdf]
            entry["memoryUsed"] = vram
            prev = samples.get((cid, bdf))
            samples[(cid, bdf)] = (now or time.time(), gfx)
            if prev is not None and gfx and now and now > prev[0]:
                entry["dutyCycle"] = max(0, min(100, int(round((gfx - prev[1]) / ((now - prev[0]) * 1e9) * 100))))
        out.append(entry)
    return out


SIM_CPU = "kubemark.amd.com/cpu-millicores"       # stub runtime: simulated usage (kubemark)
SIM_MEM = "kubemark.amd.com/memory-bytes"
SIM_GPU = "kubemark.amd.com/gpu-utilization"


def _proc_usage(pid):
    """(cumulative CPU ns, RSS bytes) of a process tree root (cAdvisor reads the cgroup)."""
    import os
    try:
        with open(f"/proc/{pid}/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        cpu = (int(fields[11]) + int(fields[12])) * (1_000_000_000 // os.sysconf("SC_CLK_TCK"))
        with open(f"/proc/{pid}/statm") as f:
            rss = int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE")
        return cpu, rss
    except (OSError, IndexError, ValueError):
        return None


def container_usage(kubelet, pod, cid, now):
    """{usageNanoCores, usageCoreNanoSeconds, workingSetBytes} for one container."""
    ann = pod["metadata"].get("annotations") or {}
    if SIM_CPU in ann or SIM_MEM in ann:
        milli = float(ann.get(SIM_CPU, 0))
        return {"usageNanoCores": int(milli * 1e6), "usageCoreNanoSeconds": 0, "workingSetBytes": int(float(ann.get(SIM_MEM, 0)))}
    meta = (getattr(kubelet.runtime, "meta", {}) or {}).get(cid) or {}
    proc = meta.get("proc")
    if proc is None or getattr(proc, "returncode", 1) is not None:
        return None
    u = _proc_usage(proc.pid)
    if u is None:
        return None
    cpu, rss = u
    prev = kubelet._cpu_samples.get(cid)
    kubelet._cpu_samples[cid] = (now, cpu)
    nano_cores = int((cpu - prev[1]) / max(1e-9, now - prev[0])) if prev and now > prev[0] else 0
    return {"usageNanoCores": nano_cores, "usageCoreNanoSeconds": cpu, "workingSetBytes": rss}


def summary(kubelet):
    now = now_rfc3339()
    t = time.time()
    if not hasattr(kubelet, "_cpu_samples"):
        kubelet._cpu_samples = {}
    pods = []
    node_cpu = node_mem = 0
    usage = gpu_process_usage(kubelet)
    for st in kubelet.pods.values():
        pod = st.pod
        md = pod["metadata"]
        containers = []
        for c in (pod.get("spec") or {}).get("containers") or ():
            ids = core.pod_extended_resource_assigned(core.AMD_GPU, c, pod) if c.get("extendedResourceRequests") else []
            cs = {"name": c["name"], "startTime": st.start_time, "cpu": {"time": now}, "memory": {"time": now}}
            cid = st.containers.get(c["name"])
            u = container_usage(kubelet, pod, cid, t) if cid else None
            if u is not None:
                cs["cpu"].update(usageNanoCores=u["usageNanoCores"], usageCoreNanoSeconds=u["usageCoreNanoSeconds"])
                cs["memory"].update(workingSetBytes=u["workingSetBytes"], usageBytes=u["workingSetBytes"])
                node_cpu += u["usageNanoCores"]
                node_mem += u["workingSetBytes"]
            acc = accelerator_stats(kubelet, ids, usage, cid, t)
            sim_gpu = (md.get("annotations") or {}).get(SIM_GPU)
            if acc and sim_gpu is not None:
                for a in acc:
                    a["dutyCycle"] = int(float(sim_gpu))
            if acc:
                cs["accelerators"] = acc
            containers.append(cs)
        pods.append({"podRef": {"name": md["name"], "namespace": md.get("namespace", ""), "uid": md["uid"]},
                     "startTime": st.start_time, "containers": containers})
    return {"node": {"nodeName": kubelet.node_name, "startTime": now,
                     "cpu": {"time": now, "usageNanoCores": node_cpu}, "memory": {"time": now, "workingSetBytes": node_mem},
                     "systemContainers": [{"name": "kubelet", "startTime": now}]},
            "pods": pods, "time": time.time()}


def _read(path, default=""):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return default


def machine_info(kubelet):
    """/spec: cAdvisor `MachineInfo` (num_cores, memory_capacity, machine_id, system_uuid,
    boot_id, topology by NUMA node) for this node, plus the AMD accelerators the device plugin
    advertises (the role cAdvisor's accelerator collector plays). Capacity values are the
    kubelet's own (hollow nodes report their configured capacity)."""
    import os

    from ..api.quantity import parse_quantity
    cap = kubelet.capacity
    topo = []
    node_dir = "/sys/devices/system/node"
    try:
        nodes = sorted(int(d[4:]) for d in os.listdir(node_dir) if d.startswith("node") and d[4:].isdigit())
    except OSError:
        nodes = []
    for n in nodes:
        cpus = _read(f"{node_dir}/node{n}/cpulist")
        mem = 0
        for ln in _read(f"{node_dir}/node{n}/meminfo").splitlines():
            if "MemTotal" in ln:
                mem = int(ln.split()[-2]) * 1024
        topo.append({"node_id": n, "memory": mem, "cpulist": cpus})
    accels = []
    for dev_id, dev in sorted(_gpu_index(kubelet.dm).items()):
        attrs = dev.get("attributes") or {}
        accels.append({"make": "amd", "model": attrs.get("amd.com/product", ""), "id": dev_id,
                       "arch": attrs.get("amd.com/arch", ""), "numa_node": attrs.get("amd.com/numa", ""),
                       "xgmi_hive": attrs.get("amd.com/xgmi-hive", ""),
                       "memory_total_mib": int(attrs.get("amd.com/memory", "0") or 0), "health": dev.get("health", "")})
    return {"num_cores": int(parse_quantity(str(cap["cpu"])).value),
            "memory_capacity": int(parse_quantity(str(cap["memory"])).value),
            "machine_id": _read("/etc/machine-id") or kubelet.node_name,
            "system_uuid": _read("/sys/class/dmi/id/product_uuid") or kubelet.node_name,
            "boot_id": _read("/proc/sys/kernel/random/boot_id"),
            "topology": topo, "accelerators": accels, "cloud_provider": "None", "instance_type": "Unknown"}


def _du(path):
    """(bytes, inodes) under `path` (no symlink following)."""
    import os
    total = files = 0
    for root, dirs, names in os.walk(path, followlinks=False):
        for n in names + dirs:
            try:
                st = os.lstat(os.path.join(root, n))
            except OSError:
                continue
            total += st.st_blocks * 512 if st.st_blocks else st.st_size
            files += 1
    return total, files


def pod_eviction_stats(kubelet, pod):
    """Per-pod usage for the eviction manager's ranking (`makeSignalObservations` statsFunc):
    memory = the containers' working set; disk / inodes = local emptyDir volumes plus container
    logs (no dedicated image fs); volumes = emptyDir usage by name. None when the pod is not
    tracked (ranked first, like the reference's missing stats)."""
    import os
    st = kubelet.pods.get(pod["metadata"].get("uid"))
    if st is None:
        return None
    ann = pod["metadata"].get("annotations") or {}
    mem = 0
    if SIM_MEM in ann:
        mem = int(float(ann.get(SIM_MEM, 0)))
    else:
        meta = getattr(kubelet.runtime, "meta", {}) or {}
        for cid in st.containers.values():
            proc = (meta.get(cid) or {}).get("proc") if cid else None
            if proc is not None and getattr(proc, "returncode", 1) is None:
                u = _proc_usage(proc.pid)
                if u is not None:
                    mem += u[1]
    disk = inodes = 0
    vols, per_container = {}, {}
    base = os.path.join(kubelet.volumes.pod_dir(pod), "volumes")
    for v in (pod.get("spec") or {}).get("volumes") or ():
        if "emptyDir" in v and (v.get("emptyDir") or {}).get("medium") != "Memory":
            b, n = _du(os.path.join(base, v["name"]))
            vols[v["name"]] = b
            disk += b
            inodes += n
    logs = getattr(kubelet, "container_log_dir", None)
    if logs and os.path.isdir(logs):
        md = pod["metadata"]
        prefix = f"{md['name']}_{md.get('namespace', 'default')}_"
        try:
            for name in os.listdir(logs):
                if name.startswith(prefix):
                    try:
                        size = os.stat(os.path.join(logs, name)).st_size
                    except OSError:
                        continue
                    disk += size
                    inodes += 1
                    cname = name[len(prefix):].rsplit("-", 1)[0]
                    per_container[cname] = per_container.get(cname, 0) + size
        except OSError:
            pass
    return {"memory": mem, "disk": disk, "inodes": inodes, "volumes": vols, "containers": per_container}
