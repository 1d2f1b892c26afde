"""amd-smi → Prometheus exporter (replaces the DCGM exporter of the NVIDIA stack; the reference
README promises DCGM → Prometheus → Grafana but ships none of it, `README.md:54-55`).

Per GPU (AMD SMI through the native shim): activity, memory-controller activity, VRAM used /
total, power and cap, hotspot / HBM temperature, ECC correctable / uncorrectable counters,
xGMI links up, GFX clock, health. Per pod: which GPUs it holds — taken from the allocation
record (`spec.extendedResources[].assigned`, via the kubelet's pods endpoint or the API), not
from a devices cgroup scan like cAdvisor's NVML collector (`accelerators/nvidia.go:172-207`).

Serves `/metrics` on :9400 (the DCGM exporter's port) for Prometheus to scrape.
"""
from __future__ import annotations

import json
import logging
import time

from ..api import core
from ..native import amdsmi
from ..utils.httpserver import HTTPServer, Response

log = logging.getLogger("amd-smi-exporter")


def _esc(v):
    return str(v).replace("\\", "\\\\").replace('"', '\\"')


def _labels(d):
    return "{" + ",".join(f'{k}="{_esc(v)}"' for k, v in d.items()) + "}"


GPU_METRICS = [
    ("amd_gpu_gfx_activity_percent", "gauge", "GFX engine activity (%)", lambda m: m.gfx_activity),
    ("amd_gpu_umc_activity_percent", "gauge", "Memory controller activity (%)", lambda m: m.umc_activity),
    ("amd_gpu_vram_used_bytes", "gauge", "HBM used (bytes)", lambda m: m.vram_used_bytes),
    ("amd_gpu_vram_total_bytes", "gauge", "HBM total (bytes)", lambda m: m.vram_total_bytes),
    ("amd_gpu_power_watts", "gauge", "Socket power (W)", lambda m: m.power_w),
    ("amd_gpu_power_cap_watts", "gauge", "Power cap (W)", lambda m: m.power_limit_w),
    ("amd_gpu_temperature_hotspot_celsius", "gauge", "Hotspot temperature (C)", lambda m: m.temp_hotspot_c),
    ("amd_gpu_temperature_hbm_celsius", "gauge", "HBM temperature (C)", lambda m: m.temp_mem_c),
    ("amd_gpu_ecc_correctable_total", "counter", "Correctable ECC errors", lambda m: m.ecc_correctable),
    ("amd_gpu_ecc_uncorrectable_total", "counter", "Uncorrectable ECC errors", lambda m: m.ecc_uncorrectable),
    ("amd_gpu_xgmi_links_up", "gauge", "xGMI links up", lambda m: m.xgmi_links_up),
    ("amd_gpu_xgmi_links_total", "gauge", "xGMI links present", lambda m: m.xgmi_links_total),
    ("amd_gpu_sclk_mhz", "gauge", "GFX clock (MHz)", lambda m: m.sclk_mhz),
]


class AMDSMIExporter:
    def __init__(self, smi: amdsmi.SMI | None = None, node_name="", pods_fn=None, health_fn=None, stats_fn=None):
        self.smi = smi or amdsmi.SMI()
        self.node = node_name
        self.gpus = self.smi.gpus()
        self.pods_fn = pods_fn          # async () -> list of pods on this node (allocation records)
        self.health_fn = health_fn      # (device id) -> "Healthy"/"Unhealthy"
        self.stats_fn = stats_fn        # async () -> the kubelet's /stats/summary (per-container VRAM)
        self.http = None
        self.scrapes = 0

    def _gpu_labels(self, g):
        return {"gpu": g.index, "uuid": g.device_id_str, "bdf": g.bdf, "product": g.product, "arch": g.arch,
                "xgmi_hive": f"{g.xgmi_hive_id:x}", "numa": g.numa_node, "node": self.node}

    async def collect(self) -> str:
        self.scrapes += 1
        lines = []
        t0 = time.perf_counter()
        per_gpu = [(g, self.smi.metrics(g.index)) for g in self.gpus]
        for name, typ, help_, fn in GPU_METRICS:
            lines.append(f"# HELP {name} {help_}")
            lines.append(f"# TYPE {name} {typ}")
            for g, mt in per_gpu:
                lines.append(f"{name}{_labels(self._gpu_labels(g))} {fn(mt)}")
        lines.append("# HELP amd_gpu_healthy 1 if the device plugin reports the GPU Healthy")
        lines.append("# TYPE amd_gpu_healthy gauge")
        for g, mt in per_gpu:
            if self.health_fn is not None:
                h = self.health_fn(g.device_id_str) == core.HEALTHY
            else:
                h = mt.ecc_uncorrectable == 0 and mt.xgmi_links_up >= min(mt.xgmi_links_total, 7)
            lines.append(f"amd_gpu_healthy{_labels(self._gpu_labels(g))} {1 if h else 0}")
        if self.pods_fn is not None:
            lines.append("# HELP amd_gpu_pod_allocated 1 for each (pod, GPU) allocation on this node")
            lines.append("# TYPE amd_gpu_pod_allocated gauge")
            by_id = {g.device_id_str: g for g in self.gpus}
            try:
                pods = await self.pods_fn()
            except Exception as e:  # scrape must not fail because the kubelet is down
                log.warning("pod attribution unavailable: %s", e)
                pods = []
            for p in pods:
                if core.pod_is_terminal(p):
                    continue
                for c in (p.get("spec") or {}).get("containers") or ():
                    if not c.get("extendedResourceRequests"):
                        continue
                    for did in core.pod_extended_resource_assigned(core.AMD_GPU, c, p):
                        g = by_id.get(did)
                        lab = {"namespace": p["metadata"].get("namespace", ""), "pod": p["metadata"]["name"],
                               "container": c["name"], "uuid": did, "gpu": g.index if g else "", "node": self.node}
                        lines.append(f"amd_gpu_pod_allocated{_labels(lab)} 1")
        if self.stats_fn is not None:
            # per-container attribution is the kubelet's (AMD SMI process list joined with the
            # runtime's container processes): the exporter republishes it per pod
            try:
                summ = await self.stats_fn()
            except Exception as e:  # scrape must not fail because the kubelet is down
                log.warning("per-pod GPU usage unavailable: %s", e)
                summ = {}
            by_id = {g.device_id_str: g for g in self.gpus}
            rows = []
            for p in summ.get("pods") or ():
                ref = p.get("podRef") or {}
                for c in p.get("containers") or ():
                    for a in c.get("accelerators") or ():
                        g = by_id.get(a.get("id"))
                        lab = {"namespace": ref.get("namespace", ""), "pod": ref.get("name", ""), "container": c.get("name", ""),
                               "uuid": a.get("id", ""), "gpu": g.index if g else "", "node": self.node}
                        rows.append((lab, a))
            lines.append("# HELP amd_gpu_pod_vram_bytes HBM used by the container's own GPU processes (bytes)")
            lines.append("# TYPE amd_gpu_pod_vram_bytes gauge")
            for lab, a in rows:
                lines.append(f"amd_gpu_pod_vram_bytes{_labels(lab)} {int(a.get('memoryUsed', 0))}")
            lines.append("# HELP amd_gpu_pod_gfx_busy_percent the container's share of the gfx engine (%)")
            lines.append("# TYPE amd_gpu_pod_gfx_busy_percent gauge")
            for lab, a in rows:
                lines.append(f"amd_gpu_pod_gfx_busy_percent{_labels(lab)} {int(a.get('dutyCycle', 0))}")
        lines.append("# TYPE amd_smi_exporter_scrape_seconds gauge")
        lines.append(f"amd_smi_exporter_scrape_seconds {time.perf_counter() - t0:.6f}")
        return "\n".join(lines) + "\n"

    async def _handle(self, req):
        if req.path == "/metrics":
            return Response(200, (await self.collect()).encode(), "text/plain; version=0.0.4")
        if req.path == "/healthz":
            return Response(200, b"ok", "text/plain")
        if req.path == "/gpus":
            return Response(200, json.dumps([self._gpu_labels(g) | {"vram_total_mb": g.vram_total_mb} for g in self.gpus]).encode())
        return Response(404, b"not found", "text/plain")

    async def start(self, host="0.0.0.0", port=9400):
        self.http = HTTPServer(self._handle)
        return await self.http.start(host, port)

    async def stop(self):
        if self.http:
            await self.http.stop()


def kubelet_stats_fn(kubelet_url):
    from ..client.http import HTTPClient

    async def fn():
        c = HTTPClient(kubelet_url)
        try:
            st, body = await c.request("GET", "/stats/summary")
        finally:
            await c.close()
        return json.loads(body) if st == 200 else {}
    return fn


def kubelet_pods_fn(kubelet_url):
    from ..client.http import HTTPClient

    async def fn():
        c = HTTPClient(kubelet_url)
        try:
            st, body = await c.request("GET", "/pods")
        finally:
            await c.close()
        return json.loads(body).get("items", []) if st == 200 else []
    return fn

