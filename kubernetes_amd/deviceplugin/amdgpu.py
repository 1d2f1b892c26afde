"""The `amd.com/gpu` device plugin for MI355X (gfx950, 288 GB HBM3E).

Replaces the out-of-tree NVIDIA plugin the reference targets (NVML enumeration,
`NVIDIA_VISIBLE_DEVICES`, nvidia-container-runtime routing). Here:
  * enumeration + health come from AMD SMI through the native shim (`native/amdsmi_shim`);
  * each device advertises vendor-prefixed attributes (api.proto:99 "Attributes must start
    by vendor name") used by the scheduler's selectors and topology-aware allocator:
      amd.com/arch=gfx950  amd.com/product=MI355X  amd.com/memory=<MiB>  amd.com/hbm=288Gi
      amd.com/xgmi-hive=<hex>  amd.com/numa=<n>  amd.com/bdf  amd.com/render-minor
      amd.com/index  amd.com/partition=SPX|CPX…  amd.com/ecc=<uncorrectable>  amd.com/compute-units
      amd.com/socket (physical package)  amd.com/partition-id  amd.com/memory-partition=NPS1|NPS2
  * InitContainer injects the shared `/dev/kfd` plus one `/dev/dri/renderD<minor>` per GPU
    (no vendor runtime, no NVML/CUDA shim) and, optionally, the ROCm userspace read-only;
    `AMD_VISIBLE_DEVICES` lists the host HIP ordinals (informational, like
    NVIDIA_VISIBLE_DEVICES) — a non-isolating runtime turns it into HIP_VISIBLE_DEVICES.
  * burn-in (optional, deviceplugin/burnin.py): each GPU runs the framework's HIP vector_add,
    MFMA GEMM and HBM-copy kernels before it is offered; it stays Unhealthy until it passes,
    and the measured TFLOP/s and GB/s become attributes (`amd.com/mfma-tflops`, `amd.com/hbm-gbps`);
  * health: a device turns Unhealthy when its uncorrectable ECC count rises above the
    baseline seen at start, when an xGMI link goes down, or (real backend) when its render
    node disappears; the change is pushed on every open ListAndWatch stream.
"""
from __future__ import annotations

import asyncio
import logging
import os

from ..api import core
from ..native import amdsmi
from . import api
from .burnin import FAILED, PASSED, PENDING
from .server import DevicePluginServer, device

ATTR_BURN_IN = "amd.com/burn-in"          # pending / passed / failed
ATTR_MFMA_TFLOPS = "amd.com/mfma-tflops"  # measured bf16 MFMA GEMM throughput
ATTR_HBM_GBPS = "amd.com/hbm-gbps"        # measured HBM copy bandwidth
ATTR_MFMA_FP8_TFLOPS = "amd.com/mfma-fp8-tflops"   # measured fp8 (e4m3, block-scaled MFMA) GEMM throughput
ATTR_XGMI_P2P_GBPS = "amd.com/xgmi-p2p-gbps"        # slowest measured peer copy to a hive peer

log = logging.getLogger("amdgpu-plugin")


def xgmi_peer_map(smi: amdsmi.SMI, gpus) -> dict:
    """Pairwise xGMI connectivity inside each hive, from the SMI link table
    (`amdsmi_topo_get_link_type` + `amdsmi_is_P2P_accessible`): device index ->
    (hive-local package index, bitmask of hive-local indices it reaches over a direct xGMI link).
    A package is indexed by its rank among the hive's packages (ordered by socket); compute
    partitions of one package share its index and reach each other on-package."""
    by_hive: dict = {}
    for g in gpus:
        by_hive.setdefault(g.xgmi_hive_id, set()).add(g.socket if g.socket >= 0 else g.index)
    local = {h: {s: k for k, s in enumerate(sorted(socks))} for h, socks in by_hive.items()}
    rep = {}                                  # (hive, socket) -> one device index of that package
    for g in gpus:
        rep.setdefault((g.xgmi_hive_id, g.socket if g.socket >= 0 else g.index), g.index)
    out = {}
    for g in gpus:
        sock = g.socket if g.socket >= 0 else g.index
        me = local[g.xgmi_hive_id][sock]
        mask = 1 << me
        for other, k in local[g.xgmi_hive_id].items():
            if other == sock:
                continue
            lk = smi.link(g.index, rep[(g.xgmi_hive_id, other)])
            if lk.type == amdsmi.LINK_XGMI and lk.p2p:
                mask |= 1 << k
        out[g.index] = (me, mask)
    return out


def gpu_attributes(g: amdsmi.GPU, m: amdsmi.Metrics | None = None, peers: tuple | None = None) -> dict:
    # usable VRAM is reported a few MiB below the 288 GB HBM3E stack size: round up to GiB
    hbm_gib = -(-g.vram_total_mb // 1024)
    attrs = {
        core.ATTR_ARCH: g.arch or "unknown",
        core.ATTR_PRODUCT: g.product,
        core.ATTR_MEMORY: str(g.vram_total_mb),
        core.ATTR_HBM: f"{hbm_gib}Gi",
        core.ATTR_HIVE: f"{g.xgmi_hive_id:x}",
        core.ATTR_NUMA: str(g.numa_node),
        core.ATTR_BDF: g.bdf,
        core.ATTR_RENDER_MINOR: str(g.render_minor),
        core.ATTR_CARD_MINOR: str(g.card_minor),
        core.ATTR_INDEX: str(g.hip_id if g.hip_id >= 0 else g.index),
        core.ATTR_PARTITION: g.compute_partition or "SPX",
        core.ATTR_CUS: str(g.compute_units),
        # compute partitions (DPX/QPX/CPX) of one package share its socket: the scheduler packs
        # multi-partition requests onto as few packages as possible
        core.ATTR_SOCKET: str(g.socket if g.socket >= 0 else g.index),
    }
    if g.partition_id >= 0:
        attrs[core.ATTR_PARTITION_ID] = str(g.partition_id)
    if g.memory_partition:
        attrs[core.ATTR_MEMORY_PARTITION] = g.memory_partition
    if m is not None:
        attrs[core.ATTR_ECC] = str(m.ecc_uncorrectable)
        attrs[core.ATTR_XGMI_LINKS] = str(m.xgmi_links_up)
    if peers is not None:
        attrs[core.ATTR_XGMI_NODE] = str(peers[0])
        attrs[core.ATTR_XGMI_PEERS] = f"{peers[1]:x}"
    return attrs


class AMDGPUPlugin(DevicePluginServer):
    def __init__(self, plugins_dir: str, smi: amdsmi.SMI | None = None, socket_name="amdgpu.sock",
                 health_interval=5.0, dev_root="/dev", rocm_mount: str | None = None, indices=None,
                 check_dev_nodes: bool | None = None, init_timeout=10, burn_in=None, link_probe=None,
                 link_min_gbps=None):
        self.smi = smi or amdsmi.SMI()
        # optional xGMI link probe (deviceplugin/linkprobe.py): hip ordinals -> ProbeResult;
        # links measured below link_min_gbps leave the published link graph
        from .linkprobe import DEFAULT_MIN_GBPS
        self.link_probe = link_probe
        self.link_min_gbps = DEFAULT_MIN_GBPS if link_min_gbps is None else link_min_gbps
        self._weak: set = set()
        self._p2p: dict = {}                      # device index -> slowest measured peer copy GB/s
        self._probe_task = None
        # optional acceptance test (deviceplugin/burnin.py): devices stay Unhealthy until it
        # passes; `burn_in` is a BurnIn or any object with run(hip_index) -> BurnInResult
        self.burn_in = burn_in
        self._burn: dict[str, object] = {}        # device id -> BurnInResult (absent = pending)
        self._burn_task = None
        self.dev_root = dev_root
        self.rocm_mount = rocm_mount
        self.health_interval = health_interval
        self.check_dev_nodes = (not self.smi.is_fake) if check_dev_nodes is None else check_dev_nodes
        all_gpus = self.smi.gpus()
        self.gpus = [g for g in all_gpus if indices is None or g.index in indices]
        self.by_id = {g.device_id_str: g for g in self.gpus}
        # published per device so the scheduler places a multi-GPU set on a clique of the link
        # graph, not merely on devices with enough links (a 6/7-link GPU must not be paired with
        # the one peer it cannot reach)
        self._all_gpus = all_gpus
        self.peers = self._peer_map()
        self._ecc_base = {}
        self._health = {}
        devs = []
        for g in self.gpus:
            m = self.smi.metrics(g.index)
            self._ecc_base[g.index] = m.ecc_uncorrectable
            self._links_base = getattr(self, "_links_base", {})
            self._links_base[g.index] = m.xgmi_links_up
            h = self._check(g, m)
            self._health[g.device_id_str] = h
            devs.append(self._device(g, m, h))
        labels = {}
        if self.gpus:
            g0 = self.gpus[0]
            labels = {"amd.com/gpu.arch": g0.arch, "amd.com/gpu.product": g0.product,
                      "amd.com/gpu.count": str(len(self.gpus)),
                      "amd.com/gpu.hbm": f"{-(-g0.vram_total_mb // 1024)}Gi"}
        super().__init__(core.AMD_GPU, os.path.join(plugins_dir, "amd.com", socket_name), devs,
                         init_timeout=init_timeout, labels=labels)
        self._health_task = None

    # -- health -------------------------------------------------------------
    def _peer_map(self):
        from .linkprobe import prune_peers
        peers = xgmi_peer_map(self.smi, self._all_gpus)
        hip_of = {g.index: (g.hip_id if g.hip_id >= 0 else g.index) for g in self._all_gpus}
        return prune_peers(peers, hip_of, self._weak)

    async def run_link_probe(self):
        """Measure peer-to-peer copies inside each hive of this plugin's GPUs; weak links leave
        the peer map (pushed to the kubelet like any health change). Returns the weak pairs."""
        loop = asyncio.get_running_loop()
        by_hive: dict = {}
        for g in self.gpus:
            by_hive.setdefault(g.xgmi_hive_id, []).append(g)
        weak = set()
        for hive, gs in by_hive.items():
            hips = sorted({g.hip_id if g.hip_id >= 0 else g.index for g in gs})
            r = await loop.run_in_executor(None, self.link_probe, hips)
            if r.error:
                log.warning("xGMI link probe of hive %x skipped: %s", hive, r.error)
                continue
            w = r.weak_pairs(self.link_min_gbps)
            for pair in w:
                log.error("xGMI link %s measured below %.0f GB/s: removed from the link graph",
                          "<->".join(str(x) for x in sorted(pair)), self.link_min_gbps)
            weak |= w
            for g in gs:
                h = g.hip_id if g.hip_id >= 0 else g.index
                vals = [v for (a, b), v in r.pairs.items() if a == h or b == h]
                if vals:
                    self._p2p[g.index] = min(vals)
        self._weak = weak
        self.poll_health(force=True)
        return weak

    def _device(self, g: amdsmi.GPU, m: amdsmi.Metrics, health: str):
        attrs = gpu_attributes(g, m, self.peers.get(g.index))
        if g.index in self._p2p:
            attrs[ATTR_XGMI_P2P_GBPS] = str(int(self._p2p[g.index]))
        if self.burn_in is not None:
            r = self._burn.get(g.device_id_str)
            attrs[ATTR_BURN_IN] = PENDING if r is None else (PASSED if r.ok else FAILED)
            if r is not None and r.tflops:
                attrs[ATTR_MFMA_TFLOPS] = str(int(r.tflops))
                attrs[ATTR_HBM_GBPS] = str(int(r.hbm_gbps))
                if r.fp8_tflops:
                    attrs[ATTR_MFMA_FP8_TFLOPS] = str(int(r.fp8_tflops))
        return device(g.device_id_str, health, attrs)

    def _check(self, g: amdsmi.GPU, m: amdsmi.Metrics) -> str:
        if self.burn_in is not None:
            r = self._burn.get(g.device_id_str)
            if r is None or not r.ok:
                return api.UNHEALTHY
        if m.ecc_uncorrectable > self._ecc_base.get(g.index, 0):
            return api.UNHEALTHY
        if m.xgmi_links_up < self._links_base.get(g.index, 0):
            return api.UNHEALTHY
        if self.check_dev_nodes and not os.path.exists(os.path.join(self.dev_root, "dri", f"renderD{g.render_minor}")):
            return api.UNHEALTHY
        return api.HEALTHY

    def poll_health(self, force=False) -> bool:
        """Re-evaluate health; push a new list if anything changed. Returns True if changed."""
        changed = False
        devs = []
        peers = self._peer_map()
        if peers != self.peers:
            log.warning("xGMI peer map changed: %s -> %s", self.peers, peers)
            self.peers = peers
            changed = True
        for g in self.gpus:
            m = self.smi.metrics(g.index)
            h = self._check(g, m)
            if h != self._health.get(g.device_id_str):
                log.warning("device %s health %s -> %s", g.device_id_str, self._health.get(g.device_id_str), h)
                self._health[g.device_id_str] = h
                changed = True
            devs.append(self._device(g, m, h))
        if changed or force:
            self.update(devs)
        return changed

    async def run_burn_in(self):
        """Run the acceptance test on every device (one worker thread per GPU: the HIP calls
        release the GIL and each thread binds its own device), publishing each result as it
        lands. Returns {device id: BurnInResult}."""
        loop = asyncio.get_running_loop()
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(max(1, len(self.gpus)), thread_name_prefix="burn-in")

        async def one(g):
            r = await loop.run_in_executor(pool, self.burn_in.run, g.hip_id if g.hip_id >= 0 else g.index)
            self._burn[g.device_id_str] = r
            if r.ok:
                log.info("burn-in passed on %s: %.0f TFLOP/s MFMA bf16, %.0f fp8, %.0f GB/s HBM (%.1f s)",
                         g.device_id_str, r.tflops, r.fp8_tflops, r.hbm_gbps, r.seconds)
            else:
                log.error("burn-in FAILED on %s: %s", g.device_id_str, r.reason)
            self.poll_health(force=True)
        try:
            await asyncio.gather(*(one(g) for g in self.gpus))
        finally:
            pool.shutdown(wait=False)
        return dict(self._burn)

    async def _health_loop(self):
        while True:
            await asyncio.sleep(self.health_interval)
            try:
                self.poll_health()
            except Exception:
                log.exception("health poll failed")

    async def start(self):
        await super().start()
        if self.health_interval:
            self._health_task = asyncio.ensure_future(self._health_loop())
        if self.burn_in is not None or self.link_probe is not None:
            self._burn_task = asyncio.ensure_future(self._acceptance())
        return self

    async def _acceptance(self):
        """Burn-in first (it owns the GPUs while it runs), then the link probe."""
        if self.burn_in is not None:
            await self.run_burn_in()
        if self.link_probe is not None:
            await self.run_link_probe()

    async def stop(self, grace=0.1):
        if self._health_task:
            self._health_task.cancel()
        if self._burn_task:
            self._burn_task.cancel()
        await super().stop(grace)

    # -- allocation hooks -------------------------------------------------------------
    def _gpus_for(self, ids):
        out = []
        for i in ids:
            g = self.by_id.get(i)
            if g is None:
                raise ValueError(f"unknown device {i}")
            out.append(g)
        return out

    async def admit_pod(self, request) -> dict:
        ids = set()
        for c in list(request.init_containers.values()) + list(request.containers.values()):
            ids.update(c.devices)
        gpus = self._gpus_for(sorted(ids))  # raises -> gRPC error -> kubelet rejects the pod
        for g in gpus:
            if self._health.get(g.device_id_str) != api.HEALTHY:
                raise ValueError(f"device {g.device_id_str} is unhealthy")
        if not gpus:
            return {}
        return {"amd.com/gpu-devices": ",".join(g.device_id_str for g in gpus),
                "amd.com/xgmi-hive": ",".join(sorted({f"{g.xgmi_hive_id:x}" for g in gpus}))}

    async def init_container(self, container) -> dict:
        gpus = self._gpus_for(list(container.devices))
        if not gpus:
            return {}
        kfd = os.path.join(self.dev_root, "kfd")
        devs = [{"container_path": "/dev/kfd", "host_path": kfd, "permissions": "rw"}]
        for g in gpus:
            node = f"renderD{g.render_minor}"
            devs.append({"container_path": f"/dev/dri/{node}", "host_path": os.path.join(self.dev_root, "dri", node),
                         "permissions": "rw"})
        mounts = []
        if self.rocm_mount:
            mounts.append({"container_path": self.rocm_mount, "host_path": self.rocm_mount, "read_only": True})
        ordinals = ",".join(str(g.hip_id if g.hip_id >= 0 else g.index) for g in gpus)
        envs = {"AMD_VISIBLE_DEVICES": ordinals,
                "AMD_GPU_DEVICE_IDS": ",".join(g.device_id_str for g in gpus),
                "AMD_GPU_ARCH": gpus[0].arch}
        return {"envs": envs, "mounts": mounts, "devices": devs,
                "annotations": {"amd.com/gpu-render-nodes": ",".join(f"renderD{g.render_minor}" for g in gpus)}}
