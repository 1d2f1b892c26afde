"""ctypes binding for `libkamd_smi.so` (native/amdsmi_shim).

Two backends behind one API:
  * real — AMD SMI (`libamd_smi.so` dlopen()ed by the shim) on a GPU host;
  * fake — a JSON fixture (default: 8 x MI355X in one xGMI hive, `FIXTURE_8X_MI355X`).

Used by the amd.com/gpu device plugin (enumeration + health), the kubelet summary
stats (per-container accelerator stats, the role of cAdvisor's NVML collector
`vendor/github.com/google/cadvisor/accelerators/nvidia.go`) and the amd-smi exporter.
"""
from __future__ import annotations

import ctypes
import json
import os
import tempfile
import threading
from dataclasses import dataclass, field

from . import LIB_DIR

STR = 128
BACKEND_NONE, BACKEND_AMDSMI, BACKEND_FAKE = 0, 1, 2
LINK_UNKNOWN, LINK_PCIE, LINK_XGMI = 0, 1, 2


class _Info(ctypes.Structure):
    _fields_ = [
        ("index", ctypes.c_int32), ("uuid", ctypes.c_char * STR), ("bdf", ctypes.c_char * 32),
        ("market_name", ctypes.c_char * STR), ("arch", ctypes.c_char * 32), ("vendor_id", ctypes.c_uint32),
        ("device_id", ctypes.c_uint64), ("vram_total_mb", ctypes.c_uint64), ("compute_units", ctypes.c_uint32),
        ("render_minor", ctypes.c_int32), ("card_minor", ctypes.c_int32), ("hsa_id", ctypes.c_int32),
        ("hip_id", ctypes.c_int32), ("xgmi_hive_id", ctypes.c_uint64), ("xgmi_node_id", ctypes.c_uint64),
        ("numa_node", ctypes.c_int32), ("kfd_id", ctypes.c_uint64), ("partition_id", ctypes.c_int32),
        ("compute_partition", ctypes.c_char * 32), ("serial", ctypes.c_char * STR),
        ("socket", ctypes.c_int32), ("memory_partition", ctypes.c_char * 16),
    ]


class _Link(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("hops", ctypes.c_uint64), ("weight", ctypes.c_uint64), ("p2p", ctypes.c_int32)]


class _Metrics(ctypes.Structure):
    _fields_ = [
        ("gfx_activity", ctypes.c_uint32), ("umc_activity", ctypes.c_uint32), ("vram_used_bytes", ctypes.c_uint64),
        ("vram_total_bytes", ctypes.c_uint64), ("power_w", ctypes.c_uint32), ("power_limit_w", ctypes.c_uint32),
        ("temp_hotspot_c", ctypes.c_int64), ("temp_mem_c", ctypes.c_int64), ("ecc_correctable", ctypes.c_uint64),
        ("ecc_uncorrectable", ctypes.c_uint64), ("xgmi_links_total", ctypes.c_uint32), ("xgmi_links_up", ctypes.c_uint32),
        ("sclk_mhz", ctypes.c_uint32),
    ]


class _Proc(ctypes.Structure):
    _fields_ = [("pid", ctypes.c_uint32), ("name", ctypes.c_char * STR), ("vram_bytes", ctypes.c_uint64),
                ("gfx_ns", ctypes.c_uint64), ("cu_occupancy", ctypes.c_uint32)]


@dataclass
class GPU:
    index: int
    uuid: str
    bdf: str
    market_name: str
    arch: str
    vendor_id: int
    device_id: int
    vram_total_mb: int
    compute_units: int
    render_minor: int
    card_minor: int
    hsa_id: int
    hip_id: int
    xgmi_hive_id: int
    xgmi_node_id: int
    numa_node: int
    kfd_id: int
    partition_id: int
    compute_partition: str
    serial: str
    socket: int = -1               # physical package: compute partitions of one MI355X share it
    memory_partition: str = ""     # NPS1 / NPS2

    @property
    def product(self) -> str:
        """Marketing product name. AMD SMI may report a generic market name ("AMD Radeon
        Graphics") on some drivers; the PCI device id is authoritative for CDNA4 parts."""
        by_id = {0x75A0: "MI350X", 0x75A3: "MI355X", 0x74A1: "MI300X", 0x74A5: "MI325X"}
        if self.device_id in by_id:
            return by_id[self.device_id]
        if "MI" in self.market_name:
            return self.market_name.split()[-1]
        return {"gfx950": "MI355X", "gfx942": "MI300X"}.get(self.arch, self.market_name or "unknown")

    @property
    def device_id_str(self) -> str:
        """Stable plugin device ID (Device.ID, ≤63 chars): prefer the ASIC UUID. Compute
        partitions of one package may share its UUID, so a partition's ID carries `-p<id>`."""
        suffix = f"-p{self.partition_id}" if self.compute_partition not in ("", "SPX") and self.partition_id >= 0 else ""
        if self.uuid:
            base = self.uuid if self.uuid.startswith("GPU-") else "GPU-" + self.uuid
            return base[:63 - len(suffix)] + suffix
        return f"GPU-{self.bdf or self.index}"


@dataclass
class Metrics:
    gfx_activity: int = 0
    umc_activity: int = 0
    vram_used_bytes: int = 0
    vram_total_bytes: int = 0
    power_w: int = 0
    power_limit_w: int = 0
    temp_hotspot_c: int = 0
    temp_mem_c: int = 0
    ecc_correctable: int = 0
    ecc_uncorrectable: int = 0
    xgmi_links_total: int = 0
    xgmi_links_up: int = 0
    sclk_mhz: int = 0


@dataclass
class Link:
    type: int
    hops: int
    weight: int
    p2p: bool


@dataclass
class Proc:
    pid: int
    name: str
    vram_bytes: int
    gfx_ns: int
    cu_occupancy: int


_lib = None
_lock = threading.Lock()


# logical devices per MI355X package in each compute-partition mode (8 XCDs per package)
PARTITIONS_PER_SOCKET = {"SPX": 1, "DPX": 2, "QPX": 4, "CPX": 8}


class SMIError(RuntimeError):
    pass


def lib_path():
    return os.path.join(LIB_DIR, "libkamd_smi.so")


def _load():
    global _lib
    if _lib is None:
        p = lib_path()
        if not os.path.exists(p):
            raise SMIError(f"{p} not built: run `python -m kubernetes_amd.native.build`")
        L = ctypes.CDLL(p)
        L.kamd_init.argtypes = [ctypes.c_char_p]
        L.kamd_device_info.argtypes = [ctypes.c_int, ctypes.POINTER(_Info)]
        L.kamd_link.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(_Link)]
        L.kamd_metrics.argtypes = [ctypes.c_int, ctypes.POINTER(_Metrics)]
        L.kamd_process_list.argtypes = [ctypes.c_int, ctypes.POINTER(_Proc), ctypes.c_int]
        L.kamd_fake_set_ecc.argtypes = [ctypes.c_int, ctypes.c_uint64]
        L.kamd_fake_set_links_up.argtypes = [ctypes.c_int, ctypes.c_uint32]
        L.kamd_fake_set_link.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.kamd_fake_set_procs.argtypes = [ctypes.c_int, ctypes.POINTER(_Proc), ctypes.c_int]
        L.kamd_last_error.restype = ctypes.c_char_p
        _lib = L
    return _lib


def _s(b):
    return b.decode(errors="replace") if isinstance(b, bytes) else b


class SMI:
    """Process-wide handle. `SMI(fixture=path)` selects the fake backend."""

    def __init__(self, fixture: str | None = None):
        self.L = _load()
        with _lock:
            b = self.L.kamd_init(fixture.encode() if fixture else None)
        if b == 0:
            raise SMIError(_s(self.L.kamd_last_error()))
        self.backend = b
        self.fixture = fixture

    @property
    def is_fake(self):
        return self.backend == BACKEND_FAKE

    def count(self) -> int:
        return self.L.kamd_device_count()

    def gpu(self, i) -> GPU:
        info = _Info()
        if self.L.kamd_device_info(i, ctypes.byref(info)) != 0:
            raise SMIError(_s(self.L.kamd_last_error()))
        return GPU(**{f: _s(getattr(info, f)) for f, _ in _Info._fields_})

    def gpus(self) -> list[GPU]:
        return [self.gpu(i) for i in range(self.count())]

    def link(self, a, b) -> Link:
        lk = _Link()
        self.L.kamd_link(a, b, ctypes.byref(lk))
        return Link(lk.type, lk.hops, lk.weight, bool(lk.p2p))

    def metrics(self, i) -> Metrics:
        mt = _Metrics()
        self.L.kamd_metrics(i, ctypes.byref(mt))
        return Metrics(**{f: getattr(mt, f) for f, _ in _Metrics._fields_})

    def processes(self, i, max_procs=256) -> list[Proc]:
        arr = (_Proc * max_procs)()
        n = self.L.kamd_process_list(i, arr, max_procs)
        return [Proc(arr[k].pid, _s(arr[k].name), arr[k].vram_bytes, arr[k].gfx_ns, arr[k].cu_occupancy) for k in range(n)]

    def fake_set_ecc(self, i, n):
        return self.L.kamd_fake_set_ecc(i, n)

    def fake_set_links_up(self, i, n):
        return self.L.kamd_fake_set_links_up(i, n)

    def fake_set_link(self, a, b, xgmi: bool):
        """Fake backend: bring the xGMI link between devices a and b up or down (both ways)."""
        t = LINK_XGMI if xgmi else LINK_PCIE
        return self.L.kamd_fake_set_link(a, b, t) | self.L.kamd_fake_set_link(b, a, t)

    def fake_set_procs(self, i, procs):
        """Fake backend: the GPU process list of device i, [(pid, name, vram_bytes, gfx_ns)]."""
        arr = (_Proc * max(1, len(procs)))()
        for k, (pid, name, vram, gfx) in enumerate(procs):
            arr[k].pid, arr[k].name, arr[k].vram_bytes, arr[k].gfx_ns = pid, name.encode()[:STR - 1], vram, gfx
        return self.L.kamd_fake_set_procs(i, arr, len(procs))

    def topology(self):
        n = self.count()
        return [[self.link(i, j) for j in range(n)] for i in range(n)]


def mi355x_fixture(n=8, hive_id=0x3C4D5E6F7081, hives=1, partition="SPX", numa_per=4, seed="node0",
                   memory_partition="NPS1", links_down=()) -> dict:
    """Fixture for an n-GPU MI355X UBB node (8 OAMs, all-to-all xGMI: 7 links per GPU).
    `hives` > 1 splits the GPUs into several hives (to exercise hive-aware allocation).

    `partition` is the compute-partition mode: SPX exposes each package as one device, DPX /
    QPX / CPX split its 8 XCDs into 2 / 4 / 8 logical devices, each with its own render node,
    1/k of the CUs and 1/k of the HBM (as AMD SMI reports a partition). Partitions of one
    package share `socket` and its xGMI links. `links_down`: package pairs (a, b) whose direct xGMI
    link is down (the pair is reachable over PCIe only; both report one link fewer)."""
    per = PARTITIONS_PER_SOCKET.get(partition, 1)
    devs = []
    per_hive = max(1, n // hives)
    for i in range(n):
        h = hive_id + (i // per_hive)
        for p in range(per):
            k = i * per + p
            uid = f"{seed}-{i:02d}ff-75a3-00{i}0-9c1e-{0x5f3c0000 + i:08x}"
            devs.append({
                "uuid": uid, "bdf": f"0000:{0x05 + 0x10 * i:02x}:00.{p}", "market_name": "AMD Instinct MI355X",
                "arch": "gfx950", "device_id": 0x75A3, "vram_total_mb": 294912 // per, "compute_units": 256 // per,
                "render_minor": 128 + k, "card_minor": k, "hsa_id": k, "hip_id": k, "xgmi_hive_id": h,
                "xgmi_node_id": i, "numa_node": i // numa_per, "partition": partition, "partition_id": p,
                "socket": i, "memory_partition": memory_partition, "serial": f"{seed}-SN{i:04d}",
                "xgmi_links_total": 7,
                "xgmi_links_up": (7 if per_hive == 8 else per_hive - 1) - sum(1 for a, b in links_down if i in (a, b)),
            })
    links = []
    for a, b in links_down:
        for pa in range(per):
            for pb in range(per):
                links += [[a * per + pa, b * per + pb, LINK_PCIE, 2, 40], [b * per + pb, a * per + pa, LINK_PCIE, 2, 40]]
    return {"devices": devs, "links": links}


_FIXTURE_CACHE = {}


def fixture_file(n=8, **kw) -> str:
    key = (n, tuple(sorted((k, tuple(map(tuple, v)) if k == "links_down" else v) for k, v in kw.items())))
    p = _FIXTURE_CACHE.get(key)
    if p and os.path.exists(p):
        return p
    fd, p = tempfile.mkstemp(prefix=f"kamd-fixture-{n}-", suffix=".json")
    with os.fdopen(fd, "w") as f:
        json.dump(mi355x_fixture(n, **kw), f)
    _FIXTURE_CACHE[key] = p
    return p
