"""kubelet equivalent: node registration/status, admission, per-pod workers, runtime sync,
status reporting, graceful deletion, and the device-manager wiring of the fork (F10).

Parity map:
  * `pkg/kubelet/kubelet.go` — NewMainKubelet admit handlers (:898), syncLoop (:1772),
    HandlePodAdditions (:1990), syncPod (:1441), dispatchWork (:1950);
  * `pkg/kubelet/pod_workers.go:153-195` — one serialized worker per pod UID;
  * `pkg/kubelet/lifecycle/predicate.go:32-80` — device manager AdmitPod runs BEFORE
    GeneralPredicates; rejection marks the pod Failed;
  * `pkg/kubelet/kubelet_node_status.go:552-553,608-623` — `Capacity[r]` and
    `Status.ExtendedResources[r]` from the device manager. Fix (quirk Q6): capacity counts
    only Healthy devices; the full device map (with health) goes to `extendedResources`;
  * `pkg/kubelet/kubelet_pods.go:453-471` — sandbox annotations from the plugin's AdmitPod
    response, container run options from InitContainer;
  * `pkg/kubelet/status/status_manager.go` — status writes; final delete once containers died.

Event-driven instead of the reference's fixed periods: pod changes are
pushed by the watch into the pod's worker immediately (no 1 s sync tick), container exits come
from the runtime (no 1 s PLEG relist wait), and a device-capacity change triggers a node status
write within `status_debounce` (no 10 s wait) — periodic heartbeat and resync remain.
"""
from __future__ import annotations

import asyncio
import itertools
import logging
import os
import tempfile
import time

from ..api import core
from ..api.meta import now_rfc3339, parse_rfc3339
from ..api.quantity import parse_quantity
from ..client.events import EventRecorder
from ..client.informer import Informer
from ..client.rest import APIStatusError, is_conflict, is_not_found
from ..utils.httpserver import HTTPServer, Response, StreamResponse
from ..utils.metrics import MICRO_BUCKETS, Registry
from .devicemanager.manager import AdmitError, ManagerStub
from .podstatus import generate_pod_initialized_condition, generate_pod_ready_condition, normalize_status
from .lifecycle import HandlerRunner
from .prober import ProbeManager
from .runtimestate import NETWORK_READY, RUNTIME_READY, RuntimeState, ready_condition, update_runtime_up
from .runtime.base import CREATED, EXITED, RUNNING, UNKNOWN, RunContainerOptions
from .qos import oom_score_adj
from .volumes import VolumeError, VolumeManager, make_absolute_path
from ..utils.tasks import spawn

log = logging.getLogger("kubelet")
CONTROLLER_MANAGED_ATTACH = "volumes.kubernetes.io/controller-managed-attach-detach"
# setNode*Condition -> recordNodeStatusEvent reasons
_NODE_STATUS_EVENTS = {("Ready", "True"): "NodeReady", ("Ready", "False"): "NodeNotReady",
                       ("MemoryPressure", "True"): "NodeHasInsufficientMemory",
                       ("MemoryPressure", "False"): "NodeHasSufficientMemory",
                       ("DiskPressure", "True"): "NodeHasDiskPressure", ("DiskPressure", "False"): "NodeHasNoDiskPressure",
                       ("OutOfDisk", "True"): "NodeOutOfDisk", ("OutOfDisk", "False"): "NodeHasSufficientDisk"}

_ip_counter = itertools.count(2)


BOOTSTRAP_CHECKPOINT = "node.kubernetes.io/bootstrap-checkpoint"
MIN_KILL_GRACE_SECONDS = 2.0        # kuberuntime minimumGracePeriodInSeconds




def expand(s, *contexts):
    """`third_party/forked/golang/expansion` Expand: a single left-to-right scan — `$$` is an
    escaped `$`, `$(NAME)` (NAME = everything up to the next `)`) is replaced from the first
    context that defines it and kept verbatim otherwise, an unclosed `$(` and any other `$x` are
    literal; values are not re-expanded."""
    s = str(s)
    out, i, n = [], 0, len(s)
    while i < n:
        ch = s[i]
        if ch != "$" or i + 1 >= n:
            out.append(ch)
            i += 1
            continue
        nxt = s[i + 1]
        if nxt == "$":
            out.append("$")
            i += 2
        elif nxt == "(":
            close = s.find(")", i + 2)
            if close < 0:
                out.append("$(")
                i += 2
            else:
                name = s[i + 2:close]
                for ctx in contexts:
                    if name in ctx:
                        out.append(ctx[name])
                        break
                else:
                    out.append(f"$({name})")
                i = close + 1
        else:
            out.append("$" + nxt)
            i += 2
    return "".join(out)


class PodState:
    __slots__ = ("uid", "pod", "sandbox", "containers", "init_containers", "admitted", "rejected", "start_time",
                 "restarts", "ip", "terminated", "deleted", "last_status", "running_at", "first_seen", "volumes",
                 "waiting", "net_mounts", "net_setup", "previous", "backoff", "adopted", "deadline_armed",
                 "final_deleted", "requests")

    def __init__(self, pod):
        self.uid = pod["metadata"]["uid"]
        self.pod = pod
        self.sandbox = None
        self.containers: dict[str, str] = {}       # name -> cid (current)
        self.init_containers: dict[str, str] = {}
        self.admitted = False
        self.rejected = None
        self.start_time = None
        self.restarts: dict[str, int] = {}
        n = next(_ip_counter)
        self.ip = f"10.{(n >> 16) & 255}.{(n >> 8) & 255}.{n & 255}"
        self.terminated = False
        self.deleted = False
        self.last_status = None
        self.running_at = None
        self.first_seen = time.time()
        self.volumes = None            # {volume name: host path} once mounted
        self.waiting: dict[str, tuple] = {}   # container -> (reason, message) while it cannot start
        self.net_mounts = []                  # /etc/hosts + /etc/resolv.conf bind mounts
        self.net_setup = False                # network plugin SetUpPod done for the sandbox
        self.previous: dict[str, str] = {}    # container name -> last dead instance (logs --previous)
        self.backoff: dict[str, list] = {}    # container name -> [next restart allowed at, current delay]
        self.adopted = False                  # sandbox/containers found in the runtime after a kubelet restart
        self.deadline_armed = False           # a resync is scheduled at spec.activeDeadlineSeconds
        self.final_deleted = False            # the grace-0 delete was accepted; later events need no other
        self.requests = None                  # core.pod_requests, once: container resources are immutable


def _field_path(pod, c):
    """`ref.GetPartialReference` fieldPath of a container (`spec.containers{name}`)."""
    spec = pod.get("spec") or {}
    if any(ic.get("name") == c["name"] for ic in spec.get("initContainers") or ()):
        return f"spec.initContainers{{{c['name']}}}"
    return f"spec.containers{{{c['name']}}}"


def now_rfc3339_nano(t=None):
    t = time.time() if t is None else t
    return time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(t)) + f".{int((t % 1) * 1e9):09d}Z"


class Kubelet:
    def __init__(self, client, node_name, runtime, device_manager=None, cpu="128", memory="2Ti", pods=110,
                 labels=None, node_status_update_frequency=10.0, status_debounce=0.02, http_port=None,
                 emit_events=True, register=True, metrics=None, address="127.0.0.1", max_status_inflight=64,
                 root_dir=None, cpu_manager_policy="none", cpu_topology=None, reserved_cpus=1,
                 pod_manifest_path=None, eviction_hard=None, eviction_signals=None, eviction_interval=10.0,
                 image_service=None, image_gc=None, image_backoff=10.0, network_plugin=None, dns=None,
                 hostports=None, container_gc=None, crash_backoff=(10.0, 300.0), dynamic_config_dir=None,
                 bootstrap_checkpoint_path=None, volume_plugin_dir="/usr/libexec/kubernetes/kubelet-plugins/volume/exec",
                 manifest_url=None, manifest_url_headers=None, kube_reserved=None, system_reserved=None,
                 cgroup_root=None, allowed_unsafe_sysctls=(), service_env=True, master_service_namespace="default", container_log_dir=None,
                 event_qps=5.0, event_burst=10, auth=None, node_log_dir="/var/log", tls=None, read_only_port=None,
                 healthz_port=None, healthz_address="127.0.0.1", debugging_handlers=True, node_ip=None,
                 register_taints=(), register_schedulable=True, provider_id="", allow_privileged=True,
                 host_sources=None, eviction_soft=None, eviction_soft_grace_period=None, eviction_minimum_reclaim=None,
                 eviction_max_pod_grace_period=0, eviction_pressure_transition_period=0.0,
                 allocatable_ignore_eviction=False, serialize_image_pulls=False, registry_qps=0.0, registry_burst=10,
                 file_check_frequency=20.0, http_check_frequency=20.0, sync_frequency=60.0, cpu_cfs_quota=True,
                 enforce_node_allocatable=True):
        self.file_check_frequency, self.http_check_frequency = file_check_frequency, http_check_frequency
        # --sync-frequency: how often running pods' configMap / secret / downwardAPI / projected
        # volumes are re-projected (`kubelet.go` syncLoop's periodic sync, 1m)
        self.sync_frequency = sync_frequency
        self.cpu_cfs_quota = cpu_cfs_quota      # --cpu-cfs-quota=false: CPU limits set no cpu.max
        self.enforce_node_allocatable = enforce_node_allocatable   # --enforce-node-allocatable=none: False
        self.client = client
        # :10250 serving (cmd/kubelet/app/server.go): TLS = (cert file, key file, client CA file or
        # None) or None for plain HTTP; --read-only-port (unauthenticated, no debugging handlers)
        # and --healthz-port listeners; --enable-debugging-handlers=false drops exec/attach/
        # port-forward/run/logs/containerLogs/pprof/configz from the server
        self.tls = tls
        self.read_only_port, self.healthz_port, self.healthz_address = read_only_port, healthz_port, healthz_address
        self.debugging_handlers = debugging_handlers
        self.ro_http = self.healthz_http = None
        # registration: --node-ip, --register-with-taints, --register-schedulable, --provider-id
        self.node_ip = node_ip
        self.register_taints = [dict(t) for t in register_taints or ()]
        self.register_schedulable = register_schedulable
        self.provider_id = provider_id
        # --allow-privileged and --host-{network,pid,ipc}-sources (pkg/kubelet/util/capabilities):
        # which pod sources ("api", "file", "http"; "*" = all) may use host namespaces
        self.allow_privileged = allow_privileged
        self.host_sources = host_sources or {}
        self.auth = auth                      # server_auth.KubeletAuth for the :10250 API (None: open)
        self.node_log_dir = node_log_dir      # served read-only under /logs/
        self._last_status_loop = time.monotonic()
        # /var/log/containers/<pod>_<ns>_<container>-<id>.log symlinks to the runtime's log
        # files (kuberuntime legacyLogSymlink): what node logging agents tail
        self.container_log_dir = container_log_dir
        self._log_links: dict[str, str] = {}      # container id -> symlink path
        from .preemption import CriticalPodAdmissionHandler
        from .sysctl import SysctlAdmitHandler
        self.sysctls = SysctlAdmitHandler(allowed_unsafe_sysctls)
        self.cgroup_root = cgroup_root            # --cgroup-root with --cgroups-per-qos (None: off)
        self.cgroups = None
        self.service_env = service_env            # inject {SVC}_SERVICE_HOST/... (pkg/kubelet/envvars)
        self.svc_informer = None
        self._svc_env_cache: dict = {}        # namespace -> ((ns, services generation), env vars)
        from .network import NetworkPlugin
        self.network = network_plugin or NetworkPlugin()
        self.dns = dns                       # network.DNSConfigurer or None
        self.master_service_namespace = master_service_namespace   # --master-service-namespace
        self.hostports = hostports           # network.HostportManager or None
        self.container_gc = container_gc     # ContainerGC policy dict or None
        self.crash_backoff = crash_backoff   # (initial, max) restart back-off, kubelet.go backOffPeriod/MaxContainerBackOff
        self.pod_cidr = None
        self.pod_checkpoints = None
        if bootstrap_checkpoint_path:
            from ..utils.checkpoint import CheckpointManager
            self.pod_checkpoints = CheckpointManager(bootstrap_checkpoint_path)
        self.dynamic = None
        if dynamic_config_dir:
            from .kubeletconfig import DynamicConfig
            self.dynamic = DynamicConfig(self, dynamic_config_dir)
        self.pod_manifest_path = pod_manifest_path
        self.manifest_url, self.manifest_url_headers = manifest_url, manifest_url_headers
        self.reserved = [dict(kube_reserved or {}), dict(system_reserved or {})]
        self.static_pods = None
        self.eviction = None
        self.eviction_interval = eviction_interval
        self.allocatable_ignore_eviction = allocatable_ignore_eviction
        if eviction_hard or eviction_soft:
            from .eviction import EvictionManager, parse_threshold_config
            th = parse_threshold_config(("pods",) if enforce_node_allocatable else (), eviction_hard or "",
                                        eviction_soft or "", eviction_soft_grace_period or "",
                                        eviction_minimum_reclaim or "")
            self.eviction = EvictionManager(th, eviction_signals, pressure_transition_period=eviction_pressure_transition_period,
                                            max_pod_grace=eviction_max_pod_grace_period)
        self.cpu_manager = None
        if cpu_manager_policy == "static":
            from .cpumanager import CPUTopology, StaticPolicy
            self.cpu_manager = StaticPolicy(cpu_topology or CPUTopology.discover(), reserved_cpus,
                                            os.path.join(root_dir or tempfile.gettempdir(), f"cpu_manager_state.{node_name}"))
        self.root_dir = root_dir or os.path.join(tempfile.gettempdir(), f"kamd-kubelet-{node_name}")
        self.volumes = VolumeManager(client, os.path.join(self.root_dir, "pods"), os.path.join(self.root_dir, "plugins"),
                                     node_name, flex_plugins_dir=volume_plugin_dir)
        self.probes = ProbeManager(runtime, self._on_readiness, self._on_liveness_failure,
                                   on_probe_failure=self._on_probe_failure)
        self.node_name = node_name
        self.runtime = runtime
        self.dm = device_manager or ManagerStub()
        self.capacity = {"cpu": str(cpu), "memory": str(memory), "pods": str(pods)}
        self.labels = dict(labels or {})
        self.status_freq = node_status_update_frequency
        self.status_debounce = status_debounce
        self.http_port = http_port
        self.register = register
        self.address = address
        self.pods: dict[str, PodState] = {}
        self.by_key: dict[str, str] = {}
        self._workers: dict[str, asyncio.Task] = {}
        self._pending: dict[str, tuple] = {}
        self._tasks = []
        self._adoptable: dict = {}
        self.orphan_grace = 10.0   # s after the first sync before unknown runtime pods are removed
        self.adopted_pods = 0
        self._status_dirty = asyncio.Event()
        self.volumes.on_in_use_change = self._status_dirty.set
        self._status_sem = asyncio.Semaphore(max_status_inflight)
        self._status_inflight: dict[str, asyncio.Task] = {}
        self._status_next: dict[str, tuple] = {}
        # event writes are rate limited like the reference kubelet's event client
        # (--event-qps 5 / --event-burst 10; 0 = unlimited)
        self.recorder = EventRecorder(client, "kubelet", node_name, workers=2, enabled=emit_events,
                                      qps=event_qps, burst=event_burst)
        self.metrics = metrics or Registry()
        m = self.metrics
        self.m_start = m.histogram("kubelet_pod_start_latency_microseconds",
                                   "Latency in microseconds for a single pod to go from pending to running",
                                   (), MICRO_BUCKETS)
        self.m_worker = m.histogram("kubelet_pod_worker_latency_microseconds", "Pod worker sync latency",
                                    ("operation_type",), MICRO_BUCKETS)
        self.m_runtime_ops = m.counter("kubelet_runtime_operations", "Runtime operations", ("operation_type",))
        self.m_running = m.gauge("kubelet_running_pod_count", "Running pods", ())
        self.informer = Informer(client, "pods", field_selector=f"spec.nodeName={node_name}")
        self.http = None
        self.node_uid = None
        self.runtime.on_exit(self._on_container_exit)
        # image manager (pkg/kubelet/images): the CRI image service of a remote runtime, or an
        # in-process image store for the in-process runtimes
        if image_service is None:
            image_service = getattr(runtime, "images", None)
        if image_service is None:
            from ..cri.server import ImageStore, LocalImageService, host_image_resolver, stub_image_resolver
            image_service = LocalImageService(ImageStore(stub_image_resolver if runtime.name == "stub" else host_image_resolver))
        from .images import ImageGCManager, ImageManager
        self.image_service = image_service
        self._node_images: list = []
        self._cond_transitions: dict = {}      # condition type -> (status, lastTransitionTime)
        self.runtime_state = RuntimeState()     # runtime.go: NodeReady's runtime/network errors
        self.images = ImageManager(image_service, self.recorder, backoff_initial=image_backoff,
                                   secret_getter=lambda ns, name: self.client.get("secrets", name, ns),
                                   serialize=serialize_image_pulls, qps=registry_qps, burst=registry_burst)
        self.image_gc = None
        if image_gc:
            self.image_gc = ImageGCManager(image_service, int(image_gc.get("capacity_bytes", 0)), self._images_in_use,
                                           image_gc.get("high", 85), image_gc.get("low", 80), image_gc.get("min_age", 120.0),
                                           last_used=self.images.last_used)
            self.image_gc_period = float(image_gc.get("period", 300.0))
        self.preemption = CriticalPodAdmissionHandler(self.active_pods, self._preempt, self.recorder)
        self.started = asyncio.Event()
        self.plugin_labels = {}
        self.informer_node_labels = {}
        self._stopped = False
        self.smi = None   # set by the node agent when the real/fake AMD SMI is available (stats)
        self.isolation = None   # runtime.isolation_status(): node condition IsolationUnavailable

    # ------------------------------------------------------------------
    # lifecycle
    async def run(self):
        """Start everything; returns once the node is registered and pods are syncing."""
        self.recorder.start()
        if self.http_port is not None:
            ctx = None
            if self.tls:
                from ..utils.tlsutil import server_context
                ctx = server_context(*self.tls)
            self.http = HTTPServer(self._http)
            self.http_port = await self.http.start(self.address, self.http_port, ssl=ctx)
        if self.read_only_port is not None:
            self.ro_http = HTTPServer(self._http_readonly)
            self.read_only_port = await self.ro_http.start(self.address, self.read_only_port)
        if self.healthz_port is not None:
            self.healthz_http = HTTPServer(self._http_healthz)
            self.healthz_port = await self.healthz_http.start(self.healthz_address, self.healthz_port)
        await self.dm.start(self.active_pods)
        self.dm.add_capacity_listener(lambda r: self._status_dirty.set())
        if self.cgroup_root:
            from .cgroups import CgroupManager
            alloc = self._allocatable(self.capacity)
            self.cgroups = CgroupManager(self.cgroup_root, {
                "cpu": parse_quantity(str(alloc["cpu"])).milli_value(),
                "memory": parse_quantity(str(alloc["memory"])).value} if self.enforce_node_allocatable else {},
                cpu_cfs_quota=self.cpu_cfs_quota).start()
        if self.service_env:
            self.svc_informer = Informer(self.client, "services")
            self.svc_informer.start()
        self._wire_dns()
        if self.volumes.recorder is None:
            self.volumes.recorder = lambda obj, typ, reason, msg: self.recorder.event(obj, typ, reason, msg)
        await self.update_runtime_up()
        if self.register:
            await self._register_node()
        if self.pod_checkpoints is not None:
            restored = self._restore_checkpointed_pods()
            if restored:
                log.info("started %d pods from bootstrap checkpoints", restored)
        if hasattr(self.runtime, "start"):
            await self.runtime.start()
        self.isolation = self.runtime.isolation_status()
        if self.isolation is not None and not self.isolation["enforced"]:
            log.warning("%s: %s", self.isolation["reason"], self.isolation["message"])
            self._status_dirty.set()
        try:
            # kubelet restart: what the runtime still runs is adopted, not started again
            self._adoptable = await self.runtime.pod_states()
        except Exception as e:  # noqa: BLE001 - a runtime that cannot list starts from scratch
            log.warning("listing runtime pods for adoption failed: %s", e)
            self._adoptable = {}
        self.informer.add_handler(self._on_add, self._on_update, self._on_delete)
        self.informer.start()
        self._tasks.append(asyncio.ensure_future(self._node_status_loop()))
        self._tasks.append(asyncio.ensure_future(self._runtime_up_loop()))
        if self.sync_frequency and self.sync_frequency > 0:
            self._tasks.append(asyncio.ensure_future(self._volume_sync_loop()))
        await self.informer.wait_synced(60)
        if self._adoptable:
            self._tasks.append(asyncio.ensure_future(self._remove_orphans(self.orphan_grace)))
        if self.pod_manifest_path or self.manifest_url:
            from .config import StaticPodSource
            period = min([f for f, on in ((self.file_check_frequency, self.pod_manifest_path),
                                          (self.http_check_frequency, self.manifest_url)) if on])
            self.static_pods = StaticPodSource(self, self.pod_manifest_path, period=period, url=self.manifest_url,
                                               url_headers=self.manifest_url_headers)
            self.static_pods.start()
        if self.eviction is not None:
            self._tasks.append(asyncio.ensure_future(self._eviction_loop()))
        if self.image_gc is not None:
            self._tasks.append(asyncio.ensure_future(self._image_gc_loop()))
        if self.container_gc is not None:
            self._tasks.append(asyncio.ensure_future(self._container_gc_loop()))
        self.started.set()

    def _images_in_use(self):
        return {c.get("image", "") for s in self.pods.values() if not s.deleted
                for c in list((s.pod.get("spec") or {}).get("containers") or ()) +
                list((s.pod.get("spec") or {}).get("initContainers") or ())}

    async def _image_gc_loop(self):
        """image_gc_manager.go: `Start` detects images right away (stamped with the zero time, so
        images present before a kubelet restart are reclaimable at once) and then every period;
        `kubelet.StartGarbageCollection` runs GarbageCollect every ImageGCPeriod (5 min)."""
        if self.image_gc.recorder is None:
            node_ref = {"kind": "Node", "metadata": {"name": self.node_name, "uid": self.node_name}}
            self.image_gc.recorder = lambda typ, reason, msg: self.recorder.event(node_ref, typ, reason, msg)
        try:
            await self.image_gc.detect()
        except Exception as e:
            log.warning("image detection failed: %s", e)
        while not self._stopped:
            await asyncio.sleep(self.image_gc_period)
            try:
                freed = await self.image_gc.garbage_collect()
                if freed:
                    log.info("image GC freed %d bytes", freed)
            except Exception as e:
                log.warning("image garbage collection failed: %s", e)

    def _wire_eviction_reclaim(self):
        """`buildResourceToNodeReclaimFuncs` (no dedicated image fs): the disk resources are
        reclaimed by deleting terminated containers, then unused images (bytes freed counted for
        the space signals only); node events go to the node."""
        ev = self.eviction
        if getattr(ev, "_kubelet_stats", False) is False and ev.usage_fn is None:
            from .stats import pod_eviction_stats
            ev.stats_fn = lambda pod: pod_eviction_stats(self, pod)
            ev._kubelet_stats = True
        if ev.recorder is None:
            node_ref = {"kind": "Node", "metadata": {"name": self.node_name, "uid": self.node_name}}
            ev.recorder = lambda obj, typ, reason, msg: self.recorder.event(obj or node_ref, typ, reason, msg)
        if ev.reclaim_fns:
            return
        fns_space, fns_inodes = [], []

        async def containers():
            # `DeleteAllUnusedContainers`: the GC policy, plus every dead container of terminated pods
            await self.garbage_collect_containers(evict_terminated=True)
            return 0
        fns_space.append(containers)
        fns_inodes.append(containers)
        if getattr(self, "image_gc", None) is not None:
            async def images(report=True):
                freed = await self.image_gc.delete_unused_images()
                return freed if report else 0
            fns_space.append(images)
            fns_inodes.append(lambda: images(False))
        ev.reclaim_fns = {"nodefs": fns_space, "imagefs": fns_space, "nodefsInodes": fns_inodes,
                          "imagefsInodes": fns_inodes}

    async def _eviction_loop(self):
        """eviction_manager.go synchronize(): observe, set pressure conditions, evict <= 1 pod."""
        last_conds = set()
        while not self._stopped:
            running = [s.pod for s in self.pods.values() if s.admitted and not s.terminated and not s.rejected]
            self._wire_eviction_reclaim()
            victim, msg, grace, event_msg = await self.eviction.synchronize(running)
            conds = set(self.eviction.conditions)
            if conds != last_conds:
                last_conds = conds
                self._status_dirty.set()
            if victim is not None:
                st = self.pods.get(victim["metadata"]["uid"])
                if st is not None:
                    self.recorder.event(victim, "Warning", "Evicted", event_msg or msg)
                    await self._kill_pod(st, grace)
                    await self._write_status(st, {"phase": core.POD_FAILED, "reason": "Evicted", "message": msg,
                                                  "conditions": (victim.get("status") or {}).get("conditions") or []})
            await asyncio.sleep(self.eviction_interval)

    async def stop(self):
        self._stopped = True
        self._status_dirty.set()
        self.informer.stop()
        if self.svc_informer is not None:
            self.svc_informer.stop()
        if self.static_pods is not None:
            self.static_pods.stop()
        for t in self._tasks:
            t.cancel()
        for t in list(self._workers.values()):
            t.cancel()
        self.probes.stop()
        if self.hostports is not None:
            self.hostports.close()
        await self.dm.stop()
        self.recorder.stop()
        for srv in (self.http, self.ro_http, self.healthz_http):
            if srv:
                await srv.stop()

    def active_pods(self):
        return [s.pod for s in self.pods.values() if not s.terminated and not s.rejected]

    # ------------------------------------------------------------------
    # node registration & status
    def _node_object(self):
        labels = {"kubernetes.io/hostname": self.node_name, "beta.kubernetes.io/os": "linux",
                  "beta.kubernetes.io/arch": "amd64"}
        labels.update(self.plugin_labels)
        labels.update(self.labels)
        spec = {}
        if self.register_taints:
            spec["taints"] = [dict(t) for t in self.register_taints]
        if not self.register_schedulable:
            spec["unschedulable"] = True
        if self.provider_id:
            spec["providerID"] = self.provider_id
        # --enable-controller-attach-detach (always on here): the attach/detach controller, not
        # this kubelet, attaches the node's volumes (`kubelet_node_status.go` initialNode)
        node = {"apiVersion": "v1", "kind": "Node",
                "metadata": {"name": self.node_name, "labels": labels,
                             "annotations": {CONTROLLER_MANAGED_ATTACH: "true"}},
                "spec": spec, "status": self._node_status()}
        return node

    def _node_status(self):
        cap, _removed = self.dm.get_capacity()
        capacity = dict(self.capacity)
        ers = {}
        for rname, dom in cap.items():
            healthy = sum(1 for d in dom["resources"].values() if d.get("health") == core.HEALTHY)
            capacity[rname] = str(healthy)
            ers[rname] = dom
        # plugin labels (e.g. amd.com/gpu.product=MI355X) become node labels
        now = now_rfc3339()
        mem_p = self.eviction is not None and self.eviction.has("MemoryPressure")
        disk_p = self.eviction is not None and self.eviction.has("DiskPressure")
        cond = self._condition
        ready = cond("Ready", *ready_condition(self._ready_errors()), now)
        alloc = self._allocatable(capacity)
        self.volumes.allocatable = alloc        # downward API: a missing limit reads as allocatable
        self.volumes.host_ip = self.node_ip or self.address
        st = {"capacity": capacity, "allocatable": alloc,
              "conditions": [
                  cond("OutOfDisk", "False", "KubeletHasSufficientDisk", "kubelet has sufficient disk space available", now),
                  cond("MemoryPressure", "True", "KubeletHasInsufficientMemory", "kubelet has insufficient memory available", now)
                  if mem_p else
                  cond("MemoryPressure", "False", "KubeletHasSufficientMemory", "kubelet has sufficient memory available", now),
                  cond("DiskPressure", "True", "KubeletHasDiskPressure", "kubelet has disk pressure", now) if disk_p else
                  cond("DiskPressure", "False", "KubeletHasNoDiskPressure", "kubelet has no disk pressure", now),
                  ready],
              "addresses": [{"type": "InternalIP", "address": self.node_ip or self.address},
                            {"type": "Hostname", "address": self.node_name}],
              "daemonEndpoints": {"kubeletEndpoint": {"Port": self.http_port or 0}},
              "nodeInfo": dict(self._host_info(), kubeletVersion="v1.9.0-amd.0", kubeProxyVersion="v1.9.0-amd.0",
                               containerRuntimeVersion=f"{self.runtime.name}://1.0", operatingSystem="linux",
                               architecture="amd64")}
        if self._node_images:
            st["images"] = self._node_images
        if self.dynamic is not None:
            st["conditions"].append(dict(self.dynamic.condition, lastHeartbeatTime=now, lastTransitionTime=now))
        iso = getattr(self, "isolation", None)
        if iso is not None:
            # a node whose runtime cannot give pods a private /dev says so instead of letting GPU
            # pods silently share every render node of the host
            st["conditions"].append({"type": "IsolationUnavailable", "status": "False" if iso["enforced"] else "True",
                                     "reason": iso["reason"], "message": iso["message"],
                                     "lastHeartbeatTime": now, "lastTransitionTime": now})
        if ers:
            st["extendedResources"] = ers
        # volumes this node has mounted (or is about to): the attach/detach controller does not
        # detach them (`kubelet_node_status.go` setNodeVolumesInUseStatus)
        st["volumesInUse"] = self.volumes.volumes_in_use() or None
        return st

    def _condition(self, ctype, status, reason, message, now):
        """A node condition whose lastTransitionTime moves only when its status changes
        (`kubelet_node_status.go` setNodeReadyCondition / setNodeMemoryPressureCondition / ...);
        lastHeartbeatTime is every update."""
        prev = self._cond_transitions.get(ctype)
        transition = prev[1] if prev is not None and prev[0] == status else now
        self._cond_transitions[ctype] = (status, transition)
        if prev is None or prev[0] != status:
            ev = _NODE_STATUS_EVENTS.get((ctype, status))
            # recordNodeStatusEvent: "Node <name> status is now: <event>" (Ready only on a change)
            if ev and (ctype != "Ready" or prev is not None):
                node_ref = {"kind": "Node", "metadata": {"name": self.node_name, "uid": self.node_name}}
                self.recorder.event(node_ref, "Normal", ev, f"Node {self.node_name} status is now: {ev}")
        return {"type": ctype, "status": status, "reason": reason, "message": message,
                "lastHeartbeatTime": now, "lastTransitionTime": transition}

    _HOST_INFO = None

    @classmethod
    def _host_info(cls):
        """`setNodeStatusMachineInfo` / `setNodeStatusVersionInfo`: machine, boot and OS
        identity of the host (read once)."""
        if cls._HOST_INFO is None:
            def read(path):
                try:
                    with open(path) as f:
                        return f.read().strip()
                except OSError:
                    return ""
            os_image = ""
            for line in read("/etc/os-release").splitlines():
                if line.startswith("PRETTY_NAME="):
                    os_image = line.split("=", 1)[1].strip().strip('"')
            cls._HOST_INFO = {"machineID": read("/etc/machine-id"), "systemUUID": read("/sys/class/dmi/id/product_uuid"),
                              "bootID": read("/proc/sys/kernel/random/boot_id"), "kernelVersion": os.uname().release,
                              "osImage": os_image}
        return dict(cls._HOST_INFO)

    async def _refresh_node_images(self):
        """`setNodeStatusImages`: the node's images, largest first, at most 50
        (`maxImagesInNodeStatus`), each with its tags and digests."""
        lister = getattr(self.image_service, "list_images", None)
        if lister is None:
            return
        try:
            imgs = await lister()
        except Exception as e:      # noqa: BLE001 - the reference logs and keeps the old list
            log.debug("listing images for node status failed: %s", e)
            return
        out = []
        for i in sorted(imgs or (), key=lambda i: -int(i.get("size", 0) or 0))[:50]:
            names = list(i.get("repoTags") or ()) + list(i.get("repoDigests") or ())
            if names:
                out.append({"names": names, "sizeBytes": int(i.get("size", 0) or 0)})
        self._node_images = out

    def _allocatable(self, capacity):
        """`pkg/kubelet/cm/node_container_manager.go` GetNodeAllocatableReservation:
        allocatable = capacity − kube-reserved − system-reserved − hard eviction threshold
        (memory.available), floored at zero."""
        if not any(self.reserved) and (self.eviction is None or self.allocatable_ignore_eviction):
            return dict(capacity)
        out = dict(capacity)
        for res in ("cpu", "memory", "ephemeral-storage"):
            if res not in capacity:
                continue
            total = parse_quantity(str(capacity[res]))
            cut = sum(parse_quantity(str(r[res])).milli_value() for r in self.reserved if res in r)
            if res == "memory" and self.eviction is not None and not self.allocatable_ignore_eviction:
                cut += self.eviction.hard_memory_bytes() * 1000
            left = max(0, total.milli_value() - cut)
            out[res] = f"{left}m" if res == "cpu" else str(left // 1000)
        return out

    def _collect_plugin_labels(self):
        labels = {}
        h = getattr(self.dm, "handler", None)
        if h is not None:
            for e in h.endpoints.values():
                labels.update(e.labels)
        self.plugin_labels = labels

    async def _register_node(self):
        self._collect_plugin_labels()
        node = self._node_object()
        for attempt in range(50):
            try:
                got = await self.client.create("nodes", node)
                self._published_ers = set(node["status"].get("extendedResources") or ())
                self.node_uid = got["metadata"]["uid"]
                self._observe_pod_cidr(got)
                return
            except APIStatusError as e:
                if e.code == 409:
                    # tryRegisterWithAPIServer: the node was registered before; reconcile the
                    # default labels and the controller-managed attach-detach annotation (plus
                    # the device plugins' labels, which describe this node's hardware)
                    cur = await self.client.get("nodes", self.node_name)
                    md = cur["metadata"]
                    md["labels"] = dict(md.get("labels") or {})
                    md["annotations"] = dict(md.get("annotations") or {})
                    changed = reconcile_cmad_annotation(node, cur)
                    changed = update_default_labels(node, cur) or changed
                    for k, v in self.plugin_labels.items():
                        if md["labels"].get(k) != v:
                            md["labels"][k] = v
                            changed = True
                    if changed:
                        cur = await self.client.update("nodes", cur)
                    cur["status"] = node["status"]
                    await self.client.update_status("nodes", cur)
                    self.node_uid = cur["metadata"]["uid"]
                    return
                raise
            except (ConnectionError, OSError):
                await asyncio.sleep(0.2)

    def apply_config(self, cfg):
        """Hot-apply a (dynamic) KubeletConfiguration; None restores the local configuration."""
        if not hasattr(self, "_local_config"):
            self._local_config = {"pods": self.capacity["pods"], "status_freq": self.status_freq, "eviction": self.eviction,
                                  "container_gc": self.container_gc, "dns": self.dns,
                                  "image_gc": (self.image_gc.high, self.image_gc.low) if self.image_gc else None}
        if cfg is None:
            lc = self._local_config
            self.capacity["pods"], self.status_freq = lc["pods"], lc["status_freq"]
            self.eviction, self.container_gc, self.dns = lc["eviction"], lc["container_gc"], lc["dns"]
            self._wire_dns()
            if self.image_gc is not None and lc["image_gc"]:
                self.image_gc.high, self.image_gc.low = lc["image_gc"]
            self._status_dirty.set()
            return
        from .kubeletconfig import eviction_string, to_kwargs
        kw = to_kwargs(cfg)
        self.capacity["pods"] = str(kw["pods"])
        self.status_freq = kw["node_status_update_frequency"]
        self.container_gc = kw["container_gc"]
        if "dns" in kw:
            self.dns = kw["dns"]
            self._wire_dns()
        if self.image_gc is not None:
            self.image_gc.high = int(cfg["imageGCHighThresholdPercent"])
            self.image_gc.low = int(cfg["imageGCLowThresholdPercent"])
        ev = eviction_string(cfg.get("evictionHard"))
        if ev:
            from .eviction import EvictionManager, parse_thresholds
            self.eviction = EvictionManager(parse_thresholds(ev), getattr(self.eviction, "signals_fn", None))
        self._status_dirty.set()

    def _observe_pod_cidr(self, node):
        """`updatePodCIDR`: hand the node's spec.podCIDR to the network plugin once it appears."""
        if self.dynamic is not None:
            spawn(self.dynamic.observe_node(node))
        cidr = ((node or {}).get("spec") or {}).get("podCIDR")
        if cidr and cidr != self.pod_cidr:
            self.pod_cidr = cidr
            self.network.set_pod_cidr(cidr)
            self._status_dirty.set()

    def _device_status_patch(self, st):
        """A merge patch only ever adds map keys, so device state that went away must be
        spelled out (`pkg/kubelet/kubelet_node_status.go:608-623` zeroes the capacity of the
        resources `GetCapacity` reports removed):
          * a resource published before but gone now: capacity/allocatable "0" and its
            `extendedResources` entry deleted (null);
          * a resource still present: its domain is sent with `$patch: replace`, so device IDs
            the plugin dropped disappear instead of lingering as Healthy on the server (the
            scheduler cache allocates from that map)."""
        st = dict(st)
        ers = st.get("extendedResources") or {}
        gone = getattr(self, "_published_ers", set()) - set(ers)
        if not ers and not gone:
            return st
        out = {r: dict(dom, **{"$patch": "replace"}) for r, dom in ers.items()}
        if gone:
            st["capacity"] = dict(st["capacity"])
            st["allocatable"] = dict(st["allocatable"])
            for r in gone:
                st["capacity"][r] = "0"
                st["allocatable"][r] = "0"
                out[r] = None
        st["extendedResources"] = out
        return st

    async def update_node_status(self):
        self._collect_plugin_labels()
        await self._refresh_node_images()
        st = self._node_status()
        try:
            # strategic merge (conditions keyed by type), as the reference's PatchNodeStatus, so
            # conditions owned by others (node-problem-detector) survive the kubelet's heartbeat
            patch = {"status": self._device_status_patch(st)}
            got = await self.client.patch("nodes", self.node_name, patch, None, "strategic", "status")
            self._published_ers = set(st.get("extendedResources") or ())
            self._observe_pod_cidr(got)
            if self.plugin_labels:
                cur = self.informer_node_labels
                if any(cur.get(k) != v for k, v in self.plugin_labels.items()):
                    await self.client.patch("nodes", self.node_name, {"metadata": {"labels": self.plugin_labels}})
                    self.informer_node_labels = {**cur, **self.plugin_labels}
        except APIStatusError as e:
            if is_not_found(e) and self.register:
                await self._register_node()
            else:
                log.warning("node status update failed: %s", e)
        except (ConnectionError, OSError) as e:
            log.warning("node status update failed: %s", e)

    def _wire_dns(self):
        """The DNS configurer reports on this node (`dns.NewConfigurer(recorder, nodeRef, nodeIP,
        ...)`); a configurer shared between kubelets is copied first. A configured resolv.conf is
        checked against the search-line limits once (`CheckLimitsForResolvConf`)."""
        if self.dns is None or getattr(self.dns, "_owner", None) is self:
            return
        import copy
        self.dns = copy.copy(self.dns)
        self.dns._owner = self
        node_ref = {"kind": "Node", "metadata": {"name": self.node_name, "uid": self.node_name}}
        self.dns.node_ref = node_ref
        self.dns.node_ip = self.node_ip or self.address
        self.dns.recorder = lambda obj, typ, reason, msg: self.recorder.event(obj or node_ref, typ, reason, msg)
        if self.dns.resolv_conf:
            self.dns.check_limits_for_resolv_conf()

    def _ready_errors(self):
        """runtimeErrors() + networkErrors(); the network plugin lives in the kubelet here, so its
        status stands in for the runtime's NetworkReady when the runtime reports none."""
        rs = self.runtime_state
        errs = rs.runtime_errors() + rs.network_errors()
        if not rs.network_errors():
            net_err = self.network.status()
            if net_err:
                errs.append(f"runtime network not ready: NetworkReady=false reason:NetworkPluginNotReady "
                            f"message:{net_err}")
        return errs

    async def update_runtime_up(self):
        """`Kubelet.updateRuntimeUp`: the runtime's Status() conditions (an in-process runtime
        without one is up whenever the kubelet runs)."""
        fn = getattr(self.runtime, "status", None)
        status = err = None
        if fn is None:
            status = {RUNTIME_READY: (True, "", ""), NETWORK_READY: (True, "", "")}
        else:
            try:
                raw = await fn()
                status = None if raw is None else {
                    k: (v if isinstance(v, tuple) else (bool(v), "", "")) for k, v in raw.items()}
            except Exception as e:  # noqa: BLE001 - a failed sanity check only goes stale
                err = e
                log.warning("container runtime sanity check failed: %s", e)
        before = ready_condition(self._ready_errors())[0]
        update_runtime_up(self.runtime_state, status, error=err)
        if ready_condition(self._ready_errors())[0] != before:
            self._status_dirty.set()

    async def _runtime_up_loop(self):
        while not self._stopped:
            await asyncio.sleep(5.0)
            await self.update_runtime_up()
            if self.runtime_state.last_sync + self.runtime_state.threshold <= time.time() + 5.0:
                self._status_dirty.set()        # about to go stale: report it on time

    async def _node_status_loop(self):
        # exits on the _stopped flag, not only on cancellation: on Python 3.10 asyncio.wait_for
        # can swallow a CancelledError that races with the inner future completing
        last = 0.0
        while not self._stopped:
            self._last_status_loop = time.monotonic()
            timeout = max(0.0, self.status_freq - (time.monotonic() - last))
            try:
                await asyncio.wait_for(self._status_dirty.wait(), timeout)
                await asyncio.sleep(self.status_debounce)  # coalesce bursts of device updates
            except asyncio.TimeoutError:
                pass
            self._status_dirty.clear()
            if self._stopped:
                return
            await self.update_node_status()
            last = time.monotonic()

    # ------------------------------------------------------------------
    # pod event dispatch (podWorkers)
    def _on_add(self, pod):
        self._dispatch(pod, "add")

    def _on_update(self, old, pod):
        self._dispatch(pod, "update")

    def _on_delete(self, pod):
        self._dispatch(pod, "delete")

    def _dispatch(self, pod, op):
        uid = pod["metadata"]["uid"]
        if self.pod_checkpoints is not None:
            self._checkpoint_pod(pod, op)
        self._pending[uid] = (pod, op)
        if uid not in self._workers:
            self._workers[uid] = asyncio.ensure_future(self._worker(uid))

    def _checkpoint_pod(self, pod, op):
        """`pkg/kubelet/checkpoint`: pods annotated `node.kubernetes.io/bootstrap-checkpoint: "true"`
        are kept on disk so a restarting kubelet can run them before the API is reachable
        (self-hosted control planes)."""
        key = "Pod" + pod["metadata"]["uid"]
        ann = (pod["metadata"].get("annotations") or {}).get(BOOTSTRAP_CHECKPOINT)
        if op == "delete" or ann != "true" or core.pod_is_terminal(pod):
            self.pod_checkpoints.remove(key)
        else:
            self.pod_checkpoints.create(key, {"version": "v1", "pod": pod})

    def _restore_checkpointed_pods(self):
        n = 0
        for _, ck in self.pod_checkpoints.load_all():
            pod = ck.get("pod")
            if pod and (pod.get("spec") or {}).get("nodeName") in (None, "", self.node_name):
                pod.setdefault("spec", {})["nodeName"] = self.node_name
                self._dispatch(pod, "add")
                n += 1
        return n

    def _on_container_exit(self, pod_uid, cid):
        st = self.pods.get(pod_uid)
        if st is not None and not st.deleted and pod_uid not in self._pending:
            self._dispatch(st.pod, "sync")

    async def _worker(self, uid):
        try:
            while uid in self._pending:
                pod, op = self._pending.pop(uid)
                t0 = time.perf_counter()
                try:
                    await self.sync_pod(pod, op)
                except Exception:
                    log.exception("sync pod %s failed", pod["metadata"].get("name"))
                self.m_worker.labels(op).observe((time.perf_counter() - t0) * 1e6)
        finally:
            self._workers.pop(uid, None)

    # ------------------------------------------------------------------
    # admission
    @staticmethod
    def _requests(st):
        if st.requests is None:
            st.requests = core.pod_requests(st.pod)
        return st.requests

    def _admit_allocatable(self):
        """Node allocatable as quantities, recomputed when capacity or reservations change."""
        key = (tuple(sorted(self.capacity.items())), id(self.eviction))
        hit = getattr(self, "_alloc_cache", None)
        if hit is None or hit[0] != key:
            alloc = self._allocatable(dict(self.capacity))
            hit = (key, {k: parse_quantity(str(v)) for k, v in alloc.items()})
            self._alloc_cache = hit
        return hit[1]

    def _general_predicates(self, pod, node_labels=None):
        """`lifecycle/predicate.go` predicateAdmitHandler with `GeneralPredicates` against this
        node's allocatable and the other active pods: the pod count, cpu / memory /
        ephemeral-storage (extended resources are the device manager's, as the reference
        removes the ones the node does not advertise), HostName, host ports and the node
        selector plus required node affinity. Returns (reason, message) or None."""
        uid = pod["metadata"]["uid"]
        me = self.pods.get(uid)
        need = self._requests(me) if me is not None else core.pod_requests(pod)
        spec = pod.get("spec") or {}
        want_ports = _host_ports(spec)
        used: dict = {}
        ports = set()
        n = 0
        for other in self.pods.values():
            if other.terminated or other.rejected or other.uid == uid:
                continue
            n += 1
            for k, v in self._requests(other).items():
                used[k] = used[k] + v if k in used else v
            if want_ports:
                ports.update(_host_ports(other.pod.get("spec") or {}))
        alloc = self._admit_allocatable()
        pods_cap = int(alloc["pods"].value) if "pods" in alloc else int(self.capacity["pods"])
        if n + 1 > pods_cap:
            return "OutOfpods", (f"Node didn't have enough resource: pods, requested: 1, used: {n}, "
                                 f"capacity: {pods_cap}")
        for k in ("cpu", "memory", "ephemeral-storage"):
            v = need.get(k)
            if v is None or k not in alloc or not v.value:
                continue
            u = used.get(k)
            total = u + v if u is not None else v
            if total > alloc[k]:
                milli = k == "cpu"
                f = (lambda q: q.milli_value()) if milli else (lambda q: int(q.value))
                return f"OutOf{k}", (f"Node didn't have enough resource: {k}, requested: {f(v)}, used: "
                                     f"{f(u) if u is not None else 0}, capacity: {f(alloc[k])}")
        if spec.get("nodeName") and spec["nodeName"] != self.node_name:
            return "HostName", "Predicate HostName failed"
        for ip, proto, port in want_ports:
            for oip, oproto, oport in ports:
                if oport == port and oproto == proto and (ip == oip or "0.0.0.0" in (ip, oip)):
                    return "PodFitsHostPorts", "Predicate PodFitsHostPorts failed"
        sel = spec.get("nodeSelector") or {}
        terms = _node_affinity_required(spec)
        if sel or terms is not None:
            labels = node_labels if node_labels is not None else self._node_object()["metadata"]["labels"]
            if any(labels.get(k) != v for k, v in sel.items()) or (
                    terms is not None and not _node_affinity_matches(terms, labels, self.node_name)):
                return "MatchNodeSelector", "Predicate MatchNodeSelector failed"
        return None

    def _shortfall(self, pod) -> dict:
        """Resources this pod lacks on the node ({cpu: milli, memory: bytes, pods: n}), the input
        of critical-pod preemption."""
        need = core.pod_requests(pod)
        used = {"cpu": 0, "memory": 0}
        n = 0
        for other in self.active_pods():
            if other["metadata"]["uid"] == pod["metadata"]["uid"]:
                continue
            n += 1
            for k, v in core.pod_requests(other).items():
                if k in used:
                    used[k] += v.milli_value() if k == "cpu" else v.value
        out = {}
        if n + 1 > int(self.capacity["pods"]):
            out["pods"] = n + 1 - int(self.capacity["pods"])
        for k in ("cpu", "memory"):
            if k in need and k in self.capacity:
                cap = parse_quantity(self.capacity[k])
                cap_v = cap.milli_value() if k == "cpu" else cap.value
                want = need[k].milli_value() if k == "cpu" else need[k].value
                if used[k] + want > cap_v:
                    out[k] = used[k] + want - cap_v
        return out

    async def _preempt(self, victim, status):
        st = self.pods.get(victim["metadata"]["uid"])
        if st is None:
            return
        # before the kill: the victim's container exits re-dispatch its sync, which must neither
        # restart them nor report the pod live again
        st.rejected = status.get("reason") or "Preempting"
        await self._kill_pod(st, 0)
        st.terminated = True
        await self._write_status(st, dict(status, conditions=(victim.get("status") or {}).get("conditions") or []))

    def _can_run_pod(self, pod):
        """`canRunPod`: privileged containers need --allow-privileged; host network / PID / IPC
        need the pod's source in --host-{network,pid,ipc}-sources."""
        spec = pod.get("spec") or {}
        uid = pod["metadata"].get("uid", "")
        if not self.allow_privileged:
            for c in list(spec.get("containers") or ()) + list(spec.get("initContainers") or ()):
                if (c.get("securityContext") or {}).get("privileged"):
                    return "Forbidden", f"pod with UID {uid!r} specified privileged container, but is disallowed"
        source = ((pod["metadata"].get("annotations") or {}).get("kubernetes.io/config.source") or "api")
        for field, what in (("hostNetwork", "host networking"), ("hostPID", "host PID"), ("hostIPC", "host ipc")):
            allowed = self.host_sources.get(field)
            if spec.get(field) and allowed is not None and "*" not in allowed and source not in allowed:
                return "Forbidden", f"pod with UID {uid!r} specified {what}, but is disallowed"
        return None

    async def _admit(self, st: PodState):
        pod = st.pod
        r = self._can_run_pod(pod)
        if r is not None:
            return r
        r = self.sysctls.admit(pod)
        if r is not None:
            return r
        try:
            await self.dm.admit_pod(pod)
        except AdmitError as e:
            return "UnexpectedAdmissionError", f"Pod admission failed: {e}"
        r = self._general_predicates(pod)
        if r is not None and r[0] == "MatchNodeSelector":
            # labels set on the Node object through the API (kubectl label node ...) count too:
            # the reference admits against the node from its lister, not its registration labels
            try:
                api_node = await self.client.get("nodes", self.node_name)
                r = self._general_predicates(pod, (api_node.get("metadata") or {}).get("labels") or {})
            except (APIStatusError, ConnectionError, OSError):
                pass
        if r is not None and r[0] in ("OutOfcpu", "OutOfmemory", "OutOfpods"):
            # `pkg/kubelet/preemption`: a critical pod evicts lower-QoS pods instead of failing
            try:
                if await self.preemption.handle_admission_failure(pod, self._shortfall(pod)):
                    r = self._general_predicates(pod)
            except ValueError as e:
                log.warning("critical pod %s: preemption impossible: %s", pod["metadata"].get("name"), e)
        if r is None and self.eviction is not None:
            r = self.eviction.admit(pod)
        return r

    # ------------------------------------------------------------------
    # sync
    async def sync_pod(self, pod, op):
        uid = pod["metadata"]["uid"]
        st = self.pods.get(uid)
        if op == "delete":
            if st is not None:
                st.deleted = True          # before the kill: container-exit callbacks must not resync it
                await self._kill_pod(st, 0)
                await self._teardown_network(st)
                if st.volumes:
                    await self.volumes.unpublish(st.pod)
                    self.volumes.teardown(st.pod)
                    st.volumes = None
                st.deleted = True
                self.pods.pop(uid, None)
                self.by_key.pop(_key(pod), None)
                self.dm.delete_pod(uid)
                if self.cgroups is not None:
                    self.cgroups.destroy_pod(uid)
                for cid in list(st.containers.values()) + list(st.init_containers.values()) + list(st.previous.values()):
                    if cid:
                        self._unlink_log(cid)
            return
        if st is None:
            # an internal resync (container exit, back-off timer) of a pod already deleted must
            # not resurrect it: only informer add/update events create pod state
            if core.pod_is_terminal(pod) or op == "sync":
                return
            st = self.pods[uid] = PodState(pod)
            if getattr(self.runtime, "shares_host_network", False) or (pod.get("spec") or {}).get("hostNetwork"):
                st.ip = self.address     # no network namespace: the pod is reachable on the node address
            self.by_key[_key(pod)] = uid
            if self._adoptable:
                await self._adopt(st)
        else:
            st.pod = pod
        md = pod["metadata"]
        if md.get("deletionTimestamp"):
            await self._kill_pod(st, md.get("deletionGracePeriodSeconds") or 0)
            await self._finalize_deletion(st)
            return
        if st.rejected or st.terminated:
            return
        if not st.admitted:
            r = await self._admit(st)
            if r is not None:
                reason, msg = r
                st.rejected = reason
                if st.adopted:
                    await self._kill_pod(st, 0)
                # rejectPod: the event carries the message, the status "Pod " + message
                self.recorder.event(pod, "Warning", reason, msg)
                await self._write_status(st, {"phase": core.POD_FAILED, "reason": reason, "message": "Pod " + msg,
                                              "conditions": (pod.get("status") or {}).get("conditions") or []})
                return
            st.admitted = True
            # an adopted pod (kubelet restart) keeps its status.startTime: activeDeadlineSeconds
            # counts from it (active_deadline.go)
            st.start_time = st.start_time or now_rfc3339()
        if await self._enforce_active_deadline(st):
            return
        await self._sync_containers(st)

    async def _enforce_active_deadline(self, st: PodState) -> bool:
        """`pkg/kubelet/active_deadline.go`: a pod active on the node longer than
        spec.activeDeadlineSeconds (counted from status.startTime) is killed and fails with reason
        DeadlineExceeded. Before the deadline a resync is armed for the moment it passes."""
        ads = (st.pod.get("spec") or {}).get("activeDeadlineSeconds")
        start = parse_rfc3339(st.start_time) if st.start_time else None
        if ads is None or start is None:
            return False
        left = start + float(ads) - time.time()
        if left > 0:
            if not st.deadline_armed:
                st.deadline_armed = True
                asyncio.get_running_loop().call_later(left + 0.01, self._resync, st.uid)
            return False
        msg = "Pod was active on the node longer than the specified deadline"
        st.rejected = "DeadlineExceeded"
        self.recorder.event(st.pod, "Normal", "DeadlineExceeded", msg)
        await self._kill_pod(st, 0)
        await self._write_status(st, {"phase": core.POD_FAILED, "reason": "DeadlineExceeded", "message": msg,
                                      "conditions": (st.pod.get("status") or {}).get("conditions") or []})
        return True

    async def _sync_containers(self, st: PodState):
        pod = st.pod
        spec = pod.get("spec") or {}
        rt = self.runtime
        if st.volumes is None:
            if spec.get("volumes"):
                try:
                    st.volumes = await self.volumes.setup(pod, self.node_name, st.ip)
                except (VolumeError, APIStatusError, OSError) as e:
                    # volumemanager WaitForAttachAndMount: report, retry on the next sync
                    self.recorder.event(pod, "Warning", "FailedMount", f"Unable to mount volumes for pod: {e}")
                    await self._report(st)
                    asyncio.get_running_loop().call_later(2.0, self._resync, st.uid)
                    return
            else:
                st.volumes = {}
        if st.sandbox is None:
            if self.cgroups is not None:
                self.cgroups.ensure_pod(pod)
            ann = {}
            pr = self.dm.pod_resources(pod)
            if pr:
                ann.update(pr["annotations"])
            st.sandbox = await rt.run_pod_sandbox(pod, ann)
            self.m_runtime_ops.labels("run_podsandbox").inc()
            st.net_setup = False
        if not st.net_setup:
            if not await self._setup_network(st):
                return
        # init containers, sequentially
        for c in spec.get("initContainers") or ():
            cid = st.init_containers.get(c["name"])
            if cid is None:
                cid = await self._start(st, c)
                st.init_containers[c["name"]] = cid
                if cid is None:
                    await self._report(st)
                    return
            cs = rt.container_status(cid)
            if cs is None or cs.state != EXITED:
                await self._report(st)
                return  # wait for the exit event
            if cs.exit_code != 0:
                if spec.get("restartPolicy", "Always") == "Never":
                    st.terminated = True
                    await self._report(st)
                    return
                del st.init_containers[c["name"]]
                st.restarts[c["name"]] = st.restarts.get(c["name"], 0) + 1
                await self._report(st)
                self._dispatch(pod, "sync")
                return
        policy = spec.get("restartPolicy", "Always")
        for c in spec.get("containers") or ():
            cid = st.containers.get(c["name"])
            if cid is not None:
                cs = rt.container_status(cid)
                if cs is not None and cs.state != RUNNING:
                    restart = should_container_be_restarted(policy, cs)
                    if restart and not md_deleting(pod) and self._in_backoff(st, c, cs):
                        continue
                    if restart and not md_deleting(pod):
                        st.restarts[c["name"]] = st.restarts.get(c["name"], 0) + 1
                        # keep one dead instance per container (container GC's MaxPerPodContainer=1)
                        old = st.previous.get(c["name"])
                        if old is not None:
                            await rt.remove_container(old)
                            self._unlink_log(old)
                        st.previous[c["name"]] = cid
                        cid = None
            if cid is None:
                st.containers[c["name"]] = await self._start(st, c)
        await self._report(st)

    def _link_log(self, pod, cname, cid):
        cs = self.runtime.container_status(cid)
        target = getattr(cs, "log_path", "") if cs is not None else ""
        if not target:
            return
        md = pod["metadata"]
        # the id part must not contain '-' (logging agents split `<container>-<id>` at the last one)
        bare = "".join(ch for ch in cid.split("://", 1)[-1] if ch.isalnum())
        link = os.path.join(self.container_log_dir, f"{md['name']}_{md.get('namespace', 'default')}_{cname}-{bare}.log")
        try:
            os.makedirs(self.container_log_dir, exist_ok=True)
            if os.path.lexists(link):
                os.unlink(link)
            os.symlink(os.path.abspath(target), link)
            self._log_links[cid] = link
        except OSError as e:
            log.warning("container log symlink %s: %s", link, e)

    def _unlink_log(self, cid):
        link = self._log_links.pop(cid, None)
        if link:
            try:
                os.unlink(link)
            except OSError:
                pass

    def current_config(self):
        """KubeletConfiguration (kubeletconfig/v1alpha1) of the running kubelet (/configz)."""
        return {"kind": "KubeletConfiguration", "apiVersion": "kubeletconfig/v1alpha1",
                "maxPods": int(self.capacity["pods"]), "nodeStatusUpdateFrequency": f"{self.status_freq:g}s",
                "eventRecordQPS": self.recorder.qps, "eventBurst": self.recorder.burst,
                "cpuManagerPolicy": "static" if self.cpu_manager is not None else "none",
                "cgroupsPerQOS": self.cgroups is not None, "cgroupRoot": self.cgroup_root or "",
                "kubeReserved": self.reserved[0], "systemReserved": self.reserved[1],
                "podManifestPath": self.pod_manifest_path or "", "featureGates": {"DevicePlugins": True}}

    def running_pods(self):
        """/runningpods/: pods as the container runtime sees them (`kubelet.GetRunningPods`)."""
        items = []
        for st in self.pods.values():
            running = []
            for name, cid in st.containers.items():
                cs = self.runtime.container_status(cid) if cid else None
                if cs is not None and cs.state == RUNNING:
                    running.append((name, cid))
            if not running:
                continue
            md = st.pod["metadata"]
            images = {c["name"]: c.get("image", "") for c in (st.pod.get("spec") or {}).get("containers") or ()}
            items.append({"metadata": {"name": md["name"], "namespace": md.get("namespace", ""), "uid": md["uid"]},
                          "spec": {"containers": [{"name": n, "image": images.get(n, "")} for n, _ in running]},
                          "status": {"containerStatuses": [{"name": n, "containerID": c} for n, c in running]}})
        return {"kind": "PodList", "apiVersion": "v1", "metadata": {}, "items": items}

    def _node_logs(self, rel):
        """/logs/: read-only view of the node's log directory (`server.go` getLogs)."""
        from ..utils.httpserver import log_dir_response
        return log_dir_response(self.node_log_dir, rel)

    async def _container_logs(self, cid, tail, q):
        """`/containerLogs` (`server.go` getContainerLogs + kuberuntime ReadLogs): tailLines,
        limitBytes, follow (the file is followed while the container runs), timestamps (lines
        read while following carry their arrival time: the runtimes write raw output files with
        no per-line times), sinceSeconds / sinceTime (a file not written since then yields
        nothing, otherwise all of it: the same file-level granularity)."""
        from ..api.meta import parse_rfc3339
        from .logs import is_structured, read_logs
        limit = int(q.get("limitBytes") or 0)
        path = getattr(self.runtime, "log_path", lambda c: None)(cid)
        since = None
        if q.get("sinceSeconds"):
            since = time.time() - float(q["sinceSeconds"])
        elif q.get("sinceTime"):
            since = parse_rfc3339(q["sinceTime"])
        if path and q.get("follow") not in ("true", "1") and os.path.exists(path):
            # a CRI runtime's own log file (`<time> <stream> <tag> <log>` or docker JSON):
            # ReadLogs with per-record times
            with open(path, "rb") as f:
                first = f.readline()
            if first and is_structured(first):
                with open(path, "rb") as f:
                    raw = f.read()
                return Response(200, read_logs(raw, tail, since, q.get("timestamps") in ("true", "1"), limit or None),
                                "text/plain")
        data = await self.runtime.container_logs(cid, tail)
        if since is not None and path and os.path.exists(path) and os.path.getmtime(path) < since:
            data = b""
        stamp = q.get("timestamps") in ("true", "1")
        if stamp and data:
            # lines already written carry the file's last write time (file-level granularity)
            mt = os.path.getmtime(path) if path and os.path.exists(path) else time.time()
            ts = now_rfc3339_nano(mt).encode() + b" "
            data = b"".join(ts + ln for ln in data.splitlines(keepends=True))
        if limit:
            data = data[:limit]
        if q.get("follow") not in ("true", "1") or not path:
            return Response(200, data, "text/plain")
        runtime = self.runtime

        async def follow(w):
            sent = len(data)
            if data:
                w.write(data)
            pos = os.path.getsize(path) if os.path.exists(path) else 0
            while True:
                try:
                    st = runtime.container_status(cid)
                except (KeyError, OSError):
                    st = None
                running = st is not None and st.state == RUNNING
                if os.path.exists(path):
                    with open(path, "rb") as f:
                        f.seek(pos)
                        chunk = f.read(1 << 20)
                    if chunk:
                        pos += len(chunk)
                        if stamp:
                            now = now_rfc3339_nano()
                            chunk = b"".join(now.encode() + b" " + ln for ln in chunk.splitlines(keepends=True))
                        if limit:
                            chunk = chunk[:max(0, limit - sent)]
                        if chunk:
                            w.write(chunk)
                            sent += len(chunk)
                        if limit and sent >= limit:
                            return
                        continue
                if not running:
                    return
                await asyncio.sleep(0.1)
        return StreamResponse(follow, "text/plain")

    def _service_env(self, pod):
        if self.svc_informer is None or not self.svc_informer.synced.is_set():
            return []
        from .envvars import service_env
        ns = pod["metadata"].get("namespace", "default")
        key = (ns, self.svc_informer.store.generation)
        hit = self._svc_env_cache.get(ns)
        if hit is not None and hit[0] == key:
            return list(hit[1])
        env = service_env(self.svc_informer.list(), ns, self.master_service_namespace)
        self._svc_env_cache[ns] = (key, env)
        return list(env)

    async def _start(self, st, c):
        from .images import ImagePullError
        try:
            await self.images.ensure_image_exists(st.pod, c)
            st.waiting.pop(c["name"], None)
        except ImagePullError as e:
            st.waiting[c["name"]] = (e.reason, e.message)
            await self._report(st)
            asyncio.get_running_loop().call_later(max(0.05, self.images.retry_after(c.get("image", ""))),
                                                  self._resync, st.uid)
            return None
        try:
            opts = RunContainerOptions.from_device_opts(await self.dm.init_container(st.pod, c))
        except Exception as e:
            self.recorder.event(st.pod, "Warning", "Failed", f"Error: device plugin InitContainer failed: {e}")
            return None
        spec_c = c
        opts.attempt = st.restarts.get(c["name"], 0)
        cfg_fn = getattr(self.image_service, "image_config", None)
        cfg = cfg_fn(c.get("image", "")) if cfg_fn is not None else None
        err = _apply_security_context(st.pod, c, opts, image_user(cfg) if cfg is not None else None)
        if err:
            # kuberuntime_container.go: verifyRunAsNonRoot fails the start with CreateContainerConfigError
            st.waiting[c["name"]] = ("CreateContainerConfigError", err)
            self.recorder.event(st.pod, "Warning", "Failed", f"Error: {err}", field_path=_field_path(st.pod, c))
            await self._report(st)
            return None
        # makeMounts: no kubelet /etc/hosts (or resolv.conf) over a path the container mounts itself
        own = {make_absolute_path(m.get("mountPath", "")) for m in c.get("volumeMounts") or ()}
        opts.mounts.extend(m for m in st.net_mounts if m["containerPath"] not in own)
        opts.oom_score_adj = oom_score_adj(st.pod, c, parse_quantity(self.capacity["memory"]).value)
        if self.cgroups is not None:
            opts.cgroup_parent = self.cgroups.pod_dir(st.pod)
        svc_env = self._service_env(st.pod)
        if svc_env or c.get("volumeMounts") or c.get("envFrom") or any(
                "valueFrom" in e or "$(" in str(e.get("value", "")) for e in c.get("env") or ()):
            try:
                spec_c = dict(c, env=await self.volumes.env_for(st.pod, c, self.node_name, st.ip, base_env=svc_env),
                              envFrom=[])
                for m in self.volumes.mounts_for(c, st.volumes or {}):
                    opts.mounts.append(m)
                for m in c.get("volumeMounts") or ():
                    opts.envs.append({"name": "KUBERNETES_VOLUME_" + m["name"].upper().replace("-", "_"),
                                      "value": (st.volumes or {}).get(m["name"], "")})
            except (VolumeError, APIStatusError) as e:
                self.recorder.event(st.pod, "Warning", "Failed", f"Error: {e}")
                asyncio.get_running_loop().call_later(2.0, self._resync, st.uid)
                return None
        if any("$(" in str(x) for x in (spec_c.get("command") or []) + (spec_c.get("args") or [])):
            # `kubecontainer.ExpandContainerCommandAndArgs`: $(VAR) from the container's resolved
            # environment; unknown references stay as written, $$ escapes
            cmd, args = expand_container_command_and_args(spec_c, spec_c.get("env") or ())
            spec_c = dict(spec_c, command=cmd or [], args=args or [])
        if self.cpu_manager is not None:
            from .cpumanager import format_cpulist
            try:
                cpus = self.cpu_manager.allocate(st.pod, c, self._gpu_numa(st.pod))
            except ValueError as e:
                self.recorder.event(st.pod, "Warning", "Failed", f"Error: cpu manager: {e}")
                return None
            opts.envs.append({"name": "KAMD_CPUSET", "value": format_cpulist(cpus)})
            opts.annotations.append({"name": "io.kubernetes.cpuset", "value": format_cpulist(cpus)})
        try:
            cid = await self.runtime.create_container(st.sandbox, st.pod, spec_c, opts)
            self.m_runtime_ops.labels("create_container").inc()
            # kuberuntime_container.go startContainer: CreatedContainer / StartedContainer events
            self.recorder.event(st.pod, "Normal", "Created", "Created container", field_path=_field_path(st.pod, c))
            await self.runtime.start_container(cid)
            self.m_runtime_ops.labels("start_container").inc()
            self.recorder.event(st.pod, "Normal", "Started", "Started container", field_path=_field_path(st.pod, c))
        except Exception as e:
            self.recorder.event(st.pod, "Warning", "Failed", f"Error: {e}")
            return None
        if self.container_log_dir:
            self._link_log(st.pod, c["name"], cid)
        post = ((c.get("lifecycle") or {}).get("postStart"))
        if post:
            # kuberuntime_container.go startContainer: a failed postStart handler is reported on
            # the container and kills it
            msg, err = await HandlerRunner(self.runtime).run(cid, st.pod, c, post, st.ip)
            if err is not None:
                self.recorder.event(st.pod, "Warning", "FailedPostStartHook", msg, field_path=_field_path(st.pod, c))
                await self.runtime.stop_container(cid, 0)
                return cid
        if c.get("livenessProbe") or c.get("readinessProbe"):
            self.probes.start(st.uid, st.pod, c, cid)
        return cid

    def _gpu_numa(self, pod):
        """NUMA nodes of the devices assigned to the pod (amd.com/numa attribute)."""
        assigned = core.pod_assigned_devices(pod)
        if not assigned:
            return ()
        store = getattr(self.dm, "store", None)
        res = getattr(store, "resources", {}) if store is not None else {}
        out = set()
        for rn, ids in assigned.items():
            devs = (res.get(rn) or {}).get("resources") or {}
            for i in ids:
                n = ((devs.get(i) or {}).get("attributes") or {}).get(core.ATTR_NUMA)
                if n is not None and str(n).isdigit():
                    out.add(int(n))
        return tuple(sorted(out))

    _PROJECTED = ("configMap", "secret", "downwardAPI", "projected")

    async def _volume_sync_loop(self):
        """Periodic pod sync of projected volumes: ConfigMap / Secret updates (and optional
        sources appearing), label / annotation changes reach running containers' files."""
        while True:
            await asyncio.sleep(self.sync_frequency)
            for st in list(self.pods.values()):
                if st.terminated or not st.volumes:
                    continue
                vols = (st.pod.get("spec") or {}).get("volumes") or ()
                if not any(k in v for v in vols for k in self._PROJECTED):
                    continue
                try:
                    await self.volumes.refresh(st.pod, self.node_name, st.ip)
                except (VolumeError, APIStatusError, OSError) as e:
                    log.debug("volume refresh of %s failed: %s", st.pod["metadata"].get("name"), e)

    def _resync(self, uid):
        st = self.pods.get(uid)
        if st is not None and not st.terminated and uid not in self._pending:
            self._dispatch(st.pod, "sync")

    def _on_readiness(self, uid, cname, ok):
        st = self.pods.get(uid)
        if st is not None:
            self._resync(uid)

    def _on_probe_failure(self, uid, cname, kind, msg):
        st = self.pods.get(uid)
        if st is not None:
            self.recorder.event(st.pod, "Warning", "Unhealthy", f"{kind.capitalize()} probe failed: {msg}",
                                field_path=f"spec.containers{{{cname}}}")

    def _on_liveness_failure(self, uid, cname, cid, msg):
        st = self.pods.get(uid)
        if st is None or st.containers.get(cname) != cid:
            return
        self.recorder.event(st.pod, "Normal", "Killing", f"Killing container {cname}: failed liveness probe")

        async def kill():
            await self.runtime.stop_container(cid, 0)
            self._resync(uid)
        spawn(kill())

    def _in_backoff(self, st: PodState, c, cs):
        """kuberuntime `doBackOff`: the first restart is immediate; later ones wait
        initial·2^k (capped). A container that ran for 2×max before failing starts over."""
        init, cap = self.crash_backoff
        if not init:
            return False
        now = time.monotonic()
        ent = st.backoff.get(c["name"])
        ran = (cs.finished_at or 0) - (cs.started_at or 0)
        if ent is not None and ran > 2 * cap:
            ent = None
        if ent is None:
            st.backoff[c["name"]] = [now + init, init]
            st.waiting.pop(c["name"], None)
            return False
        if now < ent[0]:
            md = st.pod["metadata"]
            st.waiting[c["name"]] = ("CrashLoopBackOff", f"Back-off {ent[1]:g}s restarting failed container={c['name']} "
                                                         f"pod={md['name']}_{md.get('namespace', 'default')}({st.uid})")
            asyncio.get_running_loop().call_later(ent[0] - now + 0.01, self._resync, st.uid)
            return True
        delay = min(ent[1] * 2, cap)
        st.backoff[c["name"]] = [now + delay, delay]
        st.waiting.pop(c["name"], None)
        return False

    async def garbage_collect_containers(self, now=None, policy=None, evict_terminated=False):
        """`pkg/kubelet/kuberuntime/kuberuntime_gc.go` evictContainers over the runtime's
        containers (see `containers_to_evict`). Instances the kubelet still reports a live pod's
        status from (the latest of each container) count toward the limits but are never removed
        here; they go with the pod. Containers of no tracked pod belong to deleted pods. Returns
        the removed container ids."""
        pol = policy if policy is not None else (self.container_gc or {})
        now = now or time.time()
        rt = self.runtime
        recs, owner, current = [], {}, set()
        for st in self.pods.values():
            for name, cid in list(st.containers.items()) + list(st.init_containers.items()):
                if cid:
                    current.add(cid)
            for name, cid in list(st.containers.items()) + list(st.init_containers.items()) + list(st.previous.items()):
                if not cid or cid in owner:
                    continue
                cs = rt.container_status(cid)
                if cs is None:
                    if st.previous.get(name) == cid:
                        st.previous.pop(name, None)
                    continue
                owner[cid] = (st, name)
                recs.append((cid, st.uid, name, cs.created_at, cs.state))
        for cs in list(rt.list_containers()):
            if cs.id not in owner:
                recs.append((cs.id, "", cs.name, cs.created_at, cs.state))

        def deleted(uid):
            st = self.pods.get(uid) if uid else None
            return st is None or st.deleted

        def terminated(uid):
            st = self.pods.get(uid)
            return st is not None and st.terminated

        out = []
        for cid in containers_to_evict(recs, pol, now, deleted, terminated, evict_terminated):
            if cid in current:
                continue
            await rt.remove_container(cid)
            self._unlink_log(cid)
            ent = owner.get(cid)
            if ent is not None and ent[0].previous.get(ent[1]) == cid:
                ent[0].previous.pop(ent[1], None)
            out.append(cid)
        return out

    async def _container_gc_loop(self):
        period = float((self.container_gc or {}).get("period", 60.0))
        while not self._stopped:
            await asyncio.sleep(period)
            try:
                await self.garbage_collect_containers()
            except Exception as e:  # noqa: BLE001 - GC failures are logged and retried
                log.warning("container garbage collection failed: %s", e)

    async def _adopt(self, st: PodState):
        """Take over the sandbox and containers the runtime still runs for this pod after a
        kubelet restart (kuberuntime `computePodActions` keeps running containers whose pod is
        known). Device admission (AdmitPod) still runs again — the fork rebuilds its per-pod
        plugin state that way — but nothing is restarted."""
        ps = self._adoptable.pop(st.uid, None)
        if not ps:
            return
        ready = [sb for sb in ps["sandboxes"] if sb[1]]
        if not ready:
            for sid, _, _ in ps["sandboxes"]:           # a dead sandbox: start the pod afresh
                await self.runtime.remove_pod_sandbox(sid)
            return
        sid, _, ip = ready[-1]
        for osid, _, _ in ps["sandboxes"]:
            if osid != sid:
                await self.runtime.remove_pod_sandbox(osid)
        spec = st.pod.get("spec") or {}
        init_names = {c["name"] for c in spec.get("initContainers") or ()}
        names = {c["name"] for c in spec.get("containers") or ()}
        by_name: dict = {}
        for name, cid, attempt, created, csid in ps["containers"]:
            if csid == sid and (name in names or name in init_names):
                by_name.setdefault(name, []).append((created, attempt, cid))
        st.sandbox = sid
        st.adopted = True
        self.adopted_pods += 1
        for name, lst in by_name.items():
            lst.sort()
            _, attempt, cid = lst[-1]
            if name in init_names:
                st.init_containers[name] = cid
            else:
                st.containers[name] = cid
                if len(lst) > 1:
                    st.previous[name] = lst[-2][2]
            st.restarts[name] = int(attempt or 0)
        status = st.pod.get("status") or {}
        st.start_time = status.get("startTime") or now_rfc3339()
        host_net = bool(spec.get("hostNetwork")) or getattr(self.runtime, "shares_host_network", False)
        if not host_net:
            st.ip = ip or status.get("podIP") or st.ip
            if self.hostports is not None:
                self.hostports.add(st.pod, st.ip)
        st.net_mounts = self._pod_net_files(st, st.pod)
        st.net_setup = True
        log.info("adopted running pod %s (sandbox %s, %d containers)", st.pod["metadata"].get("name"), sid,
                 len(st.containers))

    async def _remove_orphans(self, grace):
        """Runtime pods no source knows about once the kubelet has synced (deleted while it was
        down): stop and remove them, like the kubelet's cleanup of orphaned pods."""
        await asyncio.sleep(grace)
        left, self._adoptable = self._adoptable, {}
        for uid, ps in left.items():
            if uid in self.pods:
                continue
            for sid, _, _ in ps["sandboxes"]:
                try:
                    await self.runtime.stop_pod_sandbox(sid)
                    await self.runtime.remove_pod_sandbox(sid)
                except Exception as e:  # noqa: BLE001 - best effort
                    log.warning("removing orphaned sandbox %s: %s", sid, e)

    async def _setup_network(self, st: PodState):
        """SetUpPod through the network plugin (own-netns runtimes), host ports, and the
        kubelet-managed /etc/hosts + /etc/resolv.conf."""
        from .network import NetworkError
        pod = st.pod
        host_net = bool((pod.get("spec") or {}).get("hostNetwork")) or getattr(self.runtime, "shares_host_network", False)
        try:
            if not host_net:
                ip = await self.network.setup_pod(pod, st.sandbox, getattr(self.runtime, "netns_of", lambda s: "")(st.sandbox))
                if ip:
                    st.ip = ip
                if self.hostports is not None:
                    self.hostports.add(pod, st.ip)
        except NetworkError as e:
            self.recorder.event(pod, "Warning", "FailedCreatePodSandBox", f"Failed to set up pod network: {e}")
            await self.runtime.remove_pod_sandbox(st.sandbox)
            st.sandbox = None
            await self._report(st)
            asyncio.get_running_loop().call_later(2.0, self._resync, st.uid)
            return False
        st.net_mounts = self._pod_net_files(st, pod)
        st.net_setup = True
        return True

    def _pod_net_files(self, st, pod):
        """The kubelet-managed /etc/hosts (+ resolv.conf with cluster DNS) of the pod's containers;
        a runtime that never applies mounts (the hollow stub) gets none written."""
        pod_dir = os.path.join(self.root_dir, "pods", st.uid)
        if self.dns is not None:
            return self.dns.write_pod_files(pod_dir, pod, st.ip)
        if getattr(self.runtime, "name", "") == "stub":
            return []
        from .network import DNSConfigurer
        return DNSConfigurer(resolv_conf=None).write_pod_files(pod_dir, pod, st.ip, hosts_only=True)

    async def _teardown_network(self, st: PodState):
        if not st.net_setup:
            return
        st.net_setup = False
        if self.hostports is not None:
            self.hostports.remove(st.pod)
        host_net = bool((st.pod.get("spec") or {}).get("hostNetwork")) or getattr(self.runtime, "shares_host_network", False)
        if not host_net and st.sandbox is not None:
            try:
                await self.network.teardown_pod(st.pod, st.sandbox)
            except Exception as e:  # noqa: BLE001 - teardown is best effort, like the reference
                log.warning("network teardown for %s: %s", st.uid, e)

    async def _kill_pod(self, st: PodState, grace):
        self.probes.remove_pod(st.uid)
        if self.cpu_manager is not None:
            self.cpu_manager.release_pod(st.uid)
        rt = self.runtime
        spec = st.pod.get("spec") or {}
        by_name = {c["name"]: c for c in spec.get("containers") or ()}
        runner = HandlerRunner(rt)
        pre = [(name, cid, (by_name[name].get("lifecycle") or {}).get("preStop")) for name, cid in st.containers.items()
               if cid is not None and name in by_name]
        hooks = [(name, cid, h) for name, cid, h in pre if h]
        # kuberuntime_container.go killContainer (:574-599): the grace period is the deletion's
        # (else the pod's terminationGracePeriodSeconds), minus the preStop hook's run time, and
        # never below 2 s; grace 0 is this kubelet's internal immediate kill (the reference's
        # gracePeriodOverride)
        budget = float(grace if grace is not None else spec.get("terminationGracePeriodSeconds", 30))
        t_hooks = time.monotonic()
        if hooks and budget > 0:
            # preStop handlers run (concurrently) within the grace period before the stop signal
            async def hook(name, cid, h):
                msg, err = await runner.run(cid, st.pod, by_name[name], h, st.ip)
                if err is not None:
                    self.recorder.event(st.pod, "Warning", "FailedPreStopHook", msg,
                                        field_path=_field_path(st.pod, by_name[name]))
            try:
                await asyncio.wait_for(asyncio.gather(*(hook(*x) for x in hooks)), max(budget, 0.5))
            except asyncio.TimeoutError:
                pass
        timeout = 0.0 if budget <= 0 else max(budget - (time.monotonic() - t_hooks), MIN_KILL_GRACE_SECONDS)
        stops = []
        for name, cid in list(st.containers.items()) + list(st.init_containers.items()):
            if cid is not None:
                cs = rt.container_status(cid)
                if cs is not None and cs.state != EXITED:
                    # kuberuntime_container.go killContainer: KillingContainer event
                    self.recorder.event(st.pod, "Normal", "Killing", f"Killing container with id {cid}:Need to kill Pod",
                                        field_path=_field_path(st.pod, {"name": name}))
                stops.append(rt.stop_container(cid, timeout))
        if stops:
            # killContainersWithSyncResult: every container is stopped in parallel
            await asyncio.gather(*stops)
        if st.sandbox is not None:
            await rt.stop_pod_sandbox(st.sandbox)
        st.terminated = True

    async def _finalize_deletion(self, st: PodState):
        """Containers are dead: report final status, then remove the pod object (grace 0)."""
        pod = st.pod
        md = pod["metadata"]
        await self._teardown_network(st)
        if st.sandbox is not None:
            await self.runtime.remove_pod_sandbox(st.sandbox)     # removes its containers too
            st.sandbox = None
            for cid in list(st.containers.values()) + list(st.init_containers.values()) + list(st.previous.values()):
                if cid:
                    self._unlink_log(cid)
        if st.volumes:
            await self.volumes.unpublish(pod)
            self.volumes.teardown(pod)
            st.volumes = None
        if st.final_deleted:
            # every later update of the terminating pod (our own status write, the delete's
            # MODIFIED) lands here again; one accepted grace-0 delete is enough (status_manager
            # deletes once the pod `canBeDeleted`)
            return
        try:
            await self.client.delete("pods", md["name"], md.get("namespace"), grace_period=0, uid=md["uid"],
                                     decode=False)
            st.final_deleted = True
        except APIStatusError as e:
            if is_not_found(e) or is_conflict(e):
                st.final_deleted = True
            else:
                log.warning("final delete of %s failed: %s", md["name"], e)

    # ------------------------------------------------------------------
    # status
    def _compute_status(self, st: PodState):
        pod = st.pod
        spec = pod.get("spec") or {}
        rt = self.runtime
        statuses, init_statuses = [], []
        for c in spec.get("containers") or ():
            cid = st.containers.get(c["name"])
            cs = rt.container_status(cid) if cid else None
            prev = st.previous.get(c["name"])
            pcs = rt.container_status(prev) if prev and prev != cid else None
            s = _container_status(c, cs, st.restarts.get(c["name"], 0), st.waiting.get(c["name"]), pcs)
            statuses.append(s)
            if cs is not None and cs.state == RUNNING:
                if c.get("readinessProbe") and not self.probes.ready(st.uid, c["name"]):
                    s["ready"] = False
        for c in spec.get("initContainers") or ():
            cid = st.init_containers.get(c["name"])
            cs = rt.container_status(cid) if cid else None
            ics = _container_status(c, cs, st.restarts.get(c["name"], 0), st.waiting.get(c["name"]))
            # prober_manager.go UpdatePodStatus: an init container is ready once it exited 0
            ics["ready"] = cs is not None and cs.state == EXITED and cs.exit_code == 0
            init_statuses.append(ics)
        phase = get_phase(spec, statuses, init_statuses)
        now = now_rfc3339()
        old_conds = {c["type"]: c for c in (pod.get("status") or {}).get("conditions") or ()}

        def cond(c):
            prev = old_conds.get(c["type"])
            c["lastProbeTime"] = None
            c["lastTransitionTime"] = prev["lastTransitionTime"] if prev and prev.get("status") == c["status"] else now
            return c

        # status_manager.go SetPodStatus: Initialized and Ready from generate.go
        ready_c = generate_pod_ready_condition(spec, statuses, phase)
        # generateAPIPodStatus: Initialized, Ready, PodScheduled (1.9 has no ContainersReady)
        conds = [cond(generate_pod_initialized_condition(spec, init_statuses, phase)),
                 cond(ready_c),
                 cond({"type": core.COND_POD_SCHEDULED, "status": "True"})]
        status = {"phase": phase, "conditions": conds, "hostIP": self.address, "podIP": st.ip,
                  "startTime": st.start_time, "containerStatuses": statuses,
                  "qosClass": (pod.get("status") or {}).get("qosClass", "BestEffort")}
        if init_statuses:
            status["initContainerStatuses"] = init_statuses
        if phase in (core.POD_SUCCEEDED, core.POD_FAILED):
            st.terminated = True
        return normalize_status(pod, status)

    async def _report(self, st: PodState):
        status = self._compute_status(st)
        if status["phase"] == core.POD_RUNNING and st.running_at is None:
            st.running_at = time.time()
            created = parse_rfc3339(st.pod["metadata"].get("creationTimestamp")) or st.first_seen
            self.m_start.observe(max(0.0, st.running_at - st.first_seen) * 1e6)
            self.m_running.set(sum(1 for s in self.pods.values() if s.running_at and not s.terminated))
            del created
        if st.terminated and st.sandbox is not None and status["phase"] in (core.POD_SUCCEEDED, core.POD_FAILED):
            await self.runtime.stop_pod_sandbox(st.sandbox)
            if self.cpu_manager is not None:
                self.cpu_manager.release_pod(st.uid)
        await self._write_status(st, status)

    async def _write_status(self, st: PodState, status):
        if st.last_status == status:
            return
        st.last_status = status
        uid = st.uid
        self._status_next[uid] = (st.pod, status)
        if uid not in self._status_inflight:
            self._status_inflight[uid] = asyncio.ensure_future(self._status_writer(uid))

    async def _status_writer(self, uid):
        try:
            while uid in self._status_next:
                pod, status = self._status_next.pop(uid)
                md = pod["metadata"]
                async with self._status_sem:
                    try:
                        await self.client.patch("pods", md["name"], {"status": status}, md.get("namespace"), "merge", "status")
                    except APIStatusError as e:
                        if not is_not_found(e):
                            log.warning("status update of %s failed: %s", md["name"], e)
                    except (ConnectionError, OSError) as e:
                        log.warning("status update of %s failed: %s", md["name"], e)
        finally:
            self._status_inflight.pop(uid, None)

    # ------------------------------------------------------------------
    # HTTP (kubelet server :10250 subset)
    # debugging handlers (`server.go` InstallDebuggingHandlers): absent from the read-only server
    # and with --enable-debugging-handlers=false
    DEBUG_PATHS = ("/run/", "/exec/", "/attach/", "/portForward/", "/containerLogs/", "/logs", "/runningpods",
                   "/debug/pprof", "/configz", "/cri/")

    async def _http(self, req):
        if self.auth is not None:
            denied = await self.auth.check(req)
            if denied is not None:
                return Response(denied[0], denied[1].encode(), "text/plain")
        return await self._serve(req, self.debugging_handlers)

    async def _http_readonly(self, req):
        """--read-only-port: no authentication, GET only, no debugging handlers."""
        if req.method not in ("GET", "HEAD"):
            return Response(405, b"method not allowed", "text/plain")
        return await self._serve(req, False)

    async def _http_healthz(self, req):
        if req.path in ("/healthz", "/healthz/ping"):
            return Response(200, b"ok", "text/plain")
        return Response(404, b"not found", "text/plain")

    async def _serve(self, req, debugging):
        p = req.path
        if not debugging and p.startswith(self.DEBUG_PATHS):
            return Response(404, b"not found", "text/plain")
        if p in ("/healthz", "/healthz/ping"):
            return Response(200, b"ok", "text/plain")
        if p == "/healthz/syncloop":
            age = time.monotonic() - self._last_status_loop
            limit = max(60.0, 3 * self.status_freq)
            return (Response(200, b"ok", "text/plain") if age < limit else
                    Response(500, f"sync loop has not run for {age:.0f}s".encode(), "text/plain"))
        if p == "/spec" or p == "/spec/":
            from .stats import machine_info
            return Response(200, codec_dumpb(machine_info(self)))
        if p == "/configz":
            return Response(200, codec_dumpb({"kubeletconfig": self.current_config()}))
        if p.rstrip("/") == "/runningpods":
            return Response(200, codec_dumpb(self.running_pods()))
        if p == "/logs" or p.startswith("/logs/"):
            return self._node_logs(p[len("/logs"):].lstrip("/"))
        if p == "/metrics":
            return Response(200, self.metrics.render(), "text/plain; version=0.0.4")
        from ..api import codec
        if p == "/pods":
            return Response(200, codec.dumpb({"kind": "PodList", "apiVersion": "v1",
                                              "items": [s.pod for s in self.pods.values()]}))
        if p.startswith("/containerLogs/"):
            parts = p.split("/")
            if len(parts) >= 5:
                ns, name, cname = parts[2], parts[3], parts[4]
                uid = self.by_key.get(f"{ns}/{name}")
                st = self.pods.get(uid) if uid else None
                if st is None:
                    return Response(404, b"pod not found", "text/plain")
                if not cname:
                    cname = ((st.pod.get("spec") or {}).get("containers") or [{}])[0].get("name", "")
                if req.query.get("previous") in ("true", "1"):
                    cid = st.previous.get(cname)
                    if cid is None:
                        return Response(400, f'previous terminated container "{cname}" in pod "{name}" not found'.encode(),
                                        "text/plain")
                else:
                    cid = st.containers.get(cname) or st.init_containers.get(cname)
                if cid is None:
                    return Response(404, b"container not found", "text/plain")
                tail = int(req.query["tailLines"]) if "tailLines" in req.query else None
                return await self._container_logs(cid, tail, req.query)
        if p == "/stats/summary":
            from .stats import summary
            return Response(200, codec.dumpb(summary(self)))
        if p.startswith("/debug/pprof"):
            from ..utils.profiling import handle_debug
            return await handle_debug(req)
        from . import server_streaming
        r = await server_streaming.handle(self, req)
        if r is not None:
            return r
        return Response(404, b"not found", "text/plain")


def codec_dumpb(obj):
    from ..api import codec
    return codec.dumpb(obj)


def md_deleting(pod):
    return bool(pod["metadata"].get("deletionTimestamp"))


def _key(pod):
    return f"{pod['metadata'].get('namespace', '')}/{pod['metadata']['name']}"


def _ts(t):
    return now_rfc3339(t) if t else None


DEFAULT_NODE_LABELS = ("kubernetes.io/hostname", "failure-domain.beta.kubernetes.io/zone",
                       "failure-domain.beta.kubernetes.io/region", "beta.kubernetes.io/instance-type",
                       "beta.kubernetes.io/os", "beta.kubernetes.io/arch")


def update_default_labels(initial, existing) -> bool:
    """`Kubelet.updateDefaultLabels` (kubelet_node_status.go:159): each default label the kubelet
    has an opinion on is copied onto the existing node (an empty value deletes it); other labels
    stay. Returns whether the existing node changed."""
    want = (initial.get("metadata") or {}).get("labels") or {}
    have = existing["metadata"].setdefault("labels", {})
    changed = False
    for k in DEFAULT_NODE_LABELS:
        if k not in want:
            continue
        if have.get(k, "") != want[k]:
            have[k] = want[k]
            changed = True
        if have.get(k, "") == "":
            have.pop(k, None)
    return changed


def reconcile_cmad_annotation(node, existing) -> bool:
    """`reconcileCMADAnnotationWithExistingNode`: the controller-managed attach-detach annotation
    of the existing node follows the one just built (removed when the kubelet does not set it)."""
    new = (node.get("metadata") or {}).get("annotations") or {}
    have = existing["metadata"].setdefault("annotations", {})
    if new.get(CONTROLLER_MANAGED_ATTACH, "") == have.get(CONTROLLER_MANAGED_ATTACH, ""):
        return False
    if CONTROLLER_MANAGED_ATTACH in new:
        have[CONTROLLER_MANAGED_ATTACH] = new[CONTROLLER_MANAGED_ATTACH]
    else:
        have.pop(CONTROLLER_MANAGED_ATTACH, None)
    return True


def containers_to_evict(containers, policy, now, is_deleted, is_terminated, evict_terminated=False,
                        all_sources_ready=True):
    """`containerGC.evictContainers` (pkg/kubelet/kuberuntime/kuberuntime_gc.go) as a pure
    selection. `containers`: (id, pod uid, container name, createdAt, state). Non-running
    containers created at least `min_age` ago form evict units per (pod, container), newest
    first. Units of deleted pods (and of terminated ones with `evict_terminated`) go entirely;
    then each unit keeps `max_per_pod_container` (if >= 0); then, over `max_containers` (if >=
    0), every unit is cut to max(1, max_containers // units) and, still over, the oldest
    containers across units go. Returns the ids to remove, in removal order."""
    min_age = float(policy.get("min_age", 0.0))
    per = int(policy.get("max_per_pod_container", 1))
    total = int(policy.get("max_containers", -1))
    units: dict = {}
    for cid, uid, name, created, state in containers:
        if state == RUNNING or created > now - min_age:
            continue
        units.setdefault((uid, name) if uid else ("", cid), []).append((created, cid))
    for lst in units.values():
        lst.sort(key=lambda e: e[0], reverse=True)
    out = []

    def remove_oldest(lst, n):
        if n <= 0:
            return lst
        keep = len(lst) - n
        out.extend(cid for _, cid in reversed(lst[keep:]))
        return lst[:keep]

    if all_sources_ready:
        for key in list(units):
            uid = key[0]
            if is_deleted(uid) or (evict_terminated and is_terminated(uid)):
                lst = units.pop(key)
                remove_oldest(lst, len(lst))
    if per >= 0:
        for key in units:
            units[key] = remove_oldest(units[key], len(units[key]) - per)
    n = sum(len(v) for v in units.values())
    if total >= 0 and n > total:
        each = max(1, total // len(units)) if units else 1
        for key in units:
            units[key] = remove_oldest(units[key], len(units[key]) - each)
        flat = sorted((e for v in units.values() for e in v), key=lambda e: e[0], reverse=True)
        remove_oldest(flat, len(flat) - total)
    return out


def expand_container_command_and_args(container, envs):
    """`kubecontainer.ExpandContainerCommandAndArgs` (helpers.go:130): every command and args
    entry through `expand` with the container's resolved environment (`EnvVarsToMap`: a later
    variable of the same name wins). Returns (command, args), each None when the container has
    none."""
    m = {}
    for e in envs:
        m[e["name"]] = str(e.get("value", ""))
    cmd = [expand(str(x), m) for x in container.get("command") or ()] or None
    args = [expand(str(x), m) for x in container.get("args") or ()] or None
    return cmd, args


def _host_ports(spec):
    """(hostIP, protocol, hostPort) of every container port with a hostPort."""
    out = []
    for c in spec.get("containers") or ():
        for p in c.get("ports") or ():
            if p.get("hostPort"):
                out.append((p.get("hostIP") or "0.0.0.0", p.get("protocol") or "TCP", int(p["hostPort"])))
    return out


def _node_affinity_required(spec):
    aff = (spec.get("affinity") or {}).get("nodeAffinity") or {}
    req = aff.get("requiredDuringSchedulingIgnoredDuringExecution")
    return None if req is None else (req.get("nodeSelectorTerms") or [])


def _node_affinity_matches(terms, labels, node_name):
    """`nodeMatchesNodeSelectorTerms`: any term whose expressions (and metadata.name fields)
    all match; a term with neither matches nothing."""
    from ..api.labels import SelectorError, node_selector_requirements_as_selector
    for t in terms:
        exprs, fields = t.get("matchExpressions") or [], t.get("matchFields") or []
        if not exprs and not fields:
            continue
        try:
            if exprs and not node_selector_requirements_as_selector(exprs).matches(labels):
                continue
        except SelectorError:
            continue
        if any(f.get("key") == "metadata.name" and (
                (f.get("operator") == "In" and node_name not in (f.get("values") or [])) or
                (f.get("operator") == "NotIn" and node_name in (f.get("values") or []))) for f in fields):
            continue
        return True
    return False


def should_container_be_restarted(policy, status) -> bool:
    """`kubecontainer.ShouldContainerBeRestarted` (pkg/kubelet/container/helpers.go:58) over the
    latest instance's status (an object with `.state` / `.exit_code`, or None): never started ->
    start; running -> no; unknown or created-but-not-started -> always; dead -> by restartPolicy
    (Never: no, OnFailure: only a non-zero exit, Always: yes)."""
    if status is None:
        return True
    if status.state == RUNNING:
        return False
    if status.state in (UNKNOWN, CREATED):
        return True
    if policy == "Never":
        return False
    if policy == "OnFailure" and status.exit_code == 0:
        return False
    return True


def get_phase(spec, statuses, init_statuses=()):
    """`kubelet_pods.go` GetPhase over v1 container statuses: a failed init container fails a
    Never pod; initialization in progress or a waiting container (one with no previous
    termination) keeps it Pending; running containers with none unknown -> Running; all stopped
    (a waiting container with a last termination counts as stopped) -> Running for Always,
    Succeeded when every one exited 0, Failed for Never, else Running (OnFailure restarts)."""
    by_name = {s["name"]: s for s in statuses or ()}
    init_by_name = {s["name"]: s for s in init_statuses or ()}
    pending_init = failed_init = 0
    for c in spec.get("initContainers") or ():
        s = init_by_name.get(c["name"])
        st = (s or {}).get("state") or {}
        last = ((s or {}).get("lastState") or {}).get("terminated")
        if s is None or "running" in st:
            pending_init += 1
        elif "terminated" in st:
            if st["terminated"].get("exitCode", 0) != 0:
                failed_init += 1
        elif "waiting" in st and last is not None:
            if last.get("exitCode", 0) != 0:
                failed_init += 1
        else:
            pending_init += 1
    unknown = running = waiting = stopped = succeeded = 0
    for c in spec.get("containers") or ():
        s = by_name.get(c["name"])
        st = (s or {}).get("state") or {}
        if s is None or not st:
            unknown += 1
        elif "running" in st:
            running += 1
        elif "terminated" in st:
            stopped += 1
            if st["terminated"].get("exitCode", 0) == 0:
                succeeded += 1
        elif "waiting" in st:
            if ((s.get("lastState") or {}).get("terminated")) is not None:
                stopped += 1
            else:
                waiting += 1
        else:
            unknown += 1
    policy = spec.get("restartPolicy", "Always")
    if failed_init and policy == "Never":
        return core.POD_FAILED
    if pending_init or waiting:
        return core.POD_PENDING
    if running and not unknown:
        return core.POD_RUNNING
    if not running and stopped and not unknown:
        if policy == "Always":
            return core.POD_RUNNING
        if stopped == succeeded:
            return core.POD_SUCCEEDED
        if policy == "Never":
            return core.POD_FAILED
        return core.POD_RUNNING
    return core.POD_PENDING


def _last_state(pcs):
    """lastState.terminated from the previous (dead) instance of a restarted container."""
    if pcs is None or pcs.state != EXITED:
        return None
    return {"terminated": {"exitCode": pcs.exit_code, "reason": pcs.reason or ("Completed" if pcs.exit_code == 0
                                                                               else "Error"),
                           "startedAt": _ts(pcs.started_at), "finishedAt": _ts(pcs.finished_at),
                           "containerID": pcs.id}}


def _container_status(c, cs, restarts, waiting=None, pcs=None):
    s = _container_status_now(c, cs, restarts, waiting)
    if "lastState" not in s:
        last = _last_state(pcs)
        if last is not None:
            s["lastState"] = last
        elif cs is None and restarts > 0:
            # between a restart's kill and the new container: the previous instance is gone from
            # the runtime, but the container did terminate (keeps the pod from flapping to Pending)
            s["lastState"] = {"terminated": {"exitCode": 0, "reason": "Unknown"}}
    return s


def _container_status_now(c, cs, restarts, waiting=None):
    s = {"name": c["name"], "image": c.get("image", ""), "imageID": "", "restartCount": restarts, "ready": False}
    if cs is not None and waiting and waiting[0] == "CrashLoopBackOff" and cs.state == EXITED:
        s["containerID"] = cs.id
        s["state"] = {"waiting": {"reason": waiting[0], "message": waiting[1]}}
        s["lastState"] = {"terminated": {"exitCode": cs.exit_code, "reason": cs.reason or "Error",
                                         "startedAt": _ts(cs.started_at), "finishedAt": _ts(cs.finished_at),
                                         "containerID": cs.id}}
        return s
    if cs is None:
        if waiting:
            s["state"] = {"waiting": {"reason": waiting[0], "message": waiting[1]}}
        else:
            s["state"] = {"waiting": {"reason": "ContainerCreating"}}
        return s
    s["containerID"] = cs.id
    if cs.state == RUNNING:
        s["state"] = {"running": {"startedAt": _ts(cs.started_at)}}
        s["ready"] = True
    elif cs.state == EXITED:
        s["state"] = {"terminated": {"exitCode": cs.exit_code, "reason": cs.reason or ("Completed" if cs.exit_code == 0 else "Error"),
                                     "startedAt": _ts(cs.started_at), "finishedAt": _ts(cs.finished_at),
                                     "containerID": cs.id}}
        msg = cs.message
        if not msg and cs.exit_code and c.get("terminationMessagePolicy") == "FallbackToLogsOnError":
            msg = _log_tail(getattr(cs, "log_path", ""))
        if msg:
            s["state"]["terminated"]["message"] = msg
    else:
        s["state"] = {"waiting": {"reason": "ContainerCreating"}}
    return s


def _apply_security_context(pod, c, opts, image_user=None):
    """`pkg/kubelet/kuberuntime/security_context.go`: the container's securityContext overrides the
    pod's. runAsUser / runAsGroup become the process identity; the pod's fsGroup and
    supplementalGroups are supplemental groups (security_context.go:58-66), never the primary
    group; privileged, capabilities and readOnlyRootFilesystem go to the runtime; runAsNonRoot is
    verified (`verifyRunAsNonRoot`). Returns an error string."""
    psc = (pod.get("spec") or {}).get("securityContext") or {}
    csc = c.get("securityContext") or {}
    uid = csc.get("runAsUser", psc.get("runAsUser"))
    gid = csc.get("runAsGroup", psc.get("runAsGroup"))
    non_root = csc.get("runAsNonRoot", psc.get("runAsNonRoot"))
    if uid is not None:
        opts.run_as_user = int(uid)
    if gid is not None:
        opts.run_as_group = int(gid)
    groups = [int(g) for g in psc.get("supplementalGroups") or ()]
    if psc.get("fsGroup") is not None and int(psc["fsGroup"]) not in groups:
        groups.append(int(psc["fsGroup"]))
    opts.supplemental_groups = groups
    opts.privileged = bool(csc.get("privileged"))
    caps = csc.get("capabilities") or {}
    opts.cap_add = list(caps.get("add") or ())
    opts.cap_drop = list(caps.get("drop") or ())
    opts.readonly_rootfs = bool(csc.get("readOnlyRootFilesystem"))
    if image_user is None:
        # no image metadata: the entrypoint inherits the runtime's identity
        image_user = (os.geteuid(), "")
    return verify_run_as_non_root(non_root, uid, *image_user)


def image_user(config) -> tuple:
    """`getImageUser`: (uid, username) from an image config's User ("uid", "uid:gid" or a name);
    (None, "") when the image sets none, which runs as root (uid 0)."""
    user = str((config or {}).get("User") or "").split(":", 1)[0]
    if not user:
        return 0, ""
    try:
        return int(user), ""
    except ValueError:
        return None, user


def verify_run_as_non_root(run_as_non_root, run_as_user, image_uid, image_username="") -> str:
    """`verifyRunAsNonRoot` (kuberuntime/security_context.go:78) over the effective security
    context: "" when allowed, else the error."""
    if not run_as_non_root:
        return ""
    if run_as_user is not None:
        return "container's runAsUser breaks non-root policy" if int(run_as_user) == 0 else ""
    if image_uid is not None and int(image_uid) == 0:
        return "container has runAsNonRoot and image will run as root"
    if image_uid is None and image_username:
        return (f"container has runAsNonRoot and image has non-numeric user ({image_username}), cannot verify user "
                f"is non-root")
    return ""


def _log_tail(path, max_bytes=2048, max_lines=80):
    """`kuberuntime_container.go` FallbackToLogsOnError: the last 80 lines / 2 KiB of the log of a
    container that failed without writing a termination message."""
    if not path:
        return ""
    try:
        with open(path, "rb") as f:
            f.seek(0, os.SEEK_END)
            size = f.tell()
            f.seek(max(0, size - max_bytes))
            data = f.read()
    except OSError:
        return ""
    return "\n".join(data.decode(errors="replace").splitlines()[-max_lines:])
