"""In-process local cluster (the role of `hack/local-up-cluster.sh` and the integration-test
master of `test/integration/framework/master_utils.go`): API server + scheduler + N kubelets,
each with the amd.com/gpu device plugin (fake AMD SMI fixture, or the real one on a GPU box)
registering over the real gRPC/unix-socket path.
"""
from __future__ import annotations

import asyncio
import os
import shutil
import tempfile

from .apiserver.server import APIServer
from .client.rest import Client
from .deviceplugin.amdgpu import AMDGPUPlugin
from .kubelet.devicemanager.manager import ManagerImpl
from .kubelet.kubelet import Kubelet
from .kubelet.runtime.process import ProcessRuntime
from .kubelet.runtime.stub import StubRuntime
from .native import amdsmi
from .scheduler.scheduler import Scheduler


class NodeHandle:
    def __init__(self, name, kubelet, plugin, dm, runtime, plugins_dir):
        self.name, self.kubelet, self.plugin, self.dm, self.runtime, self.plugins_dir = (
            name, kubelet, plugin, dm, runtime, plugins_dir)


DNS_ADDR = "127.0.0.153"     # a loopback address of its own: the cluster DNS of LocalCluster(dns=True)


class LocalCluster:
    def __init__(self, nodes=1, gpus_per_node=8, runtime="stub", real_gpus=False, hives=1, workdir=None,
                 emit_events=True, payload=None, admission_plugins=None, scheduler_kwargs=None, kubelet_http=False,
                 health_interval=0.0, rocm_mount=None, controllers=None, controller_options=None, kubelet_kwargs=None,
                 partition="SPX", burn_in=None, dev_root="/dev", isolation=None, links_down=(), image_service=None,
                 dns=False):
        self.n_nodes = nodes
        self.gpus = gpus_per_node
        self.runtime_kind = runtime
        self.real = real_gpus
        self.hives = hives
        self.partition = partition             # fake backend: SPX/DPX/QPX/CPX compute partitions
        self.burn_in = burn_in                 # deviceplugin.burnin.BurnIn: gate GPUs on the HIP acceptance test
        self.dev_root = dev_root               # where the plugin finds /dev/kfd + /dev/dri (tests: mknod'd nodes)
        self.isolation = isolation             # process runtime: "auto" | "required" | "off"
        self.links_down = tuple(tuple(x) for x in links_down)   # fake backend: failed xGMI links
        # process runtime: node dir -> images.service.ImageService (OCI store + registry pulls)
        self.image_service = image_service
        self.own_dir = workdir is None
        self.dir = workdir or tempfile.mkdtemp(prefix="kamd-cluster-")
        self.emit_events = emit_events
        self.payload = payload
        self.admission = admission_plugins
        self.scheduler_kwargs = scheduler_kwargs or {}
        self.kubelet_http = kubelet_http
        self.health_interval = health_interval
        self.rocm_mount = rocm_mount
        self.api = None
        self.url = None
        self.client = None
        self.scheduler = None
        self.nodes: list[NodeHandle] = []
        self._sched_task = None
        self.smi = None
        self.controllers = controllers            # None = no controller manager; list/["*"] = enabled set
        self.controller_options = controller_options or {}
        self.kubelet_kwargs = kubelet_kwargs or {}
        self.cm = None
        # dns=True: the cluster DNS add-on on DNS_ADDR:53 (needs root to bind port 53; without
        # it no DNS runs) and every kubelet writes pods' resolv.conf for it (--cluster-dns)
        self.dns = dns
        self.dns_server = None

    async def start(self):
        self.api = APIServer(admission_plugins=self.admission)
        port = await self.api.start()
        self.url = f"http://127.0.0.1:{port}"
        self.client = Client(self.url)
        if self.gpus:
            fixture = None if self.real else amdsmi.fixture_file(self.gpus, hives=self.hives, partition=self.partition,
                                                                 links_down=self.links_down)
            self.smi = amdsmi.SMI(fixture=fixture)
        if self.dns and os.geteuid() == 0:
            from .addons.dns import DNSServer
            from .kubelet.network import DNSConfigurer
            self.dns_server = DNSServer(Client(self.url))
            await self.dns_server.start(DNS_ADDR, 53)
            self.kubelet_kwargs.setdefault("dns", DNSConfigurer(cluster_dns=[DNS_ADDR]))
            await self.client.create("services", {"metadata": {"name": "kube-dns", "namespace": "kube-system",
                                                               "labels": {"k8s-app": "kube-dns"}},
                                                  "spec": {"ports": [{"name": "dns", "port": 53, "protocol": "UDP"},
                                                                     {"name": "dns-tcp", "port": 53}]}},
                                     "kube-system")
        self.scheduler = Scheduler(Client(self.url), emit_events=self.emit_events, **self.scheduler_kwargs)
        self._sched_task = asyncio.ensure_future(self.scheduler.run())
        for i in range(self.n_nodes):
            await self.add_node(f"node-{i}" if not self.real else f"mi355x-{i}")
        await self.wait_nodes_ready()
        if self.controllers is not None:
            from .controllers.manager import ControllerManager
            self.cm = ControllerManager(Client(self.url), self.controllers, self.controller_options)
            await self.cm.start()
        return self

    async def add_node(self, name, runtime=None):
        ndir = os.path.join(self.dir, name)
        plugins_dir = os.path.join(ndir, "device-plugin", "plugins")
        os.makedirs(plugins_dir, exist_ok=True)
        dm = ManagerImpl(plugins_dir)
        if runtime is not None:
            rt = runtime
        elif self.runtime_kind == "process":
            rt = ProcessRuntime(os.path.join(ndir, "runtime"), isolation=self.isolation,
                                images=self.image_service(os.path.join(ndir, "images")) if self.image_service else None)
        else:
            rt = StubRuntime(payload=self.payload)
        kl = Kubelet(Client(self.url), name, rt, dm, emit_events=self.emit_events,
                     http_port=0 if self.kubelet_http else None, root_dir=ndir, **self.kubelet_kwargs)
        kl.smi = self.smi
        plugin = None
        await kl.run()
        if self.gpus:
            plugin = AMDGPUPlugin(plugins_dir, smi=self.smi, health_interval=self.health_interval,
                                  rocm_mount=self.rocm_mount, burn_in=self.burn_in, dev_root=self.dev_root)
            await plugin.start()
        h = NodeHandle(name, kl, plugin, dm, rt, plugins_dir)
        self.nodes.append(h)
        return h

    async def wait_nodes_ready(self, timeout=30):
        want = self.gpus
        loop = asyncio.get_running_loop()
        end = loop.time() + timeout
        while loop.time() < end:
            ok = 0
            for n in self.nodes:
                ni = self.scheduler.cache.nodes.get(n.name)
                if ni is not None and ni.node is not None and (not want or ni.gpu_total >= (len(n.plugin.gpus) if n.plugin else 0)):
                    ok += 1
            if ok == len(self.nodes):
                return
            await asyncio.sleep(0.02)
        raise TimeoutError("nodes not ready in the scheduler cache")

    async def wait_pod(self, name, ns="default", phase="Running", timeout=30):
        loop = asyncio.get_running_loop()
        end = loop.time() + timeout
        pod = None
        while loop.time() < end:
            try:
                pod = await self.client.get("pods", name, ns)
            except Exception:
                pod = None
            if pod is not None and (pod.get("status") or {}).get("phase") == phase:
                return pod
            await asyncio.sleep(0.02)
        raise TimeoutError(f"pod {ns}/{name} not {phase}: {pod and pod.get('status')}")

    async def wait_for(self, pred, timeout=30, interval=0.02):
        loop = asyncio.get_running_loop()
        end = loop.time() + timeout
        last = None
        while loop.time() < end:
            last = await pred()
            if last:
                return last
            await asyncio.sleep(interval)
        raise TimeoutError(f"condition not met (last={last!r})")

    async def stop(self):
        if self.cm is not None:
            await self.cm.stop()
        for n in self.nodes:
            if n.plugin:
                await n.plugin.stop()
            await n.kubelet.stop()
            if hasattr(n.runtime, "kill_all"):
                # the kubelet leaves containers running across its own restarts (adoption); a
                # torn-down cluster must not leave them behind
                await n.runtime.kill_all()
        if self.scheduler:
            await self.scheduler.stop()
        if self.dns_server is not None:
            await self.dns_server.stop()
        if self._sched_task:
            self._sched_task.cancel()
        if self.client:
            await self.client.close()
        if self.api:
            await self.api.stop()
        if self.own_dir:
            shutil.rmtree(self.dir, ignore_errors=True)

    async def __aenter__(self):
        return await self.start()

    async def __aexit__(self, *exc):
        await self.stop()
