"""kubemark hollow nodes that advertise MI355X GPUs.

Parity: `cmd/kubemark/hollow-node.go:46-160` / `pkg/kubemark/hollow_kubelet.go:49-100` — a real
kubelet code path over a fake runtime. The reference's hollow kubelet uses the stub container
manager and therefore advertises NO devices (`pkg/kubelet/cm/container_manager_stub.go:73-75`);
here every hollow node runs the real DeviceManager and a real amd.com/gpu device plugin over
gRPC/unix sockets, backed by the fake AMD SMI fixture (8 x MI355X, one xGMI hive), so GPU
scheduling and admission are exercised at scale.
"""
from __future__ import annotations

import asyncio
import os
import shutil
import tempfile

from ..client.rest import Client
from ..deviceplugin.amdgpu import AMDGPUPlugin
from ..kubelet.devicemanager.manager import ManagerImpl
from ..kubelet.kubelet import Kubelet
from ..kubelet.runtime.stub import StubRuntime
from ..native import amdsmi


class HollowCluster:
    """A set of hollow nodes sharing one process / event loop / API client pool."""

    def __init__(self, master, count, prefix="hollow", gpus=8, hives=1, payload=None, workdir=None,
                 emit_events=False, status_freq=10.0, max_conns=32, partition="SPX", links_down=(),
                 content_type="application/vnd.kubernetes.protobuf"):
        self.master = master
        self.count = count
        self.prefix = prefix
        self.gpus = gpus
        self.hives = hives
        self.links_down = tuple(tuple(x) for x in links_down)
        self.partition = partition
        self.payload = payload
        self.own_dir = workdir is None
        self.dir = workdir or tempfile.mkdtemp(prefix=f"kamd-{prefix}-")
        self.emit_events = emit_events
        self.status_freq = status_freq
        self.client = Client(master, max_conns=max_conns, content_type=content_type)
        self.nodes = []
        self.plugins = []
        self.smi = None

    async def start(self):
        if self.gpus:
            self.smi = amdsmi.SMI(fixture=amdsmi.fixture_file(self.gpus, hives=self.hives, partition=self.partition,
                                                              links_down=self.links_down))
        for i in range(self.count):
            name = f"{self.prefix}-{i}"
            pdir = os.path.join(self.dir, name, "plugins")
            os.makedirs(pdir, exist_ok=True)
            dm = ManagerImpl(pdir)
            kl = Kubelet(self.client, name, StubRuntime(payload=self.payload), dm, emit_events=self.emit_events,
                         node_status_update_frequency=self.status_freq,
                         labels={"kubemark": "true", "kubemark.amd.com/host": self.prefix})
            kl.smi = self.smi
            await kl.run()
            self.nodes.append(kl)
            if self.gpus:
                p = AMDGPUPlugin(pdir, smi=self.smi, health_interval=0)
                await p.start()
                self.plugins.append(p)
        return self

    async def wait_registered(self, timeout=60):
        loop = asyncio.get_running_loop()
        end = loop.time() + timeout
        while loop.time() < end:
            if all(p.registered.is_set() for p in self.plugins):
                return
            await asyncio.sleep(0.02)
        raise TimeoutError("device plugins did not register")

    async def stop(self):
        for p in self.plugins:
            await p.stop()
        for k in self.nodes:
            await k.stop()
        await self.client.close()
        if self.own_dir:
            shutil.rmtree(self.dir, ignore_errors=True)
