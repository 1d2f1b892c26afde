"""ProxyServer: informers -> proxy state -> proxier sync loop, plus health checks and metrics.

Parity: `cmd/kube-proxy/app/server.go:424` (`ProxyServer.Run`: service/endpoints config
handlers, `SyncLoop`, healthz on `--healthz-bind-address` :10256, metrics :10249,
`--proxy-mode` iptables | ipvs | userspace), `pkg/proxy/healthcheck/healthcheck.go`
(per-service health-check node port for `externalTrafficPolicy: Local`: 200 with the local
endpoint count, 503 when there are none) and `healthcheck.HealthzServer` (200 while the last
successful sync is recent, 503 otherwise), metric
`kubeproxy_sync_proxy_rules_latency_microseconds` (`pkg/proxy/metrics`).
"""
from __future__ import annotations

import asyncio
import json
import logging
import time

from ..client.informer import InformerFactory, resync_period
from ..utils.httpserver import HTTPServer, Response
from ..utils.metrics import MICRO_BUCKETS, Registry
from ..utils.tasks import spawn
from .config import ProxyState

log = logging.getLogger("kube-proxy")


class ServiceHealthServer:
    """One listener per `healthCheckNodePort` of an `externalTrafficPolicy: Local` service."""

    def __init__(self, state: ProxyState, bind="127.0.0.1"):
        self.state = state
        self.bind = bind
        self.servers: dict[int, tuple] = {}   # port -> (HTTPServer, (ns, name))

    async def sync(self):
        want = {}
        for spn, info in self.state.services.items():
            if info.only_local and info.health_check_node_port:
                want[info.health_check_node_port] = (spn.namespace, spn.name)
        for port in list(self.servers):
            if port not in want:
                await self.servers.pop(port)[0].stop()
        for port, nsname in want.items():
            if port in self.servers:
                continue
            srv = HTTPServer(self._handler(nsname))
            try:
                await srv.start(self.bind, port)
            except OSError as e:
                log.warning("can't open health check port %d: %s", port, e)
                continue
            self.servers[port] = (srv, nsname)

    def local_endpoints(self, ns, name):
        return sum(1 for spn, eps in self.state.endpoints.items() if (spn.namespace, spn.name) == (ns, name)
                   for e in eps if e.is_local)

    def _handler(self, nsname):
        async def h(req):
            n = self.local_endpoints(*nsname)
            body = json.dumps({"service": {"namespace": nsname[0], "name": nsname[1]}, "localEndpoints": n}).encode()
            return Response(200 if n else 503, body)
        return h

    async def stop(self):
        for srv, _ in self.servers.values():
            await srv.stop()
        self.servers.clear()


class ProxyServer:
    def __init__(self, client, hostname, mode="iptables", cluster_cidr="", masquerade_all=False, sync_period=30.0,
                 min_sync_period=0.0, node_ips=("127.0.0.1",), healthz_port=None, metrics_port=None,
                 iptables=None, ipvs=None, ipvs_scheduler="rr", bind="127.0.0.1", open_node_ports=True,
                 masquerade_bit=14, resync=0.0, profiling=False):
        self.client = client
        self.hostname = hostname
        self.mode = mode
        self.state = ProxyState(hostname)
        if mode == "iptables":
            from .iptables import IptablesProxier
            self.proxier = IptablesProxier(self.state, iptables, cluster_cidr, masquerade_all, masquerade_bit=masquerade_bit,
                                           node_ips=node_ips, min_sync_period=min_sync_period)
        elif mode == "ipvs":
            from .ipvs import IPVSProxier
            self.proxier = IPVSProxier(self.state, ipvs, ipvs_scheduler, node_ips, min_sync_period)
        elif mode == "userspace":
            from .userspace import UserspaceProxier
            self.proxier = UserspaceProxier(self.state, bind, open_node_ports=open_node_ports)
        else:
            raise ValueError(f"unknown proxy mode {mode!r}")
        self.sync_period = sync_period
        self.min_sync_period = min_sync_period
        self.health = ServiceHealthServer(self.state, bind)
        self.healthz_port = healthz_port
        self.metrics_port = metrics_port
        self.bind = bind
        self.metrics = Registry()
        self.m_sync = self.metrics.histogram("kubeproxy_sync_proxy_rules_latency_microseconds",
                                             "SyncProxyRules latency", (), MICRO_BUCKETS)
        # --config-sync-period: the service/endpoints informers resync every [p, 2p)
        self.factory = InformerFactory(client, resync_period(resync))
        self.profiling = profiling
        self._dirty = asyncio.Event()
        self._task = None
        self._http = []
        self.last_sync = 0.0
        self.synced = asyncio.Event()

    async def start(self):
        self.state.attach(self.factory.get("services"), self.factory.get("endpoints"))
        self.state.listeners.append(self._dirty.set)
        self.factory.start()
        await self.factory.wait_for_cache_sync(60)
        for port, handler in ((self.healthz_port, self._healthz), (self.metrics_port, self._metrics)):
            if port is not None:
                srv = HTTPServer(handler)
                await srv.start(self.bind, port)
                self._http.append(srv)
        await self.sync()
        self._task = spawn(self._loop())
        return self

    async def sync(self):
        t0 = time.perf_counter()
        r = self.proxier.sync(force=True)
        if asyncio.iscoroutine(r):
            await r
        await self.health.sync()
        self.m_sync.observe((time.perf_counter() - t0) * 1e6)
        self.last_sync = time.time()
        self.synced.set()

    async def _loop(self):
        while True:
            try:
                await asyncio.wait_for(self._dirty.wait(), self.sync_period)
            except asyncio.TimeoutError:
                pass
            if self.min_sync_period:
                wait = self.min_sync_period - (time.time() - self.last_sync)
                if wait > 0:
                    await asyncio.sleep(wait)
            self._dirty.clear()
            try:
                await self.sync()
            except Exception:
                log.exception("proxy rules sync failed")

    async def wait_synced_with(self, pred, timeout=10.0):
        end = time.monotonic() + timeout
        while time.monotonic() < end:
            if pred():
                return True
            await asyncio.sleep(0.02)
        return False

    async def _healthz(self, req):
        now = time.time()
        ok = self.last_sync and now - self.last_sync <= 2 * max(self.sync_period, 1.0)
        body = json.dumps({"lastUpdated": self.last_sync, "currentTime": now}).encode()
        return Response(200 if ok else 503, body)

    async def _metrics(self, req):
        if req.path.startswith("/debug/pprof") and self.profiling:     # --profiling
            from ..utils.profiling import handle_debug
            return await handle_debug(req)
        return Response(200, self.metrics.render(), "text/plain; version=0.0.4")

    async def stop(self):
        if self._task is not None:
            self._task.cancel()
        self.factory.stop()
        await self.health.stop()
        for s in self._http:
            await s.stop()
        close = getattr(self.proxier, "close", None)
        if close is not None:
            await close()
