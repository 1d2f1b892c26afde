"""Userspace proxier: an in-process TCP/UDP load balancer per service port.

Parity: `pkg/proxy/userspace/proxier.go` (one listening "proxy socket" per service port,
`OnServiceUpdate` opens/closes sockets, endpoint dial retries with `endpointDialTimeouts`
250 ms / 500 ms / 1 s / 2 s resetting session affinity on failure), `proxysocket.go`
(TCP: accept, dial, copy both ways; UDP: one upstream socket per client with an idle timeout,
`udpIdleTimeout` 250 ms refreshed by traffic) and `roundrobin.go` (`LoadBalancerRR`: round-robin
over the ready endpoints, ClientIP affinity with a TTL, affinity kept across endpoint updates for
endpoints that remain).

In the reference, iptables REDIRECT/DNAT rules steer `clusterIP:port` (the "portal") and node
ports into the proxy sockets. Here the proxy sockets carry the traffic directly: each service
port listens on `listen_ip:<proxy port>` (`portal(cluster_ip, port)` returns it) and, for
NodePort services, also on the node port itself — so the service is reachable for real.
"""
from __future__ import annotations

import asyncio
import logging
import time

from ..utils.tasks import spawn
from .config import ProxyState, ServicePortName

log = logging.getLogger("proxy.userspace")

DIAL_TIMEOUTS = (0.25, 0.5, 1.0, 2.0)
UDP_IDLE_TIMEOUT = 0.25


class NoEndpoints(Exception):
    pass


class LoadBalancerRR:
    def __init__(self, clock=time.monotonic):
        self.clock = clock
        self.services: dict = {}    # spn -> {"endpoints": [str], "index": int, "affinity": str, "ttl": s, "map": {}}

    def new_service(self, spn, affinity="None", ttl=10800):
        st = self.services.setdefault(spn, {"endpoints": [], "index": 0, "map": {}})
        st["affinity"], st["ttl"] = affinity, ttl

    def delete_service(self, spn):
        self.services.pop(spn, None)

    def has_endpoints(self, spn):
        st = self.services.get(spn)
        return bool(st and st["endpoints"])

    def next_endpoint(self, spn, src_ip=None, reset_affinity=False):
        st = self.services.get(spn)
        if not st or not st["endpoints"]:
            raise NoEndpoints(f"no endpoints available for service {spn}")
        sticky = st.get("affinity") == "ClientIP" and src_ip is not None
        now = self.clock()
        if sticky and not reset_affinity:
            a = st["map"].get(src_ip)
            if a is not None and now - a[1] < st["ttl"] and a[0] in st["endpoints"]:
                st["map"][src_ip] = (a[0], now)
                return a[0]
        ep = st["endpoints"][st["index"] % len(st["endpoints"])]
        st["index"] = (st["index"] + 1) % len(st["endpoints"])
        if sticky:
            st["map"][src_ip] = (ep, now)
        return ep

    def update_endpoints(self, spn, endpoints):
        st = self.services.setdefault(spn, {"endpoints": [], "index": 0, "map": {}, "affinity": "None", "ttl": 10800})
        if st["endpoints"] != endpoints:
            st["endpoints"] = list(endpoints)
            st["index"] = 0
            st["map"] = {ip: v for ip, v in st["map"].items() if v[0] in endpoints}

    def cleanup_sticky(self):
        now = self.clock()
        for st in self.services.values():
            st["map"] = {ip: v for ip, v in st["map"].items() if now - v[1] < st.get("ttl", 10800)}


class _UDPRelay(asyncio.DatagramProtocol):
    def __init__(self, proxier, spn, listen):
        self.proxier, self.spn, self.listen = proxier, spn, listen
        self.transport = None
        self.clients: dict = {}   # client addr -> (upstream transport, last activity)

    def connection_made(self, transport):
        self.transport = transport

    def datagram_received(self, data, addr):
        c = self.clients.get(addr)
        if c is not None:
            c[0].sendto(data)
            self.clients[addr] = (c[0], time.monotonic())
            return
        spawn(self._new_client(data, addr))

    async def _new_client(self, data, addr):
        loop = asyncio.get_running_loop()
        try:
            ep = self.proxier.lb.next_endpoint(self.spn, addr[0])
        except NoEndpoints:
            return
        host, port = ep.rsplit(":", 1)
        relay = self

        class Up(asyncio.DatagramProtocol):
            def datagram_received(self, d, _):
                relay.transport.sendto(d, addr)
                if addr in relay.clients:
                    relay.clients[addr] = (relay.clients[addr][0], time.monotonic())

        t, _ = await loop.create_datagram_endpoint(Up, remote_addr=(host, int(port)))
        self.clients[addr] = (t, time.monotonic())
        t.sendto(data)
        loop.call_later(self.proxier.udp_idle_timeout, self._expire, addr)

    def _expire(self, addr):
        c = self.clients.get(addr)
        if c is None:
            return
        idle = time.monotonic() - c[1]
        if idle >= self.proxier.udp_idle_timeout:
            c[0].close()
            self.clients.pop(addr, None)
        else:
            asyncio.get_running_loop().call_later(self.proxier.udp_idle_timeout - idle, self._expire, addr)

    def close(self):
        for t, _ in self.clients.values():
            t.close()
        self.clients.clear()
        if self.transport:
            self.transport.close()


class UserspaceProxier:
    def __init__(self, state: ProxyState, listen_ip="127.0.0.1", node_port_ip="0.0.0.0", open_node_ports=True,
                 udp_idle_timeout=UDP_IDLE_TIMEOUT):
        self.state = state
        self.listen_ip = listen_ip
        self.node_port_ip = node_port_ip
        self.open_node_ports = open_node_ports
        self.udp_idle_timeout = udp_idle_timeout
        self.lb = LoadBalancerRR()
        self.sockets: dict = {}      # spn -> {"info": ServiceInfo, "servers": [...], "port": int, "node_port": int}
        self.syncs = 0
        self.connections = 0
        self._lock = asyncio.Lock()

    def portal(self, cluster_ip, port, protocol="TCP"):
        """The local address serving `cluster_ip:port` (what the reference's portal rules redirect to)."""
        for spn, s in self.sockets.items():
            i = s["info"]
            if i.cluster_ip == cluster_ip and i.port == int(port) and i.protocol == protocol:
                return self.listen_ip, s["port"]
        return None

    def service_port(self, spn):
        s = self.sockets.get(spn)
        return None if s is None else s["port"]

    async def sync(self, force=False):
        async with self._lock:
            st = self.state
            for spn in list(self.sockets):
                info = st.services.get(spn)
                s = self.sockets[spn]
                if info is None or (info.cluster_ip, info.port, info.protocol, info.node_port) != \
                        (s["info"].cluster_ip, s["info"].port, s["info"].protocol, s["info"].node_port):
                    self._close(spn)
            for spn, info in st.services.items():
                self.lb.new_service(spn, info.session_affinity, info.sticky_seconds)
                self.lb.update_endpoints(spn, [e.endpoint for e in st.endpoints.get(spn) or ()])
                if spn not in self.sockets:
                    await self._open(spn, info)
                else:
                    self.sockets[spn]["info"] = info
            for spn in list(self.lb.services):
                if spn not in st.services:
                    self.lb.delete_service(spn)
            self.lb.cleanup_sticky()
            self.syncs += 1
        return True

    async def _open(self, spn: ServicePortName, info):
        loop = asyncio.get_running_loop()
        servers = []
        if info.protocol == "UDP":
            t, proto = await loop.create_datagram_endpoint(lambda: _UDPRelay(self, spn, None), local_addr=(self.listen_ip, 0))
            port = t.get_extra_info("sockname")[1]
            servers.append(proto)
            if info.node_port and self.open_node_ports:
                try:
                    _, p2 = await loop.create_datagram_endpoint(lambda: _UDPRelay(self, spn, None),
                                                                local_addr=(self.node_port_ip, info.node_port))
                    servers.append(p2)
                except OSError as e:
                    log.warning("can't open node port %d for %s: %s", info.node_port, spn, e)
        else:
            srv = await asyncio.start_server(lambda r, w: self._tcp(spn, r, w), self.listen_ip, 0)
            port = srv.sockets[0].getsockname()[1]
            servers.append(srv)
            if info.node_port and self.open_node_ports:
                try:
                    servers.append(await asyncio.start_server(lambda r, w: self._tcp(spn, r, w), self.node_port_ip,
                                                              info.node_port, reuse_address=True))
                except OSError as e:
                    log.warning("can't open node port %d for %s: %s", info.node_port, spn, e)
        self.sockets[spn] = {"info": info, "servers": servers, "port": port}

    def _close(self, spn):
        s = self.sockets.pop(spn, None)
        if s is None:
            return
        for srv in s["servers"]:
            srv.close()

    async def _dial(self, spn, src_ip):
        reset = False
        for timeout in DIAL_TIMEOUTS:
            ep = self.lb.next_endpoint(spn, src_ip, reset)
            host, port = ep.rsplit(":", 1)
            try:
                return await asyncio.wait_for(asyncio.open_connection(host, int(port)), timeout)
            except (OSError, asyncio.TimeoutError):
                reset = True   # the sticky endpoint failed: pick another one
        raise ConnectionError(f"failed to connect to an endpoint of {spn}")

    async def _tcp(self, spn, reader, writer):
        from ..cri.server import splice
        peer = writer.get_extra_info("peername") or ("", 0)
        try:
            ur, uw = await self._dial(spn, peer[0])
        except (NoEndpoints, ConnectionError) as e:
            log.debug("%s", e)
            writer.close()
            return
        self.connections += 1
        await splice(reader, writer, ur, uw)

    async def close(self):
        for spn in list(self.sockets):
            self._close(spn)
