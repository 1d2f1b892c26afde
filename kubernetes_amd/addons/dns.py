"""Cluster DNS add-on (the kube-dns / `cluster/addons/dns` equivalent).

Serves the Kubernetes DNS schema from API informers, over UDP and TCP:
  * `<svc>.<ns>.svc.<domain>` A → the service's clusterIP, or for a headless service the ready
    endpoint addresses; ExternalName services answer a CNAME;
  * `<hostname>.<svc>.<ns>.svc.<domain>` A for named endpoints of headless services
    (StatefulSet pods);
  * `_<port>._<proto>.<svc>.<ns>.svc.<domain>` SRV (+ additional A records);
  * `<a-b-c-d>.<ns>.pod.<domain>` A;
  * `<d>.<c>.<b>.<a>.in-addr.arpa` PTR for service cluster IPs and named endpoints;
  * anything outside the cluster domain is forwarded to the upstream resolvers (kube-dns's
    dnsmasq stage) — no upstream configured → REFUSED.
Parity: the record schema of kube-dns `pkg/dns/dns.go` (skydns tree), TTL 30 s, NXDOMAIN for
unknown names inside the domain. The DNS wire format (RFC 1035, compression pointers on read)
is implemented here directly.
"""
from __future__ import annotations

import asyncio
import ipaddress
import logging
import struct

log = logging.getLogger("dns")

A, NS, CNAME, SOA, PTR, TXT, AAAA, SRV, ANY = 1, 2, 5, 6, 12, 16, 28, 33, 255
NOERROR, FORMERR, SERVFAIL, NXDOMAIN, NOTIMP, REFUSED = 0, 1, 2, 3, 4, 5
TTL = 30


# ------------------------------------------------------------------------------------ wire format
def _read_name(buf, off):
    labels, jumped, end = [], False, None
    for _ in range(128):
        ln = buf[off]
        if ln == 0:
            off += 1
            break
        if ln & 0xC0 == 0xC0:
            ptr = struct.unpack_from("!H", buf, off)[0] & 0x3FFF
            if not jumped:
                end = off + 2
            jumped, off = True, ptr
            continue
        labels.append(buf[off + 1:off + 1 + ln].decode("ascii", "replace"))
        off += 1 + ln
    return ".".join(labels).lower(), (end if jumped else off)


def _name(n):
    out = b""
    for lab in n.strip(".").split("."):
        if lab:
            b = lab.encode()
            out += bytes([len(b)]) + b
    return out + b"\x00"


def parse_query(data):
    qid, flags, qd, an, ns, ar = struct.unpack_from("!6H", data, 0)
    off, qs = 12, []
    for _ in range(qd):
        name, off = _read_name(data, off)
        qtype, qclass = struct.unpack_from("!HH", data, off)
        off += 4
        qs.append((name, qtype, qclass))
    return qid, flags, qs


def _rr(name, typ, rdata, ttl=TTL):
    return _name(name) + struct.pack("!HHIH", typ, 1, ttl, len(rdata)) + rdata


def rdata_for(typ, value):
    if typ == A:
        return ipaddress.IPv4Address(value).packed
    if typ in (CNAME, PTR, NS):
        return _name(value)
    if typ == SRV:
        prio, weight, port, target = value
        return struct.pack("!HHH", prio, weight, port) + _name(target)
    if typ == TXT:
        b = value.encode()
        return bytes([len(b)]) + b
    if typ == SOA:
        mname, rname, serial = value
        return _name(mname) + _name(rname) + struct.pack("!IIIII", serial, 28800, 7200, 604800, TTL)
    raise ValueError(typ)


def build_response(qid, flags, q, rcode, answers=(), additional=(), authority=()):
    rd = flags & 0x0100
    hdr = struct.pack("!6H", qid, 0x8000 | 0x0400 | rd | 0x0080 | rcode, 1 if q else 0, len(answers), len(authority),
                      len(additional))
    body = (_name(q[0]) + struct.pack("!HH", q[1], q[2])) if q else b""
    for lst in (answers, authority, additional):
        for name, typ, val in lst:
            body += _rr(name, typ, rdata_for(typ, val))
    return hdr + body


def build_query(qid, name, qtype):
    return struct.pack("!6H", qid, 0x0100, 1, 0, 0, 0) + _name(name) + struct.pack("!HH", qtype, 1)


def parse_answers(data):
    """(rcode, [(name, type, value)]) of a response: A/CNAME/PTR/SRV decoded."""
    qid, flags, qd, an, ns, ar = struct.unpack_from("!6H", data, 0)
    off = 12
    for _ in range(qd):
        _, off = _read_name(data, off)
        off += 4
    out = []
    for _ in range(an + ns + ar):
        name, off = _read_name(data, off)
        typ, _cls, _ttl, ln = struct.unpack_from("!HHIH", data, off)
        off += 10
        rdata_off = off
        if typ == A:
            val = str(ipaddress.IPv4Address(data[off:off + 4]))
        elif typ in (CNAME, PTR, NS):
            val, _ = _read_name(data, off)
        elif typ == SRV:
            p, w, port = struct.unpack_from("!HHH", data, off)
            tgt, _ = _read_name(data, off + 6)
            val = (p, w, port, tgt)
        else:
            val = data[off:off + ln]
        out.append((name, typ, val))
        off = rdata_off + ln
    return flags & 0xF, out


# ------------------------------------------------------------------------------------ records
class Records:
    """Name → records view over the services / endpoints informers."""

    def __init__(self, domain="cluster.local"):
        self.domain = domain.strip(".").lower()
        self.services: dict[str, dict] = {}
        self.endpoints: dict[str, dict] = {}

    def _svc_fqdn(self, ns, name):
        return f"{name}.{ns}.svc.{self.domain}"

    def _ep_addrs(self, ns, name):
        ep = self.endpoints.get(f"{ns}/{name}") or {}
        for sub in ep.get("subsets") or ():
            for a in sub.get("addresses") or ():
                yield a, sub.get("ports") or []

    def _ep_name(self, a):
        if a.get("hostname"):
            return a["hostname"]
        return "-".join(a["ip"].split("."))     # kube-dns hashes; dashed IP keeps names readable and stable

    def lookup(self, qname, qtype):
        """(rcode, answers, additional)."""
        qname = qname.strip(".").lower()
        if qname.endswith(".in-addr.arpa"):
            return self._ptr(qname, qtype)
        if qname != self.domain and not qname.endswith("." + self.domain):
            return None
        rel = qname[:-len(self.domain)].rstrip(".")
        parts = rel.split(".") if rel else []
        if len(parts) >= 2 and parts[-1] == "pod" and len(parts) == 3:
            ip = parts[0].replace("-", ".")
            try:
                ipaddress.IPv4Address(ip)
            except ValueError:
                return NXDOMAIN, [], []
            return NOERROR, ([(qname, A, ip)] if qtype in (A, ANY) else []), []
        if len(parts) < 3 or parts[-1] != "svc":
            return (NOERROR if self._is_prefix(parts) else NXDOMAIN), [], []
        ns, name = parts[-2], parts[-3]
        svc = self.services.get(f"{ns}/{name}")
        lead = parts[:-3]
        if svc is None:
            return NXDOMAIN, [], []
        spec = svc.get("spec") or {}
        if not lead:
            if spec.get("type") == "ExternalName":
                return NOERROR, [(qname, CNAME, spec.get("externalName", ""))], []
            if qtype not in (A, ANY, SRV):
                return NOERROR, [], []
            if qtype == SRV:
                return self._srv(qname, svc, None, None)
            ip = spec.get("clusterIP")
            if ip and ip != "None":
                return NOERROR, [(qname, A, ip)], []
            return NOERROR, [(qname, A, a["ip"]) for a, _ in self._ep_addrs(ns, name)], []
        if len(lead) == 2 and lead[0].startswith("_") and lead[1].startswith("_"):
            return self._srv(qname, svc, lead[0][1:], lead[1][1:])
        if len(lead) == 1:
            for a, _ in self._ep_addrs(ns, name):
                if self._ep_name(a) == lead[0]:
                    return NOERROR, ([(qname, A, a["ip"])] if qtype in (A, ANY) else []), []
        return NXDOMAIN, [], []

    def _is_prefix(self, parts):
        if not parts:
            return True
        if parts[-1] in ("svc", "pod"):
            if len(parts) == 1:
                return True
            if len(parts) == 2:
                return any(k.split("/")[0] == parts[0] for k in self.services)
        return False

    def _srv(self, qname, svc, port_name, proto):
        md = svc["metadata"]
        ns, name = md["namespace"], md["name"]
        spec = svc.get("spec") or {}
        headless = spec.get("clusterIP") in (None, "", "None")
        ans, add = [], []
        for p in spec.get("ports") or ():
            if port_name is not None and (p.get("name") or "") != port_name:
                continue
            if proto is not None and p.get("protocol", "TCP").lower() != proto:
                continue
            if headless:
                for a, eports in self._ep_addrs(ns, name):
                    tgt = f"{self._ep_name(a)}.{self._svc_fqdn(ns, name)}"
                    port = next((e.get("port") for e in eports if e.get("name", "") == p.get("name", "")), p.get("port"))
                    ans.append((qname, SRV, (10, 100, int(port), tgt)))
                    add.append((tgt, A, a["ip"]))
            else:
                tgt = self._svc_fqdn(ns, name)
                ans.append((qname, SRV, (10, 100, int(p["port"]), tgt)))
                add.append((tgt, A, spec["clusterIP"]))
        return (NOERROR if ans else NXDOMAIN), ans, add

    def _ptr(self, qname, qtype):
        octets = qname[:-len(".in-addr.arpa")].split(".")
        if len(octets) != 4:
            return None
        ip = ".".join(reversed(octets))
        for k, svc in self.services.items():
            if (svc.get("spec") or {}).get("clusterIP") == ip:
                ns, name = k.split("/")
                return NOERROR, [(qname, PTR, self._svc_fqdn(ns, name))], []
        for k in self.endpoints:
            ns, name = k.split("/")
            for a, _ in self._ep_addrs(ns, name):
                if a["ip"] == ip and a.get("hostname"):
                    return NOERROR, [(qname, PTR, f"{a['hostname']}.{self._svc_fqdn(ns, name)}")], []
        return None


# ------------------------------------------------------------------------------------ server
class _UDP(asyncio.DatagramProtocol):
    def __init__(self, srv):
        self.srv = srv

    def connection_made(self, transport):
        self.transport = transport

    def datagram_received(self, data, addr):
        t = asyncio.ensure_future(self._reply(data, addr))
        self.srv._tasks.add(t)                     # strong ref until done
        t.add_done_callback(self.srv._tasks.discard)

    async def _reply(self, data, addr):
        try:
            resp = await self.srv.answer(data)
        except Exception:  # noqa: BLE001 - one bad query must not stop the server
            log.exception("dns query failed")
            return
        if resp:
            self.transport.sendto(resp, addr)


class DNSServer:
    def __init__(self, client=None, domain="cluster.local", upstreams=(), records=None):
        self.client = client
        self.records = records or Records(domain)
        self.upstreams = list(upstreams)
        self.udp = self.tcp = None
        self.port = None
        self._tasks = set()
        self._informers = []
        self.queries = 0

    async def start(self, host="127.0.0.1", port=0):
        if self.client is not None:
            from ..client.informer import Informer
            for res, store in (("services", self.records.services), ("endpoints", self.records.endpoints)):
                inf = Informer(self.client, res)

                def put(*objs, store=store):
                    o = objs[-1]
                    store[f"{o['metadata']['namespace']}/{o['metadata']['name']}"] = o

                def drop(o, store=store):
                    store.pop(f"{o['metadata']['namespace']}/{o['metadata']['name']}", None)
                inf.add_handler(put, put, drop)
                inf.start()
                self._informers.append(inf)
            for inf in self._informers:
                await inf.wait_synced(30)
        loop = asyncio.get_running_loop()
        self.tcp = await asyncio.start_server(self._tcp_conn, host, port)
        self.port = self.tcp.sockets[0].getsockname()[1]
        self.udp, _ = await loop.create_datagram_endpoint(lambda: _UDP(self), local_addr=(host, self.port))
        return self.port

    async def _tcp_conn(self, reader, writer):
        try:
            while True:
                hdr = await reader.readexactly(2)
                data = await reader.readexactly(struct.unpack("!H", hdr)[0])
                resp = await self.answer(data)
                writer.write(struct.pack("!H", len(resp)) + resp)
                await writer.drain()
        except (asyncio.IncompleteReadError, ConnectionError):
            pass
        finally:
            writer.close()

    async def answer(self, data):
        self.queries += 1
        try:
            qid, flags, qs = parse_query(data)
        except (struct.error, IndexError):
            return None
        if flags & 0x8000 or len(qs) != 1:
            return build_response(struct.unpack_from("!H", data)[0], flags, qs[0] if qs else None, FORMERR)
        q = qs[0]
        r = self.records.lookup(q[0], q[1])
        if r is None:
            return await self._forward(data, qid, flags, q)
        rcode, ans, add = r
        auth = []
        if not ans and rcode in (NOERROR, NXDOMAIN):
            d = self.records.domain
            auth = [(d, SOA, (f"ns.dns.{d}", f"hostmaster.{d}", 1))]
        return build_response(qid, flags, q, rcode, ans, add, auth)

    async def _forward(self, data, qid, flags, q):
        loop = asyncio.get_running_loop()
        for up in self.upstreams:
            host, _, port = up.partition(":")
            fut = loop.create_future()

            class P(asyncio.DatagramProtocol):
                def datagram_received(self, d, addr):
                    if not fut.done():
                        fut.set_result(d)

                def error_received(self, exc):
                    if not fut.done():
                        fut.set_exception(exc)
            tr, _ = await loop.create_datagram_endpoint(P, remote_addr=(host, int(port or 53)))
            try:
                tr.sendto(data)
                return await asyncio.wait_for(fut, 2.0)
            except (asyncio.TimeoutError, OSError):
                continue
            finally:
                tr.close()
        return build_response(qid, flags, q, REFUSED if not self.upstreams else SERVFAIL)

    async def stop(self):
        for inf in self._informers:
            inf.stop()
        if self.udp is not None:
            self.udp.close()
        if self.tcp is not None:
            self.tcp.close()
            await self.tcp.wait_closed()
        for t in list(self._tasks):
            t.cancel()


async def resolve(server, port, name, qtype=A, tcp=False, timeout=2.0):
    """Tiny stub resolver for tests and `kubectl` helpers: returns (rcode, records)."""
    q = build_query(0x4B38, name, qtype)
    loop = asyncio.get_running_loop()
    if tcp:
        r, w = await asyncio.open_connection(server, port)
        w.write(struct.pack("!H", len(q)) + q)
        await w.drain()
        n = struct.unpack("!H", await r.readexactly(2))[0]
        data = await r.readexactly(n)
        w.close()
        return parse_answers(data)
    fut = loop.create_future()

    class P(asyncio.DatagramProtocol):
        def datagram_received(self, d, addr):
            if not fut.done():
                fut.set_result(d)
    tr, _ = await loop.create_datagram_endpoint(P, remote_addr=(server, port))
    try:
        tr.sendto(q)
        return parse_answers(await asyncio.wait_for(fut, timeout))
    finally:
        tr.close()
