"""Exec / attach / port-forward sessions over the Kubernetes WebSocket channel protocols, shared by
the kubelet server, the CRI streaming server and (as an upgrade-aware proxy) the API server.

Parity:
  * options from the query — `input`, `output`, `error`, `tty` = "1", at least one stream,
    stderr dropped under a tty (`pkg/kubelet/server/remotecommand/httpstream.go:49-74`);
  * channels 0 stdin, 1 stdout, 2 stderr, 3 error/status, 4 resize (JSON `{"Width","Height"}`);
    an empty message on the lowest writable channel once the streams are up
    (`remotecommand/websocket.go:44-113`);
  * exit status: v4 protocols write a metav1.Status JSON on channel 3 — Success, or Failure with
    reason NonZeroExitCode and cause ExitCode=<rc>; older protocols write only a failure
    message (`remotecommand/exec.go:50-78`, `httpstream.go:426-447`);
  * port-forward: query `ports` (comma lists, repeatable), a data + error channel pair per port,
    each opened by the port as uint16 little-endian (`pkg/kubelet/server/portforward/websocket.go`);
  * `UpgradeAwareHandler`: the API server and a CRI-backed kubelet relay the client's upgrade
    request to the next hop and splice the raw connection (`apimachinery/pkg/util/proxy`).

Extension beyond 1.9: `v5.channel.k8s.io` (later Kubernetes) adds channel 255 = "close channel
<n>", which is how a client signals stdin EOF without closing the socket; v4 clients end stdin
by closing the connection.
"""
from __future__ import annotations

import asyncio
import json
import logging
from urllib.parse import parse_qs, urlsplit

from ..utils.httpserver import Response, UpgradeResponse
from ..utils.websocket import (BASE64_CHANNEL, CHANNEL, V4_BASE64_CHANNEL, V4_CHANNEL, ChannelConn, WebSocket,
                               handshake_headers, is_websocket_request, negotiate)

log = logging.getLogger("remotecommand")

V5_CHANNEL = "v5.channel.k8s.io"
EXEC_PROTOCOLS = ("", CHANNEL, BASE64_CHANNEL, V4_CHANNEL, V4_BASE64_CHANNEL, V5_CHANNEL)
PORTFORWARD_PROTOCOLS = ("", V4_CHANNEL, V4_BASE64_CHANNEL)
STDIN, STDOUT, STDERR, ERROR, RESIZE, CLOSE = 0, 1, 2, 3, 4, 255


class Options:
    __slots__ = ("stdin", "stdout", "stderr", "tty")

    def __init__(self, stdin=False, stdout=True, stderr=True, tty=False):
        self.stdin, self.stdout, self.stderr, self.tty = stdin, stdout, stderr and not tty, tty


def options_from_query(qs: str) -> Options:
    q = parse_qs(qs or "", keep_blank_values=True)
    flag = lambda k: (q.get(k) or [""])[-1] in ("1", "true")     # noqa: E731
    o = Options(flag("input") or flag("stdin"), flag("output") or flag("stdout"),
                flag("error") or flag("stderr"), flag("tty"))
    if not (o.stdin or o.stdout or o.stderr):
        raise ValueError("you must specify at least 1 of stdin, stdout, stderr")
    return o


def ports_from_query(qs: str) -> list[int]:
    q = parse_qs(qs or "", keep_blank_values=True)
    vals = (q.get("ports") or []) + (q.get("port") or [])
    if not vals:
        raise ValueError('query parameter "port" is required')
    out = []
    for v in vals:
        if not v:
            raise ValueError('query parameter "port" cannot be empty')
        for p in v.split(","):
            try:
                n = int(p)
            except ValueError:
                raise ValueError(f'unable to parse "{v}" as a port') from None
            if not 0 < n < 65536:
                raise ValueError(f'port "{v}" must be > 0')
            out.append(n)
    return out


def exit_status(rc: int | None, error: str | None = None) -> dict:
    if error is not None:
        return {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure",
                "message": error, "reason": "InternalError", "code": 500}
    if rc == 0:
        return {"metadata": {}, "status": "Success"}
    return {"metadata": {}, "status": "Failure", "message": f"command terminated with non-zero exit code: {rc}",
            "reason": "NonZeroExitCode", "details": {"causes": [{"reason": "ExitCode", "message": str(rc)}]}}


def rc_from_status(payload: bytes) -> int:
    """Client side: the exit code carried by a v4 status message (0 when Success)."""
    try:
        st = json.loads(payload)
    except ValueError:
        return 1
    if st.get("status") == "Success":
        return 0
    for c in (st.get("details") or {}).get("causes") or ():
        if c.get("reason") == "ExitCode":
            try:
                return int(c.get("message"))
            except (TypeError, ValueError):
                break
    return 1


class _Pipe:
    """Async byte-chunk iterator fed by the socket reader (stdin / resize); None ends it."""

    def __init__(self):
        self.q: asyncio.Queue = asyncio.Queue()
        self.closed = False

    def feed(self, data):
        if not self.closed:
            self.q.put_nowait(data)

    def close(self):
        if not self.closed:
            self.closed = True
            self.q.put_nowait(None)

    def __aiter__(self):
        return self

    async def __anext__(self):
        d = await self.q.get()
        if d is None:
            self.q.put_nowait(None)
            raise StopAsyncIteration
        return d


async def serve_exec(conn: ChannelConn, opts: Options, executor):
    """Run one exec/attach session. `executor(stdin, stdout, stderr, tty, resize) -> rc`:
    stdin / resize are async iterators (None when not requested), stdout / stderr async
    callables (None when not requested)."""
    stdin = _Pipe() if opts.stdin else None
    resize = _Pipe() if opts.tty else None
    first = STDOUT if opts.stdout else (STDERR if opts.stderr else ERROR)
    await conn.write(first, b"")

    async def reader():
        try:
            while True:
                m = await conn.read()
                if m is None:
                    break
                ch, data = m
                if ch == STDIN and stdin is not None:
                    stdin.feed(data)
                elif ch == RESIZE and resize is not None:
                    try:
                        sz = json.loads(data)
                        resize.feed((int(sz.get("Width", 0)), int(sz.get("Height", 0))))
                    except (ValueError, TypeError, AttributeError):
                        pass
                elif ch == CLOSE and conn.protocol == V5_CHANNEL and data[:1] == bytes([STDIN]) and stdin is not None:
                    stdin.close()
        finally:
            for p in (stdin, resize):
                if p is not None:
                    p.close()
    rtask = asyncio.ensure_future(reader())

    def sink(ch):
        async def w(data):
            if data:
                await conn.write(ch, data)
        return w
    err = None
    rc = None
    try:
        rc = await executor(stdin, sink(STDOUT) if opts.stdout else None, sink(STDERR) if opts.stderr else None,
                            opts.tty, resize)
    except (ConnectionError, asyncio.CancelledError):
        rtask.cancel()
        raise
    except Exception as e:  # noqa: BLE001 - reported to the client as an InternalError status
        log.warning("exec failed: %s", e)
        err = f"error executing command in container: {e}"
    try:
        if conn.v4 or conn.protocol == V5_CHANNEL:
            await conn.write(ERROR, json.dumps(exit_status(rc, err)).encode())
        elif err is not None or rc:
            await conn.write(ERROR, (err or f"command terminated with non-zero exit code: {rc}").encode())
        await conn.close()
    except (ConnectionError, RuntimeError):
        pass
    rtask.cancel()


async def serve_portforward(conn: ChannelConn, ports, dial):
    """`dial(port) -> (reader, writer)` to the pod's port; one connection per requested port."""
    socks: dict[int, tuple] = {}
    for i, p in enumerate(ports):
        pb = int(p).to_bytes(2, "little")
        await conn.write(2 * i, pb)
        await conn.write(2 * i + 1, pb)

    async def open_one(i, port):
        try:
            socks[i] = await dial(port)
        except OSError as e:
            await conn.write(2 * i + 1, f"error forwarding port {port} to pod: {e}".encode())
            return
        r, _w = socks[i]
        try:
            while True:
                d = await r.read(65536)
                if not d:
                    break
                await conn.write(2 * i, d)
        except (ConnectionError, RuntimeError):
            pass
    pumps = [asyncio.ensure_future(open_one(i, p)) for i, p in enumerate(ports)]
    try:
        while True:
            m = await conn.read()
            if m is None:
                break
            ch, data = m
            i = ch // 2
            if ch % 2 == 0 and i in socks and data:
                w = socks[i][1]
                w.write(data)
                await w.drain()
    except (ConnectionError, RuntimeError):
        pass
    finally:
        for t in pumps:
            t.cancel()
        for _r, w in socks.values():
            try:
                w.close()
            except RuntimeError:
                pass
        await conn.close()


def exec_response(req, opts_qs, executor, protocols=EXEC_PROTOCOLS):
    """HTTP-server response for a WebSocket exec/attach request (400 on bad options/protocol)."""
    try:
        opts = options_from_query(opts_qs)
    except ValueError as e:
        return Response(400, str(e).encode(), "text/plain")
    proto = negotiate(req.headers, protocols)
    if proto is None:
        return Response(400, f"requested protocol(s) are not supported; supports {list(protocols)}".encode(),
                        "text/plain")

    async def run(reader, writer):
        await serve_exec(ChannelConn(WebSocket(reader, writer), proto), opts, executor)
    return UpgradeResponse(run, "websocket", handshake_headers(req.headers, proto))


def portforward_response(req, dial):
    try:
        ports = ports_from_query(req.qs)
    except ValueError as e:
        return Response(400, str(e).encode(), "text/plain")
    proto = negotiate(req.headers, PORTFORWARD_PROTOCOLS)
    if proto is None:
        return Response(400, b"requested protocol(s) are not supported", "text/plain")

    async def run(reader, writer):
        await serve_portforward(ChannelConn(WebSocket(reader, writer), proto), ports, dial)
    return UpgradeResponse(run, "websocket", handshake_headers(req.headers, proto))


async def accept_raw(reader, writer, headers, supported):
    """Server handshake on a raw asyncio connection whose request head is already read (the CRI
    streaming server) -> ChannelConn, or None after a 400 reply."""
    proto = negotiate(headers, supported)
    if proto is None:
        writer.write(b"HTTP/1.1 400 Bad Request\r\nContent-Length: 0\r\n\r\n")
        await writer.drain()
        return None
    extra = "".join("%s: %s\r\n" % kv for kv in handshake_headers(headers, proto).items())
    writer.write(("HTTP/1.1 101 Switching Protocols\r\nConnection: Upgrade\r\nUpgrade: websocket\r\n%s\r\n"
                  % extra).encode())
    await writer.drain()
    return ChannelConn(WebSocket(reader, writer), proto)


HOP_HEADERS = {"host", "content-length", "transfer-encoding"}


def upgrade_proxy_response(req, url: str, extra_headers=None, ssl_context=None):
    """Relay an upgrade request (WebSocket) to `url` — path and query of the next hop — and
    splice both directions once the backend answered; the backend's reply (101 or an error) goes
    to the client verbatim."""
    from .server import splice
    u = urlsplit(url)

    async def run(reader, writer):
        try:
            tls = None
            if u.scheme == "https":
                from ..utils.tlsutil import unverified_client_context
                tls = ssl_context or unverified_client_context()
            ur, uw = await asyncio.open_connection(u.hostname, u.port or (443 if tls else 80), ssl=tls)
        except OSError as e:
            msg = f"error dialing backend: {e}".encode()
            writer.write(b"HTTP/1.1 503 Service Unavailable\r\nContent-Type: text/plain\r\nContent-Length: %d\r\n\r\n%s"
                         % (len(msg), msg))
            await writer.drain()
            return
        target = (u.path or "/") + (("?" + u.query) if u.query else "")
        lines = [f"GET {target} HTTP/1.1", f"Host: {u.hostname}:{u.port}"]
        for k, v in req.headers.items():
            if k not in HOP_HEADERS and not k.startswith("authorization"):
                lines.append(f"{k}: {v}")
        lines += [f"{k}: {v}" for k, v in (extra_headers or {}).items()]
        uw.write(("\r\n".join(lines) + "\r\n\r\n").encode())
        await uw.drain()
        try:
            head = await ur.readuntil(b"\r\n\r\n")
        except (asyncio.IncompleteReadError, asyncio.LimitOverrunError, ConnectionError):
            uw.close()
            return
        writer.write(head)
        if b" 101 " not in head.split(b"\r\n", 1)[0] + b" ":
            # refused upgrade: relay the reply and end the connection (never splice a client
            # onto a backend keep-alive connection)
            n = 0
            for ln in head.split(b"\r\n"):
                if ln.lower().startswith(b"content-length:"):
                    n = int(ln.split(b":", 1)[1])
            if n:
                try:
                    writer.write(await ur.readexactly(n))
                except (asyncio.IncompleteReadError, ConnectionError):
                    pass
            await writer.drain()
            uw.close()
            return
        await splice(reader, writer, ur, uw)
    return UpgradeResponse(run, None)


__all__ = ["Options", "options_from_query", "ports_from_query", "exit_status", "rc_from_status", "serve_exec",
           "serve_portforward", "exec_response", "portforward_response", "accept_raw", "upgrade_proxy_response",
           "is_websocket_request", "EXEC_PROTOCOLS", "PORTFORWARD_PROTOCOLS", "V5_CHANNEL"]


# -- SPDY/3.1 (what kubectl and client-go of 1.9 speak) ---------------------------------------------
SPDY_EXEC_PROTOCOLS = ("v4.channel.k8s.io", "v3.channel.k8s.io", "v2.channel.k8s.io", "channel.k8s.io")
SPDY_PORTFORWARD_PROTOCOL = "portforward.k8s.io"
STREAM_CREATION_TIMEOUT = 30.0


def is_spdy_request(headers) -> bool:
    return "upgrade" in headers.get("connection", "").lower() and \
        headers.get("upgrade", "").lower().startswith("spdy/3.1")


def is_upgrade_request(headers) -> bool:
    """A WebSocket or SPDY upgrade (what the API server relays to the kubelet untouched)."""
    return is_websocket_request(headers) or is_spdy_request(headers)


def spdy_negotiate(headers, supported):
    """`httpstream.Handshake`: the first client protocol (in the client's order) the server
    supports; "" when the client asked for none (Kubernetes 1.0 clients); None = no match."""
    offered = [p.strip() for p in headers.get("x-stream-protocol-version", "").split(",") if p.strip()]
    if not offered:
        return ""
    for p in offered:
        if p in supported:
            return p
    return None


def _refuse(offered, supported):
    body = (f"unable to upgrade: unable to negotiate protocol: client supports {offered}, "
            f"server accepts {list(supported)}").encode()
    return Response(403, body, "text/plain", {"X-Accepted-Stream-Protocol-Versions": ", ".join(supported)})


async def _json_objects(stream):
    """Consecutive JSON values on a stream (the resize stream of remotecommand v3+)."""
    dec = json.JSONDecoder()
    buf = ""
    while True:
        d = await stream.read()
        if not d:
            return
        buf += d.decode(errors="replace")
        while buf.strip():
            try:
                obj, end = dec.raw_decode(buf.lstrip())
            except ValueError:
                break
            buf = buf.lstrip()[end:]
            yield obj


async def serve_spdy_exec(reader, writer, proto: str, opts: Options, executor):
    """One exec/attach session over SPDY (`remotecommand/httpstream.go` v1-v4 handlers): the
    client opens an error stream plus one per requested stdio stream (and `resize` under a tty
    for v3+), told apart by their `streamType` header."""
    from ..utils import spdy
    want = {"error"} | ({"stdin"} if opts.stdin else set()) | ({"stdout"} if opts.stdout else set()) | \
        ({"stderr"} if opts.stderr else set()) | ({"resize"} if opts.tty and proto in SPDY_EXEC_PROTOCOLS[:2] else set())
    streams: dict = {}
    ready = asyncio.Event()

    async def on_stream(st):
        await st.reply()
        streams[st.header("streamtype")] = st
        if want <= set(streams):
            ready.set()
    conn = spdy.Connection(reader, writer, server=True, on_stream=on_stream)
    serving = asyncio.ensure_future(conn.serve())
    try:
        try:
            await asyncio.wait_for(ready.wait(), STREAM_CREATION_TIMEOUT)
        except asyncio.TimeoutError:
            log.warning("exec: timed out waiting for client streams (have %s, want %s)", sorted(streams), sorted(want))
            return

        async def stdin_chunks():
            while True:
                d = await streams["stdin"].read()
                if not d:
                    return
                yield d

        async def sizes():
            async for obj in _json_objects(streams["resize"]):
                try:
                    yield int(obj.get("Width", 0)), int(obj.get("Height", 0))
                except (TypeError, ValueError, AttributeError):
                    continue

        def sink(name):
            async def w(data):
                if data:
                    await streams[name].write(data)
            return w
        rc, err = None, None
        try:
            rc = await executor(stdin_chunks() if opts.stdin else None, sink("stdout") if opts.stdout else None,
                                sink("stderr") if opts.stderr else None, opts.tty,
                                sizes() if "resize" in want else None)
        except (ConnectionError, asyncio.CancelledError):
            raise
        except Exception as e:  # noqa: BLE001 - reported on the error stream
            log.warning("exec failed: %s", e)
            err = f"error executing command in container: {e}"
        try:
            if proto == "v4.channel.k8s.io":
                await streams["error"].write(json.dumps(exit_status(rc, err)).encode())
            elif err is not None or rc:
                await streams["error"].write((err or f"command terminated with non-zero exit code: {rc}").encode())
            for name in ("stdout", "stderr", "error"):
                if name in streams:
                    await streams[name].close()
        except (ConnectionError, RuntimeError):
            pass
    finally:
        await conn.close()
        serving.cancel()


async def serve_spdy_portforward(reader, writer, dial):
    """Port forwarding over SPDY (`portforward/httpstream.go`): the client opens a `data` and an
    `error` stream per connection, paired by the `requestID` header, for the port in `port`."""
    from ..utils import spdy
    pairs: dict = {}
    tasks = []

    async def forward(port, data, error):
        try:
            r, w = await dial(port)
        except OSError as e:
            try:
                await error.write(f"error forwarding port {port} to pod: {e}".encode())
                await error.close()
                await data.close()
            except (ConnectionError, RuntimeError):
                pass
            return

        async def up():
            try:
                while True:
                    d = await data.read()
                    if not d:
                        break
                    w.write(d)
                    await w.drain()
            except (ConnectionError, RuntimeError):
                pass
            finally:
                try:
                    w.write_eof()
                except (OSError, RuntimeError):
                    pass
        t = asyncio.ensure_future(up())
        try:
            while True:
                d = await r.read(65536)
                if not d:
                    break
                await data.write(d)
        except (ConnectionError, RuntimeError):
            pass
        finally:
            try:
                await data.close()
                await error.close()
            except (ConnectionError, RuntimeError):
                pass
            await asyncio.wait([t], timeout=5)
            w.close()

    async def on_stream(st):
        await st.reply()
        rid = st.header("requestid") or str(st.id)
        p = pairs.setdefault(rid, {})
        p[st.header("streamtype")] = st
        if "data" in p and "error" in p:
            try:
                port = int(p["data"].header("port") or p["error"].header("port"))
            except ValueError:
                await p["error"].write(b"invalid port")
                await p["error"].close()
                return
            tasks.append(asyncio.ensure_future(forward(port, p["data"], p["error"])))
    conn = spdy.Connection(reader, writer, server=True, on_stream=on_stream)
    try:
        await conn.serve()
    finally:
        for t in tasks:
            t.cancel()
        await conn.close()


def spdy_exec_response(req, executor):
    try:
        opts = options_from_query(req.qs)
    except ValueError as e:
        return Response(400, str(e).encode(), "text/plain")
    proto = spdy_negotiate(req.headers, SPDY_EXEC_PROTOCOLS)
    if proto is None:
        return _refuse(req.headers.get("x-stream-protocol-version", ""), SPDY_EXEC_PROTOCOLS)

    async def run(reader, writer):
        await serve_spdy_exec(reader, writer, proto or "channel.k8s.io", opts, executor)
    return UpgradeResponse(run, "SPDY/3.1", {"X-Stream-Protocol-Version": proto} if proto else None)


def spdy_portforward_response(req, dial):
    proto = spdy_negotiate(req.headers, (SPDY_PORTFORWARD_PROTOCOL,))
    if proto is None:
        return _refuse(req.headers.get("x-stream-protocol-version", ""), (SPDY_PORTFORWARD_PROTOCOL,))

    async def run(reader, writer):
        await serve_spdy_portforward(reader, writer, dial)
    return UpgradeResponse(run, "SPDY/3.1", {"X-Stream-Protocol-Version": proto} if proto else None)


async def accept_raw_spdy(writer, headers, supported):
    """SPDY upgrade on a raw connection (CRI streaming server) -> protocol, or None after 403."""
    proto = spdy_negotiate(headers, supported)
    if proto is None:
        r = _refuse(headers.get("x-stream-protocol-version", ""), supported)
        writer.write(b"HTTP/1.1 403 Forbidden\r\nContent-Length: %d\r\n\r\n%s" % (len(r.body), r.body))
        await writer.drain()
        return None
    extra = f"X-Stream-Protocol-Version: {proto}\r\n" if proto else ""
    writer.write(f"HTTP/1.1 101 Switching Protocols\r\nConnection: Upgrade\r\nUpgrade: SPDY/3.1\r\n{extra}\r\n".encode())
    await writer.drain()
    return proto
