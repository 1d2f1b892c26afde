"""Minimal, fast asyncio HTTP/1.1 server (keep-alive, pipelining-safe, chunked streaming).

The reference's apiserver runs Go's net/http with HTTP/2; here the control plane lives on
host sockets (SURVEY §2.4 "Distributed comms backend"), so the transport is a lean
Protocol-based HTTP/1.1 implementation: one parse per request, no per-request
allocations beyond the header dict, responses written with a single `transport.write`.
"""
from __future__ import annotations

import asyncio
import time
import logging
from urllib.parse import parse_qs, unquote

log = logging.getLogger("httpserver")

# largest request body read into memory (Content-Length or chunked); larger is a 413 and the
# connection closes. Objects are far smaller (the store keeps values under ~1.5 MiB like etcd);
# this bounds what one connection can make the server buffer.
MAX_BODY = 64 << 20

REASONS = {
    200: "OK", 201: "Created", 202: "Accepted", 204: "No Content", 400: "Bad Request",
    401: "Unauthorized", 403: "Forbidden", 404: "Not Found", 405: "Method Not Allowed",
    406: "Not Acceptable", 409: "Conflict", 410: "Gone", 413: "Payload Too Large",
    415: "Unsupported Media Type", 422: "Unprocessable Entity", 429: "Too Many Requests",
    431: "Request Header Fields Too Large", 500: "Internal Server Error", 501: "Not Implemented", 503: "Service Unavailable", 504: "Gateway Timeout",
}


class Request:
    __slots__ = ("method", "path", "raw_path", "query", "qs", "headers", "body", "transport", "user", "info", "served_gv",
                 "insecure", "obj")

    def __init__(self, method, target, headers, body, transport):
        self.method = method
        if "?" in target:
            p, qs = target.split("?", 1)
            self.query = {k: v[-1] for k, v in parse_qs(qs, keep_blank_values=True).items()}
        else:
            p, self.query, qs = target, {}, ""
        self.qs = qs
        self.raw_path = p
        self.path = unquote(p)
        self.headers = headers
        self.body = body
        self.transport = transport
        self.user = None
        self.info = None
        self.served_gv = None
        self.insecure = False      # arrived on the API server's insecure listener
        self.obj = None            # the body, already decoded (protobuf request bodies)


class Response:
    __slots__ = ("status", "body", "content_type", "headers", "entry")

    def __init__(self, status=200, body=b"", content_type="application/json", headers=None, entry=None):
        self.status = status
        self.body = body if isinstance(body, (bytes, bytearray)) else str(body).encode()
        self.content_type = content_type
        self.headers = headers
        self.entry = entry         # the cache entry the body came from (protobuf negotiation)


class StreamResponse:
    """Returned by a handler that wants to stream (watch). `run(writer)` is awaited with a
    ChunkWriter; the connection is closed afterwards."""

    __slots__ = ("run", "content_type")

    def __init__(self, run, content_type="application/json"):
        self.run = run
        self.content_type = content_type


class UpgradeResponse:
    """Returned by a handler that switches the connection to another protocol
    (`Connection: Upgrade`): `101 Switching Protocols` is sent, then `run(reader, writer)` owns
    the raw byte stream (stream-style reader/writer over the same transport). `headers` are
    added to the 101 reply (WebSocket accept key / sub-protocol); `protocol=None` writes no reply
    at all — `run` owns the whole response (an upgrade-aware proxy relays the backend's)."""

    __slots__ = ("run", "protocol", "headers")

    def __init__(self, run, protocol="tcp", headers=None):
        self.run = run
        self.protocol = protocol
        self.headers = headers


class HandoffResponse:
    """Returned by a handler that gives the whole connection to another process: `run(fd)`
    receives a duplicate of the client socket (e.g. to pass it with SCM_RIGHTS); this server
    then forgets the connection without writing anything (the other process owns the reply)."""

    __slots__ = ("run",)

    def __init__(self, run):
        self.run = run


class ChunkWriter:
    __slots__ = ("transport", "closed", "_proto")

    def __init__(self, transport, proto):
        self.transport = transport
        self._proto = proto
        self.closed = False

    def write(self, data: bytes):
        if self.closed or self.transport.is_closing():
            self.closed = True
            return False
        self.transport.write(b"%x\r\n%s\r\n" % (len(data), data))
        return True

    async def drain(self):
        await self._proto.drain()

    def end(self):
        if not self.closed and not self.transport.is_closing():
            self.transport.write(b"0\r\n\r\n")
        self.closed = True

    def wait_closed(self):
        """Future resolved when the peer closes the connection."""
        p = self._proto
        if p.close_fut is None:
            p.close_fut = asyncio.get_running_loop().create_future()
            if self.transport.is_closing():
                p.close_fut.set_result(None)
        return p.close_fut


_CHUNK_SIZE = __import__("re").compile(rb"[0-9A-Fa-f]{1,16}")
MAX_CHUNKS = 1 << 16          # chunks per request body


class _ChunkState:
    """Where a chunked body's parse stopped: `pos` = next unparsed byte, `need` = bytes of the
    current chunk still to arrive (None: a size line is next)."""
    __slots__ = ("start", "pos", "need", "parts", "size", "chunks", "framing", "trailer", "eol")

    def __init__(self, start):
        self.start = self.pos = start
        self.need = None
        self.parts = []
        self.size = self.chunks = self.framing = 0
        self.trailer = False
        self.eol = 0


class _Conn(asyncio.Protocol):
    def __init__(self, server):
        self.server = server
        self.buf = bytearray()
        self.transport = None
        self.pending = []
        self.busy = False
        self.streaming = False
        self._paused = False
        self._drain_waiter = None
        self.close_fut = None
        self.deadline = 0.0         # loop time the in-flight request must answer by (0 = none)
        self.chunked = None         # _ChunkState of a chunked request body being received
        self.rejected = None        # (status, why) answered after the pipelined requests before it

    def connection_made(self, transport):
        self.transport = transport
        self.server._conns.add(self)

    def connection_lost(self, exc):
        self.server._conns.discard(self)
        self.streaming = False
        if self.close_fut is not None and not self.close_fut.done():
            self.close_fut.set_result(None)
        if self._drain_waiter and not self._drain_waiter.done():
            self._drain_waiter.set_result(None)

    def pause_writing(self):
        self._paused = True

    def resume_writing(self):
        self._paused = False
        if self._drain_waiter and not self._drain_waiter.done():
            self._drain_waiter.set_result(None)

    async def drain(self):
        if self._paused and not self.transport.is_closing():
            self._drain_waiter = asyncio.get_running_loop().create_future()
            await self._drain_waiter

    def data_received(self, data):
        if self.rejected is not None:
            return                  # nothing after a framing error starts a request
        self.buf += data
        while True:
            req = self._parse()
            if req is None:
                break
            self.pending.append(req)
        if self.pending and not self.busy:
            self.busy = True
            # the loop only keeps weak references to tasks: hold this one until it finishes
            t = asyncio.ensure_future(self._serve())
            self.server._tasks.add(t)
            t.add_done_callback(self.server._tasks.discard)

    def _reject(self, status, why):
        """Answer a request this server will not read (bad framing, too large) and close: after
        a framing error nothing later on the connection can be trusted to start a request. The
        answer goes out after the responses of requests pipelined before it (HTTP/1.1 keeps
        responses in request order); reading stops now."""
        self.rejected = (status, why)
        self.chunked = None
        del self.buf[:]
        self.transport.pause_reading()
        if not self.pending and not self.busy:
            self._write_reject()

    def _write_reject(self):
        status, why = self.rejected
        body = b'{"kind":"Status","apiVersion":"v1","metadata":{},"status":"Failure","message":"%s","code":%d}' % (
            why.encode(), status)
        if not self.transport.is_closing():
            self.transport.write(b"HTTP/1.1 %d %s\r\nContent-Type: application/json\r\nContent-Length: %d\r\n"
                                 b"Connection: close\r\n\r\n%s" % (status, REASONS.get(status, "Error").encode(),
                                                                      len(body), body))
            self.transport.close()

    def _chunked_body(self, start):
        """(body, end offset) of a complete chunked request body at buf[start:], None while
        incomplete; raises ValueError on bad framing, OverflowError over the size limit. The
        parse state lives on the connection (`_ChunkState`), so every byte is parsed once however
        many reads the body arrives in."""
        st = self.chunked
        if st is None or st.start != start:
            st = self.chunked = _ChunkState(start)
        buf = self.buf
        limit = self.server.max_body
        while True:
            pos = st.pos
            if st.trailer:
                tend = buf.find(b"\r\n\r\n", st.eol) if buf[st.eol + 2:st.eol + 4] != b"\r\n" else st.eol
                if tend < 0:
                    if len(buf) - st.eol > 8192:
                        raise ValueError("trailer section too long")
                    return None
                self.chunked = None
                return b"".join(st.parts), tend + 4
            if st.need is None:
                eol = buf.find(b"\r\n", pos, pos + 1026)
                if eol < 0:
                    if len(buf) - pos > 1024:
                        raise ValueError("chunk size line too long")
                    return None
                tok = bytes(buf[pos:eol]).split(b";", 1)[0].strip()
                if not _CHUNK_SIZE.fullmatch(tok):       # RFC 7230 §4.1: 1*HEXDIG, nothing else
                    raise ValueError("malformed chunk size")
                n = int(tok, 16)
                st.size += n
                st.framing += eol + 2 - pos
                if st.size > limit:
                    raise OverflowError
                st.chunks += 1
                if st.chunks > MAX_CHUNKS or st.framing > max(64 << 10, limit // 4):
                    raise OverflowError
                if n == 0:
                    st.trailer, st.eol = True, eol
                    continue
                st.need, st.pos = n, eol + 2
                continue
            n = st.need
            if len(buf) < pos + n + 2:
                return None
            if buf[pos + n:pos + n + 2] != b"\r\n":
                raise ValueError("chunk not terminated by CRLF")
            st.parts.append(bytes(buf[pos:pos + n]))
            st.need, st.pos = None, pos + n + 2

    def _parse(self):
        buf = self.buf
        end = buf.find(b"\r\n\r\n")
        if end < 0:
            if len(buf) > 1 << 20:
                self._reject(431, "request header fields too large")
            return None
        head = bytes(buf[:end]).decode("latin-1")
        lines = head.split("\r\n")
        try:
            method, target, _ = lines[0].split(" ", 2)
        except ValueError:
            self.transport.close()
            return None
        headers = {}
        for ln in lines[1:]:
            k, _, v = ln.partition(":")
            k = k.strip().lower()
            # repeated headers combine into one comma-separated list (RFC 7230 §3.2.2), e.g.
            # several X-Stream-Protocol-Version offers
            headers[k] = headers[k] + ", " + v.strip() if k in headers else v.strip()
        te = headers.get("transfer-encoding")
        if te is not None:
            # RFC 7230 §3.3.3: chunked must be the final coding; it overrides Content-Length
            if te.strip().lower() != "chunked":         # other codings are not implemented
                self._reject(501, "unsupported transfer-encoding")
                return None
            try:
                got = self._chunked_body(end + 4)
            except OverflowError:
                self._reject(413, "request body too large")
                return None
            except ValueError:
                self._reject(400, "malformed chunked request body")
                return None
            if got is None:
                return None
            body, stop = got
            self.chunked = None
            del buf[:stop]
            headers.pop("transfer-encoding", None)
            headers["content-length"] = str(len(body))
            return Request(method, target, headers, body, self.transport)
        cl = headers.get("content-length", "0") or "0"
        if not cl.isdigit():
            # negative, non-numeric or differing repeated values: the body's end is unknown
            self._reject(400, "invalid content-length")
            return None
        clen = int(cl)
        if clen > self.server.max_body:
            self._reject(413, "request body too large")
            return None
        if len(buf) < end + 4 + clen:
            return None
        body = bytes(buf[end + 4:end + 4 + clen])
        del buf[:end + 4 + clen]
        return Request(method, target, headers, body, self.transport)

    async def _serve(self):
        try:
            while self.pending:
                req = self.pending.pop(0)
                srv = self.server
                if srv.request_timeout and not (srv.long_running is not None and srv.long_running(req)):
                    self.deadline = srv.loop_time() + srv.request_timeout
                try:
                    resp = await self.server.handler(req)
                except Exception as e:  # pragma: no cover - defensive
                    log.exception("handler error")
                    resp = Response(500, b'{"kind":"Status","status":"Failure","message":%s,"code":500}' % repr(str(e)).encode())
                self.deadline = 0.0
                if self.transport.is_closing():
                    return              # includes a request the timeout sweeper already answered
                if isinstance(resp, UpgradeResponse):
                    await self._upgrade(resp)
                    return
                if isinstance(resp, HandoffResponse):
                    import os
                    # earlier pipelined responses still buffered here must reach the peer first
                    for _ in range(200):
                        if self.transport.is_closing() or not self.transport.get_write_buffer_size():
                            break
                        await asyncio.sleep(0.005)
                    if self.transport.is_closing():
                        return
                    sock = self.transport.get_extra_info("socket")
                    fd = os.dup(sock.fileno())
                    try:
                        resp.run(fd)
                    except OSError:
                        log.exception("connection handoff failed")
                    finally:
                        os.close(fd)
                    # close only this process's descriptor: the peer's process now holds the socket
                    self.transport.abort()
                    return
                if isinstance(resp, StreamResponse):
                    self.streaming = True
                    self.transport.write(
                        ("HTTP/1.1 200 OK\r\nContent-Type: %s\r\nTransfer-Encoding: chunked\r\n"
                         "Cache-Control: no-cache, private\r\n\r\n" % resp.content_type).encode())
                    w = ChunkWriter(self.transport, self)
                    try:
                        await resp.run(w)
                    except (ConnectionError, asyncio.CancelledError):
                        pass
                    finally:
                        w.end()
                        self.streaming = False
                    self.transport.close()
                    return
                hdr = "HTTP/1.1 %d %s\r\nContent-Type: %s\r\nContent-Length: %d\r\n" % (
                    resp.status, REASONS.get(resp.status, "OK"), resp.content_type, len(resp.body))
                if resp.headers:
                    hdr += "".join("%s: %s\r\n" % kv for kv in resp.headers.items())
                close = req.headers.get("connection", "").lower() == "close"
                if close:
                    hdr += "Connection: close\r\n"
                self.transport.write(hdr.encode() + b"\r\n" + resp.body)
                if close:
                    self.transport.close()
                    return
        finally:
            self.busy = False
            if self.rejected is not None and not self.pending:
                self._write_reject()

    async def _upgrade(self, resp):
        loop = asyncio.get_running_loop()
        reader = asyncio.StreamReader(loop=loop)
        proto = asyncio.StreamReaderProtocol(reader, loop=loop)
        if resp.protocol is not None:
            extra = "".join("%s: %s\r\n" % kv for kv in (resp.headers or {}).items())
            self.transport.write(("HTTP/1.1 101 Switching Protocols\r\nConnection: Upgrade\r\nUpgrade: %s\r\n%s\r\n"
                                  % (resp.protocol, extra)).encode())
        rest = bytes(self.buf)
        self.buf.clear()
        self.transport.set_protocol(proto)
        proto.connection_made(self.transport)
        if rest:
            reader.feed_data(rest)
        writer = asyncio.StreamWriter(self.transport, proto, reader, loop)
        self.streaming = True
        # StreamReaderProtocol references its reader only weakly: keep both ends reachable
        self.upgraded = (reader, writer)
        try:
            await resp.run(reader, writer)
        except (ConnectionError, asyncio.CancelledError):
            pass
        finally:
            self.streaming = False
            self.upgraded = None
            self.transport.close()
            self.server._conns.discard(self)   # connection_lost now goes to the new protocol


class HTTPServer:
    """`request_timeout` (seconds): a request not answered in time gets `timeout_response` and its
    connection is closed, while the handler runs on and its late response is dropped (Go's
    http.TimeoutHandler, the API server's --request-timeout); `long_running(req)` exempts
    watches, streams and proxies. One sweeper per server checks the deadlines, so a request pays
    only a clock read."""

    def __init__(self, handler, request_timeout=None, long_running=None, timeout_response=None):
        self.handler = handler
        self._server = None
        self._conns = set()
        self._tasks = set()
        self.port = None
        self.request_timeout = request_timeout
        self.long_running = long_running
        self.timeout_response = timeout_response or Response(504, b"request timed out", "text/plain")
        self._sweeper = None
        self.loop_time = time.monotonic
        self.max_body = MAX_BODY

    async def _sweep(self):
        period = max(0.05, min(1.0, self.request_timeout / 4))
        while True:
            await asyncio.sleep(period)
            now = self.loop_time()
            for c in list(self._conns):
                if c.deadline and now > c.deadline and c.transport is not None and not c.transport.is_closing():
                    r = self.timeout_response
                    c.transport.write(("HTTP/1.1 %d %s\r\nContent-Type: %s\r\nContent-Length: %d\r\nConnection: close\r\n\r\n"
                                       % (r.status, REASONS.get(r.status, "OK"), r.content_type, len(r.body))).encode()
                                      + r.body)
                    c.deadline = 0.0
                    c.transport.close()

    async def start(self, host="127.0.0.1", port=0, ssl=None, reuse_port=False):
        """reuse_port: several worker processes listen on one port; the kernel spreads
        incoming connections across them (SO_REUSEPORT)."""
        loop = asyncio.get_running_loop()
        self._server = await loop.create_server(lambda: _Conn(self), host, port, ssl=ssl, backlog=4096,
                                                reuse_address=True, reuse_port=reuse_port or None)
        self.port = self._server.sockets[0].getsockname()[1]
        if self.request_timeout and self._sweeper is None:
            self._sweeper = asyncio.ensure_future(self._sweep())
        return self.port

    async def start_unix(self, path):
        loop = asyncio.get_running_loop()
        self._server = await loop.create_unix_server(lambda: _Conn(self), path)
        return path

    async def stop(self):
        if self._sweeper is not None:
            self._sweeper.cancel()
            self._sweeper = None
        if self._server:
            self._server.close()
            for c in list(self._conns):
                if c.transport:
                    c.transport.close()
            await self._server.wait_closed()


def log_dir_response(base_dir: str, rel: str) -> "Response":
    """Read-only view of a log directory (`/logs/` of the kubelet and the API server,
    `server.go` getLogs / `routes.Logs`): directory listings and file contents, never a path
    outside `base_dir`."""
    import os
    base = os.path.realpath(base_dir)
    target = os.path.realpath(os.path.join(base, rel))
    if target != base and not target.startswith(base + os.sep):
        return Response(403, b"path escapes the log directory", "text/plain")
    if os.path.isdir(target):
        try:
            names = sorted(os.listdir(target))
        except OSError as e:
            return Response(403, str(e).encode(), "text/plain")
        return Response(200, "".join(n + ("/" if os.path.isdir(os.path.join(target, n)) else "") + "\n"
                                     for n in names).encode(), "text/plain")
    try:
        with open(target, "rb") as f:
            return Response(200, f.read(), "text/plain")
    except OSError:
        return Response(404, b"not found", "text/plain")
