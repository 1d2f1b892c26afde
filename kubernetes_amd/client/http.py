"""Asyncio HTTP/1.1 client with a keep-alive connection pool and chunked watch streams.

Plays the role of client-go's `rest.Request` transport (`staging/src/k8s.io/client-go/rest/request.go:486-745`).
Supports `http://host:port`, `https://` (ssl context) and `unix:///path.sock` endpoints.
"""
from __future__ import annotations

import asyncio
import ssl as _ssl
from urllib.parse import urlparse


class HTTPError(Exception):
    def __init__(self, status, body):
        super().__init__(f"HTTP {status}: {body[:500]!r}")
        self.status = status
        self.body = body


class _Conn:
    __slots__ = ("reader", "writer")

    def __init__(self, reader, writer):
        self.reader, self.writer = reader, writer

    def close(self):
        try:
            self.writer.close()
        except Exception:
            pass


async def _read_response(reader):
    line = await reader.readline()
    if not line:
        raise ConnectionError("connection closed")
    parts = line.split(b" ", 2)
    status = int(parts[1])
    headers = {}
    while True:
        h = await reader.readline()
        if h in (b"\r\n", b"\n", b""):
            break
        k, _, v = h.decode("latin-1").partition(":")
        headers[k.strip().lower()] = v.strip()
    return status, headers


async def _read_body(reader, headers, status=200, method="GET"):
    if headers.get("transfer-encoding", "").lower() == "chunked":
        out = bytearray()
        while True:
            ln = await reader.readline()
            n = int(ln.strip().split(b";")[0], 16)
            if n == 0:
                await reader.readline()
                break
            out += await reader.readexactly(n)
            await reader.readline()
        return bytes(out)
    if "content-length" not in headers and method != "HEAD" and status >= 200 and status not in (204, 304):
        # no length and not chunked: the body runs to the end of the connection (RFC 7230
        # 3.3.3 rule 7 — HTTP/1.0 servers such as Python's http.server); never reuse it
        headers["connection"] = "close"
        return await reader.read()
    n = int(headers.get("content-length", "0") or 0)
    return await reader.readexactly(n) if n else b""


class HTTPClient:
    def __init__(self, base_url: str, token: str | None = None, ssl_context=None, max_conns: int = 16,
                 timeout: float = 60.0):
        self.base_url = base_url
        u = urlparse(base_url)
        self.unix = u.scheme == "unix"
        self.path_prefix = ""
        if self.unix:
            self.sock_path = u.path
            self.host_header = "localhost"
        else:
            self.host = u.hostname or "127.0.0.1"
            self.port = u.port or (443 if u.scheme == "https" else 80)
            self.host_header = f"{self.host}:{self.port}"
            self.path_prefix = u.path.rstrip("/")
        self.ssl = ssl_context
        if u.scheme == "https" and ssl_context is None:
            self.ssl = _ssl.create_default_context()
            self.ssl.check_hostname = False
            self.ssl.verify_mode = _ssl.CERT_NONE
        self.token = token
        self.default_headers = ""      # preformatted lines sent on every request (impersonation, basic auth)
        self._idle: list[_Conn] = []
        self._sem = asyncio.Semaphore(max_conns)
        self.timeout = timeout
        self._closed = False

    def set_default_headers(self, headers: dict):
        self.default_headers = "".join(f"{k}: {v}\r\n" for k, v in headers.items() if v)

    def set_ssl_context(self, ctx):
        """Swap the TLS context (client-certificate rotation): idle connections made with the
        old credential are closed; new connections present the new certificate."""
        self.ssl = ctx
        idle, self._idle = self._idle, []
        for c in idle:
            c.close()

    async def _open(self):
        if self.unix:
            r, w = await asyncio.open_unix_connection(self.sock_path, limit=1 << 24)
        else:
            r, w = await asyncio.open_connection(self.host, self.port, ssl=self.ssl, limit=1 << 24)
        return _Conn(r, w)

    def _head(self, method, path, body, content_type, extra):
        h = f"{method} {self.path_prefix}{path} HTTP/1.1\r\nHost: {self.host_header}\r\n"
        if self.token:
            h += f"Authorization: Bearer {self.token}\r\n"
        if self.default_headers:
            h += self.default_headers
        if body is not None:
            h += f"Content-Type: {content_type}\r\nContent-Length: {len(body)}\r\n"
        if extra:
            h += "".join(f"{k}: {v}\r\n" for k, v in extra.items())
        return (h + "\r\n").encode()

    async def request(self, method, path, body: bytes | None = None, content_type="application/json", headers=None):
        status, _hdrs, data = await self.request_full(method, path, body, content_type, headers)
        return status, data

    async def request_full(self, method, path, body: bytes | None = None, content_type="application/json",
                           headers=None):
        """Like request(), also returning the response headers (lower-case names)."""
        async with self._sem:
            for attempt in range(2):
                conn = self._idle.pop() if self._idle else None
                fresh = conn is None
                if conn is None:
                    conn = await self._open()
                try:
                    conn.writer.write(self._head(method, path, body, content_type, headers) + (body or b""))
                    status, hdrs = await asyncio.wait_for(_read_response(conn.reader), self.timeout)
                    data = await _read_body(conn.reader, hdrs, status, method)
                except (ConnectionError, asyncio.IncompleteReadError, OSError):
                    conn.close()
                    if fresh or attempt:
                        raise
                    continue  # stale keep-alive connection; retry once on a new one
                except asyncio.TimeoutError:
                    conn.close()
                    raise
                if hdrs.get("connection", "").lower() == "close":
                    conn.close()
                else:
                    self._idle.append(conn)
                return status, hdrs, data

    async def open_raw(self, method, path, headers=None, body=None):
        """Send one request on a dedicated connection and return (status, headers, reader,
        writer) with the body unread — for exec streams and `Upgrade: tcp` port-forward tunnels."""
        conn = await self._open()
        conn.writer.write(self._head(method, path, body, "application/octet-stream", headers) + (body or b""))
        await conn.writer.drain()
        status, hdrs = await _read_response(conn.reader)
        return status, hdrs, conn.reader, conn.writer

    async def stream(self, method, path, headers=None, frames=None):
        """Open a streaming GET; returns (status, async iterator of batches, closer, content
        type). A batch is a list of complete lines — or, when the response is a
        length-delimited stream (`...;stream=watch` protobuf) and `frames` is given, whatever
        `frames(buffer) -> (items, bytes consumed)` makes of the complete frames received."""
        conn = await self._open()
        conn.writer.write(self._head(method, path, None, None, headers))
        status, hdrs = await _read_response(conn.reader)
        if status != 200:
            body = await _read_body(conn.reader, hdrs)
            conn.close()
            raise HTTPError(status, body)
        chunked = hdrs.get("transfer-encoding", "").lower() == "chunked"
        ctype = hdrs.get("content-type", "")
        framed = frames is not None and "stream=watch" in ctype and "protobuf" in ctype
        reader = conn.reader

        async def batches():
            """Lists of complete lines (or frames): everything that arrived in one read is
            parsed and handed over at once (a watch server coalesces events per send), so a
            consumer pays one await per batch, not per event."""
            raw = bytearray()
            pay = bytearray()
            done = False
            try:
                while not done:
                    data = await reader.read(1 << 18)
                    if not data:
                        done = True
                    elif chunked:
                        raw += data
                        pos = 0
                        while True:
                            j = raw.find(b"\r\n", pos)
                            if j < 0:
                                break
                            n = int(bytes(raw[pos:j]).split(b";")[0].strip() or b"0", 16)
                            if n == 0:
                                done = True
                                break
                            end = j + 2 + n
                            if len(raw) < end + 2:
                                break
                            pay += raw[j + 2:end]
                            pos = end + 2
                        if pos:
                            del raw[:pos]
                    else:
                        pay += data
                    if framed:
                        if len(pay) >= 4:
                            items, used = frames(pay)
                            if used:
                                del pay[:used]
                            if items:
                                yield items
                        continue
                    k = pay.rfind(b"\n")
                    if k >= 0:
                        out = [ln for ln in bytes(pay[:k]).split(b"\n") if ln.strip()]
                        del pay[:k + 1]
                        if out:
                            yield out
            except (ConnectionError, asyncio.IncompleteReadError, OSError, ValueError):
                return

        return status, batches(), conn.close, ctype

    async def close(self):
        self._closed = True
        for c in self._idle:
            c.close()
        self._idle.clear()
