"""SPDY/3.1 framing — the multiplexed transport under `kubectl exec / attach / port-forward / cp`
of Kubernetes 1.9 (client-go `tools/remotecommand` SPDY executor, `httpstream/spdy`, the vendored
`docker/spdystream`).

  * an HTTP request with `Connection: Upgrade`, `Upgrade: SPDY/3.1` (and the sub-protocol in
    repeated `X-Stream-Protocol-Version` headers) is answered `101 Switching Protocols`, after
    which both ends exchange SPDY frames on the connection;
  * control frames: `1 | version(15)=3 | type(16) | flags(8) | length(24) | body`; data frames:
    `0 | stream id(31) | flags(8) | length(24) | payload`, flag 0x01 = FIN;
  * SYN_STREAM (1) / SYN_REPLY (2) / HEADERS (8) carry a header block: a 32-bit pair count,
    then 32-bit-length-prefixed lowercase names and values (several values NUL-separated),
    deflated with ONE zlib stream per direction for the whole connection, preset with the SPDY/3
    dictionary, each block ended by a sync flush;
  * RST_STREAM (3), SETTINGS (4), PING (6, echoed), GOAWAY (7), WINDOW_UPDATE (9). Like
    spdystream, no flow-control windows are enforced (WINDOW_UPDATE is read and ignored).

The streams of a session are opened by the client (odd ids); the server answers each with an
empty SYN_REPLY, as the kubelet's stream handler does.
"""
from __future__ import annotations

import asyncio
import struct
import zlib

VERSION = 3
SYN_STREAM, SYN_REPLY, RST_STREAM, SETTINGS, PING, GOAWAY, HEADERS, WINDOW_UPDATE = 1, 2, 3, 4, 6, 7, 8, 9
FLAG_FIN = 0x01
RST_PROTOCOL_ERROR, RST_INVALID_STREAM, RST_REFUSED_STREAM, RST_CANCEL = 1, 2, 3, 5
MAX_FRAME = (1 << 24) - 1
# one decompressed header block (a compressed frame could otherwise inflate ~1000x) and the
# streams one session may hold open (exec/attach use 3-5, port-forward 2 per port)
MAX_HEADER_BLOCK = 1 << 20
MAX_STREAMS = 1024          # concurrently OPEN streams per session (closed ones are forgotten)

# The SPDY/3 header-compression dictionary (draft-mbelshe-httpbis-spdy-00 §2.6.10.1): the common
# header names and values, each as a 32-bit big-endian length + bytes, then a run of status
# lines, dates and media types. Both ends must preset zlib with exactly these 1423 bytes.
_DICT_WORDS = (
    "options,head,post,put,delete,trace,accept,accept-charset,accept-encoding,accept-language,"
    "accept-ranges,age,allow,authorization,cache-control,connection,content-base,content-encoding,"
    "content-language,content-length,content-location,content-md5,content-range,content-type,date,"
    "etag,expect,expires,from,host,if-match,if-modified-since,if-none-match,if-range,"
    "if-unmodified-since,last-modified,location,max-forwards,pragma,proxy-authenticate,"
    "proxy-authorization,range,referer,retry-after,server,te,trailer,transfer-encoding,upgrade,"
    "user-agent,vary,via,warning,www-authenticate,method,get,status,200 OK,version,HTTP/1.1,url,"
    "public,set-cookie,keep-alive,origin")
_DICT_TAIL = (
    "100101201202205206300302303304305306307402405406407408409410411412413414415416417502504505"
    "203 Non-Authoritative Information204 No Content301 Moved Permanently400 Bad Request"
    "401 Unauthorized403 Forbidden404 Not Found500 Internal Server Error501 Not Implemented"
    "503 Service UnavailableJan Feb Mar Apr May Jun Jul Aug Sept Oct Nov Dec 00:00:00 "
    "Mon, Tue, Wed, Thu, Fri, Sat, Sun, GMTchunked,text/html,image/png,image/jpg,image/gif,"
    "application/xml,application/xhtml+xml,text/plain,text/javascript,publicprivatemax-age="
    "gzip,deflate,sdchcharset=utf-8charset=iso-8859-1,utf-,*,enq=0.")


def _dictionary() -> bytes:
    words = _DICT_WORDS.split(",")
    return b"".join(struct.pack(">I", len(w)) + w.encode() for w in words) + _DICT_TAIL.encode()


DICTIONARY = _dictionary()


class SpdyError(Exception):
    pass


def encode_block(headers: dict) -> bytes:
    """{name: [values]} -> uncompressed header block."""
    out = [struct.pack(">I", len(headers))]
    for name, values in headers.items():
        n = name.lower().encode()
        v = b"\x00".join(x.encode() if isinstance(x, str) else x for x in (values if isinstance(values, (list, tuple)) else [values]))
        out += [struct.pack(">I", len(n)), n, struct.pack(">I", len(v)), v]
    return b"".join(out)


def decode_block(data: bytes) -> dict:
    (n,), i = struct.unpack_from(">I", data, 0), 4
    out = {}
    for _ in range(n):
        (ln,) = struct.unpack_from(">I", data, i)
        name = data[i + 4:i + 4 + ln].decode("latin-1")
        i += 4 + ln
        (lv,) = struct.unpack_from(">I", data, i)
        out.setdefault(name, []).extend(x.decode("latin-1") for x in data[i + 4:i + 4 + lv].split(b"\x00"))
        i += 4 + lv
    return out


def control_frame(ftype: int, flags: int, body: bytes) -> bytes:
    return struct.pack(">HHI", 0x8000 | VERSION, ftype, (flags << 24) | len(body)) + body


def data_frame(sid: int, flags: int, payload: bytes) -> bytes:
    return struct.pack(">II", sid & 0x7FFFFFFF, (flags << 24) | len(payload)) + payload


class Stream:
    def __init__(self, conn, sid, headers):
        self.conn, self.id, self.headers = conn, sid, headers
        self._q: asyncio.Queue = asyncio.Queue()
        self.remote_closed = False
        self.local_closed = False
        self.reset = False
        self.replied = asyncio.Event()

    def header(self, name, default=""):
        v = self.headers.get(name.lower())
        return v[0] if v else default

    def _feed(self, data, fin):
        if data:
            self._q.put_nowait(data)
        if fin and not self.remote_closed:
            self.remote_closed = True
            self._q.put_nowait(b"")
            self.conn._forget(self)

    def _done(self):
        return self.reset or (self.remote_closed and self.local_closed)

    async def read(self) -> bytes:
        """Next chunk, b"" once the peer half-closed (or reset) the stream."""
        d = await self._q.get()
        if d == b"":
            self._q.put_nowait(b"")
        return d

    async def write(self, data: bytes, fin=False):
        if self.local_closed or self.reset:
            raise ConnectionError(f"stream {self.id} is closed")
        for i in range(0, max(1, len(data)), MAX_FRAME):
            last = i + MAX_FRAME >= len(data)
            await self.conn._send(data_frame(self.id, FLAG_FIN if (fin and last) else 0, data[i:i + MAX_FRAME]))
        if fin:
            self.local_closed = True
            self.conn._forget(self)

    async def close(self):
        """Half-close (FIN) our direction."""
        if not self.local_closed and not self.reset:
            self.local_closed = True
            self.conn._forget(self)
            await self.conn._send(data_frame(self.id, FLAG_FIN, b""))

    async def reply(self, headers=None, fin=False):
        block = self.conn._compress(encode_block(headers or {}))
        await self.conn._send(control_frame(SYN_REPLY, FLAG_FIN if fin else 0, struct.pack(">I", self.id) + block))
        if fin:
            self.local_closed = True
            self.conn._forget(self)

    async def reset_stream(self, status=RST_CANCEL):
        if not self.reset:
            self.reset = True
            self.conn._forget(self)
            await self.conn._send(control_frame(RST_STREAM, 0, struct.pack(">II", self.id, status)))


class Connection:
    """One SPDY session over an asyncio stream pair. `on_stream(stream)` is called for each
    stream the peer opens; `serve()` reads frames until the connection ends."""

    def __init__(self, reader, writer, server=True, on_stream=None):
        self.reader, self.writer, self.server = reader, writer, server
        self.on_stream = on_stream
        self.streams: dict[int, Stream] = {}
        self._next_id = 2 if server else 1
        self._zc = zlib.compressobj(9, zlib.DEFLATED, zlib.MAX_WBITS, 9, zlib.Z_DEFAULT_STRATEGY, DICTIONARY)
        self._zd = zlib.decompressobj(zlib.MAX_WBITS, DICTIONARY)
        self._wlock = asyncio.Lock()
        self.closed = asyncio.Event()
        self.goaway = False
        self.last_peer_sid = 0       # highest stream id the peer opened (GOAWAY's last-good-stream)

    def _forget(self, st):
        """A stream both sides closed (or either reset) no longer counts against MAX_STREAMS:
        the session holds open streams only."""
        if st._done() and self.streams.get(st.id) is st:
            del self.streams[st.id]

    def _compress(self, block: bytes) -> bytes:
        return self._zc.compress(block) + self._zc.flush(zlib.Z_SYNC_FLUSH)

    def _decompress(self, data: bytes) -> bytes:
        out = self._zd.decompress(data, MAX_HEADER_BLOCK)
        if self._zd.unconsumed_tail:
            raise SpdyError(f"header block inflates past {MAX_HEADER_BLOCK} bytes")
        return out

    async def _send(self, frame: bytes):
        async with self._wlock:
            self.writer.write(frame)
            await self.writer.drain()

    async def create_stream(self, headers: dict, fin=False) -> Stream:
        sid = self._next_id
        self._next_id += 2
        st = Stream(self, sid, {k.lower(): (v if isinstance(v, list) else [v]) for k, v in headers.items()})
        self.streams[sid] = st
        body = struct.pack(">IIBB", sid, 0, 0, 0) + self._compress(encode_block(headers))
        await self._send(control_frame(SYN_STREAM, FLAG_FIN if fin else 0, body))
        if fin:
            st.local_closed = True
        return st

    async def ping(self, pid=1):
        await self._send(control_frame(PING, 0, struct.pack(">I", pid)))

    async def close(self, status=0):
        if not self.goaway:
            self.goaway = True
            last = max([s for s in self.streams if (s % 2 == 1) == self.server] + [self.last_peer_sid])
            try:
                await self._send(control_frame(GOAWAY, 0, struct.pack(">II", last, status)))
            except (ConnectionError, RuntimeError):
                pass
        try:
            self.writer.close()
        except RuntimeError:
            pass

    async def serve(self):
        try:
            while True:
                head = await self.reader.readexactly(8)
                if head[0] & 0x80:
                    version, ftype, fl = struct.unpack(">HHI", head)
                    flags, length = fl >> 24, fl & 0xFFFFFF
                    body = await self.reader.readexactly(length)
                    if version & 0x7FFF != VERSION:
                        raise SpdyError(f"unsupported SPDY version {version & 0x7FFF}")
                    await self._control(ftype, flags, body)
                else:
                    sid, fl = struct.unpack(">II", head)
                    flags, length = fl >> 24, fl & 0xFFFFFF
                    payload = await self.reader.readexactly(length)
                    st = self.streams.get(sid & 0x7FFFFFFF)
                    if st is None:
                        await self._send(control_frame(RST_STREAM, 0, struct.pack(">II", sid, RST_INVALID_STREAM)))
                        continue
                    st._feed(payload, flags & FLAG_FIN)
        except (asyncio.IncompleteReadError, ConnectionError, RuntimeError, SpdyError, zlib.error, struct.error):
            pass
        finally:
            for st in list(self.streams.values()):
                st._feed(b"", True)
            self.closed.set()

    async def _control(self, ftype, flags, body):
        if ftype == SYN_STREAM:
            sid = struct.unpack_from(">I", body, 0)[0] & 0x7FFFFFFF
            headers = decode_block(self._decompress(body[10:]))
            if sid in self.streams or self.goaway:
                await self._send(control_frame(RST_STREAM, 0, struct.pack(">II", sid, RST_PROTOCOL_ERROR)))
                return
            if len(self.streams) >= MAX_STREAMS:
                await self._send(control_frame(RST_STREAM, 0, struct.pack(">II", sid, RST_REFUSED_STREAM)))
                return
            st = Stream(self, sid, headers)
            self.streams[sid] = st
            self.last_peer_sid = max(self.last_peer_sid, sid)
            if flags & FLAG_FIN:
                st._feed(b"", True)
            if self.on_stream is not None:
                try:
                    r = self.on_stream(st)
                    if asyncio.iscoroutine(r):
                        await r
                except (ConnectionError, RuntimeError):
                    raise
                except Exception:  # noqa: BLE001 - a handler bug refuses the stream, not the session
                    import logging
                    logging.getLogger("spdy").exception("stream %d handler failed", sid)
                    await st.reset_stream(RST_REFUSED_STREAM)
        elif ftype == SYN_REPLY:
            sid = struct.unpack_from(">I", body, 0)[0] & 0x7FFFFFFF
            decode_block(self._decompress(body[4:]))      # keep the shared zlib stream in step
            st = self.streams.get(sid)
            if st is not None:
                st.replied.set()
                if flags & FLAG_FIN:
                    st._feed(b"", True)
        elif ftype == HEADERS:
            sid = struct.unpack_from(">I", body, 0)[0] & 0x7FFFFFFF
            extra = decode_block(self._decompress(body[4:]))
            st = self.streams.get(sid)
            if st is not None:
                for k, v in extra.items():
                    st.headers.setdefault(k, []).extend(v)
                if flags & FLAG_FIN:
                    st._feed(b"", True)
        elif ftype == RST_STREAM:
            sid = struct.unpack_from(">I", body, 0)[0] & 0x7FFFFFFF
            st = self.streams.get(sid)
            if st is not None:
                st.reset = True
                st._feed(b"", True)
                self._forget(st)
        elif ftype == PING:
            pid = struct.unpack_from(">I", body, 0)[0]
            if (pid % 2 == 1) == self.server:          # the peer's ping: echo it
                await self._send(control_frame(PING, 0, body[:4]))
        elif ftype == GOAWAY:
            self.goaway = True
        # SETTINGS, WINDOW_UPDATE and unknown types: nothing to do (no flow control, as spdystream)


async def connect(url: str, headers=None, protocols=(), ssl=None):
    """Client upgrade -> (Connection, negotiated X-Stream-Protocol-Version). The connection's
    frames are read by a background task."""
    from urllib.parse import urlsplit
    u = urlsplit(url)
    port = u.port or (443 if u.scheme == "https" else 80)
    r, w = await asyncio.open_connection(u.hostname, port, ssl=ssl)
    target = (u.path or "/") + (("?" + u.query) if u.query else "")
    lines = [f"POST {target} HTTP/1.1", f"Host: {u.hostname}:{port}", "Connection: Upgrade", "Upgrade: SPDY/3.1",
             "Content-Length: 0"]
    lines += [f"X-Stream-Protocol-Version: {p}" for p in protocols]
    lines += [f"{k}: {v}" for k, v in (headers or {}).items()]
    w.write(("\r\n".join(lines) + "\r\n\r\n").encode())
    await w.drain()
    head = await r.readuntil(b"\r\n\r\n")
    status_line, _, rest = head.decode("latin-1").partition("\r\n")
    status = int(status_line.split(" ", 2)[1])
    hdrs = {}
    for ln in rest.split("\r\n"):
        k, _, v = ln.partition(":")
        if k:
            hdrs[k.strip().lower()] = v.strip()
    if status != 101:
        n = int(hdrs.get("content-length", "0") or 0)
        body = await r.readexactly(n) if n else b""
        w.close()
        raise SpdyError(f"upgrade refused: HTTP {status}: {body.decode(errors='replace')}")
    conn = Connection(r, w, server=False)
    conn.task = asyncio.ensure_future(conn.serve())
    return conn, hdrs.get("x-stream-protocol-version", "")
