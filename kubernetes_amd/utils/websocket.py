"""WebSocket (RFC 6455) transport and the Kubernetes channel sub-protocols.

Parity: `staging/src/k8s.io/apiserver/pkg/util/wsstream/conn.go` —
  * sub-protocols `channel.k8s.io` (each binary message = 1 channel byte + payload) and
    `base64.channel.k8s.io` (text messages: ASCII channel digit + base64 payload), plus the v4
    variants `v4.channel.k8s.io` / `v4.base64.channel.k8s.io` of remotecommand
    (`pkg/kubelet/server/remotecommand/websocket.go:36-40`), whose error channel carries a JSON
    metav1.Status instead of a bare message;
  * handshake: the first client-offered protocol that the server supports wins, no offer selects
    the "" (binary) protocol (`conn.go:111-127`);
  * `IsWebSocketRequest`: `Upgrade: websocket` and a `Connection` header containing upgrade
    (`conn.go:89-94`).

The frame codec is asyncio-native (StreamReader/StreamWriter over the upgraded HTTP
connection). Server frames are unmasked, client frames masked; ping is answered with pong,
fragmented messages are reassembled, close is echoed.
"""
from __future__ import annotations

import asyncio
import base64
import hashlib
import os
import struct
from urllib.parse import urlsplit

GUID = b"258EAFA5-E914-47DA-95CA-C5AB0DC85B11"

CHANNEL = "channel.k8s.io"
BASE64_CHANNEL = "base64.channel.k8s.io"
V4_CHANNEL = "v4." + CHANNEL
V4_BASE64_CHANNEL = "v4." + BASE64_CHANNEL

OP_CONT, OP_TEXT, OP_BINARY, OP_CLOSE, OP_PING, OP_PONG = 0x0, 0x1, 0x2, 0x8, 0x9, 0xA
MAX_MESSAGE = 64 << 20


class WebSocketError(Exception):
    pass


def accept_key(key: str) -> str:
    return base64.b64encode(hashlib.sha1(key.encode() + GUID).digest()).decode()


def is_websocket_request(headers) -> bool:
    if headers.get("upgrade", "").lower() != "websocket":
        return False
    return "upgrade" in [t.strip() for t in headers.get("connection", "").lower().split(",")]


def negotiate(headers, supported) -> str | None:
    """The sub-protocol to use, or None if the client offered only unsupported ones."""
    offered = [p.strip() for p in headers.get("sec-websocket-protocol", "").split(",") if p.strip()] or [""]
    for p in offered:
        if p in supported:
            return p
    return None


def handshake_headers(headers, protocol: str) -> dict:
    """Extra headers of the server's `101 Switching Protocols` reply."""
    out = {"Sec-WebSocket-Accept": accept_key(headers.get("sec-websocket-key", ""))}
    if protocol:
        out["Sec-WebSocket-Protocol"] = protocol
    return out


class WebSocket:
    """One RFC 6455 connection over an asyncio stream pair. `client=True` masks outgoing frames."""

    def __init__(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter, client=False):
        self.reader, self.writer, self.client = reader, writer, client
        self.closed = False
        self._wlock = asyncio.Lock()

    async def _send_frame(self, op, payload: bytes):
        n = len(payload)
        head = bytearray([0x80 | op])
        mask_bit = 0x80 if self.client else 0
        if n < 126:
            head.append(mask_bit | n)
        elif n < 1 << 16:
            head.append(mask_bit | 126)
            head += struct.pack("!H", n)
        else:
            head.append(mask_bit | 127)
            head += struct.pack("!Q", n)
        if self.client:
            key = os.urandom(4)
            head += key
            payload = _mask(payload, key)
        async with self._wlock:
            self.writer.write(bytes(head) + payload)
            await self.writer.drain()

    async def send(self, data, binary=True):
        if self.closed:
            raise ConnectionError("websocket closed")
        if isinstance(data, str):
            data, binary = data.encode(), False
        await self._send_frame(OP_BINARY if binary else OP_TEXT, bytes(data))

    async def close(self, code=1000, reason=b""):
        if self.closed:
            return
        self.closed = True
        try:
            await self._send_frame(OP_CLOSE, struct.pack("!H", code) + reason)
        except (ConnectionError, RuntimeError):
            pass

    async def _read_frame(self):
        b0, b1 = await self.reader.readexactly(2)
        fin, op, masked, n = b0 & 0x80, b0 & 0x0F, b1 & 0x80, b1 & 0x7F
        if n == 126:
            n = struct.unpack("!H", await self.reader.readexactly(2))[0]
        elif n == 127:
            n = struct.unpack("!Q", await self.reader.readexactly(8))[0]
        if n > MAX_MESSAGE:
            raise WebSocketError(f"frame of {n} bytes exceeds the limit")
        key = await self.reader.readexactly(4) if masked else None
        payload = await self.reader.readexactly(n)
        if key:
            payload = _mask(payload, key)
        return bool(fin), op, payload

    async def recv(self):
        """-> (is_binary, payload) of the next data message, or None once the peer closed."""
        parts, first_op = [], None
        while True:
            try:
                fin, op, payload = await self._read_frame()
            except (asyncio.IncompleteReadError, ConnectionError):
                self.closed = True
                return None
            if op == OP_PING:
                await self._send_frame(OP_PONG, payload)
                continue
            if op == OP_PONG:
                continue
            if op == OP_CLOSE:
                if not self.closed:
                    self.closed = True
                    try:
                        await self._send_frame(OP_CLOSE, payload[:2])
                    except (ConnectionError, RuntimeError):
                        pass
                return None
            if op != OP_CONT:
                first_op = op
            parts.append(payload)
            if sum(map(len, parts)) > MAX_MESSAGE:
                raise WebSocketError("message exceeds the limit")
            if fin:
                return first_op == OP_BINARY, b"".join(parts)


def _mask(data: bytes, key: bytes) -> bytes:
    if not data:
        return data
    n = len(data)
    k = (key * (n // 4 + 1))[:n]
    return (int.from_bytes(data, "little") ^ int.from_bytes(k, "little")).to_bytes(n, "little")


class ChannelConn:
    """The channel multiplexing of `wsstream.Conn` over one WebSocket: `write(ch, data)`;
    `read()` -> (channel, data) or None at close. base64 protocols send text frames with an
    ASCII channel digit."""

    def __init__(self, ws: WebSocket, protocol: str):
        self.ws, self.protocol = ws, protocol
        self.base64 = protocol.endswith(BASE64_CHANNEL)
        self.v4 = protocol.startswith("v4.")

    async def write(self, ch: int, data: bytes = b""):
        if self.base64:
            await self.ws.send(chr(ord("0") + ch) + base64.b64encode(data).decode(), binary=False)
        else:
            await self.ws.send(bytes([ch]) + bytes(data))

    async def read(self):
        while True:
            msg = await self.ws.recv()
            if msg is None:
                return None
            _binary, data = msg
            if not data:
                continue
            if self.base64:
                return data[0] - ord("0"), base64.b64decode(data[1:])
            return data[0], data[1:]

    async def close(self):
        await self.ws.close()


async def connect(url: str, protocols=(V4_CHANNEL,), headers=None, ssl=None):
    """Client handshake -> (ChannelConn, negotiated protocol). Raises WebSocketError with the
    HTTP status and body when the server refuses the upgrade."""
    u = urlsplit(url)
    port = u.port or (443 if u.scheme in ("https", "wss") else 80)
    r, w = await asyncio.open_connection(u.hostname, port, ssl=ssl)
    key = base64.b64encode(os.urandom(16)).decode()
    target = (u.path or "/") + (("?" + u.query) if u.query else "")
    lines = [f"GET {target} HTTP/1.1", f"Host: {u.hostname}:{port}", "Connection: Upgrade", "Upgrade: websocket",
             "Sec-WebSocket-Version: 13", f"Sec-WebSocket-Key: {key}"]
    if protocols:
        lines.append("Sec-WebSocket-Protocol: " + ", ".join(protocols))
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
        body = b""
        try:
            n = int(hdrs.get("content-length", "0") or 0)
            body = await asyncio.wait_for(r.readexactly(n) if n else r.read(65536), 2.0)
        except (asyncio.TimeoutError, asyncio.IncompleteReadError, ConnectionError):
            pass
        w.close()
        raise WebSocketError(f"upgrade refused: HTTP {status}: {body.decode(errors='replace').strip()}")
    if hdrs.get("sec-websocket-accept") != accept_key(key):
        w.close()
        raise WebSocketError("bad Sec-WebSocket-Accept")
    proto = hdrs.get("sec-websocket-protocol", "")
    return ChannelConn(WebSocket(r, w, client=True), proto), proto
