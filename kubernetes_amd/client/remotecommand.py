"""Client side of exec / attach / port-forward over WebSocket (client-go `tools/remotecommand`
and `tools/portforward` semantics on the `channel.k8s.io` protocols; see `cri/remotecommand.py`
for the server side).

  * `exec_stream` offers `v5.channel.k8s.io` (stdin EOF via the close channel), then
    `v4.channel.k8s.io` and `channel.k8s.io`; the exit code comes from the v4 status JSON on
    channel 3 (reason NonZeroExitCode, cause ExitCode), or from the bare error message of the
    pre-v4 protocols;
  * `PortForwarder` opens one WebSocket per accepted local connection with a data/error channel
    pair for the remote port (the first two bytes of each channel are the port, little-endian).
"""
from __future__ import annotations

import asyncio
import base64
import json
import os

from ..cri.remotecommand import CLOSE, ERROR, RESIZE, STDERR, STDIN, STDOUT, V5_CHANNEL, rc_from_status
from ..utils.websocket import CHANNEL, V4_CHANNEL, ChannelConn, WebSocket, WebSocketError, accept_key

EXEC_OFFER = (V5_CHANNEL, V4_CHANNEL, CHANNEL)


class StreamError(Exception):
    def __init__(self, status, message):
        super().__init__(f"HTTP {status}: {message}")
        self.status, self.message = status, message


async def ws_open(http, path, protocols=EXEC_OFFER):
    """WebSocket handshake through an HTTPClient (its TLS and credentials) -> (ChannelConn, protocol)."""
    from .http import _read_body
    key = base64.b64encode(os.urandom(16)).decode()
    st, hdrs, r, w = await http.open_raw("GET", path, {
        "Connection": "Upgrade", "Upgrade": "websocket", "Sec-WebSocket-Version": "13",
        "Sec-WebSocket-Key": key, "Sec-WebSocket-Protocol": ", ".join(protocols)})
    if st != 101:
        try:
            body = await asyncio.wait_for(_read_body(r, hdrs), 5.0)
        except (asyncio.TimeoutError, asyncio.IncompleteReadError, ConnectionError, ValueError):
            body = b""
        w.close()
        try:
            msg = json.loads(body).get("message", body.decode(errors="replace"))
        except (ValueError, AttributeError):
            msg = body.decode(errors="replace")
        raise StreamError(st, msg)
    if hdrs.get("sec-websocket-accept") != accept_key(key):
        w.close()
        raise WebSocketError("bad Sec-WebSocket-Accept")
    proto = hdrs.get("sec-websocket-protocol", "")
    return ChannelConn(WebSocket(r, w, client=True), proto), proto


async def exec_stream(http, path, stdin=None, stdout=None, stderr=None, resize=None) -> int:
    """Run an exec/attach WebSocket session. stdin / resize: async iterators of bytes /
    (width, height); stdout / stderr: callables taking bytes (sync or async). -> exit code."""
    conn, proto = await ws_open(http, path)
    v4 = proto.startswith("v4.") or proto == V5_CHANNEL
    rc = None

    async def send_stdin():
        async for d in stdin:
            await conn.write(STDIN, d)
        if proto == V5_CHANNEL:
            await conn.write(CLOSE, bytes([STDIN]))

    async def send_resize():
        async for w, h in resize:
            await conn.write(RESIZE, json.dumps({"Width": w, "Height": h}).encode())

    async def emit(sink, d):
        if sink is not None and d:
            r = sink(d)
            if asyncio.iscoroutine(r):
                await r
    tasks = []
    if stdin is not None:
        tasks.append(asyncio.ensure_future(send_stdin()))
    if resize is not None:
        tasks.append(asyncio.ensure_future(send_resize()))
    try:
        while True:
            m = await conn.read()
            if m is None:
                break
            ch, data = m
            if ch == STDOUT:
                await emit(stdout, data)
            elif ch == STDERR:
                await emit(stderr, data)
            elif ch == ERROR and data:
                if v4:
                    rc = rc_from_status(data)
                else:
                    rc = 1
                    await emit(stderr, data)
    finally:
        for t in tasks:
            t.cancel()
        await conn.close()
    return 0 if rc is None else rc


async def exec_collect(http, path, stdin_data: bytes | None = None):
    """-> (exit code, stdout, stderr) of a non-interactive exec (optionally feeding stdin_data)."""
    out, err = bytearray(), bytearray()
    src = None
    if stdin_data is not None:
        async def src_gen():
            for i in range(0, len(stdin_data), 1 << 16):
                yield stdin_data[i:i + (1 << 16)]
        src = src_gen()
    rc = await exec_stream(http, path, src, out.extend, err.extend)
    return rc, bytes(out), bytes(err)


async def forward_connection(http, path, port, reader, writer):
    """Splice one accepted local connection onto a port-forward WebSocket for `port`."""
    conn, _ = await ws_open(http, path, (V4_CHANNEL, ""))
    seen = {0: False, 1: False}

    async def up():
        try:
            while True:
                d = await reader.read(65536)
                if not d:
                    break
                await conn.write(0, d)
        except ConnectionError:
            pass
        await conn.close()          # local side closed: end the remote connection too
    t = asyncio.ensure_future(up())
    try:
        while True:
            m = await conn.read()
            if m is None:
                break
            ch, data = m
            if ch in seen and not seen[ch]:
                seen[ch] = True             # the port header of each channel
                data = data[2:]
            if ch == 0 and data:
                writer.write(data)
                await writer.drain()
            elif ch == 1 and data:
                raise StreamError(500, data.decode(errors="replace"))
    finally:
        t.cancel()
        await conn.close()
        try:
            writer.close()
        except RuntimeError:
            pass
