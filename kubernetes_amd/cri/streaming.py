"""Client side of the CRI streaming server (see `server.StreamingServer` for the protocol).

Parity: what `kubectl exec` / `kubectl port-forward` do over SPDY against the kubelet's
streaming URLs (`pkg/kubelet/server/remotecommand`, `pkg/kubelet/server/portforward`),
reduced to a framed chunked stream for exec and an HTTP `Upgrade: tcp` tunnel for port-forward.
"""
from __future__ import annotations

import asyncio
from urllib.parse import urlsplit


async def _open(url, headers="", ssl_context=None):
    u = urlsplit(url)
    ssl = None
    if u.scheme == "https":
        from ..utils.tlsutil import unverified_client_context
        ssl = ssl_context or unverified_client_context()
    r, w = await asyncio.open_connection(u.hostname, u.port or (443 if ssl else 80), ssl=ssl)
    target = u.path + (("?" + u.query) if u.query else "")
    w.write(f"GET {target} HTTP/1.1\r\nHost: {u.hostname}:{u.port}\r\n{headers}\r\n".encode())
    await w.drain()
    head = await r.readuntil(b"\r\n\r\n")
    status = int(head.split(b" ", 2)[1])
    return r, w, status, head


async def read_frames(r):
    """Decode a chunked body of exec frames -> (exit code, stdout, stderr)."""
    out, err, rc = bytearray(), bytearray(), None
    while True:
        size = int((await r.readuntil(b"\r\n")).strip(), 16)
        if size == 0:
            break
        data = await r.readexactly(size)
        await r.readexactly(2)
        ch, payload = data[0], data[1:]
        if ch == 1:
            out += payload
        elif ch == 2:
            err += payload
        elif ch == 3:
            rc = int(payload)
    return (rc if rc is not None else -1), bytes(out), bytes(err)


async def read_exec_stream(url):
    """Run an exec URL to completion -> (exit code, stdout+stderr)."""
    r, w, status, _ = await _open(url)
    try:
        if status != 200:
            raise ConnectionError(f"exec stream refused: HTTP {status}")
        rc, out, err = await read_frames(r)
        return rc, out + err
    finally:
        w.close()


async def open_port_forward(url, port, ssl_context=None):
    """Upgrade a port-forward URL into a raw tunnel -> (reader, writer)."""
    sep = "&" if "?" in url else "?"
    r, w, status, _ = await _open(f"{url}{sep}port={port}", "Connection: Upgrade\r\nUpgrade: tcp\r\n", ssl_context)
    if status != 101:
        w.close()
        raise ConnectionError(f"port-forward refused: HTTP {status}")
    return r, w
