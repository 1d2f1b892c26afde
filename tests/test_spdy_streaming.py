"""exec / port-forward over SPDY/3.1 — the transport of kubectl and client-go 1.9 — through the
API server -> kubelet -> runtime path (in-process runtime and CRI runtime), driven by a client
that opens streams the way client-go's SPDY executor does (`remotecommand/v2.go`/`v4.go`: the
error stream first, then stdin / stdout / stderr, `resize` under a tty; port-forward error+data
pairs with `port` and `requestID`).

Frame and compression details are pinned to the SPDY/3 spec: the header dictionary (1423 bytes,
adler32 0xe3c6a7c2, byte-compared with the vendored spdystream copy when the reference tree is
present), zlib FDICT headers naming that dictionary, and hand-built frames. Parity with a Go
client is unpinned here (no Go toolchain): the wire format follows the vendored
`docker/spdystream` framer read for this test.
"""
import asyncio
import json
import os
import re
import struct
import sys
import zlib
from urllib.parse import quote

import pytest

from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.cri.remote import RemoteRuntime
from kubernetes_amd.cri.server import CRIServer
from kubernetes_amd.kubelet.runtime.process import ProcessRuntime
from kubernetes_amd.utils import spdy

REF_DICT = "/root/reference/vendor/github.com/docker/spdystream/spdy/dictionary.go"


def test_dictionary_and_zlib_preset():
    assert len(spdy.DICTIONARY) == 1423 and zlib.adler32(spdy.DICTIONARY) == 0xE3C6A7C2
    if os.path.exists(REF_DICT):
        src = open(REF_DICT).read()
        body = src[src.index("[]byte{") + 7:src.rindex("}")]
        assert spdy.DICTIONARY == bytes(int(x, 16) for x in re.findall(r"0x([0-9a-fA-F]{2})", body))
    c = spdy.Connection(None, None)
    block = c._compress(spdy.encode_block({"streamType": ["stdout"], "X-Multi": ["a", "b"]}))
    assert block[0] == 0x78 and block[1] & 0x20                  # zlib header with FDICT
    assert struct.unpack(">I", block[2:6])[0] == 0xE3C6A7C2       # ... naming the SPDY dictionary
    d = zlib.decompressobj(zlib.MAX_WBITS, spdy.DICTIONARY)
    assert spdy.decode_block(d.decompress(block)) == {"streamtype": ["stdout"], "x-multi": ["a", "b"]}
    # the second block continues the same zlib stream (no new header)
    block2 = c._compress(spdy.encode_block({}))
    assert block2[:2] != b"\x78\xbb" and spdy.decode_block(d.decompress(block2)) == {}


def test_frame_layout():
    assert spdy.control_frame(spdy.PING, 0, b"\x00\x00\x00\x07") == b"\x80\x03\x00\x06\x00\x00\x00\x04\x00\x00\x00\x07"
    assert spdy.data_frame(5, spdy.FLAG_FIN, b"hi") == b"\x00\x00\x00\x05\x01\x00\x00\x02hi"
    rst = spdy.control_frame(spdy.RST_STREAM, 0, struct.pack(">II", 3, spdy.RST_CANCEL))
    assert rst[:8] == b"\x80\x03\x00\x03\x00\x00\x00\x08"


def test_header_block_bomb_ends_the_session():
    """A SYN_STREAM whose compressed header block inflates past MAX_HEADER_BLOCK ends the session
    (no stream is created, nothing is inflated past the limit); a normal block is still read."""
    async def main(block_bytes):
        c = spdy.Connection(None, None)
        reader = asyncio.StreamReader()
        peer = spdy.Connection(None, None)
        blk = peer._compress(block_bytes)
        reader.feed_data(spdy.control_frame(spdy.SYN_STREAM, 0, struct.pack(">IIBB", 1, 0, 0, 0) + blk))
        reader.feed_eof()
        c.reader = reader
        c.server = True
        seen = []
        c.on_stream = seen.append
        await asyncio.wait_for(c.serve(), 5)
        return seen
    big = spdy.encode_block({"x": ["a" * (2 * spdy.MAX_HEADER_BLOCK)]})
    assert asyncio.run(main(big)) == []
    ok = asyncio.run(main(spdy.encode_block({"streamtype": ["error"]})))
    assert len(ok) == 1 and ok[0].headers["streamtype"] == ["error"]


def test_session_outlives_max_streams_sequential_streams():
    """the MAX_STREAMS cap counts open streams only. One session opens and closes
    2 * MAX_STREAMS + 10 streams one after another (client FIN + server FIN, or a reset) and
    every one is served; the session tracks no closed stream."""
    async def main():
        served = []

        async def on_stream(st):
            async def echo():
                d = await st.read()
                if not st.reset:
                    await st.write(b"re:" + d, fin=True)
            served.append(asyncio.ensure_future(echo()))

        srv_box = {}

        async def handler(r, w):
            c = spdy.Connection(r, w, server=True, on_stream=on_stream)
            srv_box["c"] = c
            await c.serve()
        server = await asyncio.start_server(handler, "127.0.0.1", 0)
        port = server.sockets[0].getsockname()[1]
        r, w = await asyncio.open_connection("127.0.0.1", port)
        cli = spdy.Connection(r, w, server=False)
        task = asyncio.ensure_future(cli.serve())
        n = 2 * spdy.MAX_STREAMS + 10
        for i in range(n):
            st = await cli.create_stream({"streamtype": "data", "i": str(i)})
            if i % 7 == 3:
                await st.reset_stream()
                continue
            await st.write(b"x%d" % i, fin=True)
            assert await st.read() == b"re:x%d" % i
        await asyncio.sleep(0.05)
        assert len(srv_box["c"].streams) == 0 and len(cli.streams) == 0
        assert len(served) == n
        await cli.close()
        task.cancel()
        server.close()
    asyncio.run(asyncio.wait_for(main(), 60))


SLEEPER = "import time\nwhile True: time.sleep(1)\n"
ECHO = ("import socket,sys\n"
        "s=socket.socket(); s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)\n"
        "s.bind(('127.0.0.1', int(sys.argv[1]))); s.listen(8)\n"
        "while True:\n"
        "    c,_=s.accept(); d=c.recv(100)\n"
        "    if d: c.sendall(b'pong:'+d)\n"
        "    c.close()\n")


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


async def _pod(cl, node):
    port = _free_port()
    await cl.client.create("pods", {"metadata": {"name": "w", "namespace": "default"}, "spec": {"nodeName": node, "containers": [
        {"name": "main", "image": "busybox", "command": [sys.executable, "-c", SLEEPER]},
        {"name": "echo", "image": "busybox", "command": [sys.executable, "-c", ECHO, str(port)]}]}})
    await cl.wait_pod("w")
    for _ in range(250):
        try:
            _r, w = await asyncio.open_connection("127.0.0.1", port)
            w.close()
            break
        except OSError:
            await asyncio.sleep(0.02)
    return port


async def _drain(st):
    out = b""
    while True:
        d = await st.read()
        if not d:
            return out
        out += d


async def _exec(url, cmd, stdin=b"", protocols=("v4.channel.k8s.io", "v3.channel.k8s.io", "v2.channel.k8s.io",
                                                  "channel.k8s.io")):
    q = "&".join(f"command={quote(c)}" for c in cmd) + "&container=main&stdin=true&stdout=true&stderr=true"
    conn, proto = await spdy.connect(f"{url}/api/v1/namespaces/default/pods/w/exec?{q}", protocols=protocols)
    try:
        err = await conn.create_stream({"streamType": "error"})
        sin = await conn.create_stream({"streamType": "stdin"})
        sout = await conn.create_stream({"streamType": "stdout"})
        serr = await conn.create_stream({"streamType": "stderr"})
        await asyncio.wait_for(asyncio.gather(*(s.replied.wait() for s in (err, sin, sout, serr))), 10)
        if stdin:
            await sin.write(stdin)
        await sin.close()
        out, errout, status = await asyncio.wait_for(asyncio.gather(_drain(sout), _drain(serr), _drain(err)), 20)
        return proto, out, errout, status
    finally:
        await conn.close()
        conn.task.cancel()


async def _portforward(url, port):
    conn, proto = await spdy.connect(f"{url}/api/v1/namespaces/default/pods/w/portforward",
                                     protocols=("portforward.k8s.io",))
    try:
        hdr = {"port": str(port), "requestID": "0"}
        err = await conn.create_stream(dict(hdr, streamType="error"))
        data = await conn.create_stream(dict(hdr, streamType="data"))
        await data.write(b"spdy")
        got = await asyncio.wait_for(_drain(data), 10)
        return proto, got, await asyncio.wait_for(_drain(err), 10)
    finally:
        await conn.close()
        conn.task.cancel()


def _check_exec(result, proto="v4.channel.k8s.io"):
    got_proto, out, errout, status = result
    assert got_proto == proto
    assert out == b"got:line\n" and errout == b"warn\n"
    st = json.loads(status)
    assert st["reason"] == "NonZeroExitCode" and st["details"]["causes"] == [{"reason": "ExitCode", "message": "6"}]


SCRIPT = ["sh", "-c", "read x; echo got:$x; echo warn >&2; exit 6"]


def test_spdy_exec_and_portforward_inprocess(run, tmp_path):
    async def main():
        cl = LocalCluster(nodes=1, gpus_per_node=0, runtime="process", kubelet_http=True, workdir=str(tmp_path / "c"))
        await cl.start()
        try:
            port = await _pod(cl, cl.nodes[0].name)
            _check_exec(await _exec(cl.url, SCRIPT, b"line\n"))
            # pre-v4 protocol: failures are a bare message, success writes nothing
            proto, out, _e, status = await _exec(cl.url, ["sh", "-c", "exit 2"], protocols=("v2.channel.k8s.io",))
            assert proto == "v2.channel.k8s.io" and b"non-zero exit code: 2" in status
            proto, out, _e, status = await _exec(cl.url, ["echo", "ok"], protocols=("v3.channel.k8s.io",))
            assert out == b"ok\n" and status == b""
            proto, got, err = await _portforward(cl.url, port)
            assert proto == "portforward.k8s.io" and got == b"pong:spdy" and err == b""
            # unsupported protocol -> 403 listing what the server accepts
            with pytest.raises(spdy.SpdyError, match="403"):
                await spdy.connect(f"{cl.url}/api/v1/namespaces/default/pods/w/exec?command=true&stdout=true",
                                   protocols=("v9.channel.k8s.io",))
        finally:
            await cl.stop()
    run(main(), timeout=90)


def test_spdy_exec_and_portforward_over_cri(run, tmp_path):
    async def main():
        sock = str(tmp_path / "cri.sock")
        prt = ProcessRuntime(str(tmp_path / "rt"))
        srv = await CRIServer(prt, sock).start()
        rt = await RemoteRuntime(sock, relist_period=0.1).connect()
        cl = LocalCluster(nodes=0, gpus_per_node=0, kubelet_http=True, workdir=str(tmp_path / "c"))
        await cl.start()
        try:
            await cl.add_node("cri-node", runtime=rt)
            port = await _pod(cl, "cri-node")
            _check_exec(await _exec(cl.url, SCRIPT, b"line\n"))
            proto, got, err = await _portforward(cl.url, port)
            assert got == b"pong:spdy"
        finally:
            await cl.stop()
            await rt.close()
            await srv.stop()
            await prt.kill_all()
    run(main(), timeout=90)
