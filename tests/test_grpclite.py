"""grpclite: HPACK/Huffman against RFC 7541's examples, and wire interop with grpc-core (grpc.aio)
in both directions over the device-plugin services (unary, server streaming, errors, deadlines,
flow control with messages larger than the default windows and frame size)."""
import asyncio
import os
import struct
import tempfile

import grpc
import pytest

from kubernetes_amd.deviceplugin import api
from kubernetes_amd.deviceplugin.server import DevicePluginServer, device
from kubernetes_amd.utils import grpclite as gl


# -- RFC 7541 ---------------------------------------------------------------------------------

@pytest.mark.parametrize("text,hexcode", [
    (b"www.example.com", "f1e3c2e5f23a6ba0ab90f4ff"),         # C.4.1
    (b"no-cache", "a8eb10649cbf"),                            # C.4.2
    (b"custom-key", "25a849e95ba97d7f"),                      # C.4.3
    (b"custom-value", "25a849e95bb8e8b4bf"),
    (b"302", "6402"),                                          # C.6.1
    (b"private", "aec3771a4b"),
])
def test_huffman_rfc_vectors(text, hexcode):
    assert gl.huffman_encode(text).hex() == hexcode
    assert gl.huffman_decode(bytes.fromhex(hexcode)) == text


def test_huffman_every_byte_round_trips_and_bad_padding_is_rejected():
    data = bytes(range(256)) * 3
    assert gl.huffman_decode(gl.huffman_encode(data)) == data
    codes = gl.huffman_codes()
    assert codes[0] == (0x1ff8, 13) and codes[ord(" ")] == (0x14, 6) and codes[256] == (0x3fffffff, 30)
    with pytest.raises(ValueError):
        gl.huffman_decode(b"\x00")        # '0' (00000) then 3 zero bits: padding must be ones
    with pytest.raises(ValueError):
        gl.huffman_decode(b"\xff\xff\xff\xff")   # EOS inside the string


def test_hpack_decoder_rfc_request_sequences():
    # C.3: requests without Huffman; C.4: the same with Huffman — dynamic table carried over
    for seq in (["828684410f7777772e6578616d706c652e636f6d",
                 "828684be58086e6f2d6361636865",
                 "828785bf400a637573746f6d2d6b65790c637573746f6d2d76616c7565"],
                ["828684418cf1e3c2e5f23a6ba0ab90f4ff",
                 "828684be5886a8eb10649cbf",
                 "828785bf408825a849e95ba97d7f8925a849e95bb8e8b4bf"]):
        d = gl.HpackDecoder()
        r1 = d.decode(bytes.fromhex(seq[0]))
        assert r1 == [(":method", "GET"), (":scheme", "http"), (":path", "/"), (":authority", "www.example.com")]
        assert d.dyn_size == 57
        r2 = d.decode(bytes.fromhex(seq[1]))
        assert r2[-1] == ("cache-control", "no-cache") and r2[3] == (":authority", "www.example.com")
        assert d.dyn_size == 110
        r3 = d.decode(bytes.fromhex(seq[2]))
        assert r3 == [(":method", "GET"), (":scheme", "https"), (":path", "/index.html"),
                      (":authority", "www.example.com"), ("custom-key", "custom-value")]
        assert d.dyn_size == 164
        assert list(d.dyn) == [("custom-key", "custom-value"), ("cache-control", "no-cache"),
                               (":authority", "www.example.com")]


def test_hpack_eviction_and_cached_blocks_follow_the_table():
    d = gl.HpackDecoder(max_size=100)
    d.decode(bytes.fromhex("400a637573746f6d2d6b65790c637573746f6d2d76616c7565"))  # 54 bytes
    ref = bytes.fromhex("be")                    # index 62: newest dynamic entry
    assert d.decode(ref) == [("custom-key", "custom-value")]
    d.decode(bytes.fromhex("4003616263036465660a"[:-2]))   # literal abc: def (38) -> total 92
    assert d.decode(ref) == [("abc", "def")]    # same bytes, new meaning: the cache must not answer
    d.decode(bytes.fromhex("20"))                # size update to 0: evicts both
    assert d.dyn_size == 0
    with pytest.raises(ValueError):
        d.decode(ref)
    with pytest.raises(ValueError):
        d.decode(bytes.fromhex("3fe101"))        # above the advertised maximum


def test_encoded_headers_decode_and_timeouts():
    hdrs = [(":path", "/deviceplugin.DevicePlugin/AdmitPod"), ("content-type", "application/grpc"),
            ("grpc-timeout", gl._timeout_value(1.5)), ("x-custom", "v" * 300)]
    assert gl.HpackDecoder().decode(gl.encode_headers(hdrs)) == hdrs
    assert abs(gl.parse_timeout(gl._timeout_value(1.5)) - 1.5) < 1e-6
    assert gl.parse_timeout(gl._timeout_value(10)) == pytest.approx(10)
    assert len(gl._timeout_value(1e9)) <= 9


# -- interop with grpc-core --------------------------------------------------------------------

class _Plugin(DevicePluginServer):
    async def admit_pod(self, request):
        if request.pod_name == "boom":
            raise RuntimeError("plugin exploded")
        if request.pod_name == "deny":
            raise gl.RpcError(gl.StatusCode.FAILED_PRECONDITION, "no: 100% busy")
        return {"amd.com/admitted": request.pod_name, "n": str(sum(len(c.devices) for c in request.containers.values()))}

    async def init_container(self, container):
        if container.name == "slow":
            await asyncio.sleep(2)
        return {"envs": {"HIP_VISIBLE_DEVICES": ",".join(container.devices)},
                "devices": [{"container_path": "/dev/dri/renderD128", "host_path": "/dev/dri/renderD128",
                             "permissions": "rw"}]}


def _many_devices(n):
    return [device(f"gpu-{i:05d}", attributes={"amd.com/xgmi-peers": ",".join(str(j) for j in range(32)),
                                                "pad": "x" * 64}) for i in range(n)]


def _client(kind, path):
    if kind == "grpc":
        return grpc.aio.insecure_channel("unix://" + path)
    return gl.Channel("unix://" + path)


@pytest.mark.parametrize("server_t,client_t", [("lite", "grpc"), ("grpc", "lite"), ("lite", "lite")])
def test_device_plugin_calls_interoperate(server_t, client_t):
    async def main():
        d = tempfile.mkdtemp()
        sock = os.path.join(d, "p.sock")
        plugin = await _Plugin("amd.com/gpu", sock, [device("g0"), device("g1")], init_timeout=7,
                               labels={"amd.com/model": "MI355X"}, transport=server_t).start()
        ch = _client(client_t, sock)
        errors = (grpc.aio.AioRpcError,) if client_t == "grpc" else (gl.RpcError,)
        try:
            dp = api.device_plugin_stub(ch)
            ident = api.identity_stub(ch)
            info = await dp.GetPluginInfo(api.DP["GetPluginInfoRequest"](), timeout=2)
            assert info.init_timeout == 7 and dict(info.labels) == {"amd.com/model": "MI355X"}
            vs = await ident.GetSupportedVersions(api.PR["GetSupportedVersionsRequest"](), timeout=2)
            assert list(vs.supported_versions) == [api.VERSION]
            await ident.PluginRegistrationStatus(api.PR["RegistrationStatus"](success=True), timeout=2)
            assert plugin.registered.is_set()

            # many concurrent unary calls on one connection
            reqs = []
            for i in range(300):
                r = api.DP["AdmitPodRequest"](pod_name=f"p{i}")
                r.containers["c"].name = "c"
                r.containers["c"].devices.extend(["g0", "g1"][: 1 + i % 2])
                reqs.append(r)
            resps = await asyncio.gather(*[dp.AdmitPod(r, timeout=5) for r in reqs])
            for i, r in enumerate(resps):
                assert r.pod.annotations["amd.com/admitted"] == f"p{i}" and r.pod.annotations["n"] == str(1 + i % 2)
            assert plugin.admit_calls == 300

            ic = api.DP["InitContainerRequest"]()
            ic.container.name = "main"
            ic.container.devices.extend(["g1"])
            spec = (await dp.InitContainer(ic, timeout=2)).spec
            assert spec.envs["HIP_VISIBLE_DEVICES"] == "g1" and spec.devices[0].permissions == "rw"

            # handler errors: UNKNOWN for an exception, the status a handler aborts with (message
            # percent-encoding round trip), DEADLINE_EXCEEDED for a slow handler
            with pytest.raises(errors) as ei:
                await dp.AdmitPod(api.DP["AdmitPodRequest"](pod_name="boom"), timeout=2)
            assert ei.value.code().name == "UNKNOWN"
            if server_t == "lite":
                with pytest.raises(errors) as ei:
                    await dp.AdmitPod(api.DP["AdmitPodRequest"](pod_name="deny"), timeout=2)
                assert ei.value.code().name == "FAILED_PRECONDITION" and ei.value.details() == "no: 100% busy"
            slow = api.DP["InitContainerRequest"]()
            slow.container.name = "slow"
            with pytest.raises(errors) as ei:
                await dp.InitContainer(slow, timeout=0.2)
            assert ei.value.code().name == "DEADLINE_EXCEEDED"

            # unknown method
            bogus = ch.unary_unary("/deviceplugin.DevicePlugin/Nope", request_serializer=lambda m: m.SerializeToString(),
                                   response_deserializer=api.DP["GetPluginInfoResponse"].FromString)
            with pytest.raises(errors) as ei:
                await bogus(api.DP["GetPluginInfoRequest"](), timeout=2)
            assert ei.value.code().name == "UNIMPLEMENTED"

            # server streaming: initial list, an update larger than the default 64 KiB windows and
            # 16 KiB frames (flow control and DATA splitting both ways), then cancel
            call = dp.ListAndWatch(api.DP["ListAndWatchRequest"]())
            it = call.__aiter__()
            first = await asyncio.wait_for(it.__anext__(), 5)
            assert [x.ID for x in first.devices] == ["g0", "g1"]
            big = _many_devices(3000)
            for k in range(3):
                plugin.update(big[: 1000 * (k + 1)])
                upd = await asyncio.wait_for(it.__anext__(), 10)
                assert len(upd.devices) == 1000 * (k + 1) and upd.devices[-1].Attributes["pad"] == "x" * 64
            assert len(big[0].SerializeToString()) * 3000 > 4 * 65535
            call.cancel()
            with pytest.raises(asyncio.CancelledError):
                await asyncio.wait_for(it.__anext__(), 5)
            # large unary request (client -> server flow control)
            r = api.DP["AdmitPodRequest"](pod_name="big")
            for i in range(2000):
                r.containers[f"c{i}"].name = f"c{i}"
                r.containers[f"c{i}"].devices.extend([f"gpu-{i}-{j}-{'y' * 40}" for j in range(4)])
            assert len(r.SerializeToString()) > 300_000
            resp = await dp.AdmitPod(r, timeout=10)
            assert resp.pod.annotations["n"] == "8000"
        finally:
            await ch.close()
            await plugin.stop()
    asyncio.run(main())


def test_lite_client_errors_on_missing_server_and_server_stop():
    async def main():
        d = tempfile.mkdtemp()
        sock = os.path.join(d, "none.sock")
        ch = gl.Channel("unix://" + sock)
        dp = api.device_plugin_stub(ch)
        with pytest.raises(gl.RpcError) as ei:
            await dp.GetPluginInfo(api.DP["GetPluginInfoRequest"](), timeout=1)
        assert ei.value.code() == gl.StatusCode.UNAVAILABLE
        plugin = await _Plugin("amd.com/gpu", sock, [device("g0")]).start()
        info = await dp.GetPluginInfo(api.DP["GetPluginInfoRequest"](), timeout=1)   # re-dials
        assert info.init_timeout == 10
        call = dp.ListAndWatch(api.DP["ListAndWatchRequest"]())
        it = call.__aiter__()
        await asyncio.wait_for(it.__anext__(), 5)
        await plugin.stop()
        # the stream ends (server stopped): StopAsyncIteration or UNAVAILABLE, never a hang
        try:
            await asyncio.wait_for(it.__anext__(), 5)
        except (StopAsyncIteration, gl.RpcError):
            pass
        await ch.close()
    asyncio.run(main())


def test_lite_server_survives_malformed_peers():
    """A bad preface, a garbage frame, an HPACK block with an invalid index or a bad Huffman
    string ends only that connection (GOAWAY PROTOCOL_ERROR); the server keeps serving."""
    async def main():
        d = tempfile.mkdtemp()
        sock = os.path.join(d, "p.sock")
        plugin = await _Plugin("amd.com/gpu", sock, [device("g0")]).start()
        try:
            bad = [b"GET / HTTP/1.1\r\nHost: x\r\n\r\n" + b"\0" * 32,
                   gl.PREFACE + gl._HDR.pack((4 << 8) | gl.HEADERS, gl.F_END_HEADERS, 2) + b"\xff\xff\xff\xff",
                   gl.PREFACE + gl._HDR.pack((1 << 8) | gl.HEADERS, gl.F_END_HEADERS | gl.F_END_STREAM, 1) + b"\xfe",
                   gl.PREFACE + gl._HDR.pack((3 << 8) | gl.HEADERS, gl.F_END_HEADERS, 1) + b"\x00\x81\x00",
                   gl.PREFACE + gl._HDR.pack((6 << 8) | gl.WINDOW_UPDATE, 0, 0) + b"\x00" * 6]
            for payload in bad:
                r, w = await asyncio.open_unix_connection(sock)
                w.write(payload)
                await w.drain()
                data = b""
                while True:                       # the server closes the connection
                    chunk = await asyncio.wait_for(r.read(1 << 16), 5)
                    if not chunk:
                        break
                    data += chunk
                w.close()
                if payload.startswith(gl.PREFACE):
                    # SETTINGS, then GOAWAY(PROTOCOL_ERROR) before the close
                    frames, pos = [], 0
                    while pos + 9 <= len(data):
                        lt, _, _ = gl._HDR.unpack_from(data, pos)
                        frames.append((lt & 0xFF, data[pos + 9:pos + 9 + (lt >> 8)]))
                        pos += 9 + (lt >> 8)
                    goaway = [p for t, p in frames if t == gl.GOAWAY]
                    assert goaway and int.from_bytes(goaway[0][4:8], "big") == gl.E_PROTOCOL, frames
            ch = gl.Channel("unix://" + sock)
            info = await api.device_plugin_stub(ch).GetPluginInfo(api.DP["GetPluginInfoRequest"](), timeout=2)
            assert info.init_timeout == 10
            await ch.close()
        finally:
            await plugin.stop()
    asyncio.run(main())


def _frames(data):
    out, pos = [], 0
    while pos + 9 <= len(data):
        lt, flags, sid = gl._HDR.unpack_from(data, pos)
        out.append((lt & 0xFF, flags, sid, data[pos + 9:pos + 9 + (lt >> 8)]))
        pos += 9 + (lt >> 8)
    return out


def test_lite_server_bounds_what_a_peer_can_make_it_hold():
    """Limits a misbehaving peer hits instead of growing the server (RFC 7540 error codes):
    a frame over the advertised SETTINGS_MAX_FRAME_SIZE (FRAME_SIZE_ERROR), an endless
    CONTINUATION chain (ENHANCE_YOUR_CALM), padding longer than the frame and an out-of-range peer
    SETTINGS_MAX_FRAME_SIZE (PROTOCOL_ERROR) end that connection; a gRPC message declared over
    16 MiB and a second request message on a unary call are refused per stream
    (RST_STREAM) on a connection that stays usable. The server keeps serving throughout."""
    hdr = gl._HDR.pack

    async def main():
        d = tempfile.mkdtemp()
        sock = os.path.join(d, "p.sock")
        plugin = await _Plugin("amd.com/gpu", sock, [device("g0")]).start()
        try:
            cont = hdr((0 << 8) | gl.HEADERS, 0, 1) + b"".join(
                hdr((16000 << 8) | gl.CONTINUATION, 0, 1) + b"\x00" * 16000 for _ in range(6))
            conn_cases = [
                (hdr(((gl.MAX_FRAME + 1) << 8) | gl.DATA, 0, 1), gl.E_FRAME_SIZE),
                (cont, gl.E_CALM),
                (hdr((4 << 8) | gl.HEADERS, gl.F_END_HEADERS | gl.F_PADDED, 1) + b"\x09abc", gl.E_PROTOCOL),
                (hdr((6 << 8) | gl.SETTINGS, 0, 0) + struct.pack(">HI", gl.S_MAX_FRAME_SIZE, 100), gl.E_PROTOCOL),
            ]
            for payload, code in conn_cases:
                r, w = await asyncio.open_unix_connection(sock)
                w.write(gl.PREFACE + payload)
                try:
                    await w.drain()
                except ConnectionError:
                    pass
                data = b""
                while True:
                    try:
                        chunk = await asyncio.wait_for(r.read(1 << 16), 5)
                    except ConnectionError:
                        break
                    if not chunk:
                        break
                    data += chunk
                w.close()
                goaway = [p for t, _, _, p in _frames(data) if t == gl.GOAWAY]
                assert goaway and int.from_bytes(goaway[0][4:8], "big") == code, (code, _frames(data))

            # per-stream limits: the same connection keeps working afterwards
            ch = gl.Channel("unix://" + sock)
            stub = api.device_plugin_stub(ch)
            await stub.GetPluginInfo(api.DP["GetPluginInfoRequest"](), timeout=2)
            conn = ch._conn
            # a response stream whose peer declares a message over the limit: the call fails with
            # RESOURCE_EXHAUSTED before any of it is buffered, the stream is reset
            st = conn.streams.setdefault(99, gl._Stream(99, 0))
            conn.last_peer_sid = max(conn.last_peer_sid, 99)
            st.buf += gl._MSG.pack(0, gl.MAX_MESSAGE + 1) + b"\x00" * 10
            conn._take_messages(st)
            assert 99 not in conn.streams and st.error.code() == gl.StatusCode.RESOURCE_EXHAUSTED
            info = await stub.GetPluginInfo(api.DP["GetPluginInfoRequest"](), timeout=2)
            assert info.init_timeout == 10
            await ch.close()
        finally:
            await plugin.stop()
    asyncio.run(main())


def test_lite_client_queues_calls_over_peer_max_concurrent_streams(monkeypatch):
    """a grpclite client honours the peer's SETTINGS_MAX_CONCURRENT_STREAMS — calls over
    it wait for a free stream instead of being refused (UNAVAILABLE); and an
    INITIAL_WINDOW_SIZE change that overflows an open stream's window is a FLOW_CONTROL_ERROR."""
    monkeypatch.setattr(gl, "MAX_CONCURRENT_STREAMS", 4)

    async def main():
        d = tempfile.mkdtemp()
        sock = os.path.join(d, "p.sock")
        plugin = await _Plugin("amd.com/gpu", sock, [device("g0")]).start()
        ch = gl.Channel("unix://" + sock)
        try:
            dp = api.device_plugin_stub(ch)
            reqs = [api.DP["AdmitPodRequest"](pod_name=f"q{i}") for i in range(40)]
            resps = await asyncio.gather(*[dp.AdmitPod(r, timeout=10) for r in reqs])
            assert [r.pod.annotations["amd.com/admitted"] for r in resps] == [f"q{i}" for i in range(40)]
            assert ch._conn.peer_max_streams == 4 and not ch._conn.slot_waiters
            # window overflow through a SETTINGS delta
            conn = ch._conn
            st = conn.streams.setdefault(201, gl._Stream(201, gl._MAX_WINDOW - 10))
            with pytest.raises(gl._ConnError) as ei:
                conn._on_frame(gl.SETTINGS, 0, 0, struct.pack(">HI", gl.S_INITIAL_WINDOW_SIZE, conn.peer_initial + 100))
            assert ei.value.code == gl.E_FLOW_CONTROL
            conn.streams.pop(201, None)
        finally:
            await ch.close()
            await plugin.stop()
    asyncio.run(asyncio.wait_for(main(), 60))


def test_stream_slot_hand_off_on_cancel_and_deadline(monkeypatch):
    """a queued call that is woken for a free stream and cancelled before it opens one
    passes the slot to the next waiter (no lost wakeup), and a queued unary call honours its
    deadline while waiting for a slot (DEADLINE_EXCEEDED, nothing left queued)."""
    monkeypatch.setattr(gl, "MAX_CONCURRENT_STREAMS", 4)

    async def main():
        d = tempfile.mkdtemp()
        sock = os.path.join(d, "p.sock")
        plugin = await _Plugin("amd.com/gpu", sock, [device("g0")]).start()
        ch = gl.Channel("unix://" + sock)
        try:
            dp = api.device_plugin_stub(ch)
            await dp.AdmitPod(api.DP["AdmitPodRequest"](pod_name="warm"), timeout=5)
            conn = ch._conn
            assert conn.peer_max_streams == 4
            for sid in (1001, 1003, 1005, 1007):            # every stream slot taken
                conn.streams[sid] = gl._Stream(sid, 0)
            a = asyncio.ensure_future(conn.stream_slot())
            b = asyncio.ensure_future(conn.stream_slot())
            await asyncio.sleep(0.01)
            assert len(conn.slot_waiters) == 2
            conn.streams.pop(1001)
            conn._slot_free()                               # wakes a ...
            a.cancel()                                      # ... which is cancelled before it runs
            await asyncio.wait_for(b, 1)                    # b got the slot a never used
            assert a.cancelled() and not conn.slot_waiters
            conn.streams[1001] = gl._Stream(1001, 0)
            with pytest.raises(gl.RpcError) as ei:
                await conn.stream_slot(0.05)
            assert ei.value.code() == gl.StatusCode.DEADLINE_EXCEEDED and not conn.slot_waiters
            t0 = asyncio.get_running_loop().time()
            with pytest.raises(gl.RpcError) as ei:          # a unary call queued past its deadline
                await dp.AdmitPod(api.DP["AdmitPodRequest"](pod_name="late"), timeout=0.1)
            assert ei.value.code() == gl.StatusCode.DEADLINE_EXCEEDED
            assert asyncio.get_running_loop().time() - t0 < 1.0
            for sid in (1001, 1003, 1005, 1007):
                conn.streams.pop(sid, None)
        finally:
            await ch.close()
            await plugin.stop()
    asyncio.run(asyncio.wait_for(main(), 30))
