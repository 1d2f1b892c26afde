"""Protobuf watch streams (`application/vnd.kubernetes.protobuf;stream=watch`).

Parity: `staging/src/k8s.io/apiserver/pkg/endpoints/handlers/watch.go:72,166-226` (negotiated
stream serializer, objects embedded with the protobuf encoder, resourceVersion set) and
`apimachinery/pkg/runtime/serializer/protobuf/protobuf.go:436` (LengthDelimitedFramer: 4-byte
big-endian length + a raw-serialized metav1.WatchEvent). Checked on every watch path: the
single-process watch cache, a shared-store worker's own cache, the store's native fan-out (pods,
handed to kamd-etcd), and a 410 on a compacted resourceVersion; each protobuf stream must carry
exactly the events, objects and resourceVersions of the JSON stream beside it.
"""
import asyncio
import struct

import pytest

from kubernetes_amd.api import protobuf as pb
from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.native import pbcodec
from kubernetes_amd.client.rest import JSON, PROTOBUF, APIStatusError, Client
from kubernetes_amd.storage.remote import StoreServer


@pytest.fixture(autouse=True, params=["native", "python"])
def codec(request, monkeypatch):
    """Every test runs with the native codec and with the pure-Python one (KAMD_PBCODEC=python:
    no native library), whose watch frames must be byte-identical."""
    monkeypatch.setenv("KAMD_PBCODEC", request.param)
    pbcodec.reset()
    if request.param == "native" and pbcodec.codec() is None:
        pytest.skip("native pbcodec not built")
    yield request.param
    monkeypatch.delenv("KAMD_PBCODEC", raising=False)
    pbcodec.reset()


def _pod(name, node=None):
    p = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default", "labels": {"a": "b"}},
         "spec": {"containers": [{"name": "c", "image": "kubernetes-amd/pause"}]}}
    if node:
        p["spec"]["nodeName"] = node
    return p


def test_frame_layout_is_the_reference_wire_format():
    """4-byte big-endian length; WatchEvent{1: type, 2: RawExtension{1: k8s\\0 envelope}}."""
    env = pb.encode_object({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "x"}, "data": {"k": "v"}})
    fr = pb.watch_frame("ADDED", env)
    (n,) = struct.unpack(">I", fr[:4])
    assert n == len(fr) - 4
    body = fr[4:]
    assert body[:2] == b"\x0a\x05" and body[2:7] == b"ADDED"
    assert body[7] == 0x12                         # field 2, length-delimited
    # RawExtension{raw} with the envelope inside, magic first
    assert env in body and body[body.index(env) - 4:body.index(env)].find(b"\x0a") >= 0
    (evs, used) = pb.decode_watch_frames(fr)
    assert used == len(fr) and evs[0][0] == "ADDED" and evs[0][1]["data"] == {"k": "v"}
    # a partial frame is left for the next read
    assert pb.decode_watch_frames(fr[:-1]) == ([], 0)


def test_envelope_resource_version_rewrite():
    env = pb.encode_object({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "resourceVersion": "5",
                                                                          "labels": {"x": "y"}}})
    out = pb.envelope_with_rv(env, "12345")
    obj = pb.decode_object(out)
    assert obj["metadata"] == {"name": "p", "resourceVersion": "12345", "labels": {"x": "y"}}
    # an object without metadata gains it
    bare = pb.encode_object({"apiVersion": "v1", "kind": "Namespace", "spec": {"finalizers": ["kubernetes"]}})
    assert pb.decode_object(pb.envelope_with_rv(bare, "9"))["metadata"] == {"resourceVersion": "9"}
    assert pb.envelope_with_rv(b'{"json": 1}', "1") is None


async def _collect(stream, n, timeout=10):
    out = []

    async def go():
        async for typ, obj in stream:
            out.append((typ, obj["metadata"]["name"], obj["metadata"]["resourceVersion"],
                        (obj.get("spec") or {}).get("nodeName"), obj.get("kind")))
            if len(out) >= n:
                return
    await asyncio.wait_for(go(), timeout)
    return out


async def _exercise(writer, jc, pc, resource="pods", node=None):
    """Open a JSON and a protobuf watch side by side, write, compare."""
    fs = f"spec.nodeName={node}" if node else None
    jw = await jc.watch(resource, "default", resource_version="0", field_selector=fs)
    pw = await pc.watch(resource, "default", resource_version="0", field_selector=fs)
    assert pw.protobuf and not jw.protobuf
    await writer.create("pods", _pod("w1", node))
    await writer.patch("pods", "w1", {"metadata": {"labels": {"c": "d"}}}, "default")
    await writer.create("pods", _pod("w2", node))
    await writer.delete("pods", "w1", "default", grace_period=0)
    want = await _collect(jw, 4)
    got = await _collect(pw, 4)
    jw.close()
    pw.close()
    assert got == want
    assert [t for t, *_ in got] == ["ADDED", "MODIFIED", "ADDED", "DELETED"]
    assert all(k == "Pod" for *_, k in got)
    return got


def test_protobuf_watch_single_process_cache(run):
    async def main():
        s = APIServer()
        port = await s.start()
        url = f"http://127.0.0.1:{port}"
        jc, pc = Client(url), Client(url, content_type=PROTOBUF)
        try:
            await _exercise(jc, jc, pc)
        finally:
            await jc.close()
            await pc.close()
            await s.stop()
    run(main())


def test_protobuf_watch_gone(run):
    async def main():
        s = APIServer(watch_window=2)
        port = await s.start()
        url = f"http://127.0.0.1:{port}"
        c = Client(url, content_type=PROTOBUF)
        try:
            for i in range(6):
                await c.create("configmaps", {"metadata": {"name": f"cm{i}", "namespace": "default"}})
            with pytest.raises(APIStatusError) as ei:      # an HTTP 410 or an ERROR frame
                w = await c.watch("configmaps", "default", resource_version="1")
                async for _ in w:
                    pass
            assert ei.value.code == 410
            # the ERROR frame carries the Status as a protobuf envelope (v1/Status), as client-go's
            # protobuf stream decoder expects
            from kubernetes_amd.apiserver.cacher import error_event
            fr = error_event({"kind": "Status", "status": "Failure", "code": 410, "reason": "Expired"}, True)
            assert pb.MAGIC + b"\x0a\x0c\x0a\x02v1\x12\x06Status" in fr
            evs, _ = pb.decode_watch_frames(fr)
            assert evs[0][0] == "ERROR"
            assert {k: evs[0][1][k] for k in ("kind", "apiVersion", "status", "code", "reason")} == {
                "kind": "Status", "apiVersion": "v1", "status": "Failure", "code": 410, "reason": "Expired"}
        finally:
            await c.close()
            await s.stop()
    run(main())


@pytest.fixture
def store():
    s = StoreServer()
    addr = s.start()
    yield addr
    s.stop()


def test_protobuf_watch_shared_store_fanout_and_cache(run, store):
    """Pods are served by kamd-etcd's fan-out (handed-off socket), configmaps by the worker's
    own cache: both stream protobuf frames equal to the JSON stream."""
    async def main():
        s = APIServer(store=store)
        port = await s.start()
        url = f"http://127.0.0.1:{port}"
        jc, pc = Client(url), Client(url, content_type=PROTOBUF)
        try:
            assert "pods" in s.uncached and s.fanout is not None
            got = await _exercise(jc, jc, pc, node="node-a")       # nodeName-indexed fan-out watch
            assert all(n == "node-a" for *_, n, _ in got)
            jw = await jc.watch("configmaps", "default", resource_version="0")
            pw = await pc.watch("configmaps", "default", resource_version="0")
            assert pw.protobuf
            await jc.create("configmaps", {"metadata": {"name": "cm", "namespace": "default"}, "data": {"k": "v"}})
            a, b = await _collect(jw, 1), await _collect(pw, 1)
            assert a == b
            jw.close()
            pw.close()
        finally:
            await jc.close()
            await pc.close()
            await s.stop()
    run(main())


def test_protobuf_watch_resume_from_resource_version_fanout(run, store):
    async def main():
        s = APIServer(store=store)
        port = await s.start()
        url = f"http://127.0.0.1:{port}"
        c, pc = Client(url), Client(url, content_type=PROTOBUF)
        try:
            a = await c.create("pods", _pod("r1"))
            await c.create("pods", _pod("r2"))
            w = await pc.watch("pods", "default", resource_version=a["metadata"]["resourceVersion"])
            got = await _collect(w, 1)
            w.close()
            assert got[0][:2] == ("ADDED", "r2")
        finally:
            await c.close()
            await pc.close()
            await s.stop()
    run(main())


def test_protobuf_fanout_410_is_a_protobuf_status(run, store):
    """kamd-etcd's fan-out answers a compacted resourceVersion with an ERROR frame whose object
    is a protobuf v1/Status envelope (decodable without JSON sniffing)."""
    from kubernetes_amd.storage.remote import RemoteStore

    async def main():
        s = APIServer(store=store)
        port = await s.start()
        url = f"http://127.0.0.1:{port}"
        c, pc = Client(url), Client(url, content_type=PROTOBUF)
        try:
            assert s.fanout is not None
            for i in range(3):
                await c.create("pods", _pod(f"g{i}"))
            rv = (await c.list("pods", "default"))["metadata"]["resourceVersion"]
            rs = await RemoteStore(store).connect()
            await rs.compact(int(rv))
            w = await pc.watch("pods", "default", resource_version="2", timeout_seconds=2)
            with pytest.raises(APIStatusError) as ei:
                [x async for x in w]
            assert ei.value.code == 410 and "too old resource version" in str(ei.value)
        finally:
            await c.close()
            await pc.close()
            await s.stop()
    run(main())


def test_python_frames_match_native(monkeypatch):
    """The pure-Python fallbacks produce the native codec's bytes."""
    if pbcodec.codec() is None:
        pytest.skip("native pbcodec not built")
    env = pb.encode_object({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "d"},
                            "spec": {"nodeName": "n"}})
    st = {"kind": "Status", "status": "Failure", "message": "m", "reason": "Expired", "code": 410}
    nat = (pb.watch_frame("ADDED", env), pb.envelope_with_rv(env, "77"), pb.status_envelope(st))
    monkeypatch.setenv("KAMD_PBCODEC", "python")
    pbcodec.reset()
    try:
        py = (pb.watch_frame("ADDED", env), pb.envelope_with_rv(env, "77"), pb.status_envelope(st))
        assert py[0] == nat[0]
        assert pb.decode_object(py[1]) == pb.decode_object(nat[1])
        assert pb.decode_object(py[2]) == pb.decode_object(nat[2])
        assert pb.decode_watch_frames(nat[0] + nat[0][:5]) == pb.decode_watch_frames(py[0] + py[0][:5])
    finally:
        monkeypatch.setenv("KAMD_PBCODEC", "native")
        pbcodec.reset()


def test_json_clients_unchanged(run):
    async def main():
        s = APIServer()
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}", content_type=JSON)
        try:
            w = await c.watch("pods", "default", resource_version="0")
            assert not w.protobuf
            w.close()
        finally:
            await c.close()
            await s.stop()
    run(main())
