"""The etcd v3 CLIENT storage backend (`storage/etcd3_client.py`): the API server as an etcd v3
client, the way the reference's is (`staging/src/k8s.io/apiserver/pkg/storage/etcd3/store.go`).

Here the etcd v3 endpoint is `kamd-etcd-gateway` in front of a `kamd-etcd` store — the only etcd
v3 server in this image — so every request crosses etcd's wire API (KV.Range / KV.Txn /
Watch with prev_kv / Compact) and a real etcd cluster could be swapped in at the same URL.
Parity tests: `etcd3/store_test.go` (TestCreate / TestGuaranteedUpdate conflict / TestList
pagination / TestWatch delete with prevKV) and the API server suite run unchanged against it.
"""
import asyncio
import os
import subprocess
import sys

import pytest

from kubernetes_amd.storage import wire
from kubernetes_amd.storage.etcd3_client import INJECT_MAGIC, Etcd3Store, is_etcd3_address
from kubernetes_amd.storage.mvcc import CompactedError
from kubernetes_amd.storage.remote import StoreServer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def etcd():
    """kamd-etcd + kamd-etcd-gateway (a separate process): yields the etcd v3 URL."""
    s = StoreServer()
    addr = s.start()
    env = dict(os.environ, PYTHONPATH=ROOT)
    gw = subprocess.Popen([sys.executable, "-u", "-m", "kubernetes_amd.cmd.etcd_gateway", "--store", addr,
                           "--listen", "127.0.0.1:0"], env=env, stdout=subprocess.PIPE, text=True)
    line = gw.stdout.readline()
    assert "etcd v3 API" in line, line
    url = "http://" + line.strip().rsplit(" on ", 1)[1]
    yield url
    gw.terminate()
    gw.wait(10)
    s.stop()


def test_address_detection():
    assert is_etcd3_address("http://127.0.0.1:2379") and is_etcd3_address("https://a:1,https://b:2")
    assert not is_etcd3_address("unix:///run/kamd-etcd.sock") and not is_etcd3_address("tcp://127.0.0.1:1")


def test_kv_txn_range_watch(run, etcd):
    async def main():
        st = await Etcd3Store(etcd + "#/t1").connect()
        other = await Etcd3Store(etcd + "#/t2").connect()
        try:
            # create-if-absent, then a GuaranteedUpdate-style compare on mod revision
            r = await st.txn([(wire.CMP_MOD_REV, "/registry/pods/a/p", 0, None)], [(wire.OP_PUT, "/registry/pods/a/p", b"v1")])
            assert r.ok
            kv = await st.get("/registry/pods/a/p")
            assert kv.value == b"v1" and kv.mod_rev == r.rev and kv.version == 1
            seen = []
            r2 = await st.txn([(wire.CMP_MOD_REV, "/registry/pods/a/p", kv.mod_rev, None)],
                              [(wire.OP_PUT, "/registry/pods/a/p", b"v2")], on_ok=seen.append)
            assert r2.ok and seen == [r2.rev]
            # a stale compare fails, naming the compare and the current value
            r3 = await st.txn([(wire.CMP_ABSENT, "/kamd/devices/n/g0", 0, None),
                               (wire.CMP_MOD_REV, "/registry/pods/a/p", kv.mod_rev, None)],
                              [(wire.OP_PUT, "/registry/pods/a/p", b"v3")])
            assert not r3.ok and r3.failed == 1 and r3.current.value == b"v2"
            # device-claim compare: absent -> put; present -> fails at that index
            assert (await st.txn([(wire.CMP_ABSENT, "/kamd/devices/n/g0", 0, None)],
                                 [(wire.OP_PUT, "/kamd/devices/n/g0", b"/registry/pods/a/p")])).ok
            r4 = await st.txn([(wire.CMP_ABSENT, "/kamd/devices/n/g0", 0, None)], [(wire.OP_PUT, "/x", b"")])
            assert not r4.ok and r4.failed == 0 and r4.current.value == b"/registry/pods/a/p"
            # namespaces isolate: the other store sees nothing of t1
            assert await other.get("/registry/pods/a/p") is None
            # RV injection: the token's offsets are stored (not the token), reads see the mod revision
            tok = b"@rv-tok@"
            r5 = await st.txn([], [(wire.OP_PUT_INJECT, "/registry/configmaps/a/c",
                                    b'{"rv":"' + tok + b'","x":"' + tok + b'"}', tok)])
            c = await st.get("/registry/configmaps/a/c")
            assert c.value == b'{"rv":"%d","x":"%d"}' % (r5.rev, r5.rev)
            raw = await other._Range(__import__("kubernetes_amd.storage.etcdv3", fromlist=["M"]).M["RangeRequest"](
                key=b"/t1/registry/configmaps/a/c"))
            assert raw.kvs[0].value.startswith(INJECT_MAGIC) and tok not in raw.kvs[0].value
            # object content is never rewritten: text that looks like a marker in a plainly put
            # (e.g. protobuf) value reads back byte for byte
            odd = b"k8s\x00\x0a\x05@rv@" + INJECT_MAGIC[1:] + b"@kamd-etcd3-rv@"
            await st.txn([], [(wire.OP_PUT, "/registry/pods/a/odd", odd)])
            assert (await st.get("/registry/pods/a/odd")).value == odd
            # paged prefix range, pinned to one revision
            for i in range(25):
                await st.txn([], [(wire.OP_PUT, f"/registry/pods/b/p{i:02d}", b"x")])
            kvs, more, rev = await st.range("/registry/pods/b/")
            assert len(kvs) == 25 and not more
            page, more, _ = await st.range("/registry/pods/b/", limit=10)
            assert len(page) == 10 and more
            page2, _, _ = await st.range("/registry/pods/b/", limit=10, start_after=page[-1].key)
            assert page2[0].key == "/registry/pods/b/p10"
            # past-revision range (the gateway serves it from the store's history)
            await st.txn([], [(wire.OP_DELETE, "/registry/pods/b/p00", None)])
            then, _, at = await st.range("/registry/pods/b/", revision=rev)
            assert at == rev and len(then) == 25
            now, _, _ = await st.range("/registry/pods/b/")
            assert len(now) == 24
            # watch: replay from a revision, then live events; deletes carry the deleted value
            got = []
            done = asyncio.Event()

            def cb(t, kv):
                if t is None:
                    return
                got.append((t, kv.key, kv.value, kv.mod_rev))
                if t == 1 and kv.key == "/registry/pods/a/p":
                    done.set()
            created = await st.watch("/registry/pods/a/", kv.mod_rev, cb)
            assert created >= r2.rev
            d = await st.txn([], [(wire.OP_DELETE_TOMBSTONE, "/registry/pods/a/p", b"tomb", b"@x@")])
            await asyncio.wait_for(done.wait(), 10)
            assert got[0][:3] == (0, "/registry/pods/a/p", b"v2")                   # replayed put
            assert got[-1] == (1, "/registry/pods/a/p", b"v2", d.rev)               # delete, prev value
            # compaction: a watch from before it is refused
            await st.compact(d.rev)
            with pytest.raises(CompactedError):
                await st.watch("/registry/pods/a/", 1, cb)
        finally:
            await st.close()
            await other.close()
    run(main(), timeout=60)


def test_apiserver_on_etcd3(run, etcd):
    """An API server whose store is the etcd v3 endpoint: CRUD, conflicts, device claims,
    watches (with the deleted object), and the keys really live in etcd under its prefix."""
    from kubernetes_amd.apiserver.server import APIServer
    from kubernetes_amd.client.rest import APIStatusError, Client
    from kubernetes_amd.storage.etcdv3 import M

    async def main():
        api = APIServer(store=etcd + "#/apitest")
        port = await api.start()
        c = Client(f"http://127.0.0.1:{port}")
        raw = await Etcd3Store(etcd).connect()
        try:
            assert type(api.rstore).__name__ == "Etcd3Store" and api.fanout is None
            pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p1", "namespace": "default"},
                   "spec": {"containers": [{"name": "c", "image": "x"}]}}
            created = await c.create("pods", pod, "default")
            rv = created["metadata"]["resourceVersion"]
            r = await raw._Range(M["RangeRequest"](key=b"/apitest/registry/pods/default/p1"))
            assert r.kvs and str(r.kvs[0].mod_revision) == rv          # RV = the etcd mod revision
            got = await c.get("pods", "p1", "default")
            assert got["metadata"]["resourceVersion"] == rv
            # optimistic concurrency through etcd's Txn
            got["metadata"]["labels"] = {"a": "b"}
            await c.update("pods", got, "default")
            got["metadata"]["labels"] = {"a": "c"}
            with pytest.raises(APIStatusError) as e:
                await c.update("pods", got, "default")                  # stale resourceVersion
            assert e.value.code == 409
            # watch from the list revision sees the delete with the object
            lst = await c.list("pods", "default")
            events = []

            async def watch():
                async for etype, obj in await c.watch("pods", "default",
                                                      resource_version=lst["metadata"]["resourceVersion"]):
                    events.append({"type": etype, "object": obj})
                    if etype == "DELETED":
                        return
            t = asyncio.ensure_future(watch())
            await asyncio.sleep(0.2)
            await c.delete("pods", "p1", "default", grace_period=0)
            await asyncio.wait_for(t, 15)
            assert events[-1]["type"] == "DELETED" and events[-1]["object"]["metadata"]["name"] == "p1"
            with pytest.raises(APIStatusError) as e:
                await c.get("pods", "p1", "default")
            assert e.value.code == 404
        finally:
            await raw.close()
            await c.close()
            await api.stop()
    run(main(), timeout=60)


# every module that exercises the API server through its HTTP API (modules that inspect the
# in-process store object, or use an API server they never start, are not storage-agnostic)
SUITE = ["test_apiserver", "test_subresources", "test_api_versions", "test_validation_kinds", "test_initializers",
         "test_admission_security", "test_admission_estimation", "test_impersonation", "test_openapi_oidc_audit",
         "test_encryption", "test_autoscaling", "test_fake_client", "test_kubectl"]


def test_apiserver_suite_unchanged_on_etcd3(etcd):
    """The API server test modules, unchanged, with every APIServer() they build storing in the
    etcd v3 endpoint (each under a namespace of its own)."""
    env = dict(os.environ, KAMD_APISERVER_DEFAULT_STORE=etcd, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-p", "no:xdist"]
                       + [f"tests/{m}.py" for m in SUITE],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert " passed" in r.stdout


def test_kube_apiserver_command_with_etcd_servers(etcd, tmp_path, run):
    """`kube-apiserver --etcd-servers=http://... --etcd-prefix=/prod`: the process stores its
    objects in etcd under /prod; TLS flags are refused for the native store protocol."""
    import json as _json
    import time
    from kubernetes_amd.storage.etcdv3 import M
    pf = tmp_path / "port"
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.Popen([sys.executable, "-m", "kubernetes_amd.cmd.apiserver", "--port", "0", "--port-file", str(pf),
                          "--etcd-servers", etcd, "--etcd-prefix", "/prod"], env=env, cwd=ROOT,
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    try:
        t = time.time()
        while not pf.exists():
            assert p.poll() is None, p.stderr.read()
            assert time.time() - t < 60
            time.sleep(0.05)
        port = int(pf.read_text())

        async def main():
            from kubernetes_amd.client.rest import Client
            c = Client(f"http://127.0.0.1:{port}")
            await c.create("configmaps", {"metadata": {"name": "cfg", "namespace": "default"}, "data": {"a": "b"}},
                           "default")
            await c.close()
            raw = await Etcd3Store(etcd).connect()
            r = await raw._Range(M["RangeRequest"](key=b"/prod/registry/configmaps/default/cfg"))
            await raw.close()
            return r
        r = run(main())
        assert r.kvs and b"cfg" in r.kvs[0].value
    finally:
        p.terminate()
        p.wait(10)
    bad = subprocess.run([sys.executable, "-m", "kubernetes_amd.cmd.apiserver", "--port", "0",
                          "--etcd-servers", "unix:///nonexistent.sock", "--etcd-cafile", "/x"],
                         env=env, cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert bad.returncode != 0 and "TLS" in bad.stderr
