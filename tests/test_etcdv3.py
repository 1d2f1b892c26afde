"""etcd v3 gRPC API over kamd-etcd: KV / Txn / Watch / Lease / Status semantics as clientv3 and
etcdctl rely on them (parity: `vendor/github.com/coreos/etcd/clientv3` usage in
`staging/src/k8s.io/apiserver/pkg/storage/etcd3/store.go` — GuaranteedUpdate's
`Compare(ModRevision(key), "=", rev)` transactions, prefix ranges, watches from a revision),
including reading the live state an API server keeps in the same store."""
import asyncio

import pytest

from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client.rest import Client
from kubernetes_amd.storage.etcdv3 import M, EtcdV3Client, EtcdV3Gateway, prefix_end
from kubernetes_amd.storage.remote import StoreServer


@pytest.fixture
def store():
    s = StoreServer()
    addr = s.start()
    yield addr
    s.stop()


async def _gw(addr):
    gw = await EtcdV3Gateway(addr).start()
    return gw, EtcdV3Client(f"127.0.0.1:{gw.port}")


def test_prefix_end():
    assert prefix_end(b"/registry/pods/") == b"/registry/pods0"
    assert prefix_end(b"a\xff") == b"b" and prefix_end(b"\xff") == b"\x00"


def test_kv_range_put_delete_txn(run, store):
    async def main():
        gw, c = await _gw(store)
        try:
            r = await c.Put(M["PutRequest"](key=b"/a/1", value=b"one"))
            rev1 = r.header.revision
            await c.Put(M["PutRequest"](key=b"/a/2", value=b"two"))
            await c.Put(M["PutRequest"](key=b"/b/1", value=b"x"))
            p = await c.Put(M["PutRequest"](key=b"/a/1", value=b"uno", prev_kv=True))
            assert p.prev_kv.value == b"one" and p.prev_kv.mod_revision == rev1
            g = await c.Range(M["RangeRequest"](key=b"/a/1"))
            assert [(kv.key, kv.value, kv.version) for kv in g.kvs] == [(b"/a/1", b"uno", 2)]
            pr = await c.Range(M["RangeRequest"](key=b"/a/", range_end=prefix_end(b"/a/")))
            assert [kv.key for kv in pr.kvs] == [b"/a/1", b"/a/2"] and pr.count == 2
            lim = await c.Range(M["RangeRequest"](key=b"/", range_end=b"\x00", limit=2, keys_only=True))
            assert lim.more and lim.count == 3 and [kv.value for kv in lim.kvs] == [b"", b""]
            cnt = await c.Range(M["RangeRequest"](key=b"/", range_end=b"\x00", count_only=True))
            assert cnt.count == 3 and not cnt.kvs
            desc = await c.Range(M["RangeRequest"](key=b"/", range_end=b"\x00", sort_order=2, sort_target=3))
            assert [kv.key for kv in desc.kvs][0] == b"/a/1"              # newest mod revision first
            # GuaranteedUpdate-style CAS: compare mod revision, else read back
            cur = g.kvs[0].mod_revision
            ok = await c.Txn(M["TxnRequest"](
                compare=[M["Compare"](key=b"/a/1", target=2, result=0, mod_revision=cur)],
                success=[M["RequestOp"](request_put=M["PutRequest"](key=b"/a/1", value=b"cas"))],
                failure=[M["RequestOp"](request_range=M["RangeRequest"](key=b"/a/1"))]))
            assert ok.succeeded and ok.responses[0].WhichOneof("response") == "response_put"
            stale = await c.Txn(M["TxnRequest"](
                compare=[M["Compare"](key=b"/a/1", target=2, result=0, mod_revision=cur)],
                success=[M["RequestOp"](request_put=M["PutRequest"](key=b"/a/1", value=b"lost"))],
                failure=[M["RequestOp"](request_range=M["RangeRequest"](key=b"/a/1"))]))
            assert not stale.succeeded and stale.responses[0].response_range.kvs[0].value == b"cas"
            # create-if-absent: CREATE == 0 (the oneof carries the explicit 0)
            cr = M["Compare"](key=b"/new", target=1, result=0, create_revision=0)
            assert cr.WhichOneof("target_union") == "create_revision"
            mk = M["TxnRequest"](compare=[cr], success=[M["RequestOp"](request_put=M["PutRequest"](key=b"/new", value=b"1"))])
            assert (await c.Txn(mk)).succeeded and not (await c.Txn(mk)).succeeded
            # value / version comparisons
            vc = M["Compare"](key=b"/a/2", target=3, result=3, value=b"nope")         # NOT_EQUAL
            gt = M["Compare"](key=b"/a/1", target=0, result=1, version=1)             # version > 1
            t = await c.Txn(M["TxnRequest"](compare=[vc, gt], success=[M["RequestOp"](
                request_delete_range=M["DeleteRangeRequest"](key=b"/a/", range_end=prefix_end(b"/a/"), prev_kv=True))]))
            assert t.succeeded and t.responses[0].response_delete_range.deleted == 2
            assert sorted(kv.key for kv in t.responses[0].response_delete_range.prev_kvs) == [b"/a/1", b"/a/2"]
            d = await c.DeleteRange(M["DeleteRangeRequest"](key=b"/b/1"))
            assert d.deleted == 1
            assert (await c.Range(M["RangeRequest"](key=b"/", range_end=b"\x00"))).count == 1
        finally:
            await c.close()
            await gw.stop()
    run(main())


def test_watch_replay_filters_cancel_and_compaction(run, store):
    async def main():
        gw, c = await _gw(store)
        try:
            base = (await c.Put(M["PutRequest"](key=b"/w/a", value=b"1"))).header.revision
            await c.Put(M["PutRequest"](key=b"/w/b", value=b"2"))
            await c.Put(M["PutRequest"](key=b"/x/z", value=b"out of range"))
            q: asyncio.Queue = asyncio.Queue()

            async def reqs():
                yield M["WatchRequest"](create_request=M["WatchCreateRequest"](
                    key=b"/w/", range_end=prefix_end(b"/w/"), start_revision=base))
                yield M["WatchRequest"](create_request=M["WatchCreateRequest"](
                    key=b"/w/", range_end=prefix_end(b"/w/"), filters=[0]))             # NOPUT: deletes only
                await q.get()
                yield M["WatchRequest"](cancel_request=M["WatchCancelRequest"](watch_id=0))
                await q.get()
            call = c.Watch(reqs())
            got = []

            async def collect():
                async for resp in call:
                    got.append(resp)
            t = asyncio.ensure_future(collect())

            async def until(pred):
                for _ in range(200):
                    if pred():
                        return
                    await asyncio.sleep(0.02)
                raise AssertionError([str(g) for g in got])
            await until(lambda: sum(1 for g in got if g.created) == 2)
            await c.Put(M["PutRequest"](key=b"/w/c", value=b"3"))
            await c.DeleteRange(M["DeleteRangeRequest"](key=b"/w/a"))
            evs = lambda wid: [(e.type, e.kv.key) for g in got if g.watch_id == wid for e in g.events]  # noqa: E731
            await until(lambda: len(evs(0)) == 4 and len(evs(1)) == 1)
            assert evs(0) == [(0, b"/w/a"), (0, b"/w/b"), (0, b"/w/c"), (1, b"/w/a")]       # replay + live
            assert evs(1) == [(1, b"/w/a")]
            q.put_nowait(1)
            await until(lambda: any(g.canceled and g.watch_id == 0 for g in got))
            await c.Put(M["PutRequest"](key=b"/w/d", value=b"4"))
            await asyncio.sleep(0.2)
            assert len(evs(0)) == 4                                   # nothing after the cancel
            q.put_nowait(1)
            await t
            # a compacted start revision: created, then canceled with compact_revision
            cur = (await c.Range(M["RangeRequest"](key=b"/w/d"))).header.revision
            await c.Compact(M["CompactionRequest"](revision=cur))

            async def one():
                yield M["WatchRequest"](create_request=M["WatchCreateRequest"](key=b"/w/d", start_revision=2))
                await asyncio.sleep(0.5)
            resps = [r async for r in c.Watch(one())]
            assert resps[-1].canceled and resps[-1].compact_revision == cur
        finally:
            await c.close()
            await gw.stop()
    run(main())


def test_leases_expire_and_keepalive(run, store):
    async def main():
        gw, c = await _gw(store)
        try:
            short = (await c.LeaseGrant(M["LeaseGrantRequest"](TTL=1))).ID
            kept = (await c.LeaseGrant(M["LeaseGrantRequest"](TTL=1))).ID
            await c.Put(M["PutRequest"](key=b"/ev/1", value=b"a", lease=short))
            await c.Put(M["PutRequest"](key=b"/ev/2", value=b"b", lease=kept))
            ttl = await c.LeaseTimeToLive(M["LeaseTimeToLiveRequest"](ID=short, keys=True))
            assert ttl.grantedTTL == 1 and list(ttl.keys) == [b"/ev/1"]
            assert (await c.Range(M["RangeRequest"](key=b"/ev/1"))).kvs[0].lease == short

            async def ka():
                for _ in range(8):
                    yield M["LeaseKeepAliveRequest"](ID=kept)
                    await asyncio.sleep(0.25)
            async for r in c.LeaseKeepAlive(ka()):
                assert r.TTL == 1
            keys = [kv.key for kv in (await c.Range(M["RangeRequest"](key=b"/ev/", range_end=prefix_end(b"/ev/")))).kvs]
            assert keys == [b"/ev/2"]                                     # the short lease expired
            await c.LeaseRevoke(M["LeaseRevokeRequest"](ID=kept))
            assert (await c.Range(M["RangeRequest"](key=b"/ev/2"))).count == 0
            st = await c.Status(M["StatusRequest"]())
            assert st.version.startswith("3.") and st.header.revision == st.raftIndex
        finally:
            await c.close()
            await gw.stop()
    run(main())


def test_gateway_reads_api_server_state(run, store):
    """etcdctl-style inspection of a live cluster: what the API server wrote (protobuf storage,
    `k8s\\0` envelope behind the store's index frame) is visible under /registry."""
    async def main():
        api = APIServer(store=store)
        cl = Client(f"http://127.0.0.1:{await api.start()}")
        gw, c = await _gw(store)
        try:
            await cl.create("configmaps", {"metadata": {"name": "cm", "namespace": "default"}, "data": {"k": "v"}})
            r = await c.Range(M["RangeRequest"](key=b"/registry/configmaps/", range_end=prefix_end(b"/registry/configmaps/")))
            kv = [kv for kv in r.kvs if kv.key == b"/registry/configmaps/default/cm"][0]
            assert b"k8s\x00" in kv.value
            got = await cl.get("configmaps", "cm", "default")
            assert int(got["metadata"]["resourceVersion"]) == kv.mod_revision
        finally:
            await c.close()
            await gw.stop()
            await cl.close()
            await api.stop()
    run(main())
