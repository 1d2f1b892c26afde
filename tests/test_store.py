"""MVCC store engines: native C++ (libkamd_store.so / kamd-etcd) vs the pure-Python reference
engine, differential on random operation sequences; transactions, RV injection, tombstones,
WAL replay, and the remote protocol with watch."""
import asyncio
import random

import pytest

from kubernetes_amd.storage import wire
from kubernetes_amd.storage.mvcc import CompactedError, MVCCStore
from kubernetes_amd.storage.native_store import NativeMVCCStore
from kubernetes_amd.storage.remote import RemoteStore, StoreServer


def _snapshot(s):
    kvs, more, rev = s.range("/")
    return rev, [(kv.key, kv.value, kv.create_rev, kv.mod_rev, kv.version) for kv in kvs]


def test_differential_random_ops():
    rnd = random.Random(7)
    py, nat = MVCCStore(), NativeMVCCStore()
    keys = [f"/registry/pods/ns{i % 3}/p{i}" for i in range(40)]
    for step in range(3000):
        k = rnd.choice(keys)
        v = f"v{step}".encode()
        op = rnd.random()
        if op < 0.3:
            a, b = py.create(k, v), nat.create(k, v)
            assert (a is None) == (b is None)
            if a:
                assert a.kv.mod_rev == b.kv.mod_rev
        elif op < 0.6:
            cur = py.get(k)
            exp = cur.mod_rev if cur and rnd.random() < 0.8 else 12345
            (ok1, e1), (ok2, e2) = py.update(k, v, exp), nat.update(k, v, exp)
            assert ok1 == ok2
            if ok1:
                assert (e1.kv.mod_rev, e1.kv.version) == (e2.kv.mod_rev, e2.kv.version)
        elif op < 0.75:
            (ok1, _), (ok2, _) = py.delete(k), nat.delete(k)
            assert ok1 == ok2
        elif op < 0.85:
            k2 = rnd.choice(keys)
            cmps = [(wire.CMP_EXISTS, k, 0, None)]
            ops = [(wire.OP_PUT, k, v), (wire.OP_DELETE, k2, None)] if k2 != k else [(wire.OP_PUT, k, v)]
            r1, r2 = py.txn(cmps, ops), nat.txn(cmps, ops)
            assert (r1.ok, r1.rev, r1.failed) == (r2.ok, r2.rev, r2.failed)
        else:
            pre = f"/registry/pods/ns{rnd.randrange(3)}/"
            lim = rnd.randrange(0, 6)
            sa = rnd.choice([None, pre + "p1"])
            a, b = py.range(pre, lim, sa), nat.range(pre, lim, sa)
            assert [kv.key for kv in a[0]] == [kv.key for kv in b[0]] and a[1:] == b[1:]
        assert py.revision == nat.revision
    assert _snapshot(py) == _snapshot(nat)
    since = py.revision - 50
    e1, e2 = py.events_since(since, "/registry/"), nat.events_since(since, "/registry/")
    assert [(e.type, e.kv.key, e.kv.mod_rev) for e in e1] == [(e.type, e.kv.key, e.kv.mod_rev) for e in e2]
    assert py.count("/registry/pods/ns1/") == nat.count("/registry/pods/ns1/")


def test_txn_single_revision_and_injection():
    for s in (MVCCStore(), NativeMVCCStore()):
        tok = b"@tok123@"
        r = s.txn([(wire.CMP_ABSENT, "/a", 0, None)],
                  [(wire.OP_PUT_INJECT, "/a", b'{"rv":"@tok123@","x":"@RV@"}', tok), (wire.OP_PUT, "/b", b"@tok123@")])
        assert r.ok and r.rev == 2
        assert s.get("/a").value == b'{"rv":"2","x":"@RV@"}'
        assert s.get("/b").value == b"@tok123@"          # plain put: never rewritten
        assert s.get("/a").mod_rev == s.get("/b").mod_rev == 2
        r = s.txn([(wire.CMP_ABSENT, "/a", 0, None)], [(wire.OP_PUT, "/a", b"z")])
        assert not r.ok and r.failed == 0 and r.current.mod_rev == 2
        r = s.txn([(wire.CMP_MOD_REV, "/a", 2, None), (wire.CMP_VALUE, "/b", 0, b"nope")], [(wire.OP_DELETE, "/a", None)])
        assert not r.ok and r.failed == 1
        r = s.txn([(wire.CMP_MOD_REV, "/a", 2, None)], [(wire.OP_DELETE_TOMBSTONE, "/a", b"final@tok123@", tok)])
        assert r.ok and r.rev == 3 and s.get("/a") is None
        evs = s.events_since(2)
        assert evs[-1].type == 1 and evs[-1].kv.key == "/a"
        # no-op txn does not bump the revision
        r = s.txn([], [(wire.OP_DELETE, "/missing", None)])
        assert r.ok and s.revision == 3


def test_native_wal_replay_keeps_revisions(tmp_path):
    wal = str(tmp_path / "wal")
    s = NativeMVCCStore(wal_path=wal)
    s.create("/x", b"1")
    s.txn([], [(wire.OP_PUT, "/y", b"2"), (wire.OP_PUT, "/z", b"3")])
    s.update("/x", b"4", None)
    s.delete("/y")
    before = _snapshot(s)
    s.close()
    s2 = NativeMVCCStore(wal_path=wal)
    assert _snapshot(s2) == before and s2.revision == 5
    s2.close()
    with open(wal, "ab") as f:
        f.write(b"\x00\x01\x05\x00")  # torn tail
    s3 = NativeMVCCStore(wal_path=wal)
    assert _snapshot(s3) == before
    s3.close()


def test_compaction_native():
    s = NativeMVCCStore(history=10)
    for i in range(30):
        s.put(f"/k{i}", b"v")
    with pytest.raises(CompactedError):
        s.events_since(2)
    assert len(s.events_since(s.revision - 5)) == 5


def test_remote_store_server(run):
    srv = StoreServer()
    addr = srv.start()

    async def main():
        a, b = await RemoteStore(addr).connect(), await RemoteStore(addr).connect()
        seen = []
        rev0 = await b.watch("/registry/", 0, lambda t, kv: seen.append((t, kv.key if kv else None, kv.mod_rev if kv else None)))
        assert rev0 == 1
        r = await a.txn([(wire.CMP_ABSENT, "/registry/pods/a", 0, None)],
                        [(wire.OP_PUT_INJECT, "/registry/pods/a", b'{"rv":"#RV#"}', b"#RV#"), (wire.OP_PUT, "/dev/x", b"a")])
        assert r.ok and r.rev == 2
        kv = await a.get("/registry/pods/a")
        assert kv.value == b'{"rv":"2"}' and kv.mod_rev == 2
        r = await a.txn([(wire.CMP_ABSENT, "/dev/x", 0, None)], [(wire.OP_PUT, "/dev/x", b"b")])
        assert not r.ok and r.current.value == b"a"
        # concurrent CAS from two clients on the same revision: exactly one wins
        res = await asyncio.gather(
            a.txn([(wire.CMP_MOD_REV, "/registry/pods/a", 2, None)], [(wire.OP_PUT, "/registry/pods/a", b"A")]),
            b.txn([(wire.CMP_MOD_REV, "/registry/pods/a", 2, None)], [(wire.OP_PUT, "/registry/pods/a", b"B")]))
        assert sorted(x.ok for x in res) == [False, True]
        await a.txn([], [(wire.OP_DELETE_TOMBSTONE, "/registry/pods/a", b"gone", b"#")])
        for _ in range(100):
            if len(seen) >= 3:
                break
            await asyncio.sleep(0.01)
        assert seen == [(0, "/registry/pods/a", 2), (0, "/registry/pods/a", 3), (1, "/registry/pods/a", 4)]
        await a.txn([], [(wire.OP_PUT, "/dev/y", b"c")])
        kvs, more, rev = await a.range("/", 1)
        assert more and rev == 5 and kvs[0].key == "/dev/x"
        kvs, more, rev = await a.range("/", 1, "/dev/x")
        assert not more and [kv.key for kv in kvs] == ["/dev/y"]
        # watch with replay from a revision
        replay = []
        await a.watch("/registry/", 2, lambda t, kv: replay.append(kv.mod_rev if kv else None))
        await asyncio.sleep(0.05)
        assert replay == [3, 4]           # /dev/y is outside the watched prefix
        await a.close()
        await b.close()
    try:
        run(main())
    finally:
        srv.stop()


def test_store_server_drops_malformed_frames(run):
    """A request frame shorter than its id+op header, or one declaring more than the server's
    frame limit, ends only that connection; the store keeps serving other clients. (A zero
    length used to reach the request handler as a body length of 2^32 - 5.)"""
    import socket
    import struct as st
    srv = StoreServer()
    addr = srv.start()
    try:
        for frame in (st.pack("<I", 0) + b"\0" * 16, st.pack("<I", 4) + b"\0" * 16,
                      st.pack("<I", 0xFFFFFFF0) + b"\0" * 16):
            s = socket.socket(socket.AF_UNIX)
            s.connect(srv.socket_path)
            s.sendall(frame)
            s.settimeout(5)
            assert s.recv(64) == b""          # closed by the server, nothing answered
            s.close()
        assert srv.proc.poll() is None

        async def main():
            c = await RemoteStore(addr).connect()
            r = await c.txn([], [(wire.OP_PUT, "/registry/x", b"v")])
            assert r.ok and (await c.get("/registry/x")).value == b"v"
            await c.close()
        run(main())
    finally:
        srv.stop()
