"""Several API server workers sharing one native store (kamd-etcd): cross-worker visibility,
watch ordering, CAS retries on stale caches, and the cross-worker GPU double-assignment guard."""
import asyncio

import pytest

from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client.rest import APIStatusError, Client
from kubernetes_amd.storage.remote import StoreServer


def gpu_pod(name, n=1):
    return {"metadata": {"name": name, "namespace": "default"},
            "spec": {"containers": [{"name": "c", "image": "x", "resources": {"limits": {"amd.com/gpu": str(n)}}}]}}


@pytest.fixture
def store():
    s = StoreServer()
    addr = s.start()
    yield addr
    s.stop()


async def _workers(addr, n=2):
    servers, clients = [], []
    for _ in range(n):
        s = APIServer(store=addr)
        port = await s.start()
        servers.append(s)
        clients.append(Client(f"http://127.0.0.1:{port}"))
    return servers, clients


async def _close(servers, clients):
    for c in clients:
        await c.close()
    for s in servers:
        await s.stop()


async def _eventually(fn, timeout=5.0):
    t = asyncio.get_running_loop().time() + timeout
    while True:
        try:
            r = await fn()
            if r:
                return r
        except APIStatusError:
            pass
        if asyncio.get_running_loop().time() > t:
            raise AssertionError("condition not met")
        await asyncio.sleep(0.01)


def test_cross_worker_crud_and_watch(run, store):
    async def main():
        servers, (a, b) = await _workers(store)
        try:
            # bootstrap raced between workers: namespaces exist exactly once
            nss = (await a.list("namespaces"))["items"]
            assert sorted(n["metadata"]["name"] for n in nss) == ["default", "kube-public", "kube-system"]
            events = []
            w = await b.watch("pods", "default", "0")

            async def drain():
                async for typ, obj in w:
                    events.append((typ, obj["metadata"]["name"], obj["metadata"]["resourceVersion"]))
            t = asyncio.ensure_future(drain())
            p = await a.create("pods", gpu_pod("p1"))
            assert p["metadata"]["resourceVersion"].isdigit()
            got = await _eventually(lambda: b.get("pods", "p1", "default"))
            assert got == p                              # byte-identical object via the other worker
            await b.patch("pods", "p1", {"metadata": {"labels": {"x": "1"}}}, "default")
            await a.delete("pods", "p1", "default")
            await _eventually(lambda: asyncio.sleep(0, len(events) >= 3))
            assert [e[0] for e in events] == ["ADDED", "MODIFIED", "DELETED"]
            revs = [int(e[2]) for e in events]
            assert revs == sorted(revs)
            t.cancel()
        finally:
            await _close(servers, [a, b])
    run(main())


def test_concurrent_patches_retry_on_stale_cache(run, store):
    async def main():
        servers, (a, b) = await _workers(store)
        try:
            await a.create("configmaps", {"metadata": {"name": "cm", "namespace": "default"}, "data": {}})
            await _eventually(lambda: b.get("configmaps", "cm", "default"))
            # 40 merge patches of distinct keys racing through both workers: none may be lost
            await asyncio.gather(*((a if i % 2 else b).patch("configmaps", "cm", {"data": {f"k{i}": str(i)}}, "default")
                                   for i in range(40)))
            cm = await _eventually(lambda: a.get("configmaps", "cm", "default"))
            final = await _eventually(lambda: _if(a.get("configmaps", "cm", "default"), lambda o: len(o["data"]) == 40))
            assert final["data"] == {f"k{i}": str(i) for i in range(40)} and cm
            # a PUT with a stale resourceVersion is still a 409
            stale = dict(final, metadata=dict(final["metadata"], resourceVersion="3"))
            with pytest.raises(APIStatusError) as ei:
                await b.update("configmaps", stale)
            assert ei.value.code == 409
        finally:
            await _close(servers, [a, b])
    run(main())


async def _if(coro, pred):
    o = await coro
    return o if pred(o) else None


def test_device_claims_across_workers(run, store):
    async def main():
        servers, (a, b) = await _workers(store)
        try:
            await a.create("nodes", {"metadata": {"name": "n0"}})
            pa = await a.create("pods", gpu_pod("pa"))
            pb = await a.create("pods", gpu_pod("pb"))
            await _eventually(lambda: b.get("pods", "pb", "default"))
            era, erb = pa["spec"]["extendedResources"][0]["name"], pb["spec"]["extendedResources"][0]["name"]
            # two binds of the SAME GPU racing through different workers: exactly one wins
            res = await asyncio.gather(a.bind("default", "pa", "n0", {era: {"resources": ["GPU-0"]}}),
                                       b.bind("default", "pb", "n0", {erb: {"resources": ["GPU-0"]}}),
                                       return_exceptions=True)
            errs = [r for r in res if isinstance(r, Exception)]
            assert len(errs) == 1 and isinstance(errs[0], APIStatusError) and errs[0].code == 409
            assert "already assigned" in str(errs[0])
            winner = "pa" if not isinstance(res[0], Exception) else "pb"
            loser = "pb" if winner == "pa" else "pa"
            lerr = erb if loser == "pb" else era
            # deleting the winner releases the claim (grace 0), then the loser can bind it
            await a.delete("pods", winner, "default", grace_period=0)
            await _eventually(lambda: _absent(b, winner))
            await b.bind("default", loser, "n0", {lerr: {"resources": ["GPU-0"]}})
            p = await _eventually(lambda: _if(a.get("pods", loser, "default"), lambda o: o["spec"].get("nodeName")))
            assert p["spec"]["extendedResources"][0]["assigned"] == ["GPU-0"]
            # a terminal pod releases its devices too
            await a.patch("pods", loser, {"status": {"phase": "Succeeded"}}, "default", "merge", "status")
            pc = await a.create("pods", gpu_pod("pc"))
            await _eventually(lambda: b.get("pods", "pc", "default"))
            await b.bind("default", "pc", "n0", {pc["spec"]["extendedResources"][0]["name"]: {"resources": ["GPU-0"]}})
        finally:
            await _close(servers, [a, b])
    run(main())


def test_read_and_bind_right_after_write_on_other_worker(run, store, monkeypatch):
    """A worker that has not yet applied another worker's write must not answer 404 for it
    (pods cached on every worker here, so the cache-lag path is what runs)."""
    monkeypatch.setenv("KAMD_SHARED_CACHE_ALL", "1")

    async def main():
        servers, (a, b) = await _workers(store)
        # make worker b lag: its store events are applied 30 ms late (in order)
        rs = servers[1].rstore
        wid = next(iter(rs._watches))
        orig, backlog = rs._watches[wid], []
        loop = asyncio.get_running_loop()

        def late(t, kv):
            backlog.append((t, kv))
            loop.call_later(0.03, lambda: orig(*backlog.pop(0)))
        rs._watches[wid] = late
        try:
            await a.create("nodes", {"metadata": {"name": "n0"}})
            for i in range(10):
                p = await a.create("pods", gpu_pod(f"q{i}"))
                got = await b.get("pods", f"q{i}", "default")          # no polling
                assert got["metadata"]["uid"] == p["metadata"]["uid"]
                er = p["spec"]["extendedResources"][0]["name"]
                p2 = await a.create("pods", gpu_pod(f"r{i}"))
                await b.bind("default", f"r{i}", "n0", {p2["spec"]["extendedResources"][0]["name"]: {"resources": [f"G{i}"]}})
                assert er
            assert servers[1].m_retries.value("miss") >= 10     # the lag path really ran
        finally:
            await _close(servers, [a, b])
    run(main())


def test_watch_from_newer_list_on_lagging_worker(run, store):
    """List on a worker that is ahead, watch on one that lags: no replay of what the list had."""
    async def main():
        servers, (a, b) = await _workers(store)
        rs = servers[1].rstore
        wid = next(iter(rs._watches))
        orig, backlog = rs._watches[wid], []
        loop = asyncio.get_running_loop()

        def late(t, kv):
            backlog.append((t, kv))
            loop.call_later(0.1, lambda: orig(*backlog.pop(0)))
        rs._watches[wid] = late
        try:
            await a.create("configmaps", {"metadata": {"name": "old", "namespace": "default"}})
            lst = await a.list("configmaps", "default")
            w = await b.watch("configmaps", "default", lst["metadata"]["resourceVersion"])
            seen = []

            async def drain():
                async for typ, obj in w:
                    seen.append((typ, obj["metadata"]["name"]))
            t = asyncio.ensure_future(drain())
            await a.create("configmaps", {"metadata": {"name": "new", "namespace": "default"}})
            await asyncio.sleep(0.4)
            assert seen == [("ADDED", "new")]
            t.cancel()
        finally:
            await _close(servers, [a, b])
    run(main())


async def _absent(c, name):
    try:
        await c.get("pods", name, "default")
        return False
    except APIStatusError as e:
        return e.code == 404


def test_worker_restart_reloads_state(run, store):
    async def main():
        servers, (a,) = await _workers(store, 1)
        await a.create("pods", gpu_pod("keep"))
        await _close(servers, [a])
        servers, (b,) = await _workers(store, 1)
        try:
            p = await b.get("pods", "keep", "default")
            assert p["metadata"]["name"] == "keep"
            lst = await b.list("pods", "default")
            assert int(lst["metadata"]["resourceVersion"]) >= int(p["metadata"]["resourceVersion"])
        finally:
            await _close(servers, [b])
    run(main())


def test_native_watch_fanout_semantics(run, store):
    """Watches on shared-store workers are served by kamd-etcd's C++ fan-out: selector
    transitions (ADDED when an object starts matching, DELETED when it stops), resume from a
    resourceVersion, initial state, field selectors indexed by node, timeoutSeconds, and 410 for
    a compacted version. The same semantics as the in-process cacher (cacher.go dispatchEvent)."""
    from kubernetes_amd.storage.remote import RemoteStore

    async def main():
        servers, (a, b) = await _workers(store)
        try:
            assert servers[0].fanout is not None
            sel_events, node_events = [], []
            w1 = await b.watch("pods", "default", "0", label_selector="app=hip,tier!=db")
            w2 = await a.watch("pods", None, "0", field_selector="spec.nodeName=gpu-node-1")

            async def drain(w, out):
                async for typ, obj in w:
                    out.append((typ, obj["metadata"]["name"]))
            t1 = asyncio.ensure_future(drain(w1, sel_events))
            t2 = asyncio.ensure_future(drain(w2, node_events))
            await a.create("pods", dict(gpu_pod("x1"), metadata={"name": "x1", "namespace": "default",
                                                                  "labels": {"app": "hip"}}))
            await a.create("pods", dict(gpu_pod("x2"), metadata={"name": "x2", "namespace": "default",
                                                                  "labels": {"app": "other"}}))
            await b.patch("pods", "x2", {"metadata": {"labels": {"app": "hip"}}}, "default")      # starts matching
            await a.patch("pods", "x1", {"metadata": {"labels": {"tier": "db"}}}, "default")      # stops matching
            p = await a.get("pods", "x2", "default")
            er = p["spec"]["extendedResources"][0]["name"]
            await a.bind("default", "x2", "gpu-node-1", {er: {"resources": ["g0"]}})
            await a.delete("pods", "x2", "default", grace_period=0)
            await _eventually(lambda: asyncio.sleep(0, len(sel_events) >= 5 and len(node_events) >= 2))
            assert sel_events == [("ADDED", "x1"), ("ADDED", "x2"), ("DELETED", "x1"), ("MODIFIED", "x2"),
                                  ("DELETED", "x2")][:len(sel_events)] and len(sel_events) == 5
            assert node_events == [("ADDED", "x2"), ("DELETED", "x2")]
            # resume from a resourceVersion: exactly the later changes
            rv = (await a.list("pods", "default"))["metadata"]["resourceVersion"]
            await a.patch("pods", "x1", {"metadata": {"labels": {"more": "1"}}}, "default")
            w3 = await b.watch("pods", "default", rv, timeout_seconds=1)
            got = [(t, o["metadata"]["name"]) async for t, o in w3]        # ends at the timeout
            assert got == [("MODIFIED", "x1")]
            # a compacted version is 410 Gone, delivered as an ERROR event
            rs = await RemoteStore(store).connect()
            await rs.compact(int(rv) + 1)
            from kubernetes_amd.client.rest import APIStatusError as _E
            w4 = await a.watch("pods", "default", "2", timeout_seconds=2)
            with pytest.raises(_E) as ei:
                [x async for x in w4]
            assert ei.value.code == 410
            m = (await a.http.request("GET", "/metrics", None, "text/plain"))[1].decode()
            assert "apiserver_watch_fanout_handoffs_total" in m
            t1.cancel()
            t2.cancel()
        finally:
            await _close(servers, [a, b])
    run(main())


def test_uncached_pods_and_events_read_from_store(run, store):
    """Shared-mode workers do not cache pods/events: reads hit the store (no lag to wait for),
    the worker's store watch excludes them (progress frames still advance its revision), list
    selectors, conflicts, device claims, quota admission, TTL reaping and the non-fan-out watch
    fallback all work from the store."""
    from kubernetes_amd.storage import wire

    async def main():
        servers, (a, b) = await _workers(store)
        try:
            assert servers[0].uncached == {"pods", "events"} and servers[1].uncached == {"pods", "events"}
            await a.create("nodes", {"metadata": {"name": "n0"}})
            for i in range(5):
                p = await a.create("pods", dict(gpu_pod(f"u{i}"), metadata={"name": f"u{i}", "namespace": "default",
                                                                            "labels": {"i": str(i)}}))
                got = await b.get("pods", f"u{i}", "default")       # no polling: read from the store
                assert got == p
            assert not servers[0].caches["pods"].by_key and not servers[1].caches["pods"].by_key
            # the last writes were pods only: b's applied revision still reaches them (PROGRESS)
            rv = int(p["metadata"]["resourceVersion"])
            await asyncio.wait_for(servers[1]._wait_applied(rv), 5)
            lst = await b.list("pods", "default", label_selector="i in (1,3)")
            assert [x["metadata"]["name"] for x in lst["items"]] == ["u1", "u3"]
            assert int(lst["metadata"]["resourceVersion"]) >= rv
            lim = await b.list("pods", "default", limit=2)
            assert len(lim["items"]) == 2 and lim["metadata"].get("continue")
            # stale update → 409; fresh one works through the other worker
            cur = await a.get("pods", "u0", "default")
            with pytest.raises(APIStatusError) as ei:
                await b.update("pods", dict(cur, metadata=dict(cur["metadata"], resourceVersion="1")), "default")
            assert ei.value.code == 409
            cur["metadata"].setdefault("labels", {})["fresh"] = "1"
            assert (await b.update("pods", cur, "default"))["metadata"]["labels"]["fresh"] == "1"
            with pytest.raises(APIStatusError) as ei:
                await b.create("pods", gpu_pod("u0"))
            assert ei.value.code == 409
            # device claims across workers
            p0 = await b.get("pods", "u0", "default")
            p1 = await b.get("pods", "u1", "default")
            await a.bind("default", "u0", "n0", {p0["spec"]["extendedResources"][0]["name"]: {"resources": ["G0"]}})
            with pytest.raises(APIStatusError) as ei:
                await b.bind("default", "u1", "n0", {p1["spec"]["extendedResources"][0]["name"]: {"resources": ["G0"]}})
            assert ei.value.code == 409
            # quota admission charges status.used with the quota's resourceVersion, across workers
            await a.create("namespaces", {"metadata": {"name": "q"}})
            await a.create("resourcequotas", {"metadata": {"name": "rq", "namespace": "q"},
                                              "spec": {"hard": {"pods": "2"}}}, "q")
            await a.patch("resourcequotas", "rq", {"status": {"hard": {"pods": "2"}, "used": {"pods": "0"}}}, "q",
                          "merge", "status")

            async def counted():
                return ((await b.get("resourcequotas", "rq", "q")).get("status") or {}).get("used")
            await _eventually(counted)
            for i in range(2):
                await b.create("pods", {"metadata": {"name": f"q{i}", "namespace": "q"},
                                        "spec": {"containers": [{"name": "c", "image": "x"}]}}, "q")
            with pytest.raises(APIStatusError) as ei:
                await b.create("pods", {"metadata": {"name": "q2", "namespace": "q"},
                                        "spec": {"containers": [{"name": "c", "image": "x"}]}}, "q")
            assert ei.value.code == 403
            # watch that the fan-out cannot serve (quantity selector) → store-watch fallback
            w = await b.watch("pods", "default", "0", label_selector="i>2")
            seen = []

            async def drain():
                async for typ, obj in w:
                    seen.append((typ, obj["metadata"]["name"]))
                    if ("DELETED", "u4") in seen:
                        return
            t = asyncio.ensure_future(drain())
            await _eventually(lambda: asyncio.sleep(0, result=("ADDED", "u4") in seen))
            assert ("ADDED", "u3") in seen and not any(n in ("u0", "u1", "u2") for _, n in seen)
            await a.delete("pods", "u4", "default")
            await asyncio.wait_for(t, 5)
            w.close()
            assert servers[1].m_fanout.value("pods") == 0     # nothing above used the fan-out
            # events: uncached, TTL reaping reads them from the store
            await a.create("events", {"metadata": {"name": "e1", "namespace": "default"},
                                      "involvedObject": {"kind": "Pod", "name": "u0", "namespace": "default"},
                                      "reason": "X", "message": "m", "type": "Normal",
                                      "lastTimestamp": "2000-01-01T00:00:00Z"}, "default")
            assert (await b.get("events", "e1", "default"))["reason"] == "X"
            assert await servers[1].reap_events() == 1
            with pytest.raises(APIStatusError):
                await a.get("events", "e1", "default")
            assert not servers[0].caches["events"].by_key
            with pytest.raises(RuntimeError):
                servers[0].list_objects("pods")
            assert wire.PROGRESS == 10
        finally:
            await _close(servers, [a, b])
    run(main())


def test_shard_selection_native_matches_python(run, store):
    """`?kamdShard=i/n`: kamd-etcd's native fan-out and the API server's list filter select the
    same pods (zlib CRC-32 of namespace/name + the offset label, malformed offsets read as 0)."""
    from kubernetes_amd.api.sharding import SHARD_OFFSET_LABEL

    async def main():
        servers, (a,) = await _workers(store, 1)
        try:
            offs = ["", "1", "12", "x", "99999999999", "7"]
            for i in range(30):
                md = {"name": f"s{i}", "namespace": "default"}
                if offs[i % len(offs)]:
                    md["labels"] = {SHARD_OFFSET_LABEL: offs[i % len(offs)]}
                await a.create("pods", dict(gpu_pod(f"s{i}"), metadata=md))
            seen_all = []
            for k in range(3):
                listed = {p["metadata"]["name"] for p in
                          (await a.list("pods", "default", extra={"kamdShard": f"{k}/3"}))["items"]}
                w = await a.watch("pods", "default", "0", timeout_seconds=1, extra={"kamdShard": f"{k}/3"})
                watched = {o["metadata"]["name"] async for _, o in w}
                assert listed == watched and listed
                seen_all += listed
            assert sorted(seen_all) == sorted(f"s{i}" for i in range(30))     # a partition
            assert servers[0].m_fanout.value("pods") >= 3
            with pytest.raises(APIStatusError) as ei:
                await a.list("pods", "default", extra={"kamdShard": "3/3"})
            assert ei.value.code == 400
        finally:
            await _close(servers, [a])
    run(main())
