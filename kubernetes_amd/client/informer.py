"""Reflector + indexer + shared informer.

Parity: `staging/src/k8s.io/client-go/tools/cache/reflector.go:98,239` (ListAndWatch, resume
from last resourceVersion, relist on 410 Gone), `shared_informer.go:188,343` (handlers,
HasSynced), `store.go`/`index.go` (thread-safe store with indexers).

Handlers are plain callables invoked on the event loop in watch order; they must not block
(enqueue into a workqueue instead, as reference controllers do).
"""
from __future__ import annotations

import asyncio
import logging

from ..api import meta as m
from .rest import APIStatusError, is_gone

log = logging.getLogger("informer")


def key_func(obj):
    return m.ns_name(obj)


class Indexer:
    def __init__(self, indexers=None):
        self.items: dict[str, dict] = {}
        self.indexers = dict(indexers or {})
        self.indices: dict[str, dict[str, set]] = {n: {} for n in self.indexers}
        self.generation = 0       # bumped on every change: derived views can be cached against it

    def add_indexer(self, name, fn):
        self.indexers[name] = fn
        idx = self.indices[name] = {}
        for k, o in self.items.items():
            for v in fn(o) or ():
                idx.setdefault(v, set()).add(k)

    def _unindex(self, key, obj):
        for n, fn in self.indexers.items():
            idx = self.indices[n]
            for v in fn(obj) or ():
                s = idx.get(v)
                if s:
                    s.discard(key)
                    if not s:
                        del idx[v]

    def _index(self, key, obj):
        for n, fn in self.indexers.items():
            idx = self.indices[n]
            for v in fn(obj) or ():
                idx.setdefault(v, set()).add(key)

    def put(self, key, obj):
        self.generation += 1
        old = self.items.get(key)
        if old is not None and self.indexers:
            self._unindex(key, old)
        self.items[key] = obj
        if self.indexers:
            self._index(key, obj)
        return old

    def delete(self, key):
        self.generation += 1
        old = self.items.pop(key, None)
        if old is not None and self.indexers:
            self._unindex(key, old)
        return old

    def get(self, key):
        return self.items.get(key)

    def list(self):
        return list(self.items.values())

    def by_index(self, name, value):
        return [self.items[k] for k in self.indices.get(name, {}).get(value, ())]

    def keys(self):
        return list(self.items.keys())


class Informer:
    def __init__(self, client, resource, namespace=None, label_selector=None, field_selector=None,
                 indexers=None, watch_timeout=300, extra_query=None, resync_period=0.0):
        self.client = client
        # resync (`sharedIndexInformer` resyncCheckPeriod): every period each cached object is
        # re-delivered as an update with old == new, so level-driven handlers re-examine state
        # that no watch event touched; 0 = off
        self.resync_period = resync_period
        self._resync_task = None
        self.extra_query = extra_query
        self.resource = resource
        self.namespace = namespace
        self.label_selector = label_selector
        self.field_selector = field_selector
        self.store = Indexer(indexers)
        self.handlers = []
        self.synced = asyncio.Event()
        self.rv = None
        self.watch_timeout = watch_timeout
        self._task = None
        self._stream = None
        self._stopped = False

    def add_handler(self, on_add=None, on_update=None, on_delete=None):
        self.handlers.append((on_add, on_update, on_delete))
        # like AddEventHandler on a running informer: replay current state
        if self.synced.is_set() and on_add:
            for o in self.store.list():
                on_add(o)

    def has_synced(self):
        return self.synced.is_set()

    def get(self, key):
        return self.store.get(key)

    def list(self):
        return self.store.list()

    def _fire(self, kind, obj, old=None):
        for h in self.handlers:
            fn = h[kind]
            if fn is None:
                continue
            try:
                if kind == 1:
                    fn(old, obj)
                else:
                    fn(obj)
            except Exception:
                log.exception("informer handler for %s failed", self.resource)

    async def _list(self):
        items, rv = await self.client.list_all(self.resource, self.namespace, self.label_selector, self.field_selector,
                                               extra=self.extra_query)
        seen = set()
        for o in items:
            k = key_func(o)
            seen.add(k)
            old = self.store.put(k, o)
            if old is None:
                self._fire(0, o)
            elif old.get("metadata", {}).get("resourceVersion") != o["metadata"].get("resourceVersion"):
                self._fire(1, o, old)
        for k in [k for k in self.store.keys() if k not in seen]:
            old = self.store.delete(k)
            self._fire(2, old)
        self.rv = rv
        self.synced.set()

    def _handle(self, etype, obj):
        k = key_func(obj)
        self.rv = obj.get("metadata", {}).get("resourceVersion", self.rv)
        if etype == "ADDED" or etype == "MODIFIED":
            old = self.store.put(k, obj)
            if old is None:
                self._fire(0, obj)
            else:
                self._fire(1, obj, old)
        elif etype == "DELETED":
            old = self.store.delete(k)
            self._fire(2, obj if old is None else obj)

    async def run(self):
        backoff = 0.05
        while not self._stopped:
            try:
                if self.rv is None:
                    await self._list()
                st = await self.client.watch(self.resource, self.namespace, self.rv, self.label_selector,
                                             self.field_selector, self.watch_timeout, extra=self.extra_query)
                self._stream = st
                backoff = 0.05
                async for evs in st.batches():
                    for etype, obj in evs:
                        self._handle(etype, obj)
                st.close()
            except asyncio.CancelledError:
                raise
            except APIStatusError as e:
                if is_gone(e):
                    self.rv = None  # relist
                    continue
                log.warning("watch %s failed: %s", self.resource, e)
                await asyncio.sleep(backoff)
                backoff = min(backoff * 2, 2)
            except (ConnectionError, OSError) as e:
                if self._stopped:
                    return
                log.debug("watch %s connection error: %s", self.resource, e)
                await asyncio.sleep(backoff)
                backoff = min(backoff * 2, 2)

    async def _resync_loop(self):
        while not self._stopped:
            await asyncio.sleep(self.resync_period)
            if self.synced.is_set():
                for o in self.store.list():
                    self._fire(1, o, o)

    def start(self):
        self._task = asyncio.ensure_future(self.run())
        if self.resync_period > 0:
            self._resync_task = asyncio.ensure_future(self._resync_loop())
        return self._task

    async def wait_synced(self, timeout=30):
        await asyncio.wait_for(self.synced.wait(), timeout)

    def stop(self):
        self._stopped = True
        if self._stream:
            self._stream.close()
        if self._task:
            self._task.cancel()
        if self._resync_task:
            self._resync_task.cancel()


def resync_period(min_resync):
    """`ResyncPeriod(s)` of cmd/kube-controller-manager/app/controllermanager.go: a random period
    in [min, 2*min), so the informers of one process do not resync in lockstep."""
    import random
    return min_resync * (1.0 + random.random()) if min_resync > 0 else 0.0


class InformerFactory:
    """SharedInformerFactory: one informer per (resource, namespace, selectors); `resync` is the
    default resync period of the informers it makes (0 = none)."""

    def __init__(self, client, resync=0.0):
        self.client = client
        self.informers = {}
        self.resync = resync

    def get(self, resource, namespace=None, label_selector=None, field_selector=None):
        k = (resource, namespace, label_selector, field_selector)
        inf = self.informers.get(k)
        if inf is None:
            inf = self.informers[k] = Informer(self.client, resource, namespace, label_selector, field_selector,
                                               resync_period=self.resync)
        return inf

    def start(self):
        for inf in self.informers.values():
            if inf._task is None:
                inf.start()

    async def wait_for_cache_sync(self, timeout=30):
        await asyncio.gather(*(i.wait_synced(timeout) for i in self.informers.values()))

    def stop(self):
        for inf in self.informers.values():
            inf.stop()
