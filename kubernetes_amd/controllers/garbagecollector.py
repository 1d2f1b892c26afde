"""Garbage collector: an owner-reference graph over every deletable resource the API serves.

Parity: `pkg/controller/garbagecollector/`
  * monitors — one informer per resource that supports delete+list+watch, taken from discovery
    (`GetDeletableResources`, `garbagecollector.go:594`) minus `ignoredResources`
    (`graph_builder.go:354`); re-discovered every `discovery_period` (`Sync`, `:169`; the
    controller manager passes 30 s) and, sooner, whenever a CustomResourceDefinition changes;
  * the graph (`graph.go`, `graph_builder.go:processGraphChanges`) — uid -> node with owners and
    dependents; an owner that is referenced but not yet observed is a *virtual* node that is
    verified against the API server;
  * attemptToDelete (`garbagecollector.go:363 attemptToDeleteItem`) — an object is deleted only
    when none of its owners is *solid*: every owner is confirmed absent by a live GET by
    apiVersion/kind/name with a UID check (`isDangling`, `:282`) or is itself waiting for its
    dependents (foreground); solid owners plus dangling ones get the dangling references
    patched away instead (`deleteOwnerRefPatch`, `patch.go:29`);
  * foreground deletion (`processDeletingDependentsItem`, `:480`) — the owner keeps its
    `foregroundDeletion` finalizer until no dependent with `blockOwnerDeletion: true` remains;
    cycles are broken with `patchToUnblockOwnerReferences` (`patch.go:40`);
  * orphaning (`attemptToOrphanWorker`, `:531`) — dependents lose the owner reference, then the
    owner loses its `orphan` finalizer;
  * `absentOwnerCache` (`uid_cache.go`) — owners confirmed absent are not fetched again.

The reference runs the graph builder in its own goroutine fed by a channel; here informer
handlers run on the event loop in watch order, so graph updates are applied inline and only the
API-calling work (attempt-to-delete / attempt-to-orphan) goes through the rate-limited queue.
"""
from __future__ import annotations

import asyncio
import collections
import logging

from ..api import codec, meta as m
from ..client.informer import Informer
from ..client.rest import APIStatusError, is_conflict, is_not_found
from .base import Controller

log = logging.getLogger("garbagecollector")

ORPHAN = "orphan"
FOREGROUND = "foregroundDeletion"

# graph_builder.go:354
IGNORED_RESOURCES = frozenset({
    ("extensions", "replicationcontrollers"), ("", "bindings"), ("", "componentstatuses"), ("", "events"),
    ("events.k8s.io", "events"),
    ("authentication.k8s.io", "tokenreviews"), ("authorization.k8s.io", "subjectaccessreviews"),
    ("authorization.k8s.io", "selfsubjectaccessreviews"), ("authorization.k8s.io", "localsubjectaccessreviews"),
    ("authorization.k8s.io", "selfsubjectrulesreviews"), ("apiregistration.k8s.io", "apiservices"),
    ("apiextensions.k8s.io", "customresourcedefinitions"),
})

# monitored from the first sync, before discovery answers (always served, the shared informers
# most controllers use anyway); discovery adds everything else
CORE_MONITORS = ("pods", "replicasets", "deployments", "jobs", "cronjobs", "daemonsets", "statefulsets",
                 "replicationcontrollers", "controllerrevisions", "configmaps", "secrets", "services",
                 "endpoints", "poddisruptionbudgets")

_DELETABLE_VERBS = frozenset({"delete", "list", "watch"})


def deletable_resources(resource_lists, ignored=IGNORED_RESOURCES):
    """`GetDeletableResources` over discovery documents.

    `resource_lists`: APIResourceList dicts, each group's versions in preference order (the
    `/api/v1` list first). For every group/resource the first (most preferred) version serving
    it wins (`ServerPreferredResources`); sub-resources, resources without delete+list+watch and
    `ignored` group/resources are dropped, as are the extra group/versions this server serves the
    same storage under (`meta.ALIASES`: e.g. extensions/v1beta1 deployments is apps/v1 storage).
    Returns [ResourceInfo] in discovery order."""
    out, seen = [], set()
    for rl in resource_lists:
        gv = rl.get("groupVersion") or ""
        group, _, version = gv.rpartition("/")
        if not version or gv.count("/") > 1 or (gv.count("/") == 1 and not group):
            continue              # not a valid group/version: ignored (ParseGroupVersion fails)
        for r in rl.get("resources") or ():
            name = r.get("name") or ""
            if "/" in name or (group, name) in seen:
                continue
            seen.add((group, name))
            if not _DELETABLE_VERBS.issubset(r.get("verbs") or ()):
                continue
            if (group, name) in ignored:
                continue
            canon = m.BY_PLURAL.get(name) if (group, version, name) in m.ALIASES else None
            if canon is not None and canon.group != group:
                continue          # the canonical group lists the same objects
            out.append(m.ResourceInfo(group, version, r.get("kind") or "", name, bool(r.get("namespaced"))))
    return out


async def discover(client):
    """Fetch every group's resource lists (preferred version first) from the API server."""
    async def get(path):
        st, body = await client.raw("GET", path)
        if st != 200:
            raise APIStatusError(st, {"message": body[:200].decode(errors="replace")})
        return codec.loads(body)
    lists = [await get("/api/v1")]
    groups = await get("/apis")
    for g in groups.get("groups") or ():
        vs = [v["groupVersion"] for v in g.get("versions") or ()]
        pref = (g.get("preferredVersion") or {}).get("groupVersion")
        if pref in vs:
            vs.remove(pref)
            vs.insert(0, pref)
        for gv in vs:
            try:
                lists.append(await get(f"/apis/{gv}"))
            except APIStatusError as e:       # one failing group does not stop discovery
                log.debug("discovery of %s failed: %s", gv, e)
    return lists


class NotObserved(Exception):
    """A virtual node that exists but no monitor has reported yet: retried with backoff."""


class Node:
    """`graph.go node`: identity, owners as last observed, dependents, and the state bits."""
    __slots__ = ("uid", "api_version", "kind", "namespace", "name", "owners", "dependents",
                 "virtual", "being_deleted", "deleting_dependents")

    def __init__(self, uid, api_version, kind, namespace, name, owners=(), virtual=False,
                 being_deleted=False, deleting_dependents=False):
        self.uid, self.api_version, self.kind = uid, api_version, kind
        self.namespace, self.name = namespace or None, name
        self.owners = list(owners)
        self.dependents: set = set()
        self.virtual = virtual
        self.being_deleted = being_deleted
        self.deleting_dependents = deleting_dependents

    def __repr__(self):
        return f"Node({self.api_version} {self.kind} {self.namespace or ''}/{self.name} uid={self.uid}" + \
               (" virtual" if self.virtual else "") + ")"

    def blocking_dependents(self, graph):
        out = []
        for du in self.dependents:
            dep = graph.get(du)
            if dep is None:
                continue
            for ref in dep.owners:
                if ref.get("uid") == self.uid and ref.get("blockOwnerDeletion"):
                    out.append(dep)
                    break
        return out

    def unblock_patch(self):
        """`patchToUnblockOwnerReferences`: every blocking owner reference -> blockOwnerDeletion false."""
        refs = [dict(r, blockOwnerDeletion=False) for r in self.owners if r.get("blockOwnerDeletion")]
        return {"metadata": {"ownerReferences": refs, "uid": self.uid}}


def delete_owner_ref_patch(dependent_uid, *owner_uids):
    """`deleteOwnerRefPatch`: a strategic-merge patch removing the given owners (merge key uid)."""
    return {"metadata": {"ownerReferences": [{"$patch": "delete", "uid": u} for u in owner_uids],
                         "uid": dependent_uid}}


def references_diffs(old, new):
    """`referencesDiffs`: (added, removed, changed[(old, new)]) owner references by UID."""
    o = {r.get("uid"): r for r in old or ()}
    n = {r.get("uid"): r for r in new or ()}
    added = [r for u, r in n.items() if u not in o]
    removed = [r for u, r in o.items() if u not in n]
    changed = [(o[u], n[u]) for u in n if u in o and o[u] != n[u]]
    return added, removed, changed


def _deleting(obj):
    return bool((obj.get("metadata") or {}).get("deletionTimestamp"))


def _has_fin(obj, fin):
    return fin in ((obj.get("metadata") or {}).get("finalizers") or ())


class UIDCache:
    """`uid_cache.go`: a bounded LRU set of UIDs."""

    def __init__(self, size=500):
        self.size = size
        self._d = collections.OrderedDict()

    def add(self, uid):
        self._d[uid] = True
        self._d.move_to_end(uid)
        while len(self._d) > self.size:
            self._d.popitem(last=False)

    def has(self, uid):
        if uid in self._d:
            self._d.move_to_end(uid)
            return True
        return False

    def __len__(self):
        return len(self._d)


class GarbageCollector(Controller):
    name = "garbagecollector"
    workers = 20                   # --concurrent-gc-syncs

    def __init__(self, client, factory, recorder=None, discovery_period=30.0, ignored_resources=None,
                 absent_cache_size=500):
        super().__init__(client, factory, recorder)
        self.discovery_period = discovery_period
        self.ignored = frozenset(ignored_resources) if ignored_resources is not None else IGNORED_RESOURCES
        self.graph: dict[str, Node] = {}
        self.absent = UIDCache(absent_cache_size)
        self.monitors: dict[m.ResourceInfo, tuple] = {}   # ri -> (informer, owned_by_gc)
        self.kinds: dict[tuple, m.ResourceInfo] = {}      # (group, kind) -> resource for owner lookups
        self._sync_task = None
        self._resync_now = None
        self._started = False

    # -- monitors ----------------------------------------------------------------------
    def setup(self):
        for p in CORE_MONITORS:
            ri = m.BY_PLURAL.get(p)
            if ri is not None and (ri.group, ri.plural) not in self.ignored:
                self._monitor(ri)
        self.crd_inf = self.factory.get("customresourcedefinitions")
        kick = lambda *_a: self._kick()    # noqa: E731
        self.crd_inf.add_handler(kick, kick, kick)

    def _kick(self):
        if self._resync_now is not None:
            self._resync_now.set()

    def _monitor(self, ri):
        if ri in self.monitors:
            return
        shared_key = (ri.plural, None, None, None)
        canon = m.BY_PLURAL.get(ri.plural)
        if canon is not None and canon.group == ri.group and canon.version == ri.version and \
                (not self._started or shared_key in self.factory.informers):
            inf, owned = self.factory.get(ri.plural), False      # one watch shared with other controllers
        else:
            inf, owned = Informer(self.client, ri), True
        gv, kind = ri.group_version, ri.kind
        inf.add_handler(lambda o: self._on_event("add", gv, kind, o, None),
                        lambda old, new: self._on_event("update", gv, kind, new, old),
                        lambda o: self._on_event("delete", gv, kind, o, None))
        self.monitors[ri] = (inf, owned)
        self.kinds.setdefault((ri.group, ri.kind), ri)
        if owned and self._started:
            inf.start()

    def _unmonitor(self, ri):
        inf, owned = self.monitors.pop(ri)
        if owned:
            inf.stop()
        if self.kinds.get((ri.group, ri.kind)) == ri:
            del self.kinds[(ri.group, ri.kind)]

    def sync_monitors(self, resources):
        """`resyncMonitors`: start monitors for new deletable resources, stop vanished ones
        (only those this collector owns; shared informers belong to the factory)."""
        want = set(resources)
        for ri in resources:
            self._monitor(ri)
            self.kinds[(ri.group, ri.kind)] = ri
        for ri in [r for r, (_, owned) in self.monitors.items() if owned and r not in want]:
            self._unmonitor(ri)

    async def resync_discovery(self):
        if not hasattr(self.client, "raw"):
            return False                # fake clients: the compiled-in monitors only
        try:
            lists = await discover(self.client)
        except (APIStatusError, OSError, ConnectionError) as e:
            log.debug("garbage collector discovery failed: %s", e)
            return False
        res = deletable_resources(lists, self.ignored)
        for rl in lists:                 # alias group/versions still map owner kinds
            g = (rl.get("groupVersion") or "").rpartition("/")[0]
            for r in rl.get("resources") or ():
                if "/" not in (r.get("name") or "") and (g, r.get("kind")) not in self.kinds:
                    canon = m.BY_PLURAL.get(r["name"])
                    if canon is not None and canon.kind == r.get("kind"):
                        self.kinds[(g, r["kind"])] = canon
        self.sync_monitors(res)
        return True

    async def _discovery_loop(self):
        # exits on the stop flag as well as on cancellation: on Python 3.10 asyncio.wait_for can
        # swallow a CancelledError that races with the event being set, and a loop that then
        # carries on would hang the process's shutdown (asyncio.run cancels and awaits all tasks)
        while not self._gc_stopped:
            await self.resync_discovery()
            try:
                await asyncio.wait_for(self._resync_now.wait(), self.discovery_period)
                await asyncio.sleep(0.05)          # coalesce a burst of CRD events
            except asyncio.TimeoutError:
                pass
            self._resync_now.clear()

    def start(self):
        self._started = True
        for inf, owned in list(self.monitors.values()):
            if owned and inf._task is None:
                inf.start()
        self._resync_now = asyncio.Event()
        self._gc_stopped = False
        super().start()
        self._sync_task = asyncio.ensure_future(self._discovery_loop())

    def stop(self):
        self._gc_stopped = True
        super().stop()
        if self._sync_task:
            self._sync_task.cancel()
        for inf, owned in self.monitors.values():
            if owned:
                inf.stop()

    # -- graph builder (graph_builder.go processGraphChanges) ----------------------------
    def _on_event(self, etype, api_version, kind, obj, old):
        md = obj.get("metadata") or {}
        uid = md.get("uid")
        if not uid:
            return
        n = self.graph.get(uid)
        if n is not None:
            n.virtual = False                       # markObserved
        if etype in ("add", "update"):
            owners = list(md.get("ownerReferences") or ())
            if n is None:
                n = Node(uid, api_version, kind, md.get("namespace"), md.get("name"), owners,
                         being_deleted=_deleting(obj), deleting_dependents=_deleting(obj) and _has_fin(obj, FOREGROUND))
                self.graph[uid] = n
                self._add_to_owners(n, owners)
            else:
                if n.api_version != api_version or n.kind != kind or n.name != md.get("name"):
                    # a virtual node, now observed: adopt the object's own identity
                    n.api_version, n.kind, n.name = api_version, kind, md.get("name")
                    n.namespace = md.get("namespace") or None
                added, removed, changed = references_diffs(n.owners, owners)
                if added or removed or changed:
                    self._unblocked_owners(removed, changed)
                    n.owners = owners
                    self._add_to_owners(n, added)
                    for ref in removed:
                        on = self.graph.get(ref.get("uid"))
                        if on is not None:
                            on.dependents.discard(uid)
                if _deleting(obj):
                    n.being_deleted = True
            self._transitions(old, obj, n)
        elif etype == "delete":
            if n is None:
                return
            self._remove(n)
            if n.dependents:
                self.absent.add(uid)
            for du in n.dependents:
                self._attempt_delete(du)
            for ref in n.owners:
                on = self.graph.get(ref.get("uid"))
                if on is not None and on.deleting_dependents:
                    self._attempt_delete(on.uid)

    def _add_to_owners(self, n, refs):
        for ref in refs:
            ou = ref.get("uid")
            if not ou:
                continue
            on = self.graph.get(ou)
            if on is None:
                on = Node(ou, ref.get("apiVersion", ""), ref.get("kind", ""), n.namespace, ref.get("name", ""),
                          virtual=True)
                self.graph[ou] = on
                on.dependents.add(n.uid)
                self._attempt_delete(ou)          # verify the owner against the API server
            else:
                on.dependents.add(n.uid)

    def _remove(self, n):
        self.graph.pop(n.uid, None)
        for ref in n.owners:
            on = self.graph.get(ref.get("uid"))
            if on is not None:
                on.dependents.discard(n.uid)

    def _unblocked_owners(self, removed, changed):
        """`addUnblockedOwnersToDeleteQueue`."""
        for ref in removed:
            if ref.get("blockOwnerDeletion") and ref.get("uid") in self.graph:
                self._attempt_delete(ref["uid"])
        for o, n in changed:
            if o.get("blockOwnerDeletion") and not n.get("blockOwnerDeletion") and n.get("uid") in self.graph:
                self._attempt_delete(n["uid"])

    def _transitions(self, old, obj, n):
        """`processTransitions`: deletion starting with the orphan / foreground finalizer."""
        if not _deleting(obj) or (old is not None and _deleting(old)):
            return
        if _has_fin(obj, ORPHAN):
            self.queue.add(f"o|{n.uid}")
            return
        if _has_fin(obj, FOREGROUND):
            n.deleting_dependents = True
            for du in n.dependents:
                self._attempt_delete(du)
            self._attempt_delete(n.uid)

    def _attempt_delete(self, uid):
        self.queue.add(f"d|{uid}")

    # -- workers --------------------------------------------------------------------------
    async def sync(self, key):
        kind, uid = key.split("|", 1)
        n = self.graph.get(uid)
        if n is None:
            return
        if kind == "o":
            await self.attempt_to_orphan(n)
            return
        await self.attempt_to_delete_item(n)
        if n.virtual and uid in self.graph:
            # not yet observed through a monitor: look again later, with backoff (issue 56121)
            raise NotObserved(n)

    def resource_for(self, api_version, kind):
        """RESTMapping of an owner reference: discovered kinds first, then the compiled-in
        kinds of the same group (or of a group serving the same storage under an alias)."""
        group = api_version.rpartition("/")[0]
        ri = self.kinds.get((group, kind))
        if ri is not None:
            return ri
        ri = m.BY_KIND.get(kind)
        if ri is not None and (ri.group == group or any(g == group and p == ri.plural for (g, _v, p) in m.ALIASES)):
            return ri
        raise LookupError(f"no resource for {api_version} {kind} (not discovered yet)")

    def _handle(self, ri):
        """The resource argument the client takes: the plural for registered resources."""
        canon = m.BY_PLURAL.get(ri.plural)
        return ri.plural if canon is not None and canon.group == ri.group else ri

    async def _get(self, api_version, kind, namespace, name):
        ri = self.resource_for(api_version, kind)
        return await self.client.get(self._handle(ri), name, namespace if ri.namespaced else None)

    async def is_dangling(self, ref, n):
        """(dangling, owner): absent from the API server or present under another UID."""
        ou = ref.get("uid")
        if self.absent.has(ou):
            return True, None
        try:
            owner = await self._get(ref.get("apiVersion", ""), ref.get("kind", ""), n.namespace, ref.get("name", ""))
        except APIStatusError as e:
            if is_not_found(e):
                self.absent.add(ou)
                return True, None
            raise
        if m.uid_of(owner) != ou:
            self.absent.add(ou)
            return True, None
        return False, owner

    async def classify_references(self, n, refs):
        solid, dangling, waiting = [], [], []
        for ref in refs:
            d, owner = await self.is_dangling(ref, n)
            if d:
                dangling.append(ref)
            elif _deleting(owner) and _has_fin(owner, FOREGROUND):
                waiting.append(ref)
            else:
                solid.append(ref)
        return solid, dangling, waiting

    def _virtual_delete(self, n):
        """`enqueueVirtualDeleteEvent`: the object does not exist; drop it from the graph."""
        self._on_event("delete", n.api_version, n.kind, {"metadata": {"uid": n.uid}}, None)
        self.graph.pop(n.uid, None)

    async def attempt_to_delete_item(self, n):
        if n.being_deleted and not n.deleting_dependents:
            return
        try:
            latest = await self._get(n.api_version, n.kind, n.namespace, n.name)
        except APIStatusError as e:
            if is_not_found(e):
                self._virtual_delete(n)
                n.virtual = False
                return
            raise
        if m.uid_of(latest) != n.uid:
            self._virtual_delete(n)
            n.virtual = False
            return
        if n.deleting_dependents:
            await self.process_deleting_dependents(n)
            return
        refs = (latest.get("metadata") or {}).get("ownerReferences") or []
        if not refs:
            return
        solid, dangling, waiting = await self.classify_references(n, refs)
        if solid:
            if not dangling and not waiting:
                return
            await self._patch_refs_away(n, latest, [r["uid"] for r in dangling + waiting])
            return
        if waiting and n.dependents:
            for du in list(n.dependents):
                dep = self.graph.get(du)
                if dep is not None and dep.deleting_dependents:
                    # cycle guard: stop blocking our owners, then delete in the foreground
                    await self._patch(n, n.unblock_patch(), latest)
                    break
            await self._delete(n, "Foreground")
            return
        if _has_fin(latest, ORPHAN):
            policy = "Orphan"
        elif _has_fin(latest, FOREGROUND):
            policy = "Foreground"
        else:
            policy = "Background"
        await self._delete(n, policy)

    async def process_deleting_dependents(self, n):
        blocking = n.blocking_dependents(self.graph)
        if not blocking:
            await self.remove_finalizer(n, FOREGROUND)
            return
        for dep in blocking:
            if not dep.deleting_dependents:
                self._attempt_delete(dep.uid)

    async def attempt_to_orphan(self, owner):
        for du in list(owner.dependents):
            dep = self.graph.get(du)
            if dep is None:
                continue
            try:
                await self._patch_refs_away(dep, None, [owner.uid])
            except APIStatusError as e:
                if not is_not_found(e):
                    raise
        await self.remove_finalizer(owner, ORPHAN)

    # -- API writes -----------------------------------------------------------------------
    async def _delete(self, n, policy):
        ri = self.resource_for(n.api_version, n.kind)
        try:
            await self.client.delete(self._handle(ri), n.name, n.namespace if ri.namespaced else None,
                                     propagation=policy, uid=n.uid)
        except APIStatusError as e:
            if not (is_not_found(e) or e.code == 409):
                raise

    async def _patch(self, n, patch, latest=None):
        ri = self.resource_for(n.api_version, n.kind)
        ns = n.namespace if ri.namespaced else None
        if m.BY_PLURAL.get(ri.plural) in m.BUILTIN and self._handle(ri) == ri.plural:
            return await self.client.patch(ri.plural, n.name, patch, ns, patch_type="strategic")
        # custom resources take no strategic-merge patch: send the resulting list as a merge patch
        if latest is None:
            latest = await self.client.get(self._handle(ri), n.name, ns)
        refs = list((latest.get("metadata") or {}).get("ownerReferences") or ())
        p = patch["metadata"]["ownerReferences"]
        drop = {x["uid"] for x in p if x.get("$patch") == "delete"}
        repl = {x["uid"]: x for x in p if x.get("$patch") != "delete"}
        refs = [repl.get(r.get("uid"), r) for r in refs if r.get("uid") not in drop]
        return await self.client.patch(self._handle(ri), n.name,
                                       {"metadata": {"ownerReferences": refs or None}}, ns)

    async def _patch_refs_away(self, n, latest, owner_uids):
        return await self._patch(n, delete_owner_ref_patch(n.uid, *owner_uids), latest)

    async def remove_finalizer(self, n, fin):
        """GET + PUT with conflict retry (`removeFinalizer`, `operations.go`)."""
        ri = self.resource_for(n.api_version, n.kind)
        ns = n.namespace if ri.namespaced else None
        for _ in range(5):
            try:
                cur = await self.client.get(self._handle(ri), n.name, ns)
            except APIStatusError as e:
                if is_not_found(e):
                    return
                raise
            if m.uid_of(cur) != n.uid:
                return
            fins = [f for f in cur["metadata"].get("finalizers") or () if f != fin]
            if len(fins) == len(cur["metadata"].get("finalizers") or ()):
                return
            cur["metadata"]["finalizers"] = fins or None
            try:
                await self.client.update(self._handle(ri), cur, ns)
                return
            except APIStatusError as e:
                if is_not_found(e):
                    return
                if not is_conflict(e):
                    raise
        raise RuntimeError(f"removing finalizer {fin} from {n}: too many conflicts")
