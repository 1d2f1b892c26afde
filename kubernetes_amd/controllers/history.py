"""ControllerRevision history for DaemonSets and StatefulSets.

Parity: `pkg/controller/history/controller_history.go` — a revision is a ControllerRevision named
`<owner>-<hash>` owned (controller ref) by the workload, labelled `controller-revision-hash`,
with `data` = the pod template patch and a monotonically increasing `revision`; an existing
revision whose data equals the current template is reused (and re-numbered to the newest, as
on a rollback); revisions beyond `revisionHistoryLimit` (default 10) are pruned oldest first,
never the current one.
"""
from __future__ import annotations

import hashlib
import json

from ..client.rest import APIStatusError, is_already_exists, is_not_found

REVISION_HASH = "controller-revision-hash"


def revision_hash(template) -> str:
    return hashlib.sha256(json.dumps(template or {}, sort_keys=True).encode()).hexdigest()[:10]


def sort_controller_revisions(revisions):
    """`SortControllerRevisions`: by revision number (stable for equal numbers)."""
    return sorted(revisions or (), key=lambda r: int(r.get("revision", 0)))


def next_revision(revisions) -> int:
    """`NextRevision`: one past the highest revision, 1 for an empty history."""
    return max((int(r.get("revision", 0)) for r in revisions or ()), default=0) + 1


def equal_revision(a, b) -> bool:
    """`EqualRevision`: the same hash label (when both carry one) and the same data."""
    if a is None or b is None:
        return a is b
    ha = (a["metadata"].get("labels") or {}).get(REVISION_HASH)
    hb = (b["metadata"].get("labels") or {}).get(REVISION_HASH)
    if ha is not None and hb is not None and ha != hb:
        return False
    return (a.get("data") or {}) == (b.get("data") or {})


def find_equal_revisions(revisions, needle):
    """`FindEqualRevisions`: the revisions equal to `needle`."""
    return [r for r in revisions or () if equal_revision(r, needle)]


def revisions_of(lister_items, owner_uid):
    out = [r for r in lister_items
           if any(o.get("uid") == owner_uid and o.get("controller") for o in r["metadata"].get("ownerReferences") or ())]
    return sort_controller_revisions(out)


async def ensure_revision(client, owner, kind, template, existing, limit=10):
    """The ControllerRevision for `template` (created or promoted), pruning old history beyond
    `limit` (None: no pruning here — the caller truncates with `truncate_history`)."""
    md = owner["metadata"]
    ns, h = md["namespace"], revision_hash(template)
    name = f"{md['name']}-{h}"
    newest = max((int(r.get("revision", 0)) for r in existing), default=0)
    # `FindEqualRevisions`: one of ours with this hash and this template (its name may carry a
    # collision suffix)
    cur = next((r for r in existing if r["metadata"]["name"] == name
                or ((r["metadata"].get("labels") or {}).get(REVISION_HASH) == h
                    and ((r.get("data") or {}).get("spec") or {}).get("template") == template)), None)
    if cur is None:
        cur = await _create_revision(client, owner, kind, template, name, h, newest + 1)
    elif int(cur.get("revision", 0)) < newest:
        # rolled back to an older template: it becomes the newest revision again
        cur = await client.patch("controllerrevisions", cur["metadata"]["name"], {"revision": newest + 1}, ns)
    if limit is None:
        return cur
    keep = [r for r in existing if r["metadata"]["name"] != cur["metadata"]["name"]]
    excess = len(keep) + 1 - max(1, limit)
    for r in sorted(keep, key=lambda r: int(r.get("revision", 0)))[:max(0, excess)]:
        try:
            await client.delete("controllerrevisions", r["metadata"]["name"], ns)
        except APIStatusError as e:
            if not is_not_found(e):
                raise
    return cur


async def _create_revision(client, owner, kind, template, name, h, number):
    """`CreateControllerRevision` with collision handling: an existing revision of the same name
    is reused when it holds the same template and is ours or an orphan (then adopted —
    `AdoptControllerRevision`, e.g. the history of a set deleted with orphan propagation and
    re-created); one owned by another controller, or holding other data, bumps a collision
    count into the name and the create is retried."""
    md = owner["metadata"]
    ns = md["namespace"]
    ref = {"apiVersion": "apps/v1", "kind": kind, "name": md["name"], "uid": md["uid"], "controller": True,
           "blockOwnerDeletion": True}
    collision = 0
    while True:
        rname = name if collision == 0 else f"{name}-{collision}"
        rev = {"apiVersion": "apps/v1", "kind": "ControllerRevision",
               "metadata": {"name": rname, "namespace": ns, "labels": {REVISION_HASH: h}, "ownerReferences": [ref]},
               "data": {"spec": {"template": template}}, "revision": number}
        try:
            return await client.create("controllerrevisions", rev, ns)
        except APIStatusError as e:
            if not is_already_exists(e):
                raise
        got = await client.get("controllerrevisions", rname, ns)
        same = ((got.get("data") or {}).get("spec") or {}).get("template") == template
        owner_ref = next((r for r in got["metadata"].get("ownerReferences") or () if r.get("controller")), None)
        if same and owner_ref is not None and owner_ref.get("uid") == md["uid"]:
            return got
        if same and owner_ref is None:
            refs = list(got["metadata"].get("ownerReferences") or ()) + [ref]
            return await client.patch("controllerrevisions", rname,
                                      {"metadata": {"ownerReferences": refs, "uid": got["metadata"].get("uid")}}, ns)
        collision += 1
        if collision > 16:
            raise RuntimeError(f"controller revision {name}: too many hash collisions")


async def truncate_history(client, revisions, live, limit):
    """`truncateHistory` (stateful_set_control.go:124) / `cleanupHistory` (daemon/update.go:110):
    delete non-live revisions (live = the current and update revisions and every pod's), oldest
    first, until at most `limit` of them remain."""
    history = sorted((r for r in revisions if r["metadata"]["name"] not in live),
                     key=lambda r: int(r.get("revision", 0)))
    for r in history[:max(0, len(history) - max(0, int(limit)))]:
        try:
            await client.delete("controllerrevisions", r["metadata"]["name"], r["metadata"]["namespace"])
        except APIStatusError as e:
            if not is_not_found(e):
                raise
