"""PATCH support: JSON merge patch (RFC 7386), JSON patch (RFC 6902) and strategic merge
patch (the merge-key subset of `staging/src/k8s.io/apimachinery/pkg/util/strategicpatch`).
"""
from __future__ import annotations

import copy

# patchMergeKey per list field (from the struct tags in core/v1 types.go)
MERGE_KEYS = {
    "containers": "name", "initContainers": "name", "volumes": "name", "env": "name",
    "volumeMounts": "mountPath", "ports": "containerPort", "conditions": "type",
    "imagePullSecrets": "name", "ownerReferences": "uid", "taints": "key", "addresses": "type",
    "tolerations": None, "finalizers": None, "extendedResources": "name", "containerStatuses": "name",
    "initContainerStatuses": "name", "hostAliases": "ip",
}


def merge_patch(target, patch):
    if not isinstance(patch, dict):
        return patch  # the decoded patch document is owned by the request: share, don't copy
    if not isinstance(target, dict):
        target = {}
    out = dict(target)
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out


def strategic_merge_patch(target, patch, field=None):
    if not isinstance(patch, dict):
        if isinstance(patch, list) and isinstance(target, list):
            return _merge_list(target, patch, field)
        return patch  # the decoded patch document is owned by the request: share, don't copy
    if patch.get("$patch") == "replace":
        p = dict(patch)
        p.pop("$patch")
        return p
    if not isinstance(target, dict):
        target = {}
    out = dict(target)
    for k, v in patch.items():
        if k.startswith("$"):
            continue
        if k.startswith("$setElementOrder/"):
            continue
        if v is None:
            out.pop(k, None)
        elif isinstance(v, list):
            out[k] = _merge_list(out.get(k) or [], v, k)
        else:
            out[k] = strategic_merge_patch(out.get(k), v, k)
    return out


def _merge_list(target, patch, field):
    key = MERGE_KEYS.get(field)
    if key is None or not all(isinstance(x, dict) for x in patch):
        if field == "finalizers" or (field in MERGE_KEYS and MERGE_KEYS[field] is None and field != "tolerations"):
            # primitive lists with merge strategy: union
            res = list(target)
            for x in patch:
                if x not in res:
                    res.append(x)
            return res
        return patch  # the decoded patch document is owned by the request: share, don't copy
    res = [dict(x) if isinstance(x, dict) else x for x in target]
    for item in patch:
        kv = item.get(key)
        idx = next((i for i, x in enumerate(res) if isinstance(x, dict) and x.get(key) == kv), None)
        if item.get("$patch") == "delete":
            if idx is not None:
                res.pop(idx)
            continue
        if idx is None:
            res.append(strategic_merge_patch({}, item))
        else:
            res[idx] = strategic_merge_patch(res[idx], item)
    return res


class JSONPatchError(ValueError):
    pass


def _ptr(path):
    if path == "":
        return []
    if not path.startswith("/"):
        raise JSONPatchError(f"invalid path {path!r}")
    return [p.replace("~1", "/").replace("~0", "~") for p in path[1:].split("/")]


def _walk(doc, parts):
    cur = doc
    for p in parts:
        if isinstance(cur, list):
            cur = cur[int(p)]
        else:
            cur = cur[p]
    return cur


def json_patch(doc, ops):
    doc = copy.deepcopy(doc)
    for op in ops:
        kind = op.get("op")
        parts = _ptr(op.get("path", ""))
        try:
            if kind == "test":
                if _walk(doc, parts) != op.get("value"):
                    raise JSONPatchError(f"test failed at {op.get('path')}")
                continue
            if kind in ("move", "copy"):
                val = copy.deepcopy(_walk(doc, _ptr(op["from"])))
                if kind == "move":
                    fparts = _ptr(op["from"])
                    parent = _walk(doc, fparts[:-1])
                    if isinstance(parent, list):
                        parent.pop(int(fparts[-1]))
                    else:
                        del parent[fparts[-1]]
                op = {"op": "add", "path": op["path"], "value": val}
                kind = "add"
            parent = _walk(doc, parts[:-1]) if parts else None
            last = parts[-1] if parts else None
            if kind == "add":
                if parent is None:
                    doc = op["value"]
                elif isinstance(parent, list):
                    if last == "-":
                        parent.append(op["value"])
                    else:
                        parent.insert(int(last), op["value"])
                else:
                    parent[last] = op["value"]
            elif kind == "remove":
                if isinstance(parent, list):
                    parent.pop(int(last))
                else:
                    del parent[last]
            elif kind == "replace":
                if parent is None:
                    doc = op["value"]
                elif isinstance(parent, list):
                    parent[int(last)] = op["value"]
                else:
                    if last not in parent:
                        raise JSONPatchError(f"replace of missing path {op.get('path')}")
                    parent[last] = op["value"]
            else:
                raise JSONPatchError(f"unknown op {kind!r}")
        except (KeyError, IndexError, ValueError, TypeError) as e:
            if isinstance(e, JSONPatchError):
                raise
            raise JSONPatchError(f"{kind} {op.get('path')}: {e}") from e
    return doc


def apply_patch(content_type: str, target, patch):
    ct = (content_type or "").split(";")[0].strip()
    if ct == "application/json-patch+json":
        if not isinstance(patch, list):
            raise JSONPatchError("json patch must be a list")
        return json_patch(target, patch)
    if ct == "application/merge-patch+json":
        return merge_patch(target, patch)
    if ct in ("application/strategic-merge-patch+json", "application/apply-patch+yaml"):
        return strategic_merge_patch(target, patch)
    raise ValueError(f"unsupported patch type {ct!r}")


def create_merge_patch(original, modified):
    """The RFC 7386 merge patch turning `original` into `modified` (what `kubectl edit
    --output-patch` prints; `jsonmergepatch.CreateThreeWayJSONMergePatch` with no base)."""
    if not isinstance(original, dict) or not isinstance(modified, dict):
        return modified
    out = {}
    for k in original:
        if k not in modified:
            out[k] = None
    for k, v in modified.items():
        if k not in original:
            out[k] = v
        elif original[k] != v:
            out[k] = create_merge_patch(original[k], v) if isinstance(v, dict) and isinstance(original[k], dict) else v
    return out
