"""Topology-aware extended-resource (device) allocator — the scheduler's ER step (fork F4),
re-designed for MI355X xGMI hives.

Reference behaviour (`plugin/pkg/scheduler/core/extended_resources.go:42-183`): for every
surviving node, greedily take the first N devices (Go map iteration order) that match the
pod's attribute selector; no health check; no topology.

MI355X-first design:
  * only Healthy devices are candidates (the kubelet would reject the others anyway);
  * selectors are quantity-aware (`amd.com/hbm Gt 256Gi`, `amd.com/memory Gt 200000`);
  * an N-GPU request is placed inside ONE xGMI hive — RCCL rings are per-link bound, so an
    N-GPU job wants N GPUs that can drive N-1 links each. The hive with the fewest free
    devices that still fits is chosen (best fit: keeps whole hives free for big jobs);
    inside it, a NUMA node that holds the whole set is preferred; the chosen packages must be
    pairwise linked: the plugin publishes each device's hive index and the bitmask of hive
    peers it reaches over an up xGMI link (`amd.com/xgmi-node` / `amd.com/xgmi-peers`, from
    `amdsmi_topo_get_link_type`), and the set must be a clique of that graph — a GPU that
    booted with 6/7 links is never paired with the peer it cannot reach. (Devices without the
    peer attributes fall back to "at least N-1 healthy xGMI links each".)
  * single-GPU pods pack into the most-used hive / NUMA node first (anti-fragmentation);
  * compute partitions (SPX/DPX/QPX/CPX: 1/2/4/8 logical devices per package, sharing its
    `amd.com/socket`) — partitions of one package talk over the on-package fabric, so a
    k-partition request takes the fewest packages (whole free packages first, the tail
    best-fit into the package with the fewest free partitions that holds it); a 1-partition
    pod fills partly used packages before opening a fresh one. The xGMI link requirement
    counts packages, not partitions (a CPX request for 8 spans one package: no links needed);
  * `amd.com/xgmi-policy` pod annotation: `required` (fail rather than span hives) or
    `preferred` (default: span hives only when no single hive fits, with a low score);
  * deterministic order (device index) instead of map order.
Returns a binding `{er_name: {"resources": [ids]}}` plus a 0..10 topology score used by the
`XGMITopology` priority.
"""
from __future__ import annotations

from itertools import combinations

from ..api import core
from ..api.labels import SelectorError, node_selector_requirements_as_selector

# logical devices per MI355X package per compute-partition mode (8 XCDs per package)
PARTITIONS_PER_SOCKET = {"SPX": 1, "DPX": 2, "QPX": 4, "CPX": 8}

POLICY_ANNOTATION = "amd.com/xgmi-policy"
REQUIRED, PREFERRED = "required", "preferred"


class Request:
    """One pod-level extended resource request, with its selector compiled once."""
    __slots__ = ("name", "rname", "count", "selector", "error")

    def __init__(self, name, rname, count, required):
        self.name, self.rname, self.count = name, rname, count
        self.error = None
        try:
            self.selector = node_selector_requirements_as_selector(required) if required else None
        except SelectorError as e:
            self.selector = None
            self.error = str(e)


def _idx(dev):
    try:
        return int((dev.get("attributes") or {}).get(core.ATTR_INDEX, 1 << 30))
    except ValueError:
        return 1 << 30


def _links(dev):
    try:
        return int((dev.get("attributes") or {}).get(core.ATTR_XGMI_LINKS, 7))
    except ValueError:
        return 0


def _pps(dev):
    return PARTITIONS_PER_SOCKET.get((dev.get("attributes") or {}).get(core.ATTR_PARTITION, "SPX"), 1)


def _need_links(dev, n):
    """xGMI links each device of an n-device set must have: one per OTHER package spanned."""
    if n <= 1:
        return 0
    p = _pps(dev)
    return n - 1 if p == 1 else -(-n // p) - 1


def _peer(dev):
    """(hive index, peer bitmask) or None when the plugin does not publish pairwise links."""
    a = dev.get("attributes") or {}
    node, peers = a.get(core.ATTR_XGMI_NODE), a.get(core.ATTR_XGMI_PEERS)
    if node is None or peers is None:
        return None
    try:
        return int(node), int(peers, 16)
    except ValueError:
        return None


def _clique(devs, n):
    """The first n-subset of devs (list of (id, dev), in preference order) whose packages are
    pairwise xGMI-linked, preferring sets inside one NUMA node; None if there is none. Returns
    (chosen, numa_fit). Small by construction: at most 8 packages per hive (C(8,4) = 70)."""
    info = [_peer(d) for _, d in devs]
    if any(x is None for x in info):
        return None
    numa = [(d.get("attributes") or {}).get(core.ATTR_NUMA, "") for _, d in devs]
    best = None
    for combo in combinations(range(len(devs)), n):
        ok = True
        for a, b in combinations(combo, 2):
            na, ma = info[a]
            nb, mb = info[b]
            if na != nb and not ((ma >> nb) & 1 and (mb >> na) & 1):
                ok = False
                break
        if not ok:
            continue
        fit = len({numa[k] for k in combo}) == 1
        if fit:
            return [devs[k] for k in combo], True
        if best is None:
            best = [devs[k] for k in combo]
    return (best, False) if best is not None else None


def _has_peers(devs):
    return bool(devs) and all(_peer(d) is not None for _, d in devs)


def _sock(did, dev):
    return (dev.get("attributes") or {}).get(core.ATTR_SOCKET, did)


def _score(free, n, numa_fit):
    # 10 for a perfect fit, decreasing with leftover fragments in the chosen hive
    return 9.0 - min(free - n, 8) / 8.0 * 4.0 + (1.0 if numa_fit else 0.0)


def fast_path(requests) -> bool:
    """Feasibility + score can be computed from the per-hive free lists alone."""
    return len(requests) == 1 and requests[0].selector is None and not requests[0].error


def feasible(requests, er, policy=PREFERRED):
    """Filter-phase check for a single selector-less request (the common case): returns
    (ok, score, reason) without materialising a binding. Must agree with `allocate()`."""
    r = requests[0]
    n = r.count
    hives = er.hive_free.get(r.rname)
    if not hives or er.nfree.get(r.rname, 0) < n:
        return False, 0, f"Insufficient {r.rname}"
    first = next((d for devs in hives.values() for d in devs.values()), None)
    if first is not None and _pps(first) > 1:
        # compute-partitioned node: the package-level plan decides feasibility and score
        cands = [(i, d) for devs in hives.values() for i, d in devs.items() if _links(d) >= _need_links(d, n)]
        if len(cands) < n:
            return False, 0, f"Insufficient {r.rname}"
        ids, sc = _pick(cands, n, policy)
        if ids is None:
            return False, 0, f"no single xGMI hive has {n} free {r.rname}"
        return True, sc, ""
    need_links = n - 1 if n > 1 else 0
    if n > 1 and first is not None and _peer(first) is not None:
        # pairwise topology published: a hive qualifies if its free devices hold a clique of n
        ok = sorted(((len(devs), h, devs) for h, devs in hives.items() if len(devs) >= n), key=lambda t: (t[0], t[1]))
        for c, _, devs in ok:
            items = sorted(devs.items(), key=lambda x: _idx(x[1]))
            got = _clique(items, n)
            if got is not None:
                return True, _score(c, n, got[1]), ""
        if sum(len(d) for d in hives.values()) < n:
            return False, 0, f"Insufficient {r.rname}"
        if policy == REQUIRED:
            return False, 0, f"no xGMI-connected set of {n} free {r.rname} in one hive"
        return True, 1.0, ""
    best = None
    total = 0
    for h, devs in hives.items():
        if need_links:
            c = sum(1 for d in devs.values() if _links(d) >= need_links)
        else:
            c = len(devs)
        total += c
        if c >= n and (best is None or (c, h) < best[:2]):
            best = (c, h, devs)
    if best is not None:
        c, _, devs = best
        numa = {}
        for d in devs.values():
            if not need_links or _links(d) >= need_links:
                k = (d.get("attributes") or {}).get(core.ATTR_NUMA, "")
                numa[k] = numa.get(k, 0) + 1
        return True, _score(c, n, any(v >= n for v in numa.values())), ""
    if total < n:
        return False, 0, f"Insufficient {r.rname}"
    if policy == REQUIRED and n > 1:
        return False, 0, f"no single xGMI hive has {n} free {r.rname}"
    return True, 1.0, ""


def allocate(requests, er, policy=PREFERRED):
    """requests: list[Request]; er: ERManager of the node.
    Returns (binding, score, reason). binding is None on failure."""
    binding = {}
    taken: set = set()
    score_sum = 0.0
    for r in requests:
        if r.error:
            return None, 0, r.error
        avail = er.available.get(r.rname)
        if not avail:
            return None, 0, f"Insufficient {r.rname}"
        sel = r.selector
        cands = []
        hf = er.hive_free.get(r.rname)
        it = ((i, d) for devs in hf.values() for i, d in devs.items()) if hf is not None else avail.items()
        for did, dev in it:
            if did in taken or dev.get("health", core.HEALTHY) != core.HEALTHY:
                continue
            attrs = dev.get("attributes") or {}
            if sel is not None and not sel.matches(attrs):
                continue
            if r.count > 1 and _peer(dev) is None and _links(dev) < _need_links(dev, r.count):
                continue
            cands.append((did, dev))
        if len(cands) < r.count:
            return None, 0, f"Insufficient {r.rname}"
        ids, s = _pick(cands, r.count, policy)
        if ids is None:
            return None, 0, f"no xGMI-connected set of {r.count} free {r.rname} in one hive"
        binding[r.name] = {"resources": ids}
        taken.update(ids)
        score_sum += s
    return binding, (score_sum / len(requests)) if requests else 10.0, ""


def _group(cands, key):
    g = {}
    for did, dev in cands:
        g.setdefault((dev.get("attributes") or {}).get(key, ""), []).append((did, dev))
    return g


def _pick(cands, n, policy):
    hives = _group(cands, core.ATTR_HIVE)
    fitting = [(len(v), h, v) for h, v in hives.items() if len(v) >= n]
    if n > 1 and fitting and all(_has_peers(v) and not any(_pps(d) > 1 for _, d in v) for _, _, v in fitting):
        # best-fit hive first, but only a hive whose free packages hold a linked n-clique
        fitting.sort(key=lambda t: (t[0], t[1]))
        for free, _, devs in fitting:
            got = _clique(sorted(devs, key=lambda x: _idx(x[1])), n)
            if got is not None:
                chosen, numa_fit = got
                return [d for d, _ in chosen], _score(free, n, numa_fit)
        fitting = []
    if fitting:
        # best fit: the hive with the fewest free devices that still holds n
        fitting.sort(key=lambda t: (t[0], t[1]))
        free, _, devs = fitting[0]
        if any(_pps(d) > 1 for _, d in devs):
            return _pick_partitions(devs, n)
        numas = _group(devs, core.ATTR_NUMA)
        nf = [(len(v), k, v) for k, v in numas.items() if len(v) >= n]
        if nf:
            nf.sort(key=lambda t: (t[0], t[1]))
            chosen = sorted(nf[0][2], key=lambda x: _idx(x[1]))[:n]
            numa_bonus = 1.0
        else:
            # fill NUMA nodes largest-first so the set spans as few as possible
            chosen = []
            for _, _, v in sorted(((len(v), k, v) for k, v in numas.items()), key=lambda t: (-t[0], t[1])):
                chosen.extend(sorted(v, key=lambda x: _idx(x[1])))
            chosen = chosen[:n]
            numa_bonus = 0.0
        return [d for d, _ in chosen], _score(free, n, numa_bonus > 0)
    if policy == REQUIRED and n > 1:
        return None, 0
    # span hives: largest hives first, deterministic
    chosen = []
    for _, _, v in sorted(((len(v), h, v) for h, v in hives.items()), key=lambda t: (-t[0], t[1])):
        chosen.extend(sorted(v, key=lambda x: _idx(x[1])))
    return [d for d, _ in chosen[:n]], 1.0


def _pick_partitions(devs, n):
    """Place n compute partitions inside one hive on the fewest packages. Whole free packages
    are taken largest-first; the tail goes to the package with the fewest free partitions that
    still holds it (best fit), so partly used packages fill up before fresh ones are opened.
    Score: 10 for a set that spans the minimum number of packages and leaves no stranded free
    partitions on them, lower for each partition left behind on a touched package."""
    socks = {}
    for did, dev in devs:
        socks.setdefault(_sock(did, dev), []).append((did, dev))
    for v in socks.values():
        v.sort(key=lambda x: _idx(x[1]))
    order = sorted(socks, key=lambda k: (-len(socks[k]), str(k)))
    chosen, rem, used, left = [], n, 0, 0
    while rem > 0 and order:
        fit = [k for k in order if len(socks[k]) >= rem]
        if fit:
            k = min(fit, key=lambda k: (len(socks[k]), str(k)))
        else:
            k = order[0]
        order.remove(k)
        take = socks[k][:rem]
        chosen.extend(take)
        left += len(socks[k]) - len(take)
        rem -= len(take)
        used += 1
    p = max(_pps(d) for _, d in devs)
    minimal = -(-n // p)
    score = 9.0 - min(left, p) / p * 4.0 + (1.0 if used <= minimal else 0.0)
    return [d for d, _ in chosen], score
