"""Node scoring. Parity: `plugin/pkg/scheduler/algorithm/priorities/*` (LeastRequested,
MostRequested, BalancedResourceAllocation, SelectorSpread, NodeAffinity, TaintToleration,
NodePreferAvoidPods, InterPodAffinity, ImageLocality, ResourceLimits) with the default weights of `algorithmprovider/defaults/defaults.go`.

MI355X additions:
  * XGMITopology   — the allocator's hive/NUMA fit score (scheduler/topology.py), weight 2;
  * GPUBinPacking  — prefer nodes whose free-GPU count after placement is smallest, so whole
                     8-GPU nodes stay free for 8-GPU jobs (device-level MostRequested), weight 1.
Each function returns a 0..10 score for one node; `normalize` rescales relative scores.
"""
from __future__ import annotations

from ..api import core
from ..api.labels import SelectorError, node_selector_requirements_as_selector

MAX = 10.0


def _unused(req, cap):
    """`calculateUnusedScore`: integer ((capacity - requested) * 10) / capacity."""
    if cap == 0 or req > cap:
        return 0
    return (cap - req) * 10 // cap


def _used(req, cap):
    """`calculateUsedScore`: integer (requested * 10) / capacity."""
    if cap == 0 or req > cap:
        return 0
    return req * 10 // cap


def least_requested(pod, pi, ni, ctx):
    return (_unused(ni.nz_cpu + pi.nz_cpu, ni.alloc_cpu) + _unused(ni.nz_mem + pi.nz_mem, ni.alloc_mem)) // 2


def most_requested(pod, pi, ni, ctx):
    return (_used(ni.nz_cpu + pi.nz_cpu, ni.alloc_cpu) + _used(ni.nz_mem + pi.nz_mem, ni.alloc_mem)) // 2


def balanced_resource_allocation(pod, pi, ni, ctx):
    """`calculateBalancedResourceAllocation`: int((1 - |cpuFraction - memFraction|) * 10); a
    fraction of a zero capacity is 1, and any fraction >= 1 scores 0."""
    c = (ni.nz_cpu + pi.nz_cpu) / ni.alloc_cpu if ni.alloc_cpu else 1.0
    m = (ni.nz_mem + pi.nz_mem) / ni.alloc_mem if ni.alloc_mem else 1.0
    if c >= 1 or m >= 1:
        return 0
    return int((1 - abs(c - m)) * MAX)


def _service_match(p, ns, sels):
    if p["metadata"].get("namespace", "default") != ns:
        return False
    lbl = p["metadata"].get("labels") or {}
    return any(all(lbl.get(k) == v for k, v in sel.items()) for sel in sels)


def selector_spread(pod, pi, ni, ctx):
    """`selector_spreading.go` CalculateSpreadPriorityMap: raw count of the pod's siblings on the
    node — pods of the same controller, or pods any of the pod's services select; normalized
    reversed later."""
    owner = ctx.owner_uid
    sels = ctx.service_selectors
    if not owner and not sels:
        return 0.0
    ns = ctx.namespace
    n = 0
    for p, _ in ni.pods.values():
        md = p["metadata"]
        if md.get("namespace", "default") != ns or md.get("deletionTimestamp"):
            continue            # a deleted predecessor does not count for spreading
        if owner and any(ref.get("uid") == owner for ref in md.get("ownerReferences") or ()):
            n += 1
        elif sels and _service_match(p, ns, sels):
            n += 1
    return n


def service_spreading(pod, pi, ni, ctx):
    """`ServiceSpreadingPriority` (defaults.go:95-106): SelectorSpread over services only (no
    controller listers) — raw count of pods the pod's services select on the node."""
    sels = ctx.service_selectors
    if not sels:
        return 0.0
    ns = ctx.namespace
    return float(sum(1 for p, _ in ni.pods.values() if _service_match(p, ns, sels)))


def equal(pod, pi, ni, ctx):
    """`EqualPriorityMap`: every node scores 1."""
    return 1.0


# -- argument-based custom priorities (Policy `priorities[].argument`) ------------------------
# `plugin/pkg/scheduler/factory/plugins.go:299-340` RegisterCustomPriorityFunction

def make_service_anti_affinity(label):
    """`selector_spreading.go:209-254` ServiceAntiAffinity: spread the pods of the pod's first
    service over the values of `label`. A node with the label scores
    10 * (servicePods - podsOnItsLabelValue) / servicePods (10 when the service has no pods);
    a node without it scores 0."""
    def service_anti_affinity(pod, pi, ni, ctx):
        v = ni.labels.get(label)
        if v is None:
            return 0.0
        counts, total = ctx.service_label_counts(label)
        if not total:
            return MAX
        return float(int(MAX * (total - counts.get(v, 0)) / total))
    service_anti_affinity.global_view = True
    return service_anti_affinity


def make_label_preference(label, presence):
    """`node_label.go` NodeLabelPrioritizer: 10 when the node has (presence) / lacks (not
    presence) the label, else 0."""
    def label_preference(pod, pi, ni, ctx):
        return MAX if (label in ni.labels) == presence else 0.0
    return label_preference


def node_affinity(pod, pi, ni, ctx):
    prefs = ctx.node_affinity_prefs
    if not prefs:
        return 0.0
    s = 0.0
    for weight, sel in prefs:
        if sel.matches(ni.labels):
            s += weight
    return s


def taint_toleration(pod, pi, ni, ctx):
    if not ni.taints:
        return 0.0
    tols = [t for t in (pod.get("spec") or {}).get("tolerations") or () if t.get("effect") in (None, "", core.TAINT_PREFER_NO_SCHEDULE)]
    return float(sum(1 for t in ni.taints if t.get("effect") == core.TAINT_PREFER_NO_SCHEDULE and not core.tolerates(tols, t)))


_AVOID_CACHE: dict = {}


def _avoided_controllers(raw):
    """{(kind, uid)} of a node's `scheduler.alpha.kubernetes.io/preferAvoidPods` annotation
    (`v1helper.GetAvoidPodsFromNodeAnnotations`); a malformed annotation avoids nothing."""
    hit = _AVOID_CACHE.get(raw)
    if hit is None:
        import json
        hit = set()
        try:
            for a in (json.loads(raw) or {}).get("preferAvoidPods") or ():
                pc = (a.get("podSignature") or {}).get("podController")
                if pc:
                    hit.add((pc.get("kind"), pc.get("uid")))
        except (ValueError, AttributeError, TypeError):
            hit = set()
        if len(_AVOID_CACHE) > 1024:
            _AVOID_CACHE.clear()
        _AVOID_CACHE[raw] = hit
    return hit


def node_prefer_avoid_pods(pod, pi, ni, ctx):
    """`node_prefer_avoid_pods.go` NodePreferAvoidPodsPriorityMap: 0 on a node whose
    preferAvoidPods annotation names the pod's controlling ReplicationController / ReplicaSet
    (by kind and uid), else 10; other controller kinds are ignored."""
    if ctx.owner_kind not in ("ReplicationController", "ReplicaSet") or not ctx.owner_uid:
        return MAX
    anns = ((ni.node or {}).get("metadata") or {}).get("annotations") or {}
    raw = anns.get("scheduler.alpha.kubernetes.io/preferAvoidPods")
    if not raw:
        return MAX
    return 0.0 if (ctx.owner_kind, ctx.owner_uid) in _avoided_controllers(raw) else MAX


def xgmi_topology(pod, pi, ni, ctx):
    return ctx.topo_scores.get(ni.name, MAX)


def gpu_bin_packing(pod, pi, ni, ctx):
    total = ni.gpu_total
    if not total or not pi.er:
        return 0.0
    need = sum(r[2] for r in pi.er if r[1] == core.AMD_GPU)
    free_after = ni.er.free_count(core.AMD_GPU) - need
    if free_after < 0:
        return 0.0
    return MAX * (1.0 - free_after / total)


MIN_IMG, MAX_IMG = 23 * 1024 * 1024, 1000 * 1024 * 1024


def image_locality(pod, pi, ni, ctx):
    """`image_locality.go`: total size of the pod's images already on the node, mapped to
    1..10 between 23 MB and 1000 MB (0 below)."""
    if not ni.images:
        return 0.0
    total = 0
    for c in (pod.get("spec") or {}).get("containers") or ():
        total += ni.images.get(c.get("image", ""), 0)
    if total < MIN_IMG:
        return 0.0
    if total >= MAX_IMG:
        return MAX
    return float(int(MAX * (total - MIN_IMG) / (MAX_IMG - MIN_IMG)) + 1)


def resource_limits(pod, pi, ni, ctx):
    """`resource_limits.go`: 1 when the node's allocatable can satisfy the pod's cpu or memory limit."""
    cpu, mem = pi.limits
    if (cpu and ni.alloc_cpu >= cpu) or (mem and ni.alloc_mem >= mem):
        return 1.0
    return 0.0


def inter_pod_affinity(pod, pi, ni, ctx):
    """`interpod_affinity.go` CalculateInterPodAffinityPriority for the incoming pod's preferred
    terms: +weight per matching pod in the node's topology domain (affinity), −weight (anti);
    min-max normalized to 0..10."""
    s = 0.0
    for weight, key, counts in ctx.pod_affinity_counts():
        if not key:                       # empty topologyKey: counts per node (--failure-domains)
            s += weight * counts.get(ni.name, 0)
            continue
        v = ni.labels.get(key)
        if v is not None:
            s += weight * counts.get(v, 0)
    return s


# name -> (fn, reverse normalization?, normalize? True | False | "minmax")
PRIORITIES = {
    "LeastRequestedPriority": (least_requested, False, False),
    "MostRequestedPriority": (most_requested, False, False),
    "BalancedResourceAllocation": (balanced_resource_allocation, False, False),
    "SelectorSpreadPriority": (selector_spread, True, "spread"),
    "NodeAffinityPriority": (node_affinity, False, True),
    "TaintTolerationPriority": (taint_toleration, True, True),
    "NodePreferAvoidPodsPriority": (node_prefer_avoid_pods, False, False),
    "XGMITopologyPriority": (xgmi_topology, False, False),
    "GPUBinPackingPriority": (gpu_bin_packing, False, False),
    "ImageLocalityPriority": (image_locality, False, False),
    "ResourceLimitsPriority": (resource_limits, False, False),
    "InterPodAffinityPriority": (inter_pod_affinity, False, "minmax"),
    "ServiceSpreadingPriority": (service_spreading, True, "spread"),
    "EqualPriority": (equal, False, False),
}

DEFAULT_PRIORITIES = {
    "LeastRequestedPriority": 1, "BalancedResourceAllocation": 1, "SelectorSpreadPriority": 1,
    "NodeAffinityPriority": 1, "TaintTolerationPriority": 1, "NodePreferAvoidPodsPriority": 10000,
    "InterPodAffinityPriority": 1,
    "XGMITopologyPriority": 2, "GPUBinPackingPriority": 1,
}


def compile_node_affinity_prefs(pod):
    aff = ((pod.get("spec") or {}).get("affinity") or {}).get("nodeAffinity") or {}
    out = []
    for t in aff.get("preferredDuringSchedulingIgnoredDuringExecution") or ():
        try:
            sel = node_selector_requirements_as_selector((t.get("preference") or {}).get("matchExpressions") or [])
        except SelectorError:
            continue
        out.append((float(t.get("weight", 0)), sel))
    return out


def normalize_minmax(scores):
    """`CalculateInterPodAffinityPriority` reduce: int(10 * (v - min) / (max - min)) where min and
    max start at 0 (interpod_affinity.go: `var maxCount, minCount float64`), so with only
    positive counts a node scores in proportion to its count; 0 when all equal."""
    lo, hi = min(0, min(scores, default=0)), max(0, max(scores, default=0))
    if hi == lo:
        return [0 for _ in scores]
    return [int(MAX * (v - lo) / (hi - lo)) for v in scores]


def normalize(scores, reverse):
    """`NormalizeReduce(MaxPriority, reverse)`: integer 10 * score / max (reversed: 10 minus
    that); with every score 0, reverse gives everyone 10."""
    mx = max(scores) if scores else 0
    if mx <= 0:
        return [int(MAX) if reverse else 0 for _ in scores]
    out = []
    for s in scores:
        v = int(MAX) * int(s) // int(mx) if float(s).is_integer() and float(mx).is_integer() else int(MAX * s / mx)
        out.append(int(MAX) - v if reverse else v)
    return out


ZONE_WEIGHTING = 2.0 / 3.0      # selector_spreading.go zoneWeighting


def zone_key(ni):
    """`utilnode.GetZoneKey`: region + ":\x00:" + zone from the failure-domain labels; "" when
    neither is set."""
    region = ni.labels.get("failure-domain.beta.kubernetes.io/region", "")
    zone = ni.labels.get("failure-domain.beta.kubernetes.io/zone", "")
    if not region and not zone:
        return ""
    return region + ":\x00:" + zone


def normalize_spread(counts, nodes):
    """`CalculateSpreadPriorityReduce`: 10 * (maxByNode - count) / maxByNode, blended 1/3 : 2/3
    with the same score over zones when the nodes carry zone labels; int() at the end."""
    max_node = max(counts) if counts else 0
    by_zone: dict = {}
    zones = [zone_key(ni) for ni in nodes]
    for z, c in zip(zones, counts):
        if z:
            by_zone[z] = by_zone.get(z, 0) + c
    max_zone = max(by_zone.values()) if by_zone else 0
    out = []
    for z, c in zip(zones, counts):
        f = MAX
        if max_node > 0:
            f = MAX * ((max_node - c) / max_node)
        if by_zone and z:
            zs = MAX
            if max_zone > 0:
                zs = MAX * ((max_zone - by_zone[z]) / max_zone)
            f = f * (1.0 - ZONE_WEIGHTING) + ZONE_WEIGHTING * zs
        out.append(int(f))
    return out
