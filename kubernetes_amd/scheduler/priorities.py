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


def least_requested(pod, pi, ni, ctx):
    def f(req, cap):
        if cap == 0 or req > cap:
            return 0.0
        return (cap - req) * MAX / cap
    return (f(ni.nz_cpu + pi.nz_cpu, ni.alloc_cpu) + f(ni.nz_mem + pi.nz_mem, ni.alloc_mem)) / 2


def most_requested(pod, pi, ni, ctx):
    def f(req, cap):
        if cap == 0 or req > cap:
            return 0.0
        return req * MAX / cap
    return (f(ni.nz_cpu + pi.nz_cpu, ni.alloc_cpu) + f(ni.nz_mem + pi.nz_mem, ni.alloc_mem)) / 2


def balanced_resource_allocation(pod, pi, ni, ctx):
    if not ni.alloc_cpu or not ni.alloc_mem:
        return 0.0
    c = (ni.nz_cpu + pi.nz_cpu) / ni.alloc_cpu
    m = (ni.nz_mem + pi.nz_mem) / ni.alloc_mem
    if c >= 1 or m >= 1:
        return 0.0
    return MAX - abs(c - m) * MAX


def selector_spread(pod, pi, ni, ctx):
    """Raw count of sibling pods (same controller) on the node; normalized reversed later."""
    owner = ctx.owner_uid
    if not owner:
        return 0.0
    n = 0
    for p, _ in ni.pods.values():
        for ref in p["metadata"].get("ownerReferences") or ():
            if ref.get("uid") == owner:
                n += 1
                break
    return float(n)


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


def node_prefer_avoid_pods(pod, pi, ni, ctx):
    ann = ((ni.node or {}).get("metadata") or {}).get("annotations") or {}
    if "scheduler.alpha.kubernetes.io/preferAvoidPods" not in ann or not ctx.owner_uid:
        return MAX
    return 0.0 if ctx.owner_uid in ann["scheduler.alpha.kubernetes.io/preferAvoidPods"] else MAX


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
        v = ni.labels.get(key)
        if v is not None:
            s += weight * counts.get(v, 0)
    return s


# name -> (fn, reverse normalization?, normalize? True | False | "minmax")
PRIORITIES = {
    "LeastRequestedPriority": (least_requested, False, False),
    "MostRequestedPriority": (most_requested, False, False),
    "BalancedResourceAllocation": (balanced_resource_allocation, False, False),
    "SelectorSpreadPriority": (selector_spread, True, True),
    "NodeAffinityPriority": (node_affinity, False, True),
    "TaintTolerationPriority": (taint_toleration, True, True),
    "NodePreferAvoidPodsPriority": (node_prefer_avoid_pods, False, False),
    "XGMITopologyPriority": (xgmi_topology, False, False),
    "GPUBinPackingPriority": (gpu_bin_packing, False, False),
    "ImageLocalityPriority": (image_locality, False, False),
    "ResourceLimitsPriority": (resource_limits, False, False),
    "InterPodAffinityPriority": (inter_pod_affinity, False, "minmax"),
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
    lo, hi = min(scores), max(scores)
    if hi == lo:
        return [0.0 for _ in scores]
    return [MAX * (v - lo) / (hi - lo) for v in scores]


def normalize(scores, reverse):
    mx = max(scores) if scores else 0
    if mx <= 0:
        return [MAX if reverse else 0.0 for _ in scores]
    if reverse:
        return [MAX * (mx - s) / mx for s in scores]
    return [MAX * s / mx for s in scores]
