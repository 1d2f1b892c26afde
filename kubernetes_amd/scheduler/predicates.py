"""Fit predicates. Parity: `plugin/pkg/scheduler/algorithm/predicates/predicates.go:202-1465`
(PodFitsResources :583-690, GeneralPredicates :965, host ports, node selector/affinity, taints,
memory/disk pressure, node condition, inter-pod affinity) and the default provider set
(`plugin/pkg/scheduler/algorithmprovider/defaults/defaults.go:67-255`); the volume predicates live
in `volumes.py`.

Every predicate has signature `(pod, PodInfo, NodeInfo, ctx) -> reason or None`.
"""
from __future__ import annotations

from ..api import core
from ..api.labels import SelectorError, label_selector_as_selector, node_selector_requirements_as_selector


def check_node_condition(pod, pi, ni, ctx):
    """`predicates.go:1414` CheckNodeConditionPredicate: Ready must be True, OutOfDisk and
    NetworkUnavailable False, and the node schedulable (a pod tolerating the
    `node.kubernetes.io/unschedulable` taint may still go there, as later releases allow)."""
    if ni.node is None:
        return "node(s) had unknown conditions"
    if not ni.ready:
        return "node(s) were not ready"
    if ni.cond_reason:
        return ni.cond_reason
    if ni.unschedulable and not ctx.tolerates_unschedulable:
        return "node(s) were unschedulable"
    return None


def pod_fits_resources(pod, pi, ni, ctx):
    """`PodFitsResources` (predicates.go:583-690): the pod count, then every resource the pod
    requests that does not fit — all of them, as the reference's InsufficientResourceError
    list (a tuple when more than one)."""
    if len(ni.pods) + 1 > ni.alloc_pods:
        return "Insufficient pods"
    short = []
    if pi.milli_cpu and ni.req_cpu + pi.milli_cpu > ni.alloc_cpu:
        short.append("Insufficient cpu")
    if pi.memory and ni.req_mem + pi.memory > ni.alloc_mem:
        short.append("Insufficient memory")
    if pi.ephemeral and ni.alloc_eph and ni.req_eph + pi.ephemeral > ni.alloc_eph:
        short.append("Insufficient ephemeral-storage")
    for k, v in pi.scalars.items():
        if ni.req_scalars.get(k, 0) + v > ni.alloc_scalars.get(k, 0):
            short.append(f"Insufficient {k}")
    if not short:
        return None
    return short[0] if len(short) == 1 else tuple(short)


def pod_fits_host(pod, pi, ni, ctx):
    want = (pod.get("spec") or {}).get("nodeName")
    if want and want != ni.name:
        return "node(s) didn't match the requested hostname"
    return None


def pod_fits_host_ports(pod, pi, ni, ctx):
    for ip, proto, port in pi.ports:
        for oip, oproto, oport in ni.ports:
            if oport == port and oproto == proto and (ip == oip or "0.0.0.0" in (ip, oip)):
                return "node(s) didn't have free ports for the requested pod ports"
    return None


def _node_affinity_terms(pod):
    """None without a required node selector; else its terms — an empty / missing term list
    matches no node (`predicates.go` podMatchesNodeLabels / nodeMatchesNodeSelectorTerms)."""
    aff = ((pod.get("spec") or {}).get("affinity") or {}).get("nodeAffinity") or {}
    req = aff.get("requiredDuringSchedulingIgnoredDuringExecution")
    if req is None:
        return None
    return req.get("nodeSelectorTerms") or []


def _term_matches(term, ni):
    exprs = term.get("matchExpressions") or []
    fields = term.get("matchFields") or []
    if not exprs and not fields:
        return False
    if exprs:
        try:
            if not node_selector_requirements_as_selector(exprs).matches(ni.labels):
                return False
        except SelectorError:
            return False
    for f in fields:
        if f.get("key") == "metadata.name":
            vals = f.get("values") or []
            op = f.get("operator")
            if (op == "In" and ni.name not in vals) or (op == "NotIn" and ni.name in vals):
                return False
    return True


def match_node_selector(pod, pi, ni, ctx):
    spec = pod.get("spec") or {}
    ns = spec.get("nodeSelector")
    if ns:
        labels = ni.labels
        for k, v in ns.items():
            if labels.get(k) != v:
                return "node(s) didn't match node selector"
    terms = _node_affinity_terms(pod)
    if terms is not None:
        if not any(_term_matches(t, ni) for t in terms):
            return "node(s) didn't match node selector"
    return None


def pod_tolerates_node_taints(pod, pi, ni, ctx):
    if not ni.taints:
        return None
    tols = (pod.get("spec") or {}).get("tolerations") or []
    for t in ni.taints:
        if t.get("effect") not in (core.TAINT_NO_SCHEDULE, core.TAINT_NO_EXECUTE):
            continue
        if not core.tolerates(tols, t):
            return "node(s) had taints that the pod didn't tolerate"
    return None


def check_node_memory_pressure(pod, pi, ni, ctx):
    if ni.mem_pressure and pi.milli_cpu == 0 and pi.memory == 0:
        return "node(s) had memory pressure"
    return None


def check_node_disk_pressure(pod, pi, ni, ctx):
    if ni.disk_pressure:
        return "node(s) had disk pressure"
    return None


def _pod_matches_term(pod_labels, pod_ns, term, owner_ns):
    nss = term.get("namespaces") or [owner_ns]
    if pod_ns not in nss:
        return False
    try:
        return label_selector_as_selector(term.get("labelSelector")).matches(pod_labels)
    except SelectorError:
        return False


def match_inter_pod_affinity(pod, pi, ni, ctx):
    """Required pod (anti-)affinity by topologyKey; also honours existing pods' anti-affinity."""
    spec = pod.get("spec") or {}
    aff = spec.get("affinity") or {}
    pa = (aff.get("podAffinity") or {}).get("requiredDuringSchedulingIgnoredDuringExecution") or []
    paa = (aff.get("podAntiAffinity") or {}).get("requiredDuringSchedulingIgnoredDuringExecution") or []
    ns = pod["metadata"].get("namespace", "default")
    labels = pod["metadata"].get("labels") or {}
    if not pa and not paa and not ctx.any_anti_affinity:
        return None
    by_topo = ctx.pods_by_topology
    for term in pa:
        key = term.get("topologyKey", "")
        val = ni.labels.get(key)
        if val is None:
            return "node(s) didn't match pod affinity rules"
        ok = any(_pod_matches_term(p["metadata"].get("labels") or {}, p["metadata"].get("namespace"), term, ns)
                 for p in by_topo(key, val))
        if not ok:
            # the first pod of a group may land anywhere if it matches its own term and no
            # other pod in the cluster does (predicates.go satisfiesPodsAffinityAntiAffinity)
            if ctx.any_pod_matches(term, ns) or not _pod_matches_term(labels, ns, term, ns):
                return "node(s) didn't match pod affinity rules"
    for term in paa:
        key = term.get("topologyKey", "")
        val = ni.labels.get(key)
        if val is None:
            continue
        for p in by_topo(key, val):
            if _pod_matches_term(p["metadata"].get("labels") or {}, p["metadata"].get("namespace"), term, ns):
                return "node(s) didn't match pod anti-affinity rules"
    # symmetric: existing pods' anti-affinity against this pod
    if ctx.any_anti_affinity:
        for p, term in ctx.anti_affinity_terms:
            key = term.get("topologyKey", "")
            val = ni.labels.get(key)
            if val is None:
                continue
            pnode = ctx.node_of(p)
            if pnode is None or pnode.labels.get(key) != val:
                continue
            if _pod_matches_term(labels, ns, term, p["metadata"].get("namespace", "default")):
                return "node(s) didn't satisfy existing pods anti-affinity rules"
    return None


def general_predicates(pod, pi, ni, ctx):
    """`predicates.go:965` GeneralPredicates: the non-critical PodFitsResources plus the
    essential PodFitsHost, PodFitsHostPorts and PodMatchNodeSelector (`:1000-1040`) in one."""
    for fn in (pod_fits_resources, pod_fits_host, pod_fits_host_ports, match_node_selector):
        r = fn(pod, pi, ni, ctx)
        if r:
            return r
    return None


# -- argument-based custom predicates (Policy `predicates[].argument`) ------------------------
# `plugin/pkg/scheduler/factory/plugins.go:198-240` RegisterCustomFitPredicate; each Policy
# entry registers a fresh closure under its own name.

def make_labels_presence(labels, presence):
    """`predicates.go` NewNodeLabelPredicate / CheckNodeLabelPresence: with presence=true every
    label must exist on the node, with presence=false none may (values are not looked at)."""
    labels = list(labels or ())

    def labels_presence(pod, pi, ni, ctx):
        for lbl in labels:
            if (lbl in ni.labels) != presence:
                return "node(s) didn't have the requested labels"
        return None
    return labels_presence


def make_service_affinity(labels):
    """`predicates.go:829-922` ServiceAffinity: the pod's service-mates share the values of
    `labels`. Values come first from the pod's own nodeSelector; the missing ones are taken from
    the node of the first already-placed pod of the pod's services (pods in the namespace whose
    labels carry the pod's labels, when any service selects the pod); the node must then match
    them all. The first pod of a service may land anywhere."""
    labels = list(labels or ())

    def service_affinity(pod, pi, ni, ctx):
        sel = (pod.get("spec") or {}).get("nodeSelector") or {}
        want = {lbl: sel[lbl] for lbl in labels if lbl in sel}
        if len(want) < len(labels):
            first = ctx.service_affinity_first_node()
            if first is not None:
                for lbl in labels:
                    if lbl not in want and lbl in first.labels:
                        want[lbl] = first.labels[lbl]
        for k, v in want.items():
            if ni.labels.get(k) != v:
                return "node(s) didn't match service affinity"
        return None
    service_affinity.global_view = True
    return service_affinity


from . import volumes as V  # noqa: E402

PREDICATES = {
    "CheckNodeCondition": check_node_condition,
    "HostName": pod_fits_host,
    "PodFitsResources": pod_fits_resources,
    "PodFitsHostPorts": pod_fits_host_ports,
    "PodFitsPorts": pod_fits_host_ports,          # the deprecated name (defaults.go:67), same predicate
    "GeneralPredicates": general_predicates,
    "MatchNodeSelector": match_node_selector,
    "PodToleratesNodeTaints": pod_tolerates_node_taints,
    "CheckNodeMemoryPressure": check_node_memory_pressure,
    "CheckNodeDiskPressure": check_node_disk_pressure,
    "MatchInterPodAffinity": match_inter_pod_affinity,
    "NoDiskConflict": V.no_disk_conflict,
    "MaxEBSVolumeCount": V.max_volume_count("ebs"),
    "MaxGCEPDVolumeCount": V.max_volume_count("gce-pd"),
    "MaxAzureDiskVolumeCount": V.max_volume_count("azure-disk"),
    "NoVolumeZoneConflict": V.no_volume_zone_conflict,
    "CheckVolumeBinding": V.check_volume_binding,
}

# predicates that only ever reject pods carrying volumes (skipped for volume-less pods)
VOLUME_PREDICATES = {"NoDiskConflict", "MaxEBSVolumeCount", "MaxGCEPDVolumeCount", "MaxAzureDiskVolumeCount",
                     "NoVolumeZoneConflict", "CheckVolumeBinding"}

# evaluation order: cheap & selective first (predicates ordering in later reference versions)
DEFAULT_PREDICATES = ["CheckNodeCondition", "HostName", "PodFitsResources", "MatchNodeSelector",
                      "PodFitsHostPorts", "PodToleratesNodeTaints", "CheckNodeMemoryPressure",
                      "CheckNodeDiskPressure", "NoVolumeZoneConflict", "MaxEBSVolumeCount", "MaxGCEPDVolumeCount",
                      "MaxAzureDiskVolumeCount", "NoDiskConflict", "CheckVolumeBinding", "MatchInterPodAffinity"]
