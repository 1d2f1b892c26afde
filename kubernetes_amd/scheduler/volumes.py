"""Volume-aware scheduling: predicates over pod volumes and the volume binder.

Parity:
  * `NoDiskConflict` (`plugin/pkg/scheduler/algorithm/predicates/predicates.go:243-300`
    `isVolumeConflict`: GCE PD unless both read-only, EBS always, RBD shared monitor+pool+image
    unless both read-only, iSCSI same IQN unless both read-only);
  * `MaxEBSVolumeCount` / `MaxGCEPDVolumeCount` / `MaxAzureDiskVolumeCount` (`:302-480`
    `MaxPDVolumeCountChecker`: distinct volume ids on the node, direct and through PVC→PV;
    defaults 39 / 16 / 16, `KUBE_MAX_PD_VOLS` overrides);
  * `NoVolumeZoneConflict` (`:482-580`: PV zone/region labels must equal the node's; zone values
    may name several zones joined by `__`);
  * `CheckVolumeBinding` (`:1480+` with `plugin/pkg/scheduler/volumebinder/volume_binder.go`
    and `pkg/controller/volume/persistentvolume/scheduler_binder.go`): bound claims need the PV's
    node affinity to match; unbound claims of a `WaitForFirstConsumer` class need an available
    matching PV whose node affinity matches, or a provisioner; the binder assumes the chosen PVs
    and writes their `claimRef` (or the claim's `selected-node` annotation for provisioning)
    before the pod binding is posted.

Only pods that carry such volumes pay anything: `VolumeInfo` is empty for the others and each
predicate returns at its first line.
"""
from __future__ import annotations

import json
import os

from ..api.labels import SelectorError, node_selector_requirements_as_selector
from ..controllers.volume import NODE_AFFINITY_ANN, best_match, claim_class

ZONE_LABEL = "failure-domain.beta.kubernetes.io/zone"
REGION_LABEL = "failure-domain.beta.kubernetes.io/region"
SELECTED_NODE_ANN = "volume.kubernetes.io/selected-node"
WAIT = "WaitForFirstConsumer"

MAX_VOLUMES = {"ebs": 39, "gce-pd": 16, "azure-disk": 16}


class VolumeLister:
    """Claim / volume / class views fed by the scheduler's informers."""

    def __init__(self):
        self.pvcs: dict[str, dict] = {}
        self.pvs: dict[str, dict] = {}
        self.classes: dict[str, dict] = {}
        self.assumed_pvs: dict[str, dict] = {}     # PV name -> claimRef assumed by this scheduler

    def pvc(self, ns, name):
        return self.pvcs.get(f"{ns}/{name}")

    def pv_of(self, pvc):
        vn = ((pvc or {}).get("spec") or {}).get("volumeName")
        return self.pvs.get(vn) if vn else None

    def available_pvs(self):
        for name, pv in self.pvs.items():
            if name in self.assumed_pvs:
                continue
            yield pv


class VolumeInfo:
    __slots__ = ("disks", "claims")

    def __init__(self, pod):
        disks, claims = [], []
        for v in (pod.get("spec") or {}).get("volumes") or ():
            if "persistentVolumeClaim" in v:
                claims.append(v["persistentVolumeClaim"].get("claimName"))
                continue
            d = _disk_of(v)
            if d:
                disks.append(d)
        self.disks = disks
        self.claims = claims

    def __bool__(self):
        return bool(self.disks or self.claims)


def _disk_of(src):
    """(kind, identity, read_only, extra) for the disk-like sources the predicates know."""
    if src.get("gcePersistentDisk"):
        g = src["gcePersistentDisk"]
        return ("gce-pd", g.get("pdName"), bool(g.get("readOnly")), None)
    if src.get("awsElasticBlockStore"):
        return ("ebs", src["awsElasticBlockStore"].get("volumeID"), False, None)
    if src.get("azureDisk"):
        return ("azure-disk", src["azureDisk"].get("diskName"), bool(src["azureDisk"].get("readOnly")), None)
    if src.get("rbd"):
        r = src["rbd"]
        return ("rbd", (r.get("pool", "rbd"), r.get("image")), bool(r.get("readOnly")), frozenset(r.get("monitors") or ()))
    if src.get("iscsi"):
        i = src["iscsi"]
        return ("iscsi", i.get("iqn"), bool(i.get("readOnly")), None)
    return None


def _vi(pod, pi):
    vi = getattr(pi, "volumes", None)
    if vi is None:
        vi = VolumeInfo(pod)
    return vi


def _conflict(a, b):
    ka, ida, roa, exa = a
    kb, idb, rob, exb = b
    if ka != kb or ida != idb:
        return False
    if ka == "ebs":
        return True
    if ka == "rbd" and not (exa & exb):
        return False
    return not (roa and rob)


def no_disk_conflict(pod, pi, ni, ctx):
    vi = _vi(pod, pi)
    if not vi.disks:
        return None
    for other, opi in ni.pods.values():
        for d in _vi(other, opi).disks:
            for mine in vi.disks:
                if _conflict(mine, d):
                    return "node(s) had no available disk"
    return None


def _limit(kind):
    env = os.environ.get("KUBE_MAX_PD_VOLS")
    if env and env.isdigit():
        return int(env)
    return MAX_VOLUMES[kind]


def _volume_ids(pod, pi, kind, lister, ns):
    out = set()
    vi = _vi(pod, pi)
    for d in vi.disks:
        if d[0] == kind:
            out.add(d[1])
    for c in vi.claims:
        pvc = lister.pvc(ns, c) if lister else None
        pv = lister.pv_of(pvc) if pvc else None
        if pv is None:
            # an unbound or missing claim may become a volume of this kind: count it once
            if _claim_counts(lister, pvc, kind):
                out.add(("claim", ns, c))
            continue
        d = _disk_of(pv.get("spec") or {})
        if d and d[0] == kind:
            out.add(d[1])
    return out


def _claim_counts(lister, pvc, kind):
    """An unbound claim counts against every disk kind (the reference gives it a random id),
    unless its class's provisioner is known to make another kind."""
    if lister is None or pvc is None:
        return True
    cls = lister.classes.get(claim_class(pvc))
    prov = (cls or {}).get("provisioner", "")
    want = {"ebs": "kubernetes.io/aws-ebs", "gce-pd": "kubernetes.io/gce-pd", "azure-disk": "kubernetes.io/azure-disk"}[kind]
    return not prov or prov == want


def max_volume_count(kind):
    def pred(pod, pi, ni, ctx):
        vi = _vi(pod, pi)
        if not vi:
            return None
        lister = getattr(ctx, "volumes", None)
        new = _volume_ids(pod, pi, kind, lister, pod["metadata"].get("namespace", "default"))
        if not new:
            return None
        existing = set()
        for other, opi in ni.pods.values():
            existing |= _volume_ids(other, opi, kind, lister, other["metadata"].get("namespace", "default"))
        if len(existing | new) > _limit(kind):
            return "node(s) exceed max volume count"
        return None
    pred.__name__ = f"max_{kind.replace('-', '_')}_volume_count"
    return pred


def _zones(v):
    return set(v.split("__")) if v else set()


def no_volume_zone_conflict(pod, pi, ni, ctx):
    vi = _vi(pod, pi)
    if not vi.claims:
        return None
    nz, nr = ni.labels.get(ZONE_LABEL), ni.labels.get(REGION_LABEL)
    if nz is None and nr is None:
        return None
    lister = getattr(ctx, "volumes", None)
    if lister is None:
        return None
    ns = pod["metadata"].get("namespace", "default")
    for c in vi.claims:
        pv = lister.pv_of(lister.pvc(ns, c))
        if pv is None:
            continue
        labels = pv["metadata"].get("labels") or {}
        if ZONE_LABEL in labels and nz is not None and nz not in _zones(labels[ZONE_LABEL]):
            return "node(s) had no available volume zone"
        if REGION_LABEL in labels and nr is not None and nr not in _zones(labels[REGION_LABEL]):
            return "node(s) had no available volume zone"
    return None


def pv_node_terms(pv):
    """The PV's required node selector terms (`spec.nodeAffinity` or the 1.9 alpha annotation)."""
    na = (pv.get("spec") or {}).get("nodeAffinity")
    if na is None:
        ann = (pv["metadata"].get("annotations") or {}).get(NODE_AFFINITY_ANN)
        if ann:
            try:
                na = json.loads(ann)
            except ValueError:
                return [{"matchExpressions": [{"key": "__invalid__", "operator": "Exists"}]}]
    if not na:
        return None
    req = na.get("required") or na.get("requiredDuringSchedulingIgnoredDuringExecution") or {}
    return req.get("nodeSelectorTerms") or None


def pv_fits_node(pv, labels):
    terms = pv_node_terms(pv)
    if not terms:
        return True
    for t in terms:
        try:
            if node_selector_requirements_as_selector(t.get("matchExpressions") or []).matches(labels):
                return True
        except SelectorError:
            continue
    return False


def _delayed(lister, pvc):
    cls = lister.classes.get(claim_class(pvc))
    return bool(cls) and cls.get("volumeBindingMode") == WAIT


def find_pv_for(lister, pvc, labels, taken=()):
    cands = [pv for pv in lister.available_pvs() if pv["metadata"]["name"] not in taken and pv_fits_node(pv, labels)]
    return best_match(cands, pvc)


def check_volume_binding(pod, pi, ni, ctx):
    vi = _vi(pod, pi)
    if not vi.claims:
        return None
    lister = getattr(ctx, "volumes", None)
    if lister is None:
        return None
    ns = pod["metadata"].get("namespace", "default")
    taken = set()
    for c in vi.claims:
        pvc = lister.pvc(ns, c)
        if pvc is None:
            return f'persistentvolumeclaim "{c}" not found'
        pv = lister.pv_of(pvc)
        if (pvc.get("spec") or {}).get("volumeName"):
            if pv is None:
                return "node(s) had volume node affinity conflict"
            if not pv_fits_node(pv, ni.labels):
                return "node(s) had volume node affinity conflict"
            continue
        if not _delayed(lister, pvc):
            return "pod has unbound PersistentVolumeClaims"
        sel = (pvc.get("metadata") or {}).get("annotations", {}).get(SELECTED_NODE_ANN)
        if sel:
            if sel != ni.name:
                return "node(s) didn't find available persistent volumes to bind"
            continue
        pv = find_pv_for(lister, pvc, ni.labels, taken)
        if pv is not None:
            taken.add(pv["metadata"]["name"])
            continue
        cls = lister.classes.get(claim_class(pvc)) or {}
        if cls.get("provisioner") and cls.get("provisioner") != "kubernetes.io/no-provisioner":
            continue
        return "node(s) didn't find available persistent volumes to bind"
    return None


def plan_bindings(lister, pod, node_labels, node_name):
    """Volume decisions for the chosen node: [(kind, pvc, pv_or_None)] where kind is 'bind'
    (write the PV's claimRef) or 'provision' (annotate the claim with the selected node)."""
    ns = pod["metadata"].get("namespace", "default")
    out, taken = [], set()
    for c in VolumeInfo(pod).claims:
        pvc = lister.pvc(ns, c)
        if pvc is None or (pvc.get("spec") or {}).get("volumeName") or not _delayed(lister, pvc):
            continue
        if (pvc["metadata"].get("annotations") or {}).get(SELECTED_NODE_ANN):
            continue
        pv = find_pv_for(lister, pvc, node_labels, taken)
        if pv is not None:
            taken.add(pv["metadata"]["name"])
            out.append(("bind", pvc, pv))
        else:
            out.append(("provision", pvc, None))
    return out
