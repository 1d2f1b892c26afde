"""Scheduling-hint and storage admission plugins.

  * LimitPodHardAntiAffinityTopology — `plugin/pkg/admission/antiaffinity/admission.go:50-80`:
    required pod anti-affinity terms may only use `kubernetes.io/hostname` as topologyKey.
  * InitialResources — `plugin/pkg/admission/initialresources/admission.go:35-215`: containers
    that set neither a request nor a limit for cpu/memory get the `--ir-percentile` (90) of the
    historical usage of the same image, searched in the reference's widening order (image:tag
    this week → image:tag this month → image (any tag) this month, in the namespace when
    `namespaceOnly`, across namespaces otherwise) until `samplesThreshold` (30) samples are
    found; the pod is annotated `kubernetes.io/initial-resources`. The reference reads
    influxdb/gcm (heapster); here the data source is a JSON-lines usage history that the
    metrics-server appends to (`MetricsServer(history_path=...)`). `amd.com/gpu` is a device
    count and is never estimated.
  * PersistentVolumeLabel — `plugin/pkg/admission/persistentvolume/label/admission.go:77-130`
    labels new cloud disks with their zone/region. Without a cloud, the on-prem equivalent
    labels node-pinned volumes (local, hostPath with required node affinity) with the zone and
    region labels of the node they live on, so the scheduler's NoVolumeZoneConflict predicate
    works for them.
  * PVCProtection — `plugin/pkg/admission/persistentvolumeclaim/pvcprotection`: every new claim
    carries the `kubernetes.io/pvc-protection` finalizer, so a claim in use by a pod is not
    removed before the pod (the controller in `controllers/volume.py` lifts it).
"""
from __future__ import annotations

import json
import logging
import os
import time

from . import CREATE, UPDATE, AdmissionError, Plugin, register

log = logging.getLogger("admission")

HOSTNAME_LABEL = "kubernetes.io/hostname"
ZONE_LABEL = "failure-domain.beta.kubernetes.io/zone"
REGION_LABEL = "failure-domain.beta.kubernetes.io/region"
PVC_PROTECTION = "kubernetes.io/pvc-protection"
IR_ANNOTATION = "kubernetes.io/initial-resources"
SAMPLES_THRESHOLD = 30
WEEK = 7 * 24 * 3600.0
MONTH = 30 * 24 * 3600.0


def _pod_containers(spec):
    return [("container", c) for c in spec.get("containers") or []] + \
           [("init container", c) for c in spec.get("initContainers") or []]


@register
class LimitPodHardAntiAffinityTopology(Plugin):
    name = "LimitPodHardAntiAffinityTopology"
    operations = (CREATE, UPDATE)

    def validate(self, a):
        if a.resource != "pods" or a.subresource:
            return
        anti = (((a.obj.get("spec") or {}).get("affinity") or {}).get("podAntiAffinity") or {})
        for term in anti.get("requiredDuringSchedulingIgnoredDuringExecution") or []:
            key = term.get("topologyKey", "")
            if key != HOSTNAME_LABEL:
                raise AdmissionError(
                    f"affinity.PodAntiAffinity.RequiredDuringScheduling has TopologyKey {key} "
                    f"but only key {HOSTNAME_LABEL} is allowed", 403)


class UsageHistory:
    """Data source for InitialResources: per-container usage samples
    `{"ts", "namespace", "image", "cpu" (millicores), "memory" (bytes)}`, one JSON object per
    line. `usage_percentile` is the reference's `dataSource.GetUsagePercentile`
    (`initialresources/data_source.go`): returns (value, n_samples)."""

    def __init__(self, path=None, samples=None):
        self.path = path
        self._samples = list(samples or [])
        self._mtime = None

    def record(self, namespace, image, cpu_millis, mem_bytes, ts=None):
        s = {"ts": ts if ts is not None else time.time(), "namespace": namespace, "image": image,
             "cpu": int(cpu_millis), "memory": int(mem_bytes)}
        if self.path:
            with open(self.path, "a") as f:
                f.write(json.dumps(s) + "\n")
            self._mtime = None
        else:
            self._samples.append(s)

    def samples(self):
        if not self.path:
            return self._samples
        try:
            mt = os.stat(self.path).st_mtime_ns
        except FileNotFoundError:
            return []
        if mt != self._mtime:
            out = []
            with open(self.path) as f:
                for line in f:
                    line = line.strip()
                    if line:
                        try:
                            out.append(json.loads(line))
                        except ValueError:
                            continue
            self._samples, self._mtime = out, mt
        return self._samples

    def usage_percentile(self, kind, perc, image, namespace, exact_tag, start, end):
        vals = []
        for s in self.samples():
            if not (start <= s.get("ts", 0) <= end) or kind not in s:
                continue
            if namespace and s.get("namespace") != namespace:
                continue
            img = s.get("image", "")
            if exact_tag:
                if img != image:
                    continue
            elif img.split(":")[0] != image:
                continue
            vals.append(s[kind])
        if not vals:
            return 0, 0
        vals.sort()
        # nearest-rank percentile, as influxdb's PERCENTILE()
        idx = max(0, min(len(vals) - 1, -(-len(vals) * int(perc) // 100) - 1))
        return vals[idx], len(vals)


@register
class InitialResources(Plugin):
    name = "InitialResources"
    operations = (CREATE,)

    def __init__(self, server=None, config=None):
        super().__init__(server, config)
        cfg = self.config
        self.percentile = int(cfg.get("percentile", 90))
        self.ns_only = bool(cfg.get("namespaceOnly", False))
        src = cfg.get("source")
        self.source = src if isinstance(src, UsageHistory) else UsageHistory(cfg.get("historyFile"))

    def _estimate(self, kind, image, ns):
        end = time.time()
        base = image.split(":")[0]
        if self.ns_only:
            order = [(image, ns, True, WEEK), (image, ns, True, MONTH), (base, ns, False, MONTH)]
        else:
            order = [(image, ns, True, WEEK), (image, "", True, WEEK), (image, "", True, MONTH),
                     (base, "", False, MONTH)]
        usage = samples = 0
        for img, n, exact, span in order:
            usage, samples = self.source.usage_percentile(kind, self.percentile, img, n, exact, end - span, end)
            if samples >= SAMPLES_THRESHOLD:
                break
        if samples <= 0:
            return None
        return f"{usage}m" if kind == "cpu" else str(usage)

    def admit(self, a):
        if a.resource != "pods" or a.subresource:
            return
        spec = a.obj.get("spec") or {}
        ns = a.namespace or a.obj.get("metadata", {}).get("namespace", "")
        notes = []
        for what, c in _pod_containers(spec):
            res = c.setdefault("resources", {})
            req, lim = res.get("requests") or {}, res.get("limits") or {}
            done = []
            for kind in ("cpu", "memory"):
                if kind in req or kind in lim:
                    continue
                q = self._estimate(kind, c.get("image", ""), ns)
                if q is not None:
                    req[kind] = q
                    done.append(kind)
            if done:
                res["requests"] = req
                notes.append(", ".join(sorted(done)) + f" request for {what} {c.get('name')}")
        if notes:
            ann = a.obj.setdefault("metadata", {}).setdefault("annotations", {})
            ann[IR_ANNOTATION] = "Initial Resources plugin set: " + "; ".join(notes)


def _volume_node(pv):
    """Node name a node-pinned PV lives on: required node affinity on kubernetes.io/hostname."""
    from ...scheduler.volumes import pv_node_terms
    for term in pv_node_terms(pv) or []:
        for e in term.get("matchExpressions") or []:
            if e.get("key") == HOSTNAME_LABEL and e.get("operator") == "In" and len(e.get("values") or []) == 1:
                return e["values"][0]
    ann = (pv.get("metadata") or {}).get("annotations") or {}
    return ann.get("volume.alpha.kubernetes.io/node") or ann.get("kubernetes.io/hostname")


@register
class PersistentVolumeLabel(Plugin):
    name = "PersistentVolumeLabel"
    operations = (CREATE,)

    def admit(self, a):
        if a.resource != "persistentvolumes" or a.subresource or not self.server:
            return
        spec = a.obj.get("spec") or {}
        if not any(k in spec for k in ("local", "hostPath", "csi")):
            return
        node_name = _volume_node(a.obj)
        if not node_name:
            return
        node = self.server.get_object("nodes", None, node_name)
        if node is None:
            return
        nl = node.get("metadata", {}).get("labels") or {}
        labels = a.obj.setdefault("metadata", {}).setdefault("labels", {})
        for k in (ZONE_LABEL, REGION_LABEL):
            if k in nl and k not in labels:
                labels[k] = nl[k]


@register
class PVCProtection(Plugin):
    name = "PVCProtection"
    operations = (CREATE,)

    def admit(self, a):
        if a.resource != "persistentvolumeclaims" or a.subresource:
            return
        fins = a.obj.setdefault("metadata", {}).setdefault("finalizers", [])
        if PVC_PROTECTION not in fins:
            fins.append(PVC_PROTECTION)

