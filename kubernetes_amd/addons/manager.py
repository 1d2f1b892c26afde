"""Add-on manager (`cluster/addons/addon-manager/kube-addons.sh`).

Every `period` seconds the manifests in the add-on directory (YAML / JSON, multi-document) are
applied according to their `addonmanager.kubernetes.io/mode` label:
  * `Reconcile`   — created when missing and kept equal to the manifest (the live object's
    spec/data/rules are overwritten); objects carrying the label but no longer present in the
    directory are pruned;
  * `EnsureExists` — created when missing, never modified afterwards;
  * no label — ignored (the reference skips unlabelled add-ons since 1.9).
The default add-ons for this framework are the cluster DNS and the amd.com/gpu device-plugin
DaemonSet (`cluster/addons/device-plugins/nvidia-gpu` in the reference).
"""
from __future__ import annotations

import asyncio
import json
import logging
import os

import yaml

from ..api import meta as m
from ..client.rest import APIStatusError, is_not_found

log = logging.getLogger("addon-manager")
MODE = "addonmanager.kubernetes.io/mode"
RECONCILE, ENSURE = "Reconcile", "EnsureExists"
# fields the manager owns on Reconcile add-ons (everything but metadata/status)
_OWNED = ("spec", "data", "binaryData", "rules", "subjects", "roleRef", "type", "stringData", "webhooks", "secrets")


def load_dir(path):
    out = []
    for root, _, files in os.walk(path):
        for fn in sorted(files):
            if not fn.endswith((".yaml", ".yml", ".json")):
                continue
            with open(os.path.join(root, fn)) as f:
                text = f.read()
            docs = [json.loads(text)] if fn.endswith(".json") else list(yaml.safe_load_all(text))
            for d in docs:
                if not isinstance(d, dict):
                    continue
                if d.get("kind", "").endswith("List") and "items" in d:
                    out.extend(d["items"])
                else:
                    out.append(d)
    return out


def _ri(obj):
    return next((r for r in m.BY_PLURAL.values() if r.kind == obj.get("kind")), None)


class AddonManager:
    def __init__(self, client, addon_dir, period=60.0):
        self.client = client
        self.dir = addon_dir
        self.period = period
        self.applied = 0
        self.pruned = 0

    async def reconcile_once(self):
        want = {}
        for o in load_dir(self.dir):
            mode = ((o.get("metadata") or {}).get("labels") or {}).get(MODE)
            ri = _ri(o)
            if mode not in (RECONCILE, ENSURE) or ri is None:
                continue
            ns = (o["metadata"].get("namespace") or "kube-system") if ri.namespaced else None
            if ri.namespaced:
                o["metadata"]["namespace"] = ns
            want[(ri.plural, ns, o["metadata"]["name"])] = (ri, o, mode)
            try:
                cur = await self.client.get(ri.plural, o["metadata"]["name"], ns)
            except APIStatusError as e:
                if not is_not_found(e):
                    raise
                await self.client.create(ri.plural, o, ns)
                self.applied += 1
                continue
            if mode == ENSURE:
                continue
            changed = False
            for k in _OWNED:
                if k in o and cur.get(k) != o[k]:
                    cur[k] = o[k]
                    changed = True
            labels = dict(cur["metadata"].get("labels") or {})
            if any(labels.get(k) != v for k, v in (o["metadata"].get("labels") or {}).items()):
                labels.update(o["metadata"].get("labels") or {})
                cur["metadata"]["labels"] = labels
                changed = True
            if changed:
                await self.client.update(ri.plural, cur, ns)
                self.applied += 1
        # prune Reconcile add-ons whose manifest disappeared
        kinds = {ri.plural for ri, _, _ in want.values()}
        for plural in kinds | {"deployments", "daemonsets", "services", "configmaps", "serviceaccounts"}:
            ri = m.BY_PLURAL.get(plural)
            if ri is None:
                continue
            try:
                lst = await self.client.list(ri.plural, None, f"{MODE}={RECONCILE}")
            except APIStatusError:
                continue
            for o in lst.get("items") or ():
                ns = o["metadata"].get("namespace") if ri.namespaced else None
                if (ri.plural, ns, o["metadata"]["name"]) not in want:
                    try:
                        await self.client.delete(ri.plural, o["metadata"]["name"], ns)
                        self.pruned += 1
                    except APIStatusError as e:
                        if not is_not_found(e):
                            raise

    async def run(self):
        while True:
            try:
                await self.reconcile_once()
            except Exception as e:  # noqa: BLE001 - keep reconciling
                log.warning("add-on reconcile failed: %s", e)
            await asyncio.sleep(self.period)


def default_addons(cluster_dns_ip="10.96.0.10", domain="cluster.local", master="http://127.0.0.1:8080",
                   elasticsearch="http://elasticsearch-logging.kube-system:9200"):
    """Manifests for the built-in add-ons (written by `kubeadm` / local-up). `master` is the API
    server URL the hostNetwork add-ons (node-problem-detector) talk to."""
    lab = {MODE: RECONCILE}
    import sys

    from ..deviceplugin.api import DEVICE_MANAGER_PATH
    return [
        {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": "kube-dns", "namespace": "kube-system",
                                                                    "labels": dict(lab)}},
        {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "kube-dns", "namespace": "kube-system",
                                                             "labels": dict(lab, **{"k8s-app": "kube-dns"})},
         "spec": {"selector": {"k8s-app": "kube-dns"}, "clusterIP": cluster_dns_ip,
                  "ports": [{"name": "dns", "port": 53, "protocol": "UDP"}, {"name": "dns-tcp", "port": 53, "protocol": "TCP"}]}},
        {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "kube-dns", "namespace": "kube-system",
                                                                     "labels": dict(lab, **{"k8s-app": "kube-dns"})},
         "spec": {"replicas": 1, "selector": {"matchLabels": {"k8s-app": "kube-dns"}},
                  "template": {"metadata": {"labels": {"k8s-app": "kube-dns"}},
                               "spec": {"serviceAccountName": "kube-dns", "dnsPolicy": "Default",
                                        "containers": [{"name": "kubedns", "image": "kubernetes-amd/hyperkube",
                                                        "command": [sys.executable, "-m", "kubernetes_amd.cmd.dns",
                                                                    "--domain", domain, "--port", "53"]}]}}}},
        {"apiVersion": "apps/v1", "kind": "DaemonSet",
         "metadata": {"name": "amd-gpu-device-plugin", "namespace": "kube-system",
                      "labels": dict(lab, **{"k8s-app": "amd-gpu-device-plugin"})},
         "spec": {"selector": {"matchLabels": {"k8s-app": "amd-gpu-device-plugin"}},
                  "template": {"metadata": {"labels": {"k8s-app": "amd-gpu-device-plugin"},
                                            "annotations": {"scheduler.alpha.kubernetes.io/critical-pod": ""}},
                               "spec": {"hostNetwork": True, "priorityClassName": "system-node-critical",
                                        "tolerations": [{"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"}],
                                        "nodeSelector": {"feature.node.kubernetes.io/amd-gpu": "true"},
                                        "containers": [{"name": "amd-gpu-device-plugin", "image": "kubernetes-amd/hyperkube",
                                                        "command": [sys.executable, "-m", "kubernetes_amd.cmd.device_plugin"],
                                                        "volumeMounts": [{"name": "dp", "mountPath": DEVICE_MANAGER_PATH}]}],
                                        # the fork's kubelet watches <DeviceManagerPath>/plugins (quirk Q5:
                                        # the reference's GKE add-on mounts the upstream path and never registers)
                                        "volumes": [{"name": "dp", "hostPath": {"path": DEVICE_MANAGER_PATH}}]}}}},
        {"apiVersion": "apps/v1", "kind": "DaemonSet",
         "metadata": {"name": "node-problem-detector", "namespace": "kube-system",
                      "labels": dict(lab, **{"k8s-app": "node-problem-detector"})},
         "spec": {"selector": {"matchLabels": {"k8s-app": "node-problem-detector"}},
                  "template": {"metadata": {"labels": {"k8s-app": "node-problem-detector"}},
                               "spec": {"hostNetwork": True,
                                        "tolerations": [{"operator": "Exists", "effect": "NoSchedule"}],
                                        "containers": [{"name": "node-problem-detector", "image": "kubernetes-amd/hyperkube",
                                                        "command": [sys.executable, "-m", "kubernetes_amd.cmd.npd",
                                                                    "--master", master, "--kernel-log", "/var/log/kern.log", "--amd-smi"],
                                                        "env": [{"name": "NODE_NAME",
                                                                 "valueFrom": {"fieldRef": {"fieldPath": "spec.nodeName"}}}],
                                                        "volumeMounts": [{"name": "log", "mountPath": "/var/log", "readOnly": True}]}],
                                        "volumes": [{"name": "log", "hostPath": {"path": "/var/log"}}]}}}},
        # cluster/addons/fluentd-elasticsearch: node logging agent shipping /var/log/containers
        {"apiVersion": "apps/v1", "kind": "DaemonSet",
         "metadata": {"name": "log-shipper", "namespace": "kube-system",
                      "labels": dict(lab, **{"k8s-app": "log-shipper"})},
         "spec": {"selector": {"matchLabels": {"k8s-app": "log-shipper"}},
                  "template": {"metadata": {"labels": {"k8s-app": "log-shipper"}},
                               "spec": {"hostNetwork": True, "priorityClassName": "system-node-critical",
                                        "tolerations": [{"operator": "Exists", "effect": "NoSchedule"}],
                                        "containers": [{"name": "log-shipper", "image": "kubernetes-amd/hyperkube",
                                                        "command": [sys.executable, "-m", "kubernetes_amd.cmd.log_shipper",
                                                                    "--master", master, "--log-dir", "/var/log/containers",
                                                                    "--pos-file", "/var/log/es-containers.log.pos",
                                                                    "--elasticsearch", elasticsearch],
                                                        "env": [{"name": "NODE_NAME",
                                                                 "valueFrom": {"fieldRef": {"fieldPath": "spec.nodeName"}}}],
                                                        "volumeMounts": [{"name": "log", "mountPath": "/var/log"}]}],
                                        "volumes": [{"name": "log", "hostPath": {"path": "/var/log"}}]}}}},
        # cluster/addons/dashboard: read-only web UI (GPU allocation per node/device, pods, warnings)
        {"apiVersion": "apps/v1", "kind": "Deployment",
         "metadata": {"name": "kubernetes-dashboard", "namespace": "kube-system",
                      "labels": dict(lab, **{"k8s-app": "kubernetes-dashboard"})},
         "spec": {"replicas": 1, "selector": {"matchLabels": {"k8s-app": "kubernetes-dashboard"}},
                  "template": {"metadata": {"labels": {"k8s-app": "kubernetes-dashboard"}},
                               "spec": {"hostNetwork": True,
                                        "containers": [{"name": "dashboard", "image": "kubernetes-amd/hyperkube",
                                                        "command": [sys.executable, "-m", "kubernetes_amd.cmd.dashboard",
                                                                    "--master", master, "--port", "9090"]}]}}}},
        {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "kubernetes-dashboard", "namespace": "kube-system",
                                                             "labels": dict(lab, **{"k8s-app": "kubernetes-dashboard"})},
         "spec": {"selector": {"k8s-app": "kubernetes-dashboard"}, "ports": [{"port": 80, "targetPort": 9090}]}},
        # cluster/addons/storage-class: the default class (node-local host-path provisioner)
        {"apiVersion": "storage.k8s.io/v1", "kind": "StorageClass",
         "metadata": {"name": "standard", "labels": {MODE: ENSURE},
                      "annotations": {"storageclass.beta.kubernetes.io/is-default-class": "true"}},
         "provisioner": "kubernetes.io/host-path", "reclaimPolicy": "Delete"},
    ]
