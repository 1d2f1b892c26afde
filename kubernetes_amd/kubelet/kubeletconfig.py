"""Kubelet configuration files and Dynamic Kubelet Config.

Parity:
  * `pkg/kubelet/apis/kubeletconfig/v1alpha1/types.go` — the `KubeletConfiguration` object
    (`kubeletconfig/v1alpha1`); the subset the MI355X kubelet uses is mapped to constructor
    arguments by `to_kwargs`, with the reference's defaults (`defaults.go`) and validation
    (`validation/validation.go`: percentages in range, low ≤ high, positive periods).
  * `pkg/kubelet/kubeletconfig/controller.go` (Dynamic Kubelet Config, alpha in 1.9): the node's
    `spec.configSource.configMapRef` names a ConfigMap whose `kubelet` key holds a
    KubeletConfiguration; the kubelet downloads it, checkpoints it under
    `--dynamic-config-dir/checkpoints/<uid>/kubelet`, records the assignment in
    `store/current` and validates it. A valid config is applied (hot-reloadable fields in
    place, like the reference's restart would); an invalid one is rejected and the
    last-known-good (`store/last-known-good`) stays in force. The outcome is reported as the
    `KubeletConfigOk` node condition.
"""
from __future__ import annotations

import json
import logging
import os

import yaml

log = logging.getLogger("kubelet.config")

API_VERSION = "kubeletconfig/v1alpha1"

DEFAULTS = {
    "maxPods": 110,
    "nodeStatusUpdateFrequency": "10s",
    "imageGCHighThresholdPercent": 85,
    "imageGCLowThresholdPercent": 80,
    "evictionHard": {"memory.available": "100Mi"},
    "cpuManagerPolicy": "none",
    "clusterDomain": "cluster.local",
    "clusterDNS": [],
    "podManifestPath": "",
    "minimumContainerTTLDuration": "0s",
    "maxPerPodContainerCount": 1,
    "maxContainerCount": -1,
    "eventRecordQPS": 5,
    "eventBurst": 10,
}


class ConfigError(ValueError):
    pass


def parse_duration(v):
    if isinstance(v, (int, float)):
        return float(v)
    total, num = 0.0, ""
    units = {"h": 3600.0, "m": 60.0, "s": 1.0}
    s = str(v)
    i = 0
    while i < len(s):
        ch = s[i]
        if ch.isdigit() or ch == ".":
            num += ch
        elif s[i:i + 2] == "ms":
            total += float(num or 0) / 1000
            num = ""
            i += 1
        elif ch in units:
            total += float(num or 0) * units[ch]
            num = ""
        else:
            raise ConfigError(f"invalid duration {v!r}")
        i += 1
    if num:
        total += float(num)
    return total


def load(text):
    doc = yaml.safe_load(text) if text.strip() else {}
    if not isinstance(doc, dict):
        raise ConfigError("KubeletConfiguration must be an object")
    if doc.get("kind", "KubeletConfiguration") != "KubeletConfiguration":
        raise ConfigError(f"unexpected kind {doc.get('kind')!r}")
    cfg = dict(DEFAULTS)
    cfg.update({k: v for k, v in doc.items() if k not in ("kind", "apiVersion")})
    validate(cfg)
    return cfg


def validate(cfg):
    errs = []
    for k in ("imageGCHighThresholdPercent", "imageGCLowThresholdPercent"):
        if not 0 <= int(cfg[k]) <= 100:
            errs.append(f"{k} ({cfg[k]}) must be between 0 and 100")
    if int(cfg["imageGCLowThresholdPercent"]) > int(cfg["imageGCHighThresholdPercent"]):
        errs.append("imageGCLowThresholdPercent must not exceed imageGCHighThresholdPercent")
    if int(cfg["maxPods"]) < 0:
        errs.append("maxPods must not be negative")
    try:
        if parse_duration(cfg["nodeStatusUpdateFrequency"]) <= 0:
            errs.append("nodeStatusUpdateFrequency must be greater than zero")
    except ConfigError as e:
        errs.append(str(e))
    if cfg["cpuManagerPolicy"] not in ("none", "static"):
        errs.append(f"cpuManagerPolicy {cfg['cpuManagerPolicy']!r} is not one of none, static")
    if errs:
        raise ConfigError("invalid configuration: " + "; ".join(errs))


def eviction_string(ev):
    return ",".join(f"{k}<{v}" for k, v in (ev or {}).items())


def to_kwargs(cfg):
    """Kubelet constructor arguments for a KubeletConfiguration."""
    from .network import DNSConfigurer
    kw = {"pods": int(cfg["maxPods"]), "node_status_update_frequency": parse_duration(cfg["nodeStatusUpdateFrequency"]),
          "cpu_manager_policy": cfg["cpuManagerPolicy"], "eviction_hard": eviction_string(cfg["evictionHard"]) or None,
          "container_gc": {"min_age": parse_duration(cfg["minimumContainerTTLDuration"]),
                           "max_per_pod_container": int(cfg["maxPerPodContainerCount"]),
                           "max_containers": int(cfg["maxContainerCount"])},
          "event_qps": float(cfg["eventRecordQPS"]), "event_burst": int(cfg["eventBurst"])}
    if cfg.get("clusterDNS"):
        kw["dns"] = DNSConfigurer(cfg["clusterDNS"], cfg["clusterDomain"])
    if cfg.get("podManifestPath"):
        kw["pod_manifest_path"] = cfg["podManifestPath"]
    return kw


def _read_ref(config_dir, name):
    try:
        with open(os.path.join(config_dir, "store", name)) as f:
            return json.load(f).get("uid")
    except (OSError, ValueError):
        return None


def startup_checkpoint(config_dir):
    """Config to start with: the assigned checkpoint if valid, else last-known-good, else None
    (the restart path of `controller.go` `Bootstrap`)."""
    for uid in (_read_ref(config_dir, "current"), _read_ref(config_dir, "last-known-good")):
        if uid:
            try:
                with open(os.path.join(config_dir, "checkpoints", uid, "kubelet")) as f:
                    return load(f.read())
            except (OSError, ConfigError) as e:
                log.warning("checkpoint %s unusable: %s", uid, e)
    return None


class DynamicConfig:
    """Checkpoint store + controller for `spec.configSource`."""

    def __init__(self, kubelet, config_dir):
        self.kl = kubelet
        self.dir = config_dir
        os.makedirs(os.path.join(config_dir, "store"), exist_ok=True)
        self.current_uid = self._read("current")
        self.lkg_uid = self._read("last-known-good")
        self.condition = {"type": "KubeletConfigOk", "status": "True", "reason": "using local config",
                          "message": "using local config"}
        self._busy = False

    def _read(self, name):
        return _read_ref(self.dir, name)

    def _write(self, name, ref):
        p = os.path.join(self.dir, "store", name)
        with open(p + ".tmp", "w") as f:
            json.dump(ref, f)
        os.replace(p + ".tmp", p)

    def checkpoint_path(self, uid):
        return os.path.join(self.dir, "checkpoints", uid, "kubelet")

    def startup_config(self):
        return startup_checkpoint(self.dir)

    async def observe_node(self, node):
        src = ((node or {}).get("spec") or {}).get("configSource") or {}
        ref = src.get("configMapRef") or src.get("configMap")
        if not ref:
            if self.current_uid is not None:
                self.current_uid = None
                self._write("current", {})
                self.kl.apply_config(None)
                self.condition = {"type": "KubeletConfigOk", "status": "True", "reason": "using local config",
                                  "message": "using local config"}
                self.kl._status_dirty.set()
            return
        uid = ref.get("uid") or ""
        if uid == self.current_uid and self.condition.get("status") == "True" or self._busy:
            return
        self._busy = True
        try:
            await self._sync(ref)
        finally:
            self._busy = False
            self.kl._status_dirty.set()

    async def _sync(self, ref):
        ns, name = ref.get("namespace", "kube-system"), ref.get("name")
        try:
            cm = await self.kl.client.get("configmaps", name, ns)
        except Exception as e:  # noqa: BLE001 - API failures are reported in the condition
            self.condition = {"type": "KubeletConfigOk", "status": "False", "reason": "failed to download config",
                              "message": f"failed to download ConfigMap {ns}/{name}: {e}"}
            return
        uid = cm["metadata"].get("uid", "")
        if ref.get("uid") and ref["uid"] != uid:
            self.condition = {"type": "KubeletConfigOk", "status": "False", "reason": "invalid config source",
                              "message": f"configMapRef.uid {ref['uid']} does not match ConfigMap UID {uid}"}
            return
        text = (cm.get("data") or {}).get("kubelet", "")
        path = self.checkpoint_path(uid)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            f.write(text)
        self.current_uid = uid
        self._write("current", {"uid": uid, "namespace": ns, "name": name})
        try:
            cfg = load(text)
        except ConfigError as e:
            self.condition = {"type": "KubeletConfigOk", "status": "False", "reason": "failed to validate current config",
                              "message": f"{e}; using last-known-good ({self.lkg_uid or 'local'})"}
            return
        self.kl.apply_config(cfg)
        self.lkg_uid = uid
        self._write("last-known-good", {"uid": uid, "namespace": ns, "name": name})
        self.condition = {"type": "KubeletConfigOk", "status": "True", "reason": "passing all checks",
                          "message": f"using current (UID: {uid})"}
