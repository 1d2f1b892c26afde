"""Feature gates. Parity: `staging/src/k8s.io/apiserver/pkg/util/feature/feature_gate.go:77-297`
(`--feature-gates=K=V,...`, Alpha/Beta/GA maturity, defaults) and the kube registry
`pkg/features/kube_features.go` — incl. the fork's `DevicePlugins` Beta/true (:76,252).
"""
from __future__ import annotations

from dataclasses import dataclass

ALPHA, BETA, GA = "ALPHA", "BETA", "GA"


@dataclass(frozen=True)
class FeatureSpec:
    default: bool
    maturity: str


DEFAULTS = {
    "DevicePlugins": FeatureSpec(True, BETA),              # fork: Beta, on
    "ResourceV2": FeatureSpec(True, BETA),                 # pod-level extended resources (fork F1/F2)
    "XGMITopologyAwareAllocation": FeatureSpec(True, BETA),
    "EventDrivenKubelet": FeatureSpec(True, BETA),         # watch/exit-event driven pod sync
    # pod priority and scheduler preemption: alpha and off in the reference; on by default here
    # (a GPU cluster's high-priority training jobs preempt batch work), PodPriority=false turns
    # scheduler preemption and priority-aware eviction ranking off
    "PodPriority": FeatureSpec(True, ALPHA),
    "TaintBasedEvictions": FeatureSpec(False, ALPHA),     # node controller taints instead of deleting
    "TaintNodesByCondition": FeatureSpec(False, ALPHA),   # NoSchedule taints mirror node conditions
    "ExpandPersistentVolumes": FeatureSpec(False, ALPHA),
    "CPUManager": FeatureSpec(True, BETA),
    "HugePages": FeatureSpec(True, BETA),
    "Accelerators": FeatureSpec(False, ALPHA),             # legacy in-kubelet NVIDIA path: not provided
    # critical pods (kube-system + critical-pod annotation) are admitted under node pressure, are
    # never evicted when static, and may preempt on admission. On by default here (the
    # reference's alpha default is off): the AMD device-plugin DaemonSet is a critical pod, and a
    # node must not evict the agent that advertises its GPUs.
    "ExperimentalCriticalPodAnnotation": FeatureSpec(True, ALPHA),
    "LocalStorageCapacityIsolation": FeatureSpec(False, ALPHA),   # emptyDir sizeLimit / ephemeral-storage limits
    "CustomPodDNS": FeatureSpec(False, ALPHA),            # dnsPolicy None and spec.dnsConfig
}


class FeatureGate:
    def __init__(self, known=None):
        self.known = dict(known or DEFAULTS)
        self.enabled = {k: v.default for k, v in self.known.items()}

    def set(self, spec: str):
        for kv in (spec or "").split(","):
            kv = kv.strip()
            if not kv:
                continue
            k, _, v = kv.partition("=")
            k = k.strip()
            if k not in self.known:
                raise ValueError(f"unrecognized feature gate: {k}")
            v = v.strip().lower()
            if v not in ("true", "false"):
                raise ValueError(f"invalid value of {k}: {v}, err: strconv.ParseBool")
            self.enabled[k] = v == "true"
        return self

    def __call__(self, name) -> bool:
        if name not in self.enabled:
            raise KeyError(f"feature {name} is not registered")
        return self.enabled[name]

    def known_features(self):
        return [f"{k}=true|false ({v.maturity} - default={str(v.default).lower()})" for k, v in sorted(self.known.items())]


DefaultFeatureGate = FeatureGate()
