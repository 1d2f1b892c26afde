"""Scheduler policy and component configuration.

Parity:
  * `plugin/pkg/scheduler/api/types.go:38-129` — `Policy{predicates[{name}], priorities[{name,
    weight}], extenders[...], hardPodAffinitySymmetricWeight}` from a file
    (`--policy-config-file`) or a ConfigMap (`--policy-configmap`, key `policy.cfg`,
    `--policy-configmap-namespace` default kube-system);
  * `plugin/pkg/scheduler/algorithmprovider/defaults/defaults.go` — `--algorithm-provider`:
    `DefaultProvider`, and `ClusterAutoscalerProvider` (MostRequested instead of
    LeastRequested, to pack nodes);
  * `pkg/apis/componentconfig/types.go:45-86` — `KubeSchedulerConfiguration` (`--config`):
    schedulerName, algorithmSource{provider | policy{file{path} | configMap{namespace,name}}},
    leaderElection{leaderElect}, clientConnection{kubeconfig, qps, burst},
    healthzBindAddress / metricsBindAddress, disablePreemption, percentageOfNodesToScore.
"""
from __future__ import annotations

import json

import yaml

from . import predicates as P
from . import priorities as PR

PROVIDERS = {
    "DefaultProvider": lambda: (list(P.DEFAULT_PREDICATES), dict(PR.DEFAULT_PRIORITIES)),
    "ClusterAutoscalerProvider": lambda: (
        list(P.DEFAULT_PREDICATES),
        {("MostRequestedPriority" if k == "LeastRequestedPriority" else k): v for k, v in PR.DEFAULT_PRIORITIES.items()}),
}


class PolicyError(ValueError):
    pass


def parse_policy(pol):
    """(predicates | None, priorities | None, extender configs) from a Policy object."""
    if isinstance(pol, (str, bytes)):
        pol = json.loads(pol) if str(pol).lstrip().startswith("{") else yaml.safe_load(pol)
    if pol.get("kind", "Policy") != "Policy":
        raise PolicyError(f"expected kind Policy, got {pol.get('kind')!r}")
    preds = None
    if pol.get("predicates") is not None:
        preds = [p["name"] for p in pol["predicates"]]
        unknown = [n for n in preds if n not in P.PREDICATES]
        if unknown:
            raise PolicyError(f"unknown predicates {unknown}")
    prios = None
    if pol.get("priorities") is not None:
        prios = {p["name"]: int(p.get("weight", 1)) for p in pol["priorities"]}
        unknown = [n for n in prios if n not in PR.PRIORITIES]
        if unknown:
            raise PolicyError(f"unknown priorities {unknown}")
        bad = [n for n, w in prios.items() if w <= 0]
        if bad:
            raise PolicyError(f"priority weights must be positive: {bad}")
    return preds, prios, list(pol.get("extenders") or [])


def load_component_config(text):
    cfg = yaml.safe_load(text) or {}
    if cfg.get("kind", "KubeSchedulerConfiguration") != "KubeSchedulerConfiguration":
        raise PolicyError(f"expected KubeSchedulerConfiguration, got {cfg.get('kind')!r}")
    return cfg


async def resolve_algorithm(client, provider=None, policy_file=None, policy_configmap=None,
                            policy_configmap_namespace="kube-system"):
    """(predicates, priorities, extender configs) for the configured algorithm source."""
    if policy_file:
        with open(policy_file) as f:
            return parse_policy(f.read())
    if policy_configmap:
        cm = await client.get("configmaps", policy_configmap, policy_configmap_namespace)
        data = (cm.get("data") or {}).get("policy.cfg")
        if not data:
            raise PolicyError(f"ConfigMap {policy_configmap_namespace}/{policy_configmap} has no policy.cfg")
        return parse_policy(data)
    name = provider or "DefaultProvider"
    if name not in PROVIDERS:
        raise PolicyError(f"unknown algorithm provider {name!r} (have {sorted(PROVIDERS)})")
    preds, prios = PROVIDERS[name]()
    return preds, prios, []
