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


class Algorithm(tuple):
    """(predicates | None, priorities | None, extender configs) — unpacks as a 3-tuple — plus
    the Policy's hardPodAffinitySymmetricWeight (None when the Policy does not set it)."""
    hard_pod_affinity_symmetric_weight = None

    def __new__(cls, preds, prios, extenders, hard_weight=None):
        self = super().__new__(cls, (preds, prios, extenders))
        self.hard_pod_affinity_symmetric_weight = hard_weight
        return self


def _custom_predicate(entry):
    """`factory/plugins.go:198-240`: an entry with an argument builds a new predicate under the
    entry's own name; exactly one argument kind may be given (`validatePredicateOrDie`)."""
    arg = entry.get("argument") or {}
    kinds = [k for k in ("serviceAffinity", "labelsPresence") if arg.get(k) is not None]
    if len(kinds) != 1:
        raise PolicyError(f"predicate {entry['name']!r}: exactly one of serviceAffinity, labelsPresence "
                          f"must be set in its argument")
    if kinds[0] == "serviceAffinity":
        labels = arg["serviceAffinity"].get("labels") or []
        return P.make_service_affinity(labels)
    lp = arg["labelsPresence"]
    return P.make_labels_presence(lp.get("labels") or [], bool(lp.get("presence", False)))


def _custom_priority(entry, weight):
    """`factory/plugins.go:299-340`: serviceAntiAffinity{label} or labelPreference{label,presence}."""
    arg = entry.get("argument") or {}
    kinds = [k for k in ("serviceAntiAffinity", "labelPreference") if arg.get(k) is not None]
    if len(kinds) != 1:
        raise PolicyError(f"priority {entry['name']!r}: exactly one of serviceAntiAffinity, labelPreference "
                          f"must be set in its argument")
    if kinds[0] == "serviceAntiAffinity":
        label = arg["serviceAntiAffinity"].get("label")
        if not label:
            raise PolicyError(f"priority {entry['name']!r}: serviceAntiAffinity needs a label")
        return (weight, PR.make_service_anti_affinity(label), False, False)
    lp = arg["labelPreference"]
    if not lp.get("label"):
        raise PolicyError(f"priority {entry['name']!r}: labelPreference needs a label")
    return (weight, PR.make_label_preference(lp["label"], bool(lp.get("presence", False))), False, False)


def parse_policy(pol):
    """Policy (`plugin/pkg/scheduler/api/types.go:38-129`) -> Algorithm.

    predicates: a list of registry names, or (name, fn) for an argument-based entry;
    priorities: name -> weight, or name -> (weight, fn, reverse, normalize) for an
    argument-based entry. Unknown names without an argument are an error, as is a
    non-positive priority weight (`validation.go` ValidatePolicy)."""
    if isinstance(pol, (str, bytes)):
        pol = json.loads(pol) if str(pol).lstrip().startswith("{") else yaml.safe_load(pol)
    if pol.get("kind", "Policy") != "Policy":
        raise PolicyError(f"expected kind Policy, got {pol.get('kind')!r}")
    preds = None
    if pol.get("predicates") is not None:
        preds, unknown = [], []
        for e in pol["predicates"]:
            if e.get("argument") is not None:
                preds.append((e["name"], _custom_predicate(e)))
            elif e["name"] in P.PREDICATES:
                preds.append(e["name"])
            else:
                unknown.append(e["name"])
        if unknown:
            raise PolicyError(f"unknown predicates {unknown}")
    prios = None
    if pol.get("priorities") is not None:
        prios, unknown, bad = {}, [], []
        for e in pol["priorities"]:
            w = int(e.get("weight", 1))
            if w <= 0:
                bad.append(e["name"])
            if e.get("argument") is not None:
                prios[e["name"]] = _custom_priority(e, w)
            elif e["name"] in PR.PRIORITIES:
                prios[e["name"]] = w
            else:
                unknown.append(e["name"])
        if unknown:
            raise PolicyError(f"unknown priorities {unknown}")
        if bad:
            raise PolicyError(f"priority weights must be positive: {bad}")
    hw = pol.get("hardPodAffinitySymmetricWeight")
    if hw is not None and not 0 <= int(hw) <= 100:
        raise PolicyError("hardPodAffinitySymmetricWeight must be in the range 0-100")
    binders = 0
    for e in pol.get("extenders") or []:
        if not e.get("urlPrefix"):
            raise PolicyError("extender needs a urlPrefix")
        if int(e.get("weight", 1)) <= 0 and e.get("prioritizeVerb"):
            raise PolicyError(f"extender {e['urlPrefix']}: weight must be positive")
        if e.get("bindVerb") or e.get("BindVerb"):
            binders += 1
    if binders > 1:     # api/validation/validation.go:37-48
        raise PolicyError(f"Only one extender can implement bind, found {binders}")
    return Algorithm(preds, prios, list(pol.get("extenders") or []), None if hw is None else int(hw))


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
    return Algorithm(preds, prios, [])
