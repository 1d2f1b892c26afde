"""core/v1 constants and the fork's ResourceV2 ("extended resources") helpers.

Parity:
  * ER types: `staging/src/k8s.io/api/core/v1/types.go:2202-2204, 2631-2640, 2885, 3848-3850, 4011-4057, 4493-4495`
  * ER helpers: `pkg/apis/core/v1/helper/helpers.go:465-534`
  * defaults: `pkg/apis/core/v1/defaults.go:164-180`

MI355X mapping: the device resource is `amd.com/gpu`; per-device
attributes are vendor-prefixed (`amd.com/arch=gfx950`, `amd.com/memory=<MiB>`,
`amd.com/hbm=288Gi`, `amd.com/xgmi-hive=<id>`, `amd.com/numa`, `amd.com/render-minor`, ...).
"""
from __future__ import annotations

from .labels import node_selector_requirements_as_selector
from .quantity import Quantity, parse_quantity

AMD_GPU = "amd.com/gpu"
HEALTHY = "Healthy"
UNHEALTHY = "Unhealthy"

# device attribute keys advertised by the amd.com/gpu plugin
ATTR_ARCH = "amd.com/arch"                # gfx950
ATTR_PRODUCT = "amd.com/product"          # MI355X
ATTR_MEMORY = "amd.com/memory"            # MiB, integer (reference-style numeric attr)
ATTR_HBM = "amd.com/hbm"                  # quantity string, e.g. 288Gi
ATTR_HIVE = "amd.com/xgmi-hive"           # xGMI hive id (hex)
ATTR_NUMA = "amd.com/numa"
ATTR_BDF = "amd.com/bdf"
ATTR_RENDER_MINOR = "amd.com/render-minor"
ATTR_CARD_MINOR = "amd.com/card-minor"
ATTR_INDEX = "amd.com/index"
ATTR_PARTITION = "amd.com/partition"      # SPX / DPX / QPX / CPX
ATTR_SOCKET = "amd.com/socket"            # physical package: partitions of one MI355X share it
ATTR_PARTITION_ID = "amd.com/partition-id"
ATTR_MEMORY_PARTITION = "amd.com/memory-partition"   # NPS1 / NPS2
ATTR_ECC = "amd.com/ecc"                  # uncorrectable ECC count
ATTR_CUS = "amd.com/compute-units"
ATTR_UUID = "amd.com/uuid"
ATTR_XGMI_LINKS = "amd.com/xgmi-links"    # number of active xGMI links
ATTR_XGMI_NODE = "amd.com/xgmi-node"      # the package's index inside its hive (0..7)
ATTR_XGMI_PEERS = "amd.com/xgmi-peers"    # hex bitmask of hive indices reachable over an up xGMI link

POD_PENDING, POD_RUNNING, POD_SUCCEEDED, POD_FAILED, POD_UNKNOWN = (
    "Pending", "Running", "Succeeded", "Failed", "Unknown")

COND_POD_SCHEDULED = "PodScheduled"
COND_READY = "Ready"
COND_INITIALIZED = "Initialized"
COND_CONTAINERS_READY = "ContainersReady"

NODE_READY = "Ready"
TAINT_NO_SCHEDULE = "NoSchedule"
TAINT_PREFER_NO_SCHEDULE = "PreferNoSchedule"
TAINT_NO_EXECUTE = "NoExecute"

BASIC_RESOURCES = ("cpu", "memory", "ephemeral-storage", "pods")


# ---------------------------------------------------------------------------
# resources

def is_extended_resource_name(name: str) -> bool:
    """`helper.IsExtendedResourceName`: fully qualified, not kubernetes.io / requests. prefixed."""
    if "/" not in name or name.startswith("requests."):
        return False
    domain = name.split("/", 1)[0]
    return not (domain == "kubernetes.io" or domain.endswith(".kubernetes.io"))


def container_requests(c) -> dict:
    """Effective requests (limits default requests, like the reference defaulter)."""
    res = c.get("resources") or {}
    req = dict(res.get("requests") or {})
    for k, v in (res.get("limits") or {}).items():
        req.setdefault(k, v)
    return req


def pod_requests(pod) -> dict[str, Quantity]:
    """Sum of container requests, max'd with each init container
    (`predicates.GetResourceRequest`, plugin/pkg/scheduler/algorithm/predicates/predicates.go)."""
    spec = pod.get("spec") or {}
    total: dict[str, Quantity] = {}
    for c in spec.get("containers") or ():
        for k, v in container_requests(c).items():
            qv = parse_quantity(v) if isinstance(v, str) else Quantity(v)
            total[k] = total[k] + qv if k in total else qv
    for c in spec.get("initContainers") or ():
        for k, v in container_requests(c).items():
            qv = parse_quantity(v) if isinstance(v, str) else Quantity(v)
            if k not in total or qv > total[k]:
                total[k] = qv
    return total


# ---------------------------------------------------------------------------
# ResourceV2 helpers

def extended_requirements_as_selector(reqs):
    return node_selector_requirements_as_selector(reqs)


def pod_extended_resource_name(per) -> str:
    """`PodExtendedResourceName`: exactly one limit key."""
    limits = ((per.get("resources") or {}).get("limits")) or {}
    if len(limits) != 1:
        raise ValueError(f"unexpected limits length: {len(limits)} != 1")
    return next(iter(limits))


def pod_extended_resource_count(per) -> int:
    name = pod_extended_resource_name(per)
    return parse_quantity(str(per["resources"]["limits"][name])).int_value()


def pod_extended_resource_index(name, ers) -> int:
    for i, r in enumerate(ers or ()):
        if r.get("name") == name:
            return i
    raise KeyError(f"Could not find PodExtendedResource {name}")


def pod_extended_resource_assigned(rname, container, pod) -> list[str]:
    """`PodExtendedResourceAssigned(rName, c, p)`: IDs assigned to a container's ER requests
    restricted to resource `rname` (the reference ignores rname — a latent bug when a
    container references two resources; we filter)."""
    ers = (pod.get("spec") or {}).get("extendedResources") or []
    ids: list[str] = []
    for req in container.get("extendedResourceRequests") or ():
        per = ers[pod_extended_resource_index(req, ers)]
        if rname is None or pod_extended_resource_name(per) == rname:
            ids.extend(per.get("assigned") or ())
    return ids


def pod_assigned_devices(pod) -> dict[str, list[str]]:
    """resource name -> all assigned device IDs of the pod."""
    out: dict[str, list[str]] = {}
    for per in (pod.get("spec") or {}).get("extendedResources") or ():
        a = per.get("assigned")
        if not a:
            continue
        try:
            rn = pod_extended_resource_name(per)
        except ValueError:
            continue
        out.setdefault(rn, []).extend(a)
    return out


def set_defaults_pod(pod):
    """Defaults relevant to the fork (`pkg/apis/core/v1/defaults.go:164-180`) plus the
    handful of PodSpec defaults the scheduler/kubelet rely on."""
    spec = pod.setdefault("spec", {})
    spec.setdefault("restartPolicy", "Always")
    spec.setdefault("schedulerName", "default-scheduler")
    spec.setdefault("dnsPolicy", "ClusterFirst")
    spec.setdefault("terminationGracePeriodSeconds", 30)
    for c in (spec.get("containers") or []) + (spec.get("initContainers") or []):
        c.setdefault("imagePullPolicy", "Always" if str(c.get("image", "")).endswith(":latest") or ":" not in str(c.get("image", "")) else "IfNotPresent")
        c.setdefault("terminationMessagePath", "/dev/termination-log")
        res = c.get("resources")
        if res and res.get("limits"):
            req = res.setdefault("requests", {})
            for k, v in res["limits"].items():
                req.setdefault(k, v)
    for per in spec.get("extendedResources") or ():
        res = per.setdefault("resources", {})
        lim = res.get("limits")
        if lim is None:
            continue
        req = res.setdefault("requests", {})
        for k, v in lim.items():
            req.setdefault(k, v)
        per.setdefault("affinity", {})
    st = pod.setdefault("status", {})
    st.setdefault("phase", POD_PENDING)
    return pod


def get_condition(status, ctype):
    for c in (status or {}).get("conditions") or ():
        if c.get("type") == ctype:
            return c
    return None


def set_condition(status, cond):
    conds = status.setdefault("conditions", [])
    for i, c in enumerate(conds):
        if c.get("type") == cond["type"]:
            if c.get("status") == cond.get("status"):
                cond = dict(cond)
                cond["lastTransitionTime"] = c.get("lastTransitionTime", cond.get("lastTransitionTime"))
            conds[i] = cond
            return
    conds.append(cond)


def node_is_ready(node) -> bool:
    c = get_condition(node.get("status"), NODE_READY)
    return c is not None and c.get("status") == "True"


def pod_is_terminal(pod) -> bool:
    return (pod.get("status") or {}).get("phase") in (POD_SUCCEEDED, POD_FAILED)


def tolerates(tolerations, taint) -> bool:
    """`v1helper.TolerationsTolerateTaint`."""
    for t in tolerations or ():
        eff = t.get("effect")
        if eff and eff != taint.get("effect"):
            continue
        op = t.get("operator", "Equal")
        key = t.get("key")
        if key and key != taint.get("key"):
            continue
        if not key and op != "Exists":
            continue
        if op == "Exists" or t.get("value", "") == taint.get("value", ""):
            return True
    return False


_VOLUME_SECRET_REFS = ("cephfs", "flexVolume", "rbd", "scaleIO", "iscsi", "storageos")


def pod_secret_names(pod) -> list[str]:
    """Every secret a pod references, in `VisitPodSecretNames` order
    (`pkg/api/v1/pod/util.go:58-145`): image pull secrets; envFrom / secretKeyRef of init
    containers then containers; secret, projected, azureFile and the secretRef of cephfs /
    flexVolume / rbd / scaleIO / iscsi / storageos volumes."""
    spec = pod.get("spec") or {}
    out = [r.get("name", "") for r in spec.get("imagePullSecrets") or ()]
    for c in (spec.get("initContainers") or []) + (spec.get("containers") or []):
        for ef in c.get("envFrom") or ():
            if ef.get("secretRef") is not None:
                out.append(ef["secretRef"].get("name", ""))
        for e in c.get("env") or ():
            ref = (e.get("valueFrom") or {}).get("secretKeyRef")
            if ref is not None:
                out.append(ref.get("name", ""))
    for v in spec.get("volumes") or ():
        if v.get("secret") is not None:
            out.append(v["secret"].get("secretName", ""))
        elif v.get("projected") is not None:
            out += [s["secret"].get("name", "") for s in v["projected"].get("sources") or () if s.get("secret") is not None]
        elif v.get("azureFile") is not None:
            if v["azureFile"].get("secretName"):
                out.append(v["azureFile"]["secretName"])
        else:
            for k in _VOLUME_SECRET_REFS:
                if v.get(k) is not None:
                    ref = v[k].get("secretRef")
                    if ref is not None:
                        out.append(ref.get("name", ""))
                    break
    return out
