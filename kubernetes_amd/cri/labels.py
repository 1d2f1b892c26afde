"""Labels and annotations the kubelet puts on CRI sandboxes and containers
(`pkg/kubelet/kuberuntime/labels.go`), and their readers.

Sandboxes carry the pod's labels plus its name / namespace / UID, and the pod's annotations.
Containers carry the pod identity and container name as labels; their annotations hold the
container hash, restart count, termination-message path and policy, the pod's deletion and
termination grace periods, the preStop handler and the container ports (JSON), so a restarted
kubelet can stop a container it no longer has the spec for. Device-plugin annotations come first
and are overridden by the kubelet's own. The container hash is FNV-1a (32 bit) over the
canonical JSON of the container spec, printed in hex (the reference hashes Go's spew dump of the
struct, which has no portable equivalent).
"""
from __future__ import annotations

import json

from .api import CONTAINER_NAME, POD_NAME, POD_NAMESPACE, POD_UID

POD_DELETION_GRACE_PERIOD = "io.kubernetes.pod.deletionGracePeriod"
POD_TERMINATION_GRACE_PERIOD = "io.kubernetes.pod.terminationGracePeriod"
CONTAINER_HASH = "io.kubernetes.container.hash"
CONTAINER_RESTART_COUNT = "io.kubernetes.container.restartCount"
CONTAINER_TERMINATION_MESSAGE_PATH = "io.kubernetes.container.terminationMessagePath"
CONTAINER_TERMINATION_MESSAGE_POLICY = "io.kubernetes.container.terminationMessagePolicy"
CONTAINER_PRESTOP_HANDLER = "io.kubernetes.container.preStopHandler"
CONTAINER_PORTS = "io.kubernetes.container.ports"


def hash_container(container) -> int:
    data = json.dumps(container, sort_keys=True, separators=(",", ":")).encode()
    h = 0x811C9DC5
    for b in data:
        h = ((h ^ b) * 0x01000193) & 0xFFFFFFFF
    return h


def new_pod_labels(pod) -> dict:
    md = pod.get("metadata") or {}
    labels = dict(md.get("labels") or {})
    labels.update({POD_NAME: md.get("name", ""), POD_NAMESPACE: md.get("namespace", ""), POD_UID: md.get("uid", "")})
    return labels


def new_pod_annotations(pod) -> dict:
    return dict((pod.get("metadata") or {}).get("annotations") or {})


def new_container_labels(container, pod) -> dict:
    md = pod.get("metadata") or {}
    return {POD_NAME: md.get("name", ""), POD_NAMESPACE: md.get("namespace", ""), POD_UID: md.get("uid", ""),
            CONTAINER_NAME: container.get("name", "")}


def new_container_annotations(container, pod, restart_count, device_annotations=()) -> dict:
    ann = {a["name"]: a["value"] for a in device_annotations or ()}
    ann[CONTAINER_HASH] = format(hash_container(container), "x")
    ann[CONTAINER_RESTART_COUNT] = str(int(restart_count))
    ann[CONTAINER_TERMINATION_MESSAGE_PATH] = container.get("terminationMessagePath", "")
    ann[CONTAINER_TERMINATION_MESSAGE_POLICY] = container.get("terminationMessagePolicy", "")
    md, spec = pod.get("metadata") or {}, pod.get("spec") or {}
    if md.get("deletionGracePeriodSeconds") is not None:
        ann[POD_DELETION_GRACE_PERIOD] = str(int(md["deletionGracePeriodSeconds"]))
    if spec.get("terminationGracePeriodSeconds") is not None:
        ann[POD_TERMINATION_GRACE_PERIOD] = str(int(spec["terminationGracePeriodSeconds"]))
    pre = (container.get("lifecycle") or {}).get("preStop")
    if pre is not None:
        ann[CONTAINER_PRESTOP_HANDLER] = json.dumps(pre, separators=(",", ":"))
    if container.get("ports"):
        ann[CONTAINER_PORTS] = json.dumps(container["ports"], separators=(",", ":"))
    return ann


def pod_sandbox_info_from_labels(labels) -> dict:
    ids = (POD_NAME, POD_NAMESPACE, POD_UID)
    return {"podName": labels.get(POD_NAME, ""), "podNamespace": labels.get(POD_NAMESPACE, ""),
            "podUID": labels.get(POD_UID, ""), "labels": {k: v for k, v in labels.items() if k not in ids}}


def container_info_from_labels(labels) -> dict:
    return {"podName": labels.get(POD_NAME, ""), "podNamespace": labels.get(POD_NAMESPACE, ""),
            "podUID": labels.get(POD_UID, ""), "containerName": labels.get(CONTAINER_NAME, "")}


def _int(ann, key, default=0):
    try:
        return int(ann[key]) if key in ann else default
    except ValueError:
        return default


def container_info_from_annotations(ann) -> dict:
    """getContainerInfoFromAnnotations: unparsable values read as zero / None."""
    try:
        h = int(ann.get(CONTAINER_HASH, "0"), 16)
    except ValueError:
        h = 0
    out = {"hash": h, "restartCount": _int(ann, CONTAINER_RESTART_COUNT),
           "terminationMessagePath": ann.get(CONTAINER_TERMINATION_MESSAGE_PATH, ""),
           "terminationMessagePolicy": ann.get(CONTAINER_TERMINATION_MESSAGE_POLICY, ""),
           "podDeletionGracePeriod": _int(ann, POD_DELETION_GRACE_PERIOD, None),
           "podTerminationGracePeriod": _int(ann, POD_TERMINATION_GRACE_PERIOD, None),
           "preStopHandler": None, "containerPorts": None}
    for key, field in ((CONTAINER_PRESTOP_HANDLER, "preStopHandler"), (CONTAINER_PORTS, "containerPorts")):
        if key in ann:
            try:
                out[field] = json.loads(ann[key])
            except ValueError:
                pass
    return out


def container_log_path(container_name, restart_count) -> str:
    """`BuildContainerLogsPath`: <container>/<restartCount>.log under the pod log directory."""
    return f"{container_name}/{int(restart_count)}.log"
