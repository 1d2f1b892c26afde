"""Kubernetes protobuf wire/storage format for the core/v1 objects, including the fork's
ResourceV2 fields, and the `k8s\\x00` + runtime.Unknown envelope.

Parity:
  * envelope: `staging/src/k8s.io/apimachinery/pkg/runtime/serializer/protobuf/protobuf.go:42`
    (magic `0x6b 0x38 0x73 0x00`) + `runtime.Unknown{typeMeta=1{apiVersion=1,kind=2}, raw=2,
    contentEncoding=3, contentType=4}` (`staging/src/k8s.io/apimachinery/pkg/runtime/types.go:112-124`);
  * field numbers: `staging/src/k8s.io/api/core/v1/generated.proto` — fork fields Container 22,
    PodSpec 27, NodeStatus 11, ObjectReference 8 (`extendedResourceBinding`), PodExtendedResource
    1..5, ExtendedResourceDomain / ExtendedResource / ExtendedResourceList;
  * value encodings: meta/v1 Time `{seconds=1, nanos=2}`, resource.Quantity `{string=1}`,
    intstr.IntOrString `{type=1, intVal=2, strVal=3}`; maps as repeated entry messages with
    keys in sorted order (the generated marshalers sort map keys) and fields in ascending
    field-number order, so encoding is deterministic.
Gogo-embedded structs whose JSON is inlined (Volume.VolumeSource, *VolumeSource's
LocalObjectReference, ...) are marked `inline`.

Pure-Python codec (no protoc in this image): a compact schema table drives both directions.
"""
from __future__ import annotations

import datetime as _dt

MAGIC = b"k8s\x00"

# field kinds
S, B, I64, I32, MSG, MAPS, MAPM, RS, RM, RI64, TIME, QTY, IOS, INL, BYTES = (
    "s", "b", "i64", "i32", "m", "mapS", "mapM", "rs", "rm", "ri64", "time", "qty", "ios", "inline", "bytes")

# message -> [(json name, field number, kind, message type)]
SCHEMA: dict[str, list] = {
    # --- meta/v1 ----------------------------------------------------------
    "ObjectMeta": [("name", 1, S, None), ("generateName", 2, S, None), ("namespace", 3, S, None),
                   ("selfLink", 4, S, None), ("uid", 5, S, None), ("resourceVersion", 6, S, None),
                   ("generation", 7, I64, None), ("creationTimestamp", 8, TIME, None),
                   ("deletionTimestamp", 9, TIME, None), ("deletionGracePeriodSeconds", 10, I64, None),
                   ("labels", 11, MAPS, None), ("annotations", 12, MAPS, None),
                   ("ownerReferences", 13, RM, "OwnerReference"), ("finalizers", 14, RS, None),
                   ("clusterName", 15, S, None)],
    "OwnerReference": [("kind", 1, S, None), ("name", 3, S, None), ("uid", 4, S, None), ("apiVersion", 5, S, None),
                       ("controller", 6, B, None), ("blockOwnerDeletion", 7, B, None)],
    "ListMeta": [("selfLink", 1, S, None), ("resourceVersion", 2, S, None), ("continue", 3, S, None)],
    "LabelSelector": [("matchLabels", 1, MAPS, None), ("matchExpressions", 2, RM, "LabelSelectorRequirement")],
    "LabelSelectorRequirement": [("key", 1, S, None), ("operator", 2, S, None), ("values", 3, RS, None)],
    # --- core/v1 pod ------------------------------------------------------------
    "Pod": [("metadata", 1, MSG, "ObjectMeta"), ("spec", 2, MSG, "PodSpec"), ("status", 3, MSG, "PodStatus")],
    "PodList": [("metadata", 1, MSG, "ListMeta"), ("items", 2, RM, "Pod")],
    "PodSpec": [("volumes", 1, RM, "Volume"), ("containers", 2, RM, "Container"), ("restartPolicy", 3, S, None),
                ("terminationGracePeriodSeconds", 4, I64, None), ("activeDeadlineSeconds", 5, I64, None),
                ("dnsPolicy", 6, S, None), ("nodeSelector", 7, MAPS, None), ("serviceAccountName", 8, S, None),
                ("serviceAccount", 9, S, None), ("nodeName", 10, S, None), ("hostNetwork", 11, B, None),
                ("hostPID", 12, B, None), ("hostIPC", 13, B, None), ("securityContext", 14, MSG, "PodSecurityContext"),
                ("imagePullSecrets", 15, RM, "LocalObjectReference"), ("hostname", 16, S, None),
                ("subdomain", 17, S, None), ("affinity", 18, MSG, "Affinity"), ("schedulerName", 19, S, None),
                ("initContainers", 20, RM, "Container"), ("automountServiceAccountToken", 21, B, None),
                ("tolerations", 22, RM, "Toleration"), ("hostAliases", 23, RM, "HostAlias"),
                ("priorityClassName", 24, S, None), ("priority", 25, I32, None),
                ("extendedResources", 27, RM, "PodExtendedResource")],
    "Container": [("name", 1, S, None), ("image", 2, S, None), ("command", 3, RS, None), ("args", 4, RS, None),
                  ("workingDir", 5, S, None), ("ports", 6, RM, "ContainerPort"), ("env", 7, RM, "EnvVar"),
                  ("resources", 8, MSG, "ResourceRequirements"), ("volumeMounts", 9, RM, "VolumeMount"),
                  ("livenessProbe", 10, MSG, "Probe"), ("readinessProbe", 11, MSG, "Probe"),
                  ("terminationMessagePath", 13, S, None), ("imagePullPolicy", 14, S, None),
                  ("securityContext", 15, MSG, "SecurityContext"), ("stdin", 16, B, None), ("stdinOnce", 17, B, None),
                  ("tty", 18, B, None), ("terminationMessagePolicy", 20, S, None),
                  ("extendedResourceRequests", 22, RS, None)],
    "ContainerPort": [("name", 1, S, None), ("hostPort", 2, I32, None), ("containerPort", 3, I32, None),
                      ("protocol", 4, S, None), ("hostIP", 5, S, None)],
    "EnvVar": [("name", 1, S, None), ("value", 2, S, None), ("valueFrom", 3, MSG, "EnvVarSource")],
    "EnvVarSource": [("fieldRef", 1, MSG, "ObjectFieldSelector"), ("resourceFieldRef", 2, MSG, "ResourceFieldSelector"),
                     ("configMapKeyRef", 3, MSG, "ConfigMapKeySelector"), ("secretKeyRef", 4, MSG, "SecretKeySelector")],
    "ObjectFieldSelector": [("apiVersion", 1, S, None), ("fieldPath", 2, S, None)],
    "ResourceFieldSelector": [("containerName", 1, S, None), ("resource", 2, S, None), ("divisor", 3, QTY, None)],
    "ConfigMapKeySelector": [(None, 1, INL, "LocalObjectReference"), ("key", 2, S, None), ("optional", 3, B, None)],
    "SecretKeySelector": [(None, 1, INL, "LocalObjectReference"), ("key", 2, S, None), ("optional", 3, B, None)],
    "LocalObjectReference": [("name", 1, S, None)],
    "ResourceRequirements": [("limits", 1, MAPM, "Quantity"), ("requests", 2, MAPM, "Quantity")],
    "VolumeMount": [("name", 1, S, None), ("readOnly", 2, B, None), ("mountPath", 3, S, None), ("subPath", 4, S, None),
                    ("mountPropagation", 5, S, None)],
    "Volume": [("name", 1, S, None), (None, 2, INL, "VolumeSource")],
    "VolumeSource": [("hostPath", 1, MSG, "HostPathVolumeSource"), ("emptyDir", 2, MSG, "EmptyDirVolumeSource"),
                     ("secret", 6, MSG, "SecretVolumeSource"),
                     ("persistentVolumeClaim", 10, MSG, "PersistentVolumeClaimVolumeSource"),
                     ("configMap", 19, MSG, "ConfigMapVolumeSource")],
    "HostPathVolumeSource": [("path", 1, S, None), ("type", 2, S, None)],
    "EmptyDirVolumeSource": [("medium", 1, S, None), ("sizeLimit", 2, QTY, None)],
    "SecretVolumeSource": [("secretName", 1, S, None), ("items", 2, RM, "KeyToPath"), ("defaultMode", 3, I32, None),
                           ("optional", 4, B, None)],
    "ConfigMapVolumeSource": [(None, 1, INL, "LocalObjectReference"), ("items", 2, RM, "KeyToPath"),
                              ("defaultMode", 3, I32, None), ("optional", 4, B, None)],
    "PersistentVolumeClaimVolumeSource": [("claimName", 1, S, None), ("readOnly", 2, B, None)],
    "KeyToPath": [("key", 1, S, None), ("path", 2, S, None), ("mode", 3, I32, None)],
    "Probe": [(None, 1, INL, "Handler"), ("initialDelaySeconds", 2, I32, None), ("timeoutSeconds", 3, I32, None),
              ("periodSeconds", 4, I32, None), ("successThreshold", 5, I32, None), ("failureThreshold", 6, I32, None)],
    "Handler": [("exec", 1, MSG, "ExecAction"), ("httpGet", 2, MSG, "HTTPGetAction"), ("tcpSocket", 3, MSG, "TCPSocketAction")],
    "ExecAction": [("command", 1, RS, None)],
    "HTTPGetAction": [("path", 1, S, None), ("port", 2, IOS, None), ("host", 3, S, None), ("scheme", 4, S, None)],
    "TCPSocketAction": [("port", 1, IOS, None), ("host", 2, S, None)],
    "PodSecurityContext": [("runAsUser", 2, I64, None), ("runAsNonRoot", 3, B, None),
                           ("supplementalGroups", 4, RI64, None), ("fsGroup", 5, I64, None)],
    "SecurityContext": [("capabilities", 1, MSG, "Capabilities"), ("privileged", 2, B, None), ("runAsUser", 4, I64, None),
                        ("runAsNonRoot", 5, B, None), ("readOnlyRootFilesystem", 6, B, None),
                        ("allowPrivilegeEscalation", 7, B, None)],
    "Capabilities": [("add", 1, RS, None), ("drop", 2, RS, None)],
    "Toleration": [("key", 1, S, None), ("operator", 2, S, None), ("value", 3, S, None), ("effect", 4, S, None),
                   ("tolerationSeconds", 5, I64, None)],
    "HostAlias": [("ip", 1, S, None), ("hostnames", 2, RS, None)],
    "Affinity": [("nodeAffinity", 1, MSG, "NodeAffinity"), ("podAffinity", 2, MSG, "PodAffinity"),
                 ("podAntiAffinity", 3, MSG, "PodAntiAffinity")],
    "NodeAffinity": [("requiredDuringSchedulingIgnoredDuringExecution", 1, MSG, "NodeSelector"),
                     ("preferredDuringSchedulingIgnoredDuringExecution", 2, RM, "PreferredSchedulingTerm")],
    "NodeSelector": [("nodeSelectorTerms", 1, RM, "NodeSelectorTerm")],
    "NodeSelectorTerm": [("matchExpressions", 1, RM, "NodeSelectorRequirement")],
    "NodeSelectorRequirement": [("key", 1, S, None), ("operator", 2, S, None), ("values", 3, RS, None)],
    "PreferredSchedulingTerm": [("weight", 1, I32, None), ("preference", 2, MSG, "NodeSelectorTerm")],
    "PodAffinity": [("requiredDuringSchedulingIgnoredDuringExecution", 1, RM, "PodAffinityTerm"),
                    ("preferredDuringSchedulingIgnoredDuringExecution", 2, RM, "WeightedPodAffinityTerm")],
    "PodAntiAffinity": [("requiredDuringSchedulingIgnoredDuringExecution", 1, RM, "PodAffinityTerm"),
                        ("preferredDuringSchedulingIgnoredDuringExecution", 2, RM, "WeightedPodAffinityTerm")],
    "PodAffinityTerm": [("labelSelector", 1, MSG, "LabelSelector"), ("namespaces", 2, RS, None), ("topologyKey", 3, S, None)],
    "WeightedPodAffinityTerm": [("weight", 1, I32, None), ("podAffinityTerm", 2, MSG, "PodAffinityTerm")],
    # fork ResourceV2
    "PodExtendedResource": [("name", 1, S, None), ("resources", 2, MSG, "ResourceRequirements"),
                            ("affinity", 3, MSG, "ExtendedResourceAffinity"), ("annotations", 4, MAPS, None),
                            ("assigned", 5, RS, None)],
    "ExtendedResourceAffinity": [("required", 1, RM, "NodeSelectorRequirement")],   # ResourceSelector
    "ExtendedResourceDomain": [("resources", 1, MAPM, "ExtendedResource")],
    "ExtendedResource": [("id", 1, S, None), ("health", 2, S, None), ("attributes", 3, MAPS, None)],
    "ExtendedResourceList": [("resources", 1, RS, None)],
    "PodStatus": [("phase", 1, S, None), ("conditions", 2, RM, "PodCondition"), ("message", 3, S, None),
                  ("reason", 4, S, None), ("hostIP", 5, S, None), ("podIP", 6, S, None), ("startTime", 7, TIME, None),
                  ("containerStatuses", 8, RM, "ContainerStatus"), ("qosClass", 9, S, None),
                  ("initContainerStatuses", 10, RM, "ContainerStatus")],
    "PodCondition": [("type", 1, S, None), ("status", 2, S, None), ("lastProbeTime", 3, TIME, None),
                     ("lastTransitionTime", 4, TIME, None), ("reason", 5, S, None), ("message", 6, S, None)],
    "ContainerStatus": [("name", 1, S, None), ("state", 2, MSG, "ContainerState"), ("lastState", 3, MSG, "ContainerState"),
                        ("ready", 4, B, None), ("restartCount", 5, I32, None), ("image", 6, S, None),
                        ("imageID", 7, S, None), ("containerID", 8, S, None)],
    "ContainerState": [("waiting", 1, MSG, "ContainerStateWaiting"), ("running", 2, MSG, "ContainerStateRunning"),
                       ("terminated", 3, MSG, "ContainerStateTerminated")],
    "ContainerStateWaiting": [("reason", 1, S, None), ("message", 2, S, None)],
    "ContainerStateRunning": [("startedAt", 1, TIME, None)],
    "ContainerStateTerminated": [("exitCode", 1, I32, None), ("signal", 2, I32, None), ("reason", 3, S, None),
                                 ("message", 4, S, None), ("startedAt", 5, TIME, None), ("finishedAt", 6, TIME, None),
                                 ("containerID", 7, S, None)],
    # --- node -------------------------------------------------------------------
    "Node": [("metadata", 1, MSG, "ObjectMeta"), ("spec", 2, MSG, "NodeSpec"), ("status", 3, MSG, "NodeStatus")],
    "NodeSpec": [("podCIDR", 1, S, None), ("externalID", 2, S, None), ("providerID", 3, S, None),
                 ("unschedulable", 4, B, None), ("taints", 5, RM, "Taint")],
    "Taint": [("key", 1, S, None), ("value", 2, S, None), ("effect", 3, S, None), ("timeAdded", 4, TIME, None)],
    "NodeStatus": [("capacity", 1, MAPM, "Quantity"), ("allocatable", 2, MAPM, "Quantity"), ("phase", 3, S, None),
                   ("conditions", 4, RM, "NodeCondition"), ("addresses", 5, RM, "NodeAddress"),
                   ("daemonEndpoints", 6, MSG, "NodeDaemonEndpoints"), ("nodeInfo", 7, MSG, "NodeSystemInfo"),
                   ("volumesInUse", 9, RS, None), ("extendedResources", 11, MAPM, "ExtendedResourceDomain")],
    "NodeCondition": [("type", 1, S, None), ("status", 2, S, None), ("lastHeartbeatTime", 3, TIME, None),
                      ("lastTransitionTime", 4, TIME, None), ("reason", 5, S, None), ("message", 6, S, None)],
    "NodeAddress": [("type", 1, S, None), ("address", 2, S, None)],
    "NodeDaemonEndpoints": [("kubeletEndpoint", 1, MSG, "DaemonEndpoint")],
    "DaemonEndpoint": [("Port", 1, I32, None)],
    "NodeSystemInfo": [("machineID", 1, S, None), ("systemUUID", 2, S, None), ("bootID", 3, S, None),
                       ("kernelVersion", 4, S, None), ("osImage", 5, S, None), ("containerRuntimeVersion", 6, S, None),
                       ("kubeletVersion", 7, S, None), ("kubeProxyVersion", 8, S, None), ("operatingSystem", 9, S, None),
                       ("architecture", 10, S, None)],
    # --- binding / refs / namespace / event / configmap --------------------------
    "Binding": [("metadata", 1, MSG, "ObjectMeta"), ("target", 2, MSG, "ObjectReference")],
    "ObjectReference": [("kind", 1, S, None), ("namespace", 2, S, None), ("name", 3, S, None), ("uid", 4, S, None),
                        ("apiVersion", 5, S, None), ("resourceVersion", 6, S, None), ("fieldPath", 7, S, None),
                        ("extendedResourceBinding", 8, MAPM, "ExtendedResourceList")],
    "Namespace": [("metadata", 1, MSG, "ObjectMeta"), ("spec", 2, MSG, "NamespaceSpec"), ("status", 3, MSG, "NamespaceStatus")],
    "NamespaceSpec": [("finalizers", 1, RS, None)],
    "NamespaceStatus": [("phase", 1, S, None)],
    "Event": [("metadata", 1, MSG, "ObjectMeta"), ("involvedObject", 2, MSG, "ObjectReference"), ("reason", 3, S, None),
              ("message", 4, S, None), ("source", 5, MSG, "EventSource"), ("firstTimestamp", 6, TIME, None),
              ("lastTimestamp", 7, TIME, None), ("count", 8, I32, None), ("type", 9, S, None)],
    "EventSource": [("component", 1, S, None), ("host", 2, S, None)],
    "ConfigMap": [("metadata", 1, MSG, "ObjectMeta"), ("data", 2, MAPS, None)],
}

KIND_MESSAGE = {"Pod": "Pod", "Node": "Node", "Namespace": "Namespace", "Binding": "Binding", "Event": "Event",
                "ConfigMap": "ConfigMap", "PodList": "PodList"}

_BY_NUM = {m: {f[1]: f for f in fields} for m, fields in SCHEMA.items()}
_SORTED = {m: sorted(fields, key=lambda f: f[1]) for m, fields in SCHEMA.items()}


class ProtobufError(ValueError):
    pass


# ---------------------------------------------------------------------------
# wire primitives
def _varint(n: int) -> bytes:
    if n < 0:
        n += 1 << 64
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(num, wt):
    return _varint((num << 3) | wt)


def _ld(num, payload: bytes) -> bytes:
    return _key(num, 2) + _varint(len(payload)) + payload


def _read_varint(buf, i):
    shift = n = 0
    while True:
        if i >= len(buf):
            raise ProtobufError("truncated varint")
        b = buf[i]
        i += 1
        n |= (b & 0x7F) << shift
        if not b & 0x80:
            return n, i
        shift += 7


def _parse_time(s):
    if s is None:
        return None
    t = _dt.datetime.fromisoformat(s.replace("Z", "+00:00"))
    ts = t.timestamp()
    sec = int(ts // 1)
    return sec, int(round((ts - sec) * 1e9)) if t.microsecond else 0


def _fmt_time(sec, nanos):
    t = _dt.datetime.fromtimestamp(sec, _dt.timezone.utc)
    if nanos:
        t = t.replace(microsecond=nanos // 1000)
        return t.strftime("%Y-%m-%dT%H:%M:%S.%fZ")
    return t.strftime("%Y-%m-%dT%H:%M:%SZ")


# ---------------------------------------------------------------------------
def encode_message(msg: str, obj: dict) -> bytes:
    out = bytearray()
    for name, num, kind, typ in _SORTED[msg]:
        if kind == INL:
            sub = encode_message(typ, obj)
            out += _ld(num, sub)
            continue
        if name not in obj:
            continue
        v = obj[name]
        if v is None:
            continue
        if kind == S:
            out += _ld(num, str(v).encode())
        elif kind == B:
            out += _key(num, 0) + (b"\x01" if v else b"\x00")
        elif kind in (I64, I32):
            out += _key(num, 0) + _varint(int(v))
        elif kind == MSG:
            out += _ld(num, encode_message(typ, v))
        elif kind == TIME:
            sec, nanos = _parse_time(v)
            t = _key(1, 0) + _varint(sec)
            if nanos:
                t += _key(2, 0) + _varint(nanos)
            out += _ld(num, t)
        elif kind == QTY:
            out += _ld(num, _ld(1, str(v).encode()))
        elif kind == IOS:
            if isinstance(v, int):
                out += _ld(num, _key(1, 0) + _varint(0) + _key(2, 0) + _varint(v))
            else:
                out += _ld(num, _key(1, 0) + _varint(1) + _key(2, 0) + _varint(0) + _ld(3, str(v).encode()))
        elif kind == RS:
            for x in v:
                out += _ld(num, str(x).encode())
        elif kind == RI64:
            for x in v:
                out += _key(num, 0) + _varint(int(x))
        elif kind == RM:
            for x in v:
                out += _ld(num, encode_message(typ, x))
        elif kind == MAPS:
            for k in sorted(v):
                out += _ld(num, _ld(1, k.encode()) + _ld(2, str(v[k]).encode()))
        elif kind == MAPM:
            for k in sorted(v):
                if typ == "Quantity":
                    val = _ld(1, str(v[k]).encode())
                else:
                    val = encode_message(typ, v[k])
                out += _ld(num, _ld(1, k.encode()) + _ld(2, val))
    return bytes(out)


def _fields(buf):
    i = 0
    n = len(buf)
    while i < n:
        k, i = _read_varint(buf, i)
        num, wt = k >> 3, k & 7
        if wt == 0:
            v, i = _read_varint(buf, i)
        elif wt == 2:
            ln, i = _read_varint(buf, i)
            v = buf[i:i + ln]
            if len(v) != ln:
                raise ProtobufError("truncated field")
            i += ln
        elif wt == 5:
            v = buf[i:i + 4]
            i += 4
        elif wt == 1:
            v = buf[i:i + 8]
            i += 8
        else:
            raise ProtobufError(f"unsupported wire type {wt}")
        yield num, wt, v


def _signed(v, bits=64):
    return v - (1 << 64) if v >= 1 << 63 else v


def decode_message(msg: str, buf: bytes, out=None) -> dict:
    out = {} if out is None else out
    byn = _BY_NUM[msg]
    for num, wt, v in _fields(buf):
        f = byn.get(num)
        if f is None:
            continue  # unknown field: skipped (forward compatible)
        name, _, kind, typ = f
        if kind == INL:
            decode_message(typ, v, out)
        elif kind == S:
            out[name] = bytes(v).decode()
        elif kind == B:
            out[name] = bool(v)
        elif kind in (I64, I32):
            out[name] = _signed(v)
        elif kind == MSG:
            out[name] = decode_message(typ, v)
        elif kind == TIME:
            sec = nanos = 0
            for n2, _, x in _fields(v):
                if n2 == 1:
                    sec = _signed(x)
                elif n2 == 2:
                    nanos = x
            out[name] = _fmt_time(sec, nanos)
        elif kind == QTY:
            out[name] = next((bytes(x).decode() for n2, _, x in _fields(v) if n2 == 1), "0")
        elif kind == IOS:
            t = iv = 0
            sv = ""
            for n2, _, x in _fields(v):
                if n2 == 1:
                    t = x
                elif n2 == 2:
                    iv = _signed(x)
                elif n2 == 3:
                    sv = bytes(x).decode()
            out[name] = iv if t == 0 else sv
        elif kind == RS:
            out.setdefault(name, []).append(bytes(v).decode())
        elif kind == RI64:
            out.setdefault(name, []).append(_signed(v))
        elif kind == RM:
            out.setdefault(name, []).append(decode_message(typ, v))
        elif kind in (MAPS, MAPM):
            k = val = None
            for n2, _, x in _fields(v):
                if n2 == 1:
                    k = bytes(x).decode()
                elif n2 == 2:
                    val = x
            m = out.setdefault(name, {})
            if kind == MAPS:
                m[k] = bytes(val or b"").decode()
            elif typ == "Quantity":
                m[k] = next((bytes(x).decode() for n2, _, x in _fields(val or b"") if n2 == 1), "0")
            else:
                m[k] = decode_message(typ, val or b"")
    return out


# ---------------------------------------------------------------------------
def encode_unknown(api_version: str, kind: str, raw: bytes) -> bytes:
    tm = _ld(1, api_version.encode()) + _ld(2, kind.encode())
    return MAGIC + _ld(1, tm) + _ld(2, raw) + _ld(3, b"") + _ld(4, b"")


def decode_unknown(data: bytes):
    if data[:4] != MAGIC:
        raise ProtobufError("missing k8s protobuf magic")
    api_version = kind = ""
    raw = b""
    for num, _, v in _fields(data[4:]):
        if num == 1:
            for n2, _, x in _fields(v):
                if n2 == 1:
                    api_version = bytes(x).decode()
                elif n2 == 2:
                    kind = bytes(x).decode()
        elif num == 2:
            raw = bytes(v)
    return api_version, kind, raw


def encode_object(obj: dict) -> bytes:
    kind = obj.get("kind", "")
    msg = KIND_MESSAGE.get(kind)
    if msg is None:
        raise ProtobufError(f"no protobuf schema for kind {kind!r}")
    body = {k: v for k, v in obj.items() if k not in ("kind", "apiVersion")}
    return encode_unknown(obj.get("apiVersion", "v1"), kind, encode_message(msg, body))


def decode_object(data: bytes) -> dict:
    api_version, kind, raw = decode_unknown(data)
    msg = KIND_MESSAGE.get(kind)
    if msg is None:
        raise ProtobufError(f"no protobuf schema for kind {kind!r}")
    out = {"kind": kind, "apiVersion": api_version}
    out.update(decode_message(msg, raw))
    return out


def supported(kind: str) -> bool:
    return kind in KIND_MESSAGE


# storage codec hooks (codec.StorageCodec)
def encode_storage(obj):
    if supported(obj.get("kind", "")):
        return encode_object(obj)
    from .codec import dumpb
    return dumpb(obj)


def decode_storage(data):
    return decode_object(data)
