"""kubectl output printers: human tables, describe, json/yaml/name/jsonpath/custom-columns.

Parity: `pkg/printers` (table handlers per kind, `-o wide`, describe). Fork gap closed
(SURVEY §7.4 item 5): pods show their assigned GPUs and nodes their device inventory with
health and MI355X attributes.
"""
from __future__ import annotations

import json
import re
import time

import yaml

from ..api import core
from ..api.meta import parse_rfc3339


def age(ts):
    t = parse_rfc3339(ts)
    if t is None:
        return "<unknown>"
    d = max(0, int(time.time() - t))
    if d < 120:
        return f"{d}s"
    if d < 7200:
        return f"{d // 60}m"
    if d < 172800:
        return f"{d // 3600}h"
    return f"{d // 86400}d"


def pod_status_and_restarts(p):
    """`printPod` (pkg/printers/internalversion/printers.go): the STATUS column — Init:i/n,
    Init:<reason>, Init:ExitCode:n while initializing; otherwise the last container's waiting
    or terminated reason (ExitCode:n / Signal:n without one), Completed shown as Running while a
    container still runs; Terminating (Unknown for a pod on an unreachable node) once deleted —
    and the RESTARTS count of the containers it looked at."""
    st = p.get("status") or {}
    spec = p.get("spec") or {}
    reason = st.get("reason") or st.get("phase") or "Unknown"
    restarts = 0
    initializing = False
    n_init = len(spec.get("initContainers") or ())
    for i, c in enumerate(st.get("initContainerStatuses") or ()):
        restarts += int(c.get("restartCount", 0))
        s = c.get("state") or {}
        term, wait = s.get("terminated"), s.get("waiting")
        if term is not None and term.get("exitCode", 0) == 0:
            continue
        if term is not None:
            if not term.get("reason"):
                reason = f"Init:Signal:{term['signal']}" if term.get("signal") else f"Init:ExitCode:{term.get('exitCode', 0)}"
            else:
                reason = "Init:" + term["reason"]
        elif wait is not None and wait.get("reason") and wait["reason"] != "PodInitializing":
            reason = "Init:" + wait["reason"]
        else:
            reason = f"Init:{i}/{n_init}"
        initializing = True
        break
    if not initializing:
        restarts = 0
        has_running = False
        for c in reversed(st.get("containerStatuses") or ()):
            restarts += int(c.get("restartCount", 0))
            s = c.get("state") or {}
            term, wait = s.get("terminated"), s.get("waiting")
            if wait is not None and wait.get("reason"):
                reason = wait["reason"]
            elif term is not None and term.get("reason"):
                reason = term["reason"]
            elif term is not None:
                reason = f"Signal:{term['signal']}" if term.get("signal") else f"ExitCode:{term.get('exitCode', 0)}"
            elif c.get("ready") and s.get("running") is not None:
                has_running = True
        if reason == "Completed" and has_running:
            reason = "Running"
    if p["metadata"].get("deletionTimestamp"):
        reason = "Unknown" if st.get("reason") == "NodeLost" else "Terminating"
    return reason, restarts


def pod_status(p):
    return pod_status_and_restarts(p)[0]


def pod_gpus(p):
    return [i for per in (p.get("spec") or {}).get("extendedResources") or () for i in per.get("assigned") or ()]


def table(rows, headers):
    rows = [[str(c) for c in r] for r in rows]
    widths = [max([len(h)] + [len(r[i]) for r in rows]) for i, h in enumerate(headers)]
    out = ["   ".join(h.ljust(w) for h, w in zip(headers, widths)).rstrip()]
    for r in rows:
        out.append("   ".join(c.ljust(w) for c, w in zip(r, widths)).rstrip())
    return "\n".join(out)


def _g(o, *path, default=None):
    for k in path:
        o = (o or {}).get(k) if isinstance(o, dict) else None
    return default if o is None else o


def _svc_external(o):
    spec = o.get("spec") or {}
    ips = list(spec.get("externalIPs") or ())
    if spec.get("type") == "LoadBalancer":
        ing = [i.get("ip") or i.get("hostname") for i in _g(o, "status", "loadBalancer", "ingress", default=[])]
        ips = ing + ips if ing else (ips or ["<pending>"])
    elif spec.get("type") == "ExternalName":
        return spec.get("externalName", "")
    return ",".join(ips) or "<none>"


def _svc_ports(o):
    out = []
    for p in _g(o, "spec", "ports", default=[]):
        s = str(p.get("port"))
        if p.get("nodePort"):
            s += f":{p['nodePort']}"
        out.append(f"{s}/{p.get('protocol', 'TCP')}")
    return ",".join(out) or "<none>"


def _endpoints(o):
    addrs = []
    for ss in o.get("subsets") or ():
        ports = [p.get("port") for p in ss.get("ports") or ()] or [None]
        for a in ss.get("addresses") or ():
            for port in ports:
                addrs.append(a.get("ip") + (f":{port}" if port is not None else ""))
    if not addrs:
        return "<none>"
    shown = ",".join(addrs[:3])
    return shown + (f" + {len(addrs) - 3} more..." if len(addrs) > 3 else "")


def _modes(modes):
    short = {"ReadWriteOnce": "RWO", "ReadOnlyMany": "ROX", "ReadWriteMany": "RWX"}
    return ",".join(short.get(m, m) for m in modes or ())


def _hpa_targets(o):
    st, spec = o.get("status") or {}, o.get("spec") or {}
    want = spec.get("targetCPUUtilizationPercentage")
    cur = st.get("currentCPUUtilizationPercentage")
    if want is None:
        return "<none>"
    return f"{'<unknown>' if cur is None else f'{cur}%'}/{want}%"


def _csr_condition(o):
    conds = [c.get("type") for c in _g(o, "status", "conditions", default=[])]
    if _g(o, "status", "certificate") and "Approved" in conds:
        conds.append("Issued")
    return ",".join(conds) or "Pending"


def _pdb_val(v):
    return "N/A" if v is None else str(v)


# `pkg/printers/internalversion/printers.go` column sets (NAME first, AGE last)
_COLUMNS = {
    "Service": (["NAME", "TYPE", "CLUSTER-IP", "EXTERNAL-IP", "PORT(S)", "AGE"],
                lambda o: [_g(o, "spec", "type", default="ClusterIP"), _g(o, "spec", "clusterIP", default="<none>") or "<none>",
                           _svc_external(o), _svc_ports(o)]),
    "Endpoints": (["NAME", "ENDPOINTS", "AGE"], lambda o: [_endpoints(o)]),
    "ServiceAccount": (["NAME", "SECRETS", "AGE"], lambda o: [len(o.get("secrets") or ())]),
    "Secret": (["NAME", "TYPE", "DATA", "AGE"], lambda o: [o.get("type", "Opaque"), len(o.get("data") or {})]),
    "ConfigMap": (["NAME", "DATA", "AGE"], lambda o: [len(o.get("data") or {}) + len(o.get("binaryData") or {})]),
    "DaemonSet": (["NAME", "DESIRED", "CURRENT", "READY", "UP-TO-DATE", "AVAILABLE", "NODE SELECTOR", "AGE"],
                  lambda o: [_g(o, "status", "desiredNumberScheduled", default=0), _g(o, "status", "currentNumberScheduled", default=0),
                             _g(o, "status", "numberReady", default=0), _g(o, "status", "updatedNumberScheduled", default=0),
                             _g(o, "status", "numberAvailable", default=0),
                             ",".join(f"{k}={v}" for k, v in sorted(_g(o, "spec", "template", "spec", "nodeSelector", default={}).items()))
                             or "<none>"]),
    "StatefulSet": (["NAME", "DESIRED", "CURRENT", "AGE"],
                    lambda o: [_g(o, "spec", "replicas", default=1), _g(o, "status", "replicas", default=0)]),
    "CronJob": (["NAME", "SCHEDULE", "SUSPEND", "ACTIVE", "LAST SCHEDULE", "AGE"],
                lambda o: [_g(o, "spec", "schedule", default=""), str(bool(_g(o, "spec", "suspend", default=False))),
                           len(_g(o, "status", "active", default=[])),
                           age(_g(o, "status", "lastScheduleTime")) if _g(o, "status", "lastScheduleTime") else "<none>"]),
    "HorizontalPodAutoscaler": (["NAME", "REFERENCE", "TARGETS", "MINPODS", "MAXPODS", "REPLICAS", "AGE"],
                                lambda o: [f"{_g(o, 'spec', 'scaleTargetRef', 'kind', default='')}/{_g(o, 'spec', 'scaleTargetRef', 'name', default='')}",
                                           _hpa_targets(o), _g(o, "spec", "minReplicas", default=1),
                                           _g(o, "spec", "maxReplicas", default=0), _g(o, "status", "currentReplicas", default=0)]),
    "PodDisruptionBudget": (["NAME", "MIN AVAILABLE", "MAX UNAVAILABLE", "ALLOWED DISRUPTIONS", "AGE"],
                            lambda o: [_pdb_val(_g(o, "spec", "minAvailable")), _pdb_val(_g(o, "spec", "maxUnavailable")),
                                       _g(o, "status", "disruptionsAllowed", default=0)]),
    "PersistentVolume": (["NAME", "CAPACITY", "ACCESS MODES", "RECLAIM POLICY", "STATUS", "CLAIM", "STORAGECLASS", "REASON", "AGE"],
                         lambda o: [_g(o, "spec", "capacity", "storage", default=""), _modes(_g(o, "spec", "accessModes")),
                                    _g(o, "spec", "persistentVolumeReclaimPolicy", default="Retain"),
                                    _g(o, "status", "phase", default=""),
                                    (f"{_g(o, 'spec', 'claimRef', 'namespace')}/{_g(o, 'spec', 'claimRef', 'name')}"
                                     if _g(o, "spec", "claimRef") else ""),
                                    _g(o, "spec", "storageClassName", default=""), _g(o, "status", "reason", default="")]),
    "PersistentVolumeClaim": (["NAME", "STATUS", "VOLUME", "CAPACITY", "ACCESS MODES", "STORAGECLASS", "AGE"],
                              lambda o: [_g(o, "status", "phase", default=""), _g(o, "spec", "volumeName", default=""),
                                         _g(o, "status", "capacity", "storage", default=""),
                                         _modes(_g(o, "status", "accessModes")), _g(o, "spec", "storageClassName", default="")]),
    "StorageClass": (["NAME", "PROVISIONER", "AGE"],
                     lambda o: [o.get("provisioner", "")]),
    "CertificateSigningRequest": (["NAME", "REQUESTOR", "CONDITION", "AGE"],
                                  lambda o: [_g(o, "spec", "username", default=""), _csr_condition(o)]),
    "Ingress": (["NAME", "HOSTS", "ADDRESS", "PORTS", "AGE"],
                lambda o: [",".join(r.get("host", "") for r in _g(o, "spec", "rules", default=[]) if r.get("host")) or "*",
                           ",".join(i.get("ip", "") for i in _g(o, "status", "loadBalancer", "ingress", default=[])),
                           "80, 443" if _g(o, "spec", "tls") else "80"]),
    "PriorityClass": (["NAME", "VALUE", "GLOBAL-DEFAULT", "AGE"],
                      lambda o: [o.get("value", 0), str(bool(o.get("globalDefault", False))).lower()]),
}
_CLUSTER_SCOPED = {"Node", "Namespace", "PersistentVolume", "StorageClass", "CertificateSigningRequest", "PriorityClass",
                   "ClusterRole", "ClusterRoleBinding", "PodSecurityPolicy", "CustomResourceDefinition", "APIService"}


def rows_for(kind, items, wide=False, all_ns=False):
    if kind == "Pod":
        h = ["NAME", "READY", "STATUS", "RESTARTS", "AGE"]
        if wide:
            h += ["IP", "NODE", "GPUS"]
        rows = []
        for p in items:
            cs = (p.get("status") or {}).get("containerStatuses") or []
            n = len((p.get("spec") or {}).get("containers") or [])
            status, restarts = pod_status_and_restarts(p)
            r = [p["metadata"]["name"], f"{sum(1 for c in cs if c.get('ready'))}/{n}", status,
                 restarts, age(p["metadata"].get("creationTimestamp"))]
            if wide:
                g = pod_gpus(p)
                r += [(p.get("status") or {}).get("podIP", "<none>"), (p.get("spec") or {}).get("nodeName") or "<none>",
                      ",".join(x[-8:] for x in g) or "<none>"]
            rows.append(r)
    elif kind == "Node":
        h = ["NAME", "STATUS", "ROLES", "AGE", "VERSION", "GPU"]
        if wide:
            h += ["INTERNAL-IP", "GPU-PRODUCT", "ARCH", "HBM"]
        rows = []
        for n in items:
            ready = core.get_condition(n.get("status"), "Ready")
            s = "Ready" if ready and ready.get("status") == "True" else "NotReady"
            if (n.get("spec") or {}).get("unschedulable"):
                s += ",SchedulingDisabled"
            cap = (n.get("status") or {}).get("capacity") or {}
            devs = ((n.get("status") or {}).get("extendedResources") or {}).get(core.AMD_GPU, {}).get("resources") or {}
            # `findNodeRoles`: node-role.kubernetes.io/<role> labels and the kubernetes.io/role label
            labels = n["metadata"].get("labels") or {}
            roles = sorted({k.split("/", 1)[1] for k in labels if k.startswith("node-role.kubernetes.io/") and "/" in k}
                           | ({labels["kubernetes.io/role"]} if labels.get("kubernetes.io/role") else set()))
            r = [n["metadata"]["name"], s, ",".join(r_ for r_ in roles if r_) or "<none>", age(n["metadata"].get("creationTimestamp")),
                 ((n.get("status") or {}).get("nodeInfo") or {}).get("kubeletVersion", ""),
                 f"{cap.get(core.AMD_GPU, '0')}/{len(devs)}"]
            if wide:
                attrs = next(iter(devs.values()), {}).get("attributes", {}) if devs else {}
                ip = next((a["address"] for a in (n.get("status") or {}).get("addresses") or () if a.get("type") == "InternalIP"), "")
                r += [ip, attrs.get(core.ATTR_PRODUCT, "<none>"), attrs.get(core.ATTR_ARCH, "<none>"), attrs.get(core.ATTR_HBM, "<none>")]
            rows.append(r)
    elif kind in ("ReplicaSet", "ReplicationController"):
        h = ["NAME", "DESIRED", "CURRENT", "READY", "AGE"]
        rows = [[o["metadata"]["name"], (o.get("spec") or {}).get("replicas", 1), (o.get("status") or {}).get("replicas", 0),
                 (o.get("status") or {}).get("readyReplicas", 0), age(o["metadata"].get("creationTimestamp"))] for o in items]
    elif kind == "Deployment":
        h = ["NAME", "DESIRED", "CURRENT", "UP-TO-DATE", "AVAILABLE", "AGE"]
        rows = [[o["metadata"]["name"], (o.get("spec") or {}).get("replicas", 1), (o.get("status") or {}).get("replicas", 0),
                 (o.get("status") or {}).get("updatedReplicas", 0), (o.get("status") or {}).get("availableReplicas", 0),
                 age(o["metadata"].get("creationTimestamp"))] for o in items]
    elif kind == "Job":
        h = ["NAME", "DESIRED", "SUCCESSFUL", "AGE"]
        rows = [[o["metadata"]["name"], (o.get("spec") or {}).get("completions", 1), (o.get("status") or {}).get("succeeded", 0),
                 age(o["metadata"].get("creationTimestamp"))] for o in items]
    elif kind == "Event":
        # kubectl 1.9 `printEvent` columns
        h = ["LAST SEEN", "FIRST SEEN", "COUNT", "NAME", "KIND", "SUBOBJECT", "TYPE", "REASON", "SOURCE", "MESSAGE"]
        rows = []
        for o in items:
            io, src = o.get("involvedObject") or {}, o.get("source") or {}
            rows.append([age(o.get("lastTimestamp")), age(o.get("firstTimestamp")), o.get("count", 1), io.get("name", ""),
                         io.get("kind", ""), io.get("fieldPath", ""), o.get("type", ""), o.get("reason", ""),
                         ", ".join(x for x in (src.get("component", ""), src.get("host", "")) if x),
                         o.get("message", "")])
    elif kind == "Namespace":
        h = ["NAME", "STATUS", "AGE"]
        rows = [[o["metadata"]["name"], (o.get("status") or {}).get("phase", ""), age(o["metadata"].get("creationTimestamp"))] for o in items]
    elif kind in _COLUMNS:
        h, fn = _COLUMNS[kind]
        h = list(h)
        rows = [[o["metadata"]["name"]] + fn(o) + [age(o["metadata"].get("creationTimestamp"))] for o in items]
        if wide and kind == "Service":
            h.append("SELECTOR")
            for o, r in zip(items, rows):
                sel = (o.get("spec") or {}).get("selector") or {}
                r.append(",".join(f"{k}={v}" for k, v in sorted(sel.items())) or "<none>")
    else:
        h = ["NAME", "AGE"]
        rows = [[o["metadata"]["name"], age(o["metadata"].get("creationTimestamp"))] for o in items]
    if all_ns and kind not in _CLUSTER_SCOPED:
        h = ["NAMESPACE"] + h
        rows = [[o["metadata"].get("namespace", "")] + r for o, r in zip(items, rows)]
    return rows, h


def jsonpath(obj, expr):
    """A useful subset of kubectl jsonpath: {.a.b[0].c}, {.items[*].metadata.name}, literal text."""
    def ev(path, cur):
        toks = re.findall(r"\.([^.\[\]]+)|\[(\*|\d+)\]", path)
        vals = [cur]
        for name, idx in toks:
            nxt = []
            for v in vals:
                if name:
                    if isinstance(v, dict) and name in v:
                        nxt.append(v[name])
                elif idx == "*":
                    if isinstance(v, list):
                        nxt.extend(v)
                else:
                    if isinstance(v, list) and int(idx) < len(v):
                        nxt.append(v[int(idx)])
            vals = nxt
        return vals

    out = []
    for lit, path in re.findall(r"([^{]*)(?:\{([^}]*)\})?", expr):
        out.append(lit)
        if path:
            vals = ev(path, obj)
            out.append(" ".join(json.dumps(v) if isinstance(v, (dict, list)) else str(v) for v in vals))
    return "".join(out)


def render(objs, output, kind=None, wide=False, all_ns=False, list_obj=None, sort_by="", no_headers=False,
           show_labels=False, label_columns=(), show_kind=False):
    """Objects in `-o` form. Table options (`pkg/printers/humanreadable.go` PrintOptions):
    --sort-by (JSONPath; numbers and quantities compare as numbers), --no-headers,
    --show-labels, -L label columns, --show-kind (kind/name)."""
    if sort_by:
        objs = sort_objects(objs, sort_by)
        if list_obj is not None:
            list_obj = dict(list_obj, items=objs)
    if output == "json":
        return json.dumps(list_obj if list_obj is not None else (objs[0] if len(objs) == 1 else {"kind": "List", "apiVersion": "v1", "items": objs}), indent=4)
    if output == "yaml":
        return yaml.safe_dump(list_obj if list_obj is not None else (objs[0] if len(objs) == 1 else {"kind": "List", "apiVersion": "v1", "items": objs}), sort_keys=False).rstrip()
    if output == "name":
        return "\n".join(f"{(o.get('kind') or kind or '').lower()}/{o['metadata']['name']}" for o in objs)
    for pre in ("jsonpath-file=", "custom-columns-file=", "go-template-file=", "templatefile="):
        if output and output.startswith(pre):
            with open(output[len(pre):]) as f:
                body = f.read()
            if pre == "custom-columns-file=":
                # a header line of names and a line of JSONPath specs (`customcolumn.go`)
                lines = [ln.split() for ln in body.splitlines() if ln.strip()]
                if len(lines) != 2 or len(lines[0]) != len(lines[1]):
                    raise SystemExit("error: custom-columns-file needs a header line and a spec line of equal width")
                output = "custom-columns=" + ",".join(f"{h}:{p}" for h, p in zip(*lines))
            else:
                output = {"jsonpath-file=": "jsonpath=", "go-template-file=": "go-template=",
                          "templatefile=": "go-template="}[pre] + body
            break
    if output and output.startswith(("go-template=", "template=")):
        from .gotemplate import TemplateError
        from .gotemplate import render as gotemplate
        target = list_obj if list_obj is not None else (objs[0] if len(objs) == 1 else
                                                         {"kind": "List", "apiVersion": "v1", "items": objs})
        try:
            return gotemplate(output.split("=", 1)[1], target)
        except TemplateError as e:
            raise SystemExit(f"error: error executing template {output.split('=', 1)[1]!r}: {e}")
    if output and output.startswith("jsonpath="):
        target = list_obj if list_obj is not None else (objs[0] if len(objs) == 1 else {"items": objs})
        return jsonpath(target, output[len("jsonpath="):])
    if output and output.startswith("custom-columns="):
        cols = [c.split(":", 1) for c in output[len("custom-columns="):].split(",")]
        rows = [[jsonpath(o, "{" + p + "}") or "<none>" for _, p in cols] for o in objs]
        return table(rows, [h for h, _ in cols])
    if not objs:
        return "No resources found."
    rows, h = rows_for(kind or objs[0].get("kind"), objs, wide or output == "wide", all_ns)
    name_col = h.index("NAME") if "NAME" in h else None
    if show_kind and name_col is not None:
        k = (kind or objs[0].get("kind") or "").lower()
        rows = [r[:name_col] + [f"{k}/{r[name_col]}"] + r[name_col + 1:] for r in rows]
    cols = []
    for spec in label_columns or ():
        cols += [c for c in spec.split(",") if c]
    if cols:
        h = h + [c.rsplit("/", 1)[-1].upper() for c in cols]
        rows = [list(r) + [((o.get("metadata") or {}).get("labels") or {}).get(c, "") for c in cols]
                for r, o in zip(rows, objs)]
    if show_labels:
        h = h + ["LABELS"]
        rows = [list(r) + [",".join(f"{k}={v}" for k, v in sorted(((o.get("metadata") or {}).get("labels") or {}).items()))
                           or "<none>"] for r, o in zip(rows, objs)]
    text = table(rows, h)
    if no_headers:
        text = "\n".join(text.splitlines()[1:])
    return text


def sort_objects(objs, expr):
    from ..api.quantity import parse_quantity
    path = expr if expr.startswith("{") else "{" + expr + "}"

    def key(o):
        v = jsonpath(o, path)
        try:
            return (0, float(v), "")
        except (TypeError, ValueError):
            pass
        try:
            return (0, float(parse_quantity(str(v)).milli_value()) / 1000.0, "")
        except (ValueError, AttributeError):
            return (1, 0.0, str(v))
    return sorted(objs, key=key)


def describe(obj, events=(), ctx=None):
    """`kubectl describe` text; `ctx` carries related objects from `describe.gather()`."""
    from . import describe as dsc
    kind = obj.get("kind")
    md = obj["metadata"]
    lines = [f"Name:         {md['name']}"]
    if md.get("namespace"):
        lines.append(f"Namespace:    {md['namespace']}")
    lines.append(f"Labels:       {', '.join(f'{k}={v}' for k, v in (md.get('labels') or {}).items()) or '<none>'}")
    lines.append(f"Annotations:  {', '.join(f'{k}={v}' for k, v in (md.get('annotations') or {}).items()) or '<none>'}")
    lines.append(f"CreationTimestamp: {md.get('creationTimestamp')}")
    if kind == "Pod":
        spec, st = obj.get("spec") or {}, obj.get("status") or {}
        # `describePod`: the phase (Terminating once deleted), then Reason / Message when set
        phase = "Terminating" if md.get("deletionTimestamp") else st.get("phase", "")
        lines += [f"Node:         {spec.get('nodeName') or '<none>'}", f"Status:       {phase}"]
        if st.get("reason"):
            lines.append(f"Reason:       {st['reason']}")
        if st.get("message"):
            lines.append(f"Message:      {st['message']}")
        lines += [f"IP:           {st.get('podIP', '')}", f"QoS Class:    {st.get('qosClass', '')}"]
        ers = spec.get("extendedResources") or []
        if ers:
            lines.append("Extended Resources:")
            for per in ers:
                lim = (per.get("resources") or {}).get("limits") or {}
                lines.append(f"  {per.get('name')}:")
                lines.append(f"    Request:   {', '.join(f'{k}={v}' for k, v in lim.items())}")
                req = (per.get("affinity") or {}).get("required") or []
                if req:
                    lines.append("    Affinity:  " + "; ".join(f"{r.get('key')} {r.get('operator')} {','.join(r.get('values') or [])}" for r in req))
                lines.append(f"    Assigned:  {', '.join(per.get('assigned') or []) or '<pending>'}")
        lines.append("Containers:")
        cstat = {c["name"]: c for c in st.get("containerStatuses") or ()}
        for c in spec.get("containers") or ():
            lines.append(f"  {c['name']}:")
            lines.append(f"    Image:   {c.get('image')}")
            s = cstat.get(c["name"], {})
            if s:
                state = next(iter((s.get("state") or {}).keys()), "unknown")
                lines.append(f"    State:   {state.capitalize()}")
                lines.append(f"    Ready:   {s.get('ready')}")
                lines.append(f"    Restart Count: {s.get('restartCount', 0)}")
            if c.get("extendedResourceRequests"):
                lines.append(f"    Extended Resource Requests: {', '.join(c['extendedResourceRequests'])}")
        lines.append("Conditions:")
        for cd in st.get("conditions") or ():
            lines.append(f"  {cd.get('type'):<16} {cd.get('status')}")
        lines += dsc.pod_extra(obj, ctx or {})
    elif kind == "Node":
        st = obj.get("status") or {}
        lines.append("Conditions:")
        for cd in st.get("conditions") or ():
            lines.append(f"  {cd.get('type'):<16} {cd.get('status'):<8} {cd.get('reason', '')}")
        lines.append("Capacity:")
        for k, v in (st.get("capacity") or {}).items():
            lines.append(f"  {k}: {v}")
        lines.append("Allocatable:")
        for k, v in (st.get("allocatable") or {}).items():
            lines.append(f"  {k}: {v}")
        for rn, dom in (st.get("extendedResources") or {}).items():
            lines.append(f"Extended Resources ({rn}):")
            for did, d in sorted(((dom or {}).get("resources") or {}).items(), key=lambda kv: kv[1].get("attributes", {}).get(core.ATTR_INDEX, "")):
                a = d.get("attributes") or {}
                extra = ""
                if a.get(core.ATTR_PARTITION, "SPX") != "SPX":
                    extra += (f" partition={a.get(core.ATTR_PARTITION)}/{a.get(core.ATTR_PARTITION_ID, '?')}"
                              f"@socket{a.get(core.ATTR_SOCKET, '?')}")
                if a.get("amd.com/burn-in"):
                    extra += f" burn-in={a['amd.com/burn-in']}"
                    if a.get("amd.com/mfma-tflops"):
                        extra += (f" (bf16 {a['amd.com/mfma-tflops']} / fp8 {a.get('amd.com/mfma-fp8-tflops', '-')} TF/s,"
                                  f" HBM {a.get('amd.com/hbm-gbps', '-')} GB/s)")
                lines.append(f"  {did}  {d.get('health')}  {a.get(core.ATTR_PRODUCT, '')} {a.get(core.ATTR_ARCH, '')} "
                             f"hbm={a.get(core.ATTR_HBM, '')} hive={a.get(core.ATTR_HIVE, '')} numa={a.get(core.ATTR_NUMA, '')} "
                             f"render=renderD{a.get(core.ATTR_RENDER_MINOR, '?')}{extra}")
        taints = (obj.get("spec") or {}).get("taints") or []
        lines.append(f"Taints:       {', '.join(t['key'] + ':' + t['effect'] for t in taints) or '<none>'}")
        lines.append(f"Unschedulable: {bool((obj.get('spec') or {}).get('unschedulable'))}")
        lines += dsc.node_extra(obj, ctx or {})
    else:
        extra = dsc.sections(obj, ctx)
        lines += extra if extra is not None else dsc.fallback(obj)
    if events:
        # `DescribeEvents`: Type, Reason, Age, From, Message
        lines.append("Events:")
        rows = [[e.get("type", ""), e.get("reason", ""), age(e.get("lastTimestamp")),
                 ", ".join(x for x in ((e.get("source") or {}).get("component", ""), (e.get("source") or {}).get("host", "")) if x),
                 e.get("message", "")] for e in events]
        lines += ["  " + ln for ln in table(rows, ["Type", "Reason", "Age", "From", "Message"]).splitlines()]
    else:
        lines.append("Events:       <none>")
    return "\n".join(lines)
