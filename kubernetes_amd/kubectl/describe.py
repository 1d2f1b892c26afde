"""Per-kind `kubectl describe` sections.

Parity: `pkg/printers/internalversion/describe.go` — DeploymentDescriber (replicas summary,
strategy, pod template, conditions, old/new ReplicaSets), ReplicaSet / ReplicationController /
Job / DaemonSet / StatefulSet (selector, desired vs current, pods status by phase), Service
(type, IP, ports with target and node ports, endpoints, session affinity), Secret (data sizes
only — values are never printed), ConfigMap (data), Namespace (status, resource quotas and
limit ranges), ServiceAccount (mountable secrets, tokens, image pull secrets), PV / PVC,
HorizontalPodAutoscaler, Endpoints, CronJob; and the extra Pod (container ports, limits /
requests, env, mounts, volumes, node selectors, tolerations) and Node (addresses, system info,
non-terminated pods, allocated resources) sections.

`gather()` fetches what a describer needs beyond the object itself (owned pods, ReplicaSets,
endpoints, quotas, pods on a node); `sections()` renders without I/O.
"""
from __future__ import annotations

import yaml

from ..api import core
from ..api import meta as m
from ..api.quantity import QuantityError, parse_quantity

_MODES = {"ReadWriteOnce": "RWO", "ReadOnlyMany": "ROX", "ReadWriteMany": "RWX"}


def _q(v) -> float:
    try:
        return float(parse_quantity(str(v)))
    except QuantityError:
        return 0.0


def _kv(d):
    return ",".join(f"{k}={v}" for k, v in sorted((d or {}).items())) or "<none>"


def _selector(sel):
    if not sel:
        return "<none>"
    if "matchLabels" in sel or "matchExpressions" in sel:
        parts = [f"{k}={v}" for k, v in sorted((sel.get("matchLabels") or {}).items())]
        for e in sel.get("matchExpressions") or ():
            op = e.get("operator")
            if op in ("In", "NotIn"):
                parts.append(f"{e['key']} {op.lower()} ({','.join(e.get('values') or ())})")
            else:
                parts.append(e["key"] if op == "Exists" else "!" + e["key"])
        return ",".join(parts) or "<none>"
    return _kv(sel)


async def _owned_pods(client, obj, sel):
    ns = obj["metadata"].get("namespace")
    try:
        pods = (await client.list("pods", ns, sel))["items"]
    except Exception:        # noqa: BLE001 - describe degrades to the object alone
        return []
    uid = obj["metadata"].get("uid")
    return [p for p in pods if not uid or (m.controller_of(p) or {}).get("uid") in (uid, None)]


async def gather(client, obj) -> dict:
    kind, md = obj.get("kind"), obj["metadata"]
    ns = md.get("namespace")
    spec = obj.get("spec") or {}
    ctx = {}
    try:
        if kind in ("ReplicaSet", "ReplicationController", "Job", "DaemonSet", "StatefulSet"):
            sel = spec.get("selector") or {}
            labels = sel.get("matchLabels", {}) if "matchLabels" in sel or "matchExpressions" in sel else sel
            ctx["pods"] = await _owned_pods(client, obj, _kv(labels) if labels and "matchExpressions" not in sel else None)
        elif kind == "Deployment":
            rss = (await client.list("replicasets", ns))["items"]
            ctx["replicasets"] = [r for r in rss if (m.controller_of(r) or {}).get("uid") == md.get("uid")]
        elif kind == "Service":
            try:
                ctx["endpoints"] = await client.get("endpoints", md["name"], ns)
            except Exception:    # noqa: BLE001
                ctx["endpoints"] = None
        elif kind == "Node":
            ctx["pods"] = [p for p in (await client.list("pods", None, field_selector=f"spec.nodeName={md['name']}"))["items"]
                           if not core.pod_is_terminal(p)]
        elif kind == "Namespace":
            ctx["quotas"] = (await client.list("resourcequotas", md["name"]))["items"]
            ctx["limitranges"] = (await client.list("limitranges", md["name"]))["items"]
    except Exception:            # noqa: BLE001 - RBAC may hide related objects
        pass
    return ctx


def _pods_status(pods):
    c = {"Running": 0, "Pending": 0, "Succeeded": 0, "Failed": 0}
    for p in pods:
        ph = (p.get("status") or {}).get("phase", "Pending")
        c[ph] = c.get(ph, 0) + 1
    return f"{c['Running']} Running / {c['Pending']} Waiting / {c['Succeeded']} Succeeded / {c['Failed']} Failed"


def _template(tpl, indent="  "):
    out = [f"{indent}Labels:  {_kv((tpl.get('metadata') or {}).get('labels'))}", f"{indent}Containers:"]
    for c in (tpl.get("spec") or {}).get("containers") or ():
        out += [indent + "  " + ln for ln in _container(c)]
    vols = (tpl.get("spec") or {}).get("volumes") or []
    out.append(f"{indent}Volumes:" + ("  <none>" if not vols else ""))
    out += [indent + "  " + ln for v in vols for ln in _volume(v)]
    return out


def _container(c, status=None):
    out = [f"{c['name']}:", f"  Image:      {c.get('image', '')}"]
    ports = c.get("ports") or []
    out.append("  Port:       " + (", ".join(f"{p['containerPort']}/{p.get('protocol', 'TCP')}" for p in ports) or "<none>"))
    hp = [p for p in ports if p.get("hostPort")]
    if hp:
        out.append("  Host Port:  " + ", ".join(f"{p['hostPort']}/{p.get('protocol', 'TCP')}" for p in hp))
    if c.get("command"):
        out.append("  Command:")
        out += ["    " + x for x in c["command"]]
    if c.get("args"):
        out.append("  Args:")
        out += ["    " + x for x in c["args"]]
    res = c.get("resources") or {}
    for k in ("limits", "requests"):
        if res.get(k):
            out.append(f"  {k.capitalize()}:")
            out += [f"    {rk}:  {rv}" for rk, rv in sorted(res[k].items())]
    env = c.get("env") or []
    out.append("  Environment:" + ("  <none>" if not env else ""))
    for e in env:
        if "value" in e:
            out.append(f"    {e['name']}:  {e['value']}")
        else:
            src = e.get("valueFrom") or {}
            ref = next(iter(src.items()), ("", {}))
            desc = ", ".join(f"{k}={v}" for k, v in sorted((ref[1] or {}).items()))
            out.append(f"    {e['name']}:  <set to {ref[0]} {desc}>")
    mounts = c.get("volumeMounts") or []
    out.append("  Mounts:" + ("  <none>" if not mounts else ""))
    out += [f"    {vm['mountPath']} from {vm['name']} ({'ro' if vm.get('readOnly') else 'rw'})" for vm in mounts]
    return out


def _volume(v):
    name = v.get("name")
    src = next(((k, s) for k, s in v.items() if k != "name"), ("", {}))
    out = [f"{name}:", f"  Type:  {src[0]}"]
    for k, val in sorted((src[1] or {}).items()):
        if not isinstance(val, (dict, list)):
            out.append(f"  {k[:1].upper() + k[1:]}:  {val}")
    return out


def _conditions(st, cols=("type", "status", "reason")):
    conds = (st or {}).get("conditions") or []
    if not conds:
        return []
    out = ["Conditions:", "  " + "  ".join(f"{c.capitalize():<14}" for c in cols).rstrip()]
    for cd in conds:
        out.append("  " + "  ".join(f"{str(cd.get(c, '')):<14}" for c in cols).rstrip())
    return out


def pod_extra(obj, ctx):
    spec = obj.get("spec") or {}
    out = ["Container Details:"]
    for c in spec.get("containers") or ():
        out += ["  " + ln for ln in _container(c)]
    vols = spec.get("volumes") or []
    out.append("Volumes:" + ("  <none>" if not vols else ""))
    out += ["  " + ln for v in vols for ln in _volume(v)]
    out.append(f"Node-Selectors:  {_kv(spec.get('nodeSelector'))}")
    tols = spec.get("tolerations") or []
    out.append("Tolerations:     " + (", ".join(
        f"{t.get('key', '')}{'=' + t['value'] if t.get('value') else ''}:{t.get('effect', '')}"
        + (f" for {t['tolerationSeconds']}s" if t.get("tolerationSeconds") is not None else "") for t in tols) or "<none>"))
    return out


def node_extra(obj, ctx):
    st = obj.get("status") or {}
    out = ["Addresses:"] + [f"  {a['type']}:  {a['address']}" for a in st.get("addresses") or ()]
    ni = st.get("nodeInfo") or {}
    if ni:
        out.append("System Info:")
        for k in ("machineID", "systemUUID", "bootID", "kernelVersion", "osImage", "containerRuntimeVersion",
                  "kubeletVersion", "kubeProxyVersion", "operatingSystem", "architecture"):
            if k in ni:
                out.append(f" {k[:1].upper() + k[1:]}:  {ni[k]}")
    if (obj.get("spec") or {}).get("podCIDR"):
        out.append(f"PodCIDR:      {obj['spec']['podCIDR']}")
    pods = ctx.get("pods")
    if pods is not None:
        alloc = st.get("allocatable") or {}
        out.append(f"Non-terminated Pods:  ({len(pods)} in total)")
        out.append("  Namespace  Name  CPU Requests  CPU Limits  Memory Requests  Memory Limits")
        tot = {"cr": 0.0, "cl": 0.0, "mr": 0.0, "ml": 0.0, "gpu": 0}
        for p in pods:
            cr = cl = 0.0
            mr = ml = 0.0
            for c in (p.get("spec") or {}).get("containers") or ():
                r = c.get("resources") or {}
                cr += _q((r.get("requests") or {}).get("cpu", "0"))
                cl += _q((r.get("limits") or {}).get("cpu", "0"))
                mr += _q((r.get("requests") or {}).get("memory", "0"))
                ml += _q((r.get("limits") or {}).get("memory", "0"))
                tot["gpu"] += int(_q((r.get("limits") or {}).get(core.AMD_GPU, "0")))
            for per in (p.get("spec") or {}).get("extendedResources") or ():
                tot["gpu"] += int(_q(((per.get("resources") or {}).get("limits") or {}).get(core.AMD_GPU, "0")))
            tot["cr"] += cr
            tot["cl"] += cl
            tot["mr"] += mr
            tot["ml"] += ml
            out.append(f"  {p['metadata'].get('namespace', '')}  {p['metadata']['name']}  {int(cr * 1000)}m  "
                       f"{int(cl * 1000)}m  {int(mr)}  {int(ml)}")
        acpu = _q(alloc.get("cpu", "0")) or 1
        amem = _q(alloc.get("memory", "0")) or 1
        out.append("Allocated resources:")
        out.append(f"  CPU Requests  {int(tot['cr'] * 1000)}m ({int(100 * tot['cr'] / acpu)}%)  "
                   f"CPU Limits  {int(tot['cl'] * 1000)}m ({int(100 * tot['cl'] / acpu)}%)")
        out.append(f"  Memory Requests  {int(tot['mr'])} ({int(100 * tot['mr'] / amem)}%)  "
                   f"Memory Limits  {int(tot['ml'])} ({int(100 * tot['ml'] / amem)}%)")
        if core.AMD_GPU in alloc:
            out.append(f"  {core.AMD_GPU}  {tot['gpu']}/{alloc[core.AMD_GPU]}")
    return out


def _deployment(obj, ctx):
    spec, st = obj.get("spec") or {}, obj.get("status") or {}
    strat = spec.get("strategy") or {}
    out = [f"Selector:               {_selector(spec.get('selector'))}",
           f"Replicas:               {spec.get('replicas', 1)} desired | {st.get('updatedReplicas', 0)} updated | "
           f"{st.get('replicas', 0)} total | {st.get('availableReplicas', 0)} available | "
           f"{st.get('unavailableReplicas', 0)} unavailable",
           f"StrategyType:           {strat.get('type', 'RollingUpdate')}",
           f"MinReadySeconds:        {spec.get('minReadySeconds', 0)}"]
    ru = strat.get("rollingUpdate") or {}
    if strat.get("type", "RollingUpdate") == "RollingUpdate":
        out.append(f"RollingUpdateStrategy:  {ru.get('maxUnavailable', '25%')} max unavailable, {ru.get('maxSurge', '25%')} max surge")
    if spec.get("paused"):
        out.append("Paused:                 true")
    out.append("Pod Template:")
    out += _template(spec.get("template") or {})
    out += _conditions(st, ("type", "status", "reason"))
    rss = ctx.get("replicasets")
    if rss is not None:
        rev = (obj["metadata"].get("annotations") or {}).get("deployment.kubernetes.io/revision")
        def revision(r):
            return int((r["metadata"].get("annotations") or {}).get("deployment.kubernetes.io/revision") or 0)
        if rev is not None:
            new = [r for r in rss if str(revision(r)) == rev]
        else:                    # newest revision owns the current template
            new = sorted(rss, key=revision)[-1:]
        old = [r for r in rss if r not in new and ((r.get("spec") or {}).get("replicas") or 0) > 0]

        def fmt(rs):
            return ", ".join(f"{r['metadata']['name']} ({(r.get('status') or {}).get('replicas', 0)}/"
                             f"{(r.get('spec') or {}).get('replicas', 0)} replicas created)" for r in rs) or "<none>"
        out += [f"OldReplicaSets:  {fmt(old)}", f"NewReplicaSet:   {fmt(new)}"]
    return out


def _replicated(obj, ctx):
    spec, st = obj.get("spec") or {}, obj.get("status") or {}
    out = [f"Selector:     {_selector(spec.get('selector'))}"]
    k = obj.get("kind")
    if k == "DaemonSet":
        out += [f"Desired Number of Nodes Scheduled: {st.get('desiredNumberScheduled', 0)}",
                f"Current Number of Nodes Scheduled: {st.get('currentNumberScheduled', 0)}",
                f"Number of Nodes Scheduled with Up-to-date Pods: {st.get('updatedNumberScheduled', 0)}",
                f"Number of Nodes Scheduled with Available Pods: {st.get('numberAvailable', 0)}",
                f"Number of Nodes Misscheduled: {st.get('numberMisscheduled', 0)}"]
    elif k == "Job":
        out += [f"Parallelism:  {spec.get('parallelism', 1)}", f"Completions:  {spec.get('completions', '<unset>')}",
                f"Start Time:   {st.get('startTime', '<unset>')}"]
        if spec.get("activeDeadlineSeconds"):
            out.append(f"Active Deadline Seconds:  {spec['activeDeadlineSeconds']}s")
    else:
        if k == "StatefulSet":
            out.append(f"Update Strategy:  {(spec.get('updateStrategy') or {}).get('type', 'OnDelete')}")
        out.append(f"Replicas:     {st.get('replicas', 0)} current / {spec.get('replicas', 1)} desired")
    if "pods" in ctx:
        out.append(f"Pods Status:  {_pods_status(ctx['pods'])}")
    out.append("Pod Template:")
    out += _template(spec.get("template") or {})
    out += _conditions(st)
    return out


def _cronjob(obj, ctx):
    spec, st = obj.get("spec") or {}, obj.get("status") or {}
    return [f"Schedule:                    {spec.get('schedule')}",
            f"Concurrency Policy:          {spec.get('concurrencyPolicy', 'Allow')}",
            f"Suspend:                     {spec.get('suspend', False)}",
            f"Starting Deadline Seconds:   {spec.get('startingDeadlineSeconds', '<unset>')}",
            f"Last Schedule Time:          {st.get('lastScheduleTime', '<unset>')}",
            "Active Jobs:                 " + (", ".join(a.get("name", "") for a in st.get("active") or ()) or "<none>")]


def _service(obj, ctx):
    spec = obj.get("spec") or {}
    out = [f"Selector:          {_kv(spec.get('selector'))}", f"Type:              {spec.get('type', 'ClusterIP')}",
           f"IP:                {spec.get('clusterIP', '')}"]
    if spec.get("externalIPs"):
        out.append(f"External IPs:      {','.join(spec['externalIPs'])}")
    ing = ((obj.get("status") or {}).get("loadBalancer") or {}).get("ingress") or []
    if ing:
        out.append("LoadBalancer Ingress:  " + ", ".join(i.get("ip") or i.get("hostname", "") for i in ing))
    if spec.get("externalName"):
        out.append(f"External Name:     {spec['externalName']}")
    ep = ctx.get("endpoints")
    for p in spec.get("ports") or ():
        name = p.get("name") or "<unset>"
        out.append(f"Port:              {name}  {p['port']}/{p.get('protocol', 'TCP')}")
        out.append(f"TargetPort:        {p.get('targetPort', p['port'])}/{p.get('protocol', 'TCP')}")
        if p.get("nodePort"):
            out.append(f"NodePort:          {name}  {p['nodePort']}/{p.get('protocol', 'TCP')}")
        if "endpoints" in ctx:
            addrs = []
            for sub in (ep or {}).get("subsets") or ():
                port = next((q["port"] for q in sub.get("ports") or () if q.get("name", "") == p.get("name", "")), None)
                addrs += [f"{a['ip']}:{port}" for a in sub.get("addresses") or () if port is not None]
            out.append(f"Endpoints:         {','.join(addrs) or '<none>'}")
    out.append(f"Session Affinity:  {spec.get('sessionAffinity', 'None')}")
    if spec.get("externalTrafficPolicy"):
        out.append(f"External Traffic Policy:  {spec['externalTrafficPolicy']}")
    return out


def _secret(obj, ctx):
    import base64
    out = [f"Type:  {obj.get('type', 'Opaque')}", "", "Data", "===="]
    for k, v in sorted((obj.get("data") or {}).items()):
        try:
            n = len(base64.b64decode(v or ""))
        except ValueError:
            n = len(v or "")
        out.append(f"{k}:  {n} bytes")
    return out


def _configmap(obj, ctx):
    out = ["", "Data", "===="]
    for k, v in sorted((obj.get("data") or {}).items()):
        out += [f"{k}:", "----", str(v)]
    return out


def _namespace(obj, ctx):
    out = [f"Status:  {(obj.get('status') or {}).get('phase', 'Active')}"]
    quotas = ctx.get("quotas")
    if quotas is not None:
        if not quotas:
            out.append("\nNo resource quota.")
        for q in quotas:
            out += ["", "Resource Quotas", f" Name:    {q['metadata']['name']}", " Resource  Used  Hard", " --------  ---   ---"]
            st = q.get("status") or {}
            for r, h in sorted(((st.get("hard") or (q.get("spec") or {}).get("hard")) or {}).items()):
                out.append(f" {r}  {(st.get('used') or {}).get(r, '0')}  {h}")
    lrs = ctx.get("limitranges")
    if lrs is not None:
        if not lrs:
            out.append("\nNo resource limits.")
        for lr in lrs:
            out += ["", f"Resource Limits ({lr['metadata']['name']})", " Type  Resource  Min  Max  Default Request  Default Limit"]
            for it in (lr.get("spec") or {}).get("limits") or ():
                res = set((it.get("min") or {})) | set(it.get("max") or {}) | set(it.get("default") or {}) | \
                    set(it.get("defaultRequest") or {})
                for r in sorted(res):
                    out.append(f" {it.get('type')}  {r}  {(it.get('min') or {}).get(r, '-')}  {(it.get('max') or {}).get(r, '-')}  "
                               f"{(it.get('defaultRequest') or {}).get(r, '-')}  {(it.get('default') or {}).get(r, '-')}")
    return out


def _serviceaccount(obj, ctx):
    secrets = [s.get("name") for s in obj.get("secrets") or ()]
    tokens = [s for s in secrets if "-token-" in (s or "")]
    return [f"Image pull secrets:  {', '.join(s.get('name', '') for s in obj.get('imagePullSecrets') or ()) or '<none>'}",
            f"Mountable secrets:   {', '.join(secrets) or '<none>'}",
            f"Tokens:              {', '.join(tokens) or '<none>'}"]


def _pv(obj, ctx):
    spec, st = obj.get("spec") or {}, obj.get("status") or {}
    claim = spec.get("claimRef") or {}
    src = next(((k, v) for k, v in spec.items() if k not in (
        "capacity", "accessModes", "claimRef", "persistentVolumeReclaimPolicy", "storageClassName", "mountOptions",
        "volumeMode", "nodeAffinity")), ("", {}))
    return [f"StorageClass:    {spec.get('storageClassName', '')}", f"Status:          {st.get('phase', '')}",
            f"Claim:           {claim.get('namespace', '')}/{claim.get('name', '')}" if claim else "Claim:",
            f"Reclaim Policy:  {spec.get('persistentVolumeReclaimPolicy', 'Retain')}",
            f"Access Modes:    {','.join(_MODES.get(x, x) for x in spec.get('accessModes') or ())}",
            f"Capacity:        {(spec.get('capacity') or {}).get('storage', '')}",
            "Source:", f"    Type:  {src[0]}"] + [f"    {k}:  {v}" for k, v in sorted((src[1] or {}).items())
                                                   if not isinstance(v, (dict, list))]


def _pvc(obj, ctx):
    spec, st = obj.get("spec") or {}, obj.get("status") or {}
    return [f"StorageClass:  {spec.get('storageClassName', '')}", f"Status:        {st.get('phase', '')}",
            f"Volume:        {spec.get('volumeName', '')}",
            f"Capacity:      {(st.get('capacity') or {}).get('storage', '')}",
            f"Access Modes:  {','.join(_MODES.get(x, x) for x in st.get('accessModes') or ())}"]


def _hpa(obj, ctx):
    spec, st = obj.get("spec") or {}, obj.get("status") or {}
    ref = spec.get("scaleTargetRef") or {}
    out = [f"Reference:  {ref.get('kind')}/{ref.get('name')}"]
    if spec.get("targetCPUUtilizationPercentage") is not None:
        out.append(f"Metrics:  ( current / target )\n  resource cpu on pods  (as a percentage of request):  "
                   f"{st.get('currentCPUUtilizationPercentage', '<unknown>')}% / {spec['targetCPUUtilizationPercentage']}%")
    for mt in spec.get("metrics") or ():
        r = mt.get("resource") or {}
        out.append(f"Metrics:  resource {r.get('name')} on pods:  target {r.get('targetAverageUtilization')}%")
    out += [f"Min replicas:      {spec.get('minReplicas', 1)}", f"Max replicas:      {spec.get('maxReplicas')}",
            f"Current replicas:  {st.get('currentReplicas', 0)}", f"Desired replicas:  {st.get('desiredReplicas', 0)}"]
    return out + _conditions(st)


def _endpoints(obj, ctx):
    out = ["Subsets:"]
    for sub in obj.get("subsets") or ():
        out.append("  Addresses:          " + (",".join(a["ip"] for a in sub.get("addresses") or ()) or "<none>"))
        out.append("  NotReadyAddresses:  " + (",".join(a["ip"] for a in sub.get("notReadyAddresses") or ()) or "<none>"))
        out.append("  Ports:")
        out += [f"    {p.get('name', '<unset>')}  {p['port']}  {p.get('protocol', 'TCP')}" for p in sub.get("ports") or ()]
    return out


DESCRIBERS = {
    "Deployment": _deployment, "ReplicaSet": _replicated, "ReplicationController": _replicated, "Job": _replicated,
    "DaemonSet": _replicated, "StatefulSet": _replicated, "CronJob": _cronjob, "Service": _service, "Secret": _secret,
    "ConfigMap": _configmap, "Namespace": _namespace, "ServiceAccount": _serviceaccount, "PersistentVolume": _pv,
    "PersistentVolumeClaim": _pvc, "HorizontalPodAutoscaler": _hpa, "Endpoints": _endpoints,
}


def sections(obj, ctx) -> list[str] | None:
    """-> the kind-specific lines, or None when there is no dedicated describer (the caller
    then falls back to a YAML dump of spec / status)."""
    fn = DESCRIBERS.get(obj.get("kind"))
    if fn is None:
        return None
    return fn(obj, ctx or {})


def fallback(obj):
    out = []
    for k in ("spec", "status"):
        if k in obj:
            out.append(f"{k.capitalize()}:")
            out += ["  " + ln for ln in yaml.safe_dump(obj[k], sort_keys=False).rstrip().splitlines()]
    return out
