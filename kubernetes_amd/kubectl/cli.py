"""kubectl — command-line client.

Parity: the cobra tree of `pkg/kubectl/cmd/cmd.go:216+` — create, apply, get, describe, delete,
logs, label, annotate, patch, replace, scale, cordon, uncordon, drain, taint, top, rollout
(status / history / undo), run, expose, version, api-versions, api-resources, cluster-info,
config (view / use-context / set-cluster / set-context / get-contexts), explain, wait,
auth can-i; kubeconfig loading (`staging/src/k8s.io/client-go/tools/clientcmd/loader.go:52`).
exec / attach / port-forward / cp speak the WebSocket channel protocols (`v4.channel.k8s.io`,
stdin and tty with `-i` / `-t`; `client/remotecommand.py`) through the API server's pod
subresources.

    python -m kubernetes_amd.kubectl get pods -o wide
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import time

import yaml

from ..api import core, meta as m
from ..client.rest import APIStatusError, Client, is_already_exists, is_not_found, resource_path
from . import extra, printers

DEFAULT_KUBECONFIG = os.path.expanduser("~/.kube/config")


# ---------------------------------------------------------------------------
# kubeconfig
def load_kubeconfig(path=None):
    path = path or os.environ.get("KUBECONFIG") or DEFAULT_KUBECONFIG
    if not os.path.exists(path):
        return {"apiVersion": "v1", "kind": "Config", "clusters": [], "contexts": [], "users": [], "current-context": ""}, path
    with open(path) as f:
        return yaml.safe_load(f) or {}, path


def save_kubeconfig(cfg, path):
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        yaml.safe_dump(cfg, f, sort_keys=False)


def resolve_server(args):
    """-> (server, token, namespace, ssl context) from flags or the kubeconfig (client-go clientcmd)."""
    if args.server:
        return args.server, args.token, args.namespace, None
    from ..client import clientcmd
    cfg, path = load_kubeconfig(args.kubeconfig)
    r = clientcmd.resolve(cfg, args.context, os.path.dirname(os.path.abspath(path)))
    if r is None:
        return os.environ.get("KUBERNETES_MASTER", "http://127.0.0.1:8080"), args.token, args.namespace, None
    return r.server, args.token or r.token, args.namespace or r.namespace, r.ssl_context


# ---------------------------------------------------------------------------
def read_manifests(paths):
    docs = []
    for p in paths:
        files = []
        if p == "-":
            text = sys.stdin.read()
            files.append(text)
        elif os.path.isdir(p):
            for fn in sorted(os.listdir(p)):
                if fn.endswith((".yaml", ".yml", ".json")):
                    files.append(open(os.path.join(p, fn)).read())
        else:
            files.append(open(p).read())
        for text in files:
            for d in yaml.safe_load_all(text):
                if not d:
                    continue
                if d.get("kind", "").endswith("List") and "items" in d:
                    docs.extend(d["items"])
                else:
                    docs.append(d)
    return docs


def ri_for_obj(o):
    ri = m.BY_KIND.get(o.get("kind", ""))
    if ri is None:
        raise SystemExit(f"error: unable to recognize kind {o.get('kind')!r}")
    return ri


def split_targets(targets):
    """['pods', 'a', 'b'] / ['pods/a', 'nodes/b'] / ['pod,node'] -> [(ri, name|None)]"""
    out = []
    if not targets:
        raise SystemExit("error: You must specify the type of resource")
    if "/" in targets[0]:
        for t in targets:
            r, n = t.split("/", 1)
            ri = m.lookup(r)
            if ri is None:
                raise SystemExit(f'error: the server doesn\'t have a resource type "{r}"')
            out.append((ri, n))
        return out
    kinds = targets[0].split(",")
    names = targets[1:]
    for k in kinds:
        ri = m.lookup(k)
        if ri is None:
            raise SystemExit(f'error: the server doesn\'t have a resource type "{k}"')
        if names:
            out.extend((ri, n) for n in names)
        else:
            out.append((ri, None))
    return out


class Kubectl(extra.ExtraCommands):
    def __init__(self, args, out=sys.stdout):
        self.a = args
        self.out = out
        server, token, ns, ctx = resolve_server(args)
        self.server = server
        self.ns = ns or "default"
        self.client = Client(server, token=token, ssl_context=ctx)

    def p(self, *s):
        print(*s, file=self.out)

    async def discover(self):
        """RESTMapper refresh from discovery (`pkg/kubectl/cmd/util/factory`'s deferred discovery
        mapper): registers CRD / aggregated resources the static table does not know."""
        st, body = await self.client.raw("GET", "/apis")
        if st != 200:
            return
        for g in json.loads(body).get("groups") or ():
            gv = (g.get("preferredVersion") or {}).get("groupVersion")
            if not gv:
                continue
            st, body = await self.client.raw("GET", f"/apis/{gv}")
            if st != 200:
                continue
            group, version = gv.split("/", 1)
            for r in json.loads(body).get("resources") or ():
                if "/" in r["name"] or m.BY_PLURAL.get(r["name"]):
                    continue
                m.register(m.ResourceInfo(group, version, r["kind"], r["name"], bool(r.get("namespaced")),
                                          tuple(r.get("shortNames") or ())))

    def _unknown_names(self):
        a = self.a
        names = []
        for t in getattr(a, "targets", None) or []:
            names += [x.split("/", 1)[0] for x in (t.split(",") if "/" not in t else [t])]
            if "/" not in t:
                break
        if getattr(a, "resource", None):
            names.append(a.resource.split(".")[0])
        return [n for n in names if m.lookup(n) is None]

    def ns_for(self, ri, obj=None):
        if not ri.namespaced:
            return None
        if obj is not None and (obj.get("metadata") or {}).get("namespace"):
            return obj["metadata"]["namespace"]
        return self.ns

    # -- commands -----------------------------------------------------------------
    async def cmd_get(self):
        a = self.a
        if a.filename:
            objs = []
            for d in read_manifests(a.filename):
                ri = ri_for_obj(d)
                objs.append(await self.client.get(ri.plural, d["metadata"]["name"], self.ns_for(ri, d)))
            self.p(printers.render(objs, a.output, wide=a.output == "wide"))
            return
        for ri, name in split_targets(a.targets):
            ns = None if (a.all_namespaces or not ri.namespaced) else self.ns
            if a.experimental_server_print and not a.output and not a.watch:
                # the server renders the columns (meta.k8s.io Table); kubectl only aligns them
                path = resource_path(ri.plural, ns, name)
                if a.selector:
                    from urllib.parse import quote
                    path += "?labelSelector=" + quote(a.selector)
                st, body = await self.client.http.request(
                    "GET", path, None, headers={"Accept": "application/json;as=Table;v=v1alpha1;g=meta.k8s.io"})
                if st != 200:
                    raise SystemExit(f"error: {body.decode(errors='replace')}")
                t = json.loads(body)
                self.p(printers.table([r["cells"] for r in t["rows"]], [c["name"].upper() for c in t["columnDefinitions"]]))
                continue
            if name:
                if a.export:
                    st, body = await self.client.raw("GET", resource_path(ri.plural, ns, name) + "?export=true")
                    if st != 200:
                        raise SystemExit(f"error: {body.decode(errors='replace')}")
                    obj = json.loads(body)
                else:
                    obj = await self.client.get(ri.plural, name, ns)
                self.p(printers.render([obj], a.output, ri.kind, a.output == "wide"))
                continue
            lst = await self.client.list(ri.plural, ns, a.selector, a.field_selector)
            items = lst.get("items") or []
            for o in items:
                o.setdefault("kind", ri.kind)
            if a.watch:
                self.p(printers.render(items, a.output, ri.kind, a.output == "wide", a.all_namespaces))
                st = await self.client.watch(ri.plural, ns, lst["metadata"]["resourceVersion"], a.selector, a.field_selector)
                async for t, o in st:
                    rows, h = printers.rows_for(ri.kind, [o], a.output == "wide")
                    self.p(printers.table(rows, h).splitlines()[-1])
                return
            self.p(printers.render(items, a.output, ri.kind, a.output == "wide", a.all_namespaces, list_obj=lst if a.output in ("json", "yaml") else None))

    async def cmd_describe(self):
        for ri, name in split_targets(self.a.targets):
            ns = None if not ri.namespaced else self.ns
            if name:
                objs = [await self.client.get(ri.plural, name, ns)]
            else:
                objs = (await self.client.list(ri.plural, ns, self.a.selector))["items"]
            for o in objs:
                o.setdefault("kind", ri.kind)
                evs = []
                try:
                    fs = f"involvedObject.name={o['metadata']['name']},involvedObject.kind={ri.kind}"
                    evs = (await self.client.list("events", o["metadata"].get("namespace") or "default", field_selector=fs))["items"]
                except APIStatusError:
                    pass
                self.p(printers.describe(o, evs))
                self.p("")

    async def _apply_one(self, d, mode):
        ri = ri_for_obj(d)
        ns = self.ns_for(ri, d)
        if ri.namespaced:
            d.setdefault("metadata", {})["namespace"] = ns
        name = d["metadata"].get("name")
        verb = "created"
        if mode == "create":
            await self.client.create(ri.plural, d, ns)
        elif mode == "replace":
            cur = await self.client.get(ri.plural, name, ns)
            d["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
            await self.client.update(ri.plural, d, ns)
            verb = "replaced"
        else:  # apply: create or merge with last-applied annotation
            ann = "kubectl.kubernetes.io/last-applied-configuration"
            d["metadata"].setdefault("annotations", {})[ann] = json.dumps(d, sort_keys=True)
            try:
                await self.client.create(ri.plural, d, ns)
            except APIStatusError as e:
                if not is_already_exists(e):
                    raise
                await self.client.patch(ri.plural, name, d, ns, "strategic")
                verb = "configured"
        self.p(f"{ri.kind.lower()}/{name} {verb}")

    async def cmd_create(self):
        if self.a.generator:
            await self._create_generated(self.a.generator)
            return
        if not self.a.filename:
            raise SystemExit("error: must specify one of -f and a resource generator (e.g. create namespace NAME)")
        for d in read_manifests(self.a.filename):
            await self._apply_one(d, "create")

    async def cmd_apply(self):
        for d in read_manifests(self.a.filename):
            await self._apply_one(d, "apply")

    async def cmd_replace(self):
        for d in read_manifests(self.a.filename):
            await self._apply_one(d, "replace")

    async def cmd_delete(self):
        a = self.a
        targets = []
        if a.filename:
            for d in read_manifests(a.filename):
                ri = ri_for_obj(d)
                targets.append((ri, d["metadata"]["name"], self.ns_for(ri, d)))
        else:
            for ri, name in split_targets(a.targets):
                ns = self.ns if ri.namespaced else None
                if name:
                    targets.append((ri, name, ns))
                elif a.all or a.selector:
                    for o in (await self.client.list(ri.plural, ns, a.selector))["items"]:
                        targets.append((ri, o["metadata"]["name"], ns))
                else:
                    raise SystemExit("error: resource(s) were provided, but no name, label selector, or --all flag specified")
        for ri, name, ns in targets:
            try:
                await self.client.delete(ri.plural, name, ns, grace_period=a.grace_period,
                                         propagation=None if a.cascade else "Orphan")
                self.p(f'{ri.kind.lower()} "{name}" deleted')
            except APIStatusError as e:
                if is_not_found(e) and a.ignore_not_found:
                    continue
                raise

    async def cmd_logs(self):
        a = self.a
        name = a.pod.split("/", 1)[-1]
        q = f"?container={a.container}" if a.container else ""
        if a.tail is not None:
            q += ("&" if q else "?") + f"tailLines={a.tail}"
        if a.previous:
            q += ("&" if q else "?") + "previous=true"
        st, body = await self.client.raw("GET", f"/api/v1/namespaces/{self.ns}/pods/{name}/log{q}")
        if st != 200:
            raise SystemExit(f"error: {body.decode(errors='replace')}")
        self.out.write(body.decode(errors="replace"))

    async def _meta_edit(self, field):
        a = self.a
        ri = m.lookup(a.resource.split("/")[0])
        names = [a.resource.split("/", 1)[1]] if "/" in a.resource else [a.name]
        kv = a.pairs
        patch = {}
        for p in kv:
            if p.endswith("-"):
                patch[p[:-1]] = None
            else:
                k, _, v = p.partition("=")
                patch[k] = v
        for n in names:
            await self.client.patch(ri.plural, n, {"metadata": {field: patch}}, self.ns if ri.namespaced else None)
            self.p(f"{ri.kind.lower()}/{n} {'labeled' if field == 'labels' else 'annotated'}")

    async def cmd_label(self):
        await self._meta_edit("labels")

    async def cmd_annotate(self):
        await self._meta_edit("annotations")

    async def cmd_patch(self):
        a = self.a
        (ri, name), = split_targets(a.targets)
        patch = json.loads(a.patch) if a.patch.strip().startswith(("{", "[")) else yaml.safe_load(a.patch)
        await self.client.patch(ri.plural, name, patch, self.ns if ri.namespaced else None, a.type)
        self.p(f"{ri.kind.lower()}/{name} patched")

    async def cmd_scale(self):
        """`kubectl scale` (pkg/kubectl/scale.go): through the scale subresource, with the
        --current-replicas / --resource-version preconditions checked against the Scale; Jobs
        (parallelism) are patched directly."""
        a = self.a
        for ri, name in split_targets(a.targets):
            if ri.plural == "jobs":
                job = await self.client.get("jobs", name, self.ns)
                cur = (job.get("spec") or {}).get("parallelism", 1)
                if a.current_replicas is not None and a.current_replicas != cur:
                    raise SystemExit(f"error: Expected replicas to be {a.current_replicas}, was {cur}")
                await self.client.patch("jobs", name, {"spec": {"parallelism": a.replicas}}, self.ns)
            else:
                scale = await self.client.get(ri.plural, name, self.ns, subresource="scale")
                cur = (scale.get("spec") or {}).get("replicas", 0)
                if a.current_replicas is not None and a.current_replicas != cur:
                    raise SystemExit(f"error: Expected replicas to be {a.current_replicas}, was {cur}")
                if a.resource_version and a.resource_version != scale["metadata"].get("resourceVersion"):
                    raise SystemExit(f"error: Expected resourceVersion to be {a.resource_version}, "
                                     f"was {scale['metadata'].get('resourceVersion')}")
                scale["spec"] = {"replicas": a.replicas}
                await self.client.update(ri.plural, scale, self.ns, subresource="scale")
            self.p(f"{ri.kind.lower()} \"{name}\" scaled")

    async def _cordon(self, name, flag):
        await self.client.patch("nodes", name, {"spec": {"unschedulable": flag or None}})
        self.p(f"node/{name} {'cordoned' if flag else 'uncordoned'}")

    async def cmd_cordon(self):
        await self._cordon(self.a.node, True)

    async def cmd_uncordon(self):
        await self._cordon(self.a.node, False)

    async def cmd_drain(self):
        a = self.a
        await self._cordon(a.node, True)
        pods = (await self.client.list("pods", None, field_selector=f"spec.nodeName={a.node}"))["items"]
        for p in pods:
            ref = m.controller_of(p)
            if ref and ref.get("kind") == "DaemonSet" and a.ignore_daemonsets:
                continue
            if not ref and not a.force:
                raise SystemExit(f"error: pod {p['metadata']['name']} is not managed by a controller (use --force)")
            try:
                await self.client.evict(p["metadata"]["namespace"], p["metadata"]["name"], a.grace_period)
                self.p(f"pod/{p['metadata']['name']} evicted")
            except APIStatusError as e:
                if not is_not_found(e):
                    raise
        self.p(f"node/{a.node} drained")

    async def cmd_taint(self):
        a = self.a
        node = await self.client.get("nodes", a.node)
        taints = list((node.get("spec") or {}).get("taints") or [])
        for t in a.taints:
            if t.endswith("-"):
                key = t[:-1].split(":")[0].split("=")[0]
                taints = [x for x in taints if x["key"] != key]
            else:
                kv, _, eff = t.partition(":")
                k, _, v = kv.partition("=")
                taints = [x for x in taints if not (x["key"] == k and x["effect"] == eff)]
                taints.append({"key": k, "value": v, "effect": eff} if v else {"key": k, "effect": eff})
        await self.client.patch("nodes", a.node, {"spec": {"taints": taints or None}})
        self.p(f"node/{a.node} tainted")

    async def _metrics(self, path):
        st, body = await self.client.raw("GET", "/apis/metrics.k8s.io/v1beta1" + path)
        return {(i["metadata"].get("namespace"), i["metadata"]["name"]): i for i in json.loads(body).get("items") or ()} \
            if st == 200 else {}

    async def cmd_top(self):
        """`kubectl top` (`pkg/kubectl/cmd/top_node.go`, `top_pod.go`) over metrics.k8s.io, with the
        MI355X columns: allocated GPUs per node and per-pod GPU utilization."""
        a = self.a
        nodes = (await self.client.list("nodes"))["items"]
        pods = (await self.client.list("pods"))["items"]
        if a.what in ("node", "nodes"):
            nm = await self._metrics("/nodes")
            rows = []
            for n in nodes:
                name = n["metadata"]["name"]
                devs = ((n.get("status") or {}).get("extendedResources") or {}).get(core.AMD_GPU, {}).get("resources") or {}
                used = sum(len(printers.pod_gpus(p)) for p in pods if (p.get("spec") or {}).get("nodeName") == name
                           and not core.pod_is_terminal(p))
                u = (nm.get((None, name)) or {}).get("usage") or {}
                rows.append([name, u.get("cpu", "<unknown>"), u.get("memory", "<unknown>"), len(devs), used,
                             f"{(100 * used // len(devs)) if devs else 0}%",
                             sum(1 for d in devs.values() if d.get("health") != "Healthy")])
            self.p(printers.table(rows, ["NAME", "CPU(cores)", "MEMORY(bytes)", "GPUS", "GPUS-ALLOCATED", "GPU%", "UNHEALTHY"]))
        else:
            pm = await self._metrics(f"/namespaces/{self.ns}/pods")
            rows = []
            for p in pods:
                if p["metadata"].get("namespace") != self.ns or core.pod_is_terminal(p):
                    continue
                mt = pm.get((self.ns, p["metadata"]["name"])) or {}
                cpu = sum(int(str(c["usage"].get("cpu", "0m")).rstrip("m") or 0) for c in mt.get("containers") or ())
                mem = sum(int(str(c["usage"].get("memory", "0Ki")).rstrip("Ki") or 0) for c in mt.get("containers") or ())
                gpu = [c["usage"].get(core.AMD_GPU) for c in mt.get("containers") or () if core.AMD_GPU in c.get("usage", {})]
                rows.append([p["metadata"]["name"], f"{cpu}m" if mt else "<unknown>", f"{mem // 1024}Mi" if mt else "<unknown>",
                             ",".join(printers.pod_gpus(p)) or "<none>", (gpu[0] + "%") if gpu else "<none>"])
            self.p(printers.table(rows, ["NAME", "CPU(cores)", "MEMORY(bytes)", "GPUS", "GPU-UTIL"]))

    async def cmd_autoscale(self):
        """`kubectl autoscale deployment/x --min --max --cpu-percent` (`pkg/kubectl/cmd/autoscale.go`);
        `--gpu-percent` targets MI355X utilization through `spec.metrics`."""
        a = self.a
        (ri, name), = split_targets(a.targets)
        spec = {"scaleTargetRef": {"apiVersion": ri.group_version, "kind": ri.kind, "name": name},
                "maxReplicas": a.max}
        if a.min:
            spec["minReplicas"] = a.min
        if a.gpu_percent:
            spec["metrics"] = [{"type": "Resource", "resource": {"name": core.AMD_GPU, "targetAverageUtilization": a.gpu_percent}}]
        elif a.cpu_percent:
            spec["targetCPUUtilizationPercentage"] = a.cpu_percent
        await self.client.create("horizontalpodautoscalers", {"metadata": {"name": a.name or name, "namespace": self.ns},
                                                              "spec": spec}, self.ns)
        self.p(f"{ri.kind.lower()}.{ri.group or 'core'} \"{name}\" autoscaled")

    async def cmd_certificate(self):
        """`kubectl certificate approve|deny CSR...` (`pkg/kubectl/cmd/certificates.go`)."""
        a = self.a
        for n in a.names:
            csr = await self.client.get("certificatesigningrequests", n)
            conds = [c for c in (csr.get("status") or {}).get("conditions") or () if c.get("type") not in ("Approved", "Denied")]
            typ = "Approved" if a.action == "approve" else "Denied"
            conds.append({"type": typ, "reason": "KubectlApprove" if typ == "Approved" else "KubectlDeny",
                          "message": f"This CSR was {typ.lower()} by kubectl certificate {a.action}."})
            csr.setdefault("status", {})["conditions"] = conds
            await self.client.update("certificatesigningrequests", csr, subresource="approval")
            self.p(f"certificatesigningrequest.certificates.k8s.io/{n} {typ.lower()}")

    async def cmd_rollout(self):
        a = self.a
        (ri, name), = split_targets(a.targets)
        if a.action == "status":
            t = time.time()
            while True:
                d = await self.client.get(ri.plural, name, self.ns)
                st, spec = d.get("status") or {}, d.get("spec") or {}
                want = spec.get("replicas", 1)
                if st.get("updatedReplicas") == want and st.get("availableReplicas") == want and st.get("replicas") == want:
                    self.p(f'deployment "{name}" successfully rolled out')
                    return
                if not a.watch or time.time() - t > a.timeout:
                    self.p(f"Waiting for rollout to finish: {st.get('updatedReplicas', 0)} of {want} updated replicas are available...")
                    if not a.watch:
                        return
                    raise SystemExit(1)
                await asyncio.sleep(0.2)
        elif a.action in ("history", "undo") and ri.kind in ("DaemonSet", "StatefulSet"):
            from ..controllers.history import revisions_of
            obj = await self.client.get(ri.plural, name, self.ns)
            revs = revisions_of((await self.client.list("controllerrevisions", self.ns))["items"], obj["metadata"]["uid"])
            if a.action == "history":
                rows = [[int(r.get("revision", 0)), (r["metadata"].get("annotations") or {}).get(
                    "kubernetes.io/change-cause", "<none>")] for r in revs]
                self.p(printers.table(rows, ["REVISION", "CHANGE-CAUSE"]))
                return
            if len(revs) < 2 and not a.to_revision:
                raise SystemExit(f"error: no rollout history found for {ri.kind.lower()} \"{name}\"")
            target = next((r for r in revs if int(r.get("revision", 0)) == a.to_revision), None) if a.to_revision \
                else revs[-2]
            if target is None:
                raise SystemExit(f"error: unable to find specified revision {a.to_revision} in history")
            await self.client.patch(ri.plural, name, {"spec": {"template": target["data"]["spec"]["template"]}}, self.ns)
            self.p(f"{ri.kind.lower()}.apps/{name} rolled back")
        elif a.action == "history":
            uid = (await self.client.get(ri.plural, name, self.ns))["metadata"]["uid"]
            rss = [r for r in (await self.client.list("replicasets", self.ns))["items"] if (m.controller_of(r) or {}).get("uid") == uid]
            rows = sorted([[int((r["metadata"].get("annotations") or {}).get("deployment.kubernetes.io/revision", 0)), "<none>"] for r in rss])
            self.p(printers.table(rows, ["REVISION", "CHANGE-CAUSE"]))
        elif a.action == "undo":
            # DeploymentRollbacker: the extensions/v1beta1 rollback subresource
            body = {"kind": "DeploymentRollback", "apiVersion": "extensions/v1beta1", "name": name,
                    "rollbackTo": {"revision": a.to_revision or 0}}
            st, resp = await self.client.raw("POST", f"/apis/extensions/v1beta1/namespaces/{self.ns}/deployments/{name}/rollback",
                                             json.dumps(body).encode())
            if st != 200:
                raise SystemExit(f"error: {resp.decode(errors='replace')}")
            self.p(f"deployment.apps/{name} rolled back")

    async def cmd_run(self):
        a = self.a
        c = {"name": a.name, "image": a.image}
        if a.run_command:
            c["command"] = a.run_command
        if a.gpus:
            c["resources"] = {"limits": {core.AMD_GPU: str(a.gpus)}}
        pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": a.name, "namespace": self.ns, "labels": {"run": a.name}},
               "spec": {"containers": [c], "restartPolicy": a.restart}}
        await self.client.create("pods", pod, self.ns)
        self.p(f"pod/{a.name} created")

    async def cmd_expose(self):
        a = self.a
        (ri, name), = split_targets(a.targets)
        obj = await self.client.get(ri.plural, name, self.ns)
        sel = (obj["metadata"].get("labels") if ri.kind == "Pod" else
               ((obj.get("spec") or {}).get("selector") or {}).get("matchLabels")) or {}
        svc = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": a.name or name, "namespace": self.ns},
               "spec": {"selector": sel, "ports": [{"port": a.port, "targetPort": a.target_port or a.port}]}}
        await self.client.create("services", svc, self.ns)
        self.p(f"service/{a.name or name} exposed")

    async def cmd_version(self):
        st, body = await self.client.raw("GET", "/version")
        from ..apiserver.server import VERSION
        self.p(f"Client Version: {VERSION['gitVersion']}")
        if st == 200:
            self.p(f"Server Version: {json.loads(body)['gitVersion']}")

    async def cmd_api_versions(self):
        _, body = await self.client.raw("GET", "/apis")
        self.p("v1")
        for g in json.loads(body)["groups"]:
            for v in g["versions"]:
                self.p(v["groupVersion"])

    async def cmd_api_resources(self):
        rows = [[r.plural, ",".join(r.short), r.group_version, str(r.namespaced).lower(), r.kind] for r in m.RESOURCES]
        self.p(printers.table(rows, ["NAME", "SHORTNAMES", "APIVERSION", "NAMESPACED", "KIND"]))

    async def cmd_cluster_info(self):
        self.p(f"Kubernetes master is running at {self.server}")

    async def cmd_explain(self):
        ri = m.lookup(self.a.resource.split(".")[0])
        if ri is None:
            raise SystemExit(f"error: couldn't find resource for {self.a.resource}")
        self.p(f"KIND:     {ri.kind}\nVERSION:  {ri.group_version}\n")
        if ri.kind == "Pod":
            self.p("FIELDS (MI355X device model, fork ResourceV2):\n"
                   "   spec.extendedResources[]   <[]PodExtendedResource>  pod-level device requests\n"
                   "      name                    <string>  unique name referenced by containers\n"
                   "      resources.limits        <map>     exactly one entry, e.g. amd.com/gpu: 4\n"
                   "      affinity.required[]     <[]ResourceSelector> key/operator(In,NotIn,Exists,DoesNotExist,Gt,Lt)/values\n"
                   "                              keys: amd.com/arch amd.com/product amd.com/memory amd.com/hbm\n"
                   "                                    amd.com/xgmi-hive amd.com/numa amd.com/partition amd.com/ecc\n"
                   "      assigned[]              <[]string> device IDs (written by pods/binding)\n"
                   "   spec.containers[].extendedResourceRequests <[]string> names of extendedResources")

    async def cmd_wait(self):
        a = self.a
        (ri, name), = split_targets(a.targets)
        cond = a.for_.split("=", 1)[1] if "=" in a.for_ else a.for_
        t = time.time()
        while time.time() - t < a.timeout:
            try:
                o = await self.client.get(ri.plural, name, self.ns if ri.namespaced else None)
            except APIStatusError as e:
                if a.for_ == "delete" and is_not_found(e):
                    self.p(f"{ri.kind.lower()}/{name} deleted")
                    return
                raise
            if a.for_.startswith("condition="):
                c = core.get_condition(o.get("status"), cond)
                if c and c.get("status") == "True":
                    self.p(f"{ri.kind.lower()}/{name} condition met")
                    return
            await asyncio.sleep(0.1)
        raise SystemExit(f"error: timed out waiting for the condition on {ri.plural}/{name}")

    async def cmd_auth(self):
        a = self.a
        if a.action == "reconcile":
            for d in read_manifests(a.filename or []):
                await self._reconcile(d)
            return
        ri = m.lookup(a.resource)
        st, body = await self.client.raw("GET", f"{'/api/v1' if not ri.group else f'/apis/{ri.group}/{ri.version}'}"
                                         f"{'/namespaces/' + self.ns if ri.namespaced else ''}/{ri.plural}?limit=1")
        self.p("yes" if st == 200 else "no")

    # -- streaming: exec / attach / port-forward / cp / proxy / edit ------------------------
    def _pod_path(self, name, sub):
        return f"/api/v1/namespaces/{self.ns}/pods/{name}/{sub}"

    def _stream_path(self, pod, sub, container, command=(), stdin=False, tty=False):
        from urllib.parse import urlencode
        q = [("command", c) for c in command] + ([("container", container)] if container else [])
        q += [("stdin", "true")] if stdin else []
        q += [("stdout", "true")] + ([("stderr", "true")] if not tty else []) + ([("tty", "true")] if tty else [])
        return self._pod_path(pod, sub) + "?" + urlencode(q)

    async def _exec(self, pod, container, command, stdin_data=None):
        """pods/exec over WebSocket (`v4.channel.k8s.io`) -> (exit code, stdout, stderr)
        (`pkg/kubectl/cmd/exec.go`)."""
        from ..client.remotecommand import StreamError, exec_collect
        try:
            return await exec_collect(self.client.http, self._stream_path(pod, "exec", container, command,
                                                                          stdin=stdin_data is not None), stdin_data)
        except StreamError as e:
            raise SystemExit(f"error: unable to exec in pod {pod}: {e.message}")

    async def _interactive(self, pod, sub, container, command, stdin, tty):
        """exec / attach with the local stdin (and a raw-mode terminal under -t, resized on SIGWINCH)."""
        import signal
        from ..client.remotecommand import StreamError, exec_stream
        loop = asyncio.get_running_loop()
        src = resize = None
        restore = None
        if stdin:
            q: asyncio.Queue = asyncio.Queue()
            fd = sys.stdin.fileno()

            def pump():
                while True:
                    d = os.read(fd, 65536)
                    loop.call_soon_threadsafe(q.put_nowait, d)
                    if not d:
                        return
            loop.run_in_executor(None, pump)

            async def src_gen():
                while True:
                    d = await q.get()
                    if not d:
                        return
                    yield d
            src = src_gen()
            if tty and os.isatty(fd):
                import termios
                import tty as tty_mod
                saved = termios.tcgetattr(fd)
                tty_mod.setraw(fd)
                restore = lambda: termios.tcsetattr(fd, termios.TCSADRAIN, saved)   # noqa: E731
        if tty and os.isatty(1):
            rq: asyncio.Queue = asyncio.Queue()

            def winch(*_):
                sz = os.get_terminal_size(1)
                rq.put_nowait((sz.columns, sz.lines))
            winch()
            loop.add_signal_handler(signal.SIGWINCH, winch)

            async def resize_gen():
                while True:
                    yield await rq.get()
            resize = resize_gen()
        out = self.out

        def write_out(d):
            if hasattr(out, "buffer"):
                out.buffer.write(d)
                out.flush()
            else:
                out.write(d.decode(errors="replace"))

        def write_err(d):
            sys.stderr.buffer.write(d)
            sys.stderr.flush()
        try:
            return await exec_stream(self.client.http, self._stream_path(pod, sub, container, command, stdin, tty),
                                     src, write_out, write_err, resize)
        except StreamError as e:
            raise SystemExit(f"error: unable to {'exec in' if sub == 'exec' else 'attach to'} pod {pod}: {e.message}")
        finally:
            if restore:
                restore()
            if resize is not None:
                loop.remove_signal_handler(signal.SIGWINCH)

    async def cmd_exec(self):
        a = self.a
        rest = list(a.exec_command or [])
        container = a.container
        if "--" in rest:
            pre, cmd = rest[:rest.index("--")], rest[rest.index("--") + 1:]
            i = 0
            while i < len(pre):        # flags given after the pod name but before `--`
                if pre[i] in ("-c", "--container") and i + 1 < len(pre):
                    container = pre[i + 1]
                    i += 2
                else:
                    i += 1
        else:
            cmd = rest
        if not cmd:
            raise SystemExit("error: you must specify at least one command for the container")
        if a.stdin or a.tty:
            self.rc = await self._interactive(a.pod, "exec", container, cmd, a.stdin, a.tty)
            return
        rc, out, err = await self._exec(a.pod, container, cmd)
        self.out.write(out.decode(errors="replace"))
        if err:
            sys.stderr.write(err.decode(errors="replace"))
        self.rc = rc

    async def cmd_attach(self):
        """`kubectl attach`: the container's output from now on, until it exits (with -i, stdin)."""
        a = self.a
        self.rc = await self._interactive(a.pod, "attach", a.container, (), a.stdin, a.tty)

    async def cmd_port_forward(self):
        """`kubectl port-forward POD [LOCAL:]REMOTE ...` (`pkg/kubectl/cmd/portforward.go`): one
        WebSocket (`v4.channel.k8s.io`, data + error channel per port) per local connection."""
        from ..client.remotecommand import StreamError, forward_connection
        a = self.a
        pod = a.pod.split("/", 1)[-1]
        servers, served = [], [0]
        done = asyncio.Event()
        for spec in a.ports:
            lp, _, rp = spec.partition(":")
            local, remote = (int(lp), int(rp)) if rp else (int(lp), int(lp))

            def handler(remote=remote):
                async def h(reader, writer):
                    try:
                        await forward_connection(self.client.http, self._pod_path(pod, "portforward") +
                                                 f"?ports={remote}", remote, reader, writer)
                    except (StreamError, ConnectionError) as e:
                        print(f"error forwarding port {remote}: {e}", file=sys.stderr)
                        writer.close()
                    served[0] += 1
                    if a.max_connections and served[0] >= a.max_connections:
                        done.set()
                return h
            srv = await asyncio.start_server(handler(), a.address, local)
            servers.append(srv)
            self.p(f"Forwarding from {a.address}:{srv.sockets[0].getsockname()[1]} -> {remote}")
        if hasattr(self.out, "flush"):
            self.out.flush()
        try:
            await done.wait()
        finally:
            for srv in servers:
                srv.close()

    async def cmd_cp(self):
        """`kubectl cp` over exec: pod->local streams `cat`; local->pod ships the file base64-encoded
        in the exec command (files up to 1 MiB; the reference pipes a tar stream over stdin)."""
        a = self.a
        src, dst = a.src, a.dst
        if ":" in src and not os.path.exists(src):
            pod, path = src.split(":", 1)
            rc, out, err = await self._exec(pod.split("/")[-1], a.container, ["cat", path])
            if rc != 0:
                raise SystemExit(f"error: {err.decode() or out.decode()}")
            with open(dst, "wb") as f:
                f.write(out)
            return
        pod, path = dst.split(":", 1)
        with open(src, "rb") as f:
            data = f.read()
        if len(data) > 1 << 20:
            raise SystemExit("error: kubectl cp into a pod supports files up to 1 MiB")
        import base64
        b64 = base64.b64encode(data).decode()
        rc, out, err = await self._exec(pod.split("/")[-1], a.container,
                                        ["sh", "-c", f"printf %s '{b64}' | base64 -d > '{path}'"])
        if rc != 0:
            raise SystemExit(f"error: {err.decode() or out.decode()}")

    async def cmd_proxy(self):
        """`kubectl proxy`: a local HTTP endpoint forwarding to the API server with this
        kubeconfig's credentials (`pkg/kubectl/proxy/proxy_server.go`)."""
        from ..utils.httpserver import HTTPServer, Response, StreamResponse
        a = self.a
        http = self.client.http

        async def handle(req):
            path = req.raw_path + (("?" + req.qs) if req.qs else "")
            if req.query.get("watch") in ("true", "1") or "/watch/" in req.raw_path:
                st, hdrs, r, w = await http.open_raw(req.method, path)

                async def relay(cw):
                    try:
                        while True:
                            line = await r.readuntil(b"\r\n")
                            n = int(line.strip(), 16)
                            if n == 0:
                                break
                            cw.write(await r.readexactly(n))
                            await r.readexactly(2)
                    finally:
                        w.close()
                return StreamResponse(relay, hdrs.get("content-type", "application/json"))
            st, body = await http.request(req.method, path, req.body or None,
                                          req.headers.get("content-type", "application/json"))
            return Response(st, body)
        srv = HTTPServer(handle)
        port = await srv.start(a.address, a.port)
        self.p(f"Starting to serve on {a.address}:{port}")
        if hasattr(self.out, "flush"):
            self.out.flush()
        try:
            if a.serve_seconds:
                await asyncio.sleep(a.serve_seconds)
            else:
                await asyncio.Event().wait()
        finally:
            await srv.stop()

    async def cmd_edit(self):
        """`kubectl edit`: dump YAML, run $EDITOR, PUT the result if it changed."""
        import subprocess
        import tempfile
        (ri, name), = split_targets(self.a.targets)
        obj = await self.client.get(ri.plural, name, self.ns_for(ri))
        text = yaml.safe_dump(obj, sort_keys=False)
        with tempfile.NamedTemporaryFile("w", suffix=".yaml", delete=False) as f:
            f.write(text)
            path = f.name
        try:
            editor = os.environ.get("KUBE_EDITOR") or os.environ.get("EDITOR") or "vi"
            rc = subprocess.call(editor.split() + [path])
            if rc != 0:
                raise SystemExit(f"error: editor exited with {rc}")
            with open(path) as f:
                new_text = f.read()
        finally:
            os.unlink(path)
        if new_text == text:
            self.p("Edit cancelled, no changes made.")
            return
        new = yaml.safe_load(new_text)
        await self.client.update(ri.plural, new, self.ns_for(ri))
        self.p(f"{ri.kind.lower()}/{name} edited")


def cmd_config(a):
    cfg, path = load_kubeconfig(a.kubeconfig)
    if a.action == "view":
        print(yaml.safe_dump(cfg, sort_keys=False).rstrip())
    elif a.action == "current-context":
        print(cfg.get("current-context", ""))
    elif a.action == "get-contexts":
        rows = [["*" if c["name"] == cfg.get("current-context") else "", c["name"], c["context"].get("cluster", ""),
                 c["context"].get("user", ""), c["context"].get("namespace", "")] for c in cfg.get("contexts") or ()]
        print(printers.table(rows, ["CURRENT", "NAME", "CLUSTER", "AUTHINFO", "NAMESPACE"]))
    elif a.action == "use-context":
        cfg["current-context"] = a.name
        save_kubeconfig(cfg, path)
        print(f'Switched to context "{a.name}".')
    elif a.action == "set-cluster":
        cl = [c for c in cfg.setdefault("clusters", []) if c["name"] != a.name]
        cl.append({"name": a.name, "cluster": {"server": a.server_url}})
        cfg["clusters"] = cl
        save_kubeconfig(cfg, path)
        print(f'Cluster "{a.name}" set.')
    elif a.action == "set-credentials":
        us = [u for u in cfg.setdefault("users", []) if u["name"] != a.name]
        us.append({"name": a.name, "user": {"token": a.user_token}})
        cfg["users"] = us
        save_kubeconfig(cfg, path)
        print(f'User "{a.name}" set.')
    elif a.action == "set-context":
        cs = [c for c in cfg.setdefault("contexts", []) if c["name"] != a.name]
        cs.append({"name": a.name, "context": {"cluster": a.cluster, "user": a.user, "namespace": a.ctx_namespace or "default"}})
        cfg["contexts"] = cs
        save_kubeconfig(cfg, path)
        print(f'Context "{a.name}" modified.')


def build_parser():
    ap = argparse.ArgumentParser("kubectl")
    ap.add_argument("-s", "--server")
    ap.add_argument("--token")
    ap.add_argument("--kubeconfig")
    ap.add_argument("--context")
    ap.add_argument("-n", "--namespace")
    sub = ap.add_subparsers(dest="command", required=True)

    def add(name, **kw):
        return sub.add_parser(name, **kw)

    g = add("get")
    g.add_argument("targets", nargs="*")
    g.add_argument("-o", "--output", default="")
    g.add_argument("-l", "--selector")
    g.add_argument("--field-selector")
    g.add_argument("-A", "--all-namespaces", action="store_true")
    g.add_argument("-w", "--watch", action="store_true")
    g.add_argument("-f", "--filename", action="append")
    g.add_argument("--export", action="store_true", help="strip cluster-specific fields (single objects)")
    g.add_argument("--experimental-server-print", action="store_true", help="columns rendered by the API server")
    d = add("describe")
    d.add_argument("targets", nargs="+")
    d.add_argument("-l", "--selector")
    for name in ("create", "apply", "replace"):
        c = add(name)
        c.add_argument("-f", "--filename", action="append", required=name != "create")
        if name == "create":
            c.add_argument("--dry-run", action="store_true")
            c.add_argument("-o", "--output", default="")
            c.add_argument("generator", nargs=argparse.REMAINDER)
    de = add("delete")
    de.add_argument("targets", nargs="*")
    de.add_argument("-f", "--filename", action="append")
    de.add_argument("-l", "--selector")
    de.add_argument("--all", action="store_true")
    de.add_argument("--grace-period", type=int, default=None)
    de.add_argument("--cascade", type=lambda s: s.lower() != "false", default=True)
    de.add_argument("--ignore-not-found", action="store_true")
    lg = add("logs")
    lg.add_argument("pod")
    lg.add_argument("-c", "--container")
    lg.add_argument("--tail", type=int)
    lg.add_argument("-p", "--previous", action="store_true")
    for name in ("label", "annotate"):
        la = add(name)
        la.add_argument("resource")
        la.add_argument("name", nargs="?")
        la.add_argument("pairs", nargs="+")
    pa = add("patch")
    pa.add_argument("targets", nargs="+")
    pa.add_argument("-p", "--patch", required=True)
    pa.add_argument("--type", default="strategic", choices=["strategic", "merge", "json"])
    sc = add("scale")
    sc.add_argument("targets", nargs="+")
    sc.add_argument("--replicas", type=int, required=True)
    sc.add_argument("--current-replicas", type=int, default=None)
    sc.add_argument("--resource-version", default="")
    for name in ("cordon", "uncordon"):
        add(name).add_argument("node")
    dr = add("drain")
    dr.add_argument("node")
    dr.add_argument("--ignore-daemonsets", action="store_true")
    dr.add_argument("--force", action="store_true")
    dr.add_argument("--grace-period", type=int, default=None)
    ta = add("taint")
    ta.add_argument("nodes_kw", choices=["nodes", "node", "no"])
    ta.add_argument("node")
    ta.add_argument("taints", nargs="+")
    tp = add("top")
    tp.add_argument("what", choices=["node", "nodes", "pod", "pods"])
    ro = add("rollout")
    ro.add_argument("action", choices=["status", "history", "undo"])
    ro.add_argument("targets", nargs="+")
    ro.add_argument("--to-revision", type=int, default=0)
    ro.add_argument("-w", "--watch", type=lambda s: s.lower() != "false", default=True)
    ro.add_argument("--timeout", type=float, default=300)
    rn = add("run")
    rn.add_argument("name")
    rn.add_argument("--image", required=True)
    rn.add_argument("--gpus", type=int, default=0, help="request N amd.com/gpu")
    rn.add_argument("--restart", default="Always")
    rn.add_argument("run_command", nargs="*", metavar="command")
    ex = add("expose")
    ex.add_argument("targets", nargs="+")
    ex.add_argument("--port", type=int, required=True)
    ex.add_argument("--target-port", type=int)
    ex.add_argument("--name")
    add("version")
    add("api-versions")
    add("api-resources")
    add("cluster-info")
    e = add("explain")
    e.add_argument("resource")
    w = add("wait")
    w.add_argument("targets", nargs="+")
    w.add_argument("--for", dest="for_", required=True)
    w.add_argument("--timeout", type=float, default=30)
    au = add("auth")
    au.add_argument("action", choices=["can-i", "reconcile"])
    au.add_argument("verb", nargs="?")
    au.add_argument("resource", nargs="?")
    au.add_argument("-f", "--filename", action="append")
    exq = add("exec")
    exq.add_argument("pod")
    exq.add_argument("-c", "--container")
    exq.add_argument("-i", "--stdin", action="store_true")
    exq.add_argument("-t", "--tty", action="store_true")
    exq.add_argument("exec_command", nargs=argparse.REMAINDER)
    at = add("attach")
    at.add_argument("pod")
    at.add_argument("-c", "--container")
    at.add_argument("-i", "--stdin", action="store_true")
    at.add_argument("-t", "--tty", action="store_true")
    pf = add("port-forward")
    pf.add_argument("pod")
    pf.add_argument("ports", nargs="+")
    pf.add_argument("--address", default="127.0.0.1")
    pf.add_argument("--max-connections", type=int, default=0, help=argparse.SUPPRESS)
    cpp = add("cp")
    cpp.add_argument("src")
    cpp.add_argument("dst")
    cpp.add_argument("-c", "--container")
    px = add("proxy")
    px.add_argument("-p", "--port", type=int, default=8001)
    px.add_argument("--address", default="127.0.0.1")
    px.add_argument("--serve-seconds", type=float, default=0, help=argparse.SUPPRESS)
    ed = add("edit")
    ed.add_argument("targets", nargs="+")
    aut = add("autoscale")
    aut.add_argument("targets", nargs="+")
    aut.add_argument("--min", type=int, default=0)
    aut.add_argument("--max", type=int, required=True)
    aut.add_argument("--cpu-percent", type=int, default=0)
    aut.add_argument("--gpu-percent", type=int, default=0, help="target MI355X utilization (amd.com/gpu)")
    aut.add_argument("--name")
    cert = add("certificate")
    cert.add_argument("action", choices=["approve", "deny"])
    cert.add_argument("names", nargs="+")
    extra.add_parsers(add)
    cf = add("config")
    cf.add_argument("action", choices=["view", "current-context", "get-contexts", "use-context", "set-cluster",
                                       "set-context", "set-credentials"])
    cf.add_argument("name", nargs="?")
    cf.add_argument("--server", dest="server_url")
    cf.add_argument("--cluster")
    cf.add_argument("--user")
    cf.add_argument("--token", dest="user_token")
    cf.add_argument("--namespace", dest="ctx_namespace")
    return ap


GLOBAL_FLAGS = {"-s", "--server", "--token", "--kubeconfig", "--context", "-n", "--namespace"}


def hoist_global_flags(argv):
    """kubectl accepts its persistent flags anywhere (cobra); move them before the command."""
    front, rest, i = [], [], 0
    while i < len(argv):
        t = argv[i]
        if t == "--":
            rest += argv[i:]
            break
        if t in GLOBAL_FLAGS and i + 1 < len(argv):
            front += [t, argv[i + 1]]
            i += 2
            continue
        if t.split("=", 1)[0] in GLOBAL_FLAGS and "=" in t:
            front.append(t)
            i += 1
            continue
        rest.append(t)
        i += 1
    return front + rest


def main(argv=None, out=sys.stdout):
    ap = build_parser()
    argv = hoist_global_flags(list(sys.argv[1:] if argv is None else argv))
    a = ap.parse_args(argv)
    if a.command == "config":
        cmd_config(a)
        return 0
    if a.command == "completion":
        print(extra.completion(a.shell, ap), file=out)
        return 0
    if a.command == "options":
        print(extra.OPTIONS, file=out)
        return 0
    if a.command == "plugin":
        if not a.plugin_name:
            for n, p in sorted(extra.find_plugins().items()):
                print(f"  {n:<20}{p.get('shortDesc', '')}", file=out)
            return 0
        return extra.run_plugin(a.plugin_name, a.plugin_args, {"server": a.server, "namespace": a.namespace,
                                                              "kubeconfig": a.kubeconfig, "token": a.token})
    k = Kubectl(a, out)
    k.rc = 0
    name = "cmd_" + a.command.replace("-", "_")

    async def go():
        try:
            if k._unknown_names() or getattr(a, "filename", None):
                try:
                    await k.discover()
                except (ConnectionError, OSError, ValueError):
                    pass
            await getattr(k, name)()
        finally:
            await k.client.close()
    try:
        asyncio.run(go())
    except APIStatusError as e:
        print(f"Error from server ({e.reason}): {e.status.get('message', '')}", file=sys.stderr)
        return 1
    except (ConnectionError, OSError) as e:
        print(f"The connection to the server {k.server} was refused - did you specify the right host or port? ({e})", file=sys.stderr)
        return 1
    return k.rc
