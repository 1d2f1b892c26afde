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
from . import config_cmd, extra, printers

DEFAULT_KUBECONFIG = os.path.expanduser("~/.kube/config")


# ---------------------------------------------------------------------------
# kubeconfig
def load_kubeconfig(path=None):
    """-> (merged kubeconfig, the file writes go to); KUBECONFIG may list several files."""
    cfg, files = config_cmd.load(path)
    return cfg, files[0][0]


def save_kubeconfig(cfg, path):
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        yaml.safe_dump(cfg, f, sort_keys=False)


def resolve_server(args):
    """-> (server, token, namespace, ssl context) from flags or the kubeconfig (client-go clientcmd)."""
    server, token, ns, ctx = _resolve_kubeconfig(args)
    # --insecure-skip-tls-verify / --certificate-authority / --client-certificate / --client-key
    # override the kubeconfig's TLS material (clientcmd ConfigOverrides)
    ca, cert, key = (getattr(args, f, None) for f in ("certificate_authority", "client_certificate", "client_key"))
    if server.startswith("https") and (getattr(args, "insecure_skip_tls_verify", False) or ca or cert):
        from ..utils.tlsutil import client_context
        ctx = client_context(None if getattr(args, "insecure_skip_tls_verify", False) else ca, cert, key)
    return server, token, ns, ctx


def _resolve_kubeconfig(args):
    if args.server:
        return args.server, args.token, args.namespace, None
    from ..client import clientcmd
    cfg, path = load_kubeconfig(args.kubeconfig)
    ctx_name = args.context
    if getattr(args, "cluster", None) or getattr(args, "user", None):
        # --cluster / --user override the chosen context's entries
        base = next((c for c in cfg.get("contexts") or () if c["name"] == (ctx_name or cfg.get("current-context"))),
                    {"context": {}})
        ov = dict(base.get("context") or {})
        if getattr(args, "cluster", None):
            ov["cluster"] = args.cluster
        if getattr(args, "user", None):
            ov["user"] = args.user
        cfg = dict(cfg, contexts=list(cfg.get("contexts") or ()) + [{"name": "\0override", "context": ov}])
        ctx_name = "\0override"
    r = clientcmd.resolve(cfg, ctx_name, os.path.dirname(os.path.abspath(path)))
    if r is None:
        return os.environ.get("KUBERNETES_MASTER", "http://127.0.0.1:8080"), args.token, args.namespace, None
    return r.server, args.token or r.token, args.namespace or r.namespace, r.ssl_context


# ---------------------------------------------------------------------------
def read_manifests(paths, recursive=False):
    docs = []
    for p in paths:
        files = []
        if p == "-":
            text = sys.stdin.read()
            files.append(text)
        elif os.path.isdir(p):
            walk = os.walk(p) if recursive else [(p, [], os.listdir(p))]
            for dp, _dn, fns in walk:
                for fn in sorted(fns):
                    if fn.endswith((".yaml", ".yml", ".json")):
                        files.append(open(os.path.join(dp, fn)).read())
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


# kubectl 1.9 prefixes names in multi-kind tables with the short resource name (po/…, svc/…)
_SHORT_KIND = {"Pod": "po", "Service": "svc", "Deployment": "deploy", "ReplicaSet": "rs", "ReplicationController": "rc",
               "DaemonSet": "ds", "StatefulSet": "statefulsets", "Job": "jobs", "CronJob": "cronjobs",
               "HorizontalPodAutoscaler": "hpa", "Node": "no", "Namespace": "ns", "ConfigMap": "cm", "Secret": "secrets",
               "Endpoints": "ep", "ServiceAccount": "sa", "PersistentVolume": "pv", "PersistentVolumeClaim": "pvc"}
ALL_CATEGORY = ["pods", "replicationcontrollers", "services", "daemonsets", "deployments", "replicasets",
                "statefulsets", "horizontalpodautoscalers", "jobs", "cronjobs"]


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
    kinds = []
    for k in targets[0].split(","):
        # the `all` category (`pkg/kubectl/categories.go` legacyUserResources)
        kinds += ALL_CATEGORY if k == "all" else [k]
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


def _duration_s(v) -> float:
    """--request-timeout: `0` (none), a bare number of seconds, or 1s / 2m / 3h."""
    v = str(v or "0").strip()
    if v in ("", "0"):
        return 0.0
    if v[-1].isdigit():
        return float(v)
    from ..kubelet.eviction import parse_duration
    return float(parse_duration(v))


def rollout_status(obj, revision=0):
    """-> (message, done) for a Deployment, DaemonSet or StatefulSet (`pkg/kubectl/rollout_status.go`
    DeploymentStatusViewer / DaemonSetStatusViewer / StatefulSetStatusViewer)."""
    kind, name = obj.get("kind"), obj["metadata"]["name"]
    spec, st = obj.get("spec") or {}, obj.get("status") or {}
    gen, observed = obj["metadata"].get("generation", 0), st.get("observedGeneration", 0)
    if kind == "DaemonSet":
        if (spec.get("updateStrategy") or {}).get("type", "OnDelete") != "RollingUpdate":
            raise SystemExit("error: Status is available only for RollingUpdate strategy type")
        if gen > (observed or 0):
            return "Waiting for daemon set spec update to be observed...", False
        want, upd, avail = st.get("desiredNumberScheduled", 0), st.get("updatedNumberScheduled", 0), st.get("numberAvailable", 0)
        if upd < want:
            return f"Waiting for rollout to finish: {upd} out of {want} new pods have been updated...", False
        if avail < want:
            return f"Waiting for rollout to finish: {avail} of {want} updated pods are available...", False
        return f'daemon set "{name}" successfully rolled out', True
    if kind == "StatefulSet":
        us = spec.get("updateStrategy") or {}
        if us.get("type", "RollingUpdate") == "OnDelete":
            raise SystemExit("error: OnDelete updateStrategy does not have a Status`")
        if st.get("observedGeneration") is None or gen > st["observedGeneration"]:
            return "Waiting for statefulset spec update to be observed...", False
        want = spec.get("replicas")
        if want is not None and st.get("readyReplicas", 0) < want:
            return f"Waiting for {want - st.get('readyReplicas', 0)} pods to be ready...", False
        if us.get("type") == "RollingUpdate" and us.get("rollingUpdate") is not None:
            part = us["rollingUpdate"].get("partition")
            if want is not None and part is not None and st.get("updatedReplicas", 0) < want - part:
                return (f"Waiting for partitioned roll out to finish: {st.get('updatedReplicas', 0)} out of "
                        f"{want - part} new pods have been updated..."), False
            return f"partitioned roll out complete: {st.get('updatedReplicas', 0)} new pods have been updated...", True
        if st.get("updateRevision") != st.get("currentRevision"):
            return (f"waiting for statefulset rolling update to complete {st.get('updatedReplicas', 0)} pods at "
                    f"revision {st.get('updateRevision')}..."), False
        return (f"statefulset rolling update complete {st.get('currentReplicas', 0)} pods at revision "
                f"{st.get('currentRevision')}..."), True
    if revision:
        cur = int((obj["metadata"].get("annotations") or {}).get("deployment.kubernetes.io/revision") or 0)
        if cur != revision:
            raise SystemExit(f"error: desired revision ({revision}) is different from the running revision ({cur})")
    if gen > observed:
        return "Waiting for deployment spec update to be observed...", False
    for c in st.get("conditions") or ():
        if c.get("type") == "Progressing" and c.get("reason") == "ProgressDeadlineExceeded":
            raise SystemExit(f'error: deployment "{name}" exceeded its progress deadline')
    want = spec.get("replicas")
    upd, total, avail = st.get("updatedReplicas", 0), st.get("replicas", 0), st.get("availableReplicas", 0)
    if want is not None and upd < want:
        return f'Waiting for rollout to finish: {upd} out of {want} new replicas have been updated...', False
    if total > upd:
        return f"Waiting for rollout to finish: {total - upd} old replicas are pending termination...", False
    if avail < upd:
        return f"Waiting for rollout to finish: {avail} of {upd} updated replicas are available...", False
    return f'deployment "{name}" successfully rolled out', True


class Kubectl(extra.ExtraCommands):
    def __init__(self, args, out=sys.stdout):
        self.a = args
        self.out = out
        server, token, ns, ctx = resolve_server(args)
        self.server = server
        self.ns = ns or "default"
        self.client = Client(server, token=token, ssl_context=ctx,
                             timeout=_duration_s(getattr(args, "request_timeout", "0")) or 60.0)
        hdrs = {}
        if getattr(args, "as_user", None):
            hdrs["Impersonate-User"] = args.as_user
        if getattr(args, "as_group", None):
            hdrs["Impersonate-Group"] = ",".join(args.as_group)
        if getattr(args, "username", None) and not token:
            import base64
            hdrs["Authorization"] = "Basic " + base64.b64encode(
                f"{args.username}:{args.password or ''}".encode()).decode()
        if hdrs:
            self.client.http.set_default_headers(hdrs)

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
    def _render(self, objs, kind=None, list_obj=None, all_ns=False):
        a = self.a
        return printers.render(objs, a.output, kind, a.output == "wide", all_ns, list_obj=list_obj,
                               sort_by=getattr(a, "sort_by", ""), no_headers=getattr(a, "no_headers", False),
                               show_labels=getattr(a, "show_labels", False),
                               label_columns=getattr(a, "label_columns", ()), show_kind=getattr(a, "show_kind", False))

    async def cmd_get(self):
        a = self.a
        if a.raw:
            st, body = await self.client.raw("GET", a.raw)
            if st != 200:
                raise SystemExit(f"error: {body.decode(errors='replace')}")
            self.out.write(body.decode(errors="replace") + ("" if body.endswith(b"\n") else "\n"))
            return
        if a.filename:
            objs = []
            for d in read_manifests(a.filename, a.recursive):
                ri = ri_for_obj(d)
                try:
                    objs.append(await self.client.get(ri.plural, d["metadata"]["name"], self.ns_for(ri, d)))
                except APIStatusError as e:
                    if not (a.ignore_not_found and is_not_found(e)):
                        raise
            self.p(self._render(objs))
            return
        targets = split_targets(a.targets)
        multi = len({ri.plural for ri, _ in targets}) > 1 and not any(n for _, n in targets)
        printed = False
        for ri, name in targets:
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
                    try:
                        obj = await self.client.get(ri.plural, name, ns)
                    except APIStatusError as e:
                        if a.ignore_not_found and is_not_found(e):
                            continue
                        raise
                self.p(self._render([obj], ri.kind))
                continue
            extra = {"includeUninitialized": "true"} if a.include_uninitialized else None
            lst = {"kind": f"{ri.kind}List", "items": [], "metadata": {}}
            cont = None
            while True:                    # chunked list (--chunk-size, limit/continue)
                page = await self.client.list(ri.plural, ns, a.selector, a.field_selector, limit=a.chunk_size or 0,
                                              cont=cont, extra=extra)
                lst["items"] += page.get("items") or []
                lst["metadata"] = page.get("metadata") or {}
                cont = lst["metadata"].get("continue")
                if not cont or not a.chunk_size:
                    break
            lst["apiVersion"] = page.get("apiVersion", "v1")
            if ri.kind == "Pod" and not getattr(a, "show_all", False):
                # `resource_filter.go` filterPods: a list hides terminated (Succeeded / Failed)
                # pods unless --show-all; a named pod is always shown
                lst["items"] = [p for p in lst["items"]
                                if (p.get("status") or {}).get("phase") not in ("Succeeded", "Failed")]
            items = lst["items"]
            for o in items:
                o.setdefault("kind", ri.kind)
            if a.watch or a.watch_only:
                if not a.watch_only:
                    self.p(self._render(items, ri.kind, all_ns=a.all_namespaces))
                st = await self.client.watch(ri.plural, ns, lst["metadata"]["resourceVersion"], a.selector, a.field_selector)
                async for t, o in st:
                    rows, h = printers.rows_for(ri.kind, [o], a.output == "wide")
                    self.p(printers.table(rows, h).splitlines()[-1])
                return
            if multi and (not a.output or a.output == "wide"):
                # several kinds (`get all`, `get po,svc`): each non-empty table, names as kind/name
                if items:
                    prefix = _SHORT_KIND.get(ri.kind, ri.kind.lower())
                    shown = [dict(o, metadata=dict(o["metadata"], name=f"{prefix}/{o['metadata']['name']}"))
                             for o in items]
                    if printed:
                        self.p("")
                    self.p(self._render(shown, ri.kind, all_ns=a.all_namespaces))
                    printed = True
                continue
            self.p(self._render(items, ri.kind, list_obj=lst if a.output in ("json", "yaml") else None,
                                all_ns=a.all_namespaces))
        if multi and not printed and (not a.output or a.output == "wide"):
            self.p("No resources found.")

    async def cmd_describe(self):
        a = self.a
        targets = []
        if a.filename:
            for d in read_manifests(a.filename, a.recursive):
                ri = ri_for_obj(d)
                targets.append((ri, d["metadata"]["name"], self.ns_for(ri, d)))
        else:
            targets = [(ri, name, None if not ri.namespaced or a.all_namespaces else self.ns)
                       for ri, name in split_targets(a.targets)]
        for ri, name, ns in targets:
            if name:
                objs = [await self.client.get(ri.plural, name, ns)]
            else:
                objs = (await self.client.list(ri.plural, ns, a.selector))["items"]
            for o in objs:
                o.setdefault("kind", ri.kind)
                evs = []
                from .describe import gather
                ctx = await gather(self.client, o)
                if not a.show_events:
                    self.p(printers.describe(o, [], ctx))
                    self.p("")
                    continue
                try:
                    fs = f"involvedObject.name={o['metadata']['name']},involvedObject.kind={ri.kind}"
                    evs = (await self.client.list("events", o["metadata"].get("namespace") or "default", field_selector=fs))["items"]
                except APIStatusError:
                    pass
                self.p(printers.describe(o, evs, ctx))
                self.p("")

    LAST_APPLIED = "kubectl.kubernetes.io/last-applied-configuration"
    CHANGE_CAUSE = "kubernetes.io/change-cause"

    def _record(self, d):
        """--record: the command line as the object's change-cause annotation."""
        if getattr(self.a, "record", False):
            d.setdefault("metadata", {}).setdefault("annotations", {})[self.CHANGE_CAUSE] = \
                "kubectl " + " ".join(sys.argv[1:])

    async def _wait_gone(self, ri, name, ns, timeout):
        end = time.monotonic() + timeout
        while time.monotonic() < end:
            try:
                await self.client.get(ri.plural, name, ns)
            except APIStatusError as e:
                if is_not_found(e):
                    return True
                raise
            await asyncio.sleep(0.1)
        return False

    async def _apply_one(self, d, mode):
        a = self.a
        ri = ri_for_obj(d)
        ns = self.ns_for(ri, d)
        if ri.namespaced:
            d.setdefault("metadata", {})["namespace"] = ns
        name = d["metadata"].get("name")
        self._record(d)
        if getattr(a, "save_config", False) or mode == "apply":
            d["metadata"].setdefault("annotations", {})[self.LAST_APPLIED] = json.dumps(
                {k: v for k, v in d.items() if k != "status"}, sort_keys=True)
        verb = "created"
        out = d
        if a.dry_run:
            verb = {"create": "created", "replace": "replaced"}.get(mode, "configured") + " (dry run)"
        elif mode == "create":
            out = await self.client.create(ri.plural, d, ns)
        elif mode == "replace":
            if a.force:
                # --force: delete, wait for it to be gone, create (pkg/kubectl/cmd/replace.go forceReplace)
                try:
                    await self.client.delete(ri.plural, name, ns, grace_period=None if a.grace_period < 0 else a.grace_period,
                                             propagation=None if a.cascade else "Orphan")
                except APIStatusError as e:
                    if not is_not_found(e):
                        raise
                if not await self._wait_gone(ri, name, ns, a.timeout or 60):
                    raise SystemExit(f"error: timed out waiting for {ri.plural}/{name} to be deleted")
                d["metadata"].pop("resourceVersion", None)
                out = await self.client.create(ri.plural, d, ns)
            else:
                cur = await self.client.get(ri.plural, name, ns)
                d["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
                out = await self.client.update(ri.plural, d, ns)
            verb = "replaced"
        else:  # apply: create, or patch with the difference to the last-applied configuration
            try:
                out = await self.client.create(ri.plural, d, ns)
            except APIStatusError as e:
                if not is_already_exists(e):
                    raise
                try:
                    out = await self.client.patch(ri.plural, name, d, ns, "strategic")
                except APIStatusError as pe:
                    if not (a.force and pe.code in (409, 422)):
                        raise
                    # --force: a patch the server refuses (immutable field) becomes delete + create
                    await self.client.delete(ri.plural, name, ns,
                                             grace_period=None if a.grace_period < 0 else a.grace_period)
                    await self._wait_gone(ri, name, ns, a.timeout or 60)
                    out = await self.client.create(ri.plural, d, ns)
                verb = "configured"
        if a.output:
            self.p(printers.render([out], a.output, ri.kind))
        else:
            self.p(f"{ri.kind.lower()}/{name} {verb}")
        return ri, name, ns

    async def cmd_create(self):
        a = self.a
        if a.edit:
            raise SystemExit("error: --edit is not supported here; use kubectl create -f then kubectl edit")
        if a.raw:
            if not a.filename:
                raise SystemExit("error: --raw requires -f")
            data = sys.stdin.buffer.read() if a.filename[0] == "-" else open(a.filename[0], "rb").read()
            st, body = await self.client.raw("POST", a.raw, data)
            if st >= 300:
                raise SystemExit(f"error: {body.decode(errors='replace')}")
            self.out.write(body.decode(errors="replace") + "\n")
            return
        if a.generator:
            await self._create_generated(a.generator)
            return
        if not a.filename:
            raise SystemExit("error: must specify one of -f and a resource generator (e.g. create namespace NAME)")
        for d in read_manifests(a.filename, a.recursive):
            await self._apply_one(d, "create")

    async def cmd_apply(self):
        a = self.a
        applied = set()
        for d in read_manifests(a.filename, a.recursive):
            ri, name, ns = await self._apply_one(d, "apply")
            applied.add((ri.plural, ns, name))
        if a.prune:
            await self._prune(applied)

    async def _prune(self, applied):
        """--prune (pkg/kubectl/cmd/apply.go prune): delete objects of the applied kinds that
        carry a last-applied annotation, match -l (or --all) and were not in this apply."""
        a = self.a
        if not a.selector and not a.all:
            raise SystemExit("error: all resources selected for prune without explicitly passing --all")
        kinds = {m.lookup(w.rsplit("/", 1)[-1]) for w in a.prune_whitelist} - {None} if a.prune_whitelist else \
            {m.BY_PLURAL[p] for p, _ns, _n in applied}
        namespaces = {ns for _p, ns, _n in applied}
        for ri in kinds:
            for ns in (namespaces if ri.namespaced else {None}):
                for o in (await self.client.list(ri.plural, ns, a.selector))["items"]:
                    md = o["metadata"]
                    if (ri.plural, ns, md["name"]) in applied or self.LAST_APPLIED not in (md.get("annotations") or {}):
                        continue
                    if not a.dry_run:
                        await self.client.delete(ri.plural, md["name"], ns)
                    self.p(f"{ri.kind.lower()}/{md['name']} pruned" + (" (dry run)" if a.dry_run else ""))

    async def cmd_replace(self):
        for d in read_manifests(self.a.filename, self.a.recursive):
            await self._apply_one(d, "replace")

    async def _last_applied_targets(self):
        a = self.a
        if a.filename:
            return [(ri_for_obj(d), d) for d in read_manifests(a.filename, a.recursive)]
        out = []
        for ri, name in split_targets(a.targets):
            ns = self.ns if ri.namespaced else None
            if name:
                out.append((ri, await self.client.get(ri.plural, name, ns)))
            elif a.all or a.selector:
                out += [(ri, o) for o in (await self.client.list(ri.plural, ns, a.selector))["items"]]
            else:
                raise SystemExit("error: a resource name, -l or --all is required")
        return out

    async def cmd_apply_view_last_applied(self):
        """`kubectl apply view-last-applied` (pkg/kubectl/cmd/apply_view_last_applied.go)."""
        a = self.a
        for ri, o in await self._last_applied_targets():
            if a.filename:
                o = await self.client.get(ri.plural, o["metadata"]["name"], self.ns_for(ri, o))
            ann = (o["metadata"].get("annotations") or {}).get(self.LAST_APPLIED)
            if ann is None:
                raise SystemExit(f"error: no last-applied-configuration annotation found on resource: {o['metadata']['name']}")
            cfg = json.loads(ann)
            self.p(json.dumps(cfg, indent=2) if a.output == "json" else yaml.safe_dump(cfg, sort_keys=False).rstrip())

    async def cmd_apply_set_last_applied(self):
        """`kubectl apply set-last-applied -f FILE`: overwrite the annotation with the file's
        content; without --create-annotation the object must already carry one."""
        a = self.a
        if not a.filename:
            raise SystemExit("error: -f is required for set-last-applied")
        for ri, d in await self._last_applied_targets():
            ns = self.ns_for(ri, d)
            cur = await self.client.get(ri.plural, d["metadata"]["name"], ns)
            if self.LAST_APPLIED not in (cur["metadata"].get("annotations") or {}) and not a.create_annotation:
                raise SystemExit(f"error: no last-applied-configuration annotation found on resource: "
                                 f"{d['metadata']['name']}, to create the annotation, run the command with --create-annotation")
            d = json.loads(json.dumps(d))
            (d["metadata"].get("annotations") or {}).pop(self.LAST_APPLIED, None)
            patch = {"metadata": {"annotations": {self.LAST_APPLIED: json.dumps(d, sort_keys=True, separators=(",", ":"))}}}
            if a.dry_run:
                self.p(f"{ri.kind.lower()}/{d['metadata']['name']} configured (dry run)")
                continue
            out = await self.client.patch(ri.plural, d["metadata"]["name"], patch, ns, "merge")
            self.p(printers.render([out], a.output, ri.kind) if a.output else f"{ri.kind.lower()}/{d['metadata']['name']} configured")

    async def cmd_apply_edit_last_applied(self):
        """`kubectl apply edit-last-applied`: $EDITOR over the annotation, written back."""
        import subprocess
        import tempfile
        a = self.a
        for ri, o in await self._last_applied_targets():
            if a.filename:
                o = await self.client.get(ri.plural, o["metadata"]["name"], self.ns_for(ri, o))
            ann = (o["metadata"].get("annotations") or {}).get(self.LAST_APPLIED)
            if ann is None:
                raise SystemExit(f"error: no last-applied-configuration annotation found on resource: {o['metadata']['name']}")
            cfg = json.loads(ann)
            text = json.dumps(cfg, indent=2) + "\n" if a.output == "json" else yaml.safe_dump(cfg, sort_keys=False)
            with tempfile.NamedTemporaryFile("w", suffix="." + a.output, delete=False) as f:
                f.write(text)
                path = f.name
            try:
                editor = os.environ.get("KUBE_EDITOR") or os.environ.get("EDITOR") or "vi"
                if subprocess.call(editor.split() + [path]) != 0:
                    raise SystemExit("error: editor failed")
                with open(path) as f:
                    new_text = f.read()
            finally:
                os.unlink(path)
            if new_text == text:
                self.p("Edit cancelled, no changes made.")
                continue
            new = yaml.safe_load(new_text)
            patch = {"metadata": {"annotations": {self.LAST_APPLIED: json.dumps(new, sort_keys=True, separators=(",", ":"))}}}
            await self.client.patch(ri.plural, o["metadata"]["name"], patch, o["metadata"].get("namespace"), "merge")
            self.p(f"{ri.kind.lower()}/{o['metadata']['name']} edited")

    async def cmd_delete(self):
        a = self.a
        targets = []
        if a.filename:
            for d in read_manifests(a.filename, a.recursive):
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
        grace = a.grace_period
        if a.force:
            grace = 0
            print("warning: Immediate deletion does not wait for confirmation that the running resource has been "
                  "terminated. The resource may continue to run on the cluster indefinitely.", file=sys.stderr)
        elif a.now:
            grace = 1
        deleted = []
        for ri, name, ns in targets:
            try:
                await self.client.delete(ri.plural, name, ns, grace_period=grace,
                                         propagation=None if a.cascade else "Orphan")
                self.p(f"{ri.kind.lower()}/{name}" if a.output == "name" else f'{ri.kind.lower()} "{name}" deleted')
                deleted.append((ri, name, ns))
            except APIStatusError as e:
                if is_not_found(e) and a.ignore_not_found:
                    continue
                raise
        if a.timeout:
            for ri, name, ns in deleted:
                if not await self._wait_gone(ri, name, ns, a.timeout):
                    raise SystemExit(f"error: timed out waiting for {ri.plural}/{name} to be deleted")

    async def _pods_for(self, ref, selector=None):
        """`pod`, `pod/x`, `deployment/x` (its first pod, as `logs` / `attach` resolve controller
        references) or -l SELECTOR -> pod names."""
        if selector:
            return [p["metadata"]["name"] for p in (await self.client.list("pods", self.ns, selector))["items"]]
        if not ref:
            raise SystemExit("error: expected POD or TYPE/NAME, or -l")
        kind, _, name = ref.partition("/") if "/" in ref else ("pod", "", ref)
        ri = m.lookup(kind)
        if ri is None or ri.kind == "Pod":
            return [name]
        obj = await self.client.get(ri.plural, name, self.ns)
        sel = ((obj.get("spec") or {}).get("selector") or {})
        sel = sel.get("matchLabels", sel) if isinstance(sel, dict) else {}
        pods = (await self.client.list("pods", self.ns, ",".join(f"{k}={v}" for k, v in sorted(sel.items()))))["items"]
        pods.sort(key=lambda p: (p.get("status") or {}).get("phase") != "Running")
        if not pods:
            raise SystemExit(f"error: no pods found for {ref}")
        return [pods[0]["metadata"]["name"]]

    async def cmd_logs(self):
        """`kubectl logs` (pkg/kubectl/cmd/logs.go): -c, --tail (10 by default with -l), -p,
        -f, --since / --since-time, --timestamps, --limit-bytes, TYPE/NAME and -l."""
        from urllib.parse import urlencode
        a = self.a
        pods = await self._pods_for(a.pod, a.selector)
        container = a.container or a.container_pos
        q = {}
        if container:
            q["container"] = container
        tail = a.tail if a.tail is not None else (10 if a.selector else None)
        if tail is not None and tail >= 0:
            q["tailLines"] = str(tail)
        if a.previous:
            q["previous"] = "true"
        if a.since and a.since_time:
            raise SystemExit("error: at most one of `sinceTime` or `sinceSeconds` may be specified")
        if a.since:
            from ..kubelet.eviction import parse_duration
            q["sinceSeconds"] = str(int(parse_duration(a.since)))
        if a.since_time:
            q["sinceTime"] = a.since_time
        if a.timestamps:
            q["timestamps"] = "true"
        if a.limit_bytes:
            q["limitBytes"] = str(a.limit_bytes)
        if a.follow:
            if len(pods) > 1:
                raise SystemExit("error: only one pod can be followed")
            q["follow"] = "true"
        for name in pods:
            path = f"/api/v1/namespaces/{self.ns}/pods/{name}/log" + (f"?{urlencode(q)}" if q else "")
            if a.follow:
                st, hdrs, r, w = await self.client.http.open_raw("GET", path)
                try:
                    if st != 200:
                        raise SystemExit(f"error: {(await r.read(1 << 16)).decode(errors='replace')}")
                    while True:
                        n = int((await r.readuntil(b"\r\n")).split(b";")[0].strip() or b"0", 16)
                        if n == 0:
                            break
                        self.out.write((await r.readexactly(n)).decode(errors="replace"))
                        if hasattr(self.out, "flush"):
                            self.out.flush()
                        await r.readexactly(2)
                except asyncio.IncompleteReadError:
                    pass
                finally:
                    w.close()
                continue
            st, body = await self.client.raw("GET", path)
            if st != 200:
                raise SystemExit(f"error: {body.decode(errors='replace')}")
            self.out.write(body.decode(errors="replace"))

    async def _meta_edit(self, field):
        """`kubectl label` / `annotate` (pkg/kubectl/cmd/label.go): KEY=VAL and KEY- pairs; changing
        an existing key needs --overwrite; --all / -l pick objects; --resource-version is a
        precondition; --local / --dry-run print instead of writing; label --list prints."""
        a = self.a
        pairs = list(a.pairs)
        objs = []
        if a.filename:
            pairs = [x for x in (a.resource, a.name) if x] + pairs    # with -f every positional is a pair
            for d in read_manifests(a.filename, a.recursive):
                ri = ri_for_obj(d)
                objs.append((ri, d if a.local else await self.client.get(ri.plural, d["metadata"]["name"], self.ns_for(ri, d))))
        else:
            if "/" in a.resource:
                kind, _, name = a.resource.partition("/")
            else:
                kind, name = a.resource, a.name
                if name and ("=" in name or name.endswith("-")):
                    pairs.insert(0, name)      # `kubectl label pods -l x=y k=v`: no name given
                    name = None
            ri = m.lookup(kind)
            if ri is None:
                raise SystemExit(f'error: the server doesn\'t have a resource type "{kind}"')
            ns = self.ns if ri.namespaced else None
            if name:
                objs.append((ri, await self.client.get(ri.plural, name, ns)))
            elif a.all or a.selector:
                objs += [(ri, o) for o in (await self.client.list(ri.plural, ns, a.selector))["items"]]
            else:
                raise SystemExit("error: one or more resources must be specified as <resource> <name> or <resource>/<name>")
        if field == "labels" and getattr(a, "list", False):
            for ri, o in objs:
                for k, v in sorted(((o.get("metadata") or {}).get("labels") or {}).items()):
                    self.p(f"{k}={v}")
            return
        if not pairs:
            raise SystemExit(f"error: at least one {field[:-1]} update is required")
        patch = {}
        for p in pairs:
            if p.endswith("-"):
                patch[p[:-1]] = None
            else:
                k, _, v = p.partition("=")
                patch[k] = v
        for ri, o in objs:
            md = o.get("metadata") or {}
            cur = md.get(field) or {}
            if not a.overwrite:
                for k, v in patch.items():
                    if v is not None and k in cur and cur[k] != v:
                        raise SystemExit(f"error: '{k}' already has a value ({cur[k]}), and --overwrite is false")
            n = md["name"]
            body = {"metadata": {field: patch}}
            if a.resource_version:
                body["metadata"]["resourceVersion"] = a.resource_version
            if a.local or a.dry_run:
                new = dict(cur)
                for k, v in patch.items():
                    if v is None:
                        new.pop(k, None)
                    else:
                        new[k] = v
                out = dict(o, metadata=dict(md, **{field: new}))
            else:
                out = await self.client.patch(ri.plural, n, body, md.get("namespace") if ri.namespaced else None)
            if a.output:
                self.p(printers.render([out], a.output, ri.kind))
            else:
                self.p(f"{ri.kind.lower()}/{n} {'labeled' if field == 'labels' else 'annotated'}"
                       + (" (dry run)" if a.dry_run else ""))

    async def cmd_label(self):
        await self._meta_edit("labels")

    async def cmd_annotate(self):
        await self._meta_edit("annotations")

    async def cmd_patch(self):
        a = self.a
        patch = json.loads(a.patch) if a.patch.strip().startswith(("{", "[")) else yaml.safe_load(a.patch)
        if a.filename:
            docs = read_manifests(a.filename, a.recursive)
            targets = [(ri_for_obj(d), d) for d in docs]
        else:
            targets = [(ri, name) for ri, name in split_targets(a.targets)]
        for ri, t in targets:
            name = t["metadata"]["name"] if isinstance(t, dict) else t
            if a.local or a.dry_run:
                from ..utils.patch import apply_patch
                base = t if isinstance(t, dict) and a.local else await self.client.get(ri.plural, name, self.ns if ri.namespaced else None)
                ctype = {"strategic": "application/strategic-merge-patch+json", "merge": "application/merge-patch+json",
                         "json": "application/json-patch+json"}[a.type]
                out = apply_patch(ctype, base, patch)
            else:
                out = await self.client.patch(ri.plural, name, patch, self.ns if ri.namespaced else None, a.type)
            if a.output:
                self.p(printers.render([out], a.output, ri.kind))
            else:
                self.p(f"{ri.kind.lower()}/{name} patched" + (" (dry run)" if a.dry_run else ""))

    async def cmd_scale(self):
        """`kubectl scale` (pkg/kubectl/scale.go): through the scale subresource, with the
        --current-replicas / --resource-version preconditions checked against the Scale; Jobs
        (parallelism) are patched directly."""
        a = self.a
        targets = []
        if a.filename:
            targets = [(ri_for_obj(d), d["metadata"]["name"]) for d in read_manifests(a.filename, a.recursive)]
        else:
            for ri, name in split_targets(a.targets):
                if name:
                    targets.append((ri, name))
                elif a.all or a.selector:
                    targets += [(ri, o["metadata"]["name"]) for o in (await self.client.list(ri.plural, self.ns, a.selector))["items"]]
                else:
                    raise SystemExit("error: resource(s) were provided, but no name, label selector, or --all flag specified")
        for ri, name in targets:
            if ri.plural == "jobs":
                job = await self.client.get("jobs", name, self.ns)
                cur = (job.get("spec") or {}).get("parallelism", 1)
                if a.current_replicas is not None and a.current_replicas != cur:
                    raise SystemExit(f"error: Expected replicas to be {a.current_replicas}, was {cur}")
                await self.client.patch("jobs", name, {"spec": {"parallelism": a.replicas}}, self.ns)
            else:
                # ScaleWithRetries (pkg/kubectl/scale.go): a conflict from a concurrent status
                # write is retried against the fresh Scale; the preconditions are re-checked
                for attempt in range(8):
                    scale = await self.client.get(ri.plural, name, self.ns, subresource="scale")
                    cur = (scale.get("spec") or {}).get("replicas", 0)
                    if a.current_replicas is not None and a.current_replicas != cur:
                        raise SystemExit(f"error: Expected replicas to be {a.current_replicas}, was {cur}")
                    if a.resource_version and a.resource_version != scale["metadata"].get("resourceVersion"):
                        raise SystemExit(f"error: Expected resourceVersion to be {a.resource_version}, "
                                         f"was {scale['metadata'].get('resourceVersion')}")
                    scale["spec"] = {"replicas": a.replicas}
                    try:
                        await self.client.update(ri.plural, scale, self.ns, subresource="scale")
                        break
                    except APIStatusError as e:
                        if e.code != 409 or a.resource_version or attempt == 7:
                            raise
                        await asyncio.sleep(0.01 * (attempt + 1))
            self.p(f"{ri.kind.lower()} \"{name}\" scaled")
            if a.timeout and ri.plural != "jobs":
                end = time.monotonic() + a.timeout
                while True:        # --timeout: wait until the new size is ready (ScalePrecondition + waitForReplicas)
                    o = await self.client.get(ri.plural, name, self.ns)
                    st = o.get("status") or {}
                    if int(st.get("readyReplicas", st.get("replicas", 0)) or 0) == a.replicas and \
                            int(st.get("replicas", 0) or 0) == a.replicas:
                        break
                    if time.monotonic() > end:
                        raise SystemExit(f"error: timed out waiting for {ri.plural}/{name} to reach {a.replicas} replicas")
                    await asyncio.sleep(0.2)

    async def _cordon(self, name, flag):
        await self.client.patch("nodes", name, {"spec": {"unschedulable": flag or None}})
        self.p(f"node/{name} {'cordoned' if flag else 'uncordoned'}")

    async def _cordon_all(self, flag):
        """cordon / uncordon NODE, or every node matching -l; --dry-run only reports; a node
        already in the wanted state is reported as such (`drain.go` RunCordonOrUncordon)."""
        a = self.a
        if a.selector:
            nodes = (await self.client.list("nodes", None, a.selector))["items"]
        elif a.node:
            nodes = [await self.client.get("nodes", a.node)]
        else:
            raise SystemExit("error: USAGE: cordon NODE [flags] (or -l SELECTOR)")
        word = "cordoned" if flag else "uncordoned"
        for n in nodes:
            name = n["metadata"]["name"]
            if bool((n.get("spec") or {}).get("unschedulable")) == flag:
                self.p(f"node/{name} already {word}")
            elif a.dry_run:
                self.p(f"node/{name} {word} (dry run)")
            else:
                await self._cordon(name, flag)

    async def cmd_cordon(self):
        await self._cordon_all(True)

    async def cmd_uncordon(self):
        await self._cordon_all(False)

    async def cmd_drain(self):
        """`kubectl drain` (pkg/kubectl/cmd/drain.go): cordon, then evict every pod except mirror
        pods (and DaemonSet pods with --ignore-daemonsets); unmanaged pods need --force, pods with
        emptyDir data need --delete-local-data; --timeout bounds the whole drain."""
        a = self.a
        if a.selector:
            nodes = [n["metadata"]["name"] for n in (await self.client.list("nodes", None, a.selector))["items"]]
        elif a.node:
            nodes = [a.node]
        else:
            raise SystemExit("error: USAGE: drain NODE [flags] (or -l SELECTOR)")
        end = time.monotonic() + a.timeout if a.timeout else None
        for node in nodes:
            pods = (await self.client.list("pods", None, field_selector=f"spec.nodeName={node}"))["items"]
            victims, errors = [], []
            for p in pods:
                md = p["metadata"]
                if "kubernetes.io/config.mirror" in (md.get("annotations") or {}):
                    continue                                     # static pods: the kubelet owns them
                if core.pod_is_terminal(p):
                    continue
                ref = m.controller_of(p)
                if ref and ref.get("kind") == "DaemonSet":
                    if a.ignore_daemonsets:
                        continue
                    errors.append(f"DaemonSet-managed pods (use --ignore-daemonsets to ignore): {md['name']}")
                    continue
                if not ref and not a.force:
                    errors.append(f"pods not managed by ReplicationController, ReplicaSet, Job, DaemonSet or "
                                  f"StatefulSet (use --force to override): {md['name']}")
                    continue
                if any("emptyDir" in v for v in (p.get("spec") or {}).get("volumes") or ()) and not a.delete_local_data:
                    errors.append(f"pods with local storage (use --delete-local-data to override): {md['name']}")
                    continue
                victims.append(p)
            if errors:
                raise SystemExit("error: unable to drain node " + repr(node) + ", aborting command...\n\n"
                                 + "\n".join(errors))
            if a.dry_run:
                self.p(f"node/{node} cordoned (dry run)")
                for p in victims:
                    self.p(f"pod/{p['metadata']['name']} evicted (dry run)")
                self.p(f"node/{node} drained (dry run)")
                continue
            await self._cordon(node, True)
            left = None if end is None else max(0.0, end - time.monotonic())
            try:
                await asyncio.wait_for(asyncio.gather(*(self._evict_and_wait(p) for p in victims)), left)
            except asyncio.TimeoutError:
                raise SystemExit(f"error: Drain did not complete within {a.timeout}s")
            self.p(f"node/{node} drained")

    DRAIN_RETRY = 5.0           # drain.go evictPods: sleep after 429 TooManyRequests
    DRAIN_POLL = 1.0            # kubectl.Interval for waitForDelete

    async def _evict_and_wait(self, p):
        """`evictPods` / `waitForDelete`: evict, retrying while a disruption budget refuses (429);
        then wait until the pod is gone or replaced by a new pod of the same name (UID)."""
        ns, name, uid = p["metadata"]["namespace"], p["metadata"]["name"], p["metadata"].get("uid")
        while True:
            try:
                await self.client.evict(ns, name, self.a.grace_period)
                break
            except APIStatusError as e:
                if is_not_found(e):
                    self.p(f"pod/{name} evicted")
                    return
                if e.code != 429:
                    raise SystemExit(f"error: error when evicting pod {name!r}: {e}")
                await asyncio.sleep(self.DRAIN_RETRY)
        while True:
            try:
                cur = await self.client.get("pods", name, ns)
            except APIStatusError as e:
                if not is_not_found(e):
                    raise SystemExit(f"error: error when waiting for pod {name!r} terminating: {e}")
                break
            if cur["metadata"].get("uid") != uid:
                break
            await asyncio.sleep(self.DRAIN_POLL)
        self.p(f"pod/{name} evicted")

    async def cmd_taint(self):
        """`kubectl taint` (pkg/kubectl/cmd/taint.go): KEY=VAL:EFFECT adds (an existing key+effect
        needs --overwrite), KEY:EFFECT- / KEY- remove; --all / -l for several nodes."""
        a = self.a
        specs = list(a.taints)
        if a.node and (":" in a.node or a.node.endswith("-")) and (a.all or a.selector):
            specs.insert(0, a.node)
            a.node = None
        if a.node:
            names = [a.node]
        elif a.all or a.selector:
            names = [n["metadata"]["name"] for n in (await self.client.list("nodes", None, a.selector))["items"]]
        else:
            raise SystemExit("error: at least one node (or --all / -l) is required")
        for name in names:
            node = await self.client.get("nodes", name)
            taints = list((node.get("spec") or {}).get("taints") or [])
            for t in specs:
                if t.endswith("-"):
                    key, _, eff = t[:-1].partition(":")
                    key = key.split("=")[0]
                    taints = [x for x in taints if not (x["key"] == key and (not eff or x["effect"] == eff))]
                    continue
                kv, _, eff = t.partition(":")
                if eff not in ("NoSchedule", "PreferNoSchedule", "NoExecute"):
                    raise SystemExit(f"error: invalid taint effect: {eff}, unsupported taint effect")
                k, _, v = kv.partition("=")
                if any(x["key"] == k and x["effect"] == eff for x in taints) and not a.overwrite:
                    raise SystemExit(f"error: Node {name} already has {k} taint(s) with same effect(s) and --overwrite is false")
                taints = [x for x in taints if not (x["key"] == k and x["effect"] == eff)]
                taints.append({"key": k, "value": v, "effect": eff} if v else {"key": k, "effect": eff})
            await self.client.patch("nodes", name, {"spec": {"taints": taints or None}})
            self.p(f"node/{name} tainted")

    async def _metrics(self, path):
        st, body = await self.client.raw("GET", "/apis/metrics.k8s.io/v1beta1" + path)
        return {(i["metadata"].get("namespace"), i["metadata"]["name"]): i for i in json.loads(body).get("items") or ()} \
            if st == 200 else {}

    async def cmd_top(self):
        """`kubectl top` (`pkg/kubectl/cmd/top_node.go`, `top_pod.go`) over metrics.k8s.io, with the
        MI355X columns: allocated GPUs per node and per-pod GPU utilization."""
        a = self.a
        nodes = (await self.client.list("nodes", None, a.selector if a.what.startswith("node") else None))["items"]
        pods = (await self.client.list("pods"))["items"]
        if a.name:
            nodes = [n for n in nodes if n["metadata"]["name"] == a.name]
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
            pm = await self._metrics("/pods" if a.all_namespaces else f"/namespaces/{self.ns}/pods")
            if a.selector:
                from ..api.labels import parse as parse_labels
                sel = parse_labels(a.selector)
                pods = [p for p in pods if sel.matches(p["metadata"].get("labels") or {})]
            rows = []
            for p in pods:
                pns = p["metadata"].get("namespace")
                if (not a.all_namespaces and pns != self.ns) or core.pod_is_terminal(p):
                    continue
                if a.name and p["metadata"]["name"] != a.name:
                    continue
                mt = pm.get((pns, p["metadata"]["name"])) or {}
                if a.containers:
                    for c in mt.get("containers") or ():
                        u = c.get("usage") or {}
                        rows.append(([pns] if a.all_namespaces else []) + [p["metadata"]["name"], c["name"],
                                     u.get("cpu", "<unknown>"), u.get("memory", "<unknown>"),
                                     (u[core.AMD_GPU] + "%") if core.AMD_GPU in u else "<none>"])
                    continue
                cpu = sum(int(str(c["usage"].get("cpu", "0m")).rstrip("m") or 0) for c in mt.get("containers") or ())
                mem = sum(int(str(c["usage"].get("memory", "0Ki")).rstrip("Ki") or 0) for c in mt.get("containers") or ())
                gpu = [c["usage"].get(core.AMD_GPU) for c in mt.get("containers") or () if core.AMD_GPU in c.get("usage", {})]
                rows.append(([pns] if a.all_namespaces else []) + [p["metadata"]["name"], f"{cpu}m" if mt else "<unknown>",
                             f"{mem // 1024}Mi" if mt else "<unknown>",
                             ",".join(printers.pod_gpus(p)) or "<none>", (gpu[0] + "%") if gpu else "<none>"])
            head = (["NAMESPACE"] if a.all_namespaces else []) + (
                ["POD", "NAME", "CPU(cores)", "MEMORY(bytes)", "GPU-UTIL"] if a.containers else
                ["NAME", "CPU(cores)", "MEMORY(bytes)", "GPUS", "GPU-UTIL"])
            self.p(printers.table(rows, head))

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
        hpa = {"apiVersion": "autoscaling/v1" if not a.gpu_percent else "autoscaling/v2beta1",
               "kind": "HorizontalPodAutoscaler", "metadata": {"name": a.name or name, "namespace": self.ns}, "spec": spec}
        if not a.dry_run:
            hpa = await self.client.create("horizontalpodautoscalers", hpa, self.ns)
        if a.output:
            self.p(printers.render([hpa], a.output, "HorizontalPodAutoscaler"))
            return
        self.p(f"{ri.kind.lower()}.{ri.group or 'core'} \"{name}\" autoscaled" + (" (dry run)" if a.dry_run else ""))

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
            last = None
            while True:
                d = await self.client.get(ri.plural, name, self.ns)
                msg, done = rollout_status(d, a.revision)
                if done:
                    self.p(msg)
                    return
                if msg != last:
                    self.p(msg)
                    last = msg
                if not a.watch:
                    return
                if time.time() - t > a.timeout:
                    raise SystemExit(f"error: timed out waiting for the rollout of {ri.kind.lower()} \"{name}\"")
                await asyncio.sleep(0.2)
        elif a.action in ("history", "undo") and ri.kind in ("DaemonSet", "StatefulSet"):
            from ..controllers.history import revisions_of
            obj = await self.client.get(ri.plural, name, self.ns)
            revs = revisions_of((await self.client.list("controllerrevisions", self.ns))["items"], obj["metadata"]["uid"])
            if a.action == "history" and a.revision:
                from .describe import _template
                r = next((r for r in revs if int(r.get("revision", 0)) == a.revision), None)
                if r is None:
                    raise SystemExit(f"error: unable to find the specified revision")
                self.p(f'{ri.kind.lower()} "{name}" with revision #{a.revision}\nPod Template:')
                self.p("\n".join(_template(((r.get("data") or {}).get("spec") or {}).get("template") or {})))
                return
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
        elif a.action in ("pause", "resume"):
            # `pkg/kubectl/cmd/rollout/rollout_pause.go` / `rollout_resume.go`: spec.paused
            if ri.kind != "Deployment":
                raise SystemExit(f"error: {ri.kind.lower()}s \"{name}\" {a.action} is not supported")
            want = a.action == "pause"
            d = await self.client.get(ri.plural, name, self.ns)
            if bool((d.get("spec") or {}).get("paused")) == want:
                self.p(f"deployment \"{name}\" is already {'paused' if want else 'resumed'}")
                return
            await self.client.patch(ri.plural, name, {"spec": {"paused": want}}, self.ns)
            self.p(f"deployment \"{name}\" {'paused' if want else 'resumed'}")
        elif a.action == "history":
            uid = (await self.client.get(ri.plural, name, self.ns))["metadata"]["uid"]
            rss = [r for r in (await self.client.list("replicasets", self.ns))["items"] if (m.controller_of(r) or {}).get("uid") == uid]
            if a.revision:
                from .describe import _template
                r = next((r for r in rss if int((r["metadata"].get("annotations") or {}).get(
                    "deployment.kubernetes.io/revision", 0)) == a.revision), None)
                if r is None:
                    raise SystemExit(f"error: unable to find the specified revision")
                tpl = json.loads(json.dumps((r.get("spec") or {}).get("template") or {}))
                ((tpl.get("metadata") or {}).get("labels") or {}).pop("pod-template-hash", None)
                self.p(f'deployment "{name}" with revision #{a.revision}\nPod Template:')
                self.p("\n".join(_template(tpl)))
                return
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

    def _run_object(self):
        """The object `kubectl run` generates (`pkg/kubectl/run.go`): --restart=Always ->
        Deployment (deployment/apps.v1beta1), OnFailure -> Job (job/v1), Never -> Pod
        (run-pod/v1), --schedule -> CronJob (cronjob/v1beta1); --generator picks one explicitly."""
        a = self.a
        labels = dict(kv.split("=", 1) for kv in a.labels.split(",") if kv) if a.labels else {"run": a.name}
        c = {"name": a.name, "image": a.image}
        if a.run_command:
            c["command" if a.as_command else "args"] = list(a.run_command)
        if a.env:
            c["env"] = [{"name": e.split("=", 1)[0], "value": e.split("=", 1)[1] if "=" in e else ""} for e in a.env]
        res = {}
        for key, spec in (("limits", a.limits), ("requests", a.requests)):
            if spec:
                res[key] = dict(kv.split("=", 1) for kv in spec.split(",") if kv)
        if a.gpus:
            res.setdefault("limits", {})[core.AMD_GPU] = str(a.gpus)
        if res:
            c["resources"] = res
        if a.port:
            c["ports"] = [{"containerPort": a.port} | ({"hostPort": a.hostport} if a.hostport else {})]
        elif a.hostport:
            raise SystemExit("error: --hostport requires --port to be specified")
        if a.image_pull_policy:
            c["imagePullPolicy"] = a.image_pull_policy
        if a.stdin:
            c["stdin"] = True
            c["stdinOnce"] = not a.leave_stdin_open
        if a.tty:
            c["tty"] = True
        pod_spec = {"containers": [c]}
        if a.serviceaccount:
            pod_spec["serviceAccountName"] = a.serviceaccount
        gen = a.generator or ("cronjob/v1beta1" if a.schedule else {"Always": "deployment/apps.v1beta1",
                                                                   "OnFailure": "job/v1", "Never": "run-pod/v1"}[a.restart])
        md = {"name": a.name, "namespace": self.ns, "labels": labels}
        if gen.startswith("run-pod"):
            obj = {"apiVersion": "v1", "kind": "Pod", "metadata": md, "spec": dict(pod_spec, restartPolicy=a.restart)}
        elif gen.startswith("deployment"):
            if a.restart != "Always":
                raise SystemExit(f"error: --restart={a.restart} is not valid for a Deployment")
            obj = {"apiVersion": "apps/v1beta1" if "apps" in gen else "extensions/v1beta1", "kind": "Deployment",
                   "metadata": md, "spec": {"replicas": a.replicas, "selector": {"matchLabels": labels},
                                            "template": {"metadata": {"labels": labels}, "spec": pod_spec}}}
        elif gen == "run/v1":
            # BasicReplicationController (pkg/kubectl/run.go)
            if a.restart != "Always":
                raise SystemExit(f"error: --restart={a.restart} is not valid for a ReplicationController")
            obj = {"apiVersion": "v1", "kind": "ReplicationController", "metadata": md,
                   "spec": {"replicas": a.replicas, "selector": dict(labels),
                            "template": {"metadata": {"labels": labels}, "spec": pod_spec}}}
        elif gen.startswith("job"):
            obj = {"apiVersion": "batch/v1", "kind": "Job", "metadata": md,
                   "spec": {"template": {"metadata": {"labels": labels},
                                         "spec": dict(pod_spec, restartPolicy=a.restart if a.restart != "Always" else "OnFailure")}}}
        elif gen.startswith("cronjob"):
            obj = {"apiVersion": "batch/v1beta1", "kind": "CronJob", "metadata": md,
                   "spec": {"schedule": a.schedule, "jobTemplate": {"spec": {"template": {
                       "metadata": {"labels": labels},
                       "spec": dict(pod_spec, restartPolicy=a.restart if a.restart != "Always" else "OnFailure")}}}}}
        else:
            raise SystemExit(f"error: generator {gen!r} not found")
        if a.overrides:
            from ..utils.patch import apply_patch
            obj = apply_patch("application/merge-patch+json", obj, json.loads(a.overrides))
        return obj

    async def cmd_run(self):
        a = self.a
        attach = a.attach or a.stdin
        if a.rm and not attach:
            raise SystemExit("error: --rm should only be used for attached containers")
        if a.expose and not a.port:
            raise SystemExit("error: --port must be set when exposing a service")
        obj = self._run_object()
        ri = ri_for_obj(obj)
        if a.dry_run:
            self.p(printers.render([obj], a.output, ri.kind) if a.output else f"{ri.kind.lower()}/{a.name} created (dry run)")
            return
        svc = None
        if a.expose:
            svc = {"apiVersion": "v1", "kind": "Service",
                   "metadata": {"name": a.name, "namespace": self.ns, "labels": obj["metadata"]["labels"]},
                   "spec": {"selector": obj["metadata"]["labels"], "ports": [{"port": a.port, "targetPort": a.port}]}}
            if a.service_overrides:
                from ..utils.patch import apply_patch
                svc = apply_patch("application/merge-patch+json", svc, json.loads(a.service_overrides))
            svc = await self.client.create("services", svc, self.ns)
        created = await self.client.create(ri.plural, obj, self.ns)
        if a.output:
            self.p(printers.render([created] + ([svc] if svc else []), a.output, ri.kind))
        elif not (attach and a.quiet):
            if svc:
                self.p(f"service/{a.name} created")
            self.p(f"{ri.kind.lower()}/{a.name} created")
        if not attach:
            return
        # wait for a running pod (or a finished one) and attach to it (`kubectl run -i/-t`)
        end = time.monotonic() + a.pod_running_timeout
        pod = None
        while time.monotonic() < end:
            if ri.kind == "Pod":
                pods = [await self.client.get("pods", a.name, self.ns)]
            else:
                sel = ",".join(f"{k}={v}" for k, v in sorted(obj["metadata"]["labels"].items()))
                pods = (await self.client.list("pods", self.ns, sel))["items"]
            pod = next((p for p in pods if (p.get("status") or {}).get("phase") in ("Running", "Succeeded", "Failed")), None)
            if pod is not None:
                break
            await asyncio.sleep(0.2)
        if pod is None:
            raise SystemExit(f"error: timed out waiting for the pod of {ri.kind.lower()}/{a.name} to run")
        pname = pod["metadata"]["name"]
        if pod["status"]["phase"] == "Running":
            self.rc = await self._interactive(pname, "attach", a.name, (), a.stdin, a.tty)
        else:
            st, body = await self.client.raw("GET", f"/api/v1/namespaces/{self.ns}/pods/{pname}/log")
            self.out.write(body.decode(errors="replace"))
            cs = ((pod.get("status") or {}).get("containerStatuses") or [{}])[0]
            self.rc = int((((cs.get("state") or {}).get("terminated")) or {}).get("exitCode", 0) or 0)
        if a.rm:
            await self.client.delete(ri.plural, a.name, self.ns)
            if svc:
                await self.client.delete("services", a.name, self.ns)
            self.p(f"{ri.kind.lower()} \"{a.name}\" deleted")

    async def cmd_expose(self):
        """`kubectl expose` (pkg/kubectl/cmd/expose.go, service/v2 generator): selector, ports
        (and protocols) default to the exposed object's; labels default to its labels."""
        a = self.a
        if a.filename:
            objs = [(ri_for_obj(d), await self.client.get(ri_for_obj(d).plural, d["metadata"]["name"], self.ns))
                    for d in read_manifests(a.filename, False)]
        else:
            objs = [(ri, await self.client.get(ri.plural, name, self.ns)) for ri, name in split_targets(a.targets)]
        if len(objs) != 1:
            raise SystemExit("error: expose needs exactly one resource")
        ri, obj = objs[0]
        if ri.kind not in ("Pod", "Service", "ReplicationController", "ReplicaSet", "Deployment"):
            raise SystemExit(f"error: cannot expose a {ri.kind}")
        spec, md = obj.get("spec") or {}, obj["metadata"]
        if a.selector:
            sel = dict(kv.split("=", 1) for kv in a.selector.split(",") if kv)
        elif ri.kind == "Pod":
            sel = md.get("labels") or {}
        elif ri.kind in ("Service", "ReplicationController"):
            sel = spec.get("selector") or {}
        else:
            s = spec.get("selector") or {}
            if s.get("matchExpressions"):
                raise SystemExit("error: couldn't convert expressions to a service selector")
            sel = s.get("matchLabels") or {}
        if not sel:
            raise SystemExit(f"error: couldn't find a selector for {ri.kind.lower()}/{md['name']}")
        if ri.kind == "Service":
            found = [(p["port"], p.get("protocol", "TCP")) for p in spec.get("ports") or ()]
        else:
            pod_spec = spec if ri.kind == "Pod" else ((spec.get("template") or {}).get("spec") or {})
            found = [(p["containerPort"], p.get("protocol", "TCP")) for c in pod_spec.get("containers") or ()
                     for p in c.get("ports") or ()]
        target = a.target_port or a.target_port_alias
        if a.port:
            ports = [{"port": a.port, "protocol": a.protocol}]
        elif found:
            ports = [{"port": p, "protocol": proto} for p, proto in found]
        elif a.type != "ExternalName":
            raise SystemExit("error: couldn't find port via --port flag or introspection")
        else:
            ports = []
        for i, p in enumerate(ports):
            if len(ports) > 1:
                p["name"] = f"port-{i + 1}"
            t = target if target is not None else p["port"]
            p["targetPort"] = int(t) if str(t).isdigit() else t
        labels = dict(kv.split("=", 1) for kv in a.labels.split(",") if kv) if a.labels else (md.get("labels") or {})
        svc_spec = {"selector": sel, "ports": ports}
        if a.type != "ClusterIP":
            svc_spec["type"] = a.type
        if a.external_ip:
            svc_spec["externalIPs"] = [x for x in a.external_ip.split(",") if x]
        if a.load_balancer_ip:
            svc_spec["loadBalancerIP"] = a.load_balancer_ip
        if a.session_affinity:
            svc_spec["sessionAffinity"] = a.session_affinity
        if a.cluster_ip:
            svc_spec["clusterIP"] = a.cluster_ip
        svc = {"apiVersion": "v1", "kind": "Service",
               "metadata": {"name": a.name or md["name"], "namespace": self.ns, "labels": labels}, "spec": svc_spec}
        if a.overrides:
            from ..utils.patch import apply_patch
            svc = apply_patch("application/merge-patch+json", svc, json.loads(a.overrides))
        if not a.dry_run:
            svc = await self.client.create("services", svc, self.ns)
        if a.output:
            self.p(printers.render([svc], a.output, "Service"))
        else:
            self.p(f"service/{svc['metadata']['name']} exposed" + (" (dry run)" if a.dry_run else ""))

    async def cmd_version(self):
        """`kubectl version` (--client, --short, -o json|yaml)."""
        from ..apiserver.server import VERSION
        a = self.a
        info = {"clientVersion": dict(VERSION)}
        if not a.client:
            st, body = await self.client.raw("GET", "/version")
            if st == 200:
                info["serverVersion"] = json.loads(body)
        if a.output == "json":
            self.p(json.dumps(info, indent=2))
            return
        if a.output == "yaml":
            self.p(yaml.safe_dump(info, sort_keys=False).rstrip())
            return
        for who, key in (("Client", "clientVersion"), ("Server", "serverVersion")):
            v = info.get(key)
            if v is None:
                continue
            if a.short:
                self.p(f"{who} Version: {v['gitVersion']}")
            else:
                self.p(f"{who} Version: version.Info{{" + ", ".join(f'{k[:1].upper() + k[1:]}:"{v[k]}"' for k in v) + "}")

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
        """`kubectl cluster-info` lists the master and the kube-system services labeled
        kubernetes.io/cluster-service=true (with their proxy URLs); `dump` writes nodes plus, per
        namespace, events / replicationcontrollers / services / daemonsets / deployments /
        replicasets / pods and every pod's log (`pkg/kubectl/cmd/clusterinfo_dump.go`)."""
        a = self.a
        if a.action != "dump":
            self.p(f"Kubernetes master is running at {self.server}")
            svcs = (await self.client.list("services", "kube-system", "kubernetes.io/cluster-service=true"))["items"]
            for s in svcs:
                name = (s["metadata"].get("labels") or {}).get("kubernetes.io/name") or s["metadata"]["name"]
                port = ((s.get("spec") or {}).get("ports") or [{}])[0]
                ref = s["metadata"]["name"] + (f":{port['name']}" if port.get("name") else "")
                self.p(f"{name} is running at {self.server}/api/v1/namespaces/kube-system/services/{ref}/proxy")
            self.p("\nTo further debug and diagnose cluster problems, use 'kubectl cluster-info dump'.")
            return
        out_dir = a.output_directory

        def emit(rel, data):
            text = data if isinstance(data, str) else json.dumps(data, indent=2)
            if out_dir:
                path = os.path.join(out_dir, rel)
                os.makedirs(os.path.dirname(path), exist_ok=True)
                with open(path, "w") as f:
                    f.write(text)
            else:
                self.p(text)
                if rel.endswith("logs.txt"):
                    self.p(f"==== END logs for {rel[:-len('/logs.txt')]} ====")
        emit("nodes.json", await self.client.list("nodes"))
        if a.all_namespaces:
            nss = [n["metadata"]["name"] for n in (await self.client.list("namespaces"))["items"]]
        else:
            nss = [x for x in a.namespaces.split(",") if x] or ["kube-system", self.ns]
        for ns in dict.fromkeys(nss):
            for plural in ("events", "replicationcontrollers", "services", "daemonsets", "deployments", "replicasets", "pods"):
                emit(f"{ns}/{plural}.json", await self.client.list(plural, ns))
            for p in (await self.client.list("pods", ns))["items"]:
                pn = p["metadata"]["name"]
                for c in (p.get("spec") or {}).get("containers") or ():
                    st, body = await self.client.raw("GET", f"/api/v1/namespaces/{ns}/pods/{pn}/log?container={c['name']}")
                    emit(f"{ns}/{pn}/logs.txt" if len(p["spec"]["containers"]) == 1 else f"{ns}/{pn}/{c['name']}/logs.txt",
                         body.decode(errors="replace") if st == 200 else "")
        if out_dir:
            self.p(f"Cluster info dumped to {out_dir}")

    async def cmd_explain(self):
        """`kubectl explain TYPE[.field...]` (pkg/kubectl/explain): walk the server's OpenAPI
        definition; --recursive prints the whole field tree."""
        a = self.a
        head, *field_path = a.resource.split(".")
        ri = m.lookup(head)
        if ri is None:
            raise SystemExit(f"error: couldn't find resource for {a.resource}")
        if a.api_version:
            ri = next((r for r in m.RESOURCES if r.kind == ri.kind and r.group_version == a.api_version), ri)
        self.p(f"KIND:     {ri.kind}\nVERSION:  {ri.group_version}\n")
        st, body = await self.client.raw("GET", "/openapi/v2")
        if st == 200:
            from ..apiserver.openapi import def_name
            doc = json.loads(body)
            defs = doc.get("definitions") or {}

            def resolve(sch):
                while isinstance(sch, dict) and "$ref" in sch:
                    sch = defs.get(sch["$ref"].rsplit("/", 1)[-1], {})
                if isinstance(sch, dict) and sch.get("type") == "array" and isinstance(sch.get("items"), dict):
                    return resolve(sch["items"])
                return sch or {}

            def type_of(sch):
                if "$ref" in sch:
                    return "<Object>"
                t = sch.get("type", "Object")
                return f"<[]{type_of(sch['items']).strip('<>')}>" if t == "array" and "items" in sch else f"<{t}>"
            sch = defs.get(def_name(ri), {})
            for f in field_path:
                props = resolve(sch).get("properties") or {}
                if f not in props:
                    raise SystemExit(f'error: field "{f}" does not exist')
                sch = props[f]
            if field_path:
                self.p(f"RESOURCE: {field_path[-1]} {type_of(sch)}\n")
            props = resolve(sch).get("properties") or {}
            if props:
                self.p("FIELDS:")

                def walk(pr, depth, seen):
                    for k, v in sorted(pr.items()):
                        self.p(f"{'   ' * depth}{k}\t{type_of(v)}")
                        ref = v.get("$ref") or (v.get("items") or {}).get("$ref")
                        if a.recursive and ref not in seen:
                            walk(resolve(v).get("properties") or {}, depth + 1, seen | {ref})
                walk(props, 1, frozenset())
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
        # `kubectl auth can-i VERB TYPE[/NAME] | NONRESOURCEURL` (pkg/kubectl/cmd/auth/cani.go):
        # a SelfSubjectAccessReview, so it answers for the caller's (or --as) identity
        if not a.verb or not a.resource:
            raise SystemExit("error: you must specify two or three arguments: verb, resource, and optional resourceName")
        attrs = {}
        if a.resource.startswith("/"):
            attrs = {"nonResourceAttributes": {"verb": a.verb, "path": a.resource}}
        else:
            kind, _, name = a.resource.partition("/")
            name = name or a.resource_name or ""
            ri = m.lookup(kind)
            group, plural = (ri.group, ri.plural) if ri is not None else (kind.partition(".")[2], kind.partition(".")[0])
            ra = {"verb": a.verb, "resource": plural, "group": group, "name": name,
                  "namespace": "" if a.all_namespaces or (ri is not None and not ri.namespaced) else self.ns}
            if a.subresource:
                ra["subresource"] = a.subresource
            attrs = {"resourceAttributes": ra}
        body = {"apiVersion": "authorization.k8s.io/v1", "kind": "SelfSubjectAccessReview", "spec": attrs}
        st, resp = await self.client.raw("POST", "/apis/authorization.k8s.io/v1/selfsubjectaccessreviews",
                                         json.dumps(body).encode())
        if st not in (200, 201):
            raise SystemExit(f"error: {resp.decode(errors='replace')}")
        allowed = bool((json.loads(resp).get("status") or {}).get("allowed"))
        if not a.quiet:
            self.p("yes" if allowed else "no")
        self.rc = 0 if allowed else 1

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
        if a.pod_flag:                      # deprecated `-p POD`: the positional is the command
            rest = [a.pod] + rest
            a.pod = a.pod_flag
        if rest and rest[0] == "--" and "--" not in rest[1:]:
            rest = rest[1:]
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
        pod = (await self._pods_for(a.pod))[0] if "/" in a.pod else a.pod    # TYPE/NAME: its first pod
        self.rc = await self._interactive(pod, "attach", a.container, (), a.stdin, a.tty)

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
        """`kubectl cp` (pkg/kubectl/cmd/cp.go): a tar stream over exec — local->pod feeds
        `tar xf - -C DIR` on stdin, pod->local reads `tar cf - PATH`; files and directories, with
        the source's base name re-rooted at the destination. Entries that would escape the
        destination are refused."""
        import io as _io
        import posixpath
        import tarfile
        a = self.a
        src, dst = a.src, a.dst
        if ":" in src and not os.path.exists(src):
            pod, path = src.split(":", 1)
            ns = self.ns
            if "/" in pod:
                ns, pod = pod.split("/", 1)
            saved, self.ns = self.ns, ns
            try:
                rc, out, err = await self._exec(pod, a.container, ["tar", "cf", "-", "-C", posixpath.dirname(path) or "/",
                                                                   posixpath.basename(path.rstrip("/")) or "."])
            finally:
                self.ns = saved
            if rc != 0:
                raise SystemExit(f"error: {err.decode(errors='replace') or out.decode(errors='replace')}")
            base = posixpath.basename(path.rstrip("/"))
            dest_root = os.path.abspath(dst)
            with tarfile.open(fileobj=_io.BytesIO(out), mode="r:") as tf:
                for mem in tf.getmembers():
                    rel = mem.name[len(base):].lstrip("/") if mem.name == base or mem.name.startswith(base + "/") else mem.name
                    target = os.path.abspath(os.path.join(dest_root, rel)) if rel else dest_root
                    if target != dest_root and not target.startswith(dest_root + os.sep):
                        raise SystemExit(f"error: refusing to write outside {dst}: {mem.name}")
                    if mem.isdir():
                        os.makedirs(target, exist_ok=True)
                    elif mem.isfile():
                        os.makedirs(os.path.dirname(target) or ".", exist_ok=True)
                        with open(target, "wb") as f:
                            f.write(tf.extractfile(mem).read())
                        os.chmod(target, mem.mode & 0o777)
            return
        pod, path = dst.split(":", 1)
        ns = self.ns
        if "/" in pod:
            ns, pod = pod.split("/", 1)
        if not os.path.exists(src):
            raise SystemExit(f"error: {src} doesn't exist in local filesystem")
        buf = _io.BytesIO()
        with tarfile.open(fileobj=buf, mode="w:") as tf:
            tf.add(src, arcname=posixpath.basename(path.rstrip("/")) or os.path.basename(src))
        dest_dir = posixpath.dirname(path.rstrip("/")) or "/"
        saved, self.ns = self.ns, ns
        try:
            rc, out, err = await self._exec(pod, a.container, ["tar", "xf", "-", "-C", dest_dir], stdin_data=buf.getvalue())
        finally:
            self.ns = saved
        if rc != 0:
            raise SystemExit(f"error: {err.decode(errors='replace') or out.decode(errors='replace')}")

    async def cmd_proxy(self):
        """`kubectl proxy`: a local HTTP endpoint forwarding to the API server with this
        kubeconfig's credentials (`pkg/kubectl/proxy/proxy_server.go`)."""
        from ..utils.httpserver import HTTPServer, Response, StreamResponse
        import re
        a = self.a
        http = self.client.http
        rx = lambda spec: [re.compile(x) for x in spec.split(",") if x]          # noqa: E731
        accept_hosts, accept_paths = rx(a.accept_hosts), rx(a.accept_paths)
        reject_paths, reject_methods = rx(a.reject_paths), rx(a.reject_methods)
        prefix = "/" + a.api_prefix.strip("/") + "/" if a.api_prefix.strip("/") else "/"
        www_prefix = "/" + a.www_prefix.strip("/") + "/"

        async def handle(req):
            if not a.disable_filter:        # FilterServer (pkg/kubectl/proxy/proxy_server.go)
                host = (req.headers.get("host") or "").rsplit(":", 1)[0] if not (req.headers.get("host") or "").startswith("[") \
                    else (req.headers.get("host") or "").split("]")[0] + "]"
                if not any(r.search(host) for r in accept_hosts) or not any(r.search(req.path) for r in accept_paths) \
                        or any(r.search(req.path) for r in reject_paths) or any(r.search(req.method) for r in reject_methods):
                    return Response(403, b"<h3>Unauthorized</h3>", "text/html")
            if a.www and req.path.startswith(www_prefix):
                rel = os.path.normpath(req.path[len(www_prefix):]).lstrip("/")
                full = os.path.join(os.path.abspath(a.www), rel)
                if rel.startswith("..") or not os.path.isfile(full):
                    return Response(404, b"404 page not found", "text/plain")
                import mimetypes
                with open(full, "rb") as f:
                    return Response(200, f.read(), mimetypes.guess_type(full)[0] or "application/octet-stream")
            if not req.raw_path.startswith(prefix):
                return Response(404, b"404 page not found", "text/plain")
            path = "/" + req.raw_path[len(prefix):] + (("?" + req.qs) if req.qs else "")
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
        if a.unix_socket:
            await srv.start_unix(a.unix_socket)
            self.p(f"Starting to serve on {a.unix_socket}")
        else:
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
        a = self.a
        if a.filename:
            d, = read_manifests(a.filename, False)
            ri, name = ri_for_obj(d), d["metadata"]["name"]
        else:
            (ri, name), = split_targets(a.targets)
        obj = await self.client.get(ri.plural, name, self.ns_for(ri))
        text = json.dumps(obj, indent=4) + "\n" if a.output == "json" else yaml.safe_dump(obj, sort_keys=False)
        with tempfile.NamedTemporaryFile("w", suffix="." + a.output, delete=False) as f:
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
        if a.output_patch:
            from ..utils.patch import create_merge_patch
            self.p("Patch: " + json.dumps(create_merge_patch(obj, new), sort_keys=True))
        await self.client.update(ri.plural, new, self.ns_for(ri))
        self.p(f"{ri.kind.lower()}/{name} edited")


def cmd_config(a, out=sys.stdout):
    return config_cmd.run(a, out)


def _bool(v):
    return str(v).lower() not in ("false", "0", "no")


def _common(p):
    """Flags shared by many commands: accepted for compatibility where they change nothing here."""
    p.add_argument("-R", "--recursive", action="store_true", help="process directories given with -f recursively")
    p.add_argument("--output-version", default="", help="deprecated; objects are printed in their served version")


def build_parser():
    ap = argparse.ArgumentParser("kubectl", allow_abbrev=False)   # `version --client` is no prefix of --client-key
    ap.add_argument("-s", "--server")
    ap.add_argument("--token")
    ap.add_argument("--kubeconfig")
    ap.add_argument("--context")
    ap.add_argument("--as", dest="as_user", help="impersonate this user")
    ap.add_argument("--as-group", action="append", default=[], help="impersonate this group (repeatable)")
    ap.add_argument("--cluster", dest="cluster", help="kubeconfig cluster to use")
    ap.add_argument("--user", dest="user", help="kubeconfig user to use")
    ap.add_argument("--insecure-skip-tls-verify", action="store_true")
    ap.add_argument("--certificate-authority")
    ap.add_argument("--client-certificate")
    ap.add_argument("--client-key")
    ap.add_argument("--request-timeout", default="0")
    ap.add_argument("--username")
    ap.add_argument("--password")
    ap.add_argument("-v", "--v", dest="verbosity", type=int, default=0)
    ap.add_argument("--match-server-version", action="store_true")
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
    g.add_argument("--sort-by", default="", help="JSONPath, e.g. {.metadata.name}")
    g.add_argument("-L", "--label-columns", action="append", default=[])
    g.add_argument("--show-labels", action="store_true")
    g.add_argument("--show-kind", action="store_true")
    g.add_argument("--no-headers", action="store_true")
    g.add_argument("--ignore-not-found", action="store_true")
    g.add_argument("--watch-only", action="store_true")
    g.add_argument("--raw", default="", help="GET this API path verbatim")
    g.add_argument("--chunk-size", type=int, default=500)
    g.add_argument("--include-uninitialized", action="store_true")
    g.add_argument("-a", "--show-all", action="store_true",
                   help="show all resources (by default terminated pods are hidden from lists)")
    _common(g)
    d = add("describe")
    d.add_argument("targets", nargs="*")
    d.add_argument("-l", "--selector")
    d.add_argument("-A", "--all-namespaces", action="store_true")
    d.add_argument("--show-events", type=_bool, default=True)
    d.add_argument("-f", "--filename", action="append")
    _common(d)
    for name in ("create", "apply", "replace"):
        c = add(name)
        c.add_argument("-f", "--filename", action="append", required=name != "create")
        c.add_argument("--validate", type=_bool, default=True)
        c.add_argument("--record", action="store_true")
        c.add_argument("--save-config", action="store_true")
        c.add_argument("-o", "--output", default="")
        c.add_argument("--dry-run", action="store_true")
        _common(c)
        if name == "create":
            c.add_argument("--raw", default="", help="POST the file to this API path verbatim")
            c.add_argument("--edit", action="store_true")
            c.add_argument("--windows-line-endings", action="store_true")
            c.add_argument("generator", nargs=argparse.REMAINDER)
        else:
            c.add_argument("--force", action="store_true")
            c.add_argument("--grace-period", type=int, default=-1)
            c.add_argument("--timeout", type=extra.duration, default=0)
            c.add_argument("--cascade", type=_bool, default=True)
        if name == "apply":
            c.add_argument("--prune", action="store_true")
            c.add_argument("-l", "--selector")
            c.add_argument("--all", action="store_true")
            c.add_argument("--prune-whitelist", action="append", default=[])
            c.add_argument("--overwrite", type=_bool, default=True)
            c.add_argument("--openapi-patch", type=_bool, default=True)
    for sub_ in ("view-last-applied", "set-last-applied", "edit-last-applied"):
        la_ = add("apply-" + sub_, help=argparse.SUPPRESS)
        la_.add_argument("targets", nargs="*")
        la_.add_argument("-f", "--filename", action="append")
        la_.add_argument("-o", "--output", default="yaml" if sub_ != "set-last-applied" else "",
                         choices=["yaml", "json"] if sub_ != "set-last-applied" else None)
        la_.add_argument("--all", action="store_true")
        la_.add_argument("-l", "--selector")
        la_.add_argument("--create-annotation", action="store_true")
        la_.add_argument("--dry-run", action="store_true")
        la_.add_argument("--record", action="store_true")
        _common(la_)
    de = add("delete")
    de.add_argument("targets", nargs="*")
    de.add_argument("-f", "--filename", action="append")
    de.add_argument("-l", "--selector")
    de.add_argument("--all", action="store_true")
    de.add_argument("--grace-period", type=int, default=None)
    de.add_argument("--cascade", type=lambda s: s.lower() != "false", default=True)
    de.add_argument("--ignore-not-found", action="store_true")
    de.add_argument("--force", action="store_true", help="immediate deletion (--grace-period=0)")
    de.add_argument("--now", action="store_true", help="grace period 1")
    de.add_argument("--timeout", type=extra.duration, default=0, help="wait this long for the objects to be gone")
    de.add_argument("-o", "--output", default="")
    _common(de)
    lg = add("logs")
    lg.add_argument("pod", nargs="?")
    lg.add_argument("container_pos", nargs="?", metavar="container")
    lg.add_argument("-c", "--container")
    lg.add_argument("--tail", type=int)
    lg.add_argument("-p", "--previous", action="store_true")
    lg.add_argument("-f", "--follow", action="store_true")
    lg.add_argument("--since", default="", help="e.g. 5s, 2m, 3h")
    lg.add_argument("--since-time", default="", help="RFC3339")
    lg.add_argument("--timestamps", action="store_true")
    lg.add_argument("--limit-bytes", type=int, default=0)
    lg.add_argument("-l", "--selector")
    lg.add_argument("--pod-running-timeout", type=extra.duration, default=20.0)
    lg.add_argument("--interactive", action="store_true", help="deprecated; ignored")
    for name in ("label", "annotate"):
        la = add(name)
        la.add_argument("resource")
        la.add_argument("name", nargs="?")
        la.add_argument("pairs", nargs="*")
        la.add_argument("--overwrite", action="store_true")
        la.add_argument("--all", action="store_true")
        la.add_argument("-l", "--selector")
        la.add_argument("--resource-version", default="")
        la.add_argument("--dry-run", action="store_true")
        la.add_argument("--local", action="store_true")
        la.add_argument("-f", "--filename", action="append")
        la.add_argument("-o", "--output", default="")
        la.add_argument("--record", action="store_true")
        _common(la)
        if name == "label":
            la.add_argument("--list", action="store_true")
    pa = add("patch")
    pa.add_argument("targets", nargs="*")
    pa.add_argument("-p", "--patch", required=True)
    pa.add_argument("--type", default="strategic", choices=["strategic", "merge", "json"])
    pa.add_argument("-f", "--filename", action="append")
    pa.add_argument("--local", action="store_true")
    pa.add_argument("--dry-run", action="store_true")
    pa.add_argument("-o", "--output", default="")
    pa.add_argument("--record", action="store_true")
    _common(pa)
    sc = add("scale")
    sc.add_argument("targets", nargs="*")
    sc.add_argument("--replicas", type=int, required=True)
    sc.add_argument("--current-replicas", type=int, default=None)
    sc.add_argument("--resource-version", default="")
    sc.add_argument("--all", action="store_true")
    sc.add_argument("-l", "--selector")
    sc.add_argument("--timeout", type=extra.duration, default=0, help="wait for the new size to be ready")
    sc.add_argument("-f", "--filename", action="append")
    sc.add_argument("--record", action="store_true")
    _common(sc)
    for name in ("cordon", "uncordon"):
        co = add(name)
        co.add_argument("node", nargs="?")
        co.add_argument("-l", "--selector")
        co.add_argument("--dry-run", action="store_true")
    dr = add("drain")
    dr.add_argument("node", nargs="?")
    dr.add_argument("--ignore-daemonsets", action="store_true")
    dr.add_argument("--force", action="store_true")
    dr.add_argument("--grace-period", type=int, default=None)
    dr.add_argument("--delete-local-data", action="store_true", help="also evict pods with emptyDir volumes")
    dr.add_argument("--dry-run", action="store_true")
    dr.add_argument("--timeout", type=extra.duration, default=0, help="give up after this many seconds (0 = never)")
    dr.add_argument("-l", "--selector", help="drain every node matching this label selector")
    ta = add("taint")
    ta.add_argument("nodes_kw", choices=["nodes", "node", "no"])
    ta.add_argument("node", nargs="?")
    ta.add_argument("taints", nargs="*")
    ta.add_argument("--overwrite", action="store_true")
    ta.add_argument("--all", action="store_true")
    ta.add_argument("-l", "--selector")
    ta.add_argument("--validate", type=_bool, default=True)
    tp = add("top")
    tp.add_argument("what", choices=["node", "nodes", "pod", "pods"])
    tp.add_argument("name", nargs="?")
    tp.add_argument("-l", "--selector")
    tp.add_argument("-A", "--all-namespaces", action="store_true")
    tp.add_argument("--containers", action="store_true")
    for f in ("--heapster-namespace", "--heapster-port", "--heapster-scheme", "--heapster-service"):
        tp.add_argument(f, default="", help="accepted; metrics come from metrics.k8s.io")
    ro = add("rollout")
    ro.add_argument("action", choices=["status", "history", "undo", "pause", "resume"])
    ro.add_argument("targets", nargs="+")
    ro.add_argument("--to-revision", type=int, default=0)
    ro.add_argument("--revision", type=int, default=0, help="status: the revision to wait for; history: show its template")
    ro.add_argument("-w", "--watch", type=lambda s: s.lower() != "false", default=True)
    ro.add_argument("--timeout", type=extra.duration, default=300)
    rn = add("run")
    rn.add_argument("name")
    rn.add_argument("--image", required=True)
    rn.add_argument("--gpus", type=int, default=0, help="request N amd.com/gpu")
    rn.add_argument("--restart", default="Always", choices=["Always", "OnFailure", "Never"])
    rn.add_argument("--env", action="append", default=[])
    rn.add_argument("-l", "--labels", default="")
    rn.add_argument("--port", type=int, default=0)
    rn.add_argument("--hostport", type=int, default=0)
    rn.add_argument("--expose", action="store_true", help="also create a ClusterIP service for --port")
    rn.add_argument("-r", "--replicas", type=int, default=1)
    rn.add_argument("--limits", default="")
    rn.add_argument("--requests", default="")
    rn.add_argument("--command", dest="as_command", action="store_true", help="the arguments are the command, not args")
    rn.add_argument("--rm", action="store_true")
    rn.add_argument("-i", "--stdin", action="store_true")
    rn.add_argument("-t", "--tty", action="store_true")
    rn.add_argument("--attach", action="store_true")
    rn.add_argument("--leave-stdin-open", action="store_true")
    rn.add_argument("--dry-run", action="store_true")
    rn.add_argument("-o", "--output", default="")
    rn.add_argument("--image-pull-policy", default="")
    rn.add_argument("--schedule", default="", help="create a CronJob on this schedule")
    rn.add_argument("--generator", default="")
    rn.add_argument("--overrides", default="", help="JSON merged into the generated object")
    rn.add_argument("--serviceaccount", default="")
    rn.add_argument("--quiet", action="store_true")
    rn.add_argument("--record", action="store_true")
    rn.add_argument("--pod-running-timeout", type=extra.duration, default=60.0)
    rn.add_argument("--service-generator", default="")
    rn.add_argument("--service-overrides", default="")
    rn.add_argument("run_command", nargs="*", metavar="command")
    ex = add("expose")
    ex.add_argument("targets", nargs="*")
    ex.add_argument("--port", type=int, default=0)
    ex.add_argument("--target-port")
    ex.add_argument("--name")
    ex.add_argument("--type", default="ClusterIP", choices=["ClusterIP", "NodePort", "LoadBalancer", "ExternalName"])
    ex.add_argument("--protocol", default="TCP")
    ex.add_argument("--selector", default="")
    ex.add_argument("-l", "--labels", default="")
    ex.add_argument("--external-ip", default="")
    ex.add_argument("--load-balancer-ip", default="")
    ex.add_argument("--session-affinity", default="", choices=["", "None", "ClientIP"])
    ex.add_argument("--cluster-ip", default="")
    ex.add_argument("--container-port", dest="target_port_alias", default=None)
    ex.add_argument("--dry-run", action="store_true")
    ex.add_argument("-o", "--output", default="")
    ex.add_argument("--generator", default="service/v2")
    ex.add_argument("--overrides", default="")
    ex.add_argument("--record", action="store_true")
    ex.add_argument("-f", "--filename", action="append")
    _common(ex)
    ve = add("version")
    ve.add_argument("--client", action="store_true")
    ve.add_argument("--short", action="store_true")
    ve.add_argument("-o", "--output", default="", choices=["", "json", "yaml"])
    add("api-versions")
    add("api-resources")
    ci = add("cluster-info")
    ci.add_argument("action", nargs="?", choices=["dump"])
    ci.add_argument("-A", "--all-namespaces", action="store_true")
    ci.add_argument("--namespaces", default="")
    ci.add_argument("--output-directory", default="")
    ci.add_argument("-o", "--output", default="json")
    ci.add_argument("--pod-running-timeout", type=extra.duration, default=20.0)
    e = add("explain")
    e.add_argument("resource")
    e.add_argument("--recursive", action="store_true")
    e.add_argument("--api-version", default="")
    w = add("wait")
    w.add_argument("targets", nargs="+")
    w.add_argument("--for", dest="for_", required=True)
    w.add_argument("--timeout", type=extra.duration, default=30)
    au = add("auth")
    au.add_argument("action", choices=["can-i", "reconcile"])
    au.add_argument("verb", nargs="?")
    au.add_argument("resource", nargs="?")
    au.add_argument("resource_name", nargs="?")
    au.add_argument("-f", "--filename", action="append")
    au.add_argument("-A", "--all-namespaces", action="store_true")
    au.add_argument("-q", "--quiet", action="store_true")
    au.add_argument("--subresource", default="")
    exq = add("exec")
    exq.add_argument("pod")
    exq.add_argument("-c", "--container")
    exq.add_argument("-i", "--stdin", action="store_true")
    exq.add_argument("-t", "--tty", action="store_true")
    exq.add_argument("exec_command", nargs=argparse.REMAINDER)
    exq.add_argument("-p", "--pod", dest="pod_flag", help="deprecated: the pod name")
    at = add("attach")
    at.add_argument("pod")
    at.add_argument("-c", "--container")
    at.add_argument("-i", "--stdin", action="store_true")
    at.add_argument("-t", "--tty", action="store_true")
    at.add_argument("--pod-running-timeout", type=extra.duration, default=20.0)
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
    px.add_argument("--api-prefix", default="/")
    px.add_argument("-w", "--www", default="", help="serve static files from this directory under --www-prefix")
    px.add_argument("-P", "--www-prefix", default="/static/")
    px.add_argument("--accept-hosts", default=r"^localhost$,^127\.0\.0\.1$,^\[::1\]$")
    px.add_argument("--accept-paths", default="^.*")
    px.add_argument("--reject-paths", default=r"^/api/.*/pods/.*/exec,^/api/.*/pods/.*/attach")
    px.add_argument("--reject-methods", default="^$")
    px.add_argument("--disable-filter", action="store_true")
    px.add_argument("-u", "--unix-socket", default="")
    ed = add("edit")
    ed.add_argument("targets", nargs="*")
    ed.add_argument("-o", "--output", default="yaml", choices=["yaml", "json"])
    ed.add_argument("--output-patch", action="store_true")
    ed.add_argument("--record", action="store_true")
    ed.add_argument("--validate", type=_bool, default=True)
    ed.add_argument("--windows-line-endings", action="store_true")
    ed.add_argument("-f", "--filename", action="append")
    aut = add("autoscale")
    aut.add_argument("targets", nargs="+")
    aut.add_argument("--min", type=int, default=0)
    aut.add_argument("--max", type=int, required=True)
    aut.add_argument("--cpu-percent", type=int, default=0)
    aut.add_argument("--gpu-percent", type=int, default=0, help="target MI355X utilization (amd.com/gpu)")
    aut.add_argument("--name")
    aut.add_argument("--dry-run", action="store_true")
    aut.add_argument("-o", "--output", default="")
    aut.add_argument("--generator", default="horizontalpodautoscaler/v1")
    aut.add_argument("--record", action="store_true")
    cert = add("certificate")
    cert.add_argument("action", choices=["approve", "deny"])
    cert.add_argument("names", nargs="+")
    extra.add_parsers(add)
    config_cmd.add_parser(add)
    return ap


_TRAILING = {"label": "pairs", "annotate": "pairs", "taint": "taints", "get": "targets", "describe": "targets",
             "delete": "targets", "patch": "targets", "scale": "targets", "expose": "targets", "edit": "targets",
             "rollout": "targets", "autoscale": "targets", "wait": "targets", "port-forward": "ports", "set": "targets"}

GLOBAL_FLAGS = {"-s", "--server", "--token", "--kubeconfig", "--context", "-n", "--namespace", "--as", "--as-group",
                "--cluster", "--user", "--certificate-authority", "--client-certificate", "--client-key",
                "--request-timeout", "--username", "--password", "-v", "--v"}
GLOBAL_SWITCHES = {"--insecure-skip-tls-verify", "--match-server-version"}


def hoist_global_flags(argv):
    """kubectl accepts its persistent flags anywhere (cobra); move them before the command."""
    front, rest, i = [], [], 0
    flags = GLOBAL_FLAGS
    while i < len(argv):
        t = argv[i]
        if t == "config" and not rest:
            # config's own --server / --token / --namespace (set-cluster, set-credentials,
            # set-context) shadow the global ones
            flags = {"--kubeconfig", "--context"}
        elif t == "create" and not rest:
            flags = flags - {"--user"}        # create (cluster)rolebinding --user is a subject
        if t == "--":
            rest += argv[i:]
            break
        if t in flags and i + 1 < len(argv):
            front += [t, argv[i + 1]]
            i += 2
            continue
        if t in GLOBAL_SWITCHES and flags is not None and "--context" in flags and len(flags) > 2:
            front.append(t)
            i += 1
            continue
        if t.split("=", 1)[0] in flags and "=" in t:
            front.append(t)
            i += 1
            continue
        rest.append(t)
        i += 1
    return front + rest


def _bool_flag_values(ap, argv):
    """pflag booleans take `--flag=true|false`; argparse's store_true does not: rewrite those
    tokens (before any `--`) for the flags that are booleans in some subcommand."""
    table = getattr(ap, "_kamd_bools", None)
    if table is None:
        def flags(p, nested):
            out = set()
            for act in p._actions:
                if isinstance(act, (argparse._StoreTrueAction, argparse._StoreFalseAction)):
                    out.update(o for o in act.option_strings if o.startswith("--"))
                if nested and isinstance(act, argparse._SubParsersAction):
                    for sp in act.choices.values():
                        out |= flags(sp, True)
            return out
        table = {None: flags(ap, False)}          # global flags; then per subcommand
        for act in ap._actions:
            if isinstance(act, argparse._SubParsersAction):
                for name, sp in act.choices.items():
                    table[name] = table[None] | flags(sp, True)
        ap._kamd_bools = table
    cmd = next((t for t in argv if not t.startswith("-") and t in table), None)
    bools = table.get(cmd, table[None])
    out = []
    for i, t in enumerate(argv):
        if t == "--":
            return out + argv[i:]
        if t.startswith("--") and "=" in t:
            k, v = t.split("=", 1)
            if k in bools and v.lower() in ("true", "false"):
                if v.lower() == "true":
                    out.append(k)
                continue
        out.append(t)
    return out


def main(argv=None, out=sys.stdout):
    ap = build_parser()
    argv = hoist_global_flags(list(sys.argv[1:] if argv is None else argv))
    for i_, t_ in enumerate(argv[:-1]):
        if t_ == "apply" and argv[i_ + 1] in ("view-last-applied", "set-last-applied", "edit-last-applied"):
            argv = argv[:i_] + ["apply-" + argv[i_ + 1]] + argv[i_ + 2:]   # `apply view-last-applied ...`
            break
        if not t_.startswith("-") and (i_ == 0 or not argv[i_ - 1].startswith("-")):
            break
    argv = _bool_flag_values(ap, argv)
    tail = None
    if "--" in argv and "run" in argv[:argv.index("--")]:
        argv, tail = argv[:argv.index("--")], argv[argv.index("--") + 1:]     # `run NAME ... -- CMD ARGS`
    a, extras = ap.parse_known_args(argv)
    if tail is not None:
        a.run_command = list(a.run_command or []) + tail
    if extras:
        # cobra intermixes flags and positionals (`label pods -l app=x k=v`); argparse stops
        # filling a positional list at the first flag, so the rest lands here
        dest = _TRAILING.get(a.command)
        bad = [x for x in extras if x.startswith("-") and x != "-"]
        if dest is None or bad:
            ap.error("unrecognized arguments: " + " ".join(bad or extras))
        setattr(a, dest, list(getattr(a, dest) or []) + extras)
    if a.command == "config":
        return cmd_config(a, out)
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
