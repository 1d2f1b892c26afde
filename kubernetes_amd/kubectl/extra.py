"""kubectl commands beyond the basic verbs: `create <generator>`, `set`, `rolling-update`,
`convert`, `completion`, `plugin`, `options`, `alpha diff`, `auth reconcile`.

Parity: `pkg/kubectl/cmd/create_*.go` + generators (`pkg/kubectl/{configmap,secret,secret_for_tls,
serviceaccount,rolebinding,clusterrolebinding,quota,service_basic,deployment,pdb,priorityclass}.go`),
`pkg/kubectl/cmd/set/{set_image,set_resources,set_env,set_selector,set_serviceaccount,set_subject}.go`,
`pkg/kubectl/rolling_updater.go` (deployment-key relabel of the old RC, scale new up / old down by
one while new pods become ready, rename at the end), `cmd/convert.go`, `cmd/completion.go`,
`pkg/kubectl/plugins/*` (`~/.kube/plugins/<name>/plugin.yaml`, `KUBECTL_PLUGINS_*` env),
`cmd/options.go`, `cmd/auth/reconcile.go`.
"""
from __future__ import annotations

import argparse
import asyncio
import base64
import difflib
import hashlib
import json
import os
import re
import subprocess
import sys
import time

import yaml

from ..api import meta as m
from ..client.rest import APIStatusError, is_already_exists, is_not_found


def duration(v):
    """A kubectl duration flag: seconds as a number, or a Go duration ("1s", "5m", "1m30s",
    "500ms", "1h")."""
    v = str(v).strip()
    try:
        return float(v)
    except ValueError:
        pass
    units = {"ns": 1e-9, "us": 1e-6, "µs": 1e-6, "ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0}
    parts = re.findall(r"(\d+(?:\.\d+)?)(ns|us|µs|ms|s|m|h)", v)
    if not parts or "".join(n + u for n, u in parts) != v:
        raise argparse.ArgumentTypeError(f"invalid duration {v!r}")
    return sum(float(n) * units[u] for n, u in parts)


# ------------------------------------------------------------------------------------ generators
def _kv(pairs):
    out = {}
    for p in pairs or ():
        k, _, v = p.partition("=")
        out[k] = v
    return out


def _from_files(paths):
    out = {}
    for p in paths or ():
        key, _, path = p.partition("=") if "=" in p else (None, None, p)
        if os.path.isdir(path):
            for fn in sorted(os.listdir(path)):
                fp = os.path.join(path, fn)
                if os.path.isfile(fp):
                    out[fn] = open(fp, "rb").read()
        else:
            out[key or os.path.basename(path)] = open(path, "rb").read()
    return out


def _create_parser():
    ap = argparse.ArgumentParser(prog="kubectl create")
    sub = ap.add_subparsers(dest="kind", required=True)
    x = sub.add_parser("namespace", aliases=["ns"])
    x.add_argument("name")
    x = sub.add_parser("serviceaccount", aliases=["sa"])
    x.add_argument("name")
    x = sub.add_parser("configmap", aliases=["cm"])
    x.add_argument("name")
    x.add_argument("--from-literal", action="append", default=[])
    x.add_argument("--from-file", action="append", default=[])
    x.add_argument("--from-env-file")
    x.add_argument("--append-hash", action="store_true", help="Append a hash of the configmap to its name.")
    x = sub.add_parser("secret")
    ss = x.add_subparsers(dest="secret_type", required=True)
    g = ss.add_parser("generic")
    g.add_argument("name")
    g.add_argument("--from-literal", action="append", default=[])
    g.add_argument("--from-file", action="append", default=[])
    g.add_argument("--type", default="Opaque")
    g.add_argument("--from-env-file")
    t = ss.add_parser("tls")
    t.add_argument("name")
    t.add_argument("--cert", required=True)
    t.add_argument("--key", required=True)
    d = ss.add_parser("docker-registry")
    for q in (g, t, d):
        q.add_argument("--append-hash", action="store_true", help="Append a hash of the secret to its name.")
    d.add_argument("name")
    d.add_argument("--docker-server", default="https://index.docker.io/v1/")
    d.add_argument("--docker-username", required=True)
    d.add_argument("--docker-password", required=True)
    d.add_argument("--docker-email", default="")
    x = sub.add_parser("deployment", aliases=["deploy"])
    x.add_argument("name")
    x.add_argument("--image", action="append", required=True)
    x.add_argument("--replicas", type=int, default=1)
    x.add_argument("--gpus", type=int, default=0, help="amd.com/gpu per pod")
    x = sub.add_parser("job")
    x.add_argument("name")
    x.add_argument("--image", required=True)
    x.add_argument("cmd", nargs="*")
    for kind in ("role", "clusterrole"):
        x = sub.add_parser(kind)
        x.add_argument("name")
        x.add_argument("--verb", action="append", required=True)
        x.add_argument("--resource", action="append", default=[])
        x.add_argument("--resource-name", action="append", default=[])
        if kind == "clusterrole":
            x.add_argument("--non-resource-url", action="append", default=[])
    for kind in ("rolebinding", "clusterrolebinding"):
        x = sub.add_parser(kind)
        x.add_argument("name")
        x.add_argument("--clusterrole")
        if kind == "rolebinding":
            x.add_argument("--role")
        x.add_argument("--user", action="append", default=[])
        x.add_argument("--group", action="append", default=[])
        x.add_argument("--serviceaccount", action="append", default=[])
    x = sub.add_parser("quota", aliases=["resourcequota"])
    x.add_argument("name")
    x.add_argument("--hard", default="")
    x.add_argument("--scopes", default="")
    x = sub.add_parser("service", aliases=["svc"])
    st = x.add_subparsers(dest="service_type", required=True)
    for k in ("clusterip", "nodeport", "loadbalancer", "externalname"):
        y = st.add_parser(k)
        y.add_argument("name")
        y.add_argument("--tcp", action="append", default=[])
        y.add_argument("--clusterip", default=None)
        y.add_argument("--node-port", type=int, default=0)
        y.add_argument("--external-name", default="")
    x = sub.add_parser("poddisruptionbudget", aliases=["pdb"])
    x.add_argument("name")
    x.add_argument("--selector", required=True)
    x.add_argument("--min-available")
    x.add_argument("--max-unavailable")
    x = sub.add_parser("priorityclass", aliases=["pc"])
    x.add_argument("name")
    x.add_argument("--value", type=int, required=True)
    x.add_argument("--global-default", action="store_true")
    x.add_argument("--description", default="")
    return ap


def _env_file(path):
    """`--from-env-file` (`pkg/kubectl/cmd/util/env_file.go`): KEY=VALUE lines, `#` comments
    and blank lines skipped, a bare KEY takes its value from the environment, keys must be
    valid environment variable names."""
    import re as _re
    out = {}
    if not path:
        return out
    with open(path) as f:
        for n, line in enumerate(f, 1):
            line = line.lstrip()
            if not line.strip() or line.startswith("#"):
                continue
            kk, eq, vv = line.rstrip("\n").partition("=")
            if not _re.fullmatch(r"[-._a-zA-Z][-._a-zA-Z0-9]*", kk):
                raise SystemExit(f"error: {kk!r} at line {n} of {path} is not a valid key name")
            out[kk] = vv if eq else os.environ.get(kk, "")
    return out


def _b64(v):
    return base64.b64encode(v if isinstance(v, bytes) else v.encode()).decode()


def _rules(verbs, resources, names):
    rules = {}
    for r in resources:
        res, _, grp = r.partition(".")
        rules.setdefault(grp, []).append(res)
    out = [{"apiGroups": [g], "resources": rs, "verbs": verbs} for g, rs in rules.items()]
    if names:
        for r in out:
            r["resourceNames"] = names
    return out


def _subjects(a, ns):
    out = [{"kind": "User", "apiGroup": "rbac.authorization.k8s.io", "name": u} for u in a.user]
    out += [{"kind": "Group", "apiGroup": "rbac.authorization.k8s.io", "name": g} for g in a.group]
    for s in a.serviceaccount:
        sns, _, sname = s.partition(":")
        out.append({"kind": "ServiceAccount", "namespace": sns or ns, "name": sname})
    return out


def _labels_sel(s):
    return dict(p.split("=", 1) for p in s.split(",") if p)


def _secret(a, md):
    """The Secret of `kubectl create secret generic|tls|docker-registry`."""
    if a.secret_type == "generic":
        data = {kk: _b64(v) for kk, v in _kv(a.from_literal).items()}
        data.update({kk: _b64(v) for kk, v in _from_files(a.from_file).items()})
        data.update({kk: _b64(v) for kk, v in _env_file(a.from_env_file).items()})
        return "secrets", {"apiVersion": "v1", "kind": "Secret", "metadata": md, "type": a.type, "data": data}
    if a.secret_type == "tls":
        return "secrets", {"apiVersion": "v1", "kind": "Secret", "metadata": md, "type": "kubernetes.io/tls",
                           "data": {"tls.crt": _b64(open(a.cert, "rb").read()), "tls.key": _b64(open(a.key, "rb").read())}}
    auth = _b64(f"{a.docker_username}:{a.docker_password}")
    cfg = {"auths": {a.docker_server: {"username": a.docker_username, "password": a.docker_password,
                                       "email": a.docker_email, "auth": auth}}}
    return "secrets", {"apiVersion": "v1", "kind": "Secret", "metadata": md, "type": "kubernetes.io/dockerconfigjson",
                       "data": {".dockerconfigjson": _b64(json.dumps(cfg))}}

def generate(argv, ns):
    """Object built by a `kubectl create <generator>` command line (no server round trip)."""
    a = _create_parser().parse_args(argv)
    k = a.kind
    md = {"name": a.name}
    if k in ("namespace", "ns"):
        return "namespaces", {"apiVersion": "v1", "kind": "Namespace", "metadata": md}
    md["namespace"] = ns
    if k in ("serviceaccount", "sa"):
        return "serviceaccounts", {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": md}
    if k in ("configmap", "cm"):
        data = _kv(a.from_literal)
        binary = {}
        for key, v in _from_files(a.from_file).items():
            try:
                data[key] = v.decode()
            except UnicodeDecodeError:
                binary[key] = _b64(v)
        data.update(_env_file(a.from_env_file))
        o = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": md, "data": data}
        if binary:
            o["binaryData"] = binary
        if a.append_hash:
            from .hash import config_map_hash
            md["name"] = f"{a.name}-{config_map_hash(o)}"
        return "configmaps", o
    if k == "secret":
        plural, o = _secret(a, md)
        if a.append_hash:
            from .hash import secret_hash
            md["name"] = f"{a.name}-{secret_hash(o)}"
        return plural, o

    if k in ("deployment", "deploy"):
        labels = {"app": a.name}
        ctrs = []
        for img in a.image:
            c = {"name": img.split("/")[-1].split(":")[0].split("@")[0], "image": img}
            if a.gpus:
                c["resources"] = {"limits": {"amd.com/gpu": str(a.gpus)}}
            ctrs.append(c)
        return "deployments", {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": dict(md, labels=labels),
                               "spec": {"replicas": a.replicas, "selector": {"matchLabels": labels},
                                        "template": {"metadata": {"labels": labels}, "spec": {"containers": ctrs}}}}
    if k == "job":
        c = {"name": a.name, "image": a.image}
        if a.cmd:
            c["command"] = a.cmd
        return "jobs", {"apiVersion": "batch/v1", "kind": "Job", "metadata": md,
                        "spec": {"template": {"spec": {"containers": [c], "restartPolicy": "Never"}}}}
    if k in ("role", "clusterrole"):
        rules = _rules(a.verb, a.resource, a.resource_name)
        if k == "clusterrole":
            md.pop("namespace")
            if a.non_resource_url:
                rules.append({"nonResourceURLs": a.non_resource_url, "verbs": a.verb})
            return "clusterroles", {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole", "metadata": md,
                                    "rules": rules}
        return "roles", {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role", "metadata": md, "rules": rules}
    if k in ("rolebinding", "clusterrolebinding"):
        role_kind, role = ("ClusterRole", a.clusterrole) if a.clusterrole else ("Role", getattr(a, "role", None))
        if not role:
            raise SystemExit("error: exactly one of clusterrole or role must be specified")
        o = {"apiVersion": "rbac.authorization.k8s.io/v1", "metadata": md, "subjects": _subjects(a, ns),
             "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": role_kind, "name": role}}
        if k == "clusterrolebinding":
            md.pop("namespace")
            return "clusterrolebindings", dict(o, kind="ClusterRoleBinding")
        return "rolebindings", dict(o, kind="RoleBinding")
    if k in ("quota", "resourcequota"):
        spec = {"hard": _labels_sel(a.hard)}
        if a.scopes:
            spec["scopes"] = a.scopes.split(",")
        return "resourcequotas", {"apiVersion": "v1", "kind": "ResourceQuota", "metadata": md, "spec": spec}
    if k in ("service", "svc"):
        t = {"clusterip": "ClusterIP", "nodeport": "NodePort", "loadbalancer": "LoadBalancer",
             "externalname": "ExternalName"}[a.service_type]
        ports = []
        for p in a.tcp:
            port, _, target = p.partition(":")
            e = {"name": f"{port}-{target or port}", "protocol": "TCP", "port": int(port), "targetPort": int(target or port)}
            if a.node_port and t == "NodePort":
                e["nodePort"] = a.node_port
            ports.append(e)
        spec = {"type": t, "selector": {"app": a.name}, "ports": ports}
        if t == "ExternalName":
            spec = {"type": t, "externalName": a.external_name}
        if a.clusterip is not None:
            spec["clusterIP"] = a.clusterip
        return "services", {"apiVersion": "v1", "kind": "Service", "metadata": dict(md, labels={"app": a.name}), "spec": spec}
    if k in ("poddisruptionbudget", "pdb"):
        spec = {"selector": {"matchLabels": _labels_sel(a.selector)}}
        for fld, v in (("minAvailable", a.min_available), ("maxUnavailable", a.max_unavailable)):
            if v is not None:
                spec[fld] = int(v) if v.isdigit() else v
        if "minAvailable" not in spec and "maxUnavailable" not in spec:
            spec["minAvailable"] = 1
        return "poddisruptionbudgets", {"apiVersion": "policy/v1beta1", "kind": "PodDisruptionBudget", "metadata": md,
                                        "spec": spec}
    if k in ("priorityclass", "pc"):
        md.pop("namespace")
        return "priorityclasses", {"apiVersion": "scheduling.k8s.io/v1alpha1", "kind": "PriorityClass", "metadata": md,
                                   "value": a.value, "globalDefault": a.global_default, "description": a.description}
    raise SystemExit(f"error: unknown generator {k}")


# ------------------------------------------------------------------------------------ set
def _pod_spec(obj):
    k = obj.get("kind")
    if k == "Pod":
        return obj["spec"]
    if k == "CronJob":
        return obj["spec"]["jobTemplate"]["spec"]["template"]["spec"]
    return obj["spec"]["template"]["spec"]


def _containers(spec, name):
    cs = (spec.get("initContainers") or []) + (spec.get("containers") or [])
    return [c for c in cs if name in (None, "*", c.get("name"))]


def _res_list(s):
    return {k: v for k, v in _kv(s.split(",")).items()} if s else {}


class ExtraCommands:
    """Mixed into `Kubectl` (self.client, self.ns, self.a, self.p, ns_for)."""

    async def _create_generated(self, argv):
        plural, obj = generate(argv, self.ns)
        ri = m.BY_PLURAL.get(plural) or m.lookup(plural)
        if getattr(self.a, "dry_run", False):
            self.p(yaml.safe_dump(obj, sort_keys=False) if getattr(self.a, "output", "") == "yaml" else json.dumps(obj, indent=2))
            return
        await self.client.create(ri.plural, obj, self.ns_for(ri, obj))
        self.p(f"{ri.kind.lower()}/{obj['metadata']['name']} created")

    async def _mutate(self, target, fn):
        r, _, name = target.partition("/")
        ri = m.lookup(r)
        if ri is None or not name:
            raise SystemExit(f"error: expected TYPE/NAME, got {target!r}")
        ns = self.ns_for(ri)
        # client-go RetryOnConflict with a growing pause: a controller writing the object's status
        # (a Deployment right after it was created) can win several read-modify-write races
        for attempt in range(12):
            obj = await self.client.get(ri.plural, name, ns)
            obj.setdefault("kind", ri.kind)
            if fn(obj) is False:
                return ri, obj, False
            try:
                await self.client.update(ri.plural, obj, ns)
                return ri, obj, True
            except APIStatusError as e:
                if e.code != 409:
                    raise
                await asyncio.sleep(min(0.01 * (attempt + 1), 0.1))
        raise SystemExit("error: too many conflicts")

    async def _set_split(self):
        """`set` positionals: TYPE/NAME... or TYPE NAME... (or -f / -l / --all), then KEY=VALUE /
        KEY- pairs (`serviceaccount`: the last word is the account) -> ([(ri, name|obj)], pairs)."""
        from .cli import read_manifests, ri_for_obj
        a = self.a
        toks = list(a.targets)
        if a.what == "serviceaccount":
            toks, pairs = toks[:-1], toks[-1:]
        else:
            cut = next((i for i, t in enumerate(toks) if "=" in t or (t.endswith("-") and "/" not in t)), len(toks))
            toks, pairs = toks[:cut], toks[cut:]
        out = []
        if a.filename:
            for d in read_manifests(a.filename, a.recursive):
                d.setdefault("metadata", {})
                out.append((ri_for_obj(d), d if a.local else d["metadata"]["name"]))
        elif toks and "/" in toks[0]:
            for t in toks:
                r, _, n = t.partition("/")
                ri = m.lookup(r)
                if ri is None:
                    raise SystemExit(f'error: the server doesn\'t have a resource type "{r}"')
                out.append((ri, n))
        elif toks:
            ri = m.lookup(toks[0])
            if ri is None:
                raise SystemExit(f'error: the server doesn\'t have a resource type "{toks[0]}"')
            if toks[1:]:
                out += [(ri, n) for n in toks[1:]]
            elif a.all or a.label_selector:
                items = (await self.client.list(ri.plural, self.ns_for(ri), a.label_selector))["items"]
                out += [(ri, o["metadata"]["name"]) for o in items]
            else:
                raise SystemExit("error: resource(s) were provided, but no name, label selector, or --all flag specified")
        else:
            raise SystemExit("error: one or more resources must be specified as <resource> <name> or <resource>/<name>")
        return out, pairs

    async def _set_apply(self, targets, fn, verb):
        """Run `fn` on each target: --local (files only), --dry-run (fetched, not written) or a
        conflict-retried update; print `-o` output or `<kind>/<name> <verb>`."""
        a = self.a
        for ri, t in targets:
            if isinstance(t, dict) or a.dry_run:
                obj = t if isinstance(t, dict) else await self.client.get(ri.plural, t, self.ns_for(ri))
                obj.setdefault("kind", ri.kind)
                fn(obj)
            else:
                if a.resource_version:
                    cur = await self.client.get(ri.plural, t, self.ns_for(ri))
                    if cur["metadata"].get("resourceVersion") != a.resource_version:
                        raise SystemExit(f"error: Operation cannot be fulfilled on {ri.plural} \"{t}\": "
                                         f"the object has been modified")
                ri, obj, _ = await self._mutate(f"{ri.plural}/{t}", fn)
            if a.output:
                from . import printers
                self.p(printers.render([obj], a.output, ri.kind))
            else:
                self.p(f"{ri.kind.lower()}/{obj['metadata']['name']} {verb}" + (" (dry run)" if a.dry_run else ""))

    async def _set_env(self, targets):
        """`kubectl set env` (pkg/kubectl/cmd/set/set_env.go): KEY=VAL / -e, KEY- removal,
        --from=configmap/NAME|secret/NAME (one valueFrom per key, --prefix, --keys), --list,
        --overwrite=false refuses to change an existing variable."""
        a = self.a
        pairs = list(a.pairs) + list(a.env_pairs)
        sets = {}
        for p_ in pairs:
            if "=" in p_:
                k_, v_ = p_.split("=", 1)
                sets[k_] = {"name": k_, "value": v_}
        drops = {p_[:-1] for p_ in pairs if p_.endswith("-") and "=" not in p_}
        if a.env_from:
            kind, _, src = a.env_from.partition("/")
            kind = {"cm": "configmap", "configmaps": "configmap", "secrets": "secret"}.get(kind, kind)
            if kind not in ("configmap", "secret") or not src:
                raise SystemExit("error: --from must be configmap/NAME or secret/NAME")
            o = await self.client.get("configmaps" if kind == "configmap" else "secrets", src, self.ns)
            keys = [k_ for k_ in sorted((o.get("data") or {})) if not a.keys or k_ in a.keys.split(",")]
            ref = "configMapKeyRef" if kind == "configmap" else "secretKeyRef"
            for key in keys:
                name = (a.prefix + key).upper().replace("-", "_").replace(".", "_")
                sets[name] = {"name": name, "valueFrom": {ref: {"name": src, "key": key}}}
        if a.list:
            for ri, t in targets:
                obj = t if isinstance(t, dict) else await self.client.get(ri.plural, t, self.ns_for(ri))
                self.p(f"# {ri.kind} {obj['metadata']['name']}")
                for c in _containers(_pod_spec(obj), a.containers):
                    self.p(f"# container {c['name']}")
                    for e in c.get("env") or ():
                        if "value" in e:
                            self.p(f"{e['name']}={e['value']}")
                        else:
                            vf = e.get("valueFrom") or {}
                            r = vf.get("configMapKeyRef") or vf.get("secretKeyRef") or {}
                            what = "configmap" if "configMapKeyRef" in vf else "secret" if "secretKeyRef" in vf else "field"
                            self.p(f"# {e['name']} from {what} {r.get('name', '')}, key {r.get('key', '')}")
            return

        def fn(obj):
            for c in _containers(_pod_spec(obj), a.containers):
                cur = {e["name"]: e for e in c.get("env") or ()}
                if not a.overwrite:
                    for k_, e in sets.items():
                        if k_ in cur and cur[k_] != e:
                            raise SystemExit(f"error: '{k_}' already has a value ({cur[k_].get('value', '')}), and --overwrite is false")
                env = [e for e in c.get("env") or () if e["name"] not in drops and e["name"] not in sets]
                env += list(sets.values())
                c["env"] = env
        await self._set_apply(targets, fn, "env updated")

    async def cmd_set(self):
        a = self.a
        targets, a.pairs = await self._set_split()
        if a.what == "env":
            await self._set_env(targets)
            return
        if a.what == "image":
            pairs = _kv(a.pairs)

            def fn(obj):
                spec = _pod_spec(obj)
                hit = False
                for cname, img in pairs.items():
                    for c in _containers(spec, None if cname == "*" else cname):
                        c["image"] = img
                        hit = True
                if not hit:
                    raise SystemExit(f"error: unable to find container(s) {', '.join(pairs)}")
            await self._set_apply(targets, fn, "image updated")
        elif a.what == "resources":
            def fn(obj):
                for c in _containers(_pod_spec(obj), a.containers):
                    r = c.setdefault("resources", {})
                    if a.limits:
                        r.setdefault("limits", {}).update(_res_list(a.limits))
                    if a.requests:
                        r.setdefault("requests", {}).update(_res_list(a.requests))
            await self._set_apply(targets, fn, "resource requirements updated")
        elif a.what == "serviceaccount":
            sa = a.pairs[0]

            def fn(obj):
                _pod_spec(obj)["serviceAccountName"] = sa
            await self._set_apply(targets, fn, "serviceaccount updated")
        elif a.what == "selector":
            sel = _kv(a.pairs)

            def fn(obj):
                if obj.get("kind") == "Service":
                    obj["spec"]["selector"] = sel
                else:
                    obj["spec"]["selector"] = {"matchLabels": sel}
            await self._set_apply(targets, fn, "selector updated")
        elif a.what == "subject":
            def fn(obj):
                subs = obj.setdefault("subjects", [])
                for s in _subjects(a, self.ns):
                    if s not in subs:
                        subs.append(s)
            await self._set_apply(targets, fn, "subjects updated")

    # -------------------------------------------------------------------------- rolling-update
    async def _ready(self, rc_name):
        rc = await self.client.get("replicationcontrollers", rc_name, self.ns)
        return (rc.get("status") or {}).get("readyReplicas", 0), rc

    async def cmd_rolling_update(self):
        a = self.a
        rcs = "replicationcontrollers"
        old = await self.client.get(rcs, a.old, self.ns)
        desired = old["spec"].get("replicas", 1)
        if a.filename:
            from .cli import read_manifests
            new = read_manifests(a.filename)[0]
            new.setdefault("metadata", {})["namespace"] = self.ns
        else:
            new = json.loads(json.dumps(old))
            same = all(c.get("image") == a.image for c in _containers(new["spec"]["template"]["spec"], a.container))
            if same and not a.image_pull_policy:
                raise SystemExit("error: --image-pull-policy (Always|Never|IfNotPresent) must be provided when "
                                 "--image is the same as existing container image")
            for c in _containers(new["spec"]["template"]["spec"], a.container):
                c["image"] = a.image
                if a.image_pull_policy:
                    c["imagePullPolicy"] = a.image_pull_policy
            new["metadata"] = {"name": a.new_name or "", "namespace": self.ns,
                               "labels": old["metadata"].get("labels") or {}}
            new.pop("status", None)
        key = a.deployment_label_key
        h_old = hashlib.sha256(json.dumps(old["spec"]["template"], sort_keys=True).encode()).hexdigest()[:10]
        h_new = hashlib.sha256(json.dumps(new["spec"]["template"], sort_keys=True).encode()).hexdigest()[:10]
        if h_old == h_new:
            if not getattr(a, "image_pull_policy", ""):
                raise SystemExit("error: the new controller's template is identical to the old one")
            # the same image and pull policy on purpose (roll the pods): a fresh hash still
            # separates the new controller's pods from the old ones
            h_new = hashlib.sha256(f"{h_old}-{time.time()}".encode()).hexdigest()[:10]
        rename = not new["metadata"].get("name")
        if rename:
            new["metadata"]["name"] = f"{a.old}-{h_new[:5]}"
        # 1. make the old controller and its pods distinguishable (deployment=<old hash>)
        if (old["spec"].get("selector") or {}).get(key) is None:
            sel = dict(old["spec"].get("selector") or {})
            for p in (await self.client.list("pods", self.ns, ",".join(f"{k}={v}" for k, v in sel.items())))["items"]:
                await self.client.patch("pods", p["metadata"]["name"], {"metadata": {"labels": {key: h_old}}}, self.ns)
            old["spec"]["selector"] = dict(sel, **{key: h_old})
            old["spec"]["template"]["metadata"].setdefault("labels", {})[key] = h_old
            old = await self.client.update(rcs, old, self.ns)
        # 2. the new controller starts at zero replicas
        new["spec"]["selector"] = dict({k: v for k, v in (new["spec"].get("selector") or {}).items() if k != key}, **{key: h_new})
        new["spec"]["template"].setdefault("metadata", {}).setdefault("labels", {}).update(
            {k: v for k, v in new["spec"]["selector"].items()})
        new["spec"]["replicas"] = 0
        new["metadata"].pop("resourceVersion", None)
        new["metadata"].pop("uid", None)
        try:
            await self.client.create(rcs, new, self.ns)
        except APIStatusError as e:
            if not is_already_exists(e):
                raise
        self.p(f"Created {new['metadata']['name']}")
        # 3. scale new up / old down one at a time, waiting for readiness (maxSurge 1, maxUnavailable 0)
        n_new, n_old = 0, old["spec"].get("replicas", desired)
        deadline = time.monotonic() + a.timeout
        while n_new < desired or n_old > 0:
            if n_new < desired:
                n_new += 1
                await self.client.patch(rcs, new["metadata"]["name"], {"spec": {"replicas": n_new}}, self.ns)
                self.p(f"Scaling {new['metadata']['name']} up to {n_new}")
                while (await self._ready(new["metadata"]["name"]))[0] < n_new:
                    if time.monotonic() > deadline:
                        raise SystemExit(f"error: timed out waiting for {new['metadata']['name']} to become ready")
                    await asyncio.sleep(a.poll_interval)
            if n_old > 0 and n_new + n_old > desired:
                n_old -= 1
                await self.client.patch(rcs, a.old, {"spec": {"replicas": n_old}}, self.ns)
                self.p(f"Scaling {a.old} down to {n_old}")
            elif n_new >= desired and n_old > 0:
                n_old = 0
                await self.client.patch(rcs, a.old, {"spec": {"replicas": 0}}, self.ns)
        await self.client.delete(rcs, a.old, self.ns)
        final = new["metadata"]["name"]
        if rename:
            # keep the old name: recreate under it and orphan-delete the temporary controller
            cur = await self.client.get(rcs, final, self.ns)
            cur["metadata"] = {"name": a.old, "namespace": self.ns, "labels": cur["metadata"].get("labels") or {}}
            cur.pop("status", None)
            await self.client.create(rcs, cur, self.ns)
            await self.client.delete(rcs, final, self.ns, propagation="Orphan")
            final = a.old
        self.p(f'Update succeeded. Deleting old controller: {a.old}\nreplicationcontroller "{final}" rolling updated')

    # -------------------------------------------------------------------------- convert / diff
    async def cmd_convert(self):
        from .cli import read_manifests
        out = []
        for d in read_manifests(self.a.filename):
            ri = next((x for x in m.BY_PLURAL.values() if x.kind == d.get("kind")), None)
            if ri is None:
                raise SystemExit(f"error: unknown kind {d.get('kind')}")
            want = self.a.output_version or (f"{ri.group}/{ri.version}" if ri.group else ri.version)
            d["apiVersion"] = want
            out.append(d)
        if self.a.output == "json":
            self.p(json.dumps(out[0] if len(out) == 1 else {"kind": "List", "apiVersion": "v1", "items": out}, indent=2))
        else:
            self.p(yaml.safe_dump_all(out, sort_keys=False).rstrip())

    async def cmd_alpha(self):
        from .cli import read_manifests, ri_for_obj
        rc = 0
        for d in read_manifests(self.a.filename):
            ri = ri_for_obj(d)
            try:
                live = await self.client.get(ri.plural, d["metadata"]["name"], self.ns_for(ri, d))
                ann = (live["metadata"].get("annotations") or {}).get("kubectl.kubernetes.io/last-applied-configuration")
                base = json.loads(ann) if ann else live
            except APIStatusError as e:
                if not is_not_found(e):
                    raise
                base = {}
            for o in (base, d):
                anns = (o.get("metadata") or {}).get("annotations") or {}
                anns.pop("kubectl.kubernetes.io/last-applied-configuration", None)
            a_txt = yaml.safe_dump(base, sort_keys=True).splitlines()
            b_txt = yaml.safe_dump(d, sort_keys=True).splitlines()
            diff = list(difflib.unified_diff(a_txt, b_txt, "LIVE", "LOCAL", lineterm=""))
            if diff:
                rc = 1
                self.p("\n".join(diff))
        self.rc = rc

    # -------------------------------------------------------------------------- auth reconcile
    async def _reconcile(self, d):
        from .cli import ri_for_obj
        ri = ri_for_obj(d)
        ns = self.ns_for(ri, d)
        try:
            cur = await self.client.get(ri.plural, d["metadata"]["name"], ns)
        except APIStatusError as e:
            if not is_not_found(e):
                raise
            await self.client.create(ri.plural, d, ns)
            self.p(f"{ri.kind.lower()}.rbac.authorization.k8s.io/{d['metadata']['name']} reconciled (created)")
            return
        changed = False
        if ri.kind in ("Role", "ClusterRole"):
            rules = cur.get("rules") or []
            for r in d.get("rules") or ():
                if r not in rules:
                    rules.append(r)
                    changed = True
            cur["rules"] = rules
        else:
            subs = cur.get("subjects") or []
            for s in d.get("subjects") or ():
                if s not in subs:
                    subs.append(s)
                    changed = True
            cur["subjects"] = subs
            if cur.get("roleRef") != d.get("roleRef"):
                await self.client.delete(ri.plural, d["metadata"]["name"], ns)
                await self.client.create(ri.plural, d, ns)
                self.p(f"{ri.kind.lower()}.rbac.authorization.k8s.io/{d['metadata']['name']} reconciled (recreated)")
                return
        if changed:
            await self.client.update(ri.plural, cur, ns)
        self.p(f"{ri.kind.lower()}.rbac.authorization.k8s.io/{d['metadata']['name']} reconciled")


# ------------------------------------------------------------------------------------ client-only
PLUGIN_DIRS = [os.path.join(os.path.expanduser("~"), ".kube", "plugins")]


def find_plugins():
    dirs = list(PLUGIN_DIRS)
    env = os.environ.get("KUBECTL_PLUGINS_PATH")
    if env:
        dirs = env.split(os.pathsep) + dirs
    out = {}
    for d in dirs:
        if not os.path.isdir(d):
            continue
        for name in sorted(os.listdir(d)):
            desc = os.path.join(d, name, "plugin.yaml")
            if os.path.exists(desc):
                with open(desc) as f:
                    p = yaml.safe_load(f) or {}
                p["_dir"] = os.path.join(d, name)
                out.setdefault(p.get("name", name), p)
    return out


def run_plugin(name, args, global_args):
    plugins = find_plugins()
    if name not in plugins:
        print(f"error: unknown plugin {name!r}; available: {', '.join(sorted(plugins)) or 'none'}", file=sys.stderr)
        return 1
    p = plugins[name]
    env = dict(os.environ)
    env.update({"KUBECTL_PLUGINS_CALLER": sys.argv[0], "KUBECTL_PLUGINS_DESCRIPTOR_NAME": name,
                "KUBECTL_PLUGINS_DESCRIPTOR_SHORT_DESC": p.get("shortDesc", ""),
                "KUBECTL_PLUGINS_DESCRIPTOR_COMMAND": p.get("command", ""),
                "KUBECTL_PLUGINS_CURRENT_NAMESPACE": global_args.get("namespace") or "default"})
    for k, v in global_args.items():
        if v:
            env[f"KUBECTL_PLUGINS_GLOBAL_FLAG_{k.upper().replace('-', '_')}"] = str(v)
    return subprocess.call(p["command"] + (" " + " ".join(args) if args else ""), shell=True, cwd=p["_dir"], env=env)


def completion(shell, parser):
    cmds = sorted(a for act in parser._subparsers._group_actions for a in act.choices)  # noqa: SLF001
    words = " ".join(cmds)
    if shell == "zsh":
        return f"#compdef kubectl\n_kubectl() {{ compadd {words} }}\ncompdef _kubectl kubectl\n"
    return ("# bash completion for kubectl\n_kubectl() {\n  local cur=${COMP_WORDS[COMP_CWORD]}\n"
            "  if [ $COMP_CWORD -eq 1 ]; then COMPREPLY=( $(compgen -W \"" + words + "\" -- $cur) ); "
            "else COMPREPLY=( $(compgen -f -- $cur) ); fi\n}\ncomplete -F _kubectl kubectl\n")


OPTIONS = """The following options can be passed to any command:

  -s, --server='': The address and port of the Kubernetes API server
      --token='': Bearer token for authentication to the API server
      --kubeconfig='': Path to the kubeconfig file to use for CLI requests
      --context='': The name of the kubeconfig context to use
  -n, --namespace='': If present, the namespace scope for this CLI request"""


def add_parsers(add):
    s = add("set")
    ss = s.add_subparsers(dest="what", required=True)
    for what in ("image", "resources", "env", "serviceaccount", "selector", "subject"):
        x = ss.add_parser(what)
        x.add_argument("targets", nargs="*", help="TYPE/NAME ... or TYPE NAME ..., then KEY=VALUE pairs")
        x.add_argument("--all", action="store_true")
        x.add_argument("-l", "--selector", dest="label_selector")
        x.add_argument("-f", "--filename", action="append")
        x.add_argument("-R", "--recursive", action="store_true")
        x.add_argument("--local", action="store_true")
        x.add_argument("--dry-run", action="store_true")
        x.add_argument("-o", "--output", default="")
        x.add_argument("--record", action="store_true")
        x.add_argument("--resource-version", default="")
        if what == "env":
            x.add_argument("-e", "--env", dest="env_pairs", action="append", default=[])
            x.add_argument("--list", action="store_true")
            x.add_argument("--from", dest="env_from", default="")
            x.add_argument("--prefix", default="")
            x.add_argument("--keys", default="")
            x.add_argument("--overwrite", type=lambda v: v.lower() != "false", default=True)
        x.add_argument("-c", "--containers", default=None)
        x.add_argument("--limits", default="")
        x.add_argument("--requests", default="")
        x.add_argument("--user", action="append", default=[])
        x.add_argument("--group", action="append", default=[])
        x.add_argument("--serviceaccount", action="append", default=[])
    ru = add("rolling-update")
    ru.add_argument("old")
    ru.add_argument("new_name", nargs="?", default=None)
    ru.add_argument("--image")
    ru.add_argument("--image-pull-policy", default="", choices=["", "Always", "Never", "IfNotPresent"])
    ru.add_argument("-c", "--container", default=None)
    ru.add_argument("-f", "--filename", action="append")
    ru.add_argument("--deployment-label-key", default="deployment")
    ru.add_argument("--timeout", type=duration, default=300)
    ru.add_argument("--update-period", dest="poll_interval", type=duration, default=0.1)
    cv = add("convert")
    cv.add_argument("-f", "--filename", action="append", required=True)
    cv.add_argument("--output-version", default=None)
    cv.add_argument("-o", "--output", default="yaml")
    al = add("alpha")
    al.add_argument("sub", choices=["diff"])
    al.add_argument("-f", "--filename", action="append", required=True)
    cp = add("completion")
    cp.add_argument("shell", choices=["bash", "zsh"])
    pl = add("plugin")
    pl.add_argument("plugin_name", nargs="?")
    pl.add_argument("plugin_args", nargs=argparse.REMAINDER)
    add("options")
