"""`kubectl config`: read and edit kubeconfig files.

Parity: `pkg/kubectl/cmd/config/*.go` — view (`--minify`, `--flatten`, `--raw`, `-o`),
current-context, get-contexts (`-o name`, `--no-headers`), get-clusters, use-context,
set-cluster (`--server`, `--certificate-authority`, `--embed-certs`,
`--insecure-skip-tls-verify`), set-credentials (`--token`, `--username`/`--password`,
`--client-certificate`/`--client-key`, `--embed-certs`, `--auth-provider`,
`--auth-provider-arg`), set-context (`--current`, `--cluster`, `--user`, `--namespace`),
set / unset of a dotted property path (`navigation_step_parser.go`), delete-cluster,
delete-context, rename-context.

`KUBECONFIG` may list several files separated by `:` (`clientcmd` loading rules): reads see
their merge — the first file to define a map key or a named entry wins; writes go to the
file that already holds the edited entry, else to the first file.
"""
from __future__ import annotations

import base64
import json
import os

import yaml

DEFAULT_KUBECONFIG = os.path.expanduser("~/.kube/config")
_LISTS = (("clusters", "cluster"), ("contexts", "context"), ("users", "user"))
_SECRET_FIELDS = ("certificate-authority-data", "client-certificate-data", "client-key-data")


def _empty():
    return {"apiVersion": "v1", "kind": "Config", "preferences": {}, "clusters": [], "contexts": [], "users": [],
            "current-context": ""}


def _read(path):
    if not os.path.exists(path):
        return _empty()
    with open(path) as f:
        cfg = yaml.safe_load(f) or {}
    for key, _ in _LISTS:
        cfg[key] = cfg.get(key) or []
    return cfg


def paths(explicit=None):
    if explicit:
        return [explicit]
    env = os.environ.get("KUBECONFIG")
    if env:
        return [p for p in env.split(os.pathsep) if p] or [DEFAULT_KUBECONFIG]
    return [DEFAULT_KUBECONFIG]


def load(explicit=None):
    """-> (merged config, [(path, config)])."""
    files = [(p, _read(p)) for p in paths(explicit)]
    merged = _empty()
    for _, cfg in files:
        for key, _inner in _LISTS:
            have = {e["name"] for e in merged[key]}
            merged[key] += [e for e in cfg.get(key) or () if e.get("name") not in have]
        if not merged["current-context"] and cfg.get("current-context"):
            merged["current-context"] = cfg["current-context"]
        for k, v in cfg.items():
            if k not in merged or (k == "preferences" and not merged[k]):
                merged[k] = v
    return merged, files


def _owner(files, key, name):
    for p, cfg in files:
        if any(e.get("name") == name for e in cfg.get(key) or ()):
            return p, cfg
    return files[0]


def _save(path, cfg):
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        yaml.safe_dump(cfg, f, sort_keys=False)
    os.replace(tmp, path)


def _entry(cfg, key, name, create=True):
    inner = dict(_LISTS)[key]
    for e in cfg.setdefault(key, []):
        if e.get("name") == name:
            e.setdefault(inner, {})
            return e[inner]
    if not create:
        return None
    e = {"name": name, inner: {}}
    cfg[key].append(e)
    return e[inner]


def _embed(path):
    with open(path, "rb") as f:
        return base64.b64encode(f.read()).decode()


def add_parser(add):
    cf = add("config")
    ss = cf.add_subparsers(dest="action", required=True)
    v = ss.add_parser("view")
    v.add_argument("--minify", action="store_true")
    v.add_argument("--flatten", action="store_true")
    v.add_argument("--raw", action="store_true")
    v.add_argument("-o", "--output", default="yaml", choices=["yaml", "json"])
    ss.add_parser("current-context")
    gc = ss.add_parser("get-contexts")
    gc.add_argument("name", nargs="?")
    gc.add_argument("-o", "--output", default="", choices=["", "name"])
    gc.add_argument("--no-headers", action="store_true")
    ss.add_parser("get-clusters")
    uc = ss.add_parser("use-context")
    uc.add_argument("name")
    sc = ss.add_parser("set-cluster")
    sc.add_argument("name")
    sc.add_argument("--server", dest="server_url")
    sc.add_argument("--certificate-authority")
    sc.add_argument("--embed-certs", action="store_true")
    sc.add_argument("--insecure-skip-tls-verify", choices=["true", "false"])
    sr = ss.add_parser("set-credentials")
    sr.add_argument("name")
    sr.add_argument("--token", dest="user_token")
    sr.add_argument("--username")
    sr.add_argument("--password")
    sr.add_argument("--client-certificate")
    sr.add_argument("--client-key")
    sr.add_argument("--embed-certs", action="store_true")
    sr.add_argument("--auth-provider")
    sr.add_argument("--auth-provider-arg", action="append", default=[])
    sx = ss.add_parser("set-context")
    sx.add_argument("name", nargs="?")
    sx.add_argument("--current", action="store_true")
    sx.add_argument("--cluster")
    sx.add_argument("--user")
    sx.add_argument("--namespace", dest="ctx_namespace")
    st = ss.add_parser("set")
    st.add_argument("property")
    st.add_argument("value")
    st.add_argument("--set-raw-bytes", choices=["true", "false"], default="false")
    un = ss.add_parser("unset")
    un.add_argument("property")
    for n in ("delete-cluster", "delete-context"):
        ss.add_parser(n).add_argument("name")
    rc = ss.add_parser("rename-context")
    rc.add_argument("name")
    rc.add_argument("new_name")
    return cf


def _redact(cfg):
    cfg = json.loads(json.dumps(cfg))
    for key, inner in _LISTS:
        for e in cfg.get(key) or ():
            body = e.get(inner) or {}
            for f in _SECRET_FIELDS:
                if body.get(f):
                    body[f] = "DATA+OMITTED" if key == "clusters" or f == "client-certificate-data" else "REDACTED"
            for f in ("token", "password"):
                if body.get(f):
                    body[f] = "REDACTED" if key == "users" else body[f]
    return cfg


def _minify(cfg, context=None):
    name = context or cfg.get("current-context")
    if not name:
        raise SystemExit("error: current-context must exist in order to minify")
    ctx = _entry(cfg, "contexts", name, create=False)
    if ctx is None:
        raise SystemExit(f'error: cannot locate context {name}')
    out = dict(cfg)
    out["contexts"] = [e for e in cfg["contexts"] if e["name"] == name]
    out["clusters"] = [e for e in cfg["clusters"] if e["name"] == ctx.get("cluster")]
    out["users"] = [e for e in cfg["users"] if e["name"] == ctx.get("user")]
    out["current-context"] = name
    return out


def _flatten(cfg, base_dirs):
    cfg = json.loads(json.dumps(cfg))
    for key, inner in _LISTS:
        for e in cfg.get(key) or ():
            body = e.get(inner) or {}
            for f in ("certificate-authority", "client-certificate", "client-key"):
                p = body.pop(f, None)
                if p:
                    full = p if os.path.isabs(p) else os.path.join(base_dirs.get((key, e["name"]), "."), p)
                    body[f + "-data"] = _embed(full)
    return cfg


def _set_path(cfg, prop, value):
    """`kubectl config set users.alice.token xyz`: a step through a named list picks the entry
    by name (names may contain dots: the longest matching name wins)."""
    parts = prop.split(".")
    node = cfg
    i = 0
    while i < len(parts):
        key = parts[i]
        last = i == len(parts) - 1
        if key in dict(_LISTS) and node is cfg:
            rest = parts[i + 1:]
            if not rest:
                raise SystemExit(f"error: can't set a map to a value: {prop}")
            names = {e["name"] for e in cfg[key]}
            n = next((".".join(rest[:j]) for j in range(len(rest), 0, -1) if ".".join(rest[:j]) in names), rest[0])
            j = len(n.split("."))
            if value is None and i + 1 + j == len(parts):
                cfg[key] = [e for e in cfg[key] if e["name"] != n]
                return
            node = _entry(cfg, key, n, create=value is not None)
            if node is None:
                raise SystemExit(f"error: current map key `{n}` is invalid")
            i += 1 + j
            continue
        if last:
            if value is None:
                if key not in node:
                    raise SystemExit(f"error: current map key `{key}` is invalid")
                node.pop(key)
            else:
                node[key] = value
            return
        if value is None and key not in node:
            raise SystemExit(f"error: current map key `{key}` is invalid")
        node = node.setdefault(key, {})
        i += 1


def run(a, out):
    def p(s=""):
        print(s, file=out)
    merged, files = load(getattr(a, "kubeconfig", None))
    act = a.action
    if act == "view":
        cfg = merged
        if a.minify:
            cfg = _minify(cfg, getattr(a, "context", None))
        if a.flatten:
            base = {}
            for path, fc in files:
                for key, _ in _LISTS:
                    for e in fc.get(key) or ():
                        base.setdefault((key, e["name"]), os.path.dirname(os.path.abspath(path)))
            cfg = _flatten(cfg, base)
        if not a.raw:
            cfg = _redact(cfg)
        p(json.dumps(cfg, indent=4) if a.output == "json" else yaml.safe_dump(cfg, sort_keys=False).rstrip())
        return 0
    if act == "current-context":
        if not merged.get("current-context"):
            raise SystemExit("error: current-context is not set")
        p(merged["current-context"])
        return 0
    if act == "get-contexts":
        ctxs = merged["contexts"]
        if a.name:
            ctxs = [c for c in ctxs if c["name"] == a.name]
            if not ctxs:
                raise SystemExit(f'error: context {a.name} not found')
        if a.output == "name":
            for c in ctxs:
                p(c["name"])
            return 0
        from .printers import table
        rows = [["*" if c["name"] == merged.get("current-context") else "", c["name"], (c.get("context") or {}).get("cluster", ""),
                 (c.get("context") or {}).get("user", ""), (c.get("context") or {}).get("namespace", "")] for c in ctxs]
        text = table(rows, ["CURRENT", "NAME", "CLUSTER", "AUTHINFO", "NAMESPACE"])
        p("\n".join(text.splitlines()[1:]) if a.no_headers else text)
        return 0
    if act == "get-clusters":
        p("NAME")
        for c in merged["clusters"]:
            p(c["name"])
        return 0
    if act == "use-context":
        if not any(c["name"] == a.name for c in merged["contexts"]):
            raise SystemExit(f'error: no context exists with the name: "{a.name}"')
        path, cfg = files[0]
        cfg["current-context"] = a.name
        _save(path, cfg)
        p(f'Switched to context "{a.name}".')
        return 0
    if act == "set-cluster":
        path, cfg = _owner(files, "clusters", a.name)
        existed = _entry(cfg, "clusters", a.name, create=False) is not None
        cl = _entry(cfg, "clusters", a.name)
        if a.server_url is not None:
            cl["server"] = a.server_url
        if a.insecure_skip_tls_verify is not None:
            cl["insecure-skip-tls-verify"] = a.insecure_skip_tls_verify == "true"
            if cl["insecure-skip-tls-verify"]:
                cl.pop("certificate-authority", None)
                cl.pop("certificate-authority-data", None)
        if a.certificate_authority:
            if a.embed_certs:
                cl["certificate-authority-data"] = _embed(a.certificate_authority)
                cl.pop("certificate-authority", None)
            else:
                cl["certificate-authority"] = os.path.abspath(a.certificate_authority)
                cl.pop("certificate-authority-data", None)
            cl.pop("insecure-skip-tls-verify", None)
        elif a.embed_certs:
            raise SystemExit("error: you must specify a --certificate-authority to embed")
        _save(path, cfg)
        p(f'Cluster "{a.name}" {"modified" if existed else "set"}.')
        return 0
    if act == "set-credentials":
        path, cfg = _owner(files, "users", a.name)
        existed = _entry(cfg, "users", a.name, create=False) is not None
        u = _entry(cfg, "users", a.name)
        if a.user_token is not None and (a.username or a.password):
            raise SystemExit("error: you cannot specify more than one authentication method at the same time: "
                             "--token, --username/--password")
        if a.user_token is not None:
            u["token"] = a.user_token
            u.pop("username", None), u.pop("password", None)
        if a.username is not None:
            u["username"] = a.username
            u.pop("token", None)
        if a.password is not None:
            u["password"] = a.password
        for flag, field in ((a.client_certificate, "client-certificate"), (a.client_key, "client-key")):
            if flag:
                if a.embed_certs:
                    u[field + "-data"] = _embed(flag)
                    u.pop(field, None)
                else:
                    u[field] = os.path.abspath(flag)
                    u.pop(field + "-data", None)
        if a.auth_provider:
            ap = u.setdefault("auth-provider", {})
            if ap.get("name") != a.auth_provider:
                ap.clear()
            ap["name"] = a.auth_provider
        for arg in a.auth_provider_arg:
            ap = u.setdefault("auth-provider", {})
            conf = ap.setdefault("config", {})
            if arg.endswith("-"):
                conf.pop(arg[:-1], None)
            else:
                k, _, v = arg.partition("=")
                conf[k] = v
        _save(path, cfg)
        p(f'User "{a.name}" {"modified" if existed else "set"}.')
        return 0
    if act == "set-context":
        name = merged.get("current-context") if a.current else a.name
        if not name:
            raise SystemExit("error: you must specify a non-empty context name or --current")
        if a.current and a.name:
            raise SystemExit("error: you cannot specify a context name and --current")
        path, cfg = _owner(files, "contexts", name)
        existed = _entry(cfg, "contexts", name, create=False) is not None
        c = _entry(cfg, "contexts", name)
        for val, field in ((a.cluster, "cluster"), (a.user, "user"), (a.ctx_namespace, "namespace")):
            if val is not None:
                c[field] = val
        _save(path, cfg)
        p(f'Context "{name}" {"modified" if existed else "created"}.')
        return 0
    if act in ("set", "unset"):
        path, cfg = files[0]
        value = None
        if act == "set":
            value = a.value
            if value in ("true", "false") and a.property.split(".")[-1] in ("insecure-skip-tls-verify",):
                value = value == "true"
            elif a.property.endswith("-data") and a.set_raw_bytes != "true":
                value = base64.b64encode(value.encode()).decode()
        _set_path(cfg, a.property, value)
        _save(path, cfg)
        p(f'Property "{a.property}" {"set" if act == "set" else "unset"}.')
        return 0
    if act in ("delete-cluster", "delete-context"):
        key = "clusters" if act == "delete-cluster" else "contexts"
        path, cfg = _owner(files, key, a.name)
        if _entry(cfg, key, a.name, create=False) is None:
            raise SystemExit(f"error: cannot delete {key[:-1]} {a.name}, not in {path}")
        cfg[key] = [e for e in cfg[key] if e["name"] != a.name]
        if key == "contexts" and cfg.get("current-context") == a.name:
            print(f"warning: this removed your active context, use \"kubectl config use-context\" to select a "
                  f"different one", file=out)
        _save(path, cfg)
        p(f"deleted {key[:-1]} {a.name} from {path}")
        return 0
    if act == "rename-context":
        path, cfg = _owner(files, "contexts", a.name)
        if _entry(cfg, "contexts", a.name, create=False) is None:
            raise SystemExit(f'error: cannot rename the context "{a.name}", it\'s not in {path}')
        if any(e["name"] == a.new_name for e in cfg["contexts"]):
            raise SystemExit(f'error: cannot rename the context "{a.name}", the context "{a.new_name}" already exists in {path}')
        for e in cfg["contexts"]:
            if e["name"] == a.name:
                e["name"] = a.new_name
        if cfg.get("current-context") == a.name:
            cfg["current-context"] = a.new_name
        _save(path, cfg)
        p(f'Context "{a.name}" renamed to "{a.new_name}".')
        return 0
    raise SystemExit(f"error: unknown config action {act}")
