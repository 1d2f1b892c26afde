"""kubeconfig loading / writing (client-go `tools/clientcmd`).

Parity: `staging/src/k8s.io/client-go/tools/clientcmd/loader.go:52` (`$KUBECONFIG` or
`~/.kube/config`), `api/types.go` (clusters / users / contexts / current-context), `client_config.go`
(context resolution; cluster `server`, `certificate-authority[-data]`,
`insecure-skip-tls-verify`; user `token`, `client-certificate[-data]`, `client-key[-data]`,
`username/password` basic auth unsupported). TLS material given as `-data` is written to private
temp files because Python's ssl loads certificate chains from files.
"""
from __future__ import annotations

import base64
import os
import ssl
import tempfile

import yaml

DEFAULT_KUBECONFIG = os.path.join(os.path.expanduser("~"), ".kube", "config")


def empty():
    return {"apiVersion": "v1", "kind": "Config", "clusters": [], "contexts": [], "users": [], "current-context": "",
            "preferences": {}}


def load(path=None):
    path = path or os.environ.get("KUBECONFIG") or DEFAULT_KUBECONFIG
    if not os.path.exists(path):
        return empty(), path
    with open(path) as f:
        return yaml.safe_load(f) or empty(), path


def save(cfg, path):
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    tmp = path + ".tmp"
    with open(os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600), "w") as f:
        yaml.safe_dump(cfg, f, sort_keys=False)
    os.replace(tmp, path)


def build(cluster_name, server, user_name, ca_pem=None, token=None, client_cert_pem=None, client_key_pem=None,
          namespace=None):
    """A one-context kubeconfig with embedded credentials (kubeadm's `kubeconfigutil.CreateWithCerts`)."""
    cl = {"server": server}
    if ca_pem:
        cl["certificate-authority-data"] = base64.b64encode(ca_pem.encode()).decode()
    us = {}
    if token:
        us["token"] = token
    if client_cert_pem:
        us["client-certificate-data"] = base64.b64encode(client_cert_pem.encode()).decode()
        us["client-key-data"] = base64.b64encode(client_key_pem.encode()).decode()
    ctx_name = f"{user_name}@{cluster_name}"
    ctx = {"cluster": cluster_name, "user": user_name}
    if namespace:
        ctx["namespace"] = namespace
    cfg = empty()
    cfg["clusters"] = [{"name": cluster_name, "cluster": cl}]
    cfg["users"] = [{"name": user_name, "user": us}]
    cfg["contexts"] = [{"name": ctx_name, "context": ctx}]
    cfg["current-context"] = ctx_name
    return cfg


class Resolved:
    def __init__(self, server, token=None, ssl_context=None, namespace=None, ca_pem=None):
        self.server, self.token, self.ssl_context, self.namespace, self.ca_pem = server, token, ssl_context, namespace, ca_pem


def _material(d, key, base_dir):
    if d.get(key + "-data"):
        return base64.b64decode(d[key + "-data"]).decode()
    p = d.get(key)
    if p:
        if not os.path.isabs(p):
            p = os.path.join(base_dir, p)
        with open(p) as f:
            return f.read()
    return None


def _tmpfile(text):
    fd, p = tempfile.mkstemp(prefix="kamd-kc-", suffix=".pem")
    with os.fdopen(fd, "w") as f:
        f.write(text)
    os.chmod(p, 0o600)
    return p


def resolve(cfg, context=None, base_dir="."):
    ctxname = context or cfg.get("current-context")
    ctx = next((c["context"] for c in cfg.get("contexts") or () if c["name"] == ctxname), None)
    if ctx is None:
        return None
    cl = next((c["cluster"] for c in cfg.get("clusters") or () if c["name"] == ctx.get("cluster")), {}) or {}
    us = next((u["user"] for u in cfg.get("users") or () if u["name"] == ctx.get("user")), {}) or {}
    server = cl.get("server", "")
    ctx_ssl = None
    ca = _material(cl, "certificate-authority", base_dir)
    if server.startswith("https://"):
        if cl.get("insecure-skip-tls-verify"):
            ctx_ssl = ssl.create_default_context()
            ctx_ssl.check_hostname = False
            ctx_ssl.verify_mode = ssl.CERT_NONE
        else:
            ctx_ssl = ssl.create_default_context(cadata=ca) if ca else ssl.create_default_context()
            ctx_ssl.check_hostname = False      # clusters are addressed by IP as often as by name
        cert = _material(us, "client-certificate", base_dir)
        key = _material(us, "client-key", base_dir)
        if cert and key:
            cp, kp = _tmpfile(cert), _tmpfile(key)
            try:
                ctx_ssl.load_cert_chain(cp, kp)
            finally:
                os.unlink(cp)
                os.unlink(kp)
    return Resolved(server, us.get("token"), ctx_ssl, ctx.get("namespace"), ca)


def resolve_webhook(path):
    """A webhook kubeconfig (`--*-webhook-config-file`, ImagePolicyWebhook's kubeConfigFile):
    the current context, or — with none set — the cluster and user named "" (client-go's
    non-interactive loading with empty overrides). Missing server or unreadable TLS files raise."""
    with open(path) as f:
        cfg = yaml.safe_load(f) or {}
    base = os.path.dirname(os.path.abspath(path))
    cfg = dict(cfg)
    for k in ("clusters", "users", "contexts"):
        cfg[k] = [dict(e, name=e.get("name") or "") for e in cfg.get(k) or ()]
    cur = cfg["current-context"] = cfg.get("current-context") or ""
    if not any(c["name"] == cur for c in cfg["contexts"]):
        cfg["contexts"].append({"name": cur, "context": {"cluster": "", "user": ""}})
    r = resolve(cfg, cur, base)
    if r is None or not r.server:
        raise ValueError(f"webhook kubeconfig {path}: invalid configuration: no server found")
    return r


def client_from(path=None, context=None, **kw):
    from .rest import Client
    cfg, p = load(path)
    r = resolve(cfg, context, os.path.dirname(os.path.abspath(p)))
    if r is None:
        raise ValueError(f"kubeconfig {p}: no usable context")
    return Client(r.server, token=r.token, ssl_context=r.ssl_context, **kw)
