"""kubeadm phases (see package docstring for the reference map)."""
from __future__ import annotations

import base64
import hashlib
import ipaddress
import json
import os
import random
import shutil
import socket
import string
import sys
import time

import yaml

from ..api.meta import now_rfc3339
from ..client import clientcmd
from ..native import crypto

VERSION = "v1.9.0-amd.0"
CA, APISERVER, APISERVER_KUBELET_CLIENT, SA = "ca", "apiserver", "apiserver-kubelet-client", "sa"
FRONT_PROXY_CA, FRONT_PROXY_CLIENT = "front-proxy-ca", "front-proxy-client"
ADMIN_CONF, KUBELET_CONF, CM_CONF, SCHED_CONF, BOOTSTRAP_KUBELET_CONF = (
    "admin.conf", "kubelet.conf", "controller-manager.conf", "scheduler.conf", "bootstrap-kubelet.conf")
DEFAULT_ADMISSION = ["NamespaceLifecycle", "LimitRanger", "ServiceAccount", "DefaultStorageClass",
                     "DefaultTolerationSeconds", "NodeRestriction", "ResourceV2", "ResourceQuota"]
BOOTSTRAP_GROUP = "system:bootstrappers:kubeadm:default-node-token"


def default_config(**over):
    cfg = {"apiVersion": "kubeadm.k8s.io/v1alpha1", "kind": "MasterConfiguration",
           "api": {"advertiseAddress": "127.0.0.1", "bindPort": 6443},
           "networking": {"serviceSubnet": "10.96.0.0/12", "podSubnet": "10.244.0.0/16", "dnsDomain": "cluster.local"},
           "kubernetesVersion": VERSION, "nodeName": socket.gethostname().lower(),
           "authorizationModes": ["Node", "RBAC"], "tokenTTL": "24h0m0s", "token": "",
           "certificatesDir": "/etc/kubernetes/pki", "kubernetesDir": "/etc/kubernetes",
           "etcd": {"dataDir": "/var/lib/kamd-etcd"}, "featureGates": {"DevicePlugins": True}}
    for k, v in over.items():
        if isinstance(v, dict) and isinstance(cfg.get(k), dict):
            cfg[k].update(v)
        elif v is not None:
            cfg[k] = v
    return cfg


def _write(path, data, mode=0o644):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, mode), "w") as f:
        f.write(data)


def _read(path):
    with open(path) as f:
        return f.read()


# ------------------------------------------------------------------------------------ preflight
def preflight(cfg, kind="master"):
    """Checks (`app/preflight/checks.go`): ports free, manifest dir empty, ROCm devices."""
    warnings, errors = [], []
    if kind == "master":
        s = socket.socket()
        try:
            s.bind((cfg["api"]["advertiseAddress"], cfg["api"]["bindPort"]))
        except OSError:
            errors.append(f"Port {cfg['api']['bindPort']} is in use")
        finally:
            s.close()
        mdir = os.path.join(cfg["kubernetesDir"], "manifests")
        if os.path.isdir(mdir) and os.listdir(mdir):
            errors.append(f"{mdir} is not empty")
    if not os.path.exists("/dev/kfd"):
        warnings.append("/dev/kfd not found: this node will not advertise amd.com/gpu (no ROCm kernel driver)")
    if not any(os.path.exists(p) for p in ("/opt/rocm/lib/libamd_smi.so", "/opt/rocm/lib/libamd_smi.so.1")):
        warnings.append("libamd_smi not found under /opt/rocm/lib: the amd.com/gpu device plugin needs AMD SMI")
    return warnings, errors


# ------------------------------------------------------------------------------------ certs
def _sans(cfg):
    net = ipaddress.ip_network(cfg["networking"]["serviceSubnet"], strict=False)
    svc_ip = str(net.network_address + 1)
    dom = cfg["networking"].get("dnsDomain", "cluster.local")
    names = [cfg["nodeName"], "kubernetes", "kubernetes.default", "kubernetes.default.svc", f"kubernetes.default.svc.{dom}",
             "localhost"]
    ips = sorted({svc_ip, cfg["api"]["advertiseAddress"], "127.0.0.1"})
    return tuple([f"DNS:{n}" for n in names] + [f"IP:{i}" for i in ips])


def phase_certs(cfg):
    d = cfg["certificatesDir"]
    os.makedirs(d, exist_ok=True)
    made = []

    def have(base):
        return os.path.exists(os.path.join(d, base + ".crt")) and os.path.exists(os.path.join(d, base + ".key"))

    if not have(CA):
        ca, key = crypto.self_signed_ca("kubernetes", kind="rsa")
        _write(os.path.join(d, "ca.crt"), ca)
        _write(os.path.join(d, "ca.key"), key, 0o600)
        made.append(CA)
    ca, ca_key = _read(os.path.join(d, "ca.crt")), _read(os.path.join(d, "ca.key"))
    for base, cn, orgs, usage, sans in ((APISERVER, "kube-apiserver", (), "server", _sans(cfg)),
                                        (APISERVER_KUBELET_CLIENT, "kube-apiserver-kubelet-client", ("system:masters",),
                                         "client", ())):
        if not have(base):
            key = crypto.generate_key("rsa")
            cert = crypto.issue_cert(key_pem=key, cn=cn, orgs=orgs, ca_cert=ca, ca_key=ca_key, usage=usage, sans=sans)
            _write(os.path.join(d, base + ".crt"), cert)
            _write(os.path.join(d, base + ".key"), key, 0o600)
            made.append(base)
    if not os.path.exists(os.path.join(d, "sa.key")):
        key = crypto.generate_key("rsa")
        _write(os.path.join(d, "sa.key"), key, 0o600)
        _write(os.path.join(d, "sa.pub"), crypto.public_key(key))
        made.append(SA)
    if not have(FRONT_PROXY_CA):
        fca, fkey = crypto.self_signed_ca("front-proxy-ca", kind="rsa")
        _write(os.path.join(d, "front-proxy-ca.crt"), fca)
        _write(os.path.join(d, "front-proxy-ca.key"), fkey, 0o600)
        made.append(FRONT_PROXY_CA)
    if not have(FRONT_PROXY_CLIENT):
        fca, fkey = _read(os.path.join(d, "front-proxy-ca.crt")), _read(os.path.join(d, "front-proxy-ca.key"))
        key = crypto.generate_key("rsa")
        cert = crypto.issue_cert(key_pem=key, cn="front-proxy-client", ca_cert=fca, ca_key=fkey, usage="client")
        _write(os.path.join(d, "front-proxy-client.crt"), cert)
        _write(os.path.join(d, "front-proxy-client.key"), key, 0o600)
        made.append(FRONT_PROXY_CLIENT)
    return made


def ca_cert_hash(ca_pem):
    """`sha256:<hex>` of the CA's DER SubjectPublicKeyInfo (`pubkeypin.Hash`)."""
    pub = crypto.public_key(ca_pem)
    der = base64.b64decode("".join(l for l in pub.splitlines() if not l.startswith("-----")))
    return "sha256:" + hashlib.sha256(der).hexdigest()


# ------------------------------------------------------------------------------------ kubeconfig
def server_url(cfg):
    return f"https://{cfg['api']['advertiseAddress']}:{cfg['api']['bindPort']}"


def phase_kubeconfig(cfg):
    d, kd = cfg["certificatesDir"], cfg["kubernetesDir"]
    ca, ca_key = _read(os.path.join(d, "ca.crt")), _read(os.path.join(d, "ca.key"))
    out = []
    for fn, cn, orgs in ((ADMIN_CONF, "kubernetes-admin", ("system:masters",)),
                         (KUBELET_CONF, f"system:node:{cfg['nodeName']}", ("system:nodes",)),
                         (CM_CONF, "system:kube-controller-manager", ()),
                         (SCHED_CONF, "system:kube-scheduler", ())):
        path = os.path.join(kd, fn)
        if os.path.exists(path):
            continue
        key = crypto.generate_key()
        cert = crypto.issue_cert(key_pem=key, cn=cn, orgs=orgs, ca_cert=ca, ca_key=ca_key, usage="client")
        clientcmd.save(clientcmd.build("kubernetes", server_url(cfg), cn, ca_pem=ca, client_cert_pem=cert,
                                       client_key_pem=key), path)
        out.append(fn)
    return out


# ------------------------------------------------------------------------------------ manifests
def _static_pod(name, command, host_paths=(), version=VERSION):
    vols, mounts = [], []
    for i, p in enumerate(host_paths):
        vols.append({"name": f"v{i}", "hostPath": {"path": p, "type": "DirectoryOrCreate"}})
        mounts.append({"name": f"v{i}", "mountPath": p, "readOnly": False})
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": name, "namespace": "kube-system", "labels": {"component": name, "tier": "control-plane"},
                         "annotations": {"scheduler.alpha.kubernetes.io/critical-pod": ""}},
            "spec": {"hostNetwork": True, "priorityClassName": "system-cluster-critical",
                     "containers": [{"name": name, "image": f"kubernetes-amd/hyperkube:{version}", "command": command,
                                     "volumeMounts": mounts,
                                     "livenessProbe": {"httpGet": {"host": "127.0.0.1", "path": "/healthz",
                                                                   "port": 0}, "initialDelaySeconds": 15,
                                                       "timeoutSeconds": 15, "failureThreshold": 8}}],
                     "volumes": vols}}


def kubelet_flags(pki_dir):
    """The kubelet drop-in kubeadm installs (10-kubeadm.conf): privileged pods allowed (the
    control plane and add-ons need them), x509 client authentication against the cluster CA,
    requests authorized by the API server (Webhook)."""
    return ["--allow-privileged=true", "--client-ca-file", os.path.join(pki_dir, "ca.crt"),
            "--authorization-mode", "Webhook", "--authentication-token-webhook"]


def etcd_socket(cfg):
    return os.path.join(cfg["etcd"]["dataDir"], "kamd-etcd.sock")


def etcd_manifest(cfg):
    """Local store static pod (`phases/etcd/local.go` CreateLocalEtcdStaticPodManifestFile): the
    native kamd-etcd on a unix socket in its data dir, WAL beside it; skipped when
    `etcd.endpoints` names an external store."""
    from ..api.protobuf import SCHEMA_PATH
    from ..native import BIN_DIR
    data = cfg["etcd"]["dataDir"]
    cmd = [os.path.join(BIN_DIR, "kamd-etcd"), "--listen-unix", etcd_socket(cfg), "--wal", os.path.join(data, "wal"),
           "--pb-schema", SCHEMA_PATH]
    pod = _static_pod("etcd", cmd, (data,), cfg.get("kubernetesVersion") or VERSION)
    pod["spec"]["containers"][0].pop("livenessProbe", None)   # no HTTP endpoint: the kubelet restarts it on exit
    return pod


def control_plane_manifests(cfg):
    d, kd = cfg["certificatesDir"], cfg["kubernetesDir"]
    py = [sys.executable, "-m"]
    external = list(cfg["etcd"].get("endpoints") or ())
    store = ["--etcd-servers", external[0]] if external else ["--etcd-servers", "unix://" + etcd_socket(cfg)]
    api = py + ["kubernetes_amd.cmd.apiserver", "--bind-address", cfg["api"]["advertiseAddress"],
                "--port", str(cfg["api"]["bindPort"]),
                "--tls-cert-file", os.path.join(d, "apiserver.crt"), "--tls-private-key-file", os.path.join(d, "apiserver.key"),
                "--client-ca-file", os.path.join(d, "ca.crt"), "--service-account-key-file", os.path.join(d, "sa.pub"),
                "--enable-bootstrap-token-auth", "--authorization-mode", ",".join(cfg["authorizationModes"]),
                "--admission-control", ",".join(DEFAULT_ADMISSION),
                "--service-cluster-ip-range", cfg["networking"]["serviceSubnet"],
                "--storage-media-type", "application/vnd.kubernetes.protobuf",
                "--kubelet-client-certificate", os.path.join(d, APISERVER_KUBELET_CLIENT + ".crt"),
                "--kubelet-client-key", os.path.join(d, APISERVER_KUBELET_CLIENT + ".key")] + store
    cm = py + ["kubernetes_amd.cmd.controller_manager", "--kubeconfig", os.path.join(kd, CM_CONF), "--leader-elect",
               "--service-account-private-key-file", os.path.join(d, "sa.key"), "--root-ca-file", os.path.join(d, "ca.crt"),
               "--cluster-signing-cert-file", os.path.join(d, "ca.crt"), "--cluster-signing-key-file", os.path.join(d, "ca.key"),
               "--controllers", "*,bootstrapsigner,tokencleaner", "--use-service-account-credentials", "true"]
    sched = py + ["kubernetes_amd.cmd.scheduler", "--kubeconfig", os.path.join(kd, SCHED_CONF), "--leader-elect"]
    v = cfg.get("kubernetesVersion") or VERSION
    out = {"kube-apiserver": _static_pod("kube-apiserver", api, (d, cfg["etcd"]["dataDir"]), v),
           "kube-controller-manager": _static_pod("kube-controller-manager", cm, (d, kd), v),
           "kube-scheduler": _static_pod("kube-scheduler", sched, (kd,), v)}
    if not external:
        out["etcd"] = etcd_manifest(cfg)
    return out


def phase_etcd_local(cfg):
    mdir = os.path.join(cfg["kubernetesDir"], "manifests")
    path = os.path.join(mdir, "etcd.yaml")
    _write(path, yaml.safe_dump(etcd_manifest(cfg), sort_keys=False))
    return path


def phase_manifests(cfg):
    mdir = os.path.join(cfg["kubernetesDir"], "manifests")
    os.makedirs(mdir, exist_ok=True)
    written = []
    for name, pod in control_plane_manifests(cfg).items():
        p = os.path.join(mdir, name + ".yaml")
        _write(p, yaml.safe_dump(pod, sort_keys=False))
        written.append(p)
    return written


# ------------------------------------------------------------------------------------ tokens
TOKEN_ALPHABET = string.ascii_lowercase + string.digits


def generate_token():
    r = random.SystemRandom()
    return "".join(r.choice(TOKEN_ALPHABET) for _ in range(6)) + "." + "".join(r.choice(TOKEN_ALPHABET) for _ in range(16))


def _enc(v):
    return base64.b64encode(v.encode()).decode()


def token_secret(token, ttl_seconds=86400, usages=("authentication", "signing"), groups=(BOOTSTRAP_GROUP,), description=""):
    tid, tsec = token.split(".")
    data = {"token-id": _enc(tid), "token-secret": _enc(tsec)}
    for u in usages:
        data[f"usage-bootstrap-{u}"] = _enc("true")
    if groups:
        data["auth-extra-groups"] = _enc(",".join(groups))
    if ttl_seconds:
        data["expiration"] = _enc(now_rfc3339(time.time() + ttl_seconds))
    if description:
        data["description"] = _enc(description)
    return {"apiVersion": "v1", "kind": "Secret", "type": "bootstrap.kubernetes.io/token",
            "metadata": {"name": f"bootstrap-token-{tid}", "namespace": "kube-system"}, "data": data}


def parse_ttl(s):
    if not s or s in ("0", "0s"):
        return 0
    total, num = 0.0, ""
    units = {"h": 3600, "m": 60, "s": 1}
    for ch in s:
        if ch.isdigit() or ch == ".":
            num += ch
        elif ch in units:
            total += float(num or 0) * units[ch]
            num = ""
    return int(total + float(num or 0))


async def _ensure(client, res, obj, ns=None, update=False):
    from ..client.rest import APIStatusError
    try:
        return await client.create(res, obj, ns)
    except APIStatusError as e:
        if e.code != 409:
            raise
        if update:
            cur = await client.get(res, obj["metadata"]["name"], ns or obj["metadata"].get("namespace"))
            obj["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
            return await client.update(res, obj, ns or obj["metadata"].get("namespace"))
        return None


async def phase_bootstrap_token(client, cfg, token):
    await _ensure(client, "secrets", token_secret(token, parse_ttl(cfg.get("tokenTTL", "24h")),
                                                  description="The default bootstrap token generated by 'kubeadm init'."),
                  "kube-system")
    await phase_bootstrap_token_rbac(client)


async def phase_bootstrap_token_rbac(client):
    """RBAC for bootstrap tokens: post CSRs, auto-approve node client CSRs and their rotation."""
    rb = lambda name, role, group: {"metadata": {"name": name},  # noqa: E731
                                    "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": role},
                                    "subjects": [{"kind": "Group", "name": group, "apiGroup": "rbac.authorization.k8s.io"}]}
    await _ensure(client, "clusterrolebindings", rb("kubeadm:kubelet-bootstrap", "system:node-bootstrapper", BOOTSTRAP_GROUP))
    await _ensure(client, "clusterrolebindings", rb("kubeadm:node-autoapprove-bootstrap",
                                                    "system:certificates.k8s.io:certificatesigningrequests:nodeclient",
                                                    BOOTSTRAP_GROUP))
    await _ensure(client, "clusterrolebindings", rb("kubeadm:node-autoapprove-certificate-rotation",
                                                    "system:certificates.k8s.io:certificatesigningrequests:selfnodeclient",
                                                    "system:nodes"))


async def phase_cluster_info(client, cfg):
    ca = _read(os.path.join(cfg["certificatesDir"], "ca.crt"))
    kc = clientcmd.build("", server_url(cfg), "", ca_pem=ca)
    kc["users"], kc["contexts"], kc["current-context"] = [], [], ""
    await _ensure(client, "configmaps", {"metadata": {"name": "cluster-info", "namespace": "kube-public"},
                                         "data": {"kubeconfig": yaml.safe_dump(kc, sort_keys=False)}}, "kube-public", update=True)
    await _ensure(client, "roles", {"metadata": {"name": "kubeadm:bootstrap-signer-clusterinfo", "namespace": "kube-public"},
                                    "rules": [{"apiGroups": [""], "resources": ["configmaps"], "resourceNames": ["cluster-info"],
                                               "verbs": ["get"]}]}, "kube-public")
    await _ensure(client, "rolebindings", {"metadata": {"name": "kubeadm:bootstrap-signer-clusterinfo", "namespace": "kube-public"},
                                           "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "Role",
                                                       "name": "kubeadm:bootstrap-signer-clusterinfo"},
                                           "subjects": [{"kind": "User", "name": "system:anonymous"}]}, "kube-public")


async def phase_upload_config(client, cfg):
    await _ensure(client, "configmaps", {"metadata": {"name": "kubeadm-config", "namespace": "kube-system"},
                                         "data": {"MasterConfiguration": yaml.safe_dump(cfg, sort_keys=False)}},
                  "kube-system", update=True)


async def phase_mark_master(client, node_name):
    node = await client.get("nodes", node_name)
    taints = [t for t in (node.get("spec") or {}).get("taints") or () if t.get("key") != "node-role.kubernetes.io/master"]
    taints.append({"key": "node-role.kubernetes.io/master", "effect": "NoSchedule"})
    await client.patch("nodes", node_name, {"metadata": {"labels": {"node-role.kubernetes.io/master": ""}},
                                            "spec": {"taints": taints}})


async def phase_addons(client, cfg, update=False):
    """kube-proxy (ConfigMap + DaemonSet + its RBAC) and the amd.com/gpu device plugin DaemonSet;
    `update` replaces existing DaemonSets (kubeadm upgrade moves them to the new version)."""
    py = [sys.executable, "-m"]
    version = cfg.get("kubernetesVersion") or VERSION
    await _ensure(client, "serviceaccounts", {"metadata": {"name": "kube-proxy", "namespace": "kube-system"}}, "kube-system")
    await _ensure(client, "clusterrolebindings", {"metadata": {"name": "kubeadm:node-proxier"},
                                                  "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole",
                                                              "name": "system:node-proxier"},
                                                  "subjects": [{"kind": "ServiceAccount", "name": "kube-proxy",
                                                                "namespace": "kube-system"}]})
    await _ensure(client, "configmaps", {"metadata": {"name": "kube-proxy", "namespace": "kube-system"}, "data": {
        "config.conf": yaml.safe_dump({"apiVersion": "kubeproxy.config.k8s.io/v1alpha1", "kind": "KubeProxyConfiguration",
                                       "clusterCIDR": cfg["networking"].get("podSubnet", ""), "mode": "iptables"})}},
                  "kube-system", update=True)
    ds = lambda name, cmd, labels: {"apiVersion": "apps/v1", "kind": "DaemonSet",  # noqa: E731
                                    "metadata": {"name": name, "namespace": "kube-system", "labels": labels},
                                    "spec": {"selector": {"matchLabels": labels},
                                             "template": {"metadata": {"labels": labels},
                                                          "spec": {"hostNetwork": True, "serviceAccountName": name,
                                                                   "tolerations": [{"key": "node-role.kubernetes.io/master",
                                                                                    "effect": "NoSchedule"}],
                                                                   "containers": [{"name": name, "image": f"kubernetes-amd/hyperkube:{version}",
                                                                                   "command": cmd}]}}}}
    await _ensure(client, "daemonsets", ds("kube-proxy", py + ["kubernetes_amd.cmd.proxy", "--kubeconfig",
                                                               "/var/lib/kube-proxy/kubeconfig.conf"], {"k8s-app": "kube-proxy"}),
                  "kube-system", update=update)
    await _ensure(client, "serviceaccounts", {"metadata": {"name": "amd-gpu-device-plugin", "namespace": "kube-system"}},
                  "kube-system")
    await _ensure(client, "daemonsets", ds("amd-gpu-device-plugin", py + ["kubernetes_amd.cmd.device_plugin"],
                                           {"k8s-app": "amd-gpu-device-plugin"}), "kube-system", update=update)


# ------------------------------------------------------------------------------------ join
async def discover_cluster_info(server, token, ca_hashes=(), unsafe_skip_ca_verification=False):
    """Token discovery: anonymous GET of `kube-public/cluster-info`, verify the bootstrap signer's
    JWS for this token id, optionally pin the CA; returns (kubeconfig dict, CA PEM)."""
    import hmac
    import ssl
    from ..client.rest import Client
    tid, tsec = token.split(".")
    insecure = ssl.create_default_context()
    insecure.check_hostname = False
    insecure.verify_mode = ssl.CERT_NONE
    c = Client(server, ssl_context=insecure if server.startswith("https") else None)
    try:
        cm = await c.get("configmaps", "cluster-info", "kube-public")
    finally:
        await c.close()
    data = cm.get("data") or {}
    kc_text, sig = data.get("kubeconfig"), data.get(f"jws-kubeconfig-{tid}")
    if not kc_text or not sig:
        raise PermissionError(f"there is no JWS signed token in the cluster-info ConfigMap for token id {tid!r}")
    header, _, mac = sig.partition("..")
    body = base64.urlsafe_b64encode(kc_text.encode()).rstrip(b"=")
    want = hmac.new(token.encode(), header.encode() + b"." + body, hashlib.sha256).digest()
    got = base64.urlsafe_b64decode(mac + "=" * (-len(mac) % 4))
    if not hmac.compare_digest(want, got):
        raise PermissionError("failed to verify JWS signature of received cluster info object, can't trust this API Server")
    kc = yaml.safe_load(kc_text)
    ca = base64.b64decode(kc["clusters"][0]["cluster"]["certificate-authority-data"]).decode()
    if ca_hashes and ca_cert_hash(ca) not in ca_hashes:
        raise PermissionError(f"cluster CA found in cluster-info ConfigMap is not pinned: {ca_cert_hash(ca)}")
    if not ca_hashes and not unsafe_skip_ca_verification:
        raise PermissionError("--discovery-token-ca-cert-hash is required unless --discovery-token-unsafe-skip-ca-verification")
    del tsec
    return kc, ca


async def join(server, token, node_name, kubernetes_dir, ca_hashes=(), unsafe_skip_ca_verification=False, timeout=120.0):
    from ..kubelet.certificate import bootstrap_client_certificate
    kc, ca = await discover_cluster_info(server, token, ca_hashes, unsafe_skip_ca_verification)
    cluster_server = kc["clusters"][0]["cluster"]["server"]
    boot = os.path.join(kubernetes_dir, BOOTSTRAP_KUBELET_CONF)
    clientcmd.save(clientcmd.build("kubernetes", cluster_server, "tls-bootstrap-token-user", ca_pem=ca, token=token), boot)
    _write(os.path.join(kubernetes_dir, "pki", "ca.crt"), ca)
    conf = os.path.join(kubernetes_dir, KUBELET_CONF)
    await bootstrap_client_certificate(boot, conf, node_name, os.path.join(kubernetes_dir, "pki"), timeout)
    return conf


def reset(cfg):
    """`kubeadm reset`: remove manifests, kubeconfigs, PKI and etcd data."""
    kd = cfg["kubernetesDir"]
    for sub in ("manifests", "pki"):
        shutil.rmtree(os.path.join(kd, sub), ignore_errors=True)
    for fn in (ADMIN_CONF, KUBELET_CONF, CM_CONF, SCHED_CONF, BOOTSTRAP_KUBELET_CONF):
        p = os.path.join(kd, fn)
        if os.path.exists(p):
            os.unlink(p)
    shutil.rmtree(cfg["etcd"]["dataDir"], ignore_errors=True)
    if cfg["certificatesDir"] != os.path.join(kd, "pki"):
        shutil.rmtree(cfg["certificatesDir"], ignore_errors=True)


def dump(obj):
    return json.dumps(obj, indent=1)
