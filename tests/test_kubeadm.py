"""kubeadm init phases + token discovery join + kubelet TLS bootstrap, against an in-process
API server running on exactly the certificates and flags kubeadm generated
(reference: cmd/kubeadm/app/phases/*, cmd/kubeadm/app/discovery/token/token.go)."""
import asyncio
import contextlib
import io
import os
import socket

import pytest
import yaml

from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client import clientcmd
from kubernetes_amd.client.rest import Client
from kubernetes_amd.controllers.manager import ControllerManager
from kubernetes_amd.kubeadm import cli, phases as P
from kubernetes_amd.native import crypto


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(tmp_path, port):
    return P.default_config(api={"advertiseAddress": "127.0.0.1", "bindPort": port}, nodeName="master-0",
                            certificatesDir=str(tmp_path / "k8s" / "pki"), kubernetesDir=str(tmp_path / "k8s"),
                            etcd={"dataDir": str(tmp_path / "etcd")})


def test_phases_offline(tmp_path):
    cfg = _cfg(tmp_path, 6443)
    made = P.phase_certs(cfg)
    assert set(made) == {P.CA, P.APISERVER, P.APISERVER_KUBELET_CLIENT, P.SA, P.FRONT_PROXY_CA, P.FRONT_PROXY_CLIENT}
    assert P.phase_certs(cfg) == []                           # idempotent
    pki = tmp_path / "k8s" / "pki"
    ca = (pki / "ca.crt").read_text()
    ok, msg = crypto.verify_cert((pki / "apiserver.crt").read_text(), ca)
    assert ok, msg
    assert crypto.cert_subject((pki / "apiserver-kubelet-client.crt").read_text()) == (
        "kube-apiserver-kubelet-client", ["system:masters"])
    assert oct((pki / "ca.key").stat().st_mode & 0o777) == "0o600"
    h = P.ca_cert_hash(ca)
    assert h.startswith("sha256:") and len(h) == 7 + 64 and P.ca_cert_hash(ca) == h

    assert sorted(P.phase_kubeconfig(cfg)) == sorted([P.ADMIN_CONF, P.KUBELET_CONF, P.CM_CONF, P.SCHED_CONF])
    kc, _ = clientcmd.load(str(tmp_path / "k8s" / P.KUBELET_CONF))
    r = clientcmd.resolve(kc)
    assert r.server == "https://127.0.0.1:6443" and r.ca_pem == ca
    import base64
    cert = base64.b64decode(kc["users"][0]["user"]["client-certificate-data"]).decode()
    assert crypto.cert_subject(cert) == ("system:node:master-0", ["system:nodes"])

    files = P.phase_manifests(cfg)
    api = yaml.safe_load(open([f for f in files if f.endswith("kube-apiserver.yaml")][0]))
    cmd = api["spec"]["containers"][0]["command"]
    assert "--enable-bootstrap-token-auth" in cmd and "Node,RBAC" in cmd
    adm = cmd[cmd.index("--admission-control") + 1].split(",")
    assert "ResourceV2" in adm and adm.index("NodeRestriction") < adm.index("ResourceQuota")
    assert api["spec"]["hostNetwork"] and api["metadata"]["namespace"] == "kube-system"
    # local store static pod; the API server joins it over its unix socket
    etcd = yaml.safe_load(open([f for f in files if f.endswith("etcd.yaml")][0]))
    ecmd = etcd["spec"]["containers"][0]["command"]
    assert ecmd[0].endswith("kamd-etcd") and ecmd[ecmd.index("--wal") + 1] == str(tmp_path / "etcd" / "wal")
    assert cmd[cmd.index("--etcd-servers") + 1] == "unix://" + ecmd[ecmd.index("--listen-unix") + 1]
    ext = P.control_plane_manifests(dict(cfg, etcd={"dataDir": "/x", "endpoints": ["tcp://10.0.0.5:2379"]}))
    assert "etcd" not in ext
    ecmd_api = ext["kube-apiserver"]["spec"]["containers"][0]["command"]
    assert ecmd_api[ecmd_api.index("--etcd-servers") + 1] == "tcp://10.0.0.5:2379"

    tok = P.generate_token()
    assert len(tok) == 23 and tok[6] == "."
    sec = P.token_secret(tok, 3600)
    assert sec["metadata"]["name"] == f"bootstrap-token-{tok[:6]}" and "expiration" in sec["data"]
    assert P.parse_ttl("24h0m0s") == 86400 and P.parse_ttl("1h30m") == 5400 and P.parse_ttl("0") == 0

    P.reset(cfg)
    assert not (tmp_path / "k8s" / "manifests").exists() and not pki.exists()


def test_init_join_tls_bootstrap(run, tmp_path):
    port = _free_port()
    cfg = _cfg(tmp_path, port)
    P.phase_certs(cfg)
    P.phase_kubeconfig(cfg)
    pki, kd = cfg["certificatesDir"], cfg["kubernetesDir"]
    token = P.generate_token()

    async def main():
        s = APIServer(tls_cert_file=f"{pki}/apiserver.crt", tls_private_key_file=f"{pki}/apiserver.key",
                      client_ca_file=f"{pki}/ca.crt", service_account_key_files=[f"{pki}/sa.pub"],
                      enable_bootstrap_token_auth=True, authorization_modes=("Node", "RBAC"))
        await s.start(port=port)
        admin_conf = os.path.join(kd, P.ADMIN_CONF)
        cm = ControllerManager(clientcmd.client_from(admin_conf), ["csrapproving", "csrsigning", "bootstrapsigner"],
                               {"csrsigning": {"cert_file": f"{pki}/ca.crt", "key_file": f"{pki}/ca.key"}})
        await cm.start()
        try:
            # the master's kubelet registers with its kubeadm-issued node credential
            kubelet = clientcmd.client_from(os.path.join(kd, P.KUBELET_CONF))
            await kubelet.create("nodes", {"metadata": {"name": "master-0"}})
            await kubelet.close()
            lines = []
            await cli.post_control_plane(cfg, admin_conf, token, 30, out=lines.append)
            admin = clientcmd.client_from(admin_conf)
            node = await admin.get("nodes", "master-0")
            assert node["metadata"]["labels"]["node-role.kubernetes.io/master"] == ""
            assert {"key": "node-role.kubernetes.io/master", "effect": "NoSchedule"} in node["spec"]["taints"]
            kcfg = await admin.get("configmaps", "kubeadm-config", "kube-system")
            assert yaml.safe_load(kcfg["data"]["MasterConfiguration"])["nodeName"] == "master-0"
            assert (await admin.get("daemonsets", "amd-gpu-device-plugin", "kube-system"))["metadata"]["name"]

            # wait for the bootstrap signer to sign cluster-info for our token
            for _ in range(200):
                ci = await admin.get("configmaps", "cluster-info", "kube-public")
                if f"jws-kubeconfig-{token[:6]}" in (ci.get("data") or {}):
                    break
                await asyncio.sleep(0.05)
            ca = open(f"{pki}/ca.crt").read()
            server = f"https://127.0.0.1:{port}"

            with pytest.raises(PermissionError):            # wrong CA pin
                await P.discover_cluster_info(server, token, ("sha256:" + "0" * 64,))
            with pytest.raises(PermissionError):            # unknown token id -> no signature
                await P.discover_cluster_info(server, "zzzzzz.0123456789abcdef", (P.ca_cert_hash(ca),))
            with pytest.raises(PermissionError):            # right id, wrong secret -> bad JWS
                await P.discover_cluster_info(server, token[:7] + "0123456789abcdef", (P.ca_cert_hash(ca),))

            node_dir = str(tmp_path / "node")
            conf = await P.join(server, token, "gpu-0", node_dir, (P.ca_cert_hash(ca),), timeout=20)
            kc, _ = clientcmd.load(conf)
            import base64
            cert = base64.b64decode(kc["users"][0]["user"]["client-certificate-data"]).decode()
            assert crypto.cert_subject(cert) == ("system:node:gpu-0", ["system:nodes"])
            assert crypto.verify_cert(cert, ca)[0]
            n = clientcmd.client_from(conf)
            await n.create("nodes", {"metadata": {"name": "gpu-0"}})
            from kubernetes_amd.client.rest import APIStatusError
            with pytest.raises(APIStatusError):             # NodeRestriction: cannot touch another node
                await n.patch("nodes", "master-0", {"metadata": {"labels": {"x": "y"}}})
            # client-certificate rotation over the current credential (selfnodeclient CSR)
            from kubernetes_amd.kubelet.certificate import CertificateRotator
            rot = CertificateRotator(conf, "gpu-0", str(tmp_path / "node" / "pki"), n)
            assert not await rot.maybe_rotate()              # fresh certificate: not due
            assert await rot.maybe_rotate(now=crypto.cert_not_after(cert) - 60)
            kc2, _ = clientcmd.load(conf)
            cert2 = base64.b64decode(kc2["users"][0]["user"]["client-certificate-data"]).decode()
            assert cert2 != cert and crypto.cert_subject(cert2) == ("system:node:gpu-0", ["system:nodes"])
            assert (await n.get("nodes", "gpu-0"))["metadata"]["name"] == "gpu-0"   # live client on the new cert
            await n.close()

            # kubeadm token create/list/delete through the CLI (its own event loop, in a thread)
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                rc = await asyncio.to_thread(cli.main, ["token", "create", "--kubeconfig", admin_conf, "--ttl", "1h"])
            assert rc == 0
            new_tok = buf.getvalue().strip()
            await admin.get("secrets", f"bootstrap-token-{new_tok[:6]}", "kube-system")
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                await asyncio.to_thread(cli.main, ["token", "list", "--kubeconfig", admin_conf])
            assert new_tok in buf.getvalue() and token in buf.getvalue()
            with contextlib.redirect_stdout(io.StringIO()):
                await asyncio.to_thread(cli.main, ["token", "delete", "--kubeconfig", admin_conf, new_tok])
            with pytest.raises(APIStatusError):
                await admin.get("secrets", f"bootstrap-token-{new_tok[:6]}", "kube-system")
            await admin.close()
        finally:
            await cm.stop()
            await s.stop()

    run(main(), timeout=90)


def test_local_etcd_manifest_runs(tmp_path):
    """The etcd and API server manifests' commands work together: objects written through the
    API server survive its restart because they live in the separate store process."""
    import subprocess
    import sys
    import time
    from kubernetes_amd.native import BIN_DIR
    if not os.path.exists(os.path.join(BIN_DIR, "kamd-etcd")):
        pytest.skip("kamd-etcd not built")
    cfg = _cfg(tmp_path, 0)
    (tmp_path / "etcd").mkdir()
    m = P.control_plane_manifests(cfg)
    store = subprocess.Popen(m["etcd"]["spec"]["containers"][0]["command"], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    api_cmd = m["kube-apiserver"]["spec"]["containers"][0]["command"]
    srv = api_cmd[api_cmd.index("--etcd-servers") + 1]
    procs = [store]
    try:
        sock = srv[len("unix://"):]
        for _ in range(100):
            if os.path.exists(sock):
                break
            time.sleep(0.05)

        def api():
            pf = tmp_path / "port"
            if pf.exists():
                pf.unlink()
            p = subprocess.Popen([sys.executable, "-m", "kubernetes_amd.cmd.apiserver", "--port", "0", "--port-file", str(pf),
                                  "--etcd-servers", srv], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            procs.append(p)
            for _ in range(600):
                if pf.exists() and pf.read_text().strip():
                    return p, f"http://127.0.0.1:{pf.read_text().strip()}"
                time.sleep(0.05)
            raise TimeoutError("apiserver did not start")

        async def put(url):
            c = Client(url)
            try:
                await c.create("configmaps", {"metadata": {"name": "kept", "namespace": "default"}, "data": {"a": "1"}})
            finally:
                await c.close()

        async def get(url):
            c = Client(url)
            try:
                return (await c.get("configmaps", "kept", "default"))["data"]
            finally:
                await c.close()
        p1, url = api()
        asyncio.run(put(url))
        p1.terminate()
        p1.wait(10)
        p2, url = api()
        assert asyncio.run(get(url)) == {"a": "1"}
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            p.wait(10)
