"""Service-account token controller, bootstrap signer / token cleaner, CSR approve + sign (kubelet
TLS bootstrap flow), cluster-role aggregation, TTL controller.

Parity: `pkg/controller/serviceaccount/tokens_controller_test.go`,
`pkg/controller/bootstrap/{bootstrapsigner,tokencleaner}_test.go`,
`pkg/controller/certificates/approver/sarapprove_test.go`, `signer/cfssl_signer_test.go`,
`pkg/controller/clusterroleaggregation/clusterroleaggregation_controller_test.go`,
`pkg/controller/ttl/ttl_controller_test.go`.
"""
import asyncio
import base64
import time

from kubernetes_amd.api.meta import now_rfc3339
from kubernetes_amd.apiserver.auth import User
from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client.rest import Client
from kubernetes_amd.controllers.certificates import jws_detached, ttl_for
from kubernetes_amd.controllers.manager import ControllerManager
from kubernetes_amd.native import crypto


async def eventually(fn, timeout=10.0):
    end = time.monotonic() + timeout
    while True:
        r = await fn()
        if r:
            return r
        if time.monotonic() > end:
            raise AssertionError("condition not met")
        await asyncio.sleep(0.05)


def enc(v):
    return base64.b64encode(v.encode()).decode()


def test_identity_controllers(run, tmp_path):
    sa_key = crypto.generate_key("rsa", 2048)
    (tmp_path / "sa.key").write_text(sa_key)
    ca, ca_key = crypto.self_signed_ca("kubernetes")

    async def main():
        s = APIServer(authorization_modes=("RBAC",), enable_bootstrap_token_auth=True,
                      service_account_key_files=[str(tmp_path / "sa.key")],
                      tokens={"admin": User("admin", "0", ["system:masters"])})
        port = await s.start()
        url = f"http://127.0.0.1:{port}"
        admin = Client(url, token="admin")
        cm = ControllerManager(Client(url, token="admin"), ["serviceaccount", "serviceaccount-token", "bootstrapsigner",
                                                            "tokencleaner", "csrapproving", "csrsigning",
                                                            "clusterroleaggregation", "ttl"],
                               {"serviceaccount-token": {"private_key": sa_key, "root_ca": ca},
                                "csrsigning": {"ca_cert": ca, "ca_key": ca_key}})
        await cm.start()
        try:
            # 1. every namespace's default SA gets a token secret that authenticates
            sa = await eventually(lambda: _get_sa_with_secret(admin, "default", "default"))
            sec = await admin.get("secrets", sa["secrets"][0]["name"], "default")
            assert sec["type"] == "kubernetes.io/service-account-token"
            tok = base64.b64decode(sec["data"]["token"]).decode()
            assert base64.b64decode(sec["data"]["ca.crt"]).decode() == ca
            tr = await admin.create("tokenreviews", {"spec": {"token": tok}})
            assert tr["status"]["user"]["username"] == "system:serviceaccount:default:default"

            # 2. bootstrap signer signs cluster-info; token cleaner removes expired tokens
            await admin.create("configmaps", {"metadata": {"name": "cluster-info", "namespace": "kube-public"},
                                              "data": {"kubeconfig": "apiVersion: v1\nclusters: []\n"}})
            await admin.create("secrets", {"metadata": {"name": "bootstrap-token-abcdef", "namespace": "kube-system"},
                                           "type": "bootstrap.kubernetes.io/token",
                                           "data": {"token-id": enc("abcdef"), "token-secret": enc("0123456789abcdef"),
                                                    "usage-bootstrap-signing": enc("true"),
                                                    "usage-bootstrap-authentication": enc("true")}})

            async def signed():
                ci = await admin.get("configmaps", "cluster-info", "kube-public")
                return ci["data"].get("jws-kubeconfig-abcdef")
            sig = await eventually(signed)
            assert sig == jws_detached("abcdef", "0123456789abcdef", "apiVersion: v1\nclusters: []\n")
            assert sig.count(".") == 2 and ".." in sig
            await admin.create("secrets", {"metadata": {"name": "bootstrap-token-old123", "namespace": "kube-system"},
                                           "type": "bootstrap.kubernetes.io/token",
                                           "data": {"token-id": enc("old123"), "token-secret": enc("0123456789abcdef"),
                                                    "expiration": enc(now_rfc3339(time.time() - 60))}})

            async def cleaned():
                try:
                    await admin.get("secrets", "bootstrap-token-old123", "kube-system")
                    return False
                except Exception:
                    return True
            await eventually(cleaned)

            # 3. kubelet TLS bootstrap: a bootstrap-token identity files a node client CSR,
            #    the approver (after a SubjectAccessReview) approves it, the signer issues a cert
            await admin.create("clusterroles", {"metadata": {"name": "nodeclient"}, "rules": [
                {"apiGroups": ["certificates.k8s.io"], "resources": ["certificatesigningrequests/nodeclient",
                                                                     "certificatesigningrequests"],
                 "verbs": ["create", "get", "list", "watch"]}]})
            await admin.create("clusterrolebindings", {"metadata": {"name": "bootstrappers-nodeclient"},
                "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "nodeclient"},
                "subjects": [{"kind": "Group", "name": "system:bootstrappers"}]})
            boot = Client(url, token="abcdef.0123456789abcdef")
            node_key = crypto.generate_key()
            req = crypto.make_csr(node_key, "system:node:mi355x-0", ["system:nodes"])
            await boot.create("certificatesigningrequests", {"metadata": {"name": "node-csr-1"}, "spec": {
                "request": base64.b64encode(req.encode()).decode(),
                "usages": ["digital signature", "key encipherment", "client auth"],
                "username": "forged-user"}})

            async def issued():
                c = await boot.get("certificatesigningrequests", "node-csr-1")
                return c if (c.get("status") or {}).get("certificate") else None
            csr = await eventually(issued)
            assert csr["spec"]["username"] == "system:bootstrap:abcdef"       # set by the server
            assert csr["status"]["conditions"][0]["reason"] == "AutoApproved"
            cert = base64.b64decode(csr["status"]["certificate"]).decode()
            assert crypto.cert_subject(cert) == ("system:node:mi355x-0", ["system:nodes"])
            assert crypto.verify_cert(cert, ca)[0]
            # a server-auth CSR is not auto-approved
            req2 = crypto.make_csr(node_key, "system:node:mi355x-0", ["system:nodes"])
            await boot.create("certificatesigningrequests", {"metadata": {"name": "node-csr-2"}, "spec": {
                "request": base64.b64encode(req2.encode()).decode(), "usages": ["digital signature", "server auth"]}})
            await asyncio.sleep(0.3)
            assert not (await admin.get("certificatesigningrequests", "node-csr-2")).get("status", {}).get("conditions")
            await boot.close()

            # 4. aggregated cluster roles
            await admin.create("clusterroles", {"metadata": {"name": "gpu-view", "labels": {"rbac.amd.com/aggregate-to-gpu": "true"}},
                                                "rules": [{"apiGroups": [""], "resources": ["nodes"], "verbs": ["get"]}]})
            await admin.create("clusterroles", {"metadata": {"name": "gpu-admin"}, "aggregationRule": {
                "clusterRoleSelectors": [{"matchLabels": {"rbac.amd.com/aggregate-to-gpu": "true"}}]}, "rules": []})

            async def aggregated():
                r = await admin.get("clusterroles", "gpu-admin")
                return r.get("rules")
            assert (await eventually(aggregated)) == [{"apiGroups": [""], "resources": ["nodes"], "verbs": ["get"]}]

            # 5. TTL annotation on nodes
            await admin.create("nodes", {"metadata": {"name": "n1"}})

            async def ttl():
                n = await admin.get("nodes", "n1")
                return (n["metadata"].get("annotations") or {}).get("node.alpha.kubernetes.io/ttl")
            assert await eventually(ttl) == "0"
            assert (ttl_for(50), ttl_for(400), ttl_for(900), ttl_for(1500), ttl_for(5000)) == (0, 15, 30, 60, 300)
        finally:
            await cm.stop()
            await admin.close()
            await s.stop()
    run(main(), timeout=60)


async def _get_sa_with_secret(c, ns, name):
    try:
        sa = await c.get("serviceaccounts", name, ns)
    except Exception:
        return None
    return sa if sa.get("secrets") else None


def test_ttl_boundaries_hysteresis():
    """ttl_controller_test.go TestDesiredTTL: adding past sizeMax steps up, deleting below
    sizeMin steps down — in between the TTL holds."""
    from kubernetes_amd.controllers.certificates import TTLController
    t = TTLController.__new__(TTLController)
    t.node_count, t.step = 0, 0
    t.enqueue = lambda n: None
    for _ in range(101):
        t._add({})
    assert t.desired_ttl == 15
    for _ in range(6):
        t._delete({})                 # 95 nodes: above sizeMin 90 of the 15 s step
    assert t.desired_ttl == 15
    for _ in range(6):
        t._delete({})                 # 89 nodes
    assert t.desired_ttl == 0
    assert ttl_for(20000) == 600


def test_csr_cleaner_criteria():
    """cleaner_test.go TestCleanerWithApprovedExpiredCSR table: approved+issued > 1 h, denied
    > 1 h, pending > 24 h and expired certificates are cleaned; fresh ones are kept."""
    from kubernetes_amd.controllers.certificates import CSRCleanerController as C
    now = time.time()

    def csr(created_ago, conds=(), cert=None):
        c = {"metadata": {"name": "c", "creationTimestamp": now_rfc3339(now - created_ago)},
             "status": {"conditions": [{"type": t, "lastUpdateTime": now_rfc3339(now - ago)} for t, ago in conds]}}
        if cert:
            c["status"]["certificate"] = base64.b64encode(cert.encode()).decode()
        return c
    ca, ca_key = crypto.self_signed_ca("kubernetes")
    good = crypto.issue_cert(key_pem=crypto.generate_key(), cn="system:node:a", ca_cert=ca, ca_key=ca_key, days=30)
    assert C.should_clean(csr(60)) is None
    assert C.should_clean(csr(25 * 3600)) == "pending"
    assert C.should_clean(csr(7200, [("Denied", 1800)])) is None
    assert C.should_clean(csr(7200, [("Denied", 5400)])) == "denied"
    assert C.should_clean(csr(7200, [("Approved", 5400)])) is None           # approved, not issued
    assert C.should_clean(csr(7200, [("Approved", 1800)], good)) is None
    assert C.should_clean(csr(7200, [("Approved", 5400)], good)) == "approved"
    assert C.should_clean(csr(7200, [("Approved", 1800)], good), now=now + 40 * 86400) == "approved"


def test_controller_manager_accepts_reference_controller_names():
    from kubernetes_amd.controllers.manager import CONTROLLERS, resolve
    assert {"csrcleaner", "pv-protection"} <= set(CONTROLLERS)
    assert "nodelifecycle" in resolve(["node"]) and "clusterroleaggregation" in resolve(["clusterrole-aggregation"])
    assert "nodelifecycle" not in resolve(["*", "-node"])
