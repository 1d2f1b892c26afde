"""Authentication: x509 client certificates over TLS, bootstrap tokens, service-account JWTs,
union semantics (401 for a bad token, anonymous without credentials).

Parity: `staging/src/k8s.io/apiserver/pkg/authentication/request/x509/x509_test.go`,
`plugin/pkg/auth/authenticator/token/bootstrap/bootstrap_test.go`, `pkg/serviceaccount/jwt_test.go`.
"""
import base64
import ssl
import time

import pytest

from kubernetes_amd.api.meta import now_rfc3339
from kubernetes_amd.apiserver import authn as an
from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client.rest import APIStatusError, Client
from kubernetes_amd.native import crypto


def test_jwt_roundtrip_rsa_and_ec():
    for kind in ("rsa", "ec"):
        key = crypto.generate_key(kind)
        tok = an.jwt_sign(key, {"iss": "x", "n": 1})
        assert an.jwt_verify([crypto.public_key(key)], tok) == {"iss": "x", "n": 1}
        other = crypto.public_key(crypto.generate_key(kind))
        assert an.jwt_verify([other], tok) is None
        h, b, s = tok.split(".")
        forged = h + "." + an.b64url(b'{"iss":"x","n":2}') + "." + s
        assert an.jwt_verify([crypto.public_key(key)], forged) is None


def _pki(tmp_path):
    ca, ca_key = crypto.self_signed_ca("kubernetes-ca")
    skey = crypto.generate_key()
    scert = crypto.issue_cert(key_pem=skey, cn="kube-apiserver", ca_cert=ca, ca_key=ca_key, usage="server",
                              sans=("IP:127.0.0.1", "DNS:localhost"))
    ckey = crypto.generate_key()
    ccert = crypto.issue_cert(key_pem=ckey, cn="alice", orgs=("system:masters",), ca_cert=ca, ca_key=ca_key, usage="client")
    paths = {}
    for n, v in (("ca.crt", ca), ("apiserver.crt", scert), ("apiserver.key", skey), ("alice.crt", ccert), ("alice.key", ckey)):
        p = tmp_path / n
        p.write_text(v)
        paths[n] = str(p)
    return paths


def test_x509_client_cert_auth(run, tmp_path):
    paths = _pki(tmp_path)

    async def main():
        s = APIServer(tls_cert_file=paths["apiserver.crt"], tls_private_key_file=paths["apiserver.key"],
                      client_ca_file=paths["ca.crt"], authorization_modes=("RBAC",))
        port = await s.start()
        ctx = ssl.create_default_context(cafile=paths["ca.crt"])
        ctx.load_cert_chain(paths["alice.crt"], paths["alice.key"])
        alice = Client(f"https://127.0.0.1:{port}", ssl_context=ctx)
        anon_ctx = ssl.create_default_context(cafile=paths["ca.crt"])
        anon = Client(f"https://127.0.0.1:{port}", ssl_context=anon_ctx)
        try:
            # alice is in system:masters via her certificate's O= field
            await alice.create("configmaps", {"metadata": {"name": "c", "namespace": "default"}})
            ssar = await alice.create("selfsubjectaccessreviews", {"spec": {"resourceAttributes": {"verb": "delete", "resource": "nodes"}}})
            assert ssar["status"]["allowed"]
            with pytest.raises(APIStatusError) as e:
                await anon.list("configmaps", "default")
            assert e.value.code == 403
        finally:
            await alice.close()
            await anon.close()
            await s.stop()
    run(main())


def test_bootstrap_and_service_account_tokens(run, tmp_path):
    sa_key = crypto.generate_key("rsa", 2048)
    (tmp_path / "sa.key").write_text(sa_key)

    async def main():
        s = APIServer(enable_bootstrap_token_auth=True, service_account_key_files=[str(tmp_path / "sa.key")],
                      authorization_modes=("RBAC",), tokens={"admin": __import__("kubernetes_amd.apiserver.auth", fromlist=["User"]).User(
                          "admin", "0", ["system:masters"])})
        port = await s.start()
        admin = Client(f"http://127.0.0.1:{port}", token="admin")
        try:
            enc = lambda v: base64.b64encode(v.encode()).decode()  # noqa: E731
            await admin.create("secrets", {"metadata": {"name": "bootstrap-token-abcdef", "namespace": "kube-system"},
                                           "type": "bootstrap.kubernetes.io/token",
                                           "data": {"token-id": enc("abcdef"), "token-secret": enc("0123456789abcdef"),
                                                    "usage-bootstrap-authentication": enc("true"),
                                                    "auth-extra-groups": enc("system:bootstrappers:kubeadm:default-node-token")}})
            tr = await admin.create("tokenreviews", {"spec": {"token": "abcdef.0123456789abcdef"}})
            u = tr["status"]["user"]
            assert u["username"] == "system:bootstrap:abcdef"
            assert "system:bootstrappers:kubeadm:default-node-token" in u["groups"]
            assert not (await admin.create("tokenreviews", {"spec": {"token": "abcdef.0123456789abcdeX"}}))["status"]["authenticated"]
            # expired token
            await admin.patch("secrets", "bootstrap-token-abcdef", {"stringData": None, "data": {
                "expiration": enc(now_rfc3339(time.time() - 10))}}, "kube-system")
            assert not (await admin.create("tokenreviews", {"spec": {"token": "abcdef.0123456789abcdef"}}))["status"]["authenticated"]
            # service account JWT
            sa = await admin.create("serviceaccounts", {"metadata": {"name": "builder", "namespace": "default"}})
            await admin.create("secrets", {"metadata": {"name": "builder-token-x", "namespace": "default",
                                                        "annotations": {"kubernetes.io/service-account.name": "builder"}},
                                           "type": "kubernetes.io/service-account-token"})
            tok = an.service_account_token(sa_key, sa, "builder-token-x")
            tr = await admin.create("tokenreviews", {"spec": {"token": tok}})
            assert tr["status"]["user"]["username"] == "system:serviceaccount:default:builder"
            assert "system:serviceaccounts:default" in tr["status"]["user"]["groups"]
            sac = Client(f"http://127.0.0.1:{port}", token=tok)
            with pytest.raises(APIStatusError) as e:     # authenticated but not authorized
                await sac.list("secrets", "default")
            assert e.value.code == 403
            bad = Client(f"http://127.0.0.1:{port}", token="not-a-token")
            with pytest.raises(APIStatusError) as e:
                await bad.list("pods", "default")
            assert e.value.code == 401
            await bad.close()
            # revoking the secret revokes the token (service-account lookup)
            await admin.delete("secrets", "builder-token-x", "default")
            with pytest.raises(APIStatusError) as e:
                await sac.list("secrets", "default")
            assert e.value.code == 401
            await sac.close()
        finally:
            await admin.close()
            await s.stop()
    run(main())
