"""OpenAPI v2 document, OIDC ID-token authentication, the audit webhook backend, and the
multi-worker flag pass-through (reference: routes/openapi.go, plugin/pkg/authenticator/token/oidc
oidc_test.go, plugin/pkg/audit/webhook/webhook_test.go)."""
import json
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from kubernetes_amd.apiserver import authn as an
from kubernetes_amd.apiserver.audit import AuditLogger, WebhookBackend
from kubernetes_amd.apiserver.auth import User
from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client import clientcmd
from kubernetes_amd.client.rest import APIStatusError, Client
from kubernetes_amd.native import crypto


def _serve(handler_fn):
    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def do_GET(self):
            code, body = handler_fn("GET", self.path, None)
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.end_headers()
            self.wfile.write(body)

        def do_POST(self):
            n = int(self.headers.get("Content-Length", 0))
            code, body = handler_fn("POST", self.path, self.rfile.read(n))
            self.send_response(code)
            self.end_headers()
            self.wfile.write(body)
    srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv, f"http://127.0.0.1:{srv.server_address[1]}"


def test_openapi_document(run):
    async def main():
        s = APIServer()
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        try:
            st, body = await c.raw("GET", "/openapi/v2")
            assert st == 200
            doc = json.loads(body)
            assert doc["swagger"] == "2.0"
            pods = doc["paths"]["/api/v1/namespaces/{namespace}/pods"]
            assert pods["get"]["operationId"] == "listCoreV1NamespacedPod"
            assert pods["post"]["operationId"] == "createCoreV1NamespacedPod"
            assert doc["paths"]["/apis/apps/v1/namespaces/{namespace}/deployments/{name}"]["patch"]["operationId"] == \
                "patchAppsV1NamespacedDeployment"
            assert doc["paths"]["/api/v1/nodes/{name}"]["get"]["operationId"] == "readCoreV1Node"
            pod = doc["definitions"]["io.k8s.api.core.v1.Pod"]
            assert pod["x-kubernetes-group-version-kind"] == [{"group": "", "version": "v1", "kind": "Pod"}]
            await c.create("customresourcedefinitions", {
                "apiVersion": "apiextensions.k8s.io/v1beta1", "metadata": {"name": "gpujobs.mi355x.amd.com"},
                "spec": {"group": "mi355x.amd.com", "version": "v1", "scope": "Namespaced",
                         "names": {"plural": "gpujobs", "kind": "GPUJob"},
                         "validation": {"openAPIV3Schema": {"properties": {"spec": {"properties": {
                             "gpus": {"type": "integer", "minimum": 1}}}}}}}})
            for _ in range(100):
                doc = json.loads((await c.raw("GET", "/swagger.json"))[1])
                if "com.amd.mi355x.v1.GPUJob" in doc["definitions"]:
                    break
                time.sleep(0.02)
            gj = doc["definitions"]["com.amd.mi355x.v1.GPUJob"]
            assert gj["properties"]["spec"]["properties"]["gpus"]["minimum"] == 1
            assert "/apis/mi355x.amd.com/v1/namespaces/{namespace}/gpujobs" in doc["paths"]
        finally:
            await c.close()
            await s.stop()
    run(main())


def test_jwk_round_trip():
    for kind in ("rsa", "ec"):
        key = crypto.generate_key(kind)
        jwk = an.pem_to_jwk(key, kid="k1")
        pem = an.jwk_to_pem(jwk)
        assert pem.strip() == crypto.public_key(key).strip()
        tok = an.jwt_sign(key, {"a": 1})
        assert an.jwt_verify([pem], tok) == {"a": 1}


def test_oidc_authentication(run):
    key = crypto.generate_key("rsa")
    jwks = {"keys": [an.pem_to_jwk(key, kid="main")]}
    state = {}

    def issuer(method, path, body):
        if path == "/.well-known/openid-configuration":
            return 200, json.dumps({"issuer": state["url"], "jwks_uri": state["url"] + "/keys"}).encode()
        if path == "/keys":
            return 200, json.dumps(jwks).encode()
        return 404, b"{}"
    srv, url = _serve(issuer)
    state["url"] = url

    def tok(**claims):
        base = {"iss": url, "aud": "kubernetes", "sub": "alice-id", "email": "alice@amd.com", "email_verified": True,
                "groups": ["ml-team"], "exp": time.time() + 600}
        base.update(claims)
        return an.jwt_sign(key, base)

    async def main():
        oidc = an.OIDCAuthenticator(url, "kubernetes", username_claim="email", groups_claim="groups",
                                    groups_prefix="oidc:")
        oidc._fetching.join(10)
        assert "main" in oidc.keys
        s = APIServer(authorization_modes=("RBAC",), oidc=oidc, tokens={"admin": User("admin", "0", ["system:masters"])})
        port = await s.start()
        admin = Client(f"http://127.0.0.1:{port}", token="admin")
        try:
            await admin.create("clusterrolebindings", {"metadata": {"name": "ml-view"}, "roleRef": {
                "apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "view"},
                "subjects": [{"kind": "Group", "name": "oidc:ml-team"}]})
            tr = await admin.create("tokenreviews", {"spec": {"token": tok()}})
            assert tr["status"]["authenticated"] and tr["status"]["user"]["username"] == "alice@amd.com"
            assert "oidc:ml-team" in tr["status"]["user"]["groups"]
            alice = Client(f"http://127.0.0.1:{port}", token=tok())
            await alice.list("pods", "default")                                   # view via group binding
            try:
                await alice.create("pods", {"metadata": {"name": "x"}, "spec": {"containers": [{"name": "c", "image": "i"}]}},
                                   "default")
                raise AssertionError("view must not create")
            except APIStatusError as e:
                assert e.code == 403
            await alice.close()
            for bad in (tok(aud="other"), tok(iss="https://evil"), tok(exp=time.time() - 5), tok(email_verified=False)):
                tr = await admin.create("tokenreviews", {"spec": {"token": bad}})
                assert not tr["status"].get("authenticated")
            other = crypto.generate_key("rsa")
            forged = an.jwt_sign(other, {"iss": url, "aud": "kubernetes", "email": "x@y", "exp": time.time() + 60})
            tr = await admin.create("tokenreviews", {"spec": {"token": forged}})
            assert not tr["status"].get("authenticated")
            sub_only = an.OIDCAuthenticator(url, "kubernetes", keys=oidc.keys)       # default claim: sub, prefixed
            assert sub_only.authenticate_token(tok()).name == f"{url}#alice-id"
        finally:
            await admin.close()
            await s.stop()
            srv.shutdown()
    run(main())


def test_audit_webhook_backend(run, tmp_path):
    got = []

    def sink(method, path, body):
        if method == "POST":
            got.append(json.loads(body))
        return 200, b"{}"
    srv, url = _serve(sink)
    kc = tmp_path / "audit-webhook.kubeconfig"
    clientcmd.save(clientcmd.build("audit", url + "/audit", "apiserver"), str(kc))

    async def main():
        wh = WebhookBackend(str(kc), max_batch=5, max_wait=0.05)
        audit = AuditLogger(None, webhook=wh)
        s = APIServer(audit=audit)
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        try:
            for i in range(12):
                await c.create("configmaps", {"metadata": {"name": f"cm{i}"}, "data": {}}, "default")
        finally:
            await c.close()
            await s.stop()
        audit.close()
    run(main())
    srv.shutdown()
    assert got and all(b["kind"] == "EventList" and b["apiVersion"] == "audit.k8s.io/v1beta1" for b in got)
    assert all(len(b["items"]) <= 5 for b in got)
    creates = [e for b in got for e in b["items"] if e["verb"] == "create" and e["objectRef"]["resource"] == "configmaps"]
    assert len(creates) == 12


def test_supervisor_passes_auth_flags():
    from kubernetes_amd.cmd.apiserver import _parser, passthrough_args
    a = _parser().parse_args(["--workers", "4", "--port", "6443", "--tls-cert-file", "c.crt", "--tls-private-key-file",
                              "c.key", "--client-ca-file", "ca.crt", "--enable-bootstrap-token-auth",
                              "--oidc-issuer-url", "https://idp", "--oidc-client-id", "k8s",
                              "--service-account-key-file", "a.pub", "--service-account-key-file", "b.pub",
                              "--authorization-mode", "Node,RBAC", "--anonymous-auth", "false"])
    args = passthrough_args(a)
    for flag in ("--tls-cert-file", "--client-ca-file", "--enable-bootstrap-token-auth", "--oidc-issuer-url",
                 "--authorization-mode"):
        assert flag in args
    assert args.count("--service-account-key-file") == 2
    assert "--workers" not in args and "--port" not in args
    assert args[args.index("--anonymous-auth") + 1] == "false"
