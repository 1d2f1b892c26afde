"""ImagePolicyWebhook: ported tables.

Reference: `plugin/pkg/admission/imagepolicy/admission_test.go` (TestNewFromConfig :67,
TestTLSConfig :413, TestWebhookCache :541, TestContainerCombinations :581, TestDefaultAllow
:776, TestAnnotationFiltering :869) and `config_test.go` TestConfigNormalization. The backend is
a TLS test server whose review logic is the reference's `mockService`; PKI comes from the native
crypto helpers. Durations in the config are the reference's raw numbers (seconds for the TTLs,
milliseconds for retryBackoff).
"""
import json
import ssl

import pytest

from kubernetes_amd.apiserver.admission import CREATE, AdmissionError, Attributes
from kubernetes_amd.apiserver.admission.security import (DEFAULT_ALLOW_TTL, DEFAULT_DENY_TTL, DEFAULT_RETRY_BACKOFF,
                                                         IMAGE_POLICY_FAILED_OPEN, MAX_ALLOW_TTL, MAX_DENY_TTL,
                                                         MAX_RETRY_BACKOFF, ImagePolicyWebhook,
                                                         normalize_image_policy_config)
from kubernetes_amd.native import crypto
from kubernetes_amd.utils.httpserver import HTTPServer, Response


@pytest.fixture(scope="module")
def pki(tmp_path_factory):
    d = tmp_path_factory.mktemp("pki")
    ca, ca_key = crypto.self_signed_ca("webhook-ca")
    bad_ca, _ = crypto.self_signed_ca("other-ca")
    skey = crypto.generate_key()
    scert = crypto.issue_cert(key_pem=skey, cn="images", ca_cert=ca, ca_key=ca_key, usage="server",
                              sans=("IP:127.0.0.1", "DNS:localhost"))
    ckey = crypto.generate_key()
    ccert = crypto.issue_cert(key_pem=ckey, cn="apiserver", ca_cert=ca, ca_key=ca_key, usage="client")
    out = {}
    for n, v in (("ca", ca), ("bad_ca", bad_ca), ("server_cert", scert), ("server_key", skey),
                 ("client_cert", ccert), ("client_key", ckey)):
        p = d / f"{n}.pem"
        p.write_text(v)
        out[n] = str(p)
    return out


class MockService:
    """admission_test.go mockService: allow/deny all, with "good"/"bad" image overrides."""

    def __init__(self, allow=False, status_code=200):
        self.allow, self.status_code = allow, status_code
        self.calls = 0
        self.annotations = None

    async def handler(self, req):
        self.calls += 1
        review = json.loads(req.body)
        spec = review["spec"]
        self.annotations = dict(spec.get("annotations") or {})
        if self.status_code != 200:
            return Response(self.status_code, b"{}")
        allowed = self.allow
        if spec["containers"][0]["image"] == "good":
            allowed = True
        if any(c["image"] == "bad" for c in spec["containers"]):
            allowed = False
        status = {"allowed": allowed}
        if not allowed:
            status["reason"] = "not allowed"
        return Response(200, json.dumps({"apiVersion": "imagepolicy.k8s.io/v1alpha1", "kind": "ImageReview",
                                         "status": status}).encode())


def server_ssl(pki, client_ca="ca"):
    ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
    ctx.load_cert_chain(pki["server_cert"], pki["server_key"])
    if client_ca:
        ctx.verify_mode = ssl.CERT_REQUIRED
        ctx.load_verify_locations(pki[client_ca])
    return ctx


def write_kubeconfig(tmp_path, url, ca=None, cert=None, key=None, name="kc.yaml"):
    cluster = {"server": url}
    if ca:
        cluster["certificate-authority"] = ca
    user = {}
    if cert:
        user["client-certificate"], user["client-key"] = cert, key
    p = tmp_path / name
    p.write_text(json.dumps({"clusters": [{"cluster": cluster}], "users": [{"user": user}]}))
    return str(p)


def new_webhook(tmp_path, url, pki, ttl=0, default_allow=False, client_cert=True, ca=True):
    kc = write_kubeconfig(tmp_path, url, pki["ca"] if ca else None, pki["client_cert"] if client_cert else None,
                          pki["client_key"])
    return ImagePolicyWebhook(None, {"imagePolicy": {"kubeConfigFile": kc, "allowTTL": ttl, "denyTTL": ttl,
                                                     "retryBackoff": 1, "defaultAllow": default_allow}})


def good_pod(image, init=None, annotations=None):
    spec = {"serviceAccountName": "default", "containers": [{"name": f"c{i}", "image": im}
                                                             for i, im in enumerate([image] if isinstance(image, str)
                                                                                    else image)]}
    if init:
        spec["initContainers"] = [{"name": "i", "image": init}]
    md = {"name": "p", "namespace": "namespace"}
    if annotations is not None:
        md["annotations"] = annotations
    return {"metadata": md, "spec": spec}


def attrs(pod):
    return Attributes(CREATE, "pods", "", "namespace", "p", pod)


async def validate(wh, pod):
    await wh.charge(attrs(pod))


async def serve(service, pki, client_ca="ca"):
    srv = HTTPServer(service.handler)
    port = await srv.start(ssl=server_ssl(pki, client_ca))
    return srv, f"https://127.0.0.1:{port}/review"


# -- config_test.go TestConfigNormalization ----------------------------------------------------

@pytest.mark.parametrize("cfg,want", [
    ({"allowTTL": 900, "denyTTL": 900, "retryBackoff": 150000}, {"allowTTL": 900.0, "denyTTL": 900.0,
                                                                "retryBackoff": 150.0}),
    ({"allowTTL": 0, "denyTTL": 0, "retryBackoff": 0}, {"allowTTL": DEFAULT_ALLOW_TTL, "denyTTL": DEFAULT_DENY_TTL,
                                                        "retryBackoff": DEFAULT_RETRY_BACKOFF}),
    ({"allowTTL": -1, "denyTTL": -1, "retryBackoff": -1}, {"allowTTL": 0.0, "denyTTL": 0.0, "retryBackoff": 0.0}),
    ({"allowTTL": 1, "denyTTL": 1, "retryBackoff": 1}, {"allowTTL": 1.0, "denyTTL": 1.0, "retryBackoff": 0.001}),
    ({"allowTTL": 1800, "denyTTL": 1800, "retryBackoff": 300000}, {"allowTTL": MAX_ALLOW_TTL, "denyTTL": MAX_DENY_TTL,
                                                                  "retryBackoff": MAX_RETRY_BACKOFF}),
])
def test_config_normalization(cfg, want):
    got = normalize_image_policy_config(cfg)
    for k, v in want.items():
        assert got[k] == pytest.approx(v), k


@pytest.mark.parametrize("cfg", [{"allowTTL": 1801}, {"denyTTL": 1801}, {"retryBackoff": 300001},
                                 {"allowTTL": -2}, {"denyTTL": -5}])
def test_config_out_of_range(cfg):
    with pytest.raises(ValueError, match="valid value is between"):
        normalize_image_policy_config(cfg)


def test_no_config_is_an_error():
    with pytest.raises(ValueError, match="no config specified"):
        ImagePolicyWebhook(None, None)


# -- TestNewFromConfig ---------------------------------------------------------------------------

def _kc(pki, clusters, contexts=None, current=None):
    doc = {"clusters": [{"name": n, "cluster": {"certificate-authority": ca, "server": "https://admission.example.com"}}
                        for n, ca in clusters],
           "users": [{"name": "a name", "user": {"client-certificate": pki["client_cert"],
                                                 "client-key": pki["client_key"]}}]}
    if contexts:
        doc["contexts"] = [{"name": "default", "context": {"cluster": contexts, "user": "a name"}}]
        doc["current-context"] = current or "default"
    return doc


@pytest.mark.parametrize("case,want_err", [
    ("single cluster and single user", True),
    ("multiple clusters with no context", True),
    ("multiple clusters with a context", False),
    ("cluster with bad certificate path specified", True),
])
def test_new_from_config(tmp_path, pki, case, want_err):
    docs = {
        "single cluster and single user": _kc(pki, [("foobar", pki["ca"])]),
        "multiple clusters with no context": _kc(pki, [("foobar", pki["ca"]), ("barfoo", "a bad certificate path")]),
        "multiple clusters with a context": _kc(pki, [("foobar", "a bad certificate path"), ("barfoo", pki["ca"])],
                                                contexts="barfoo"),
        "cluster with bad certificate path specified": _kc(pki, [("foobar", "a bad certificate path"),
                                                                 ("barfoo", pki["ca"])], contexts="foobar"),
    }
    p = tmp_path / "kc.json"
    p.write_text(json.dumps(docs[case]))
    cfg = {"imagePolicy": {"kubeConfigFile": str(p), "allowTTL": 500, "denyTTL": 500, "retryBackoff": 500,
                           "defaultAllow": True}}
    if want_err:
        with pytest.raises((ValueError, OSError)):
            ImagePolicyWebhook(None, cfg)
    else:
        wh = ImagePolicyWebhook(None, cfg)
        assert wh.url == "https://admission.example.com" and wh.allow_ttl == 500


# -- TestTLSConfig -------------------------------------------------------------------------------

@pytest.mark.parametrize("case,client_cert,client_ca,server_client_ca,want_allowed", [
    ("TLS setup between client and server", True, True, "ca", True),
    ("Server does not require client auth", False, True, None, True),
    ("Server does not require client auth, client provides it", True, True, None, True),
    ("Client does not trust server", True, False, "ca", False),
    ("Server does not trust client", True, True, "bad_ca", False),
])
def test_tls_config(run, tmp_path, pki, case, client_cert, client_ca, server_client_ca, want_allowed):
    async def main():
        svc = MockService(status_code=200)
        srv, url = await serve(svc, pki, server_client_ca)
        try:
            wh = new_webhook(tmp_path, url, pki, ttl=-1, client_cert=client_cert, ca=client_ca)
            pod = good_pod("img-1")
            svc.allow = True
            if not want_allowed:
                with pytest.raises(AdmissionError):
                    await validate(wh, pod)
                return
            await validate(wh, pod)
            svc.allow = False
            with pytest.raises(AdmissionError):
                await validate(wh, pod)
        finally:
            await srv.stop()
    run(main())


def test_insecure_backend_with_tls_material_fails(run, tmp_path, pki):
    """"Server is using insecure connection": an https kubeconfig against a plain-HTTP server."""
    async def main():
        svc = MockService(allow=True)
        srv = HTTPServer(svc.handler)
        port = await srv.start()
        try:
            wh = new_webhook(tmp_path, f"https://127.0.0.1:{port}/review", pki, ttl=-1)
            wh.timeout = 0.5
            with pytest.raises(AdmissionError):
                await validate(wh, good_pod("img"))
        finally:
            await srv.stop()
    run(main())


# -- TestWebhookCache ----------------------------------------------------------------------------

def test_webhook_cache(run, tmp_path, pki):
    async def main():
        svc = MockService(allow=True)
        srv, url = await serve(svc, pki)
        try:
            wh = new_webhook(tmp_path, url, pki, ttl=200)

            async def cases(pod, table):
                for code, want_err, _cached in table:
                    svc.status_code = code
                    if want_err:
                        with pytest.raises(AdmissionError):
                            await validate(wh, pod)
                    else:
                        await validate(wh, pod)

            await cases(good_pod("test"), [(500, True, False), (404, True, False), (403, True, False),
                                           (401, True, False), (200, False, False), (500, False, True)])
            # a different request calls the webhook again
            await cases(good_pod("test2"), [(500, True, False), (200, False, False), (500, False, True)])
        finally:
            await srv.stop()
    run(main())


def test_transient_failures_are_retried(run, tmp_path, pki):
    """util/webhook WithExponentialBackoff: 5xx is retried (5 steps), 4xx is not."""
    async def main():
        svc = MockService(allow=True, status_code=500)
        srv, url = await serve(svc, pki)
        try:
            wh = new_webhook(tmp_path, url, pki, ttl=-1)
            with pytest.raises(AdmissionError, match="Error contacting webhook: 500"):
                await validate(wh, good_pod("x"))
            assert svc.calls == 5
            svc.calls, svc.status_code = 0, 403
            with pytest.raises(AdmissionError):
                await validate(wh, good_pod("x"))
            assert svc.calls == 1
        finally:
            await srv.stop()
    run(main())


# -- TestContainerCombinations -------------------------------------------------------------------

@pytest.mark.parametrize("case,pod,want_allowed", [
    ("Single container allowed", good_pod("good"), True),
    ("Single container denied", good_pod("bad"), False),
    ("One good container, one bad", good_pod(["bad", "good"]), False),
    ("Multiple good containers", good_pod(["good", "good"]), True),
    ("Multiple bad containers", good_pod(["bad", "bad"]), False),
    ("Good container, bad init container", good_pod("good", init="bad"), False),
    ("Bad container, good init container", good_pod("bad", init="good"), False),
    ("Good container, good init container", good_pod("good", init="good"), True),
])
def test_container_combinations(run, tmp_path, pki, case, pod, want_allowed):
    async def main():
        svc = MockService(status_code=200)
        srv, url = await serve(svc, pki)
        try:
            wh = new_webhook(tmp_path, url, pki, ttl=0)
            if want_allowed:
                await validate(wh, pod)
            else:
                with pytest.raises(AdmissionError, match="image policy webhook backend denied one or more images: "
                                                         "not allowed"):
                    await validate(wh, pod)
        finally:
            await srv.stop()
    run(main())


# -- TestDefaultAllow ----------------------------------------------------------------------------

@pytest.mark.parametrize("image,default_allow,want_allowed", [
    ("bad", True, True), ("good", True, True), ("good", False, False), ("bad", False, False)])
def test_default_allow(run, tmp_path, pki, image, default_allow, want_allowed):
    async def main():
        svc = MockService(status_code=500)
        srv, url = await serve(svc, pki)
        try:
            wh = new_webhook(tmp_path, url, pki, ttl=0, default_allow=default_allow)
            pod = good_pod(image)
            if want_allowed:
                await validate(wh, pod)
                assert pod["metadata"]["annotations"][IMAGE_POLICY_FAILED_OPEN] == "true"
            else:
                with pytest.raises(AdmissionError):
                    await validate(wh, pod)
                assert IMAGE_POLICY_FAILED_OPEN not in (pod["metadata"].get("annotations") or {})
        finally:
            await srv.stop()
    run(main())


# -- TestAnnotationFiltering ---------------------------------------------------------------------

@pytest.mark.parametrize("annotations,out", [
    ({"test": "test", "another": "annotation", "": ""}, {}),
    ({"my.image-policy.k8s.io/test": "test", "other.image-policy.k8s.io/test2": "annotation", "test": "test",
      "another": "another", "": ""},
     {"my.image-policy.k8s.io/test": "test", "other.image-policy.k8s.io/test2": "annotation"}),
])
def test_annotation_filtering(run, tmp_path, pki, annotations, out):
    async def main():
        svc = MockService(allow=True)
        srv, url = await serve(svc, pki)
        try:
            wh = new_webhook(tmp_path, url, pki, ttl=0, default_allow=True)
            await validate(wh, good_pod("test", annotations=annotations))
            assert svc.annotations == out
        finally:
            await srv.stop()
    run(main())


def test_subresources_and_other_resources_are_ignored(run, tmp_path, pki):
    async def main():
        wh = new_webhook(tmp_path, "https://127.0.0.1:1/unreachable", pki, ttl=0)
        await wh.charge(Attributes(CREATE, "pods", "binding", "ns", "p", good_pod("bad")))
        await wh.charge(Attributes(CREATE, "configmaps", "", "ns", "c", {"metadata": {"name": "c"}}))
    run(main())


def test_apiserver_enforces_image_policy(run, tmp_path, pki):
    """End to end: the API server's chain refuses a pod with a bad image and admits a good one."""
    from kubernetes_amd.apiserver.server import APIServer
    from kubernetes_amd.client.rest import APIStatusError, Client

    async def main():
        svc = MockService(allow=False)
        srv, url = await serve(svc, pki)
        kc = write_kubeconfig(tmp_path, url, pki["ca"], pki["client_cert"], pki["client_key"])
        s = APIServer(admission_plugins=["NamespaceLifecycle", "ImagePolicyWebhook"],
                      admission_config={"ImagePolicyWebhook": {"imagePolicy": {"kubeConfigFile": kc}}})
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        try:
            with pytest.raises(APIStatusError) as e:
                await c.create("pods", {"metadata": {"name": "b"}, "spec": {"containers": [{"name": "c",
                                                                                            "image": "bad"}]}})
            assert e.value.code == 403 and "not allowed" in str(e.value)
            await c.create("pods", {"metadata": {"name": "g"}, "spec": {"containers": [{"name": "c", "image": "good"}]}})
        finally:
            await c.close()
            await s.stop()
            await srv.stop()
    run(main())
