"""One storage, many served group/versions (pkg/master: deployments under apps/v1, apps/v1beta2,
apps/v1beta1 and extensions/v1beta1; rbac v1/v1beta1/v1alpha1; ...) and version-priority
ordered discovery (apimachinery version helpers)."""
import json

from kubernetes_amd.api import meta as m
from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client.rest import Client


def test_version_priority():
    vs = ["v1alpha1", "v1", "v1beta2", "v2beta1", "v1beta1", "v2alpha1", "v10"]
    assert sorted(vs, key=m.version_priority, reverse=True) == ["v10", "v1", "v2beta1", "v1beta2", "v1beta1",
                                                                "v2alpha1", "v1alpha1"]


def test_aliased_group_versions(run):
    async def main():
        s = APIServer()
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")

        async def req(method, path, body=None):
            st, b = await c.raw(method, path, json.dumps(body).encode() if body is not None else None)
            return st, (json.loads(b) if b[:1] == b"{" else b)
        try:
            dep = {"apiVersion": "extensions/v1beta1", "kind": "Deployment", "metadata": {"name": "old"},
                   "spec": {"replicas": 1, "selector": {"matchLabels": {"a": "b"}},
                            "template": {"metadata": {"labels": {"a": "b"}},
                                         "spec": {"containers": [{"name": "c", "image": "x"}]}}}}
            st, out = await req("POST", "/apis/extensions/v1beta1/namespaces/default/deployments", dep)
            assert st == 201 and out["apiVersion"] == "extensions/v1beta1"
            for gv in ("apps/v1", "apps/v1beta2", "apps/v1beta1", "extensions/v1beta1"):
                st, got = await req("GET", f"/apis/{gv}/namespaces/default/deployments/old")
                assert st == 200 and got["apiVersion"] == gv and got["metadata"]["name"] == "old"
            st, lst = await req("GET", "/apis/apps/v1beta2/namespaces/default/deployments")
            assert lst["items"][0]["apiVersion"] == "apps/v1beta2"
            st, _ = await req("GET", "/apis/extensions/v1beta1/namespaces/default/statefulsets")
            assert st == 404                                   # not served in extensions
            st, out = await req("POST", "/apis/rbac.authorization.k8s.io/v1beta1/clusterroles",
                                {"apiVersion": "rbac.authorization.k8s.io/v1beta1", "kind": "ClusterRole",
                                 "metadata": {"name": "beta-role"}, "rules": []})
            assert st == 201
            assert (await c.get("clusterroles", "beta-role"))["apiVersion"] == "rbac.authorization.k8s.io/v1"
            st, apps = await req("GET", "/apis/apps")
            assert [v["version"] for v in apps["versions"]] == ["v1", "v1beta2", "v1beta1"]
            assert apps["preferredVersion"]["version"] == "v1"
            st, ext = await req("GET", "/apis/extensions/v1beta1")
            names = {r["name"] for r in ext["resources"]}
            assert {"deployments", "daemonsets", "replicasets", "ingresses", "podsecuritypolicies"} <= names
            st, groups = await req("GET", "/apis")
            g = {x["name"]: x for x in groups["groups"]}
            assert g["batch"]["preferredVersion"]["version"] == "v1"
            assert "v2alpha1" in [v["version"] for v in g["batch"]["versions"]]
            assert g["autoscaling"]["preferredVersion"]["version"] == "v1"
        finally:
            await c.close()
            await s.stop()
    run(main())


def test_componentstatuses_podtemplates_events_alias(run):
    from kubernetes_amd.utils.httpserver import HTTPServer, Response

    async def main():
        healthy = HTTPServer(lambda req: _ok())
        hport = await healthy.start("127.0.0.1", 0)
        s = APIServer(component_endpoints={"scheduler": f"http://127.0.0.1:{hport}/healthz",
                                           "controller-manager": "http://127.0.0.1:1/healthz"})
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        try:
            st, body = await c.raw("GET", "/api/v1/componentstatuses")
            cs = {i["metadata"]["name"]: i["conditions"][0] for i in json.loads(body)["items"]}
            assert cs["scheduler"]["status"] == "True" and cs["etcd-0"]["status"] == "True"
            assert cs["controller-manager"]["status"] == "False" and cs["controller-manager"]["error"]
            st, body = await c.raw("GET", "/api/v1/componentstatuses/scheduler")
            assert st == 200 and json.loads(body)["metadata"]["name"] == "scheduler"
            await c.create("podtemplates", {"metadata": {"name": "t"}, "template": {"spec": {"containers": [
                {"name": "c", "image": "x"}]}}}, "default")
            assert (await c.get("podtemplates", "t", "default"))["template"]["spec"]["containers"][0]["image"] == "x"
            await c.create("events", {"metadata": {"name": "e1"}, "involvedObject": {"kind": "Pod", "name": "p"},
                                      "reason": "Test", "message": "m"}, "default")
            st, body = await c.raw("GET", "/apis/events.k8s.io/v1beta1/namespaces/default/events/e1")
            assert st == 200 and json.loads(body)["apiVersion"] == "events.k8s.io/v1beta1"
        finally:
            await c.close()
            await s.stop()
            await healthy.stop()
    run(main())


async def _ok():
    from kubernetes_amd.utils.httpserver import Response
    return Response(200, b"ok", "text/plain")
