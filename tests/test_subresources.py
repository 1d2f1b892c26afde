"""Scale / rollback / proxy subresources and the per-kind create/update strategies.

Parity: `pkg/registry/extensions/deployment/storage/storage_test.go` (ScaleREST Get/Update,
RollbackREST), `pkg/registry/core/replicationcontroller/storage/storage_test.go` (autoscaling/v1
Scale), `pkg/registry/core/service/rest_test.go` (ResourceLocation: port name / number, no
endpoints), `pkg/registry/core/pod/strategy_test.go` (ResourceLocation), `pkg/registry/batch/job/
strategy_test.go` (generated selector), workload strategies' PrepareForCreate (status reset).
"""
import asyncio
import json

import pytest

from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.apiserver.subresources import legacy_proxy_path, split_scheme_name_port
from kubernetes_amd.client.rest import APIStatusError, Client

NS = "/api/v1/namespaces/default"


def _dep(name="web", replicas=2):
    return {"metadata": {"name": name, "namespace": "default"}, "spec": {
        "replicas": replicas, "selector": {"matchLabels": {"app": name}},
        "template": {"metadata": {"labels": {"app": name}}, "spec": {"containers": [{"name": "c", "image": "x"}]}}}}


async def _api():
    api = APIServer()
    c = Client(f"http://127.0.0.1:{await api.start()}")
    return api, c


async def _req(c, method, path, body=None, ctype="application/json"):
    st, data = await c.raw(method, path, None if body is None else json.dumps(body).encode(), ctype)
    return st, (json.loads(data) if data[:1] in (b"{", b"[") else data)


def test_scale_subresource(run):
    async def main():
        api, c = await _api()
        try:
            d = await c.create("deployments", _dep())
            st, sc = await _req(c, "GET", "/apis/apps/v1/namespaces/default/deployments/web/scale")
            assert st == 200 and sc["apiVersion"] == "autoscaling/v1" and sc["kind"] == "Scale"
            assert sc["spec"] == {"replicas": 2} and sc["status"]["selector"] == "app=web"
            assert sc["metadata"]["resourceVersion"] == d["metadata"]["resourceVersion"]
            st, ext = await _req(c, "GET", "/apis/extensions/v1beta1/namespaces/default/deployments/web/scale")
            assert ext["apiVersion"] == "extensions/v1beta1" and ext["status"]["selector"] == {"app": "web"}
            assert ext["status"]["targetSelector"] == "app=web"
            # PUT: spec.replicas lands on the deployment, generation bumps
            st, out = await _req(c, "PUT", "/apis/apps/v1/namespaces/default/deployments/web/scale",
                                 {"metadata": {"name": "web"}, "spec": {"replicas": 5}})
            assert st == 200 and out["spec"]["replicas"] == 5
            got = await c.get("deployments", "web", "default")
            assert got["spec"]["replicas"] == 5 and got["metadata"]["generation"] == 2
            # a stale resourceVersion is a conflict; negative replicas are invalid
            st, err = await _req(c, "PUT", "/apis/apps/v1/namespaces/default/deployments/web/scale",
                                 {"metadata": {"name": "web", "resourceVersion": sc["metadata"]["resourceVersion"]},
                                  "spec": {"replicas": 1}})
            assert st == 409, err
            st, err = await _req(c, "PUT", "/apis/apps/v1/namespaces/default/deployments/web/scale",
                                 {"metadata": {"name": "web"}, "spec": {"replicas": -1}})
            assert st == 422 and "spec.replicas" in err["message"]
            st, out = await _req(c, "PATCH", "/apis/apps/v1/namespaces/default/deployments/web/scale",
                                 {"spec": {"replicas": 3}}, "application/merge-patch+json")
            assert st == 200 and (await c.get("deployments", "web", "default"))["spec"]["replicas"] == 3
            # RC: autoscaling/v1 with the map selector printed as a string
            await c.create("replicationcontrollers", {"metadata": {"name": "rc", "namespace": "default"}, "spec": {
                "replicas": 1, "selector": {"app": "rc", "tier": "x"},
                "template": {"metadata": {"labels": {"app": "rc", "tier": "x"}},
                             "spec": {"containers": [{"name": "c", "image": "x"}]}}}})
            st, rsc = await _req(c, "GET", f"{NS}/replicationcontrollers/rc/scale")
            assert rsc["apiVersion"] == "autoscaling/v1" and rsc["status"]["selector"] == "app=rc,tier=x"
            st, _ = await _req(c, "PUT", f"{NS}/replicationcontrollers/rc/scale", {"spec": {"replicas": 4}})
            assert (await c.get("replicationcontrollers", "rc", "default"))["spec"]["replicas"] == 4
            # kinds without a scale subresource, unknown subresources: 404, never a write
            await c.create("configmaps", {"metadata": {"name": "cm", "namespace": "default"}, "data": {"a": "b"}})
            st, _ = await _req(c, "PUT", f"{NS}/configmaps/cm/scale", {"spec": {"replicas": 4}})
            assert st == 404
            st, _ = await _req(c, "PUT", f"{NS}/configmaps/cm/bogus", {"data": {"a": "overwritten"}})
            assert st == 404 and (await c.get("configmaps", "cm", "default"))["data"] == {"a": "b"}
            # discovery advertises them
            st, disc = await _req(c, "GET", "/apis/extensions/v1beta1")
            names = {r["name"] for r in disc["resources"]}
            assert {"deployments/scale", "deployments/rollback", "replicasets/scale"} <= names
            st, disc = await _req(c, "GET", "/api/v1")
            names = {r["name"] for r in disc["resources"]}
            assert {"replicationcontrollers/scale", "pods/proxy", "services/proxy", "nodes/proxy"} <= names
        finally:
            await c.close()
            await api.stop()
    run(main())


def test_deployment_rollback_subresource(run):
    async def main():
        api, c = await _api()
        try:
            await c.create("deployments", _dep())
            st, out = await _req(c, "POST", "/apis/extensions/v1beta1/namespaces/default/deployments/web/rollback",
                                 {"kind": "DeploymentRollback", "apiVersion": "extensions/v1beta1", "name": "web",
                                  "updatedAnnotations": {"kubernetes.io/change-cause": "undo"},
                                  "rollbackTo": {"revision": 1}})
            assert st == 200 and "rollback request for deployment" in out["message"]
            d = await c.get("deployments", "web", "default")
            assert d["spec"]["rollbackTo"] == {"revision": 1}
            assert d["metadata"]["annotations"]["kubernetes.io/change-cause"] == "undo"
            assert d["metadata"]["generation"] == 2
            st, _ = await _req(c, "POST", "/apis/apps/v1/namespaces/default/deployments/web/rollback",
                               {"name": "web", "rollbackTo": {"revision": 1}})
            assert st == 404                                   # no rollback in apps/v1
            st, _ = await _req(c, "POST", "/apis/apps/v1beta1/namespaces/default/deployments/web/rollback",
                               {"name": "web", "rollbackTo": {"revision": -2}})
            assert st == 422
        finally:
            await c.close()
            await api.stop()
    run(main())


async def _echo_backend():
    async def handle(r, w):
        try:
            while True:
                head = await r.readuntil(b"\r\n\r\n")
                lines = head.decode().split("\r\n")
                method, target, _ = lines[0].split(" ", 2)
                hdrs = {k.lower(): v.strip() for k, _, v in (ln.partition(":") for ln in lines[1:] if ln)}
                body = await r.readexactly(int(hdrs.get("content-length", "0")))
                out = json.dumps({"method": method, "target": target, "body": body.decode(),
                                  "x-test": hdrs.get("x-test", ""), "auth": hdrs.get("authorization", "")}).encode()
                w.write(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n%s" % (len(out), out))
                await w.drain()
        except (asyncio.IncompleteReadError, ConnectionError):
            w.close()
    srv = await asyncio.start_server(handle, "127.0.0.1", 0)
    return srv, srv.sockets[0].getsockname()[1]


def test_proxy_subresources(run):
    async def main():
        api, c = await _api()
        srv, port = await _echo_backend()
        try:
            # pod proxy: pod IP + explicit port
            await c.create("pods", {"metadata": {"name": "p", "namespace": "default"},
                                    "spec": {"containers": [{"name": "c", "image": "x"}]}})
            st, _ = await _req(c, "GET", f"{NS}/pods/p:{port}/proxy/metrics")
            assert st == 400                                   # no pod IP yet
            await c.patch("pods", "p", {"status": {"podIP": "127.0.0.1", "phase": "Running"}}, "default", "merge", "status")
            st, e = await _req(c, "GET", f"{NS}/pods/p:{port}/proxy/metrics?format=json")
            assert st == 200 and e["method"] == "GET" and e["target"] == "/metrics?format=json"
            # service proxy by port name and by port number; POST bodies and headers relayed
            await c.create("services", {"metadata": {"name": "svc", "namespace": "default"}, "spec": {
                "selector": {"app": "x"}, "ports": [{"name": "http", "port": 80, "targetPort": port}]}})
            st, _ = await _req(c, "GET", f"{NS}/services/svc:http/proxy/")
            assert st == 503                                   # no endpoints
            await c.create("endpoints", {"metadata": {"name": "svc", "namespace": "default"}, "subsets": [
                {"addresses": [{"ip": "127.0.0.1"}], "ports": [{"name": "http", "port": port}]}]})
            st, e = await _req(c, "POST", f"{NS}/services/svc:80/proxy/v1/infer", {"prompt": "hi"})
            assert st == 200 and e["method"] == "POST" and json.loads(e["body"]) == {"prompt": "hi"}
            assert e["target"] == "/v1/infer" and e["auth"] == ""
            st, e = await _req(c, "GET", f"{NS}/services/svc:http/proxy/a/b/")
            assert e["target"] == "/a/b/"
            st, _ = await _req(c, "GET", f"{NS}/services/svc:8080/proxy/")
            assert st == 503                                   # no such service port
            # deprecated /api/v1/proxy/... form
            st, e = await _req(c, "GET", f"/api/v1/proxy/namespaces/default/services/svc:http/healthz")
            assert st == 200 and e["target"] == "/healthz"
            # node proxy: the kubelet endpoint of the node
            await c.create("nodes", {"metadata": {"name": "n1"}, "status": {
                "addresses": [{"type": "InternalIP", "address": "127.0.0.1"}],
                "daemonEndpoints": {"kubeletEndpoint": {"Port": port}}}})
            st, e = await _req(c, "GET", "/api/v1/nodes/n1/proxy/stats/summary")
            assert st == 200 and e["target"] == "/stats/summary"
            st, e = await _req(c, "GET", "/api/v1/proxy/nodes/n1/pods")
            assert st == 200 and e["target"] == "/pods"
            # other kinds have no proxy
            st, _ = await _req(c, "GET", f"{NS}/configmaps/x/proxy/")
            assert st == 404
        finally:
            srv.close()
            await c.close()
            await api.stop()
    run(main())


def test_split_scheme_name_port_and_legacy_paths():
    assert split_scheme_name_port("svc") == ("", "svc", "")
    assert split_scheme_name_port("svc:http") == ("", "svc", "http")
    assert split_scheme_name_port("https:svc:443") == ("https", "svc", "443")
    with pytest.raises(Exception):
        split_scheme_name_port("a:b:c:d")
    assert legacy_proxy_path("/api/v1/proxy/namespaces/kube-system/services/dns:53/x/y") == \
        "/api/v1/namespaces/kube-system/services/dns:53/proxy/x/y"
    assert legacy_proxy_path("/api/v1/proxy/nodes/n1") == "/api/v1/nodes/n1/proxy"
    assert legacy_proxy_path("/api/v1/namespaces/default/pods") is None


def test_workload_strategies(run):
    async def main():
        api, c = await _api()
        try:
            d = _dep("s")
            d["status"] = {"replicas": 99, "readyReplicas": 99}
            got = await c.create("deployments", d)
            assert got["status"] == {} and got["metadata"]["generation"] == 1
            # annotation changes bump a deployment's generation; a status update does not
            got = await c.patch("deployments", "s", {"metadata": {"annotations": {"a": "b"}}}, "default")
            assert got["metadata"]["generation"] == 2
            got = await c.patch("deployments", "s", {"status": {"replicas": 2}}, "default", "merge", "status")
            assert got["metadata"]["generation"] == 2 and got["status"]["replicas"] == 2
            # a main-resource update cannot write status
            got = await c.patch("deployments", "s", {"status": {"replicas": 7}}, "default")
            assert got["status"]["replicas"] == 2
            # Job: generated selector unless manualSelector
            job = await c.create("jobs", {"metadata": {"name": "train", "namespace": "default"}, "spec": {
                "template": {"metadata": {"labels": {"app": "train"}},
                             "spec": {"restartPolicy": "Never", "containers": [{"name": "c", "image": "x"}]}}}})
            uid = job["metadata"]["uid"]
            assert job["spec"]["selector"] == {"matchLabels": {"controller-uid": uid}}
            assert job["spec"]["template"]["metadata"]["labels"] == {"app": "train", "controller-uid": uid,
                                                                     "job-name": "train"}
            manual = await c.create("jobs", {"metadata": {"name": "m", "namespace": "default"}, "spec": {
                "manualSelector": True, "selector": {"matchLabels": {"app": "m"}},
                "template": {"metadata": {"labels": {"app": "m"}},
                             "spec": {"restartPolicy": "Never", "containers": [{"name": "c", "image": "x"}]}}}})
            assert manual["spec"]["selector"] == {"matchLabels": {"app": "m"}}
            with pytest.raises(APIStatusError) as ei:
                await c.create("jobs", {"metadata": {"name": "bad", "namespace": "default"}, "spec": {
                    "selector": {"matchLabels": {"controller-uid": "not-mine"}},
                    "template": {"metadata": {"labels": {"controller-uid": "not-mine"}},
                                 "spec": {"restartPolicy": "Never", "containers": [{"name": "c", "image": "x"}]}}}})
            assert ei.value.code == 422
            # PV / PVC start Pending whatever the client sent
            pvc = await c.create("persistentvolumeclaims", {"metadata": {"name": "c", "namespace": "default"},
                                                            "spec": {"accessModes": ["ReadWriteOnce"],
                                                                     "resources": {"requests": {"storage": "1Gi"}}},
                                                            "status": {"phase": "Bound"}})
            assert pvc["status"] == {"phase": "Pending"}
            svc = await c.create("services", {"metadata": {"name": "lb", "namespace": "default"}, "spec": {
                "type": "LoadBalancer", "ports": [{"port": 80}]},
                "status": {"loadBalancer": {"ingress": [{"ip": "6.6.6.6"}]}}})
            assert svc["status"] == {"loadBalancer": {}}
        finally:
            await c.close()
            await api.stop()
    run(main())


def test_export(run):
    """`?export=true` (`genericregistry.Store.Export`): cluster-specific metadata stripped;
    without `exact` also the namespace, status, allocated cluster IPs / node ports, a pod's node
    and devices, and service-account token data."""
    async def main():
        api, c = await _api()
        try:
            await c.create("services", {"metadata": {"name": "np", "namespace": "default"}, "spec": {
                "type": "NodePort", "ports": [{"port": 80}]}})
            st, e = await _req(c, "GET", f"{NS}/services/np?export=true")
            assert st == 200 and "uid" not in e["metadata"] and "resourceVersion" not in e["metadata"]
            assert "namespace" not in e["metadata"] and "clusterIP" not in e["spec"]
            assert "nodePort" not in e["spec"]["ports"][0]
            st, e = await _req(c, "GET", f"{NS}/services/np?export=true&exact=true")
            assert e["metadata"]["namespace"] == "default" and e["spec"]["clusterIP"]
            await c.create("pods", {"metadata": {"name": "p", "namespace": "default"},
                                    "spec": {"containers": [{"name": "c", "image": "x"}]}})
            await c.patch("pods", "p", {"status": {"phase": "Running", "podIP": "10.1.2.3"}}, "default", "merge", "status")
            st, e = await _req(c, "GET", f"{NS}/pods/p?export=true")
            assert e["status"]["phase"] == "Pending" and "podIP" not in e["status"]
            await c.create("secrets", {"metadata": {"name": "tok", "namespace": "default",
                                                    "annotations": {"kubernetes.io/service-account.name": "default"}},
                                       "type": "kubernetes.io/service-account-token", "data": {"token": "YWJj"}})
            st, e = await _req(c, "GET", f"{NS}/secrets/tok?export=true")
            assert "data" not in e
        finally:
            await c.close()
            await api.stop()
    run(main())


def test_server_side_table(run):
    """`Accept: ...;as=Table` turns GET / LIST into a meta.k8s.io Table with kubectl's columns."""
    async def main():
        api, c = await _api()
        try:
            for n in ("a", "b"):
                await c.create("pods", {"metadata": {"name": n, "namespace": "default", "labels": {"x": "y"}},
                                        "spec": {"containers": [{"name": "c", "image": "x"}]}})
            tbl = {"Accept": "application/json;as=Table;v=v1alpha1;g=meta.k8s.io"}
            st, body = await c.http.request("GET", f"{NS}/pods", None, headers=tbl)
            t = json.loads(body)
            assert st == 200 and t["kind"] == "Table" and t["apiVersion"] == "meta.k8s.io/v1alpha1"
            names = [col["name"] for col in t["columnDefinitions"]]
            assert names[0] == "Name" and "Status" in names
            assert [r["cells"][0] for r in t["rows"]] == ["a", "b"]
            assert t["rows"][0]["object"]["kind"] == "PartialObjectMetadata"
            assert t["rows"][0]["object"]["metadata"]["labels"] == {"x": "y"}
            st, body = await c.http.request("GET", f"{NS}/pods/a?includeObject=Object", None, headers=tbl)
            t = json.loads(body)
            assert len(t["rows"]) == 1 and t["rows"][0]["object"]["kind"] == "Pod"
            st, body = await c.http.request("GET", f"{NS}/pods?includeObject=None", None, headers=tbl)
            assert "object" not in json.loads(body)["rows"][0]
            # plain JSON clients are unaffected
            assert (await c.get("pods", "a", "default"))["kind"] == "Pod"
        finally:
            await c.close()
            await api.stop()
    run(main())
