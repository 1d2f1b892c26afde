"""Protobuf wire/storage format: round trips, determinism, the `k8s\\0`
envelope, and a cross-check of the hand-written codec against google.protobuf messages
built from the same field numbers (the reference generated.proto ones)."""
from kubernetes_amd.api import protobuf as pb
from kubernetes_amd.api.codec import PROTOBUF
from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client.rest import Client
from kubernetes_amd.utils.protodesc import build

CORE = "k8s.io.api.core.v1."

POD = {
    "apiVersion": "v1", "kind": "Pod",
    "metadata": {"name": "train-0", "namespace": "ml", "uid": "9b1c", "resourceVersion": "42", "generation": 1,
                 "creationTimestamp": "2026-10-15T12:00:00Z", "labels": {"b": "2", "a": "1"},
                 "ownerReferences": [{"apiVersion": "batch/v1", "kind": "Job", "name": "train", "uid": "u1", "controller": True}]},
    "spec": {"containers": [{"name": "c", "image": "rocm/pytorch", "command": ["python", "train.py"],
                             "env": [{"name": "X", "value": "1"}],
                             "resources": {"limits": {"cpu": "4", "memory": "64Gi"}, "requests": {"cpu": "4"}},
                             "extendedResourceRequests": ["gpus"],
                             "readinessProbe": {"httpGet": {"path": "/ready", "port": 8080}, "periodSeconds": 5},
                             "ports": [{"containerPort": 8080, "protocol": "TCP"}]}],
             "volumes": [{"name": "data", "hostPath": {"path": "/data"}}, {"name": "cfg", "configMap": {"name": "cm"}}],
             "restartPolicy": "Never", "terminationGracePeriodSeconds": 30, "nodeName": "mi355x-0",
             "tolerations": [{"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"}],
             "extendedResources": [{"name": "gpus", "resources": {"limits": {"amd.com/gpu": "4"}, "requests": {"amd.com/gpu": "4"}},
                                    "affinity": {"required": [{"key": "amd.com/hbm", "operator": "Gt", "values": ["256Gi"]}]},
                                    "assigned": ["GPU-0", "GPU-1", "GPU-2", "GPU-3"]}]},
    "status": {"phase": "Running", "podIP": "10.0.0.5", "startTime": "2026-10-15T12:00:01Z",
               "conditions": [{"type": "Ready", "status": "True", "lastTransitionTime": "2026-10-15T12:00:02Z"}],
               "containerStatuses": [{"name": "c", "ready": True, "restartCount": 0,
                                      "state": {"running": {"startedAt": "2026-10-15T12:00:02Z"}}}]},
}

NODE = {"apiVersion": "v1", "kind": "Node", "metadata": {"name": "mi355x-0"},
        "spec": {"taints": [{"key": "k", "value": "v", "effect": "NoSchedule"}]},
        "status": {"capacity": {"amd.com/gpu": "8", "cpu": "256"},
                   "extendedResources": {"amd.com/gpu": {"resources": {
                       "GPU-0": {"id": "GPU-0", "health": "Healthy", "attributes": {"amd.com/arch": "gfx950", "amd.com/hbm": "288Gi"}},
                       "GPU-1": {"id": "GPU-1", "health": "Unhealthy", "attributes": {"amd.com/arch": "gfx950"}}}}},
                   "daemonEndpoints": {"kubeletEndpoint": {"Port": 10250}}}}


def test_round_trip_pod_node_binding():
    for obj in (POD, NODE, {"apiVersion": "v1", "kind": "Binding", "metadata": {"name": "p"},
                            "target": {"kind": "Node", "name": "n", "extendedResourceBinding": {"gpus": {"resources": ["a", "b"]}}}}):
        data = pb.encode_object(obj)
        assert data[:4] == b"k8s\x00"
        assert pb.decode_object(data) == obj


def test_deterministic_map_order():
    a = pb.encode_object(POD)
    p2 = dict(POD, metadata=dict(POD["metadata"], labels={"a": "1", "b": "2"}))
    assert pb.encode_object(p2) == a


def test_envelope_fields():
    data = pb.encode_object(NODE)
    api, kind, raw = pb.decode_unknown(data)
    assert (api, kind) == ("v1", "Node") and raw == pb.encode_message(CORE + "Node", {k: v for k, v in NODE.items() if k not in ("kind", "apiVersion")})


def test_cross_check_against_google_protobuf():
    """Same field numbers, built as real protobuf messages: byte-identical deterministic output."""
    M = build("k8s.io.api.core.v1", "xcheck.proto", {
        "ExtendedResourceList": [("resources", 1, "string", "rep", None)],
        "ObjectReference": [("kind", 1, "string", "opt", None), ("name", 3, "string", "opt", None),
                            ("extendedResourceBinding", 8, "message", "map", "ExtendedResourceList")],
        "ExtendedResource": [("id", 1, "string", "opt", None), ("health", 2, "string", "opt", None),
                             ("attributes", 3, "string", "map", None)],
        "ExtendedResourceDomain": [("resources", 1, "message", "map", "ExtendedResource")],
    }, syntax="proto2")
    ref = M["ObjectReference"](kind="Node", name="mi355x-0")
    ref.extendedResourceBinding["z"].resources.extend(["g3"])
    ref.extendedResourceBinding["a"].resources.extend(["g0", "g1"])
    ours = pb.encode_message(CORE + "ObjectReference", {"kind": "Node", "name": "mi355x-0",
                                                 "extendedResourceBinding": {"z": {"resources": ["g3"]},
                                                                             "a": {"resources": ["g0", "g1"]}}})
    assert ref.SerializeToString(deterministic=True) == ours
    dom = M["ExtendedResourceDomain"]()
    r = dom.resources["GPU-0"]
    r.id, r.health = "GPU-0", "Healthy"
    r.attributes["amd.com/arch"] = "gfx950"
    r.attributes["amd.com/hbm"] = "288Gi"
    ours = pb.encode_message(CORE + "ExtendedResourceDomain", {"resources": {"GPU-0": {
        "id": "GPU-0", "health": "Healthy", "attributes": {"amd.com/hbm": "288Gi", "amd.com/arch": "gfx950"}}}})
    assert dom.SerializeToString(deterministic=True) == ours
    # and google.protobuf parses ours
    back = M["ExtendedResourceDomain"].FromString(ours)
    assert back.resources["GPU-0"].attributes["amd.com/hbm"] == "288Gi"


def test_apiserver_protobuf_storage(run):
    async def main():
        s = APIServer(storage_media_type=PROTOBUF)
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        try:
            await c.create("pods", {"metadata": {"name": "p", "namespace": "default"},
                                    "spec": {"containers": [{"name": "c", "image": "x", "resources": {"limits": {"amd.com/gpu": "1"}}}]}})
            kv = s.store.get("/registry/pods/default/p")
            assert kv.value[:4] == b"k8s\x00"
            stored = pb.decode_object(kv.value)
            assert stored["spec"]["extendedResources"][0]["resources"]["limits"] == {"amd.com/gpu": "1"}
            got = await c.get("pods", "p", "default")
            assert got["metadata"]["name"] == "p"
        finally:
            await c.close()
            await s.stop()
    run(main())


def test_protobuf_content_negotiation(run):
    async def main():
        s = APIServer()
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        try:
            body = pb.encode_object({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "pp", "namespace": "default"},
                                     "spec": {"containers": [{"name": "c", "image": "x"}]}})
            st, resp = await c.http.request("POST", "/api/v1/namespaces/default/pods", body, PROTOBUF,
                                            headers={"Accept": PROTOBUF})
            assert st == 201 and resp[:4] == b"k8s\x00"
            assert pb.decode_object(resp)["metadata"]["name"] == "pp"
        finally:
            await c.close()
            await s.stop()
    run(main())
