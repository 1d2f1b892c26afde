"""Validation of every served kind (table-driven), through the API server: invalid objects get
422 Invalid with field paths; valid ones are stored; update-only rules (immutable fields) hold.

The first three cases are the objects round 2 accepted (VERDICT "What's missing" 3): a
Deployment with replicas -3, no containers and a selector that does not match its template; a
Job with parallelism -1 and restartPolicy Always; a ConfigMap with key "bad key!". Reference:
`pkg/apis/extensions/validation/validation.go:268-420`, `pkg/apis/batch/validation/validation.go:78-150`,
`pkg/apis/core/validation/validation.go:3781-3830,4376`.
"""
import pytest

from kubernetes_amd.api import validation_ext as vx
from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client.rest import APIStatusError, Client


def tpl(labels=None, restart=None, containers=True):
    spec = {"containers": [{"name": "c", "image": "busybox"}] if containers else []}
    if restart:
        spec["restartPolicy"] = restart
    return {"metadata": {"labels": labels or {"app": "a"}}, "spec": spec}


# (resource, object, expected field paths in the 422 message)
INVALID = [
    ("deployments", {"metadata": {"name": "d"}, "spec": {"replicas": -3, "selector": {"matchLabels": {"app": "x"}},
                                                         "template": tpl(containers=False)}},
     ["spec.replicas", "spec.template.metadata.labels", "spec.template.spec.containers"]),
    ("jobs", {"metadata": {"name": "j"}, "spec": {"parallelism": -1, "template": tpl(restart="Always")}},
     ["spec.parallelism", "spec.template.spec.restartPolicy"]),
    ("configmaps", {"metadata": {"name": "cm"}, "data": {"bad key!": "v"}}, ["data[bad key!]"]),
    ("deployments", {"metadata": {"name": "d2"}, "spec": {"selector": {"matchLabels": {"app": "a"}}, "template": tpl(),
                                                          "strategy": {"type": "RollingUpdate", "rollingUpdate": {
                                                              "maxUnavailable": 0, "maxSurge": 0}}}},
     ["spec.strategy.rollingUpdate.maxUnavailable"]),
    ("deployments", {"metadata": {"name": "d3"}, "spec": {"selector": {"matchLabels": {"app": "a"}}, "template": tpl(),
                                                          "strategy": {"type": "Recreate", "rollingUpdate": {}}}},
     ["spec.strategy.rollingUpdate"]),
    ("replicasets", {"metadata": {"name": "rs"}, "spec": {"selector": {"matchLabels": {"app": "b"}}, "template": tpl()}},
     ["spec.template.metadata.labels"]),
    ("daemonsets", {"metadata": {"name": "ds"}, "spec": {"template": tpl(restart="Never")}},
     ["spec.template.spec.restartPolicy"]),
    ("statefulsets", {"metadata": {"name": "ss"}, "spec": {"podManagementPolicy": "Random", "template": tpl()}},
     ["spec.podManagementPolicy"]),
    ("replicationcontrollers", {"metadata": {"name": "rc"}, "spec": {"replicas": -1, "selector": {"app": "z"},
                                                                      "template": tpl()}},
     ["spec.replicas", "spec.template.metadata.labels"]),
    ("cronjobs", {"metadata": {"name": "cj"}, "spec": {"schedule": "61 * * * *", "concurrencyPolicy": "Sometimes",
                                                       "jobTemplate": {"spec": {"template": tpl(restart="OnFailure")}}}},
     ["spec.schedule", "spec.concurrencyPolicy"]),
    ("secrets", {"metadata": {"name": "s"}, "type": "kubernetes.io/tls", "data": {"tls.crt": "YQ=="}}, ["data[tls.key]"]),
    ("secrets", {"metadata": {"name": "s2"}, "data": {"..hidden": "YQ=="}}, ["data[..hidden]"]),
    ("persistentvolumeclaims", {"metadata": {"name": "pvc"}, "spec": {"accessModes": ["ReadWriteSometimes"]}},
     ["spec.accessModes", "spec.resources[storage]"]),
    ("persistentvolumes", {"metadata": {"name": "pv"}, "spec": {"accessModes": ["ReadWriteOnce"], "capacity": {"storage": "1Gi"},
                                                                "hostPath": {"path": "/a"}, "nfs": {"server": "x", "path": "/"}}},
     ["spec.nfs"]),
    ("horizontalpodautoscalers", {"metadata": {"name": "h"}, "spec": {"scaleTargetRef": {"kind": "Deployment", "name": "d"},
                                                                       "minReplicas": 5, "maxReplicas": 2}},
     ["spec.maxReplicas"]),
    ("poddisruptionbudgets", {"metadata": {"name": "pdb"}, "spec": {"minAvailable": 1, "maxUnavailable": "150%"}},
     ["spec", "spec.maxUnavailable"]),
    ("limitranges", {"metadata": {"name": "lr"}, "spec": {"limits": [{"type": "Container", "min": {"cpu": "2"},
                                                                      "max": {"cpu": "1"}}]}},
     ["spec.limits[0].min[cpu]"]),
    ("resourcequotas", {"metadata": {"name": "rq"}, "spec": {"hard": {"pods": "-1"}, "scopes": ["Nope"]}},
     ["spec.hard[pods]", "spec.scopes[0]"]),
    ("endpoints", {"metadata": {"name": "ep"}, "subsets": [{"addresses": [{"ip": "300.1.1.1"}], "ports": [{"port": 70000}]}]},
     ["subsets[0].addresses[0].ip", "subsets[0].ports[0].port"]),
    ("roles", {"metadata": {"name": "r"}, "rules": [{"apiGroups": [""], "resources": ["pods"], "verbs": []}]},
     ["rules[0].verbs"]),
    ("rolebindings", {"metadata": {"name": "rb"}, "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "Thing",
                                                              "name": "x"}, "subjects": [{"kind": "Robot", "name": "r2"}]},
     ["roleRef.kind", "subjects[0].kind"]),
    ("clusterrolebindings", {"metadata": {"name": "crb"}, "roleRef": {"apiGroup": "rbac.authorization.k8s.io",
                                                                      "kind": "Role", "name": "x"},
                             "subjects": [{"kind": "ServiceAccount", "name": "sa"}]},
     ["roleRef.kind", "subjects[0].namespace"]),
    ("storageclasses", {"metadata": {"name": "sc"}, "reclaimPolicy": "Recycle"}, ["provisioner", "reclaimPolicy"]),
    ("priorityclasses", {"metadata": {"name": "huge"}, "value": 2_000_000_000}, ["value"]),
    ("networkpolicies", {"metadata": {"name": "np"}, "spec": {"podSelector": {}, "ingress": [{"from": [
        {"ipBlock": {"cidr": "10.0.0.0/8", "except": ["11.0.0.0/16"]}}], "ports": [{"protocol": "SCTP", "port": 0}]}]}},
     ["spec.ingress[0].from[0].ipBlock.except[0]", "spec.ingress[0].ports[0].protocol", "spec.ingress[0].ports[0].port"]),
    ("ingresses", {"metadata": {"name": "ing"}, "spec": {"rules": [{"host": "1.2.3.4", "http": {"paths": [
        {"path": "rel", "backend": {"serviceName": "Svc", "servicePort": 80}}]}}]}},
     ["spec.rules[0].host", "spec.rules[0].http.paths[0].path", "spec.rules[0].http.paths[0].backend.serviceName"]),
    ("pods", {"metadata": {"name": "p"}, "spec": {"dnsPolicy": "Sometimes",
                                                  # (a source-less volume is defaulted to emptyDir, SetDefaults_Volume)
                                                  "volumes": [{"name": "v", "emptyDir": {}, "hostPath": {"path": "/x"}}],
                                                  "tolerations": [{"operator": "Equal", "value": "x"}],
                                                  "containers": [{"name": "c", "image": "i", "env": [{"name": "1BAD=X"}],
                                                                  "volumeMounts": [{"name": "w", "mountPath": "/w"}],
                                                                  "livenessProbe": {"periodSeconds": 1}}]}},
     ["spec.dnsPolicy", "spec.volumes[0].emptyDir", "spec.tolerations[0].operator", "spec.containers[0].env[0].name",
      "spec.containers[0].volumeMounts[0].name", "spec.containers[0].livenessProbe"]),
]

VALID = [
    ("deployments", {"metadata": {"name": "ok-d"}, "spec": {"template": tpl()}}),   # selector defaulted from labels
    ("jobs", {"metadata": {"name": "ok-j"}, "spec": {"template": tpl(restart="Never")}}),
    ("configmaps", {"metadata": {"name": "ok-cm"}, "data": {"a.b-c_d": "v"}}),
    ("cronjobs", {"metadata": {"name": "ok-cj"}, "spec": {"schedule": "*/5 * * * mon-fri",
                                                          "jobTemplate": {"spec": {"template": tpl(restart="OnFailure")}}}}),
    ("statefulsets", {"metadata": {"name": "ok-ss"}, "spec": {"serviceName": "s", "template": tpl()}}),
    ("networkpolicies", {"metadata": {"name": "ok-np"}, "spec": {"podSelector": {"matchLabels": {"app": "a"}},
                                                                 "ingress": [{"ports": [{"port": 80}]}]}}),
]


def with_api(run, body):
    """Run body(client) against a fresh in-process API server on one event loop."""
    async def main():
        srv = APIServer()
        port = await srv.start()
        c = Client(f"http://127.0.0.1:{port}")
        try:
            await body(c)
        finally:
            await c.close()
            await srv.stop()
    run(main())


@pytest.mark.parametrize("resource,obj,fields", INVALID, ids=[f"{r}-{o['metadata']['name']}" for r, o, _ in INVALID])
def test_invalid_objects_are_rejected(run, resource, obj, fields):
    async def body(c):
        with pytest.raises(APIStatusError) as e:
            await c.create(resource, obj, "default")
        assert e.value.code == 422, e.value
        msg = str(e.value)
        for f in fields:
            assert f + ":" in msg, (f, msg)
    with_api(run, body)


@pytest.mark.parametrize("resource,obj", VALID, ids=[f"{r}-{o['metadata']['name']}" for r, o in VALID])
def test_valid_objects_are_stored(run, resource, obj):
    async def body(c):
        got = await c.create(resource, obj, "default")
        assert got["metadata"]["name"] == obj["metadata"]["name"]
    with_api(run, body)


def test_defaults_applied_before_validation(run):
    async def body(c):
        d = await c.create("deployments", {"metadata": {"name": "dd"}, "spec": {"template": tpl()}}, "default")
        s = d["spec"]
        assert s["replicas"] == 1 and s["selector"] == {"matchLabels": {"app": "a"}}
        assert s["strategy"] == {"type": "RollingUpdate", "rollingUpdate": {"maxUnavailable": "25%", "maxSurge": "25%"}}
        assert s["template"]["spec"]["restartPolicy"] == "Always" and s["template"]["spec"]["dnsPolicy"] == "ClusterFirst"
        j = await c.create("jobs", {"metadata": {"name": "jj"}, "spec": {"template": tpl(restart="Never")}}, "default")
        assert (j["spec"]["completions"], j["spec"]["parallelism"], j["spec"]["backoffLimit"]) == (1, 1, 6)
    with_api(run, body)


def test_update_rules_immutable_fields(run):
    async def body(c):
        d = await c.create("deployments", {"metadata": {"name": "imm"}, "spec": {"template": tpl()}}, "default")
        d["spec"]["selector"] = {"matchLabels": {"app": "a", "tier": "x"}}
        d["spec"]["template"]["metadata"]["labels"]["tier"] = "x"
        with pytest.raises(APIStatusError) as e:
            await c.update("deployments", d)
        assert e.value.code == 422 and "spec.selector: Invalid value: field is immutable" in str(e.value)
        j = await c.create("jobs", {"metadata": {"name": "jimm"}, "spec": {"template": tpl(restart="Never")}}, "default")
        j["spec"]["completions"] = 5
        with pytest.raises(APIStatusError) as e:
            await c.update("jobs", j)
        assert "spec.completions" in str(e.value)
        rb = await c.create("rolebindings", {"metadata": {"name": "rbimm"}, "roleRef": {
            "apiGroup": "rbac.authorization.k8s.io", "kind": "Role", "name": "a"}, "subjects": [{"kind": "User", "name": "u"}]},
            "default")
        rb["roleRef"]["name"] = "b"
        with pytest.raises(APIStatusError) as e:
            await c.update("rolebindings", rb)
        assert "roleRef" in str(e.value)
        s = await c.create("secrets", {"metadata": {"name": "simm"}, "data": {"a": "YQ=="}}, "default")
        s["type"] = "kubernetes.io/basic-auth"
        s["data"]["username"] = "dQ=="
        with pytest.raises(APIStatusError) as e:
            await c.update("secrets", s)
        assert "type: Invalid value: field is immutable" in str(e.value)
        ss = await c.create("statefulsets", {"metadata": {"name": "ssimm"}, "spec": {"serviceName": "a", "template": tpl()}},
                            "default")
        ss["spec"]["serviceName"] = "b"
        with pytest.raises(APIStatusError) as e:
            await c.update("statefulsets", ss)
        assert "updates to statefulset spec" in str(e.value)
    with_api(run, body)


@pytest.mark.parametrize("expr,ok", [("*/5 * * * *", True), ("0 0 1 jan *", True), ("@hourly", True), ("@every 1h30m", True),
                                     ("61 * * * *", False), ("* * *", False), ("0 25 * * *", False), ("a b c d e", False)])
def test_cron_expressions(expr, ok):
    assert vx.valid_cron(expr) is ok


# -- SetDefaults_* (pkg/apis/*/v1*/defaults.go) --------------------------------------------------

def test_scheme_defaults():
    from kubernetes_amd.api import defaults as D
    svc = D.apply("Service", {"spec": {"ports": [{"port": 80}], "type": "NodePort", "sessionAffinity": "ClientIP"}})
    sp = svc["spec"]
    assert sp["ports"][0] == {"port": 80, "protocol": "TCP", "targetPort": 80}
    assert sp["sessionAffinityConfig"] == {"clientIP": {"timeoutSeconds": 10800}} and sp["externalTrafficPolicy"] == "Cluster"
    assert D.apply("Service", {"spec": {}})["spec"] == {"sessionAffinity": "None", "type": "ClusterIP"}
    assert D.apply("Endpoints", {"subsets": [{"ports": [{"port": 1}]}]})["subsets"][0]["ports"][0]["protocol"] == "TCP"
    assert D.apply("Namespace", {"metadata": {"name": "n"}})["status"] == {"phase": "Active"}
    n = D.apply("Node", {"metadata": {"name": "n1"}, "status": {"capacity": {"cpu": "4"}}})
    assert n["spec"]["externalID"] == "n1" and n["status"]["allocatable"] == {"cpu": "4"}
    lr = D.apply("LimitRange", {"spec": {"limits": [
        {"type": "Container", "max": {"cpu": "2"}, "min": {"memory": "1Mi"}, "default": {"memory": "1Gi"}},
        {"type": "Pod", "max": {"cpu": "4"}}]}})
    c, p = lr["spec"]["limits"]
    assert c["default"] == {"memory": "1Gi", "cpu": "2"} and c["defaultRequest"] == {"memory": "1Gi", "cpu": "2"}
    assert "default" not in p
    assert D.apply("StorageClass", {})["reclaimPolicy"] == "Delete"
    wh = D.apply("ValidatingWebhookConfiguration", {"webhooks": [{"name": "w"}]})["webhooks"][0]
    assert wh["failurePolicy"] == "Ignore" and wh["namespaceSelector"] == {}
    rb = D.apply("RoleBinding", {"roleRef": {"kind": "Role", "name": "r"}, "subjects": [
        {"kind": "User", "name": "u"}, {"kind": "ServiceAccount", "name": "s"}]})
    assert rb["roleRef"]["apiGroup"] == "rbac.authorization.k8s.io"
    assert rb["subjects"][0]["apiGroup"] == "rbac.authorization.k8s.io" and "apiGroup" not in rb["subjects"][1]
    assert D.apply("CertificateSigningRequest", {"spec": {}})["spec"]["usages"] == ["digital signature",
                                                                                    "key encipherment"]
    assert D.apply("PodSecurityPolicy", {"spec": {}})["spec"]["allowPrivilegeEscalation"] is True
    pod = D.apply("Pod", {"spec": {"containers": [{"name": "c", "env": [
        {"name": "N", "valueFrom": {"fieldRef": {"fieldPath": "metadata.name"}}}]}],
        "volumes": [{"name": "a"}, {"name": "b", "rbd": {"monitors": ["m"], "image": "i"}},
                    {"name": "c", "iscsi": {"targetPortal": "t", "iqn": "q", "lun": 0}}]}})
    assert pod["spec"]["containers"][0]["env"][0]["valueFrom"]["fieldRef"]["apiVersion"] == "v1"
    a, b, c = pod["spec"]["volumes"]
    assert a == {"name": "a", "emptyDir": {}}
    assert (b["rbd"]["pool"], b["rbd"]["user"], b["rbd"]["keyring"]) == ("rbd", "admin", "/etc/ceph/keyring")
    assert c["iscsi"]["iscsiInterface"] == "default"
