"""RBAC bootstrap policy parity and per-controller service-account credentials.

Parity:
  * `plugin/pkg/auth/authorizer/rbac/bootstrappolicy/{policy,controller_policy,namespace_policy}.go`
    and their tests (`policy_test.go` TestBootstrapClusterRoles / TestClusterRoleLabel,
    `controller_policy_test.go` TestNoStarRolesForControllers);
  * `cmd/kube-controller-manager/app/controllermanager.go:133-139` — with
    `--use-service-account-credentials` each controller runs as `kube-system/<controller SA>`;
  * `test/integration/auth/rbac_test.go` shape: the controllers still do their work under RBAC,
    and a controller cannot exceed its role (the deployment controller may not read Secrets).
"""
import asyncio
import base64
import time

import pytest

from kubernetes_amd.apiserver import bootstrappolicy as bp
from kubernetes_amd.apiserver.auth import User
from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client.rest import APIStatusError, Client
from kubernetes_amd.controllers.manager import SERVICE_ACCOUNTS, ControllerManager
from kubernetes_amd.native import crypto


async def eventually(fn, timeout=15.0):
    end = time.monotonic() + timeout
    while True:
        r = await fn()
        if r:
            return r
        if time.monotonic() > end:
            raise AssertionError("condition not met")
        await asyncio.sleep(0.05)


def test_bootstrap_policy_shape():
    roles = bp.cluster_roles()
    controller_roles = [n for n in roles if n.startswith("system:controller:")]
    assert len(controller_roles) >= 26
    # TestNoStarRolesForControllers: only the aggregation controller may hold '*' verbs
    for n in controller_roles:
        if n == "system:controller:clusterrole-aggregation-controller":
            continue
        for r in roles[n]["rules"]:
            assert "*" not in r.get("verbs", ()), (n, r)
    # every controller SA the manager uses has a role + binding
    bindings = bp.cluster_role_bindings()
    for sa in set(SERVICE_ACCOUNTS.values()):
        if sa in ("bootstrap-signer", "token-cleaner"):        # namespaced roles in kube-system
            assert ("kube-system", "system:controller:" + sa) in bp.namespace_role_bindings()
            continue
        b = bindings["system:controller:" + sa]
        assert b["subjects"] == [{"kind": "ServiceAccount", "name": sa, "namespace": "kube-system"}]
    # the manager's own role is no longer */*/*
    cm = roles["system:kube-controller-manager"]["rules"]
    assert not any(r.get("verbs") == ["*"] for r in cm)
    assert {"list", "watch"} == set(next(r for r in cm if r.get("apiGroups") == ["*"])["verbs"])
    # aggregation: admin/edit/view select their aggregate-to-* parts and start filled in
    for agg in ("admin", "edit", "view"):
        sel = roles[agg]["aggregationRule"]["clusterRoleSelectors"][0]["matchLabels"]
        part = roles[f"system:aggregate-to-{agg}"]
        assert part["metadata"]["labels"].items() >= sel.items()
        assert roles[agg]["rules"] == part["rules"]
    # TestClusterRoleLabel
    for r in roles.values():
        assert r["metadata"]["labels"]["kubernetes.io/bootstrapping"] == "rbac-defaults"
    for name in ("system:heapster", "system:kube-dns", "system:auth-delegator", "system:kube-aggregator",
                 "system:persistent-volume-provisioner", "system:node-problem-detector"):
        assert name in roles
    assert bindings["system:node"]["subjects"] == []


def test_controllers_run_as_their_service_accounts(run, tmp_path):
    sa_key = crypto.generate_key("rsa", 2048)
    (tmp_path / "sa.key").write_text(sa_key)

    async def main():
        s = APIServer(authorization_modes=("RBAC",), service_account_key_files=[str(tmp_path / "sa.key")],
                      tokens={"admin": User("admin", "0", ["system:masters"]),
                              "kcm": User("system:kube-controller-manager", "1", [])})
        port = await s.start()
        url = f"http://127.0.0.1:{port}"
        admin = Client(url, token="admin")
        root = Client(url, token="kcm")
        made = []

        def factory(token):
            c = Client(url, token=token)
            made.append(c)
            return c
        cm = ControllerManager(root, ["serviceaccount-token", "serviceaccount", "deployment", "replicaset",
                                      "endpoint", "clusterroleaggregation", "namespace", "garbagecollector"],
                               {"serviceaccount-token": {"private_key": sa_key}}, sa_client_factory=factory)
        await cm.start()
        try:
            assert cm.identities["deployment"] == "system:serviceaccount:kube-system:deployment-controller"
            assert cm.identities["serviceaccount-token"] == "manager"
            # the manager's identity alone may not create pods any more
            with pytest.raises(APIStatusError) as e:
                await root.create("pods", {"metadata": {"name": "x", "namespace": "default"},
                                           "spec": {"containers": [{"name": "c", "image": "i"}]}}, "default")
            assert e.value.code == 403
            # the controllers still work under RBAC: Deployment -> ReplicaSet -> pods
            await admin.create("deployments", {
                "apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "web", "namespace": "default"},
                "spec": {"replicas": 2, "selector": {"matchLabels": {"app": "web"}},
                         "template": {"metadata": {"labels": {"app": "web"}},
                                      "spec": {"containers": [{"name": "c", "image": "nginx"}]}}}}, "default")

            async def pods():
                ps = (await admin.list("pods", "default", label_selector="app=web"))["items"]
                return ps if len(ps) == 2 else None
            await eventually(pods)
            # endpoints controller (its own SA) publishes a service's endpoints object
            await admin.create("services", {"metadata": {"name": "web", "namespace": "default"},
                                            "spec": {"selector": {"app": "web"}, "ports": [{"port": 80}]}}, "default")

            async def eps():
                try:
                    return await admin.get("endpoints", "web", "default")
                except APIStatusError:
                    return None
            await eventually(eps)
            # the aggregation controller, as its SA, folds a new aggregate-to-view role into view
            await admin.create("clusterroles", {
                "metadata": {"name": "gpu-viewer", "labels": {"rbac.authorization.k8s.io/aggregate-to-view": "true"}},
                "rules": [{"apiGroups": ["kamd.io"], "resources": ["gpuhealth"], "verbs": ["get"]}]})

            async def view_has():
                v = await admin.get("clusterroles", "view")
                return any(r.get("apiGroups") == ["kamd.io"] for r in v.get("rules") or ())
            await eventually(view_has)
            # a controller cannot exceed its role: the deployment controller may not read Secrets
            dep_client = await cm.sa_clients.client_for("deployment-controller")
            with pytest.raises(APIStatusError) as e:
                await dep_client.list("secrets", "default")
            assert e.value.code == 403
            await dep_client.list("replicasets", "default")       # ... but may read its ReplicaSets
            # namespace deletion runs as namespace-controller
            await admin.create("namespaces", {"metadata": {"name": "scratch"}})
            await admin.create("configmaps", {"metadata": {"name": "cfg", "namespace": "scratch"}}, "scratch")
            await admin.delete("namespaces", "scratch")

            async def gone():
                try:
                    await admin.get("namespaces", "scratch")
                    return False
                except APIStatusError as e:
                    return e.code == 404
            await eventually(gone)
            tok_sa = await admin.get("serviceaccounts", "deployment-controller", "kube-system")
            sec = await admin.get("secrets", tok_sa["secrets"][0]["name"], "kube-system")
            tr = await admin.create("tokenreviews", {"spec": {"token": base64.b64decode(sec["data"]["token"]).decode()}})
            assert tr["status"]["user"]["username"] == "system:serviceaccount:kube-system:deployment-controller"
        finally:
            await cm.stop()
            await admin.close()
            await root.close()
            await s.stop()
    run(main(), timeout=90)


def test_controller_manager_flag_requires_signing_key():
    from kubernetes_amd.cmd.controller_manager import main
    with pytest.raises(SystemExit) as e:
        import asyncio as _a  # noqa: F401
        main(["--master", "http://127.0.0.1:1", "--use-service-account-credentials", "true", "--port", "0"])
    assert "service-account-private-key-file" in str(e.value)
