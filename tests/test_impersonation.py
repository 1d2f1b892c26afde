"""Impersonation (`Impersonate-User` / `-Group` / `-Extra-*`) and kubectl's --as / --as-group.

Parity: `staging/src/k8s.io/apiserver/pkg/endpoints/filters/impersonation_test.go` — the
requester needs `impersonate` on users / groups / serviceaccounts / userextras; the request
then runs with the impersonated identity (service accounts gain their groups).
"""
import io

import pytest

from kubernetes_amd.apiserver.audit import AuditLogger
from kubernetes_amd.apiserver.auth import User
from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client.http import HTTPClient
from kubernetes_amd.kubectl.cli import main as kubectl


def _rbac(name, rules):
    return {"metadata": {"name": name}, "rules": rules}


def test_impersonation_filter_and_kubectl_as(run, tmp_path):
    async def main():
        tokens = {"admin-t": User("admin", "1", ["system:masters", "system:authenticated"]),
                  "dev-t": User("dev", "2", ["system:authenticated"]),
                  "imp-t": User("imp", "3", ["system:authenticated"])}
        audit_path = tmp_path / "audit.log"
        api = APIServer(authorization_modes=("RBAC",), tokens=tokens, audit=AuditLogger(str(audit_path)))
        port = await api.start()
        url = f"http://127.0.0.1:{port}"
        admin = HTTPClient(url, token="admin-t")
        try:
            import json
            # imp may impersonate user "dev" and group "gpu-team"; dev may list pods
            for kind, obj in (("clusterroles", _rbac("impersonator", [
                    {"apiGroups": [""], "resources": ["users"], "verbs": ["impersonate"], "resourceNames": ["dev"]},
                    {"apiGroups": [""], "resources": ["groups"], "verbs": ["impersonate"], "resourceNames": ["gpu-team"]},
                    {"apiGroups": [""], "resources": ["serviceaccounts"], "verbs": ["impersonate"]}])),
                              ("clusterroles", _rbac("pod-reader", [{"apiGroups": [""], "resources": ["pods"],
                                                                     "verbs": ["list", "get"]}]))):
                st, body = await admin.request("POST", "/apis/rbac.authorization.k8s.io/v1/clusterroles",
                                               json.dumps(obj).encode())
                assert st == 201, body
            for name, role, subj in (("imp-b", "impersonator", {"kind": "User", "name": "imp"}),
                                     ("dev-b", "pod-reader", {"kind": "User", "name": "dev"}),
                                     ("sa-b", "pod-reader", {"kind": "Group", "name": "system:serviceaccounts:default"})):
                b = {"metadata": {"name": name}, "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole",
                                                             "name": role}, "subjects": [subj]}
                st, body = await admin.request("POST", "/apis/rbac.authorization.k8s.io/v1/clusterrolebindings",
                                               json.dumps(b).encode())
                assert st == 201, body
            imp = HTTPClient(url, token="imp-t")
            st, _ = await imp.request("GET", "/api/v1/namespaces/default/pods")
            assert st == 403                                     # imp itself cannot list pods
            st, _ = await imp.request("GET", "/api/v1/namespaces/default/pods", headers={"Impersonate-User": "dev"})
            assert st == 200                                     # ... but as dev it can
            st, _ = await imp.request("GET", "/api/v1/namespaces/default/pods", headers={"Impersonate-User": "root"})
            assert st == 403                                     # not allowed to impersonate root
            st, _ = await imp.request("GET", "/api/v1/namespaces/default/pods",
                                      headers={"Impersonate-User": "dev", "Impersonate-Group": "system:masters"})
            assert st == 403                                     # nor to add system:masters
            st, _ = await imp.request("GET", "/api/v1/namespaces/default/pods", headers={"Impersonate-Group": "gpu-team"})
            assert st == 400                                     # groups without a user
            st, _ = await imp.request("GET", "/api/v1/namespaces/default/pods",
                                      headers={"Impersonate-User": "system:serviceaccount:default:builder"})
            assert st == 200                                     # SA identity carries system:serviceaccounts:default
            st, _ = await HTTPClient(url, token="dev-t").request(
                "GET", "/api/v1/namespaces/default/pods", headers={"Impersonate-User": "imp"})
            assert st == 403                                     # dev may not impersonate anyone
            await imp.close()
            import json as _j
            api.audit.flush() if hasattr(api.audit, "flush") else None
            evs = [_j.loads(line) for line in audit_path.read_text().splitlines() if line.strip()]
            ev = next(e for e in evs if (e.get("impersonatedUser") or {}).get("username") == "dev")
            assert ev["user"]["username"] == "imp"

            def k(*args):
                out = io.StringIO()
                return kubectl(["-s", url, "--token", "imp-t", *args], out=out), out.getvalue()
            import asyncio
            rc, _ = await asyncio.to_thread(k, "get", "pods", "--as", "dev")
            assert rc == 0
            rc, _ = await asyncio.to_thread(k, "get", "pods")
            assert rc == 1
            rc, _ = await asyncio.to_thread(k, "--as", "dev", "--as-group", "gpu-team", "get", "pods")
            assert rc == 0
        finally:
            await admin.close()
            await api.stop()
    run(main())


def test_specified_groups_are_the_complete_group_list():
    """`impersonation.go:66-124`: with Impersonate-Group headers the specified groups are the
    whole list — system:authenticated and the service-account groups are added only when no
    group is specified."""
    from kubernetes_amd.apiserver.impersonation import impersonate
    calls = []

    def allow(*a):
        calls.append(a[1:])
    me = User("imp", "3", ["system:authenticated"])
    u = impersonate({"impersonate-user": "dev", "impersonate-group": "gpu-team"}, me, allow)
    assert u.name == "dev" and list(u.groups) == ["gpu-team"]
    u = impersonate({"impersonate-user": "dev"}, me, allow)
    assert list(u.groups) == ["system:authenticated"]
    u = impersonate({"impersonate-user": "system:serviceaccount:ns1:sa"}, me, allow)
    assert list(u.groups) == ["system:serviceaccounts", "system:serviceaccounts:ns1", "system:authenticated"]
    u = impersonate({"impersonate-user": "system:serviceaccount:ns1:sa", "impersonate-group": "g1, g2"}, me, allow)
    assert list(u.groups) == ["g1", "g2"]
    u = impersonate({"impersonate-user": "system:anonymous"}, me, allow)
    assert list(u.groups) == []
    assert ("impersonate", None, "groups", "", "g2", "") in calls
