"""NamespaceExists / NamespaceAutoProvision (`plugin/pkg/admission/namespace/{exists,
autoprovision}/admission_test.go`), the webhook admission plugins gating the webhook calls, and
DenyExecOnPrivileged (`plugin/pkg/admission/exec/admission_test.go`)."""
import pytest

from kubernetes_amd.apiserver import admission as adm
from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client.rest import APIStatusError, Client


def cm(ns):
    return {"metadata": {"name": "c", "namespace": ns}, "data": {"a": "b"}}


async def _srv(plugins):
    s = APIServer(admission_plugins=plugins)
    port = await s.start()
    return s, Client(f"http://127.0.0.1:{port}")


def test_namespace_exists_refuses_missing_namespaces(run):
    async def main():
        s, c = await _srv(["NamespaceExists"])
        try:
            with pytest.raises(APIStatusError) as e:
                await c.create("configmaps", cm("nowhere"), "nowhere")
            assert e.value.code == 404
            await c.create("namespaces", {"metadata": {"name": "somewhere"}})
            await c.create("configmaps", cm("somewhere"), "somewhere")
        finally:
            await c.close()
            await s.stop()
    run(main())


def test_namespace_autoprovision_creates_the_namespace(run):
    async def main():
        s, c = await _srv(["NamespaceAutoProvision", "NamespaceLifecycle"])
        try:
            await c.create("configmaps", cm("fresh"), "fresh")
            ns = await c.get("namespaces", "fresh")
            assert ns["metadata"]["name"] == "fresh"
            await c.create("configmaps", dict(cm("fresh"), metadata={"name": "d", "namespace": "fresh"}), "fresh")
        finally:
            await c.close()
            await s.stop()
    run(main())


def test_webhooks_only_with_their_admission_plugins():
    on = APIServer(admission_plugins=list(adm.DEFAULT_PLUGINS))
    off = APIServer(admission_plugins=["NamespaceLifecycle"])
    assert on.mutating_webhooks_enabled and on.validating_webhooks_enabled
    assert not off.mutating_webhooks_enabled and not off.validating_webhooks_enabled


def test_deny_exec_on_privileged_ignores_host_namespaces():
    chain = adm.new_chain(["DenyExecOnPrivileged"])

    def attempt(spec):
        pod = {"metadata": {"name": "p", "namespace": "default"}, "spec": spec}
        a = adm.Attributes(adm.CONNECT, "pods", "exec", "default", "p", None, pod, None, "Pod")
        chain.validate(a)
    attempt({"hostPID": True, "containers": [{"name": "c"}]})          # allowed by this (older) plugin
    with pytest.raises(adm.AdmissionError):
        attempt({"containers": [{"name": "c", "securityContext": {"privileged": True}}]})
