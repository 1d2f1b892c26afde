"""Unit tests for pieces the conformance specs exercise end to end: ServiceAccount token
mounting (`plugin/pkg/admission/serviceaccount/admission.go`), `podutil.FindPort` in the
endpoints controller, close-delimited HTTP response bodies, kubectl's Go durations and
`--flag=true|false` booleans, and the process runtime's container stdin."""
import asyncio

import pytest

from kubernetes_amd.apiserver.admission.plugins import SA_MOUNT_PATH
from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client.rest import Client
from kubernetes_amd.controllers.misc import find_port


def test_find_port():
    pod = {"spec": {"containers": [{"ports": [{"name": "web", "containerPort": 8080},
                                              {"name": "dns", "containerPort": 53, "protocol": "UDP"}]}]}}
    assert find_port(pod, {"port": 80, "targetPort": "web"}) == 8080
    assert find_port(pod, {"port": 80, "targetPort": 9000}) == 9000
    assert find_port(pod, {"port": 80, "targetPort": "9001"}) == 9001
    assert find_port(pod, {"port": 80}) == 80
    assert find_port(pod, {"port": 53, "targetPort": "dns"}) is None            # TCP service port, UDP name
    assert find_port(pod, {"port": 53, "targetPort": "dns", "protocol": "UDP"}) == 53
    assert find_port(pod, {"port": 80, "targetPort": "missing"}) is None


def test_service_account_token_mount(run):
    async def main():
        s = APIServer()
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        try:
            await c.create("secrets", {"metadata": {"name": "default-token-x", "annotations": {
                "kubernetes.io/service-account.name": "default"}}, "type": "kubernetes.io/service-account-token",
                "data": {}}, "default")
            await c.create("serviceaccounts", {"metadata": {"name": "default"},
                                               "secrets": [{"name": "default-token-x"}]}, "default")
            await c.create("serviceaccounts", {"metadata": {"name": "quiet"}, "automountServiceAccountToken": False},
                           "default")

            def pod(name, **spec):
                return {"metadata": {"name": name}, "spec": dict({"containers": [{"name": "c", "image": "i"}]}, **spec)}
            p = await c.create("pods", pod("a"), "default")
            assert p["spec"]["serviceAccountName"] == "default"
            assert p["spec"]["volumes"] == [{"name": "default-token-x", "secret": {"secretName": "default-token-x",
                                                                                   "defaultMode": 420}}]
            assert p["spec"]["containers"][0]["volumeMounts"] == [
                {"name": "default-token-x", "readOnly": True, "mountPath": SA_MOUNT_PATH}]
            p = await c.create("pods", pod("b", automountServiceAccountToken=False), "default")
            assert not p["spec"].get("volumes")
            p = await c.create("pods", pod("c", serviceAccountName="quiet"), "default")
            assert not p["spec"].get("volumes")
            # an account without a token yet: admitted, nothing mounted
            await c.create("serviceaccounts", {"metadata": {"name": "fresh"}}, "default")
            p = await c.create("pods", pod("d", serviceAccountName="fresh"), "default")
            assert not p["spec"].get("volumes")
            # the mounted pod can be updated (image) without tripping spec immutability
            got = await c.get("pods", "a", "default")
            got["spec"]["containers"][0]["image"] = "i2"
            await c.update("pods", got, "default")
        finally:
            await c.close()
            await s.stop()
    run(main(), timeout=30)


def test_close_delimited_http_body(run):
    from kubernetes_amd.client.http import HTTPClient

    async def main():
        async def handle(reader, writer):
            await reader.readuntil(b"\r\n\r\n")
            writer.write(b"HTTP/1.0 200 OK\r\nContent-Type: text/plain\r\n\r\nno length here")
            await writer.drain()
            writer.close()
        srv = await asyncio.start_server(handle, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        h = HTTPClient(f"http://127.0.0.1:{port}")
        try:
            for _ in range(2):                  # the closed connection is never reused
                st, body = await h.request("GET", "/")
                assert st == 200 and body == b"no length here"
        finally:
            await h.close()
            srv.close()
    run(main(), timeout=20)


def test_kubectl_durations_and_bool_values():
    from kubernetes_amd.kubectl.cli import _bool_flag_values, build_parser
    from kubernetes_amd.kubectl.extra import duration
    assert duration("1s") == 1 and duration("5m") == 300 and duration("1m30s") == 90
    assert duration("500ms") == 0.5 and duration("2.5") == 2.5 and duration("1h") == 3600
    with pytest.raises(Exception):
        duration("5 minutes")
    ap = build_parser()
    assert _bool_flag_values(ap, ["run", "x", "--rm=true", "--attach=false", "--", "--rm=true"]) == \
        ["run", "x", "--rm", "--", "--rm=true"]
    # `set env --overwrite=false` takes a value there: not rewritten
    assert _bool_flag_values(ap, ["set", "env", "d/x", "--overwrite=false"]) == ["set", "env", "d/x", "--overwrite=false"]


def test_process_runtime_container_stdin(run, tmp_path):
    from kubernetes_amd.kubelet.runtime.base import RunContainerOptions
    from kubernetes_amd.kubelet.runtime.process import ProcessRuntime

    async def main():
        rt = ProcessRuntime(str(tmp_path / "rt"), isolation="off")
        pod = {"metadata": {"name": "p", "namespace": "d", "uid": "u-stdin"}, "spec": {}}
        sid = await rt.run_pod_sandbox(pod, {})
        c = {"name": "c", "image": "busybox", "command": ["sh", "-c", "cat; echo done"], "stdin": True, "stdinOnce": True}
        cid = await rt.create_container(sid, pod, c, RunContainerOptions())
        await rt.start_container(cid)
        await asyncio.sleep(0.3)
        assert rt.container_status(cid).state == "CONTAINER_RUNNING"       # waiting on its stdin

        async def src():
            yield b"hello "
            yield b"world\n"
        out = []

        async def sink(d):
            out.append(d)
        code = await asyncio.wait_for(rt.attach(cid, src(), sink, None, False, None), 10)
        assert code == 0 and b"".join(out) == b"hello world\ndone\n"
        await rt.remove_pod_sandbox(sid)
    run(main(), timeout=30)
