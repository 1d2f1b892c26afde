"""Probe helpers and probes against live endpoints.

Reference: `pkg/kubelet/prober/prober_test.go` — TestFormatURL, TestFindPortByName,
TestGetURLParts, TestGetTCPAddrParts, TestHTTPHeaders (a user Host header wins) and the HTTP
success range (2xx/3xx), HTTPS without verification (`probe/http/http.go` InsecureSkipVerify).
"""
import asyncio
import ssl

import pytest

from kubernetes_amd.kubelet.prober import extract_port, find_port_by_name, format_url, run_probe

CTR = {"ports": [{"name": "found", "containerPort": 93}]}


@pytest.mark.parametrize("scheme,host,port,path,want", [
    ("http", "localhost", 93, "", "http://localhost:93"), ("https", "localhost", 93, "/path", "https://localhost:93/path"),
    ("http", "localhost", 93, "?foo", "http://localhost:93?foo"),
    ("https", "localhost", 93, "/path?bar", "https://localhost:93/path?bar")])
def test_format_url(scheme, host, port, path, want):
    assert format_url(scheme, host, port, path) == want


def test_find_port_by_name():
    assert find_port_by_name({"ports": [{"name": "foo", "containerPort": 8080},
                                        {"name": "bar", "containerPort": 9000}]}, "foo") == 8080


@pytest.mark.parametrize("port,ok,want", [(-1, False, None), ("", False, None), ("-1", False, None),
                                          ("not-found", False, None), ("found", True, 93), (76, True, 76),
                                          ("118", True, 118), (70000, False, None)])
def test_extract_port(port, ok, want):
    """TestGetURLParts / TestGetTCPAddrParts share extractPort."""
    if ok:
        assert extract_port(port, CTR) == want
    else:
        with pytest.raises(ValueError):
            extract_port(port, CTR)


class _Server:
    def __init__(self, status=200, tls=None):
        self.status, self.tls, self.requests = status, tls, []

    async def handle(self, r, w):
        head = await r.readuntil(b"\r\n\r\n")
        self.requests.append(head.decode())
        w.write(f"HTTP/1.1 {self.status} X\r\nContent-Length: 0\r\n\r\n".encode())
        await w.drain()
        w.close()

    async def start(self):
        self.srv = await asyncio.start_server(self.handle, "127.0.0.1", 0, ssl=self.tls)
        return self.srv.sockets[0].getsockname()[1]


@pytest.mark.parametrize("status,ok", [(200, True), (302, True), (399, True), (400, False), (500, False)])
def test_http_probe_status_range(run, status, ok):
    async def main():
        s = _Server(status)
        port = await s.start()
        try:
            res, _ = await run_probe(None, {}, {}, "cid", {"httpGet": {"port": port, "path": "?q=1"}}, "127.0.0.1")
        finally:
            s.srv.close()
        return res, s.requests
    res, reqs = run(main())
    assert res is ok
    assert reqs[0].startswith("GET /?q=1 HTTP/1.1")


def test_http_headers_and_host_override(run):
    async def main():
        s = _Server()
        port = await s.start()
        try:
            await run_probe(None, {}, {}, "cid", {"httpGet": {"port": port, "httpHeaders": [
                {"name": "Host", "value": "example.com"}, {"name": "X-Probe", "value": "gpu"}]}}, "127.0.0.1")
        finally:
            s.srv.close()
        return s.requests[0]
    head = run(main())
    assert "Host: example.com\r\n" in head and "X-Probe: gpu\r\n" in head and "User-Agent: kube-probe/" in head


def test_https_probe_skips_verification(run, tmp_path):
    from kubernetes_amd.utils.tlsutil import self_signed_serving_cert
    cert, key = self_signed_serving_cert(str(tmp_path), "probe", ("127.0.0.1",))
    ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
    ctx.load_cert_chain(cert, key)

    async def main():
        s = _Server(200, ctx)
        port = await s.start()
        try:
            return await run_probe(None, {}, {}, "cid", {"httpGet": {"port": port, "scheme": "HTTPS"}}, "127.0.0.1")
        finally:
            s.srv.close()
    ok, msg = run(main())
    assert ok, msg


def test_http_probe_failure_message_and_success(run):
    """`pkg/probe/http/http.go` DoHTTPProbe: 200 <= code < 400 succeeds; otherwise the output is
    "HTTP probe failed with statuscode: <code>"."""
    import asyncio

    from kubernetes_amd.kubelet.prober import run_probe

    async def main():
        codes = iter([500, 302])

        async def serve(r, w):
            await r.readuntil(b"\r\n\r\n")
            w.write(f"HTTP/1.1 {next(codes)} X\r\nContent-Length: 0\r\nConnection: close\r\n\r\n".encode())
            await w.drain()
            w.close()
        srv = await asyncio.start_server(serve, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        try:
            probe = {"httpGet": {"port": port, "path": "/healthz"}, "timeoutSeconds": 5}
            assert await run_probe(None, {}, {}, "cid", probe, "127.0.0.1") == (
                False, "HTTP probe failed with statuscode: 500")
            assert (await run_probe(None, {}, {}, "cid", probe, "127.0.0.1"))[0] is True
        finally:
            srv.close()
    run(main())


def test_worker_non_running_container_fails_readiness_without_threshold(run):
    """`worker.go` doProbe: a container that is not running is not probed; its readiness result
    becomes Failure at once, and with restartPolicy Never the worker stops."""
    import asyncio
    from types import SimpleNamespace

    from kubernetes_amd.kubelet.prober import ProbeManager
    from kubernetes_amd.kubelet.runtime.base import EXITED, RUNNING

    class RT:
        state = RUNNING
        execs = 0

        def container_status(self, cid):
            return SimpleNamespace(state=self.state)

        async def exec_sync(self, cid, cmd, timeout):
            self.execs += 1
            return 0, b""

    async def main():
        rt, changes = RT(), []
        pm = ProbeManager(rt, lambda uid, c, ready: changes.append(ready), lambda *a: None)
        c = {"name": "c", "readinessProbe": {"exec": {"command": ["true"]}, "periodSeconds": 0.02,
                                             "failureThreshold": 3}}
        pod = {"spec": {"restartPolicy": "Never"}}
        pm.start("u", pod, c, "cid")
        for _ in range(100):
            if pm.ready("u", "c"):
                break
            await asyncio.sleep(0.01)
        assert pm.ready("u", "c") is True
        rt.state = EXITED
        n = rt.execs
        for _ in range(100):
            if pm.ready("u", "c") is False:
                break
            await asyncio.sleep(0.01)
        assert pm.ready("u", "c") is False and changes[-1] is False       # no 3-probe threshold
        w = pm.workers[("u", "c", "readiness")]
        await asyncio.sleep(0.1)
        assert w.task.done() and rt.execs == n                            # Never: the worker ended unprobed
        pm.stop()
    run(main())
