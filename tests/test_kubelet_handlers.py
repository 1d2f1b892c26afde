"""Lifecycle hook runner ported from `pkg/kubelet/lifecycle/handlers_test.go` (TestResolvePort*,
TestRunHandlerExec, TestRunHandlerHttp, TestRunHandlerNil, TestRunHandlerExecFailure,
TestRunHandlerHttpFailure), plus a live HTTP hook whose 500 response is not a failure."""
import asyncio

import pytest

from kubernetes_amd.kubelet.lifecycle import HandlerRunner, HookError, format_pod, http_get, resolve_port


def test_resolve_port_int():
    assert resolve_port(80, {}) == 80


def test_resolve_port_string():
    assert resolve_port("foo", {"ports": [{"name": "foo", "containerPort": 80}]}) == 80
    assert resolve_port("8080", {}) == 8080


def test_resolve_port_string_unknown():
    with pytest.raises(HookError):
        resolve_port("foo", {"ports": [{"name": "bar", "containerPort": 80}]})


class FakeCommandRunner:
    def __init__(self, rc=0, msg=b"", err=None):
        self.cmd = self.cid = None
        self.rc, self.msg, self.err = rc, msg, err

    async def exec_sync(self, cid, cmd, timeout):
        self.cid, self.cmd = cid, cmd
        if self.err:
            raise self.err
        return self.rc, self.msg


class FakeHTTP:
    def __init__(self, body="", err=None):
        self.url = None
        self.body, self.err = body, err

    async def __call__(self, url):
        self.url = url
        return self.body, self.err


POD = {"metadata": {"name": "podFoo", "namespace": "nsFoo"}}


def test_run_handler_exec(run):
    rt = FakeCommandRunner()
    c = {"name": "containerFoo", "lifecycle": {"postStart": {"exec": {"command": ["ls", "-a"]}}}}
    msg, err = run(HandlerRunner(rt, FakeHTTP()).run("test://abc1234", POD, c, c["lifecycle"]["postStart"]))
    assert err is None and rt.cid == "test://abc1234" and rt.cmd == ["ls", "-a"]


def test_run_handler_http(run):
    http = FakeHTTP()
    c = {"name": "containerFoo", "lifecycle": {"postStart": {"httpGet": {"host": "foo", "port": 8080, "path": "bar"}}}}
    msg, err = run(HandlerRunner(FakeCommandRunner(), http).run("id", POD, c, c["lifecycle"]["postStart"]))
    assert err is None and http.url == "http://foo:8080/bar"


def test_run_handler_http_defaults(run):
    http = FakeHTTP()
    c = {"name": "c", "ports": [{"name": "web", "containerPort": 8081}]}
    run(HandlerRunner(FakeCommandRunner(), http).run("id", POD, c, {"httpGet": {"port": "", "path": "x"}}, "10.1.2.3"))
    assert http.url == "http://10.1.2.3:80/x"                       # empty string port: 80, pod IP host
    run(HandlerRunner(FakeCommandRunner(), http).run("id", POD, c, {"httpGet": {"port": "web"}}, "fd00::5"))
    assert http.url == "http://[fd00::5]:8081/"
    msg, err = run(HandlerRunner(FakeCommandRunner(), http).run("id", POD, c, {"httpGet": {"port": 1}}, None))
    assert err is not None                                            # no host and no pod IP


def test_run_handler_nil(run):
    c = {"name": "containerFoo", "lifecycle": {"postStart": {}}}
    msg, err = run(HandlerRunner(FakeCommandRunner(), FakeHTTP()).run("id", POD, c, c["lifecycle"]["postStart"]))
    assert err is not None and msg.startswith("Cannot run handler: Invalid handler")


def test_run_handler_exec_failure(run):
    rt = FakeCommandRunner(err=OSError("invalid command"), msg=b"invalid command")
    c = {"name": "containerFoo"}
    h = {"exec": {"command": ["ls", "--a"]}}
    msg, err = run(HandlerRunner(rt, FakeHTTP()).run("id", POD, c, h))
    assert err is not None
    assert msg == (f'Exec lifecycle hook ([ls --a]) for Container "containerFoo" in Pod "{format_pod(POD)}" failed - '
                   f'error: invalid command, message: ""')
    rt = FakeCommandRunner(rc=2, msg=b"boom")
    msg, err = run(HandlerRunner(rt, FakeHTTP()).run("id", POD, c, h))
    assert err is not None and msg.endswith('message: "boom"')


def test_run_handler_http_failure(run):
    http = FakeHTTP(body="fake http error", err=OSError("fake http error"))
    c = {"name": "containerFoo"}
    h = {"httpGet": {"host": "foo", "port": 8080, "path": "bar"}}
    msg, err = run(HandlerRunner(FakeCommandRunner(), http).run("id", POD, c, h))
    assert err is not None and http.url == "http://foo:8080/bar"
    assert msg == (f'Http lifecycle hook (bar) for Container "containerFoo" in Pod "{format_pod(POD)}" failed - '
                   f'error: fake http error, message: "fake http error"')


def test_http_hook_any_status_is_success(run):
    async def main():
        async def serve(r, w):
            await r.readuntil(b"\r\n\r\n")
            w.write(b"HTTP/1.1 500 Internal Server Error\r\nContent-Length: 4\r\nConnection: close\r\n\r\noops")
            await w.drain()
            w.close()
        srv = await asyncio.start_server(serve, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        try:
            body, err = await http_get(f"http://127.0.0.1:{port}/hook", timeout=5)
            assert (body, err) == ("oops", None)
        finally:
            srv.close()
        body, err = await http_get(f"http://127.0.0.1:{port}/hook", timeout=5)   # closed: transport error
        assert err is not None
    run(main())
