"""Container lifecycle hooks (`pkg/kubelet/lifecycle/handlers.go` HandlerRunner).

  * exec handlers run in the container through the runtime's ExecSync; a non-zero exit is the
    error. The reference passes no timeout (a hook can hold the pod worker forever); here a hook
    gets `EXEC_HOOK_TIMEOUT` seconds.
  * httpGet handlers GET `http://<host or pod IP>:<port>/<path>`; only a transport failure is an
    error (the status code is not checked, unlike a probe). An empty string port means 80;
    `resolve_port` takes an int, a numeric string or a named container port.
  * the returned message carries the reference wording, e.g. `Exec lifecycle hook ([cmd]) for
    Container "c" in Pod "name_ns(uid)" failed - error: ..., message: "..."`.
"""
from __future__ import annotations

import asyncio

EXEC_HOOK_TIMEOUT = 120.0


class HookError(Exception):
    pass


def format_pod(pod) -> str:
    """`format.Pod`: name_namespace(uid)."""
    md = pod.get("metadata") or {}
    return f"{md.get('name', '')}_{md.get('namespace', '')}({md.get('uid', '')})"


def _go_list(cmd) -> str:
    return "[" + " ".join(str(x) for x in cmd) + "]"


def resolve_port(port, container) -> int:
    """`resolvePort`: an int is literal; a string is parsed as a number, else looked up among the
    container's named ports."""
    if isinstance(port, int) and not isinstance(port, bool):
        return port
    name = str(port)
    try:
        return int(name)
    except ValueError:
        pass
    for p in container.get("ports") or ():
        if p.get("name") == name:
            return int(p["containerPort"])
    raise HookError(f"couldn't find port: {name} in {container.get('name', '')}")


async def http_get(url, timeout=EXEC_HOOK_TIMEOUT):
    """`HttpGetter.Get` + getHttpRespBody: returns (body, error); any status code is a response,
    only a transport failure is an error."""
    try:
        return await _get(url, timeout), None
    except (OSError, asyncio.TimeoutError, ValueError) as e:
        return "", e


async def _get(url, timeout):
    from urllib.parse import urlsplit
    u = urlsplit(url)
    host, port = u.hostname, u.port or 80
    target = u.path or "/"
    if u.query:
        target += "?" + u.query
    r, w = await asyncio.wait_for(asyncio.open_connection(host, port), timeout)
    try:
        hh = f"[{host}]" if ":" in host else host
        w.write(f"GET {target} HTTP/1.1\r\nHost: {hh}:{port}\r\nUser-Agent: Go-http-client/1.1\r\n"
                f"Connection: close\r\n\r\n".encode())
        data = await asyncio.wait_for(r.read(), timeout)
    finally:
        w.close()
    _, _, body = data.partition(b"\r\n\r\n")
    return body.decode(errors="replace")


class HandlerRunner:
    def __init__(self, runtime, http_getter=http_get, exec_timeout=EXEC_HOOK_TIMEOUT):
        self.runtime = runtime
        self.http_get = http_getter
        self.exec_timeout = exec_timeout

    async def run(self, cid, pod, container, handler, pod_ip=None):
        """Returns (message, error): error None on success."""
        handler = handler or {}
        if handler.get("exec") is not None:
            cmd = list(handler["exec"].get("command") or ())
            err, out = None, b""
            try:
                rc, out = await self.runtime.exec_sync(cid, cmd, self.exec_timeout)
                if rc != 0:
                    err = HookError(f"command '{' '.join(cmd)}' exited with {rc}: ")
            except (OSError, asyncio.TimeoutError, NotImplementedError) as e:
                err = e
            if err is None:
                return "", None
            text = out.decode(errors="replace") if isinstance(out, bytes) else str(out)
            return (f"Exec lifecycle hook ({_go_list(cmd)}) for Container \"{container.get('name', '')}\" in Pod "
                    f"\"{format_pod(pod)}\" failed - error: {err}, message: \"{text}\""), err
        if handler.get("httpGet") is not None:
            h = handler["httpGet"]
            msg, err = await self._run_http(pod, container, h, pod_ip)
            if err is None:
                return msg, None
            return (f"Http lifecycle hook ({h.get('path', '')}) for Container \"{container.get('name', '')}\" in Pod "
                    f"\"{format_pod(pod)}\" failed - error: {err}, message: \"{msg}\""), err
        err = HookError(f"Invalid handler: {handler}")
        return f"Cannot run handler: {err}", err

    async def _run_http(self, pod, container, h, pod_ip):
        host = h.get("host") or ""
        if not host:
            if not pod_ip:
                return "", HookError("failed to find networking container")
            host = pod_ip
        port = h.get("port")
        try:
            port = 80 if isinstance(port, str) and port == "" else resolve_port(port, container)
        except HookError as e:
            return "", e
        hh = f"[{host}]" if ":" in host else host
        return await self.http_get(f"http://{hh}:{port}/{h.get('path', '')}")
