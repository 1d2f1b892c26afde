"""Kubelet server streaming endpoints: /exec, /attach, /run, /portForward.

Parity: `pkg/kubelet/server/server.go:303-360` (routes `/run/{ns}/{pod}/{container}`,
`/exec/{ns}/{pod}/{container}`, `/attach/...`, `/portForward/{ns}/{pod}`, with optional `{uid}`)
and `getExec`/`getPortForward` (`:600-700`): with a CRI runtime the kubelet obtains a streaming
URL from the runtime (`Exec`/`PortForward` RPCs) and proxies it; for the in-process runtimes it
serves the stream itself.

Three wire protocols:
  * SPDY/3.1 (`Upgrade: SPDY/3.1`, sub-protocol in `X-Stream-Protocol-Version`): what kubectl and
    client-go of 1.9 use — remotecommand v1-v4 (`streamType` error/stdin/stdout/stderr/resize
    streams) and `portforward.k8s.io` (data/error stream pairs per `requestID`);
  * WebSocket (`Upgrade: websocket`): the Kubernetes channel protocols `channel.k8s.io`,
    `base64.channel.k8s.io`, `v4.channel.k8s.io`, `v4.base64.channel.k8s.io` (+ `v5`) for
    exec/attach with stdin, tty and resize, and the per-port channel pairs of port-forward
    (`cri/remotecommand.py`); with a CRI runtime the upgrade is relayed to the runtime's
    streaming server;
  * the framed fallback of `cri/server.py` (chunked frames for exec, `Upgrade: tcp` tunnel for
    port-forward) for clients that do not speak WebSocket.
"""
from __future__ import annotations

import asyncio
from urllib.parse import parse_qs

from ..cri import remotecommand as rc_
from ..cri.server import splice
from ..utils.httpserver import Response, StreamResponse, UpgradeResponse
from ..utils.websocket import is_websocket_request


def _frames(rc, out):
    body = b""
    if out:
        p = b"\x01" + (out if isinstance(out, bytes) else str(out).encode())
        body += b"%x\r\n%s\r\n" % (len(p), p)
    p = b"\x03" + str(rc).encode()
    return body + b"%x\r\n%s\r\n" % (len(p), p)


def _find(kubelet, parts, with_container=True):
    """parts after the verb: ns, pod, [uid,] container"""
    if len(parts) < (3 if with_container else 2):
        return None, None, "bad path"
    ns, name = parts[0], parts[1]
    uid = kubelet.by_key.get(f"{ns}/{name}")
    st = kubelet.pods.get(uid) if uid else None
    if st is None:
        return None, None, f"pod {ns}/{name} not found"
    if not with_container:
        return st, None, None
    cname = parts[-1]
    cid = st.containers.get(cname) or st.init_containers.get(cname)
    if cid is None:
        return st, None, f"container {cname} not found in pod {ns}/{name}"
    return st, cid, None


async def handle(kubelet, req):
    """Returns a Response / StreamResponse / UpgradeResponse, or None if the path is not ours."""
    p = req.path
    verb = p.split("/", 2)[1] if p.count("/") >= 2 else ""
    if verb not in ("exec", "run", "attach", "portForward"):
        return None
    parts = [x for x in p.split("/")[2:] if x]
    rt = kubelet.runtime
    if verb != "run" and (is_websocket_request(req.headers) or rc_.is_spdy_request(req.headers)):
        return await _upgraded(kubelet, rt, req, verb, parts, spdy=rc_.is_spdy_request(req.headers))
    if verb in ("exec", "run", "attach"):
        st, cid, err = _find(kubelet, parts)
        if err:
            return Response(404, err.encode(), "text/plain")
        q = parse_qs(req.qs or "")
        cmd = q.get("command") or q.get("cmd") or []
        if verb == "run":   # /run returns the combined output as the body (runInContainer)
            rc, out = await rt.exec_sync(cid, cmd, 60)
            return Response(200 if rc == 0 else 500, out, "text/plain")
        if verb == "attach":
            data = await rt.container_logs(cid)
            return StreamResponse(_static(_frames(0, data)), "application/vnd.kamd.stream")
        if hasattr(rt, "exec_url"):
            url = await rt.exec_url(cid, cmd)
            return StreamResponse(_proxy_exec(url), "application/vnd.kamd.stream")
        rc, out = await rt.exec_sync(cid, cmd, float(q.get("timeout", ["300"])[0]))
        return StreamResponse(_static(_frames(rc, out)), "application/vnd.kamd.stream")
    # portForward
    st, _, err = _find(kubelet, parts, with_container=False)
    if err:
        return Response(404, err.encode(), "text/plain")
    port = int(req.query.get("port") or 0)
    if not port:
        return Response(400, b"port is required", "text/plain")
    if "upgrade" not in req.headers.get("connection", "").lower():
        return Response(400, b"port-forward needs Connection: Upgrade", "text/plain")
    if hasattr(rt, "port_forward_url"):
        url = await rt.port_forward_url(st.sandbox, [port])
        from ..cri.streaming import open_port_forward

        async def run(reader, writer):
            ur, uw = await open_port_forward(url, port)
            await splice(reader, writer, ur, uw)
        return UpgradeResponse(run)

    async def run_local(reader, writer):
        # in-process runtimes: pods share the host network namespace
        try:
            ur, uw = await asyncio.open_connection("127.0.0.1", port)
        except OSError:
            writer.close()
            return
        await splice(reader, writer, ur, uw)
    return UpgradeResponse(run_local)


async def _upgraded(kubelet, rt, req, verb, parts, spdy=False):
    """WebSocket or SPDY/3.1 sessions (the transport is chosen by the client's Upgrade header)."""
    if verb == "portForward":
        st, _, err = _find(kubelet, parts, with_container=False)
        if err:
            return Response(404, err.encode(), "text/plain")
        if hasattr(rt, "port_forward_url"):
            try:
                ports = [] if spdy else rc_.ports_from_query(req.qs)     # SPDY names ports per stream
            except ValueError as e:
                return Response(400, str(e).encode(), "text/plain")
            return rc_.upgrade_proxy_response(req, await rt.port_forward_url(st.sandbox, ports))
        # in-process runtimes: pods share the host network namespace
        dial = lambda port: asyncio.open_connection("127.0.0.1", port)   # noqa: E731
        return rc_.spdy_portforward_response(req, dial) if spdy else rc_.portforward_response(req, dial)
    st, cid, err = _find(kubelet, parts)
    if err:
        return Response(404, err.encode(), "text/plain")
    q = parse_qs(req.qs or "")
    cmd = q.get("command") or q.get("cmd") or []
    if verb == "exec" and not cmd:
        return Response(400, b"command is required", "text/plain")
    try:
        opts = rc_.options_from_query(req.qs)
    except ValueError as e:
        return Response(400, str(e).encode(), "text/plain")
    if hasattr(rt, "exec_url"):
        kw = dict(tty=opts.tty, stdin=opts.stdin, stdout=opts.stdout, stderr=opts.stderr)
        url = await rt.exec_url(cid, cmd, **kw) if verb == "exec" else await rt.attach_url(cid, **kw)
        return rc_.upgrade_proxy_response(req, url)
    if verb == "exec":
        async def run(stdin, stdout, stderr, tty, resize):
            return await rt.exec_interactive(cid, cmd, stdin, stdout, stderr, tty, resize)
    else:
        async def run(stdin, stdout, stderr, tty, resize):
            return await rt.attach(cid, stdin, stdout, stderr, tty, resize)
    return rc_.spdy_exec_response(req, run) if spdy else rc_.exec_response(req, req.qs, run)


def _static(raw):
    async def run(w):
        w.transport.write(raw)
    return run


def _proxy_exec(url):
    from ..cri.streaming import _open

    async def run(w):
        r, uw, status, _ = await _open(url)
        try:
            if status != 200:
                w.transport.write(_frames(126, f"exec refused by runtime: HTTP {status}".encode()))
                return
            # forward the runtime's chunked frames verbatim (already framed)
            while True:
                line = await r.readuntil(b"\r\n")
                size = int(line.strip(), 16)
                if size == 0:
                    break
                data = await r.readexactly(size + 2)
                w.transport.write(line + data)
        finally:
            uw.close()
    return run
