"""Liveness / readiness probes.

Parity: `pkg/kubelet/prober` — `prober.go` (exec via the runtime's ExecSync, HTTP GET with
success = 200 <= code < 400, TCP connect), `worker.go` (one worker per container and probe
type: `initialDelaySeconds`, `periodSeconds` (10), `timeoutSeconds` (1), `successThreshold` (1),
`failureThreshold` (3); a readiness result starts as Failure until the first success, liveness
as Success), `prober_manager.go` (results feed the container's `ready` and the kubelet kills a
container whose liveness probe fails, restarting it per the pod's restartPolicy).
"""
from __future__ import annotations

import asyncio
import logging

from .runtime.base import EXITED, RUNNING

log = logging.getLogger("kubelet.prober")


def extract_port(port, container) -> int:
    """`prober.go` extractPort: an int, a numeric string or a named container port; the result
    must be in 1..65535."""
    if isinstance(port, int) and not isinstance(port, bool):
        n = port
    elif isinstance(port, str) and port.lstrip("-").isdigit():
        n = int(port)
    elif isinstance(port, str):
        n = find_port_by_name(container, port)
    else:
        raise ValueError(f"invalid port {port!r}")
    if 0 < n < 65536:
        return n
    raise ValueError(f"invalid port number: {n}")


def find_port_by_name(container, name) -> int:
    for p in container.get("ports") or ():
        if p.get("name") == name:
            return int(p["containerPort"])
    raise ValueError(f"port {name} not found")


_port = extract_port       # the old name


def format_url(scheme, host, port, path) -> str:
    """`prober.go` formatURL: scheme://host:port plus the path (and its query)."""
    h = f"[{host}]" if ":" in host and not host.startswith("[") else host
    return f"{scheme.lower()}://{h}:{port}{path}"


def _request_target(path) -> str:
    if not path:
        return "/"
    return path if path.startswith("/") else "/" + path


async def run_probe(runtime, pod, container, cid, probe, pod_ip="127.0.0.1"):
    """Returns (success, message)."""
    timeout = float(probe.get("timeoutSeconds") or 1)
    try:
        if "exec" in probe:
            rc, out = await runtime.exec_sync(cid, probe["exec"].get("command") or [], timeout)
            return rc == 0, out.decode(errors="replace")[-256:] if isinstance(out, bytes) else str(out)
        if "httpGet" in probe:
            h = probe["httpGet"]
            host = h.get("host") or pod_ip
            port = extract_port(h.get("port"), container)
            path = _request_target(h.get("path") or "")
            ssl_ctx = None
            if (h.get("scheme") or "HTTP").upper() == "HTTPS":
                import ssl
                ssl_ctx = ssl.create_default_context()      # http.go: InsecureSkipVerify
                ssl_ctx.check_hostname = False
                ssl_ctx.verify_mode = ssl.CERT_NONE
            headers = {"Host": f"{host}:{port}", "User-Agent": "kube-probe/1.9"}
            for x in h.get("httpHeaders") or ():
                headers[x["name"]] = x["value"]             # a user Host header replaces the default
            hdrs = "".join(f"{k}: {v}\r\n" for k, v in headers.items())
            r, w = await asyncio.wait_for(asyncio.open_connection(host, port, ssl=ssl_ctx), timeout)
            try:
                w.write(f"GET {path} HTTP/1.1\r\n{hdrs}Connection: close\r\n\r\n".encode())
                line = await asyncio.wait_for(r.readline(), timeout)
            finally:
                w.close()
            parts = line.split()
            code = int(parts[1]) if len(parts) > 1 else 0
            if 200 <= code < 400:
                return True, ""
            return False, f"HTTP probe failed with statuscode: {code}"
        if "tcpSocket" in probe:
            t = probe["tcpSocket"]
            r, w = await asyncio.wait_for(asyncio.open_connection(t.get("host") or pod_ip,
                                                                  extract_port(t.get("port"), container)), timeout)
            w.close()
            return True, ""
    except (OSError, asyncio.TimeoutError, ValueError, NotImplementedError) as e:
        return False, f"probe error: {e}"
    return False, "probe has no handler"


class _Worker:
    def __init__(self, mgr, uid, pod, container, cid, kind, probe):
        self.mgr, self.uid, self.pod, self.container, self.cid, self.kind, self.probe = (
            mgr, uid, pod, container, cid, kind, probe)
        self.result = kind == "liveness"          # readiness starts "not ready"
        self.ok_run = self.fail_run = 0
        self.task = asyncio.ensure_future(self.run())

    async def run(self):
        p = self.probe
        period = float(p.get("periodSeconds") or 10)
        succ_th = int(p.get("successThreshold") or 1)
        fail_th = int(p.get("failureThreshold") or 3)
        await asyncio.sleep(float(p.get("initialDelaySeconds") or 0))
        while True:
            status_fn = getattr(self.mgr.runtime, "container_status", None)
            cs = status_fn(self.cid) if status_fn is not None else None
            if cs is not None and cs.state != RUNNING:
                # worker.go doProbe: a non-running container is not probed; readiness fails at
                # once (no threshold), and the worker ends if the container will not restart
                if self.kind == "readiness" and self.result:
                    self.result = False
                    self.ok_run = 0
                    self.mgr.changed(self, "container is not running")
                if cs.state == EXITED and (self.pod.get("spec") or {}).get("restartPolicy") == "Never":
                    return
                await asyncio.sleep(period)
                continue
            ok, msg = await run_probe(self.mgr.runtime, self.pod, self.container, self.cid, p, self.mgr.pod_ip(self.uid))
            if ok:
                self.ok_run += 1
                self.fail_run = 0
            else:
                self.fail_run += 1
                self.ok_run = 0
                self.mgr.failed(self, msg)
            new = self.result
            if ok and self.ok_run >= succ_th:
                new = True
            elif not ok and self.fail_run >= fail_th:
                new = False
            if new != self.result:
                self.result = new
                self.mgr.changed(self, msg)
                if self.kind == "liveness" and not new:
                    return   # the container is being killed; a new worker follows the restart
            await asyncio.sleep(period)

    def stop(self):
        self.task.cancel()


class ProbeManager:
    def __init__(self, runtime, on_readiness, on_liveness_failure, pod_ip=lambda uid: "127.0.0.1",
                 on_probe_failure=None):
        self.runtime = runtime
        self.on_probe_failure = on_probe_failure
        self.on_readiness = on_readiness
        self.on_liveness_failure = on_liveness_failure
        self.pod_ip = pod_ip
        self.workers: dict[tuple, _Worker] = {}   # (uid, container, kind) -> worker

    def start(self, uid, pod, container, cid):
        for kind in ("readiness", "liveness"):
            p = container.get(f"{kind}Probe")
            key = (uid, container["name"], kind)
            old = self.workers.pop(key, None)
            if old is not None:
                old.stop()
            if p:
                self.workers[key] = _Worker(self, uid, pod, container, cid, kind, p)

    def ready(self, uid, cname):
        """None when the container has no readiness probe."""
        w = self.workers.get((uid, cname, "readiness"))
        return None if w is None else w.result

    def failed(self, w, msg):
        """`prober.probe`: every failed probe is a Warning `Unhealthy` event on the container
        ("Liveness probe failed: <output>")."""
        if self.on_probe_failure is not None:
            self.on_probe_failure(w.uid, w.container["name"], w.kind, msg)

    def changed(self, w, msg):
        if w.kind == "readiness":
            self.on_readiness(w.uid, w.container["name"], w.result)
        elif not w.result:
            log.info("liveness probe of %s/%s failed: %s", w.uid, w.container["name"], msg)
            self.on_liveness_failure(w.uid, w.container["name"], w.cid, msg)

    def remove_pod(self, uid):
        for key in [k for k in self.workers if k[0] == uid]:
            self.workers.pop(key).stop()

    def stop(self):
        for w in self.workers.values():
            w.stop()
        self.workers.clear()
