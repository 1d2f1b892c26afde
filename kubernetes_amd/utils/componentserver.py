"""The insecure health/metrics endpoint of the control-plane daemons.

Parity: kube-controller-manager `--port` 10252 / `--address` and kube-scheduler `--port` 10251 /
`--address` (`cmd/kube-controller-manager/app/controllermanager.go` startHTTP,
`plugin/cmd/kube-scheduler/app/server.go` makeHealthzServer/makeMetricsServer): `/healthz`,
`/metrics` (Prometheus text), `/configz` (the component's effective configuration) and, with
`--profiling`, `/debug/pprof`. These are the URLs the API server's componentstatuses probe.
A port that is already taken is logged, not fatal: several daemons of one kind can share a
host in tests and rehearsals.
"""
from __future__ import annotations

import json
import logging

from .httpserver import HTTPServer, Response

log = logging.getLogger("componentserver")


class ComponentServer:
    def __init__(self, name, metrics=None, healthz=None, configz=None, profiling=True):
        """metrics: object with render() -> bytes/str; healthz: () -> None | error string;
        configz: () -> dict."""
        self.name = name
        self.metrics, self.healthz, self.configz, self.profiling = metrics, healthz, configz, profiling
        self.http = None
        self.port = None

    async def _handle(self, req):
        p = req.path
        if p in ("/healthz", "/healthz/ping"):
            err = self.healthz() if self.healthz is not None else None
            return Response(500, f"healthz check failed: {err}".encode(), "text/plain") if err else \
                Response(200, b"ok", "text/plain")
        if p == "/metrics":
            body = self.metrics.render() if self.metrics is not None else b""
            return Response(200, body, "text/plain; version=0.0.4")
        if p == "/configz":
            return Response(200, json.dumps({self.name: self.configz() if self.configz else {}}).encode())
        if p.startswith("/debug/pprof") and self.profiling:
            from .profiling import handle_debug
            return await handle_debug(req)
        return Response(404, b"not found", "text/plain")

    async def start(self, address="0.0.0.0", port=0):
        if port is None or port < 0:
            return None
        self.http = HTTPServer(self._handle)
        try:
            self.port = await self.http.start(address, port)
        except OSError as e:
            log.warning("%s: health/metrics endpoint %s:%s not started: %s", self.name, address, port, e)
            self.http = None
            return None
        return self.port

    async def stop(self):
        if self.http is not None:
            await self.http.stop()
