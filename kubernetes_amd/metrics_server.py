"""metrics-server: resource metrics API (`metrics.k8s.io/v1beta1`) served through API aggregation.

Parity: the `cluster/addons/metrics-server` add-on (kubernetes-incubator/metrics-server, vendored
API types in `staging/src/k8s.io/metrics/pkg/apis/metrics`): scrape every node's kubelet
`/stats/summary` each `--metric-resolution` (60 s), keep the latest sample, serve `NodeMetrics`
and `PodMetrics` (`usage: {cpu, memory}`) under `/apis/metrics.k8s.io/v1beta1/...`, registered with
the aggregator by an APIService. MI355X addition: container usage also carries
`amd.com/gpu` = GPU duty cycle in percent (averaged over the container's assigned GPUs, from the
kubelet's AMD SMI accelerator stats), so the HPA can scale on GPU utilization.
"""
from __future__ import annotations

import asyncio
import json
import logging
import time

from .api.meta import now_rfc3339
from .client.http import HTTPClient
from .utils.httpserver import HTTPServer, Response
from .utils.tasks import spawn

log = logging.getLogger("metrics-server")
GROUP, VERSION = "metrics.k8s.io", "v1beta1"


def cpu_q(nano):
    return f"{int(round(nano / 1e6))}m"


def mem_q(b):
    return f"{int(b // 1024)}Ki"


class MetricsServer:
    def __init__(self, client, resolution=60.0, history_path=None):
        self.client = client
        # JSON-lines usage history for the InitialResources admission plugin (the reference's
        # heapster → influxdb sink): one sample per container per scrape, keyed by image.
        self.history = None
        if history_path:
            from .apiserver.admission.estimation import UsageHistory
            self.history = UsageHistory(history_path)
        self.resolution = resolution
        self.nodes: dict = {}       # node -> NodeMetrics
        self.pods: dict = {}        # (ns, name) -> PodMetrics
        self.http = HTTPServer(self.handle)
        self.port = None
        self._task = None
        self.scrapes = 0

    async def scrape_once(self):
        nodes = (await self.client.list("nodes"))["items"]
        nodes_out, pods_out = {}, {}
        ts = now_rfc3339()
        for n in nodes:
            st = n.get("status") or {}
            port = ((st.get("daemonEndpoints") or {}).get("kubeletEndpoint") or {}).get("Port")
            addr = next((a["address"] for a in st.get("addresses") or () if a.get("type") == "InternalIP"), "127.0.0.1")
            if not port:
                continue
            c = HTTPClient(f"http://{addr}:{port}", timeout=10)
            try:
                code, body = await c.request("GET", "/stats/summary")
            except OSError as e:
                log.debug("scrape %s failed: %s", n["metadata"]["name"], e)
                continue
            finally:
                await c.close()
            if code != 200:
                continue
            summ = json.loads(body)
            node = summ.get("node") or {}
            nodes_out[n["metadata"]["name"]] = {
                "kind": "NodeMetrics", "apiVersion": f"{GROUP}/{VERSION}",
                "metadata": {"name": n["metadata"]["name"], "creationTimestamp": ts},
                "timestamp": ts, "window": f"{int(self.resolution)}s",
                "usage": {"cpu": cpu_q((node.get("cpu") or {}).get("usageNanoCores", 0)),
                          "memory": mem_q((node.get("memory") or {}).get("workingSetBytes", 0))}}
            for p in summ.get("pods") or ():
                ref = p["podRef"]
                cs = []
                for ctr in p.get("containers") or ():
                    usage = {"cpu": cpu_q((ctr.get("cpu") or {}).get("usageNanoCores", 0)),
                             "memory": mem_q((ctr.get("memory") or {}).get("workingSetBytes", 0))}
                    acc = ctr.get("accelerators") or []
                    if acc:
                        usage["amd.com/gpu"] = str(int(round(sum(a.get("dutyCycle", 0) for a in acc) / len(acc))))
                    cs.append({"name": ctr["name"], "usage": usage})
                pods_out[(ref["namespace"], ref["name"])] = {
                    "kind": "PodMetrics", "apiVersion": f"{GROUP}/{VERSION}",
                    "metadata": {"name": ref["name"], "namespace": ref["namespace"], "creationTimestamp": ts},
                    "timestamp": ts, "window": f"{int(self.resolution)}s", "containers": cs}
        self.nodes, self.pods = nodes_out, pods_out
        self.scrapes += 1
        if self.history is not None and pods_out:
            await self._record_history(pods_out)

    async def _record_history(self, pods_out):
        images = {}
        for p in (await self.client.list("pods"))["items"]:
            md = p["metadata"]
            for c in (p.get("spec") or {}).get("containers") or ():
                images[(md.get("namespace"), md["name"], c["name"])] = c.get("image", "")
        now = time.time()
        for (ns, name), pm in pods_out.items():
            for c in pm["containers"]:
                img = images.get((ns, name, c["name"]))
                if img:
                    self.history.record(ns, img, int(c["usage"]["cpu"].rstrip("m")),
                                        int(c["usage"]["memory"].rstrip("Ki")) * 1024, ts=now)

    async def _loop(self):
        while True:
            try:
                await self.scrape_once()
            except Exception as e:   # keep serving the last sample
                log.warning("scrape failed: %s", e)
            await asyncio.sleep(self.resolution)

    async def handle(self, req):
        parts = [p for p in req.path.split("/") if p]
        if req.path in ("/healthz", "/livez", "/readyz"):
            return Response(200, b"ok", "text/plain")
        if parts[:3] != ["apis", GROUP, VERSION]:
            return Response(404, b'{"kind":"Status","code":404}')
        rest = parts[3:]
        if not rest:
            return Response(200, json.dumps({"kind": "APIResourceList", "groupVersion": f"{GROUP}/{VERSION}", "resources": [
                {"name": "nodes", "namespaced": False, "kind": "NodeMetrics", "verbs": ["get", "list"]},
                {"name": "pods", "namespaced": True, "kind": "PodMetrics", "verbs": ["get", "list"]}]}).encode())
        if rest[0] == "nodes":
            if len(rest) > 1:
                m = self.nodes.get(rest[1])
                return Response(200, json.dumps(m).encode()) if m else Response(404, b'{"kind":"Status","code":404}')
            return Response(200, json.dumps({"kind": "NodeMetricsList", "apiVersion": f"{GROUP}/{VERSION}",
                                             "metadata": {}, "items": list(self.nodes.values())}).encode())
        ns = None
        if rest[0] == "namespaces" and len(rest) >= 3:
            ns, rest = rest[1], rest[2:]
        if rest[0] == "pods":
            if len(rest) > 1:
                m = self.pods.get((ns, rest[1]))
                return Response(200, json.dumps(m).encode()) if m else Response(404, b'{"kind":"Status","code":404}')
            items = [v for (pns, _), v in self.pods.items() if ns is None or pns == ns]
            sel = req.query.get("labelSelector")
            if sel:
                from .api.labels import parse
                s = parse(sel)
                labels = await self._pod_labels(ns)
                items = [v for v in items if s.matches(labels.get((v["metadata"]["namespace"], v["metadata"]["name"]), {}))]
            return Response(200, json.dumps({"kind": "PodMetricsList", "apiVersion": f"{GROUP}/{VERSION}",
                                             "metadata": {}, "items": items}).encode())
        return Response(404, b'{"kind":"Status","code":404}')

    async def _pod_labels(self, ns):
        lst = await self.client.list("pods", ns)
        return {(p["metadata"].get("namespace"), p["metadata"]["name"]): p["metadata"].get("labels") or {}
                for p in lst["items"]}

    async def start(self, host="127.0.0.1", port=0, register=True):
        self.port = await self.http.start(host, port)
        self._task = spawn(self._loop())
        if register:
            await self.register(host)
        return self

    async def register(self, host):
        """Service + Endpoints + APIService `v1beta1.metrics.k8s.io` (the add-on's manifests)."""
        from .client.rest import APIStatusError
        objs = [("services", {"metadata": {"name": "metrics-server", "namespace": "kube-system"},
                              "spec": {"ports": [{"port": 443, "targetPort": self.port}]}}),
                ("endpoints", {"metadata": {"name": "metrics-server", "namespace": "kube-system"},
                               "subsets": [{"addresses": [{"ip": host}], "ports": [{"port": self.port}]}]}),
                ("apiservices", {"metadata": {"name": f"{VERSION}.{GROUP}"},
                                 "spec": {"group": GROUP, "version": VERSION, "insecureSkipTLSVerify": True,
                                          "groupPriorityMinimum": 100, "versionPriority": 100,
                                          "service": {"namespace": "kube-system", "name": "metrics-server"}}})]
        for res, o in objs:
            try:
                await self.client.create(res, o)
            except APIStatusError as e:
                if e.code != 409:
                    raise
                if res == "endpoints":
                    await self.client.patch("endpoints", "metrics-server", {"subsets": o["subsets"]}, "kube-system")

    async def stop(self):
        if self._task is not None:
            self._task.cancel()
        await self.http.stop()


def main(argv=None):
    import argparse
    from .client.rest import Client
    from .cmd._common import run_until_signal, setup_logging
    ap = argparse.ArgumentParser("metrics-server")
    ap.add_argument("--master", required=True)
    ap.add_argument("--metric-resolution", type=float, default=60.0)
    ap.add_argument("--bind-address", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--usage-history-file", default=None,
                    help="append per-container usage samples (InitialResources data source)")
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    setup_logging(a.v)

    async def start():
        ms = await MetricsServer(Client(a.master), a.metric_resolution, a.usage_history_file).start(a.bind_address, a.port)
        print(f"metrics-server serving {GROUP}/{VERSION} on {a.bind_address}:{ms.port}", flush=True)
        return ms
    run_until_signal(start)


if __name__ == "__main__":
    main()
