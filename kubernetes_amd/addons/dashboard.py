"""Cluster dashboard add-on (the reference ships `cluster/addons/dashboard`, the kubernetes-dashboard
web UI). This one is read-only and GPU-first: one page per cluster, rendered on the server from the
API, with

  * nodes: readiness, GPU capacity / allocated, and per device its health, xGMI hive, NUMA node,
    compute partition and socket, burn-in result and measured TFLOP/s (`amd.com/*` attributes);
  * pods: phase, node, and the device IDs bound to them (`spec.extendedResources[].assigned`);
  * the most recent warning events.

`/` is HTML, `/api/summary` the same data as JSON (what the page is built from).

    python -m kubernetes_amd.cmd.dashboard --master http://127.0.0.1:8080 --port 9090
"""
from __future__ import annotations

import html
import json

from ..api import core
from ..client.rest import Client
from ..utils.httpserver import HTTPServer, Response


async def summary(client: Client) -> dict:
    nodes = (await client.list("nodes"))["items"]
    pods = (await client.list("pods"))["items"]
    events = (await client.list("events"))["items"]
    used = {}                      # (node, device id) -> "ns/pod"
    pod_rows = []
    for p in pods:
        md, sp, st = p["metadata"], p.get("spec") or {}, p.get("status") or {}
        devs = [i for ids in core.pod_assigned_devices(p).values() for i in ids]
        if not core.pod_is_terminal(p):
            for d in devs:
                used[(sp.get("nodeName"), d)] = f"{md.get('namespace')}/{md['name']}"
        pod_rows.append({"namespace": md.get("namespace"), "name": md["name"], "phase": st.get("phase", "Pending"),
                         "node": sp.get("nodeName") or "", "gpus": devs})
    node_rows = []
    for n in nodes:
        name, st = n["metadata"]["name"], n.get("status") or {}
        ready = any(c.get("type") == "Ready" and c.get("status") == "True" for c in st.get("conditions") or ())
        devs = ((st.get("extendedResources") or {}).get(core.AMD_GPU) or {}).get("resources") or {}
        rows = []
        for did, d in sorted(devs.items(), key=lambda kv: int((kv[1].get("attributes") or {}).get(core.ATTR_INDEX, 1 << 30))):
            a = d.get("attributes") or {}
            rows.append({"id": did, "health": d.get("health"), "hive": a.get(core.ATTR_HIVE, ""),
                         "numa": a.get(core.ATTR_NUMA, ""), "partition": a.get(core.ATTR_PARTITION, "SPX"),
                         "socket": a.get(core.ATTR_SOCKET, ""), "burn_in": a.get("amd.com/burn-in", ""),
                         "tflops": a.get("amd.com/mfma-tflops", ""), "fp8_tflops": a.get("amd.com/mfma-fp8-tflops", ""),
                         "pod": used.get((name, did), "")})
        node_rows.append({"name": name, "ready": ready, "unschedulable": bool((n.get("spec") or {}).get("unschedulable")),
                          "gpus": len(devs), "allocated": sum(1 for r in rows if r["pod"]),
                          "healthy": sum(1 for r in rows if r["health"] == core.HEALTHY), "devices": rows})
    warnings = sorted((e for e in events if e.get("type") == "Warning"),
                      key=lambda e: e.get("lastTimestamp") or "", reverse=True)[:20]
    return {"nodes": node_rows, "pods": pod_rows,
            "gpus": {"total": sum(r["gpus"] for r in node_rows), "allocated": sum(r["allocated"] for r in node_rows),
                     "healthy": sum(r["healthy"] for r in node_rows)},
            "warnings": [{"object": f"{(e.get('involvedObject') or {}).get('kind', '')}/"
                                    f"{(e.get('involvedObject') or {}).get('name', '')}",
                          "reason": e.get("reason", ""), "message": e.get("message", "")} for e in warnings]}


def render(s: dict) -> str:
    e = html.escape
    out = ["<!doctype html><html><head><meta charset='utf-8'><title>kubernetes_amd dashboard</title>",
           "<style>body{font-family:sans-serif;margin:1em}table{border-collapse:collapse;margin-bottom:1em}"
           "td,th{border:1px solid #ccc;padding:2px 6px;font-size:13px}.bad{color:#b00}</style></head><body>",
           f"<h1>GPUs: {s['gpus']['allocated']} / {s['gpus']['total']} allocated, {s['gpus']['healthy']} healthy</h1>"]
    for n in s["nodes"]:
        state = "Ready" if n["ready"] else "<span class='bad'>NotReady</span>"
        out.append(f"<h2>{e(n['name'])} — {state}{' (cordoned)' if n['unschedulable'] else ''} — "
                   f"{n['allocated']}/{n['gpus']} GPUs allocated</h2>")
        if n["devices"]:
            out.append("<table><tr><th>device</th><th>health</th><th>hive</th><th>numa</th><th>partition</th>"
                       "<th>burn-in</th><th>bf16 / fp8 TF/s</th><th>pod</th></tr>")
            for d in n["devices"]:
                cls = "" if d["health"] == core.HEALTHY else " class='bad'"
                part = d["partition"] + (f"@{d['socket']}" if d["partition"] != "SPX" else "")
                out.append(f"<tr><td>{e(d['id'])}</td><td{cls}>{e(str(d['health']))}</td><td>{e(d['hive'])}</td>"
                           f"<td>{e(d['numa'])}</td><td>{e(part)}</td><td>{e(d['burn_in'])}</td>"
                           f"<td>{e(d['tflops'])} / {e(d['fp8_tflops'])}</td><td>{e(d['pod'])}</td></tr>")
            out.append("</table>")
    out.append("<h2>Pods</h2><table><tr><th>namespace</th><th>name</th><th>phase</th><th>node</th><th>GPUs</th></tr>")
    for p in s["pods"]:
        out.append(f"<tr><td>{e(p['namespace'] or '')}</td><td>{e(p['name'])}</td><td>{e(p['phase'])}</td>"
                   f"<td>{e(p['node'])}</td><td>{e(', '.join(p['gpus']))}</td></tr>")
    out.append("</table>")
    if s["warnings"]:
        out.append("<h2>Warnings</h2><table><tr><th>object</th><th>reason</th><th>message</th></tr>")
        for w in s["warnings"]:
            out.append(f"<tr><td>{e(w['object'])}</td><td>{e(w['reason'])}</td><td>{e(w['message'])}</td></tr>")
        out.append("</table>")
    out.append("</body></html>")
    return "\n".join(out)


class Dashboard:
    def __init__(self, master, token=None):
        self.client = Client(master, token=token)
        self.http = None

    async def _handle(self, req):
        if req.path in ("/", "/index.html"):
            return Response(200, render(await summary(self.client)).encode(), "text/html; charset=utf-8")
        if req.path == "/api/summary":
            return Response(200, json.dumps(await summary(self.client)).encode())
        if req.path == "/healthz":
            return Response(200, b"ok", "text/plain")
        return Response(404, b"not found", "text/plain")

    async def start(self, host="0.0.0.0", port=9090):
        self.http = HTTPServer(self._handle)
        return await self.http.start(host, port)

    async def stop(self):
        if self.http:
            await self.http.stop()
        await self.client.close()
