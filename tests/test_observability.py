"""Audit log, utiltrace, /debug/pprof."""
import json
import logging

from kubernetes_amd.apiserver.audit import AuditLogger, Policy
from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client.http import HTTPClient
from kubernetes_amd.client.rest import Client
from kubernetes_amd.utils.trace import Trace


def test_audit_policy_levels_and_events(tmp_path, run):
    pol = Policy([
        {"level": "None", "users": ["system:kube-proxy"]},
        {"level": "None", "resources": [{"group": "", "resources": ["events"]}]},
        {"level": "RequestResponse", "resources": [{"group": "", "resources": ["pods/binding"]}]},
        {"level": "Request", "verbs": ["create"], "resources": [{"group": "", "resources": ["pods"]}]},
        {"level": "Metadata"},
    ])
    path = str(tmp_path / "audit.log")

    async def main():
        s = APIServer(audit=AuditLogger(path, pol))
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        try:
            await c.create("nodes", {"metadata": {"name": "n0"}})
            p = await c.create("pods", {"metadata": {"name": "p", "namespace": "default"},
                                        "spec": {"containers": [{"name": "c", "image": "x",
                                                                 "resources": {"limits": {"amd.com/gpu": "1"}}}]}})
            er = p["spec"]["extendedResources"][0]["name"]
            await c.bind("default", "p", "n0", {er: {"resources": ["GPU-0"]}})
            await c.get("pods", "p", "default")
            await c.list("pods", "default")
            await c.create("events", {"metadata": {"name": "e1", "namespace": "default"},
                                      "involvedObject": {"kind": "Pod", "name": "p"}, "reason": "x"})
        finally:
            await c.close()
            await s.stop()
            s.audit.close()
    run(main())
    evs = [json.loads(line) for line in open(path)]
    by = [(e["verb"], e["objectRef"]["resource"], e["objectRef"].get("subresource"), e["level"]) for e in evs]
    assert ("create", "nodes", None, "Metadata") in by
    assert ("create", "pods", None, "Request") in by
    assert ("create", "pods", "binding", "RequestResponse") in by
    assert ("get", "pods", None, "Metadata") in by and ("list", "pods", None, "Metadata") in by
    assert not [e for e in evs if e["objectRef"]["resource"] == "events"]
    create_pod = next(e for e in evs if e["verb"] == "create" and e["objectRef"]["resource"] == "pods"
                      and not e["objectRef"].get("subresource"))
    assert create_pod["requestObject"]["metadata"]["name"] == "p" and create_pod["responseStatus"]["code"] == 201
    assert create_pod["objectRef"]["namespace"] == "default"


def test_trace_logs_only_when_long(caplog):
    t = Trace("fast")
    t.step("a")
    assert not t.log_if_long(10.0)
    t2 = Trace("slow")
    t2.step("phase one")
    with caplog.at_level(logging.WARNING):
        assert t2.log_if_long(0.0)
    assert 'Trace "slow"' in caplog.text and "phase one" in caplog.text


def test_debug_pprof(run):
    async def main():
        s = APIServer()
        port = await s.start()
        h = HTTPClient(f"http://127.0.0.1:{port}")
        try:
            st, body = await h.request("GET", "/debug/pprof/profile?seconds=0.2")
            assert st == 200 and b"function calls" in body
            st, body = await h.request("GET", "/debug/pprof/goroutine")
            assert st == 200 and b"task" in body and b"thread MainThread" in body
        finally:
            await h.close()
            await s.stop()
    run(main())
