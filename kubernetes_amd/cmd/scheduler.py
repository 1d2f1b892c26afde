"""kube-scheduler entry point (reference: plugin/cmd/kube-scheduler/app/server.go:320-552)."""
from __future__ import annotations

import argparse
import asyncio
import json

from ..client.rest import Client
from ..scheduler.scheduler import Scheduler
from ._common import run_until_signal, setup_logging


def main(argv=None):
    ap = argparse.ArgumentParser("kube-scheduler")
    ap.add_argument("--master", required=True)
    ap.add_argument("--scheduler-name", default="default-scheduler")
    ap.add_argument("--policy-config-file", default=None, help="JSON Policy {predicates:[{name}], priorities:[{name,weight}]}")
    ap.add_argument("--percentage-of-nodes-to-score", type=int, default=100)
    ap.add_argument("--metrics-port", type=int, default=None)
    ap.add_argument("--no-events", action="store_true")
    ap.add_argument("--kube-api-qps", type=float, default=None)
    ap.add_argument("--leader-elect", action="store_true")
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    setup_logging(a.v)
    preds = prios = None
    if a.policy_config_file:
        with open(a.policy_config_file) as f:
            pol = json.load(f)
        preds = [p["name"] for p in pol.get("predicates") or []] or None
        if pol.get("priorities") is not None:
            prios = {p["name"]: int(p.get("weight", 1)) for p in pol["priorities"]}

    async def start():
        client = Client(a.master, qps=a.kube_api_qps, burst=int(a.kube_api_qps or 10), max_conns=64)
        s = Scheduler(client, a.scheduler_name, preds, prios, a.percentage_of_nodes_to_score,
                      emit_events=not a.no_events)
        if a.leader_elect:
            from ..client.leaderelection import LeaderElector
            le = LeaderElector(client, "kube-system", "kube-scheduler")
            await le.acquire()
        asyncio.ensure_future(s.run(metrics_port=a.metrics_port))
        return s

    run_until_signal(start)


if __name__ == "__main__":
    main()
