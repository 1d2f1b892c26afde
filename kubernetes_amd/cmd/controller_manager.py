"""kube-controller-manager entry point (reference: cmd/kube-controller-manager/app/controllermanager.go:106)."""
from __future__ import annotations

import argparse

from ..client.rest import Client
from ..controllers.manager import CONTROLLERS, ControllerManager
from ._common import run_until_signal, setup_logging


def main(argv=None):
    ap = argparse.ArgumentParser("kube-controller-manager")
    ap.add_argument("--master", required=True)
    ap.add_argument("--controllers", default="*", help=f"comma list; '*' = all of {sorted(CONTROLLERS)}, '-name' disables")
    ap.add_argument("--node-monitor-grace-period", type=float, default=40.0)
    ap.add_argument("--pod-eviction-timeout", type=float, default=300.0)
    ap.add_argument("--terminated-pod-gc-threshold", type=int, default=12500)
    ap.add_argument("--leader-elect", action="store_true")
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    setup_logging(a.v)

    async def start():
        client = Client(a.master, max_conns=64)
        if a.leader_elect:
            from ..client.leaderelection import LeaderElector
            await LeaderElector(client, "kube-system", "kube-controller-manager").acquire()
        opts = {"nodelifecycle": {"grace": a.node_monitor_grace_period, "pod_eviction_timeout": a.pod_eviction_timeout},
                "podgc": {"terminated_pod_gc_threshold": a.terminated_pod_gc_threshold}}
        return await ControllerManager(client, a.controllers.split(","), opts).start()

    run_until_signal(start)


if __name__ == "__main__":
    main()
