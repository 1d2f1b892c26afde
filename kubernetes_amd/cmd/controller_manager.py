"""kube-controller-manager entry point (reference: cmd/kube-controller-manager/app/controllermanager.go:106)."""
from __future__ import annotations

import argparse

from ..client.rest import Client
from ..controllers.manager import CONTROLLERS, ControllerManager
from ._common import run_until_signal, setup_logging


def main(argv=None):
    ap = argparse.ArgumentParser("kube-controller-manager")
    ap.add_argument("--master", default=None)
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--service-account-private-key-file", default=None)
    ap.add_argument("--root-ca-file", default=None)
    ap.add_argument("--cluster-signing-cert-file", default=None)
    ap.add_argument("--cluster-signing-key-file", default=None)
    ap.add_argument("--horizontal-pod-autoscaler-sync-period", type=float, default=30.0)
    ap.add_argument("--controllers", default="*", help=f"comma list; '*' = all of {sorted(CONTROLLERS)}, '-name' disables")
    ap.add_argument("--node-monitor-grace-period", type=float, default=40.0)
    ap.add_argument("--pod-eviction-timeout", type=float, default=300.0)
    ap.add_argument("--node-monitor-period", type=float, default=5.0)
    ap.add_argument("--node-startup-grace-period", type=float, default=60.0)
    ap.add_argument("--node-eviction-rate", type=float, default=0.1,
                    help="nodes per second whose pods are deleted on node failure in a healthy zone")
    ap.add_argument("--secondary-node-eviction-rate", type=float, default=0.01,
                    help="the rate in an unhealthy zone (0 below --large-cluster-size-threshold)")
    ap.add_argument("--large-cluster-size-threshold", type=int, default=50)
    ap.add_argument("--unhealthy-zone-threshold", type=float, default=0.55,
                    help="fraction of not-Ready nodes (at least 3) that makes a zone unhealthy")
    ap.add_argument("--enable-taint-manager", default="true", choices=("true", "false"),
                    help="evict pods from nodes with NoExecute taints they do not tolerate")
    ap.add_argument("--feature-gates", default="", help="e.g. TaintBasedEvictions=true,TaintNodesByCondition=true")
    ap.add_argument("--terminated-pod-gc-threshold", type=int, default=12500)
    ap.add_argument("--leader-elect", action="store_true")
    ap.add_argument("--allocate-node-cidrs", action="store_true")
    ap.add_argument("--cluster-cidr", default="10.244.0.0/16")
    ap.add_argument("--node-cidr-mask-size", type=int, default=24)
    ap.add_argument("--configure-cloud-routes", action="store_true",
                    help="run the route controller: program a route to every node's pod CIDR (with --allocate-node-cidrs)")
    ap.add_argument("--route-table", default="ip", choices=("ip", "memory"),
                    help="where routes go: 'ip' (ip route on this gateway host) or 'memory'")
    ap.add_argument("--route-reconciliation-period", type=float, default=10.0,
                    help="seconds between full route reconciliations (besides node events)")
    ap.add_argument("--loadbalancer-ip-range", default="",
                    help="on-prem LoadBalancer pool ('10.0.5.10-10.0.5.50' or a CIDR); enables the service controller")
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    setup_logging(a.v)
    from ..utils.features import DefaultFeatureGate
    DefaultFeatureGate.set(a.feature_gates)

    async def start():
        if a.kubeconfig:
            from ..client.clientcmd import client_from
            client = client_from(a.kubeconfig, max_conns=64)
        else:
            client = Client(a.master or "http://127.0.0.1:8080", max_conns=64)
        if a.leader_elect:
            from ..client.leaderelection import LeaderElector
            await LeaderElector(client, "kube-system", "kube-controller-manager").acquire()
        opts = {"nodelifecycle": {"grace": a.node_monitor_grace_period, "pod_eviction_timeout": a.pod_eviction_timeout,
                                  "monitor_period": a.node_monitor_period, "startup_grace": a.node_startup_grace_period,
                                  "eviction_rate": a.node_eviction_rate,
                                  "secondary_eviction_rate": a.secondary_node_eviction_rate,
                                  "large_cluster_threshold": a.large_cluster_size_threshold,
                                  "unhealthy_zone_threshold": a.unhealthy_zone_threshold,
                                  "taint_manager": a.enable_taint_manager == "true"},
                "podgc": {"terminated_pod_gc_threshold": a.terminated_pod_gc_threshold},
                "serviceaccount-token": {"private_key_file": a.service_account_private_key_file, "root_ca_file": a.root_ca_file},
                "csrsigning": {"cert_file": a.cluster_signing_cert_file, "key_file": a.cluster_signing_key_file},
                "horizontalpodautoscaling": {"sync_period": a.horizontal_pod_autoscaler_sync_period},
                "nodeipam": {"cluster_cidr": a.cluster_cidr, "node_cidr_mask_size": a.node_cidr_mask_size},
                "route": {"cluster_cidr": a.cluster_cidr, "routes": a.route_table,
                          "reconcile_period": a.route_reconciliation_period},
                "service": {"ip_range": a.loadbalancer_ip_range}}
        enabled = a.controllers.split(",")
        if a.allocate_node_cidrs:
            enabled.append("nodeipam")
            if a.configure_cloud_routes:
                enabled.append("route")
        if a.loadbalancer_ip_range:
            enabled.append("service")
        return await ControllerManager(client, enabled, opts).start()

    run_until_signal(start)


if __name__ == "__main__":
    main()
