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
    _reference_flags(ap)
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    setup_logging(a.v)
    if a.cloud_provider:
        raise SystemExit(f"kube-controller-manager: --cloud-provider={a.cloud_provider}: cloud providers are out of "
                         "scope here (LoadBalancers come from --loadbalancer-ip-range)")
    from ..utils.features import DefaultFeatureGate
    DefaultFeatureGate.set(a.feature_gates)

    async def start():
        if a.kubeconfig:
            from ..client.clientcmd import client_from
            client = client_from(a.kubeconfig, max_conns=64, qps=a.kube_api_qps, burst=a.kube_api_burst)
        else:
            client = Client(a.master or "http://127.0.0.1:8080", max_conns=64, qps=a.kube_api_qps, burst=a.kube_api_burst)
        from ..utils.componentserver import ComponentServer
        health = ComponentServer("componentconfig", profiling=a.profiling, configz=lambda: {
            k: v for k, v in vars(a).items() if not k.startswith("_")})
        if a.port:
            await health.start(a.address, a.port)
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
                "csrsigning": {"cert_file": a.cluster_signing_cert_file, "key_file": a.cluster_signing_key_file,
                               "days": max(1, int(_dur(a.experimental_cluster_signing_duration) // 86400))},
                "horizontalpodautoscaling": {"sync_period": a.horizontal_pod_autoscaler_sync_period,
                                             "tolerance": a.horizontal_pod_autoscaler_tolerance,
                                             "upscale_window": _dur(a.horizontal_pod_autoscaler_upscale_delay),
                                             "downscale_window": _dur(a.horizontal_pod_autoscaler_downscale_delay)},
                "nodeipam": {"cluster_cidr": a.cluster_cidr, "node_cidr_mask_size": a.node_cidr_mask_size},
                "route": {"cluster_cidr": a.cluster_cidr, "routes": a.route_table,
                          "reconcile_period": a.route_reconciliation_period},
                "service": {"ip_range": a.loadbalancer_ip_range}}
        if a.enable_hostpath_provisioner:
            opts["persistentvolume-binder"] = {"hostpath_root": "/tmp/hostpath_pv"}
        enabled = a.controllers.split(",")
        if not a.enable_garbage_collector:
            enabled.append("-garbagecollector")
        if a.allocate_node_cidrs:
            enabled.append("nodeipam")
            if a.configure_cloud_routes:
                enabled.append("route")
        if a.loadbalancer_ip_range:
            enabled.append("service")
        workers = {"deployment": a.concurrent_deployment_syncs, "replicaset": a.concurrent_replicaset_syncs,
                   "replicationcontroller": a.concurrent_rc_syncs, "endpoint": a.concurrent_endpoint_syncs,
                   "garbagecollector": a.concurrent_gc_syncs, "namespace": a.concurrent_namespace_syncs,
                   "resourcequota": a.concurrent_resource_quota_syncs, "service": a.concurrent_service_syncs,
                   "serviceaccount-token": a.concurrent_serviceaccount_token_syncs}
        sa_factory = None
        if a.use_service_account_credentials:
            if not a.service_account_private_key_file:
                raise SystemExit("kube-controller-manager: --use-service-account-credentials needs "
                                 "--service-account-private-key-file (the token controller mints the tokens)")
            root = client

            def sa_factory(token):
                return Client(root.url, token=token, ssl_context=root.http.ssl, max_conns=16,
                              qps=a.kube_api_qps, burst=a.kube_api_burst)
        cm = await ControllerManager(client, enabled, opts, workers=workers,
                                     start_interval=_dur(a.controller_start_interval),
                                     sa_client_factory=sa_factory).start()
        health.metrics = cm
        return cm

    run_until_signal(start)


def _dur(v):
    from ..kubelet.eviction import parse_duration
    v = str(v).strip()
    return float(v) if v.replace(".", "", 1).isdigit() else parse_duration(v)


def _bool(v):
    return str(v).lower() not in ("false", "0", "no")


def _reference_flags(ap):
    """The rest of kube-controller-manager's flags (cmd/kube-controller-manager/app/options)."""
    g = ap.add_argument_group("serving")
    g.add_argument("--port", type=int, default=10252, help="/healthz, /metrics, /configz (0 = off)")
    g.add_argument("--address", default="0.0.0.0")
    g.add_argument("--profiling", type=_bool, default=True)
    g.add_argument("--contention-profiling", type=_bool, default=False, help="accepted")
    g.add_argument("--kube-api-qps", type=float, default=20.0)
    g.add_argument("--kube-api-burst", type=int, default=30)
    g.add_argument("--kube-api-content-type", default="application/vnd.kubernetes.protobuf",
                   help="accepted; the client speaks JSON")
    g.add_argument("--controller-start-interval", default="0s")
    g.add_argument("--min-resync-period", default="12h", help="accepted; informers resync on watch restarts")
    g = ap.add_argument_group("controller workers")
    for name, d in (("deployment", 5), ("replicaset", 5), ("rc", 5), ("endpoint", 5), ("gc", 20), ("namespace", 10),
                    ("resource-quota", 5), ("service", 1), ("serviceaccount-token", 5)):
        g.add_argument(f"--concurrent-{name}-syncs", type=int, default=d)
    g = ap.add_argument_group("controller settings")
    g.add_argument("--horizontal-pod-autoscaler-upscale-delay", default="3m")
    g.add_argument("--horizontal-pod-autoscaler-downscale-delay", default="5m")
    g.add_argument("--horizontal-pod-autoscaler-tolerance", type=float, default=0.1)
    g.add_argument("--horizontal-pod-autoscaler-use-rest-clients", type=_bool, default=True,
                   help="accepted; metrics always come through the metrics API")
    g.add_argument("--experimental-cluster-signing-duration", default="8760h")
    g.add_argument("--enable-garbage-collector", type=_bool, default=True)
    g.add_argument("--enable-hostpath-provisioner", type=_bool, default=False,
                   help="dynamic hostPath volumes under /tmp/hostpath_pv (single-node testing)")
    g.add_argument("--enable-dynamic-provisioning", type=_bool, default=True, help="accepted")
    g.add_argument("--service-cluster-ip-range", default="", help="accepted")
    g.add_argument("--cidr-allocator-type", default="RangeAllocator", choices=["RangeAllocator", "CloudAllocator"])
    g.add_argument("--cluster-name", default="kubernetes")
    for f in ("--deployment-controller-sync-period", "--namespace-sync-period", "--pvclaimbinder-sync-period",
              "--resource-quota-sync-period", "--service-sync-period", "--node-sync-period",
              "--attach-detach-reconcile-sync-period"):
        g.add_argument(f, default="", help="accepted; controllers resync from watch events")
    g.add_argument("--disable-attach-detach-reconcile-sync", type=_bool, default=False, help="accepted")
    g.add_argument("--flex-volume-plugin-dir", default="/usr/libexec/kubernetes/kubelet-plugins/volume/exec/",
                   help="accepted (FlexVolume attach runs in the kubelet)")
    g.add_argument("--use-service-account-credentials", type=_bool, default=False,
                   help="run each controller as its own kube-system service account "
                        "(bound to its system:controller:<name> role)")
    for f in ("--pv-recycler-pod-template-filepath-nfs", "--pv-recycler-pod-template-filepath-hostpath"):
        g.add_argument(f, default="", help="accepted")
    for f in ("--pv-recycler-minimum-timeout-nfs", "--pv-recycler-increment-timeout-nfs",
              "--pv-recycler-minimum-timeout-hostpath", "--pv-recycler-timeout-increment-hostpath"):
        g.add_argument(f, type=int, default=0, help="accepted")
    g = ap.add_argument_group("no-ops kept for command-line compatibility")
    g.add_argument("--cloud-provider", default="")
    g.add_argument("--cloud-config", default="")
    g.add_argument("--allow-untagged-cloud", type=_bool, default=False)
    g.add_argument("--insecure-experimental-approve-all-kubelet-csrs-for-group", default="")
    g.add_argument("--deleting-pods-qps", type=float, default=0.1)
    g.add_argument("--deleting-pods-burst", type=int, default=0)
    g.add_argument("--register-retry-count", type=int, default=10)


if __name__ == "__main__":
    main()
