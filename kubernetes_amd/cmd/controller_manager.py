"""kube-controller-manager entry point (reference: cmd/kube-controller-manager/app/controllermanager.go:106)."""
from __future__ import annotations

import argparse

from ..client.rest import Client
from ..controllers.manager import CONTROLLERS, ControllerManager
from ._common import check_unsupported, deprecated_noop, run_until_signal, setup_logging, unsupported


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
    check_unsupported(ap, a)
    setup_logging(a.v)
    if a.cloud_provider:
        raise SystemExit(f"kube-controller-manager: --cloud-provider={a.cloud_provider}: cloud providers are out of "
                         "scope here (LoadBalancers come from --loadbalancer-ip-range)")
    from ..utils.features import DefaultFeatureGate
    DefaultFeatureGate.set(a.feature_gates)

    async def start():
        if a.kubeconfig:
            from ..client.clientcmd import client_from
            client = client_from(a.kubeconfig, max_conns=64, qps=a.kube_api_qps, burst=a.kube_api_burst,
                                 content_type=a.kube_api_content_type)
        else:
            client = Client(a.master or "http://127.0.0.1:8080", max_conns=64, qps=a.kube_api_qps, burst=a.kube_api_burst,
                            content_type=a.kube_api_content_type)
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
        opts["persistentvolume-binder"] = {"enable_dynamic_provisioning": a.enable_dynamic_provisioning}
        if a.enable_hostpath_provisioner:
            opts["persistentvolume-binder"]["hostpath_root"] = "/tmp/hostpath_pv"
        opts["nodeipam"]["service_cluster_ip_range"] = a.service_cluster_ip_range
        resync = {ctl: _dur(getattr(a, f[2:].replace("-", "_"))) for f, (ctl, _) in RESYNC_FLAGS.items()}
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
                              qps=a.kube_api_qps, burst=a.kube_api_burst, content_type=a.kube_api_content_type)
        if a.contention_profiling and a.profiling:
            from ..utils.profiling import enable_contention_profiling
            enable_contention_profiling()
        cm = await ControllerManager(client, enabled, opts, workers=workers,
                                     start_interval=_dur(a.controller_start_interval),
                                     sa_client_factory=sa_factory, resync=_dur(a.min_resync_period),
                                     resync_periods=resync,
                                     attach_detach_reconcile=not a.disable_attach_detach_reconcile_sync).start()
        health.metrics = cm
        return cm

    run_until_signal(start)


def _dur(v):
    from ..kubelet.eviction import parse_duration
    v = str(v).strip()
    return float(v) if v.replace(".", "", 1).isdigit() else parse_duration(v)


def _bool(v):
    return str(v).lower() not in ("false", "0", "no")


# flag -> (controller, reference default)
RESYNC_FLAGS = {"--deployment-controller-sync-period": ("deployment", "30s"),
                "--namespace-sync-period": ("namespace", "5m"),
                "--pvclaimbinder-sync-period": ("persistentvolume-binder", "15s"),
                "--resource-quota-sync-period": ("resourcequota", "5m"),
                "--service-sync-period": ("service", "5m"),
                "--attach-detach-reconcile-sync-period": ("attachdetach", "1m")}


def _reference_flags(ap):
    """The rest of kube-controller-manager's flags (cmd/kube-controller-manager/app/options)."""
    g = ap.add_argument_group("serving")
    g.add_argument("--port", type=int, default=10252, help="/healthz, /metrics, /configz (0 = off)")
    g.add_argument("--address", default="0.0.0.0")
    g.add_argument("--profiling", type=_bool, default=True)
    g.add_argument("--contention-profiling", type=_bool, default=False,
                   help="sample where the event loop blocks, served at /debug/pprof/block (with --profiling)")
    g.add_argument("--kube-api-qps", type=float, default=20.0)
    g.add_argument("--kube-api-burst", type=int, default=30)
    g.add_argument("--kube-api-content-type", default="application/vnd.kubernetes.protobuf",
                   choices=["application/json", "application/vnd.kubernetes.protobuf"],
                   help="wire format of API requests and watch streams (reference default protobuf, "
                         "`pkg/apis/componentconfig/v1alpha1/defaults.go:75`: protobuf bodies and "
                         "length-delimited protobuf watch frames, decoded natively)")
    g.add_argument("--controller-start-interval", default="0s")
    g.add_argument("--min-resync-period", default="12h",
                   help="the shared informers re-deliver every cached object every [min, 2*min)")
    g = ap.add_argument_group("controller workers")
    for name, d in (("deployment", 5), ("replicaset", 5), ("rc", 5), ("endpoint", 5), ("gc", 20), ("namespace", 10),
                    ("resource-quota", 5), ("service", 1), ("serviceaccount-token", 5)):
        g.add_argument(f"--concurrent-{name}-syncs", type=int, default=d)
    g = ap.add_argument_group("controller settings")
    g.add_argument("--horizontal-pod-autoscaler-upscale-delay", default="3m")
    g.add_argument("--horizontal-pod-autoscaler-downscale-delay", default="5m")
    g.add_argument("--horizontal-pod-autoscaler-tolerance", type=float, default=0.1)
    unsupported(g, "--horizontal-pod-autoscaler-use-rest-clients", True, _bool,
                "metrics always come through the resource metrics API (the Heapster client is not built)")
    g.add_argument("--experimental-cluster-signing-duration", default="8760h")
    g.add_argument("--enable-garbage-collector", type=_bool, default=True)
    g.add_argument("--enable-hostpath-provisioner", type=_bool, default=False,
                   help="dynamic hostPath volumes under /tmp/hostpath_pv (single-node testing)")
    g.add_argument("--enable-dynamic-provisioning", type=_bool, default=True,
                   help="false: claims only bind to existing PersistentVolumes")
    g.add_argument("--service-cluster-ip-range", default="",
                   help="node CIDR allocation (--allocate-node-cidrs) never hands out blocks overlapping it")
    unsupported(g, "--cidr-allocator-type", "RangeAllocator", str, "CloudAllocator needs a cloud provider")
    unsupported(g, "--cluster-name", "kubernetes", str, "it names cloud resources; cloud providers are out of scope")
    for f, d in RESYNC_FLAGS.items():
        g.add_argument(f, default=d[1], help=f"period of the {d[0]} controller's full resync (0 = only on events)")
    deprecated_noop(g, "--node-sync-period", "0s", str, "options.go:158-161")
    g.add_argument("--disable-attach-detach-reconcile-sync", type=_bool, default=False,
                   help="the attach/detach controller reconciles on events only")
    unsupported(g, "--flex-volume-plugin-dir", "/usr/libexec/kubernetes/kubelet-plugins/volume/exec/", str,
                "FlexVolume attach/detach runs in the kubelet, not the controller manager")
    g.add_argument("--use-service-account-credentials", type=_bool, default=False,
                   help="run each controller as its own kube-system service account "
                        "(bound to its system:controller:<name> role)")
    why = "volumes are recycled in-process by the PV controller (no recycler pod)"
    for f in ("--pv-recycler-pod-template-filepath-nfs", "--pv-recycler-pod-template-filepath-hostpath"):
        unsupported(g, f, "", str, why)
    for f, d in (("--pv-recycler-minimum-timeout-nfs", 300), ("--pv-recycler-increment-timeout-nfs", 30),
                 ("--pv-recycler-minimum-timeout-hostpath", 60), ("--pv-recycler-timeout-increment-hostpath", 30)):
        unsupported(g, f, d, int, why)
    g = ap.add_argument_group("cloud provider and deprecated flags")
    g.add_argument("--cloud-provider", default="", help="'' only: cloud providers are out of scope")
    unsupported(g, "--cloud-config", "", str, "cloud providers are out of scope")
    unsupported(g, "--allow-untagged-cloud", False, _bool, "cloud providers are out of scope")
    deprecated_noop(g, "--insecure-experimental-approve-all-kubelet-csrs-for-group", "", str, "options.go:203-204")
    deprecated_noop(g, "--deleting-pods-qps", 0.1, float, "options.go:183-184")
    deprecated_noop(g, "--deleting-pods-burst", 0, int, "options.go:185-186")
    deprecated_noop(g, "--register-retry-count", 10, int, "options.go:187-189")


if __name__ == "__main__":
    main()
