"""kubelet entry point (reference: cmd/kubelet/app/server.go:98-777)."""
from __future__ import annotations

import argparse
import logging
import os
import sys

from ..client.rest import Client
from ..deviceplugin import api
from ..kubelet.devicemanager.manager import ManagerImpl, ManagerStub
from ..kubelet.kubelet import Kubelet
from ..kubelet.runtime.process import ProcessRuntime
from ..kubelet.runtime.stub import StubRuntime
from ..utils.features import DefaultFeatureGate
from ._common import check_unsupported, deprecated_noop, run_until_signal, setup_logging, unsupported


def main(argv=None):
    ap = argparse.ArgumentParser("kubelet")
    ap.add_argument("--api-servers", "--master", dest="master", default=None)
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--bootstrap-kubeconfig", default=None,
                    help="TLS bootstrap: obtain a client certificate via a CSR with these credentials, "
                         "then write --kubeconfig")
    ap.add_argument("--hostname-override", default=os.uname().nodename)
    ap.add_argument("--root-dir", default="/var/lib/kubelet")
    ap.add_argument("--device-plugins-dir", default=None)
    ap.add_argument("--container-runtime", default="process", choices=["process", "stub", "remote"])
    ap.add_argument("--container-runtime-endpoint", default="unix:///var/run/kamd-cri.sock",
                    help="CRI endpoint for --container-runtime=remote (kamd-cri or any v1alpha1 CRI runtime)")
    ap.add_argument("--runtime-request-timeout", type=float, default=120.0)
    ap.add_argument("--pleg-relist-period", type=float, default=1.0, help="generic PLEG relist period (remote runtime)")
    ap.add_argument("--image-gc-high-threshold", type=int, default=85)
    ap.add_argument("--image-gc-low-threshold", type=int, default=80)
    ap.add_argument("--image-service", default="oci", choices=["oci", "builtin"],
                    help="process runtime images: 'oci' = OCI store + registry pulls (overlay root "
                         "filesystems under isolation), 'builtin' = built-in images / host root only")
    ap.add_argument("--insecure-registry", action="append", default=[],
                    help="registry host[:port] reached over plain HTTP (loopback registries always are)")
    ap.add_argument("--image-fs-capacity", default="0", help="image filesystem size for image GC (e.g. 100Gi; 0 = off)")
    ap.add_argument("--port", type=int, default=10250)
    ap.add_argument("--address", default="127.0.0.1")
    ap.add_argument("--node-status-update-frequency", type=float, default=10.0)
    ap.add_argument("--max-pods", type=int, default=110)
    ap.add_argument("--node-labels", default="")
    ap.add_argument("--feature-gates", default="")
    ap.add_argument("--token", default=None)
    ap.add_argument("--cpu-manager-policy", default="none", choices=["none", "static"])
    ap.add_argument("--reserved-cpus", type=int, default=1, help="CPUs kept out of the static policy's exclusive pool")
    ap.add_argument("--pod-manifest-path", default=None, help="directory of static pod manifests (JSON/YAML)")
    ap.add_argument("--eviction-hard", default="memory.available<100Mi",
                    help="hard eviction thresholds, e.g. memory.available<100Mi,nodefs.available<5%%")
    ap.add_argument("--network-plugin", default="", choices=["", "cni", "kubenet"])
    ap.add_argument("--cni-conf-dir", default="/etc/cni/net.d")
    ap.add_argument("--cni-bin-dir", default="/opt/cni/bin")
    ap.add_argument("--pod-cidr", default=None, help="standalone mode: pod CIDR when no API node spec provides one")
    ap.add_argument("--cluster-dns", default="", help="comma-separated DNS server IPs for ClusterFirst pods")
    ap.add_argument("--cluster-domain", default="cluster.local")
    ap.add_argument("--resolv-conf", default="/etc/resolv.conf")
    ap.add_argument("--hostport-holder", type=lambda v: v.lower() != "false", default=True,
                    help="open and hold the host ports of pods in their own network namespace")
    ap.add_argument("--minimum-container-ttl-duration", type=float, default=0.0)
    ap.add_argument("--maximum-dead-containers-per-container", type=int, default=1)
    ap.add_argument("--maximum-dead-containers", type=int, default=-1)
    ap.add_argument("--bootstrap-checkpoint-path", default=None,
                    help="checkpoint pods annotated node.kubernetes.io/bootstrap-checkpoint=true here")
    ap.add_argument("--volume-plugin-dir", default="/usr/libexec/kubernetes/kubelet-plugins/volume/exec",
                    help="FlexVolume driver directory (<vendor>~<driver>/<driver>)")
    ap.add_argument("--manifest-url", default=None, help="HTTP pod source (polled every 20 s)")
    ap.add_argument("--manifest-url-header", action="append", default=[], help="key:value header for --manifest-url")
    ap.add_argument("--kube-reserved", default="", help="e.g. cpu=1,memory=2Gi (subtracted from allocatable)")
    ap.add_argument("--system-reserved", default="", help="e.g. cpu=500m,memory=1Gi")
    ap.add_argument("--rotate-certificates", action="store_true",
                    help="rotate the kubelet client certificate (CSR) as it approaches expiry")
    ap.add_argument("--config", default=None, help="KubeletConfiguration file (kubeletconfig/v1alpha1)")
    ap.add_argument("--dynamic-config-dir", default=None, help="enable Dynamic Kubelet Config; checkpoints live here")
    ap.add_argument("--cgroups-per-qos", type=lambda v: v.lower() != "false", default=False,
                    help="create the QoS and pod cgroup hierarchy under --cgroup-root")
    ap.add_argument("--cgroup-root", default="/sys/fs/cgroup/kubepods.slice",
                    help="cgroup v2 directory delegated to the kubelet (with --cgroups-per-qos)")
    ap.add_argument("--experimental-allowed-unsafe-sysctls", default="",
                    help="comma-separated unsafe sysctls or prefix* patterns pods may request")
    ap.add_argument("--container-log-dir", default="/var/log/containers",
                    help="where <pod>_<namespace>_<container>-<id>.log symlinks for logging agents go ('' = off)")
    ap.add_argument("--anonymous-auth", type=lambda v: v.lower() != "false", default=True,
                    help="allow anonymous requests to the kubelet API (system:anonymous)")
    ap.add_argument("--authentication-token-webhook", action="store_true",
                    help="authenticate bearer tokens with TokenReviews against the API server")
    ap.add_argument("--authorization-mode", default="AlwaysAllow", choices=["AlwaysAllow", "Webhook"],
                    help="Webhook: SubjectAccessReview per request (resource nodes, subresource by path)")
    ap.add_argument("--event-qps", type=float, default=5.0, help="limit event creations per second (0 = unlimited)")
    ap.add_argument("--event-burst", type=int, default=10, help="burst of event creations (with --event-qps > 0)")
    _reference_flags(ap)
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    check_unsupported(ap, a)
    enforce = {x.strip() for x in a.enforce_node_allocatable.split(",") if x.strip()}
    if not enforce <= {"pods", "none"} or ("none" in enforce and len(enforce) > 1):
        ap.error(f"--enforce-node-allocatable={a.enforce_node_allocatable!r}: only 'pods' or 'none' are supported "
                 "(system-reserved/kube-reserved need their cgroups, which this kubelet does not manage)")
    setup_logging(a.v)
    DefaultFeatureGate.set(a.feature_gates)
    _host_checks(a)
    if a.node_ip:
        # setNodeAddress -> validateNodeIP: an unusable --node-ip fails here, not on every status
        from ..kubelet.network import validate_node_ip
        try:
            validate_node_ip(a.node_ip)
        except ValueError as e:
            ap.error(f"failed to validate nodeIP: {e}")

    async def start():
        if a.contention_profiling:
            from ..utils.profiling import enable_contention_profiling
            enable_contention_profiling()
        if a.experimental_bootstrap_kubeconfig and not a.bootstrap_kubeconfig:
            a.bootstrap_kubeconfig = a.experimental_bootstrap_kubeconfig
        if a.bootstrap_kubeconfig and a.kubeconfig and not os.path.exists(a.kubeconfig):
            from ..kubelet.certificate import bootstrap_client_certificate
            await bootstrap_client_certificate(a.bootstrap_kubeconfig, a.kubeconfig, a.hostname_override,
                                               os.path.join(a.root_dir, "pki"))
        if a.kubeconfig:
            from ..client.clientcmd import client_from
            client = client_from(a.kubeconfig, max_conns=32, qps=a.kube_api_qps, burst=a.kube_api_burst,
                                 content_type=a.kube_api_content_type)
        else:
            client = Client(a.master or "http://127.0.0.1:8080", token=a.token, max_conns=32, qps=a.kube_api_qps,
                            burst=a.kube_api_burst, content_type=a.kube_api_content_type)
        pdir = a.device_plugins_dir or os.path.join(a.root_dir, "device-plugin", "plugins")
        dm = ManagerImpl(pdir) if DefaultFeatureGate("DevicePlugins") else ManagerStub()
        if a.container_runtime == "remote":
            from ..cri.remote import RemoteRuntime
            if a.image_service_endpoint and a.image_service_endpoint != a.container_runtime_endpoint:
                print("kubelet: --image-service-endpoint must equal --container-runtime-endpoint here "
                      "(one CRI server serves both services)", file=sys.stderr)
                sys.exit(1)
            rt = await RemoteRuntime(a.container_runtime_endpoint, a.runtime_request_timeout, a.pleg_relist_period).connect()
        elif a.container_runtime == "process":
            images = None
            if a.image_service == "oci":
                from ..images.service import node_image_service
                images = node_image_service(os.path.join(a.root_dir, "images"), True, a.insecure_registry)
            rt = ProcessRuntime(os.path.join(a.root_dir, "runtime"), images=images)
        else:
            rt = StubRuntime()
        from ..api.quantity import parse_quantity
        cap = int(parse_quantity(a.image_fs_capacity).value) if a.image_fs_capacity not in ("", "0") else 0
        image_gc = {"capacity_bytes": cap, "high": a.image_gc_high_threshold, "low": a.image_gc_low_threshold,
                    "min_age": _duration(a.minimum_image_ttl_duration)} if cap else None
        labels = dict(kv.split("=", 1) for kv in a.node_labels.split(",") if "=" in kv)
        from ..kubelet import network as net
        plugin = net.new_plugin(a.network_plugin, os.path.join(a.root_dir, "network"), a.cni_conf_dir, a.cni_bin_dir,
                                hairpin_mode=a.hairpin_mode, mtu=getattr(a, "network_plugin_mtu", 0) or 1460)
        if a.pod_cidr:
            plugin.set_pod_cidr(a.pod_cidr)
        dns = net.DNSConfigurer(a.cluster_dns.split(","), a.cluster_domain, a.resolv_conf)
        hostports = net.HostportManager(a.hostport_holder)
        container_gc = {"min_age": a.minimum_container_ttl_duration,
                        "max_per_pod_container": a.maximum_dead_containers_per_container,
                        "max_containers": a.maximum_dead_containers}
        extra = {}
        if a.config:
            from ..kubelet.kubeletconfig import load, to_kwargs
            with open(a.config) as f:
                extra = to_kwargs(load(f.read()))
        if a.dynamic_config_dir:
            from ..kubelet.kubeletconfig import startup_checkpoint, to_kwargs
            ck = startup_checkpoint(a.dynamic_config_dir)   # restart path: start on the assigned checkpoint
            if ck is not None:
                extra.update(to_kwargs(ck))
            extra["dynamic_config_dir"] = a.dynamic_config_dir
        max_pods = a.max_pods
        if a.pods_per_core > 0:
            max_pods = min(max_pods, a.pods_per_core * (os.cpu_count() or 1))
        base = dict(pods=max_pods, node_status_update_frequency=a.node_status_update_frequency,
                    cpu_manager_policy=a.cpu_manager_policy, eviction_hard=a.eviction_hard, dns=dns,
                    pod_manifest_path=a.pod_manifest_path, container_gc=container_gc,
                    bootstrap_checkpoint_path=a.bootstrap_checkpoint_path, volume_plugin_dir=a.volume_plugin_dir,
                    manifest_url=a.manifest_url,
                    manifest_url_headers=dict(h.split(":", 1) for h in a.manifest_url_header if ":" in h),
                    kube_reserved=dict(kv.split("=", 1) for kv in a.kube_reserved.split(",") if "=" in kv),
                    system_reserved=dict(kv.split("=", 1) for kv in a.system_reserved.split(",") if "=" in kv),
                    event_qps=a.event_qps, event_burst=a.event_burst,
                    tls=_tls(a), read_only_port=a.read_only_port or None,
                    healthz_port=a.healthz_port or None, healthz_address=a.healthz_bind_address,
                    debugging_handlers=a.enable_debugging_handlers, node_ip=a.node_ip or None,
                    register_taints=_taints(a.register_with_taints), register_schedulable=a.register_schedulable,
                    provider_id=a.provider_id, allow_privileged=a.allow_privileged,
                    host_sources={"hostNetwork": _sources(a.host_network_sources), "hostPID": _sources(a.host_pid_sources),
                                  "hostIPC": _sources(a.host_ipc_sources)},
                    eviction_soft=a.eviction_soft or None, eviction_soft_grace_period=a.eviction_soft_grace_period,
                    eviction_minimum_reclaim=a.eviction_minimum_reclaim,
                    eviction_max_pod_grace_period=a.eviction_max_pod_grace_period,
                    eviction_pressure_transition_period=_duration(a.eviction_pressure_transition_period),
                    allocatable_ignore_eviction=a.experimental_allocatable_ignore_eviction,
                    serialize_image_pulls=a.serialize_image_pulls, registry_qps=a.registry_qps,
                    registry_burst=a.registry_burst, file_check_frequency=_duration(a.file_check_frequency), sync_frequency=_duration(a.sync_frequency),
                    cpu_cfs_quota=a.cpu_cfs_quota, enforce_node_allocatable="none" not in enforce,
                    http_check_frequency=_duration(a.http_check_frequency), register=a.register_node)
        if not a.anonymous_auth or a.authentication_token_webhook or a.authorization_mode != "AlwaysAllow" or a.client_ca_file:
            from ..kubelet.server_auth import KubeletAuth
            base["auth"] = KubeletAuth(client, a.hostname_override, a.anonymous_auth,
                                       a.authentication_token_webhook, a.authorization_mode,
                                       authn_ttl=_duration(a.authentication_token_webhook_cache_ttl),
                                       authz_allowed_ttl=_duration(a.authorization_webhook_cache_authorized_ttl),
                                       authz_denied_ttl=_duration(a.authorization_webhook_cache_unauthorized_ttl))
        base.update(extra)
        kl = Kubelet(client, a.hostname_override, rt, dm, labels=labels,
                     http_port=a.port if a.enable_server else None, address=a.address, root_dir=a.root_dir, reserved_cpus=a.reserved_cpus,
                     image_gc=image_gc, network_plugin=plugin, hostports=hostports,
                     cgroup_root=a.cgroup_root if a.cgroups_per_qos else None,
                     container_log_dir=a.container_log_dir or None,
                     master_service_namespace=a.master_service_namespace,
                     allowed_unsafe_sysctls=[x for x in a.experimental_allowed_unsafe_sysctls.split(",") if x], **base)
        await kl.run()
        if a.rotate_certificates and a.kubeconfig:
            import asyncio
            from ..kubelet.certificate import CertificateRotator
            rot = CertificateRotator(a.kubeconfig, a.hostname_override, os.path.join(a.root_dir, "pki"), client)
            kl._tasks.append(asyncio.ensure_future(rot.run()))
        print(f"kubelet {a.hostname_override} running (runtime={rt.name}, plugins={pdir}, port={kl.http_port}, "
              f"{'https' if kl.tls else 'http'})", flush=True)
        return kl

    run_until_signal(start)


def _duration(v) -> float:
    from ..kubelet.eviction import parse_duration
    if isinstance(v, (int, float)):
        return float(v)
    v = str(v).strip()
    return float(v) if v.replace(".", "", 1).isdigit() else parse_duration(v)


def _sources(v):
    return [x.strip() for x in (v or "").split(",") if x.strip()]


def _taints(spec):
    """`key=value:Effect` / `key:Effect`, comma separated (`--register-with-taints`)."""
    out = []
    for part in _sources(spec):
        kv, _, effect = part.rpartition(":")
        if effect not in ("NoSchedule", "PreferNoSchedule", "NoExecute") or not kv:
            raise SystemExit(f"kubelet: invalid taint {part!r} (want key=value:Effect)")
        key, _, value = kv.partition("=")
        t = {"key": key, "effect": effect}
        if value:
            t["value"] = value
        out.append(t)
    return out


def _tls(a):
    """--tls-cert-file/--tls-private-key-file, else a self-signed pair in --cert-dir
    (InitializeTLS); --client-ca-file enables x509 client authentication."""
    if not a.enable_server:
        return None
    if a.tls_cert_file:
        return (a.tls_cert_file, a.tls_private_key_file or a.tls_cert_file, a.client_ca_file)
    from ..utils.tlsutil import self_signed_serving_cert
    cert_dir = a.cert_dir or os.path.join(a.root_dir, "pki")
    cert, key = self_signed_serving_cert(cert_dir, a.hostname_override, [a.node_ip, a.address])
    return (cert, key, a.client_ca_file)


def _host_checks(a):
    from ..kubelet import hostchecks as H
    if a.cloud_provider not in ("", "external"):
        print(f"kubelet: --cloud-provider={a.cloud_provider}: cloud providers are out of scope here "
              "(use '' or 'external')", file=sys.stderr)
        sys.exit(1)
    if a.cgroup_driver not in ("cgroupfs", "systemd"):
        print(f"kubelet: unknown --cgroup-driver {a.cgroup_driver!r}", file=sys.stderr)
        sys.exit(1)
    if a.runonce:
        print("kubelet: --runonce is not supported (run the static pods with a normal kubelet)", file=sys.stderr)
        sys.exit(1)
    if a.cadvisor_port:
        logging.getLogger("kubelet").warning("--cadvisor-port: container stats are served by /stats/summary; "
                                             "no standalone cAdvisor endpoint is started")
    try:
        H.check_swap(a.fail_swap_on and a.experimental_fail_swap_on)
        H.check_kernel_defaults(a.protect_kernel_defaults)
    except H.HostCheckError as e:
        print(f"kubelet: {e}", file=sys.stderr)
        sys.exit(1)
    H.set_max_open_files(a.max_open_files)
    H.set_oom_score_adj(a.oom_score_adj)
    if a.lock_file:
        lk = H.LockFile(a.lock_file).acquire()
        if a.exit_on_lock_contention:
            lk.watch_contention(lambda: os._exit(0))


def _bool(v):
    return str(v).lower() not in ("false", "0", "no")


def _reference_flags(ap):
    """The rest of the reference kubelet's flags (cmd/kubelet/app/options/options.go). Flags whose
    subsystem does not exist here are accepted and documented as such."""
    g = ap.add_argument_group("serving")
    g.add_argument("--tls-cert-file", default=None, help="x509 serving certificate (default: self-signed in --cert-dir)")
    g.add_argument("--tls-private-key-file", default=None)
    g.add_argument("--cert-dir", default=None, help="where the self-signed serving pair goes (default <root-dir>/pki)")
    g.add_argument("--client-ca-file", default=None, help="authenticate API clients by x509 certificates of this CA")
    g.add_argument("--read-only-port", type=int, default=0,
                   help="unauthenticated read-only port (no debugging handlers); 0 = off (the reference defaults to 10255)")
    g.add_argument("--healthz-port", type=int, default=0, help="localhost /healthz port; 0 = off (reference: 10248)")
    g.add_argument("--healthz-bind-address", default="127.0.0.1")
    g.add_argument("--enable-server", type=_bool, default=True)
    g.add_argument("--enable-debugging-handlers", type=_bool, default=True,
                   help="exec/attach/port-forward/run/logs/containerLogs/pprof/configz on the server")
    g.add_argument("--authentication-token-webhook-cache-ttl", default="2m")
    g.add_argument("--authorization-webhook-cache-authorized-ttl", default="5m")
    g.add_argument("--authorization-webhook-cache-unauthorized-ttl", default="30s")
    unsupported(g, "--streaming-connection-idle-timeout", "4h", str, "exec/attach/port-forward streams end when "
                "either side closes; no idle timer")
    g = ap.add_argument_group("registration")
    g.add_argument("--register-node", type=_bool, default=True)
    g.add_argument("--register-with-taints", default="", help="key=value:Effect,... applied at registration")
    g.add_argument("--register-schedulable", type=_bool, default=True)
    g.add_argument("--node-ip", default="", help="the node's InternalIP (default: --address)")
    g.add_argument("--provider-id", default="")
    g.add_argument("--cloud-provider", default="", help="'' or 'external' (cloud providers are out of scope)")
    unsupported(g, "--cloud-config", "", str, "cloud providers are out of scope")
    g = ap.add_argument_group("admission")
    g.add_argument("--allow-privileged", type=_bool, default=False)
    g.add_argument("--host-network-sources", default="*", help="pod sources (api,file,http) allowed hostNetwork")
    g.add_argument("--host-pid-sources", default="*")
    g.add_argument("--host-ipc-sources", default="*")
    g.add_argument("--pods-per-core", type=int, default=0)
    g = ap.add_argument_group("eviction")
    g.add_argument("--eviction-soft", default="", help="e.g. memory.available<1.5Gi")
    g.add_argument("--eviction-soft-grace-period", default="", help="e.g. memory.available=1m30s")
    g.add_argument("--eviction-max-pod-grace-period", type=int, default=0)
    g.add_argument("--eviction-minimum-reclaim", default="", help="e.g. memory.available=0Mi,nodefs.available=500Mi")
    g.add_argument("--eviction-pressure-transition-period", default="5m")
    g.add_argument("--experimental-allocatable-ignore-eviction", type=_bool, default=False)
    g = ap.add_argument_group("images and pod sources")
    g.add_argument("--serialize-image-pulls", type=_bool, default=True)
    g.add_argument("--registry-qps", type=float, default=5.0)
    g.add_argument("--registry-burst", type=int, default=10)
    g.add_argument("--minimum-image-ttl-duration", default="2m")
    g.add_argument("--image-service-endpoint", default="")
    g.add_argument("--file-check-frequency", default="20s")
    g.add_argument("--http-check-frequency", default="20s")
    g.add_argument("--sync-frequency", default="1m",
                   help="period of the pod sync that re-projects configMap/secret/downwardAPI/projected volumes "
                        "(pod changes themselves resync on every watch event)")
    g = ap.add_argument_group("API client")
    g.add_argument("--kube-api-qps", type=float, default=5.0)
    g.add_argument("--kube-api-burst", type=int, default=10)
    g.add_argument("--kube-api-content-type", default="application/vnd.kubernetes.protobuf",
                   choices=["application/json", "application/vnd.kubernetes.protobuf"],
                   help="wire format of API requests and watch streams (reference default protobuf, "
                         "`pkg/apis/componentconfig/v1alpha1/defaults.go:75`: protobuf bodies and "
                         "length-delimited protobuf watch frames, decoded natively)")
    g.add_argument("--experimental-bootstrap-kubeconfig", default=None, help="deprecated alias of --bootstrap-kubeconfig")
    deprecated_noop(g, "--require-kubeconfig", False, _bool, "options.go:298")
    g = ap.add_argument_group("host")
    g.add_argument("--fail-swap-on", type=_bool, default=True)
    g.add_argument("--experimental-fail-swap-on", type=_bool, default=True, help="deprecated alias of --fail-swap-on")
    g.add_argument("--protect-kernel-defaults", type=_bool, default=False)
    g.add_argument("--max-open-files", type=int, default=1000000)
    g.add_argument("--oom-score-adj", type=int, default=-999)
    g.add_argument("--lock-file", default="")
    g.add_argument("--exit-on-lock-contention", type=_bool, default=False)
    g.add_argument("--cgroup-driver", default="cgroupfs", help="cgroupfs or systemd (both manage the cgroup v2 tree directly)")
    g.add_argument("--enforce-node-allocatable", default="pods",
                   help="'pods': node allocatable caps the kubepods cgroup (with --cgroups-per-qos); 'none': no cap")
    for f in ("--kubelet-cgroups", "--system-cgroups", "--kube-reserved-cgroup", "--system-reserved-cgroup"):
        unsupported(g, f, "", str, "system daemons are not moved into cgroups by this kubelet")
    g.add_argument("--cpu-cfs-quota", type=_bool, default=True,
                   help="enforce CPU limits with a CFS quota (cpu.max); false: limits only shape requests")
    unsupported(g, "--cpu-manager-reconcile-period", "10s", str, "CPU assignments are applied at container start")
    unsupported(g, "--experimental-qos-reserved", "", str, "alpha QOSReserved is not implemented")
    unsupported(g, "--seccomp-profile-root", "/var/lib/kubelet/seccomp", str,
                "localhost seccomp profiles are not applied by this runtime")
    g = ap.add_argument_group("networking")
    g.add_argument("--network-plugin-mtu", type=int, default=0, help="kubenet bridge MTU (0: 1460)")
    g.add_argument("--hairpin-mode", default="promiscuous-bridge", choices=["promiscuous-bridge", "hairpin-veth", "none"],
                   help="kubenet: bridge promiscuous mode, or hairpin on each pod's veth port")
    why = "the kubelet does not program KUBE-MARK-* iptables chains (kube-proxy owns the NAT rules)"
    unsupported(g, "--non-masquerade-cidr", "10.0.0.0/8", str, why)
    unsupported(g, "--make-iptables-util-chains", True, _bool, why)
    unsupported(g, "--iptables-masquerade-bit", 14, int, why)
    unsupported(g, "--iptables-drop-bit", 15, int, why)
    g = ap.add_argument_group("subsystems this kubelet does not have")
    unsupported(g, "--cadvisor-port", 0, int, "no embedded cAdvisor; stats come from the summary API")
    unsupported(g, "--chaos-chance", 0.0, float, "no fault-injecting client")
    for f, why in (("--containerized", "the kubelet runs on the host"),
                   ("--really-crash-for-testing", "test-only panic mode"),
                   ("--experimental-check-node-capabilities-before-mount", "mount utilities are not probed"),
                   ("--experimental-kernel-memcg-notification", "eviction polls memory; no memcg threshold events"),
                   ("--runonce", "run-once mode is not implemented")):
        unsupported(g, f, False, _bool, why)
    g.add_argument("--contention-profiling", type=_bool, default=False,
                   help="sample where the event loop blocks, served at /debug/pprof/block")
    deprecated_noop(g, "--enable-custom-metrics", False, _bool, "options.go:368")
    g.add_argument("--master-service-namespace", default="default",
                   help="the namespace whose kubernetes service is injected into every pod's environment")
    unsupported(g, "--keep-terminated-pod-volumes", False, _bool, "volumes of terminated pods are torn down")
    unsupported(g, "--enable-controller-attach-detach", True, _bool,
                "attach/detach is always the controller's (the kubelet only mounts)")
    for f, d in (("--experimental-mounter-path", ""), ("--init-config-dir", ""),
                 ("--volume-stats-agg-period", "1m")):
        unsupported(g, f, d, str, "not implemented by this kubelet")


if __name__ == "__main__":
    main()
