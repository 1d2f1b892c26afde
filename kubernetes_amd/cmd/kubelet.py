"""kubelet entry point (reference: cmd/kubelet/app/server.go:98-777)."""
from __future__ import annotations

import argparse
import os

from ..client.rest import Client
from ..deviceplugin import api
from ..kubelet.devicemanager.manager import ManagerImpl, ManagerStub
from ..kubelet.kubelet import Kubelet
from ..kubelet.runtime.process import ProcessRuntime
from ..kubelet.runtime.stub import StubRuntime
from ..utils.features import DefaultFeatureGate
from ._common import run_until_signal, setup_logging


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
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    setup_logging(a.v)
    DefaultFeatureGate.set(a.feature_gates)

    async def start():
        if a.bootstrap_kubeconfig and a.kubeconfig and not os.path.exists(a.kubeconfig):
            from ..kubelet.certificate import bootstrap_client_certificate
            await bootstrap_client_certificate(a.bootstrap_kubeconfig, a.kubeconfig, a.hostname_override,
                                               os.path.join(a.root_dir, "pki"))
        if a.kubeconfig:
            from ..client.clientcmd import client_from
            client = client_from(a.kubeconfig, max_conns=32)
        else:
            client = Client(a.master or "http://127.0.0.1:8080", token=a.token, max_conns=32)
        pdir = a.device_plugins_dir or os.path.join(a.root_dir, "device-plugin", "plugins")
        dm = ManagerImpl(pdir) if DefaultFeatureGate("DevicePlugins") else ManagerStub()
        if a.container_runtime == "remote":
            from ..cri.remote import RemoteRuntime
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
        image_gc = {"capacity_bytes": cap, "high": a.image_gc_high_threshold, "low": a.image_gc_low_threshold} if cap else None
        labels = dict(kv.split("=", 1) for kv in a.node_labels.split(",") if "=" in kv)
        from ..kubelet import network as net
        plugin = net.new_plugin(a.network_plugin, os.path.join(a.root_dir, "network"), a.cni_conf_dir, a.cni_bin_dir)
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
        base = dict(pods=a.max_pods, node_status_update_frequency=a.node_status_update_frequency,
                    cpu_manager_policy=a.cpu_manager_policy, eviction_hard=a.eviction_hard, dns=dns,
                    pod_manifest_path=a.pod_manifest_path, container_gc=container_gc,
                    bootstrap_checkpoint_path=a.bootstrap_checkpoint_path, volume_plugin_dir=a.volume_plugin_dir,
                    manifest_url=a.manifest_url,
                    manifest_url_headers=dict(h.split(":", 1) for h in a.manifest_url_header if ":" in h),
                    kube_reserved=dict(kv.split("=", 1) for kv in a.kube_reserved.split(",") if "=" in kv),
                    system_reserved=dict(kv.split("=", 1) for kv in a.system_reserved.split(",") if "=" in kv),
                    event_qps=a.event_qps, event_burst=a.event_burst)
        if not a.anonymous_auth or a.authentication_token_webhook or a.authorization_mode != "AlwaysAllow":
            from ..kubelet.server_auth import KubeletAuth
            base["auth"] = KubeletAuth(client, a.hostname_override, a.anonymous_auth,
                                       a.authentication_token_webhook, a.authorization_mode)
        base.update(extra)
        kl = Kubelet(client, a.hostname_override, rt, dm, labels=labels,
                     http_port=a.port, address=a.address, root_dir=a.root_dir, reserved_cpus=a.reserved_cpus,
                     image_gc=image_gc, network_plugin=plugin, hostports=hostports,
                     cgroup_root=a.cgroup_root if a.cgroups_per_qos else None,
                     container_log_dir=a.container_log_dir or None,
                     allowed_unsafe_sysctls=[x for x in a.experimental_allowed_unsafe_sysctls.split(",") if x], **base)
        await kl.run()
        if a.rotate_certificates and a.kubeconfig:
            import asyncio
            from ..kubelet.certificate import CertificateRotator
            rot = CertificateRotator(a.kubeconfig, a.hostname_override, os.path.join(a.root_dir, "pki"), client)
            kl._tasks.append(asyncio.ensure_future(rot.run()))
        print(f"kubelet {a.hostname_override} running (runtime={rt.name}, plugins={pdir}, port={kl.http_port})", flush=True)
        return kl

    run_until_signal(start)


if __name__ == "__main__":
    main()
