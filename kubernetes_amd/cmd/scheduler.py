"""kube-scheduler entry point (reference: plugin/cmd/kube-scheduler/app/server.go:320-552).

    python -m kubernetes_amd.cmd.scheduler --master URL                 # one scheduler
    python -m kubernetes_amd.cmd.scheduler --master URL --shards 4      # 4 parallel shards

`--shards N` makes this process a supervisor of N scheduler processes (`--shard-index i
--shard-count N`), each owning a hash partition of the pods and preferring a hash partition of
the nodes; bind conflicts between shards are resolved by the API server's device-claim guard
(see `kubernetes_amd/scheduler/scheduler.py`).
"""
from __future__ import annotations

import argparse
import asyncio
import signal
import subprocess
import sys
import time

from ..client.rest import Client
from ..scheduler.scheduler import Scheduler
from ..utils.features import DefaultFeatureGate
from ._common import run_until_signal, setup_logging
from ..utils.tasks import spawn


def _parser():
    ap = argparse.ArgumentParser("kube-scheduler")
    ap.add_argument("--feature-gates", default="", help="e.g. PodPriority=false (turns scheduler preemption off)")
    ap.add_argument("--master", default=None)
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--scheduler-name", default="default-scheduler")
    ap.add_argument("--policy-config-file", default=None, help="JSON Policy {predicates:[{name}], priorities:[{name,weight}]}")
    ap.add_argument("--percentage-of-nodes-to-score", type=int, default=100)
    ap.add_argument("--metrics-port", type=int, default=None)
    ap.add_argument("--no-events", action="store_true")
    ap.add_argument("--kube-api-qps", type=float, default=None)
    ap.add_argument("--leader-elect", action="store_true")
    ap.add_argument("--disable-preemption", action="store_true")
    ap.add_argument("--shards", type=int, default=1, help="run N parallel scheduler shard processes")
    ap.add_argument("--shard-index", type=int, default=0)
    ap.add_argument("--shard-count", type=int, default=1)
    ap.add_argument("--config", default=None, help="KubeSchedulerConfiguration file")
    ap.add_argument("--algorithm-provider", default=None, help="DefaultProvider | ClusterAutoscalerProvider")
    ap.add_argument("--policy-configmap", default=None, help="ConfigMap holding the Policy under policy.cfg")
    ap.add_argument("--policy-configmap-namespace", default="kube-system")
    ap.add_argument("--port", type=int, default=10251, help="/healthz and /metrics (0 = off; shard i uses port+i)")
    ap.add_argument("--address", default="0.0.0.0")
    ap.add_argument("--kube-api-burst", type=int, default=None)
    ap.add_argument("--kube-api-content-type", default="application/vnd.kubernetes.protobuf",
                    choices=["application/json", "application/vnd.kubernetes.protobuf"],
                    help="wire format of API requests and watch streams (reference default protobuf, "
                         "`pkg/apis/componentconfig/v1alpha1/defaults.go:75`: protobuf bodies and "
                         "length-delimited protobuf watch frames, decoded natively)")
    ap.add_argument("--lock-object-name", default="kube-scheduler")
    ap.add_argument("--lock-object-namespace", default="kube-system")
    ap.add_argument("--hard-pod-affinity-symmetric-weight", type=int, default=1,
                    help="score an existing pod's required pod affinity gives a matching incoming pod (0-100)")
    ap.add_argument("--failure-domains", default="kubernetes.io/hostname,failure-domain.beta.kubernetes.io/zone,"
                    "failure-domain.beta.kubernetes.io/region",
                    help="labels an empty topologyKey in a preferred pod (anti-)affinity term stands for "
                         "(deprecated in 1.9)")
    ap.add_argument("--use-legacy-policy-config", action="store_true",
                    help="read --policy-config-file even when --config is given")
    ap.add_argument("--profiling", default="true", help="serve /debug/pprof on the metrics port")
    ap.add_argument("--contention-profiling", default="false",
                    help="sample where the event loop blocks, served at /debug/pprof/block")
    ap.add_argument("-v", type=int, default=0)
    return ap


def _true(v):
    return str(v).lower() in ("true", "1", "yes")


def supervise(argv, n):
    """Run n shard processes; stop all when one exits or on SIGTERM/SIGINT."""
    base = [a for a in argv if not a.startswith("--shards")]
    if "--shards" in argv:
        i = argv.index("--shards")
        base = argv[:i] + argv[i + 2:]
    stopping = []
    signal.signal(signal.SIGTERM, lambda *_: stopping.append(1))
    signal.signal(signal.SIGINT, lambda *_: stopping.append(1))
    procs = [subprocess.Popen([sys.executable, "-m", "kubernetes_amd.cmd.scheduler", *base,
                               "--shard-index", str(i), "--shard-count", str(n)]) for i in range(n)]
    rc = 0
    try:
        while not stopping:
            if any(p.poll() is not None for p in procs):
                rc = 1
                break
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
    return rc


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    a = _parser().parse_args(argv)
    setup_logging(a.v)
    DefaultFeatureGate.set(a.feature_gates)
    if a.shards > 1:
        sys.exit(supervise(argv, a.shards))
    from ..scheduler import policy as SP
    if not 0 <= a.hard_pod_affinity_symmetric_weight <= 100:
        raise SystemExit("kube-scheduler: --hard-pod-affinity-symmetric-weight must be in 0..100")
    if a.metrics_port is None and a.port:
        a.metrics_port = a.port + a.shard_index
    legacy_policy = a.policy_config_file
    if a.config:
        with open(a.config) as f:
            cc = SP.load_component_config(f.read())
        src = cc.get("algorithmSource") or {}
        pol = src.get("policy") or {}
        a.algorithm_provider = src.get("provider") or a.algorithm_provider
        a.policy_config_file = ((pol.get("file") or {}).get("path")) or a.policy_config_file
        if pol.get("configMap"):
            a.policy_configmap = pol["configMap"].get("name")
            a.policy_configmap_namespace = pol["configMap"].get("namespace", "kube-system")
        a.scheduler_name = cc.get("schedulerName", a.scheduler_name)
        a.leader_elect = (cc.get("leaderElection") or {}).get("leaderElect", a.leader_elect)
        conn = cc.get("clientConnection") or {}
        a.kubeconfig = conn.get("kubeconfig") or a.kubeconfig
        a.kube_api_qps = conn.get("qps", a.kube_api_qps)
        a.disable_preemption = cc.get("disablePreemption", a.disable_preemption)
        a.percentage_of_nodes_to_score = cc.get("percentageOfNodesToScore", a.percentage_of_nodes_to_score)
        mb = cc.get("metricsBindAddress")
        if mb and ":" in mb:
            a.metrics_port = int(mb.rsplit(":", 1)[1])
        a.hard_pod_affinity_symmetric_weight = cc.get("hardPodAffinitySymmetricWeight", a.hard_pod_affinity_symmetric_weight)
        if a.use_legacy_policy_config and legacy_policy:
            a.policy_config_file = legacy_policy

    async def start():
        from ..scheduler.extender import HTTPExtender
        if a.kubeconfig:
            from ..client.clientcmd import client_from
            client = client_from(a.kubeconfig, qps=a.kube_api_qps, burst=a.kube_api_burst or int(a.kube_api_qps or 10),
                                 max_conns=64, content_type=a.kube_api_content_type)
        else:
            client = Client(a.master or "http://127.0.0.1:8080", qps=a.kube_api_qps,
                            burst=a.kube_api_burst or int(a.kube_api_qps or 10), max_conns=64,
                            content_type=a.kube_api_content_type)
        algo = await SP.resolve_algorithm(client, a.algorithm_provider, a.policy_config_file,
                                          a.policy_configmap, a.policy_configmap_namespace)
        preds, prios, ext_cfgs = algo
        if algo.hard_pod_affinity_symmetric_weight is not None:
            # the Policy's value wins over the flag (`factory.go:847` CreateFromConfig)
            a.hard_pod_affinity_symmetric_weight = algo.hard_pod_affinity_symmetric_weight
        extenders = [HTTPExtender.from_config(e) for e in ext_cfgs]
        s = Scheduler(client, a.scheduler_name, preds, prios, a.percentage_of_nodes_to_score,
                      emit_events=not a.no_events, extenders=extenders, shard_index=a.shard_index,
                      shard_count=a.shard_count, preemption=not a.disable_preemption and DefaultFeatureGate("PodPriority"),
                      hard_pod_affinity_symmetric_weight=a.hard_pod_affinity_symmetric_weight,
                      failure_domains=[d for d in a.failure_domains.split(",") if d])
        s.profiling = _true(a.profiling)
        if _true(a.contention_profiling):
            from ..utils.profiling import enable_contention_profiling
            enable_contention_profiling()
        if a.leader_elect:
            from ..client.leaderelection import LeaderElector
            lock = a.lock_object_name if a.shard_count == 1 else f"{a.lock_object_name}-shard-{a.shard_index}"
            le = LeaderElector(client, a.lock_object_namespace, lock)
            await le.acquire()
        spawn(s.run(metrics_port=a.metrics_port, metrics_address=a.address))
        return s

    run_until_signal(start)


if __name__ == "__main__":
    main()
