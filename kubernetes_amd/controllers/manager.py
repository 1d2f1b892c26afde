"""kube-controller-manager: runs the enabled controllers over one shared informer factory.

Parity: `cmd/kube-controller-manager/app/controllermanager.go:106-463` (controller map
`:334-363`, `--controllers` enable list with `*` and `-name`, shared informers started after
all controllers registered, optional leader election).

Credentials (`controllermanager.go:133-139`, `--use-service-account-credentials`): the shared
informers and the service-account token controller always use the manager's own client (the
`system:kube-controller-manager` role: read-only informers plus SA/secret bootstrap). With
service-account credentials every other controller runs as `kube-system/<its SA>` — bound to its
`system:controller:<name>` role by the bootstrap policy — with a client built from that
account's token (`SAControllerClientBuilder`: create the account if missing, wait for the token
controller to mint its token secret).
"""
from __future__ import annotations

import asyncio
import logging

from ..client.informer import InformerFactory, resync_period
from .daemonset import DaemonSetController, StatefulSetController
from .deployment import DeploymentController
from .job import CronJobController, JobController
from .lifecycle import GarbageCollector, NamespaceController, NodeLifecycleController, PodGCController
from .certificates import (BootstrapSignerController, ClusterRoleAggregationController, CSRApprovingController,
                           CSRCleanerController, CSRSigningController, TokenCleanerController, TokensController,
                           TTLController)
from .podautoscaler import HorizontalController
from .attachdetach import AttachDetachController, ExternalAttacher
from .network import NodeIPAMController, RouteController, ServiceLBController
from .volume import ExpandController, PersistentVolumeController, PVCProtectionController, PVProtectionController
from .misc import DisruptionController, EndpointsController, ResourceQuotaController, ServiceAccountController
from .replicaset import ReplicaSetController, ReplicationControllerController

log = logging.getLogger("controller-manager")

CONTROLLERS = {
    "replicaset": ReplicaSetController,
    "replicationcontroller": ReplicationControllerController,
    "deployment": DeploymentController,
    "job": JobController,
    "cronjob": CronJobController,
    "daemonset": DaemonSetController,
    "statefulset": StatefulSetController,
    "namespace": NamespaceController,
    "garbagecollector": GarbageCollector,
    "podgc": PodGCController,
    "nodelifecycle": NodeLifecycleController,
    "serviceaccount": ServiceAccountController,
    "endpoint": EndpointsController,
    "resourcequota": ResourceQuotaController,
    "disruption": DisruptionController,
    "horizontalpodautoscaling": HorizontalController,
    "serviceaccount-token": TokensController,
    "bootstrapsigner": BootstrapSignerController,
    "tokencleaner": TokenCleanerController,
    "csrapproving": CSRApprovingController,
    "csrsigning": CSRSigningController,
    "csrcleaner": CSRCleanerController,
    "clusterroleaggregation": ClusterRoleAggregationController,
    "ttl": TTLController,
    "persistentvolume-binder": PersistentVolumeController,
    "pvc-protection": PVCProtectionController,
    "pv-protection": PVProtectionController,
    "nodeipam": NodeIPAMController,
    "route": RouteController,
    "service": ServiceLBController,
    "attachdetach": AttachDetachController,
    "persistentvolume-expander": ExpandController,
    "csi-attacher": ExternalAttacher,
}


# `ControllersDisabledByDefault` (controllermanager.go:321: bootstrapsigner, tokencleaner — kubeadm
# names them explicitly) plus the controllers the command line enables from --allocate-node-cidrs
# / --loadbalancer-ip-range and the in-tree CSI attacher: "*" does not start these
DISABLED_BY_DEFAULT = {"bootstrapsigner", "tokencleaner", "nodeipam", "route", "service", "csi-attacher"}


# the reference's `--controllers` names (`controllermanager.go:334-363`) for controllers this
# manager runs under a different name or splits: "node" is the lifecycle half of the reference's
# node controller (CIDR allocation is `nodeipam`, enabled by --allocate-node-cidrs)
ALIASES = {"node": ("nodelifecycle",), "clusterrole-aggregation": ("clusterroleaggregation",)}


def resolve(enabled):
    def expand(e):
        return ALIASES.get(e, (e,))
    names = set()
    for e in enabled or ["*"]:
        if e == "*":
            names |= set(CONTROLLERS) - DISABLED_BY_DEFAULT
        elif e.startswith("-"):
            names.difference_update(expand(e[1:]))
        else:
            names.update(expand(e))
    for e in enabled or []:
        if e.startswith("-"):
            names.difference_update(expand(e[1:]))
    return sorted(names)


# controller -> the kube-system service account it runs as (`controller_policy.go` role names);
# controllers absent here (serviceaccount-token) always use the manager's own credentials
SERVICE_ACCOUNTS = {
    "replicaset": "replicaset-controller", "replicationcontroller": "replication-controller",
    "deployment": "deployment-controller", "job": "job-controller", "cronjob": "cronjob-controller",
    "daemonset": "daemon-set-controller", "statefulset": "statefulset-controller",
    "namespace": "namespace-controller", "garbagecollector": "generic-garbage-collector",
    "podgc": "pod-garbage-collector", "nodelifecycle": "node-controller", "nodeipam": "node-controller",
    "serviceaccount": "service-account-controller", "endpoint": "endpoint-controller",
    "resourcequota": "resourcequota-controller", "disruption": "disruption-controller",
    "horizontalpodautoscaling": "horizontal-pod-autoscaler", "bootstrapsigner": "bootstrap-signer",
    "tokencleaner": "token-cleaner", "csrapproving": "certificate-controller", "csrsigning": "certificate-controller",
    "csrcleaner": "certificate-controller",
    "clusterroleaggregation": "clusterrole-aggregation-controller", "ttl": "ttl-controller",
    "persistentvolume-binder": "persistent-volume-binder", "pvc-protection": "pvc-protection-controller",
    "pv-protection": "pv-protection-controller",
    "route": "route-controller", "service": "service-controller", "attachdetach": "attachdetach-controller",
    "persistentvolume-expander": "expand-controller", "csi-attacher": "csi-attacher",
}
SA_NAMESPACE = "kube-system"
SA_TOKEN_TYPE = "kubernetes.io/service-account-token"


class ServiceAccountClients:
    """`SAControllerClientBuilder`: a client per controller service account, authenticated with
    the account's token. `make_client(token)` builds a client against the same server."""

    def __init__(self, root, make_client, timeout=30.0):
        self.root = root
        self.make_client = make_client
        self.timeout = timeout
        self.clients = {}
        self._lock = asyncio.Lock()

    async def _token(self, sa):
        from ..client.rest import APIStatusError
        try:
            await self.root.create("serviceaccounts", {"metadata": {"name": sa, "namespace": SA_NAMESPACE}},
                                   SA_NAMESPACE)
        except APIStatusError as e:
            if e.code != 409:
                raise
        deadline = asyncio.get_running_loop().time() + self.timeout
        while True:
            acct = await self.root.get("serviceaccounts", sa, SA_NAMESPACE)
            for ref in acct.get("secrets") or ():
                try:
                    sec = await self.root.get("secrets", ref["name"], SA_NAMESPACE)
                except APIStatusError:
                    continue
                tok = (sec.get("data") or {}).get("token")
                if sec.get("type") == SA_TOKEN_TYPE and tok:
                    import base64
                    return base64.b64decode(tok).decode()
            if asyncio.get_running_loop().time() > deadline:
                raise TimeoutError(f"no token for service account {SA_NAMESPACE}/{sa} after {self.timeout:.0f}s "
                                   "(is the serviceaccount-token controller running with a signing key?)")
            await asyncio.sleep(0.1)

    async def client_for(self, sa):
        async with self._lock:
            c = self.clients.get(sa)
        if c is None:
            c = self.make_client(await self._token(sa))
            async with self._lock:
                self.clients.setdefault(sa, c)
                c = self.clients[sa]
        return c

    async def close(self):
        for c in self.clients.values():
            await c.close()


class ControllerManager:
    """`workers`: {controller name: worker count} (--concurrent-*-syncs); `start_interval`:
    seconds between controller starts (--controller-start-interval); `sa_client_factory`:
    token -> client, set for --use-service-account-credentials; `resync`: --min-resync-period
    in seconds (0 = informers never resync)."""

    def __init__(self, client, controllers=None, options=None, workers=None, start_interval=0.0,
                 sa_client_factory=None, resync=0.0, resync_periods=None, attach_detach_reconcile=True):
        self.client = client
        # --min-resync-period: the shared informers resync every [min, 2*min)
        self.factory = InformerFactory(client, resync_period(resync))
        self.controllers = []
        self.start_interval = start_interval
        self.options = options or {}
        self.workers = workers or {}
        self.resync_periods = resync_periods or {}      # controller -> full-resync seconds
        self.attach_detach_reconcile = attach_detach_reconcile
        self.names = resolve(controllers)
        self.sa_clients = ServiceAccountClients(client, sa_client_factory) if sa_client_factory else None
        self.identities = {}          # controller name -> the identity it runs as
        if self.sa_clients is None:
            for name in self.names:
                self._add(name, client)
                self.identities[name] = "manager"

    def _add(self, name, client):
        cls = CONTROLLERS[name]
        c = cls(client, self.factory, **self.options.get(name, {}))
        if self.workers.get(name):
            c.workers = int(self.workers[name])
        if self.resync_periods.get(name):
            c.resync_period = float(self.resync_periods[name])
        if name == "attachdetach":
            c.disable_reconcile_sync = not self.attach_detach_reconcile
        c.setup()
        self.controllers.append(c)
        return c

    async def _build_with_service_accounts(self):
        # the token controller (manager credentials) must run before any account has a token
        first = [n for n in self.names if n not in SERVICE_ACCOUNTS]
        for name in first:
            self._add(name, self.client)
            self.identities[name] = "manager"
        self.factory.start()
        await self.factory.wait_for_cache_sync(60)
        for c in self.controllers:
            c.start()
        rest = [n for n in self.names if n in SERVICE_ACCOUNTS]
        clients = await asyncio.gather(*(self.sa_clients.client_for(SERVICE_ACCOUNTS[n]) for n in rest))
        started = len(self.controllers)
        for name, cl in zip(rest, clients):
            self._add(name, cl)
            self.identities[name] = f"system:serviceaccount:{SA_NAMESPACE}:{SERVICE_ACCOUNTS[name]}"
        return started

    async def start(self):
        already = 0
        if self.sa_clients is not None:
            already = await self._build_with_service_accounts()
        self.factory.start()
        await self.factory.wait_for_cache_sync(60)
        for c in self.controllers[already:]:
            c.start()
            if self.start_interval:
                await asyncio.sleep(self.start_interval)
        return self

    def render_metrics(self) -> bytes:
        """Work-queue metrics per controller (`workqueue/metrics.go`: depth, adds)."""
        out = ["# TYPE workqueue_depth gauge"]
        out += [f'workqueue_depth{{name="{c.name}"}} {len(c.queue._queue)}' for c in self.controllers]
        out.append("# TYPE workqueue_adds counter")
        out += [f'workqueue_adds{{name="{c.name}"}} {c.queue.adds}' for c in self.controllers]
        out.append("# TYPE controller_syncs_total counter")
        out += [f'controller_syncs_total{{name="{c.name}"}} {c.syncs}' for c in self.controllers]
        return ("\n".join(out) + "\n").encode()

    def render(self):
        return self.render_metrics()

    def get(self, name):
        for c in self.controllers:
            if c.name == name:
                return c
        return None

    async def stop(self):
        for c in self.controllers:
            c.stop()
        self.factory.stop()
        if self.sa_clients is not None:
            await self.sa_clients.close()
        await asyncio.sleep(0)
