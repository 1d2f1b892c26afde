"""kube-controller-manager: runs the enabled controllers over one shared informer factory.

Parity: `cmd/kube-controller-manager/app/controllermanager.go:106-463` (controller map
`:334-363`, `--controllers` enable list with `*` and `-name`, shared informers started after
all controllers registered, optional leader election).
"""
from __future__ import annotations

import asyncio
import logging

from ..client.informer import InformerFactory
from .daemonset import DaemonSetController, StatefulSetController
from .deployment import DeploymentController
from .job import CronJobController, JobController
from .lifecycle import GarbageCollector, NamespaceController, NodeLifecycleController, PodGCController
from .certificates import (BootstrapSignerController, ClusterRoleAggregationController, CSRApprovingController,
                           CSRSigningController, TokenCleanerController, TokensController, TTLController)
from .podautoscaler import HorizontalController
from .attachdetach import AttachDetachController, ExternalAttacher
from .network import NodeIPAMController, RouteController, ServiceLBController
from .volume import ExpandController, PersistentVolumeController, PVCProtectionController
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
    "clusterroleaggregation": ClusterRoleAggregationController,
    "ttl": TTLController,
    "persistentvolume-binder": PersistentVolumeController,
    "pvc-protection": PVCProtectionController,
    "nodeipam": NodeIPAMController,
    "route": RouteController,
    "service": ServiceLBController,
    "attachdetach": AttachDetachController,
    "persistentvolume-expander": ExpandController,
    "csi-attacher": ExternalAttacher,
}


# like ControllersDisabledByDefault: "*" does not start these (name them explicitly, or the
# command line enables them from --allocate-node-cidrs / --loadbalancer-ip-range)
DISABLED_BY_DEFAULT = {"nodeipam", "route", "service", "csi-attacher"}


def resolve(enabled):
    names = set()
    for e in enabled or ["*"]:
        if e == "*":
            names |= set(CONTROLLERS) - DISABLED_BY_DEFAULT
        elif e.startswith("-"):
            names.discard(e[1:])
        else:
            names.add(e)
    for e in enabled or []:
        if e.startswith("-"):
            names.discard(e[1:])
    return sorted(names)


class ControllerManager:
    """`workers`: {controller name: worker count} (--concurrent-*-syncs); `start_interval`:
    seconds between controller starts (--controller-start-interval)."""

    def __init__(self, client, controllers=None, options=None, workers=None, start_interval=0.0):
        self.client = client
        self.factory = InformerFactory(client)
        self.controllers = []
        self.start_interval = start_interval
        options = options or {}
        for name in resolve(controllers):
            cls = CONTROLLERS[name]
            c = cls(client, self.factory, **options.get(name, {}))
            if workers and workers.get(name):
                c.workers = int(workers[name])
            c.setup()
            self.controllers.append(c)

    async def start(self):
        self.factory.start()
        await self.factory.wait_for_cache_sync(60)
        for c in self.controllers:
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
        await asyncio.sleep(0)
