"""DaemonSet controller: tables ported from `pkg/controller/daemon/update_test.go`
(TestDaemonSetUpdatesPods, ...WhenNewPosIsNotReady, ...AllOldPodsNotReady, ...NoTemplateChanged,
TestGetUnavailableNumbers) and the status / failed-pod cases of `daemon_controller_test.go`
(TestNumberReadyStatus, TestDaemonKillFailedPods), over the fake client; plus the round-4 probe
live: a DaemonSet with `maxUnavailable: "50%"` rolls on a real cluster.
"""
import asyncio
import copy

import pytest

from kubernetes_amd.api import meta as m
from kubernetes_amd.client.fake import FakeClient
from kubernetes_amd.client.informer import InformerFactory
from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.controllers.daemonset import DaemonSetController, HOSTNAME
from kubernetes_amd.controllers.history import REVISION_HASH, revision_hash

LABELS = {"name": "simple-daemon", "type": "production"}


def new_ds(name="foo", max_unavailable=None, min_ready=0):
    ds = {"apiVersion": "apps/v1", "kind": "DaemonSet",
          "metadata": {"name": name, "namespace": "default", "uid": f"uid-{name}", "generation": 1},
          "spec": {"selector": {"matchLabels": dict(LABELS)}, "revisionHistoryLimit": 10,
                   "updateStrategy": {"type": "OnDelete"},
                   "template": {"metadata": {"labels": dict(LABELS)},
                                "spec": {"containers": [{"name": "c", "image": "foo/bar"}]}}}}
    if max_unavailable is not None:
        ds["spec"]["updateStrategy"] = {"type": "RollingUpdate", "rollingUpdate": {"maxUnavailable": max_unavailable}}
    if min_ready:
        ds["spec"]["minReadySeconds"] = min_ready
    return ds


def node(i, labels=None, alloc=None, taints=None, conditions=None):
    name = i if isinstance(i, str) else f"node-{i}"
    n = {"apiVersion": "v1", "kind": "Node",
         "metadata": {"name": name, "labels": dict(labels or {}, **{HOSTNAME: name})},
         "spec": {},
         "status": {"conditions": conditions if conditions is not None else [{"type": "Ready", "status": "True"}]}}
    if alloc:
        n["status"]["allocatable"] = dict(alloc)
    if taints:
        n["spec"]["taints"] = list(taints)
    return n


class Harness:
    def __init__(self, ds, nodes=5, extra=()):
        nodes = [node(i) for i in range(nodes)] if isinstance(nodes, int) else list(nodes)
        self.c = FakeClient(ds, *nodes, *extra)
        self.f = InformerFactory(self.c)
        self.ctl = DaemonSetController(self.c, self.f)
        self.ctl.setup()
        self.creates, self.deletes = [], []

        def on_create(a):
            self.creates.append(a.obj)
            return False, None

        def on_delete(a):
            self.deletes.append(a.name)
            return False, None
        self.c.prepend_reactor("create", "pods", on_create)
        self.c.prepend_reactor("delete", "pods", on_delete)
        self.key = "default/" + ds["metadata"]["name"]
        self.events = []
        self.ctl.recorder.event = lambda obj, typ, reason, msg: self.events.append((reason, msg))
        self.error = None

    async def start(self):
        self.f.start()
        await self.f.wait_for_cache_sync()
        return self

    async def settle(self):
        for _ in range(3):
            await asyncio.sleep(0.002)

    async def sync_and_validate(self, creates, deletes):
        """syncAndValidateDaemonSets: one sync makes exactly this many creates and deletes."""
        self.creates.clear()
        self.deletes.clear()
        self.error = None
        try:
            await self.ctl.sync(self.key)
        except Exception as e:      # noqa: BLE001 - the reference's syncAndValidate only logs it
            self.error = e
        await self.settle()
        assert (len(self.creates), len(self.deletes)) == (creates, deletes), \
            (len(self.creates), len(self.deletes))

    def pods(self):
        return list(self.c.objects.get("pods", {}).values())

    async def mark_ready(self, since="2000-01-01T00:00:00Z"):
        for p in self.pods():
            if (p.get("status") or {}).get("phase") == "Running":
                continue
            q = copy.deepcopy(p)
            q["status"] = {"phase": "Running", "conditions": [{"type": "Ready", "status": "True",
                                                                "lastTransitionTime": since}]}
            await self.c.update("pods", q, "default")
        await self.settle()

    async def update_ds(self, fn):
        ds = copy.deepcopy(self.ctl.ds_inf.get(self.key))
        fn(ds)
        await self.c.update("daemonsets", ds, "default")
        await self.settle()

    def status(self):
        return self.ctl.ds_inf.get(self.key).get("status") or {}


def _new_image(max_unavailable):
    def fn(ds):
        ds["spec"]["template"]["spec"]["containers"][0]["image"] = "foo2/bar2"
        ds["spec"]["updateStrategy"] = {"type": "RollingUpdate", "rollingUpdate": {"maxUnavailable": max_unavailable}}
    return fn


def test_daemonset_updates_pods(run):
    async def main():
        h = await Harness(new_ds()).start()
        await h.sync_and_validate(5, 0)
        await h.mark_ready()
        await h.update_ds(_new_image(2))
        await h.sync_and_validate(0, 2)
        await h.sync_and_validate(2, 0)
        await h.mark_ready()
        await h.sync_and_validate(0, 2)
        await h.sync_and_validate(2, 0)
        await h.mark_ready()
        await h.sync_and_validate(0, 1)
        await h.sync_and_validate(1, 0)
        await h.mark_ready()
        await h.sync_and_validate(0, 0)
        assert all(p["spec"]["containers"][0]["image"] == "foo2/bar2" for p in h.pods())
        st = h.status()
        assert (st["updatedNumberScheduled"], st["numberAvailable"], st["desiredNumberScheduled"]) == (5, 5, 5)
    run(main())


def test_daemonset_updates_percentage_max_unavailable(run):
    """The round-4 wedge: `int("50%")`. 50% of 5 nodes rounds up to 3."""
    async def main():
        h = await Harness(new_ds()).start()
        await h.sync_and_validate(5, 0)
        await h.mark_ready()
        await h.update_ds(_new_image("50%"))
        await h.sync_and_validate(0, 3)
        await h.sync_and_validate(3, 0)
        await h.mark_ready()
        await h.sync_and_validate(0, 2)
    run(main())


def test_daemonset_updates_when_new_pod_is_not_ready(run):
    async def main():
        h = await Harness(new_ds()).start()
        await h.sync_and_validate(5, 0)
        await h.mark_ready()
        await h.update_ds(_new_image(3))
        await h.sync_and_validate(0, 3)
        await h.sync_and_validate(3, 0)
        await h.sync_and_validate(0, 0)     # the new pods are not ready: numUnavailable == maxUnavailable
    run(main())


def test_daemonset_updates_all_old_pods_not_ready(run):
    async def main():
        h = await Harness(new_ds()).start()
        await h.sync_and_validate(5, 0)
        await h.update_ds(_new_image(3))
        await h.sync_and_validate(0, 5)     # every old pod is unavailable: all go at once
        await h.sync_and_validate(5, 0)
        await h.sync_and_validate(0, 0)
    run(main())


def test_daemonset_updates_no_template_changed(run):
    async def main():
        h = await Harness(new_ds()).start()
        await h.sync_and_validate(5, 0)

        def fn(ds):
            ds["spec"]["updateStrategy"] = {"type": "RollingUpdate", "rollingUpdate": {"maxUnavailable": 3}}
        await h.update_ds(fn)
        await h.sync_and_validate(0, 0)
    run(main())


def _pod(name, node_name, ready=True, terminating=False):
    p = {"metadata": {"name": name, "namespace": "default", "labels": dict(LABELS)},
         "spec": {"nodeName": node_name}}
    if ready:
        p["status"] = {"phase": "Running", "conditions": [{"type": "Ready", "status": "True",
                                                           "lastTransitionTime": "2000-01-01T00:00:00Z"}]}
    if terminating:
        p["metadata"]["deletionTimestamp"] = "2000-01-01T00:00:00Z"
    return p


@pytest.mark.parametrize("name,nodes,mu,node_to_pods,exp", [
    ("No nodes", 0, 0, {}, (0, 0)),
    ("Two nodes with ready pods", 2, 1, {"node-0": [_pod("pod-0", "node-0")], "node-1": [_pod("pod-1", "node-1")]},
     (1, 0)),
    ("Two nodes, one node without pods", 2, 0, {"node-0": [_pod("pod-0", "node-0")]}, (0, 1)),
    ("Two nodes with pods, MaxUnavailable in percents", 2, "50%",
     {"node-0": [_pod("pod-0", "node-0")], "node-1": [_pod("pod-1", "node-1")]}, (1, 0)),
    ("Two nodes with pods, MaxUnavailable in percents, pod terminating", 2, "50%",
     {"node-0": [_pod("pod-0", "node-0")], "node-1": [_pod("pod-1", "node-1", terminating=True)]}, (1, 1)),
])
def test_get_unavailable_numbers(name, nodes, mu, node_to_pods, exp):
    h = Harness(new_ds("x", max_unavailable=mu), nodes=nodes)
    ds = new_ds("x", max_unavailable=mu)
    want = {f"node-{i}" for i in range(nodes)}
    assert h.ctl.unavailable_numbers(ds, want, node_to_pods) == exp, name


def test_number_ready_status_and_min_ready_seconds(run):
    """TestNumberReadyStatus + numberAvailable honouring minReadySeconds."""
    async def main():
        h = await Harness(new_ds(min_ready=3600), nodes=2).start()
        await h.sync_and_validate(2, 0)
        await h.ctl.sync(h.key)
        await h.settle()
        st = h.status()
        assert (st["numberReady"], st["numberAvailable"], st["desiredNumberScheduled"]) == (0, 0, 2)
        await h.mark_ready(since=m.now_rfc3339())           # ready just now: not yet available
        await h.ctl.sync(h.key)
        await h.settle()
        st = h.status()
        assert (st["numberReady"], st["numberAvailable"], st["numberUnavailable"]) == (2, 0, 2)
        for p in h.pods():                                   # ready for longer than minReadySeconds
            q = copy.deepcopy(p)
            q["status"]["conditions"][0]["lastTransitionTime"] = "2000-01-01T00:00:00Z"
            await h.c.update("pods", q, "default")
        await h.settle()
        await h.ctl.sync(h.key)
        await h.settle()
        st = h.status()
        assert (st["numberReady"], st["numberAvailable"], st["numberUnavailable"]) == (2, 2, 0)
    run(main())


@pytest.mark.parametrize("failed,normal,creates,deletes,events", [
    (0, 1, 0, 0, 0),       # normal (do nothing)
    (0, 0, 1, 0, 0),       # no pods (create 1)
    (1, 0, 0, 1, 1),       # 1 failed pod (kill 1); the replacement comes with the next sync
    (1, 3, 0, 3, 1),       # 1 failed pod (kill 1), 3 normal pods (kill 2)
    (2, 1, 0, 2, 2),       # 2 failed pods (kill 2), 1 normal pod
])
def test_daemon_kill_failed_pods(run, failed, normal, creates, deletes, events):
    """TestDaemonKillFailedPods; a sync that killed failed pods ends in an error (rate limit)."""
    async def main():
        ds = new_ds()
        pods = [daemon_pod(f"failed-{i}", "node-0", ds, phase="Failed") for i in range(failed)] + \
               [daemon_pod(f"normal-{i}", "node-0", ds) for i in range(normal)]
        h = await Harness(ds, nodes=1, extra=pods).start()
        await h.sync_and_validate(creates, deletes)
        assert len([e for e in h.events if e[0] == "FailedDaemonPod"]) == events
        assert (h.error is not None) == bool(failed)
        if failed and not normal:
            await h.sync_and_validate(1, 0)
    run(main())


def test_percentage_max_unavailable_rolls_live(run):
    async def main():
        async with LocalCluster(nodes=2, gpus_per_node=0, controllers=["daemonset"]) as cl:
            c = cl.client
            ds = {"apiVersion": "apps/v1", "kind": "DaemonSet", "metadata": {"name": "agent", "namespace": "default"},
                  "spec": {"selector": {"matchLabels": {"app": "agent"}},
                           "updateStrategy": {"type": "RollingUpdate", "rollingUpdate": {"maxUnavailable": "50%"}},
                           "template": {"metadata": {"labels": {"app": "agent"}},
                                        "spec": {"containers": [{"name": "c", "image": "agent:1"}]}}}}
            await c.create("daemonsets", ds)

            async def rolled(image):
                d = await c.get("daemonsets", "agent", "default")
                st = d.get("status") or {}
                ps = [p for p in (await c.list("pods", "default", label_selector="app=agent"))["items"]
                      if not p["metadata"].get("deletionTimestamp")]
                return st.get("observedGeneration") == d["metadata"]["generation"] and \
                    st.get("updatedNumberScheduled") == 2 and st.get("numberAvailable") == 2 and \
                    len(ps) == 2 and all(p["spec"]["containers"][0]["image"] == image for p in ps)
            await cl.wait_for(lambda: rolled("agent:1"), timeout=30)
            await c.patch("daemonsets", "agent", {"spec": {"template": {"spec": {"containers": [
                {"name": "c", "image": "agent:2"}]}}}}, "default", patch_type="strategic")
            await cl.wait_for(lambda: rolled("agent:2"), timeout=30)
            revs = (await c.list("controllerrevisions", "default"))["items"]
            assert len(revs) == 2 and all(REVISION_HASH in r["metadata"]["labels"] for r in revs)
    run(main(), timeout=90)


def daemon_pod(name, node_name, ds, labels=None, phase="Running", spec=None, terminating=False):
    p = {"apiVersion": "v1", "kind": "Pod",
         "metadata": {"name": name, "namespace": "default", "labels": dict(labels if labels is not None else LABELS),
                      "creationTimestamp": "2000-01-01T00:00:00Z"},
         "spec": dict(spec or {"containers": [{"name": "c", "image": "foo/bar"}]}, nodeName=node_name),
         "status": {"phase": phase}}
    if ds is not None:
        p["metadata"]["labels"][REVISION_HASH] = revision_hash(ds["spec"]["template"])
        p["metadata"]["ownerReferences"] = [{"apiVersion": "apps/v1", "kind": "DaemonSet", "name": ds["metadata"]["name"],
                                             "uid": ds["metadata"]["uid"], "controller": True}]
    if terminating:
        p["metadata"]["deletionTimestamp"] = "2000-01-01T00:00:00Z"
    return p


def resource_spec(node_name, mem, cpu):
    spec = {"containers": [{"name": "c", "image": "foo/bar", "resources": {"requests": {"memory": mem, "cpu": cpu}}}]}
    if node_name:
        spec["nodeName"] = node_name
    return spec


def with_spec(ds, spec):
    ds["spec"]["template"]["spec"] = spec
    return ds


def drain(q):
    q._heap.clear()
    while (it := q.get_nowait()) is not None:
        q.done(it)


def queued(q):
    return len(q) + len(q._heap)


NO_SCHEDULE = [{"key": "dedicated", "value": "gpu", "effect": "NoSchedule"}]
NO_EXECUTE = [{"key": "dedicated", "value": "gpu", "effect": "NoExecute"}]
STRATEGIES = [None, 1]        # OnDelete, RollingUpdate (updateStrategies())


async def _one(ds, nodes, extra=(), creates=0, deletes=0):
    h = await Harness(ds, nodes=nodes, extra=extra).start()
    await h.sync_and_validate(creates, deletes)
    return h


@pytest.mark.parametrize("mu", STRATEGIES)
def test_taints(run, mu):
    """TestNoScheduleTaintedDoesntEvicitRunningIntolerantPod, TestNoExecuteTaintedDoesEvicit...,
    TestTaintedNodeDaemonDoesNotLaunchIntolerantPod, TestTaintedNodeDaemonLaunchesToleratePod,
    TestNotReadyNodeDaemonLaunchesPod, TestUnreachableNodeDaemonLaunchesPod,
    TestTaintPressureNodeDaemonLaunchesPod."""
    async def main():
        ds = new_ds("intolerant", max_unavailable=mu)
        await _one(ds, [node("tainted", taints=NO_SCHEDULE)], [daemon_pod("keep-running-me", "tainted", ds)], 0, 0)
        await _one(ds, [node("tainted", taints=NO_EXECUTE)], [daemon_pod("stop-running-me", "tainted", ds)], 0, 1)
        await _one(ds, [node("tainted", taints=NO_SCHEDULE)], (), 0, 0)
        tol = new_ds("tolerate", max_unavailable=mu)
        tol["spec"]["template"]["spec"]["tolerations"] = [{"key": "dedicated", "operator": "Equal", "value": "gpu",
                                                          "effect": "NoSchedule"}]
        await _one(tol, [node("tainted", taints=NO_SCHEDULE)], (), 1, 0)
        await _one(tol, [node(0)], (), 1, 0)
        simple = new_ds("simple", max_unavailable=mu)
        await _one(simple, [node("nr", taints=[{"key": "node.kubernetes.io/not-ready", "effect": "NoExecute"}],
                                 conditions=[{"type": "Ready", "status": "False"}])], (), 1, 0)
        await _one(simple, [node("ur", taints=[{"key": "node.kubernetes.io/unreachable", "effect": "NoExecute"}],
                                 conditions=[{"type": "Ready", "status": "Unknown"}])], (), 1, 0)
        await _one(simple, [node("pressure", taints=[
            {"key": "node.kubernetes.io/disk-pressure", "effect": "NoSchedule"},
            {"key": "node.kubernetes.io/memory-pressure", "effect": "NoSchedule"}])], (), 1, 0)
        await _one(simple, [node("net", conditions=[{"type": "NetworkUnavailable", "status": "True"}])], (), 1, 0)
    run(main())


def test_daemonset_respects_termination(run):
    async def main():
        ds = new_ds()
        await _one(ds, [node(0)], [daemon_pod("node-0-x", "node-0", ds, terminating=True)], 0, 0)
    run(main())


@pytest.mark.parametrize("mu", STRATEGIES)
def test_insufficient_capacity(run, mu):
    """TestInsufficientCapacityNodeDaemonDoesNotLaunchPod / ...DoesNotUnscheduleRunningPod /
    TestSufficientCapacityWithTerminatedPodsDaemonLaunchesPod / TestSufficientCapacityNode...:
    an over-committed node gets no new pod (FailedPlacement) but keeps a running one."""
    async def main():
        spec = resource_spec("", "75M", "75m")
        other = daemon_pod("other", "too-much-mem", None, labels={}, spec=resource_spec("", "75M", "75m"))
        small = {"memory": "100M", "cpu": "200m", "pods": "100"}
        h = await _one(with_spec(new_ds(max_unavailable=mu), spec), [node("too-much-mem", alloc=small)], [other], 0, 0)
        assert [r for r, _ in h.events] == ["FailedPlacement"] and "Insufficient" in h.events[0][1]
        assert h.ctl.suspended == {"too-much-mem": {h.key}}
        ds = with_spec(new_ds(max_unavailable=mu), spec)
        await _one(ds, [node("too-much-mem", alloc=small)], [other, daemon_pod("mine", "too-much-mem", ds, spec=spec)], 0, 0)
        done = dict(other, status={"phase": "Succeeded"})
        h = await _one(with_spec(new_ds(max_unavailable=mu), spec), [node("too-much-mem", alloc=small)], [done], 1, 0)
        big = {"memory": "200M", "cpu": "200m", "pods": "100"}
        await _one(with_spec(new_ds(max_unavailable=mu), spec), [node("roomy", alloc=big)], [other], 1, 0)
    run(main())


def test_insufficient_capacity_elsewhere_with_node_selector(run):
    """TestInsufficientCapacityNodeSufficientCapacityWithNodeLabelDaemonLaunchPod: no event for
    a node the selector excludes anyway."""
    async def main():
        ds = with_spec(new_ds(), dict(resource_spec("", "50M", "75m"), nodeSelector={"color": "blue"}))
        h = await _one(ds, [node("not-enough", alloc={"memory": "10M", "cpu": "20m"}),
                            node("enough", labels={"color": "blue"}, alloc={"memory": "100M", "cpu": "200m"})], (), 1, 0)
        assert h.events == []
    run(main())


def test_deleting_a_pod_requeues_suspended_sets(run):
    """TestDeleteNoDaemonPod: deleting a scheduled non-daemon pod on the node frees room."""
    async def main():
        spec = resource_spec("", "50M", "50m")
        others = [daemon_pod(f"pod-{i}", "node1", None, labels={}, spec=spec) for i in range(4)]
        h = await _one(with_spec(new_ds(), spec), [node("node1", alloc={"memory": "200M", "cpu": "200m"})], others, 0, 0)
        assert h.ctl.suspended == {"node1": {h.key}}
        drain(h.ctl.queue)
        await h.c.delete("pods", "pod-0", "default")
        await asyncio.sleep(0.05)
        assert queued(h.ctl.queue) == 1
        await h.sync_and_validate(1, 0)
        assert h.ctl.suspended == {}
    run(main())


@pytest.mark.parametrize("mu", STRATEGIES)
def test_host_ports(run, mu):
    """TestPortConflictNodeDaemonDoesNotLaunchPod / TestPortConflictWithSameDaemonPodDoesNotDeletePod
    / TestNoPortConflictNodeDaemonLaunchesPod."""
    def spec(port):
        return {"containers": [{"name": "c", "image": "foo/bar", "ports": [{"containerPort": port, "hostPort": port}]}]}

    async def main():
        other = daemon_pod("other", "port-conflict", None, labels={}, spec=spec(666))
        await _one(with_spec(new_ds(max_unavailable=mu), spec(666)), [node("port-conflict")], [other], 0, 0)
        ds = with_spec(new_ds(max_unavailable=mu), spec(666))
        await _one(ds, [node("port-conflict")], [daemon_pod("foo-1", "port-conflict", ds, spec=spec(666))], 0, 0)
        other2 = daemon_pod("other", "no-port-conflict", None, labels={}, spec=spec(6661))
        await _one(with_spec(new_ds(max_unavailable=mu), spec(6662)), [node("no-port-conflict")], [other2], 1, 0)
    run(main())


def test_empty_selector_does_nothing(run):
    """TestPodIsNotDeletedByDaemonsetWithEmptyLabelSelector."""
    async def main():
        ds = new_ds()
        ds["spec"]["selector"] = {}
        ds["spec"]["template"]["spec"]["nodeSelector"] = {"foo": "bar"}
        h = await _one(ds, [node("node1")], [daemon_pod("p", "node1", None, labels={"bang": "boom"})], 0, 0)
        assert [r for r, _ in h.events] == ["SelectingAll"]
    run(main())


def test_deals_with_existing_pods(run):
    """TestDealsWithExistingPods: the oldest pod per node stays, duplicates go, owned pods whose
    labels no longer match are released (not deleted) and their nodes get a new pod."""
    async def main():
        ds = new_ds()
        pods = [daemon_pod("n1-0", "node-1", ds)] + [daemon_pod(f"n2-{i}", "node-2", ds) for i in range(2)] + \
               [daemon_pod(f"n3-{i}", "node-3", ds) for i in range(5)] + \
               [daemon_pod(f"n4-{i}", "node-4", ds, labels={"name": "other"}) for i in range(2)]
        h = await _one(ds, 5, pods, 2, 5)
        released = [p for p in h.pods() if p["metadata"]["name"].startswith("n4-")]
        assert all(not p["metadata"].get("ownerReferences") for p in released)
    run(main())


def test_adopts_matching_orphans(run):
    async def main():
        ds = new_ds()
        h = await _one(ds, 1, [daemon_pod("orphan", "node-0", None)], 0, 0)
        (p,) = h.pods()
        assert p["metadata"]["ownerReferences"][0]["uid"] == ds["metadata"]["uid"]
    run(main())


def test_selector_and_name(run):
    """TestSelectorDaemonLaunchesPods, TestSelectorDaemonDeletesUnselectedPods,
    TestNameDaemonSetLaunchesPods, TestBadNameDaemonSetDoesNothing,
    TestNameAndSelectorDaemonSetLaunchesPods, TestInconsistentNameSelectorDaemonSetDoesNothing."""
    blue = {"color": "blue"}

    async def main():
        ds = new_ds()
        ds["spec"]["template"]["spec"]["nodeSelector"] = blue
        nodes = [node(i) for i in range(4)] + [node(i, labels=blue) for i in range(4, 7)]
        await _one(ds, nodes, (), 3, 0)
        ds = new_ds()
        ds["spec"]["template"]["spec"]["nodeSelector"] = blue
        pods = [daemon_pod("a", "node-0", ds), daemon_pod("b", "node-4", ds), daemon_pod("c", "node-5", ds)]
        await _one(ds, nodes, pods, 1, 1)
        ds = new_ds()
        ds["spec"]["template"]["spec"]["nodeName"] = "node-0"
        await _one(ds, 5, (), 1, 0)
        ds = new_ds()
        ds["spec"]["template"]["spec"]["nodeName"] = "node-10"
        await _one(ds, 5, (), 0, 0)
        ds = new_ds()
        ds["spec"]["template"]["spec"].update(nodeName="node-6", nodeSelector=blue)
        await _one(ds, nodes, (), 1, 0)
        ds = new_ds()
        ds["spec"]["template"]["spec"].update(nodeName="node-0", nodeSelector=blue)
        await _one(ds, nodes, (), 0, 0)
    run(main())


@pytest.mark.parametrize("spec,pods,exp", [
    (resource_spec("", "50M", "0.5"), [], (True, True, True)),
    (resource_spec("", "200M", "0.5"), [], (True, False, True)),
    (resource_spec("other-node", "50M", "0.5"), [], (False, False, False)),
    ({"containers": [{"name": "c", "ports": [{"containerPort": 666, "hostPort": 666}]}]},
     [{"containers": [{"name": "c", "ports": [{"containerPort": 666, "hostPort": 666}]}]}], (False, False, False)),
])
def test_node_should_run_daemon_pod(spec, pods, exp):
    """TestNodeShouldRunDaemonPod."""
    from kubernetes_amd.controllers.daemonset import node_should_run
    n = node("test-node", alloc={"memory": "100M", "cpu": "1"})
    on_node = [daemon_pod(f"p{i}", "test-node", None, labels={}, spec=s) for i, s in enumerate(pods)]
    assert node_should_run(with_spec(new_ds(), spec), n, on_node)[:3] == exp


def test_update_node_enqueues_only_on_relevant_changes(run):
    """TestUpdateNode."""
    async def main():
        ds = new_ds()
        ds["spec"]["template"]["spec"]["nodeSelector"] = {"color": "blue"}
        h = await Harness(ds, nodes=[node("node1")], extra=[new_ds("plain")]).start()

        def enqueued(old, cur):
            drain(h.ctl.queue)
            h.ctl._update_node(old, cur)
            return queued(h.ctl.queue) > 0
        assert not enqueued(node("node1"), node("node1"))
        assert enqueued(node("node1"), node("node1", labels={"color": "blue"}))
        assert enqueued(node("node1", taints=NO_EXECUTE), node("node1"))
        # a heartbeat that only moves timestamps is ignored
        a = node("node1", conditions=[{"type": "Ready", "status": "True", "lastHeartbeatTime": "1"}])
        b = node("node1", conditions=[{"type": "Ready", "status": "True", "lastHeartbeatTime": "2"}])
        assert not enqueued(a, b)
    run(main())


def test_create_pod_template_tolerations(feature_gate):
    """`pkg/controller/daemon/util/daemonset_util_test.go` TestCreatePodTemplate: the not-ready /
    unreachable NoExecute and pressure NoSchedule tolerations (replacing same key+effect ones), and
    out-of-disk only for a critical pod."""
    from kubernetes_amd.controllers.daemonset import OUT_OF_DISK_TOLERATION, _with_tolerations
    spec = {"tolerations": [{"key": "node.kubernetes.io/not-ready", "operator": "Equal", "value": "x",
                             "effect": "NoExecute", "tolerationSeconds": 5}]}
    tols = _with_tolerations(spec, {"namespace": "default"})
    keys = [(t["key"], t["effect"]) for t in tols]
    assert keys.count(("node.kubernetes.io/not-ready", "NoExecute")) == 1
    assert {"key": "node.kubernetes.io/not-ready", "operator": "Exists", "effect": "NoExecute"} in tols
    assert OUT_OF_DISK_TOLERATION not in tols
    crit = {"namespace": "kube-system", "annotations": {"scheduler.alpha.kubernetes.io/critical-pod": ""}}
    assert OUT_OF_DISK_TOLERATION in _with_tolerations({}, crit)
    feature_gate.set("ExperimentalCriticalPodAnnotation=false")
    assert OUT_OF_DISK_TOLERATION not in _with_tolerations({}, crit)
