"""Leader election. Parity: `staging/src/k8s.io/client-go/tools/leaderelection/leaderelection.go`
with the Endpoints annotation lock (`resourcelock/endpointslock.go`, annotation
`control-plane.alpha.kubernetes.io/leader` holding a LeaderElectionRecord) — plus a Lease lock.

Semantics: acquire if the record is absent or expired (renewTime + leaseDuration < now); the
holder renews every `retry_period`; losing the lease (renew failed for `renew_deadline`) calls
`on_stopped_leading`.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import socket
import time

from ..api.meta import new_uid, now_rfc3339_micro, parse_rfc3339
from .rest import APIStatusError, is_conflict, is_not_found

log = logging.getLogger("leaderelection")
ANNOTATION = "control-plane.alpha.kubernetes.io/leader"


class EndpointsLock:
    resource = "endpoints"

    def __init__(self, client, ns, name):
        self.client, self.ns, self.name = client, ns, name
        self.obj = None

    async def get(self):
        try:
            self.obj = await self.client.get(self.resource, self.name, self.ns)
        except APIStatusError as e:
            if is_not_found(e):
                self.obj = None
                return None
            raise
        raw = (self.obj["metadata"].get("annotations") or {}).get(ANNOTATION)
        return json.loads(raw) if raw else None

    async def create(self, rec):
        self.obj = await self.client.create(self.resource, {"metadata": {"name": self.name, "namespace": self.ns,
                                                                         "annotations": {ANNOTATION: json.dumps(rec)}}}, self.ns)

    async def update(self, rec):
        md = dict(self.obj["metadata"])
        md["annotations"] = dict(md.get("annotations") or {}, **{ANNOTATION: json.dumps(rec)})
        self.obj = await self.client.update(self.resource, dict(self.obj, metadata=md), self.ns)


class LeaseLock(EndpointsLock):
    resource = "leases"

    async def get(self):
        try:
            self.obj = await self.client.get(self.resource, self.name, self.ns)
        except APIStatusError as e:
            if is_not_found(e):
                self.obj = None
                return None
            raise
        s = self.obj.get("spec") or {}
        return {"holderIdentity": s.get("holderIdentity", ""), "leaseDurationSeconds": s.get("leaseDurationSeconds", 15),
                "acquireTime": s.get("acquireTime"), "renewTime": s.get("renewTime"),
                "leaderTransitions": s.get("leaseTransitions", 0)}

    @staticmethod
    def _spec(rec):
        return {"holderIdentity": rec["holderIdentity"], "leaseDurationSeconds": rec["leaseDurationSeconds"],
                "acquireTime": rec["acquireTime"], "renewTime": rec["renewTime"], "leaseTransitions": rec["leaderTransitions"]}

    async def create(self, rec):
        self.obj = await self.client.create(self.resource, {"metadata": {"name": self.name, "namespace": self.ns},
                                                            "spec": self._spec(rec)}, self.ns)

    async def update(self, rec):
        self.obj = await self.client.update(self.resource, dict(self.obj, spec=self._spec(rec)), self.ns)


class LeaderElector:
    def __init__(self, client, namespace, name, identity=None, lease_duration=15.0, renew_deadline=10.0,
                 retry_period=2.0, lock="endpoints", on_started_leading=None, on_stopped_leading=None):
        self.lock = (LeaseLock if lock == "leases" else EndpointsLock)(client, namespace, name)
        self.identity = identity or f"{socket.gethostname()}_{os.getpid()}_{new_uid()[:8]}"
        self.lease_duration = lease_duration
        self.renew_deadline = renew_deadline
        self.retry_period = retry_period
        self.on_started = on_started_leading
        self.on_stopped = on_stopped_leading
        self.is_leader = False
        self._renewer = None

    async def try_acquire_or_renew(self) -> bool:
        now = time.time()
        rec = {"holderIdentity": self.identity, "leaseDurationSeconds": int(self.lease_duration),
               "acquireTime": now_rfc3339_micro(now), "renewTime": now_rfc3339_micro(now), "leaderTransitions": 0}
        try:
            old = await self.lock.get()
            if old is None:
                await self.lock.create(rec)
                return True
            renew = parse_rfc3339(old.get("renewTime")) or 0
            if old.get("holderIdentity") not in ("", self.identity) and renew + float(old.get("leaseDurationSeconds", 15)) > now:
                return False
            if old.get("holderIdentity") == self.identity:
                rec["acquireTime"] = old.get("acquireTime") or rec["acquireTime"]
                rec["leaderTransitions"] = old.get("leaderTransitions", 0)
            else:
                rec["leaderTransitions"] = int(old.get("leaderTransitions", 0)) + 1
            await self.lock.update(rec)
            return True
        except APIStatusError as e:
            if is_conflict(e) or e.code == 409:
                return False
            raise

    async def acquire(self):
        while not await self.try_acquire_or_renew():
            await asyncio.sleep(self.retry_period)
        self.is_leader = True
        log.info("%s became leader of %s", self.identity, self.lock.name)
        if self.on_started:
            self.on_started()
        self._renewer = asyncio.ensure_future(self._renew_loop())

    async def _renew_loop(self):
        last_ok = time.monotonic()
        while self.is_leader:
            await asyncio.sleep(self.retry_period)
            try:
                ok = await self.try_acquire_or_renew()
            except Exception:
                ok = False
            if ok:
                last_ok = time.monotonic()
            elif time.monotonic() - last_ok > self.renew_deadline:
                self.is_leader = False
                log.warning("%s lost leadership", self.identity)
                if self.on_stopped:
                    self.on_stopped()

    async def release(self):
        self.is_leader = False
        if self._renewer:
            self._renewer.cancel()
        try:
            old = await self.lock.get()
            if old and old.get("holderIdentity") == self.identity:
                old["holderIdentity"] = ""
                old["renewTime"] = now_rfc3339_micro(0)
                await self.lock.update(old)
        except APIStatusError:
            pass
