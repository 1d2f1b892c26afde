"""Image pulling and image garbage collection.

Parity:
  * `pkg/kubelet/images/image_manager.go` — `EnsureImageExists`: pull policy Always /
    IfNotPresent / Never (default from `pkg/apis/core/v1/defaults.go`: Always for `:latest` or
    untagged images, IfNotPresent otherwise), events Pulling / Pulled / Failed /
    ErrImageNeverPull, and a per-image exponential back-off (`ImagePullBackOff`,
    10 s doubling to 300 s: `pkg/kubelet/kubelet.go` backOffPeriod / MaxContainerBackOff);
  * `pkg/kubelet/images/image_gc_manager.go` — `GarbageCollect`: when image-fs usage exceeds
    `HighThresholdPercent` (85), delete images not used by any container, least recently
    used first and older than `MinAge`, until usage drops to `LowThresholdPercent` (80).
"""
from __future__ import annotations

import time


class ImagePullError(Exception):
    def __init__(self, reason, message):
        super().__init__(message)
        self.reason = reason
        self.message = message


def default_pull_policy(image: str) -> str:
    ref = image.split("@")[0]
    last = ref.rsplit("/", 1)[-1]
    if "@" in image:
        return "IfNotPresent"
    if ":" not in last or last.endswith(":latest"):
        return "Always"
    return "IfNotPresent"


class ImageManager:
    """`serialize` (--serialize-image-pulls, default true): one pull at a time
    (`serialImagePuller`), else concurrent pulls (`parallelImagePuller`); `qps`/`burst`
    (--registry-qps 5 / --registry-burst 10; qps 0 = unlimited): pulls go through a token bucket
    (`throttleImagePulling`), and a pull over the limit fails with "pull QPS exceeded" so the
    pod retries after its back-off, as in the reference."""

    def __init__(self, service, recorder=None, backoff_initial=10.0, backoff_max=300.0, clock=time.monotonic,
                 secret_getter=None, serialize=False, qps=0.0, burst=10):
        import asyncio
        self.service = service
        self._serial = asyncio.Lock() if serialize else None
        self.qps, self.burst = float(qps or 0), int(burst)
        self._tokens, self._t = float(burst), clock()
        # async (namespace, name) -> Secret, for the pod's imagePullSecrets keyring
        self.secret_getter = secret_getter
        self.recorder = recorder
        self.backoff_initial = backoff_initial
        self.backoff_max = backoff_max
        self.clock = clock
        self._backoff: dict[str, tuple] = {}   # image -> (next allowed time, current period)
        self.last_used: dict[str, float] = {}  # image id -> wall time
        self.pulls = 0

    def _event(self, pod, typ, reason, msg):
        if self.recorder is not None:
            self.recorder.event(pod, typ, reason, msg)

    async def ensure_image_exists(self, pod, container) -> str:
        image = container.get("image") or ""
        if not image:
            raise ImagePullError("InvalidImageName", "container has no image")
        policy = container.get("imagePullPolicy") or default_pull_policy(image)
        present = await self.service.image_status(image)
        if present is not None and policy != "Always":
            self.last_used[present["id"]] = time.time()
            # image_manager.go EnsureImageExists: "already present" is reported every time
            self._event(pod, "Normal", "Pulled", f'Container image "{image}" already present on machine')
            return present["id"]
        if policy == "Never":
            msg = f'Container image "{image}" is not present with pull policy of Never'
            self._event(pod, "Warning", "ErrImageNeverPull", msg)
            raise ImagePullError("ErrImageNeverPull", msg)
        now = self.clock()
        b = self._backoff.get(image)
        if b is not None and now < b[0]:
            msg = f'Back-off pulling image "{image}"'
            self._event(pod, "Normal", "BackOff", msg)
            raise ImagePullError("ImagePullBackOff", msg)
        self._event(pod, "Normal", "Pulling", f'pulling image "{image}"')
        try:
            if not self._take_token():
                raise RuntimeError("pull QPS exceeded")
            if self._serial is not None:
                async with self._serial:
                    ref = await self._pull(pod, image)
            else:
                ref = await self._pull(pod, image)
        except Exception as e:
            period = min(self.backoff_max, b[1] * 2) if b else self.backoff_initial
            self._backoff[image] = (now + period, period)
            self._event(pod, "Warning", "Failed", f'Failed to pull image "{image}": {e}')
            raise ImagePullError("ErrImagePull", str(e))
        self._backoff.pop(image, None)
        self.pulls += 1
        self.last_used[ref] = time.time()
        self._event(pod, "Normal", "Pulled", f'Successfully pulled image "{image}"')
        return ref

    def _take_token(self) -> bool:
        if self.qps <= 0:
            return True
        now = self.clock()
        self._tokens = min(float(self.burst), self._tokens + (now - self._t) * self.qps)
        self._t = now
        if self._tokens < 1.0:
            return False
        self._tokens -= 1.0
        return True

    async def _pull(self, pod, image):
        """`kuberuntime_image.go PullImage`: try every matching pull-secret credential in turn
        (then none), like the reference keyring lookup."""
        auths = []
        names = [s.get("name") for s in (pod.get("spec") or {}).get("imagePullSecrets") or () if s.get("name")]
        if names and self.secret_getter is not None:
            from ..images.credentials import keyring_from_secrets
            secrets = []
            for n in names:
                try:
                    secrets.append(await self.secret_getter(pod["metadata"].get("namespace", "default"), n))
                except Exception:   # noqa: BLE001 - a missing pull secret only removes a credential
                    continue
            try:
                auths = keyring_from_secrets(secrets).lookup(image)
            except ValueError:
                auths = []
        if not auths:
            return await self.service.pull_image(image)
        err = None
        for a in auths:
            try:
                return await self.service.pull_image(image, a)
            except Exception as e:  # noqa: BLE001 - the next credential may work
                err = e
        raise err

    def retry_after(self, image):
        b = self._backoff.get(image)
        return max(0.0, b[0] - self.clock()) if b else 0.0


class ImageGCManager:
    def __init__(self, service, capacity_bytes, in_use, high=85, low=80, min_age=120.0, clock=time.time,
                 last_used=None):
        """in_use() -> set of image refs/tags used by containers that exist on the node."""
        if not 0 <= low < high <= 100:
            raise ValueError("LowThresholdPercent must be less than HighThresholdPercent")
        self.service = service
        self.capacity = capacity_bytes
        self.in_use = in_use
        self.high, self.low = high, low
        self.min_age = min_age
        self.clock = clock
        self.first_seen: dict[str, float] = {}
        self.last_used = last_used if last_used is not None else {}
        self.freed_total = 0

    async def detect(self):
        imgs = await self.service.list_images()
        now = self.clock()
        used = self.in_use()
        for i in imgs:
            self.first_seen.setdefault(i["id"], now)
            if i["id"] in used or any(t in used for t in i["repoTags"]):
                self.last_used[i["id"]] = now
        return imgs

    async def garbage_collect(self):
        """Returns bytes freed."""
        fs = await self.service.image_fs_info()
        usage = fs["usedBytes"]
        if self.capacity <= 0 or usage * 100 < self.high * self.capacity:
            return 0
        target = usage - self.low * self.capacity // 100
        return await self.free_space(target)

    async def free_space(self, want):
        imgs = await self.detect()
        used = self.in_use()
        now = self.clock()
        cands = [i for i in imgs if i["id"] not in used and not any(t in used for t in i["repoTags"])]
        cands.sort(key=lambda i: (self.last_used.get(i["id"], 0.0), self.first_seen.get(i["id"], now)))
        freed = 0
        for i in cands:
            if freed >= want:
                break
            if now - self.first_seen.get(i["id"], now) < self.min_age:
                continue
            await self.service.remove_image(i["id"])
            self.first_seen.pop(i["id"], None)
            self.last_used.pop(i["id"], None)
            freed += i["size"]
        self.freed_total += freed
        return freed
