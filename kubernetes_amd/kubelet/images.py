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


def validate_image_gc_policy(high, low):
    """image_gc_manager.go NewImageGCManager checks."""
    if not 0 <= high <= 100:
        raise ValueError(f"invalid HighThresholdPercent {high}, must be in range [0-100]")
    if not 0 <= low <= 100:
        raise ValueError(f"invalid LowThresholdPercent {low}, must be in range [0-100]")
    if low > high:
        raise ValueError(f"LowThresholdPercent {low} can not be higher than HighThresholdPercent {high}")


class ImageGCError(Exception):
    pass


class ImageGCManager:
    """`pkg/kubelet/images/image_gc_manager.go` realImageGCManager.

    Records per image ID: first detected (the zero time for images present at the first
    detection, so a restarted kubelet can reclaim them at once), last used (refreshed whenever a
    container on the node uses it) and size; records of images that disappeared are dropped.
    `free_space(n)` removes unused images least-recently-used first (ties: earliest detected),
    skipping those used at or after the free time and those younger than `min_age`, until n bytes
    are freed; removal errors are collected and raised after the pass. `garbage_collect()` runs
    when image-fs usage reaches `high`% and frees down to `low`%; freeing less than that is an
    error, as is a zero-capacity filesystem.
    """

    def __init__(self, service, capacity_bytes, in_use, high=85, low=80, min_age=120.0, clock=time.time,
                 last_used=None, recorder=None):
        """in_use() -> set of image IDs / refs used by containers that exist on the node."""
        validate_image_gc_policy(high, low)
        self.service = service
        self.capacity = capacity_bytes
        self.in_use = in_use
        self.high, self.low = high, low
        self.min_age = min_age
        self.clock = clock
        self.records: dict[str, dict] = {}
        self.initialized = False
        self.freed_total = 0
        self.recorder = recorder          # (type, reason, message) -> None
        for iid, t in (last_used or {}).items():
            self.records[iid] = {"first": 0.0, "last": t, "size": 0}

    # back-compat views used by the kubelet / tests
    @property
    def first_seen(self):
        return {k: r["first"] for k, r in self.records.items()}

    @property
    def last_used(self):
        return {k: r["last"] for k, r in self.records.items()}

    @staticmethod
    def _used(img, used):
        return img["id"] in used or any(t in used for t in img.get("repoTags") or ())

    async def detect(self, detect_time=None):
        """detectImages: a first detection stamps images with the zero time."""
        if detect_time is None:
            detect_time = self.clock() if self.initialized else 0.0
        self.initialized = True
        imgs = await self.service.list_images()
        now = self.clock()
        used = self.in_use()
        current = set()
        for i in imgs:
            current.add(i["id"])
            rec = self.records.setdefault(i["id"], {"first": detect_time, "last": 0.0, "size": 0})
            if self._used(i, used):
                rec["last"] = now
            rec["size"] = int(i.get("size") or 0)
        for k in list(self.records):
            if k not in current:
                del self.records[k]
        return imgs

    async def free_space(self, want, free_time=None):
        """freeSpace: returns bytes freed; raises ImageGCError after the pass if removals failed."""
        if free_time is None:
            free_time = self.clock()
        imgs = {i["id"]: i for i in await self.detect(free_time)}
        used = self.in_use()
        cands = [(k, r) for k, r in self.records.items() if not (k in imgs and self._used(imgs[k], used))]
        cands.sort(key=lambda kr: (kr[1]["last"], kr[1]["first"]))
        freed, errors = 0, []
        for k, r in cands:
            if r["last"] >= free_time:
                continue                  # used since the free started
            if free_time - r["first"] < self.min_age:
                continue
            try:
                await self.service.remove_image(k)
            except Exception as e:        # continue despite errors
                errors.append(f"{k}: {e}")
                continue
            del self.records[k]
            freed += r["size"]
            if freed >= want:
                break
        self.freed_total += freed
        if errors:
            raise ImageGCError(f"wanted to free {want} bytes, but freed {freed} bytes space with errors in image "
                               f"deletion: {errors}")
        return freed

    async def delete_unused_images(self):
        """DeleteUnusedImages: free every unused image (eviction's image reclaim)."""
        return await self.free_space(1 << 62, self.clock())

    async def _fs_stats(self):
        fs = await self.service.image_fs_info()
        cap = int(fs.get("capacityBytes") or self.capacity or 0)
        if fs.get("availableBytes") is not None:
            avail = int(fs["availableBytes"])
        else:
            avail = cap - int(fs.get("usedBytes") or 0)
        return cap, min(max(avail, 0), cap)

    async def garbage_collect(self):
        """GarbageCollect: returns bytes freed (0 below the high threshold)."""
        cap, avail = await self._fs_stats()
        if cap <= 0:
            if self.recorder:
                self.recorder("Warning", "InvalidDiskCapacity", "invalid capacity 0 on image filesystem")
            raise ImageGCError("invalid capacity 0 on image filesystem")
        usage_pct = 100 - avail * 100 // cap
        if usage_pct < self.high:
            return 0
        amount = cap * (100 - self.low) // 100 - avail
        freed = await self.free_space(amount, self.clock())
        if freed < amount:
            msg = (f"failed to garbage collect required amount of images. Wanted to free {amount} bytes, "
                   f"but freed {freed} bytes")
            if self.recorder:
                self.recorder("Warning", "FreeDiskSpaceFailed", msg)
            raise ImageGCError(msg)
        return freed
