"""Image GC manager tables ported from `pkg/kubelet/images/image_gc_manager_test.go`.

A fake image service stands in for the runtime's image list and the image-fs stats provider;
a fake clock that advances on every read makes "time.Now()" strictly increasing, as the Go
tests rely on wall-clock ordering between detections.
"""
import pytest

from kubernetes_amd.kubelet.images import ImageGCError, ImageGCManager, validate_image_gc_policy


class FakeImages:
    def __init__(self):
        self.images = []
        self.fs = {}
        self.fs_error = None

    async def list_images(self):
        return [dict(i) for i in self.images]

    async def remove_image(self, iid):
        self.images = [i for i in self.images if i["id"] != iid]

    async def image_fs_info(self):
        if self.fs_error:
            raise self.fs_error
        return dict(self.fs)


def image_id(n):
    return f"image-{n}"


def make_image(n, size):
    return {"id": image_id(n), "size": size, "repoTags": []}


class Clock:
    def __init__(self, t=1000.0):
        self.t = t

    def __call__(self):
        self.t += 0.001
        return self.t


def manager(high=0, low=0, min_age=0.0):
    svc, clock, used = FakeImages(), Clock(), set()
    gc = ImageGCManager(svc, 0, lambda: set(used), high=high, low=low, min_age=min_age, clock=clock)
    return gc, svc, used, clock


def test_detect_images_initial_detect(run):
    gc, svc, used, clock = manager()
    svc.images = [make_image(0, 1024), make_image(1, 2048), make_image(2, 2048)]
    used |= {image_id(1), image_id(2)}               # container 1 runs a no-name image
    start = clock.t
    run(gc.detect(0.0))
    assert len(gc.records) == 3
    assert gc.records[image_id(0)] == {"first": 0.0, "last": 0.0, "size": 1024}
    for n in (1, 2):
        assert gc.records[image_id(n)]["first"] == 0.0
        assert gc.records[image_id(n)]["last"] > start


def test_detect_images_with_new_image(run):
    gc, svc, used, clock = manager()
    svc.images = [make_image(0, 1024), make_image(1, 2048)]
    used.add(image_id(1))
    run(gc.detect(0.0))
    assert len(gc.records) == 2
    svc.images = [make_image(0, 1024), make_image(1, 1024), make_image(2, 1024)]
    start = clock.t
    run(gc.detect(1.0))
    assert len(gc.records) == 3
    assert gc.records[image_id(0)]["first"] == 0.0 and gc.records[image_id(0)]["last"] == 0.0
    assert gc.records[image_id(1)]["first"] == 0.0 and gc.records[image_id(1)]["last"] > start
    assert gc.records[image_id(2)]["first"] == 1.0 and gc.records[image_id(2)]["last"] == 0.0
    assert gc.records[image_id(1)]["size"] == 1024   # size refreshed


def test_detect_images_container_stopped(run):
    gc, svc, used, clock = manager()
    svc.images = [make_image(0, 1024), make_image(1, 2048)]
    used.add(image_id(1))
    run(gc.detect(0.0))
    last = gc.records[image_id(1)]["last"]
    used.clear()
    run(gc.detect(clock()))
    assert len(gc.records) == 2
    assert gc.records[image_id(0)]["first"] == 0.0 and gc.records[image_id(0)]["last"] == 0.0
    assert gc.records[image_id(1)]["first"] == 0.0 and gc.records[image_id(1)]["last"] == last


def test_detect_images_with_removed_images(run):
    gc, svc, used, clock = manager()
    svc.images = [make_image(0, 1024), make_image(1, 2048)]
    used.add(image_id(1))
    run(gc.detect(0.0))
    assert len(gc.records) == 2
    svc.images = []
    run(gc.detect(clock()))
    assert len(gc.records) == 0


def test_free_space_images_in_use_containers_are_ignored(run):
    gc, svc, used, clock = manager()
    svc.images = [make_image(0, 1024), make_image(1, 2048)]
    used.add(image_id(1))
    assert run(gc.free_space(2048, clock())) == 1024
    assert len(svc.images) == 1


def test_delete_unused_images_remove_all_unused_images(run):
    gc, svc, used, clock = manager()
    svc.images = [make_image(0, 1024), make_image(1, 2048), make_image(2, 2048)]
    used.add(image_id(2))
    assert run(gc.delete_unused_images()) == 3072
    assert [i["id"] for i in svc.images] == [image_id(2)]


def test_free_space_remove_by_least_recently_used(run):
    gc, svc, used, clock = manager()
    svc.images = [make_image(0, 1024), make_image(1, 2048)]
    used |= {image_id(0), image_id(1)}
    run(gc.detect(0.0))
    used.discard(image_id(0))                         # 1 used more recently than 0
    run(gc.detect(clock()))
    used.clear()
    run(gc.detect(clock()))
    assert len(gc.records) == 2
    assert run(gc.free_space(1024, clock())) == 1024
    assert [i["id"] for i in svc.images] == [image_id(1)]


def test_free_space_ties_broken_by_detected_time(run):
    gc, svc, used, clock = manager()
    svc.images = [make_image(0, 1024)]
    used.add(image_id(0))
    run(gc.detect(0.0))
    svc.images = [make_image(0, 1024), make_image(1, 2048)]
    run(gc.detect(clock()))
    used.clear()
    run(gc.detect(clock()))
    assert len(gc.records) == 2
    assert run(gc.free_space(1024, clock())) == 2048
    assert len(svc.images) == 1


def test_free_space_equal_last_used_prefers_earliest_detected(run):
    """byLastUsedAndDetected: with equal lastUsed the earlier-detected image goes first."""
    gc, svc, used, clock = manager()
    svc.images = [make_image(0, 1024)]
    run(gc.detect(5.0))
    svc.images = [make_image(0, 1024), make_image(1, 1024)]
    run(gc.detect(3.0))                               # image-1 detected "earlier" (3 < 5)
    assert run(gc.free_space(1, clock())) == 1024
    assert [i["id"] for i in svc.images] == [image_id(0)]


def test_garbage_collect_below_low_threshold(run):
    gc, svc, used, clock = manager(high=90, low=80)
    svc.fs = {"availableBytes": 600, "capacityBytes": 1000}          # 40% usage
    assert run(gc.garbage_collect()) == 0


def test_garbage_collect_stats_failure(run):
    gc, svc, used, clock = manager(high=90, low=80)
    svc.fs_error = RuntimeError("error")
    with pytest.raises(RuntimeError):
        run(gc.garbage_collect())


def test_garbage_collect_below_success(run):
    gc, svc, used, clock = manager(high=90, low=80)
    svc.fs = {"availableBytes": 50, "capacityBytes": 1000}           # 95% usage, most gets freed
    svc.images = [make_image(0, 450)]
    assert run(gc.garbage_collect()) == 450


def test_garbage_collect_not_enough_freed(run):
    gc, svc, used, clock = manager(high=90, low=80)
    events = []
    gc.recorder = lambda *e: events.append(e)
    svc.fs = {"availableBytes": 50, "capacityBytes": 1000}
    svc.images = [make_image(0, 50)]
    with pytest.raises(ImageGCError, match="Wanted to free 150 bytes, but freed 50 bytes"):
        run(gc.garbage_collect())
    assert events[0][:2] == ("Warning", "FreeDiskSpaceFailed")


def test_garbage_collect_zero_capacity(run):
    gc, svc, used, clock = manager(high=90, low=80)
    events = []
    gc.recorder = lambda *e: events.append(e)
    svc.fs = {"availableBytes": 0, "capacityBytes": 0}
    with pytest.raises(ImageGCError, match="invalid capacity 0 on image filesystem"):
        run(gc.garbage_collect())
    assert events[0][1] == "InvalidDiskCapacity"


def test_garbage_collect_image_not_old_enough(run):
    svc, used = FakeImages(), {image_id(1)}
    now = [5000.0]
    gc = ImageGCManager(svc, 0, lambda: used, high=90, low=80, min_age=60.0, clock=lambda: now[0])
    svc.images = [make_image(0, 1024), make_image(1, 2048)]
    run(gc.detect(now[0]))
    assert len(gc.records) == 2
    assert run(gc.free_space(1024, now[0])) == 0      # one in use, the other too young
    assert len(svc.images) == 2
    now[0] += 60.0
    assert run(gc.free_space(1024, now[0])) == 1024
    assert len(svc.images) == 1


def test_free_space_reports_removal_errors(run):
    gc, svc, used, clock = manager()
    svc.images = [make_image(0, 10), make_image(1, 20)]

    async def boom(iid):
        if iid == image_id(0):
            raise RuntimeError("device busy")
        svc.images = [i for i in svc.images if i["id"] != iid]
    svc.remove_image = boom
    with pytest.raises(ImageGCError, match="freed 20 bytes space with errors"):
        run(gc.free_space(100, clock()))
    assert [i["id"] for i in svc.images] == [image_id(0)]


@pytest.mark.parametrize("high,low,err", [
    (2, 1, None),
    (-1, 0, "invalid HighThresholdPercent -1, must be in range [0-100]"),
    (101, 0, "invalid HighThresholdPercent 101, must be in range [0-100]"),
    (0, -1, "invalid LowThresholdPercent -1, must be in range [0-100]"),
    (0, 101, "invalid LowThresholdPercent 101, must be in range [0-100]"),
    (1, 2, "LowThresholdPercent 2 can not be higher than HighThresholdPercent 1"),
])
def test_validate_image_gc_policy(high, low, err):
    if err is None:
        validate_image_gc_policy(high, low)
        ImageGCManager(FakeImages(), 0, set, high=high, low=low)
    else:
        with pytest.raises(ValueError, match=__import__("re").escape(err)):
            validate_image_gc_policy(high, low)
        with pytest.raises(ValueError):
            ImageGCManager(FakeImages(), 0, set, high=high, low=low)
