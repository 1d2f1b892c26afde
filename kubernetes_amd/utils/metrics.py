"""Tiny Prometheus metrics library (text exposition format 0.0.4).

Every component serves `/metrics` like the reference (kubelet `pkg/kubelet/metrics/metrics.go:28-152`,
scheduler `plugin/pkg/scheduler/metrics/metrics.go:33-50`, apiserver
`staging/src/k8s.io/apiserver/pkg/endpoints/metrics/metrics.go`). A per-component
`Registry` (not a process-global one) lets several components share one process in tests
and in the kubemark harness.
"""
from __future__ import annotations

import bisect
import math
import threading

DEFAULT_BUCKETS = (0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10)
# reference scheduler/kubelet latency metrics are microsecond summaries; exponential buckets 1ms..16s
MICRO_BUCKETS = tuple(1000 * (2 ** i) for i in range(15))


def _fmt_labels(names, values, extra=None):
    parts = [f'{n}="{_esc(v)}"' for n, v in zip(names, values)]
    if extra:
        parts.append(extra)
    return "{" + ",".join(parts) + "}" if parts else ""


def _esc(v):
    return str(v).replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n")


def _num(v):
    if v == math.inf:
        return "+Inf"
    if isinstance(v, float) and v.is_integer():
        return repr(v)
    return repr(v) if isinstance(v, float) else str(v)


class _Metric:
    type = "untyped"

    def __init__(self, name, help_, labels=()):
        self.name, self.help, self.labelnames = name, help_, tuple(labels)
        self._children = {}
        self._lock = threading.Lock()

    def labels(self, *values, **kw):
        if kw:
            values = tuple(kw[n] for n in self.labelnames)
        key = tuple(str(v) for v in values)
        c = self._children.get(key)
        if c is None:
            with self._lock:
                c = self._children.setdefault(key, self._new_child())
        return c

    def _default(self):
        return self.labels() if not self.labelnames else None

    def render(self):
        out = [f"# HELP {self.name} {self.help}", f"# TYPE {self.name} {self.type}"]
        for key, c in sorted(self._children.items()):
            out.extend(c.render(self.name, self.labelnames, key))
        return out


class _CounterChild:
    __slots__ = ("v",)

    def __init__(self):
        self.v = 0.0

    def inc(self, n=1):
        self.v += n

    def set(self, v):
        self.v = v

    def dec(self, n=1):
        self.v -= n

    def render(self, name, ln, lv):
        return [f"{name}{_fmt_labels(ln, lv)} {_num(self.v)}"]


class Counter(_Metric):
    type = "counter"

    def _new_child(self):
        return _CounterChild()

    def inc(self, n=1):
        self.labels().inc(n)

    def value(self, *lv):
        return self.labels(*lv).v


class Gauge(Counter):
    type = "gauge"

    def set(self, v):
        self.labels().set(v)


class _HistChild:
    __slots__ = ("buckets", "counts", "sum", "count", "samples")

    def __init__(self, buckets):
        self.buckets = buckets
        self.counts = [0] * (len(buckets) + 1)
        self.sum = 0.0
        self.count = 0

    def observe(self, v):
        self.counts[bisect.bisect_left(self.buckets, v)] += 1
        self.sum += v
        self.count += 1

    def quantile(self, q):
        """Bucket-interpolated quantile (histogram_quantile)."""
        if not self.count:
            return float("nan")
        rank = q * self.count
        acc = 0
        lo = 0.0
        for i, c in enumerate(self.counts):
            if acc + c >= rank:
                hi = self.buckets[i] if i < len(self.buckets) else self.buckets[-1]
                if c == 0:
                    return hi
                return lo + (hi - lo) * (rank - acc) / c
            acc += c
            lo = self.buckets[i] if i < len(self.buckets) else lo
        return self.buckets[-1]

    def render(self, name, ln, lv):
        out, acc = [], 0
        for b, c in zip(self.buckets, self.counts):
            acc += c
            le = 'le="%s"' % _num(float(b))
            out.append(f"{name}_bucket{_fmt_labels(ln, lv, le)} {acc}")
        acc += self.counts[-1]
        le = 'le="+Inf"'
        out.append(f"{name}_bucket{_fmt_labels(ln, lv, le)} {acc}")
        out.append(f"{name}_sum{_fmt_labels(ln, lv)} {_num(self.sum)}")
        out.append(f"{name}_count{_fmt_labels(ln, lv)} {self.count}")
        return out


class Histogram(_Metric):
    type = "histogram"

    def __init__(self, name, help_, labels=(), buckets=DEFAULT_BUCKETS):
        super().__init__(name, help_, labels)
        self.buckets = tuple(sorted(buckets))

    def _new_child(self):
        return _HistChild(self.buckets)

    def observe(self, v):
        self.labels().observe(v)


class Registry:
    def __init__(self):
        self.metrics: list[_Metric] = []
        self.collectors = []

    def add(self, m):
        self.metrics.append(m)
        return m

    def counter(self, name, help_, labels=()):
        return self.add(Counter(name, help_, labels))

    def gauge(self, name, help_, labels=()):
        return self.add(Gauge(name, help_, labels))

    def histogram(self, name, help_, labels=(), buckets=DEFAULT_BUCKETS):
        return self.add(Histogram(name, help_, labels, buckets))

    def register_collector(self, fn):
        """fn() -> iterable of exposition lines (for dynamic metrics such as amd-smi)."""
        self.collectors.append(fn)

    def render(self) -> bytes:
        lines = []
        for m in self.metrics:
            lines.extend(m.render())
        for fn in self.collectors:
            lines.extend(fn())
        return ("\n".join(lines) + "\n").encode()
