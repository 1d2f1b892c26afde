"""utiltrace: step-timed traces that are logged only when the whole operation was slow.

Parity: `staging/src/k8s.io/apiserver/pkg/util/trace/trace.go:33-79` (`New`, `Step`,
`LogIfLong`, `TotalTime`); used around scheduling (`generic_scheduler.go:110-111`, 100 ms) and
the API server's create/update/delete paths (500 ms).
"""
from __future__ import annotations

import logging
import time

log = logging.getLogger("trace")


class Trace:
    __slots__ = ("name", "start", "steps")

    def __init__(self, name: str):
        self.name = name
        self.start = time.perf_counter()
        self.steps = []

    def step(self, msg: str):
        self.steps.append((time.perf_counter(), msg))

    def total(self) -> float:
        return time.perf_counter() - self.start

    def log_if_long(self, threshold: float, logger=None) -> bool:
        end = time.perf_counter()
        if end - self.start < threshold:
            return False
        lines = [f'Trace "{self.name}" (started {time.strftime("%H:%M:%S")}) total {1e3 * (end - self.start):.1f} ms:']
        last = self.start
        for t, msg in self.steps:
            lines.append(f"  [{1e3 * (t - self.start):.1f} ms] [{1e3 * (t - last):.1f} ms] {msg}")
            last = t
        lines.append(f'  [{1e3 * (end - self.start):.1f} ms] [{1e3 * (end - last):.1f} ms] END')
        (logger or log).warning("\n".join(lines))
        return True
