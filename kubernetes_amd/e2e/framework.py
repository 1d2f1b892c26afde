"""e2e framework: conformance-style specs that run against ANY cluster URL.

Parity: `test/e2e/framework/framework.go` (per-spec namespace created before and deleted after
each spec, client, wait helpers; `ConformanceIt` at :647 tags the conformance subset) and the
ginkgo focus/skip selection. Specs are async functions registered with `@conformance` (or
`@spec` for non-conformance / feature-gated ones such as `[Feature:GPU]`).

    python -m kubernetes_amd.e2e --server http://127.0.0.1:8080 --focus Conformance
"""
from __future__ import annotations

import asyncio
import re
import time
import traceback
import uuid

from ..client.rest import APIStatusError, Client

SPECS: list[tuple[str, object, tuple]] = []


def spec(name, *tags):
    def deco(fn):
        SPECS.append((name, fn, tags))
        return fn
    return deco


def conformance(name, *tags):
    return spec(f"[Conformance] {name}", "Conformance", *tags)


class Skip(Exception):
    """Raised by a spec whose prerequisites the cluster lacks (ginkgo's `framework.Skipf`, e.g.
    `SkipUnlessNodeCountIsAtLeast`): reported as SKIP, neither pass nor failure."""


class Framework:
    def __init__(self, client, base_name="e2e"):
        self.client = client
        self.ns = f"{base_name}-{uuid.uuid4().hex[:6]}"

    async def setup(self):
        await self.client.create("namespaces", {"metadata": {"name": self.ns, "labels": {"e2e-run": "true"}}})

    async def teardown(self):
        try:
            await self.client.delete("namespaces", self.ns)
        except APIStatusError:
            pass

    async def wait(self, pred, timeout=60.0, what="condition"):
        end = time.monotonic() + timeout
        last = None
        while time.monotonic() < end:
            try:
                last = await pred()
            except APIStatusError as e:
                last = e
                if e.code != 404:
                    raise
            if last and not isinstance(last, Exception):
                return last
            await asyncio.sleep(0.1)
        raise TimeoutError(f"timed out waiting for {what} (last={last!r:.200})")

    async def pod_phase(self, name, phases=("Running", "Succeeded"), timeout=60.0):
        async def check():
            p = await self.client.get("pods", name, self.ns)
            if (p.get("status") or {}).get("phase") == "Failed" and "Failed" not in phases:
                raise AssertionError(f"pod {name} failed: {p.get('status')}")
            return p if (p.get("status") or {}).get("phase") in phases else None
        return await self.wait(check, timeout, f"pod {self.ns}/{name} in {phases}")

    async def logs(self, name, container=None):
        q = f"?container={container}" if container else ""
        st, body = await self.client.raw("GET", f"/api/v1/namespaces/{self.ns}/pods/{name}/log{q}")
        if st != 200:
            raise AssertionError(f"logs of {name}: HTTP {st} {body[:200]!r}")
        return body.decode(errors="replace")


class Result:
    def __init__(self, name, ok, seconds, error="", skipped=False):
        self.name, self.ok, self.seconds, self.error = name, ok, seconds, error
        self.skipped = skipped


async def run_specs(server, focus=None, skip=None, token=None, ssl_context=None, timeout=180.0, out=print):
    client = Client(server, token=token, ssl_context=ssl_context)
    results = []
    try:
        for name, fn, tags in SPECS:
            label = name + "".join(f" [{t}]" for t in tags if t != "Conformance")
            if focus and not re.search(focus, label):
                continue
            if skip and re.search(skip, label):
                continue
            f = Framework(client)
            t0 = time.monotonic()
            try:
                await f.setup()
                await asyncio.wait_for(fn(f), timeout)
                results.append(Result(label, True, time.monotonic() - t0))
                out(f"  PASS  {label} ({time.monotonic() - t0:.2f}s)")
            except Skip as e:
                results.append(Result(label, True, time.monotonic() - t0, str(e), skipped=True))
                out(f"  SKIP  {label}: {e}")
            except Exception as e:  # noqa: BLE001 - a failing spec is a result, not a crash
                results.append(Result(label, False, time.monotonic() - t0, f"{type(e).__name__}: {e}\n"
                                                                          f"{traceback.format_exc(limit=3)}"))
                out(f"  FAIL  {label}: {type(e).__name__}: {e}")
            finally:
                await f.teardown()
    finally:
        await client.close()
    return results
