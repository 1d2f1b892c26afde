import asyncio
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture
def run():
    """Run a coroutine to completion on a fresh event loop."""
    def _run(coro, timeout=60):
        return asyncio.run(asyncio.wait_for(coro, timeout))
    return _run


_SESSION_START = [0.0]


@pytest.fixture
def feature_gate():
    """The process-wide feature gate, restored after the test (`--feature-gates` in-process)."""
    from kubernetes_amd.utils.features import DefaultFeatureGate
    saved = dict(DefaultFeatureGate.enabled)
    yield DefaultFeatureGate
    DefaultFeatureGate.enabled = saved


def pytest_sessionstart(session):
    import time
    _SESSION_START[0] = time.time()


def _session_tmp_roots(session):
    """Temp directories this session made: pytest's basetemp and every /tmp/kamd-* (and
    kamd-*-named tempfile.mkdtemp) directory created after the session started."""
    import glob
    import tempfile
    roots = []
    try:
        roots.append(str(session.config._tmp_path_factory.getbasetemp()))
    except Exception:  # noqa: BLE001 - no tmp_path used
        pass
    for d in glob.glob(os.path.join(tempfile.gettempdir(), "kamd-*")):
        try:
            if os.path.isdir(d) and os.stat(d).st_ctime >= _SESSION_START[0] - 1:
                roots.append(d)
        except OSError:
            pass
    return [r.rstrip("/") + "/" for r in roots]


def _orphans(me, roots):
    """Processes started during the session that are no longer its descendants (reparented to
    init: containers a stopped kubelet left running) but whose working directory or command line
    lives under one of the session's temp directories — so never anything else on the host."""
    import psutil
    mine = {p.pid for p in me.children(recursive=True)} | {me.pid}
    out = []
    for p in psutil.process_iter(["pid", "create_time", "uids", "cmdline"]):
        try:
            if p.pid in mine or p.info["create_time"] < _SESSION_START[0] - 1:
                continue
            if p.info["uids"] is None or p.info["uids"].real != os.getuid():
                continue
            where = [p.cwd()] + list(p.info["cmdline"] or ())
            if any(w.startswith(r) or w.rstrip("/") + "/" == r for w in where for r in roots):
                out.append(p)
        except (psutil.NoSuchProcess, psutil.AccessDenied, psutil.ZombieProcess):
            continue
    return out


def pytest_sessionfinish(session, exitstatus):
    """No test may leave processes behind (containers of the process runtime, store servers,
    writer processes): whatever is still a descendant of the test session at the end — or was
    started by it, got reparented, and still runs out of the session's temp directories — is
    killed and fails the run."""
    try:
        import psutil
    except ImportError:
        return
    import time
    me = psutil.Process()
    roots = _session_tmp_roots(session)
    deadline = time.time() + 5
    left = []
    while time.time() < deadline:
        left = [p for p in me.children(recursive=True) if p.is_running() and p.status() != psutil.STATUS_ZOMBIE]
        left += _orphans(me, roots) if roots else []
        if not left:
            return
        time.sleep(0.2)
    desc = []
    for p in left:
        try:
            desc.append(f"{p.pid} {' '.join(p.cmdline())[:120]}")
            for c in p.children(recursive=True):
                c.kill()
            p.kill()
        except psutil.NoSuchProcess:
            pass
    print("\nleaked processes killed at session end:\n  " + "\n  ".join(desc))
    if session.exitstatus == 0:
        session.exitstatus = 1
