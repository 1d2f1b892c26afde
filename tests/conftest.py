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


def pytest_sessionfinish(session, exitstatus):
    """No test may leave processes behind (containers of the process runtime, store servers,
    writer processes): whatever is still a descendant of the test session at the end is killed
    and fails the run."""
    try:
        import psutil
    except ImportError:
        return
    import time
    me = psutil.Process()
    deadline = time.time() + 5
    left = []
    while time.time() < deadline:
        left = [p for p in me.children(recursive=True) if p.is_running() and p.status() != psutil.STATUS_ZOMBIE]
        if not left:
            return
        time.sleep(0.2)
    desc = []
    for p in left:
        try:
            desc.append(f"{p.pid} {' '.join(p.cmdline())[:120]}")
            p.kill()
        except psutil.NoSuchProcess:
            pass
    print("\nleaked processes killed at session end:\n  " + "\n  ".join(desc))
    if session.exitstatus == 0:
        session.exitstatus = 1
