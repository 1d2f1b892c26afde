"""Race detection / sanitizer tier.

The reference runs Go's race detector on its unit tests (`KUBE_RACE=-race`,
`hack/make-rules/test.sh:107`) and forces interleavings with instrumented shims
(`pkg/kubelet/cm/devicemanager/endpoint_store_shim.go`). Here the native host code gets the
equivalent: ASan+UBSan builds of the MVCC store (a differential fuzz of the engine, and the
kamd-etcd server driven by the shared-store API-server tests), a TSan build of the AMD SMI shim
under a multi-threaded stress, and the asyncio side runs a concurrency-heavy subset in asyncio
debug mode (never-awaited coroutines and callbacks on the wrong loop fail). GPU-side sanitizers
are not available on the MI355X pool, so none of this touches the device.
"""
import os
import subprocess
import sys

import pytest

from kubernetes_amd.native import amdsmi
from kubernetes_amd.native.build import SAN_DIR, build

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN_REPORT = ("ERROR: AddressSanitizer", "ERROR: LeakSanitizer", "runtime error:", "WARNING: ThreadSanitizer")


@pytest.fixture(scope="module")
def san_build():
    build(sanitize=True, verbose=False)
    return SAN_DIR


def _clean(text):
    return not any(s in text for s in SAN_REPORT)


@pytest.mark.parametrize("seed", [1, 7, 1234])
def test_store_engine_fuzz_asan_ubsan(san_build, tmp_path, seed):
    wal = str(tmp_path / "fuzz.wal")
    r = subprocess.run([os.path.join(san_build, "asan", "store_fuzz"), "15000", str(seed), wal],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and _clean(r.stderr), r.stderr[-3000:]
    assert "OK" in r.stdout


def test_smi_shim_threads_tsan(san_build):
    fx = amdsmi.fixture_file(8, seed="tsan")
    r = subprocess.run([os.path.join(san_build, "tsan", "smi_threads"), fx, "8", "3000"],
                       capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1"))
    assert r.returncode == 0 and _clean(r.stderr), r.stderr[-3000:]


def test_shared_store_server_asan(san_build, tmp_path):
    """The multi-worker API server tests (cross-worker CAS, watches, device claims, restarts)
    and the remote store client, against the ASan/UBSan build of kamd-etcd; the server exits
    cleanly on SIGTERM so LeakSanitizer also runs."""
    logs = tmp_path / "etcd-logs"
    env = dict(os.environ, KAMD_ETCD_BIN=os.path.join(san_build, "asan", "kamd-etcd"), KAMD_ETCD_LOG_DIR=str(logs),
               ASAN_OPTIONS="detect_leaks=1 abort_on_error=0")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        "tests/test_apiserver_shared.py", "tests/test_store.py::test_remote_store_server"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    files = list(logs.iterdir())
    assert files, "the sanitized server never ran"
    for f in files:
        text = f.read_text(errors="replace")
        assert _clean(text), f"{f.name}:\n{text[-4000:]}"


def test_shared_store_server_tsan(san_build, tmp_path):
    """kamd-etcd runs a store thread and watch fan-out threads (here 3) that share the event
    queues, the KV objects' lifetimes and (per-thread slots of) their parse cache: the multi-worker
    API server suite against its TSan build."""
    logs = tmp_path / "etcd-logs"
    env = dict(os.environ, KAMD_ETCD_BIN=os.path.join(san_build, "tsan", "kamd-etcd"), KAMD_ETCD_LOG_DIR=str(logs),
               KAMD_ETCD_FAN_THREADS="3",
               TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        "tests/test_apiserver_shared.py"], cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    files = list(logs.iterdir())
    assert files, "the sanitized server never ran"
    for f in files:
        text = f.read_text(errors="replace")
        assert _clean(text), f"{f.name}:\n{text[-4000:]}"


def test_asyncio_debug_mode_devicemanager_and_scheduler():
    """asyncio debug mode over the device-manager / scheduler suites: a coroutine that is
    never awaited or a loop-thread violation is an error, not a silent warning."""
    env = dict(os.environ, PYTHONASYNCIODEBUG="1", PYTHONWARNINGS="error::RuntimeWarning")
    r = subprocess.run([sys.executable, "-X", "dev", "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        "-W", "error::RuntimeWarning", "tests/test_devicemanager.py", "tests/test_scheduler.py"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "was never awaited" not in out, out[-4000:]
    assert "Non-thread-safe operation" not in out, out[-4000:]
