"""Process- and host-level checks the kubelet runs before it starts.

Parity (`cmd/kubelet/app/server.go` run(), `pkg/kubelet/cm/container_manager_linux.go`):
* `--fail-swap-on` (default true): refuse to start while swap is enabled (`/proc/swaps` lists a
  device) — "Running with swap on is not supported, please disable swap!";
* `--protect-kernel-defaults`: refuse to start when the kernel tunables the kubelet relies on
  differ from its defaults (`setupKernelTunables` KernelTunableError): vm.overcommit_memory=1,
  vm.panic_on_oom=0, kernel.panic=10, kernel.panic_on_oops=1; without the flag the kubelet only
  logs the difference (it does not rewrite host sysctls here);
* `--max-open-files`: raise RLIMIT_NOFILE (`rlimit.RlimitNumFiles`);
* `--oom-score-adj` (-999): the kubelet's own OOM score (`oom.ApplyOOMScoreAdj(0, ...)`);
* `--lock-file` / `--exit-on-lock-contention`: hold an exclusive flock on the file for the
  kubelet's lifetime, waiting for it if another kubelet holds it; with contention-exit, leave
  as soon as another process opens the file (`watchForLockfileContention`: inotify IN_OPEN |
  IN_DELETE_SELF).
"""
from __future__ import annotations

import ctypes
import ctypes.util
import fcntl
import logging
import os
import resource
import struct
import threading

log = logging.getLogger("kubelet.hostchecks")

KERNEL_DEFAULTS = {"vm/overcommit_memory": 1, "vm/panic_on_oom": 0, "kernel/panic": 10, "kernel/panic_on_oops": 1}
IN_OPEN, IN_DELETE_SELF = 0x20, 0x400


class HostCheckError(Exception):
    pass


def swap_enabled(proc_swaps="/proc/swaps") -> bool:
    try:
        with open(proc_swaps) as f:
            lines = [ln for ln in f.read().splitlines() if ln.strip()]
    except OSError:
        return False
    return len(lines) > 1          # the first line is the header


def check_swap(fail_swap_on: bool, proc_swaps="/proc/swaps"):
    if fail_swap_on and swap_enabled(proc_swaps):
        raise HostCheckError("Running with swap on is not supported, please disable swap! or set --fail-swap-on "
                             "flag to false. /proc/swaps contained swap devices")


def kernel_default_mismatches(root="/proc/sys") -> list[str]:
    out = []
    for key, want in KERNEL_DEFAULTS.items():
        try:
            with open(os.path.join(root, key)) as f:
                got = int(f.read().strip())
        except (OSError, ValueError):
            continue
        if got != want:
            out.append(f"{key.replace('/', '.')}={got} (want {want})")
    return out


def check_kernel_defaults(protect: bool, root="/proc/sys"):
    bad = kernel_default_mismatches(root)
    if bad and protect:
        raise HostCheckError("invalid kernel flags: " + ", ".join(bad) + " (--protect-kernel-defaults)")
    for b in bad:
        log.info("kernel tunable differs from the kubelet default: %s", b)


def set_max_open_files(n: int):
    if n <= 0:
        return
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    want_hard = max(hard, n) if hard != resource.RLIM_INFINITY else hard
    try:
        resource.setrlimit(resource.RLIMIT_NOFILE, (n, want_hard))
    except (ValueError, OSError):
        # unprivileged: raise the soft limit as far as the hard one allows
        try:
            resource.setrlimit(resource.RLIMIT_NOFILE, (min(n, hard) if hard != resource.RLIM_INFINITY else n, hard))
        except (ValueError, OSError) as e:
            log.warning("could not set RLIMIT_NOFILE to %d: %s", n, e)


def set_oom_score_adj(v: int, pid="self"):
    try:
        with open(f"/proc/{pid}/oom_score_adj", "w") as f:
            f.write(str(int(v)))
    except OSError as e:     # lowering it needs CAP_SYS_RESOURCE
        log.info("could not set oom_score_adj %d: %s", v, e)


class LockFile:
    """flock-held lock file; `exit_on_contention` calls `on_contention` when another process
    opens the file (or it is deleted)."""

    def __init__(self, path: str):
        self.path = path
        self.fd = None
        self._ifd = None

    def acquire(self, blocking=True):
        os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
        self.fd = os.open(self.path, os.O_RDWR | os.O_CREAT, 0o600)
        flags = fcntl.LOCK_EX | (0 if blocking else fcntl.LOCK_NB)
        fcntl.flock(self.fd, flags)
        return self

    def watch_contention(self, on_contention):
        libc = ctypes.CDLL(ctypes.util.find_library("c") or "libc.so.6", use_errno=True)
        self._ifd = libc.inotify_init1(0o2000000)     # IN_CLOEXEC
        if self._ifd < 0:
            raise OSError(ctypes.get_errno(), "inotify_init1")
        if libc.inotify_add_watch(self._ifd, self.path.encode(), IN_OPEN | IN_DELETE_SELF) < 0:
            raise OSError(ctypes.get_errno(), "inotify_add_watch")
        ev = struct.Struct("iIII")

        def run():
            while True:
                try:
                    buf = os.read(self._ifd, 4096)
                except OSError:
                    return
                off = 0
                while off + ev.size <= len(buf):
                    _wd, mask, _c, ln = ev.unpack_from(buf, off)
                    off += ev.size + ln
                    if mask & (IN_OPEN | IN_DELETE_SELF):
                        log.warning("lock file %s contended: exiting", self.path)
                        on_contention()
                        return
        threading.Thread(target=run, name="lockfile-contention", daemon=True).start()

    def release(self):
        if self.fd is not None:
            try:
                fcntl.flock(self.fd, fcntl.LOCK_UN)
            finally:
                os.close(self.fd)
                self.fd = None
