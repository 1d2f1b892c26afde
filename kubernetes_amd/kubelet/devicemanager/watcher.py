"""PluginWatcher: discovers device-plugin sockets under `<plugins_dir>/<domain>/<socket>`.

Parity: `pkg/kubelet/apis/pluginregistration/v1beta/plugin_watcher.go:16-261` — walk the tree at
start, then react to filesystem events; files directly in the root and directories inside a
domain are rejected (`handleCreate` :222-244); emits Added(path) / Removed(path).

Implementation: Linux inotify through ctypes (event-driven, no polling), driven by the
asyncio loop's reader callback; falls back to a 100 ms poll if inotify is unavailable.
"""
from __future__ import annotations

import asyncio
import ctypes
import ctypes.util
import logging
import os
import stat
import struct

log = logging.getLogger("pluginwatcher")

IN_CREATE, IN_DELETE, IN_MOVED_FROM, IN_MOVED_TO = 0x100, 0x200, 0x40, 0x80
IN_DELETE_SELF, IN_ISDIR, IN_NONBLOCK, IN_CLOEXEC = 0x400, 0x40000000, 0o4000, 0o2000000
_EV = struct.Struct("iIII")


class PluginWatcher:
    def __init__(self, plugins_dir: str):
        self.dir = os.path.abspath(plugins_dir)
        self.added: asyncio.Queue = asyncio.Queue()
        self.removed: asyncio.Queue = asyncio.Queue()
        self._known: set[str] = set()
        self._fd = None
        self._wd: dict[int, str] = {}
        self._poll_task = None
        self._libc = None

    # -- helpers -----------------------------------------------------------
    @staticmethod
    def _is_socket(p):
        try:
            return stat.S_ISSOCK(os.stat(p).st_mode)
        except OSError:
            return False

    def _emit_add(self, path):
        if path not in self._known:
            self._known.add(path)
            self.added.put_nowait(path)

    def _emit_remove(self, path):
        if path in self._known:
            self._known.discard(path)
            self.removed.put_nowait(path)

    def _scan(self):
        """Walk <dir>/<domain>/<socket> (the reference's init walk)."""
        seen = set()
        try:
            domains = os.listdir(self.dir)
        except FileNotFoundError:
            domains = []
        for d in domains:
            dp = os.path.join(self.dir, d)
            if not os.path.isdir(dp):
                continue  # files in the root are ignored (handleCreate rule)
            self._add_watch(dp)
            for f in os.listdir(dp):
                fp = os.path.join(dp, f)
                if os.path.isdir(fp):
                    continue  # directories inside a domain are rejected
                if self._is_socket(fp):
                    seen.add(fp)
                    self._emit_add(fp)
        for p in list(self._known):
            if p not in seen:
                self._emit_remove(p)

    def _add_watch(self, path):
        if self._fd is None or path in self._wd.values():
            return
        wd = self._libc.inotify_add_watch(self._fd, path.encode(), IN_CREATE | IN_DELETE | IN_MOVED_FROM | IN_MOVED_TO | IN_DELETE_SELF)
        if wd >= 0:
            self._wd[wd] = path

    def _on_readable(self):
        try:
            data = os.read(self._fd, 1 << 16)
        except BlockingIOError:
            return
        off = 0
        rescan = False
        while off + _EV.size <= len(data):
            wd, mask, _cookie, ln = _EV.unpack_from(data, off)
            name = data[off + _EV.size: off + _EV.size + ln].rstrip(b"\0").decode()
            off += _EV.size + ln
            base = self._wd.get(wd)
            if base is None:
                continue
            full = os.path.join(base, name)
            if mask & IN_DELETE_SELF:
                self._wd.pop(wd, None)
                rescan = True
                continue
            if mask & (IN_CREATE | IN_MOVED_TO):
                if base == self.dir:
                    if mask & IN_ISDIR:
                        self._add_watch(full)
                        rescan = True
                    continue
                if not (mask & IN_ISDIR) and self._is_socket(full):
                    self._emit_add(full)
                else:
                    rescan = True  # the socket file may appear before it is a socket
            elif mask & (IN_DELETE | IN_MOVED_FROM):
                self._emit_remove(full)
        if rescan:
            self._scan()

    async def _poll(self):
        while True:
            await asyncio.sleep(0.1)
            self._scan()

    # -- public ----------------------------------------------------------------
    def start(self):
        os.makedirs(self.dir, exist_ok=True)
        try:
            self._libc = ctypes.CDLL(ctypes.util.find_library("c"), use_errno=True)
            fd = self._libc.inotify_init1(IN_NONBLOCK | IN_CLOEXEC)
            if fd < 0:
                raise OSError(ctypes.get_errno(), "inotify_init1")
            self._fd = fd
            self._add_watch(self.dir)
            asyncio.get_event_loop().add_reader(fd, self._on_readable)
        except (OSError, AttributeError) as e:
            log.warning("inotify unavailable (%s); polling %s", e, self.dir)
            self._fd = None
            self._poll_task = asyncio.ensure_future(self._poll())
        self._scan()

    def stop(self):
        if self._fd is not None:
            try:
                asyncio.get_event_loop().remove_reader(self._fd)
            except Exception:
                pass
            # closing an inotify descriptor waits out a kernel SRCU grace period (~50 ms on the
            # MI355X box, profiles/r4_gpu/cprofile): close it off the event loop so a process
            # stopping many watchers (a hollow-node process with 16+ kubelets) does not
            # serialise those waits; concurrent closes share grace periods
            import threading
            threading.Thread(target=os.close, args=(self._fd,), name="inotify-close", daemon=True).start()
            self._fd = None
        if self._poll_task:
            self._poll_task.cancel()
