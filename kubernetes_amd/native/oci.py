"""Binding for libkamd_oci.so: OCI `linux.devices` + cgroup allow rules for injected GPU nodes."""
from __future__ import annotations

import ctypes
import json
import os

from . import LIB_DIR

_lib = None


def _load():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(os.path.join(LIB_DIR, "libkamd_oci.so"))
        L.kamd_oci_devices.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
        _lib = L
    return _lib


def oci_devices(paths, access="rwm") -> dict:
    """stat() each host device node -> {"devices": [...], "allow": [...]} (OCI runtime-spec)."""
    buf = ctypes.create_string_buffer(1 << 16)
    rc = _load().kamd_oci_devices("\n".join(paths).encode(), access.encode(), buf, len(buf))
    if rc <= -100:
        raise FileNotFoundError(f"not a device node: {paths[-rc - 100]}")
    if rc < 0:
        raise RuntimeError("oci_devices: output buffer too small")
    return json.loads(buf.value.decode())
