"""Loader for the native protobuf codec (`native/pbcodec/kamd_pbcodec.cc` -> `_kamd_pbcodec`).

`codec()` returns the extension's codec object bound to the generated schema table, or None when
the extension is not built (the pure-Python codec in `api/protobuf.py` is then used). Set
KAMD_PBCODEC=python to force the Python path (tests cross-check both)."""
from __future__ import annotations

import importlib.util
import os

from . import LIB_DIR

_CODEC = False


def lib_path():
    import sysconfig
    return os.path.join(LIB_DIR, "_kamd_pbcodec" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))


def codec():
    global _CODEC
    if _CODEC is False:
        _CODEC = None
        if os.environ.get("KAMD_PBCODEC", "native") != "python" and os.path.exists(lib_path()):
            spec = importlib.util.spec_from_file_location("_kamd_pbcodec", lib_path())
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            import json
            from ..api import protobuf
            dumps = json.JSONEncoder(separators=(",", ":"), ensure_ascii=False).encode
            _CODEC = mod.Codec(protobuf.SCHEMA_PATH, protobuf.ProtobufError, dumps, json.loads)
            from ..api.meta import RESOURCES
            _CODEC.set_canonical({r.kind: r.group_version for r in RESOURCES})
    return _CODEC


def reset():
    """Re-read KAMD_PBCODEC (tests)."""
    global _CODEC
    _CODEC = False
