"""Binary encoding shared by the native store (libkamd_store.so, kamd-etcd) and its clients.

Layout documented in native/store/mvcc_store.cc. A transaction is a list of compares (all must
hold) and a list of ops applied atomically under ONE new revision — etcd's Txn(If...Then...).
"""
from __future__ import annotations

import struct

from .mvcc import KV

# compare kinds
CMP_MOD_REV, CMP_EXISTS, CMP_ABSENT, CMP_VALUE = 0, 1, 2, 3
# op kinds
OP_PUT, OP_DELETE, OP_PUT_INJECT, OP_DELETE_TOMBSTONE = 0, 1, 2, 3
# request ops
TXN, GET, RANGE, WATCH, REV, COMPACT, RANGE_AT = 1, 2, 3, 4, 5, 6, 7
# statuses
OK, FAILED, COMPACTED, NOT_FOUND, EVENT, BAD, PROGRESS = 0, 1, 3, 4, 8, 9, 10

_u32 = struct.Struct("<I")
_i64 = struct.Struct("<q")
_kvhdr = struct.Struct("<qqqI")


def _s(b: bytes) -> bytes:
    return _u32.pack(len(b)) + b


def encode_txn(cmps, ops) -> bytes:
    """cmps: [(kind, key, arg_rev, value_bytes)], ops: [(kind, key, value_bytes[, token])]."""
    parts = [struct.pack("<H", len(cmps))]
    for kind, key, arg, val in cmps:
        parts.append(bytes((kind,)) + _s(key.encode()) + _i64.pack(arg) + _s(val or b""))
    parts.append(struct.pack("<H", len(ops)))
    for op in ops:
        kind, key, val = op[0], op[1], op[2]
        parts.append(bytes((kind,)) + _s(key.encode()) + _s(val or b""))
        if kind >= OP_PUT_INJECT:
            parts.append(_s(op[3]))
    return b"".join(parts)


def decode_kv(buf, off=0):
    """Returns (KV, new_offset)."""
    cr, mr, ver, kl = _kvhdr.unpack_from(buf, off)
    off += _kvhdr.size
    key = bytes(buf[off:off + kl]).decode()
    off += kl
    (vl,) = _u32.unpack_from(buf, off)
    off += 4
    val = bytes(buf[off:off + vl])
    return KV(key, val, cr, mr, ver), off + vl


def decode_range(buf):
    """Returns (kvs, more, rev)."""
    (rev,) = _i64.unpack_from(buf, 0)
    more = buf[8] == 1
    (n,) = _u32.unpack_from(buf, 9)
    off = 13
    out = []
    for _ in range(n):
        kv, off = decode_kv(buf, off)
        out.append(kv)
    return out, more, rev


def encode_range(prefix: str, limit: int = 0, start_after: str | None = None) -> bytes:
    return _s(prefix.encode()) + _u32.pack(limit) + _s((start_after or "").encode())


def decode_failed(buf):
    """Failed-compare response: (index, current KV or None, store revision)."""
    (idx,) = struct.unpack_from("<H", buf, 0)
    off = 2
    kv = None
    if buf[off] == 1:
        kv, off = decode_kv(buf, off + 1)
    else:
        off += 1
    (rev,) = _i64.unpack_from(buf, off)
    return idx, kv, rev
