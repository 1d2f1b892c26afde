"""Scheduler-shard selection of pods (`?kamdShard=i/n` on list and watch).

With `kube-scheduler --shards n` every shard lists/watches only the unassigned pods it is
responsible for, so per-shard work is O(pods/n) instead of every shard decoding every pod event.
A pod belongs to shard `(crc32("<namespace>/<name>") + offset) % n`, where `offset` is the
integer label `scheduler.kamd.io/shard-offset` (absent = 0): a shard whose nodes cannot fit a
pod hands it to the next shard by bumping that label. The API server evaluates the selector on
the stored index fields, and `kamd-etcd`'s watch fan-out evaluates the same function natively
(requirement op 6 in native/store/mvcc_store.cc), so the hash must stay zlib's CRC-32.
"""
from __future__ import annotations

import zlib

SHARD_OFFSET_LABEL = "scheduler.kamd.io/shard-offset"
QUERY_PARAM = "kamdShard"


def parse_shard(value: str):
    """"i/n" -> (i, n); ValueError when malformed."""
    i, _, n = (value or "").partition("/")
    i, n = int(i), int(n)
    if n < 1 or not 0 <= i < n:
        raise ValueError(f"invalid {QUERY_PARAM} {value!r}: want i/n with 0 <= i < n")
    return i, n


def offset_of(labels) -> int:
    """The offset label as an int; malformed or |v| > 2^31 reads as 0 (same in the C++ side)."""
    v = (labels or {}).get(SHARD_OFFSET_LABEL, "")
    try:
        off = int(v) if isinstance(v, str) and v.strip() == v else 0
    except ValueError:
        return 0
    return off if -(1 << 31) <= off <= (1 << 31) else 0


def shard_of_key(key: str, count: int, offset: int = 0) -> int:
    return (zlib.crc32(key.encode()) + offset) % count


def shard_matches(fields, labels, index: int, count: int) -> bool:
    key = f"{fields.get('metadata.namespace', '')}/{fields.get('metadata.name', '')}"
    return shard_of_key(key, count, offset_of(labels)) == index
