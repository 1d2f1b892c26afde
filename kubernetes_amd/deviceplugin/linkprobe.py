"""xGMI link probe: measured peer-to-peer bandwidth between the node's GPUs feeds the link graph
the plugin publishes (`amd.com/xgmi-peers`), so a link that the SMI reports up but that trained
degraded (fewer lanes, lower speed, replaying errors) stops counting as a direct link for the
scheduler's clique placement.

The measurement is `xgmi-probe --p2p` (native/hip/xgmi_probe.cc): hipMemcpyPeerAsync for every
ordered pair of the GPUs it is given plus each GPU's local copy bandwidth, one JSON object.
A pair is weak when either direction measures below `min_gbps`. The reference fork has no such
check (its NVIDIA plugin trusts NVML's NVLink state); SURVEY §2.3 "link-health probe".
"""
from __future__ import annotations

import json
import logging
import os
import subprocess

from ..native import BIN_DIR

log = logging.getLogger("linkprobe")
PROBE = os.path.join(BIN_DIR, "xgmi-probe")
DEFAULT_MIN_GBPS = 25.0


class ProbeResult:
    def __init__(self, pairs=None, local=None, error=""):
        self.pairs: dict[tuple, float] = pairs or {}    # (src hip index, dst hip index) -> GB/s
        self.local: dict[int, float] = local or {}
        self.error = error

    def weak_pairs(self, min_gbps):
        """Unordered pairs {a, b} with a direction under min_gbps."""
        out = set()
        for (a, b), g in self.pairs.items():
            if g < min_gbps:
                out.add(frozenset((a, b)))
        return out


def parse(text: str, hip_ids) -> ProbeResult:
    """`xgmi-probe --p2p` output; device numbers are positions in `hip_ids` (the probe ran with
    exactly those GPUs visible)."""
    d = json.loads(text)
    pairs = {(hip_ids[p["src"]], hip_ids[p["dst"]]): float(p["GBps"]) for p in d.get("pairs") or ()}
    local = {hip_ids[x["dev"]]: float(x["GBps"]) for x in d.get("local") or ()}
    return ProbeResult(pairs, local)


def run_probe(hip_ids, mib=256, iters=10, timeout=120.0) -> ProbeResult:
    """Run the native probe on the given host HIP ordinals (and only those)."""
    if not os.access(PROBE, os.X_OK):
        return ProbeResult(error="xgmi-probe is not built")
    env = dict(os.environ, HIP_VISIBLE_DEVICES=",".join(str(i) for i in hip_ids))
    env.pop("ROCR_VISIBLE_DEVICES", None)
    try:
        r = subprocess.run([PROBE, "--p2p", str(mib), str(iters)], env=env, capture_output=True, text=True,
                           timeout=timeout)
    except (OSError, subprocess.TimeoutExpired) as e:
        return ProbeResult(error=f"xgmi-probe: {e}")
    if r.returncode != 0:
        return ProbeResult(error=f"xgmi-probe exited {r.returncode}: {r.stderr.strip()[-300:]}")
    try:
        return parse(r.stdout.strip().splitlines()[-1], list(hip_ids))
    except (ValueError, KeyError, IndexError) as e:
        return ProbeResult(error=f"xgmi-probe output: {e}")


def prune_peers(peers: dict, hip_of: dict, weak: set) -> dict:
    """Remove weak links from the peer map ({device index: (hive-local index, mask)});
    `hip_of` maps device index -> HIP ordinal (the probe's numbering)."""
    if not weak:
        return peers
    local_of = {idx: p[0] for idx, p in peers.items()}
    out = dict(peers)
    for pair in weak:
        a, b = tuple(pair)
        ia = [i for i, h in hip_of.items() if h == a]
        ib = [i for i, h in hip_of.items() if h == b]
        for x in ia:
            for y in ib:
                if x in out and y in out and local_of[x] != local_of[y]:
                    out[x] = (out[x][0], out[x][1] & ~(1 << local_of[y]))
                    out[y] = (out[y][0], out[y][1] & ~(1 << local_of[x]))
    return out
