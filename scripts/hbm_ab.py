"""A/B the HBM copy kernels (read+write bytes counted) on cuda:0."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubernetes_amd.ops import hip_kernels as h  # noqa: E402

NAMES = {0: "flat", 1: "grid-stride", 2: "x4-nontemporal", 3: "x4-plain"}
for nbytes in (1 << 30, 4 << 30):
    for variant, blocks in ((0, 0), (1, 0), (2, 16384), (3, 16384)):
        h.hbm_copy_config(variant, blocks)
        r = h.diag_hbm(0, nbytes, 20)
        print(f"{nbytes >> 20} MiB {NAMES[variant]} blocks={blocks or 'default'}: {r['GBps']:.0f} GB/s", flush=True)
h.hbm_copy_config(0, 0)
