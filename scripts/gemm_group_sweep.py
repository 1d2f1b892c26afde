"""Ping-pong GEMM: M-tile group size of the L2-friendly tile order, bf16 and fp8, bf16 output."""
import sys
import time

import torch

sys.path.insert(0, ".")
from kubernetes_amd.ops import hip_kernels as hk  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(3):
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / iters)
    return best


for M, N, K in [(4096, 4096, 4096), (8192, 8192, 8192), (16384, 8192, 8192), (16384, 16384, 4096)]:
    a8 = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.float8_e4m3fn)
    b8 = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.float8_e4m3fn)
    a16, b16 = a8.to(torch.bfloat16), b8.to(torch.bfloat16)
    flop = 2.0 * M * N * K
    line = []
    for g in (1, 2, 4, 8, 16, 32):
        hk.set_gemm_group(g)
        bf = flop / timeit(lambda: hk.gemm_bf16_nt(a16, b16, out_fp32=False)) / 1e12
        f8 = flop / timeit(lambda: hk.gemm_fp8_nt(a8, b8, out_fp32=False)) / 1e12
        line.append(f"G{g}: bf16 {bf:.0f} fp8 {f8:.0f}")
    hk.set_gemm_group(4)
    print(f"{M}x{N}x{K}: " + " | ".join(line), flush=True)
