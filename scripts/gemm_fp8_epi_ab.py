"""Ping-pong GEMM, fp8 and bf16: register epilogue (path 0 / 3) vs the LDS-staged vector epilogue
(path 4), fp32 and bf16 output; correctness vs fp32 torch first."""
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


for M, N, K in [(256, 256, 128), (768, 512, 640)]:
    a = (torch.rand(M, K, device="cuda") * 4 - 2).to(torch.float8_e4m3fn)
    b = (torch.rand(N, K, device="cuda") * 4 - 2).to(torch.float8_e4m3fn)
    ref = a.float() @ b.float().T
    for path in (0, 4):
        hk.set_gemm_path(path)
        for f32 in (True, False):
            err = (hk.gemm_fp8_nt(a, b, out_fp32=f32).float() - ref).abs().max().item() / ref.abs().max().item()
            assert err < (1e-4 if f32 else 1e-2), (M, N, K, path, f32, err)
    print(f"check {M}x{N}x{K} ok", flush=True)
for M, N, K in [(4096, 4096, 4096), (8192, 8192, 8192), (16384, 8192, 8192)]:
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.float8_e4m3fn)
    b = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.float8_e4m3fn)
    flop = 2.0 * M * N * K
    a16, b16 = a.to(torch.bfloat16), b.to(torch.bfloat16)
    res = {}
    for rep in range(2):
        for path in (0, 4):
            hk.set_gemm_path(path)
            for f32 in (False, True):
                res.setdefault(("fp8", path, f32), []).append(
                    flop / timeit(lambda: hk.gemm_fp8_nt(a, b, out_fp32=f32)) / 1e12)
        for path in (3, 4):
            hk.set_gemm_path(path)
            res.setdefault(("bf16", path, False), []).append(
                flop / timeit(lambda: hk.gemm_bf16_nt(a16, b16, out_fp32=False)) / 1e12)
    hk.set_gemm_path(0)
    print(f"{M}x{N}x{K}: " + " | ".join(f"{d} path {p} {'fp32' if f else 'bf16'} out: {max(v):.0f}"
                                          for (d, p, f), v in sorted(res.items())), flush=True)
