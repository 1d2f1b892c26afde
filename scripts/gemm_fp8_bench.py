"""fp8 (OCP e4m3) GEMM throughput: the block-scaled MFMA ping-pong kernel vs torch._scaled_mm
(hipBLASLt), and our bf16 kernel vs torch.matmul (hipBLASLt), all with bf16 output (same bytes
written). Prints one line per shape."""
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


def main():
    shapes = [(4096, 4096, 4096), (8192, 8192, 8192), (16384, 8192, 8192)]
    one = torch.tensor(1.0, device="cuda")
    for M, N, K in shapes:
        a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.float8_e4m3fn)
        b = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.float8_e4m3fn)
        flop = 2.0 * M * N * K
        ours = flop / timeit(lambda: hk.gemm_fp8_nt(a, b, out_fp32=False)) / 1e12
        try:
            theirs = flop / timeit(lambda: torch._scaled_mm(a, b.t(), scale_a=one, scale_b=one,
                                                            out_dtype=torch.bfloat16)) / 1e12
        except Exception as e:  # noqa: BLE001
            theirs = float("nan")
            print(f"torch._scaled_mm unavailable: {e}", flush=True)
        a16, b16 = a.to(torch.bfloat16), b.to(torch.bfloat16)
        bf = flop / timeit(lambda: hk.gemm_bf16_nt(a16, b16, out_fp32=False)) / 1e12
        tbf = flop / timeit(lambda: torch.matmul(a16, b16.t())) / 1e12
        err = (hk.gemm_fp8_nt(a[:1024, :], b[:1024, :]) - a[:1024].float() @ b[:1024].float().T).abs().max().item()
        print(f"{M}x{N}x{K}: fp8 ours {ours:.0f} TF/s | torch._scaled_mm {theirs:.0f} TF/s | ratio {ours / theirs:.2f} "
              f"| our bf16 {bf:.0f} TF/s vs torch.matmul bf16 {tbf:.0f} ({bf / tbf:.2f}) | max abs err vs fp32 {err:.2e}",
              flush=True)


if __name__ == "__main__":
    main()
