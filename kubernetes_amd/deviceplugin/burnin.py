"""Device acceptance test ("burn-in") run by the amd.com/gpu plugin before it offers a GPU.

The reference's device health is whatever the vendor plugin reports from NVML
(`pkg/kubelet/cm/devicemanager/manager_store.go:47-83` stores it, `:116-118` refuses to admit on
unhealthy IDs); nothing in it exercises the GPU. Here the plugin can gate every MI355X on the
framework's own HIP kernels (`native/hip/kamd_hip.hip`, via `ops/hip_kernels.py`):

  * vector_add    — the e2e workload kernel; the result must be exact;
  * MFMA GEMM     — bf16 M=N=K=`gemm_size` on the ping-pong MFMA kernel: sampled outputs are
                    checked against an fp64 host dot product (numerics) and the throughput
                    must reach `min_tflops` (a throttled / degraded part shows up here);
  * fp8 MFMA GEMM — the same on OCP e4m3 operands through the block-scaled
                    v_mfma_scale_f32_16x16x128_f8f6f4 path (`min_fp8_tflops`);
  * HBM copy      — streaming copy bandwidth must reach `min_hbm_gbps`.

A device is advertised Unhealthy (`amd.com/burn-in=pending`) until its test passes, so the
scheduler never binds a pod to a GPU that has not been validated; the measured numbers are
published as device attributes (`amd.com/mfma-tflops`, `amd.com/mfma-fp8-tflops`,
`amd.com/hbm-gbps`) that pod selectors can use. Thresholds default to roughly half of what a
healthy MI355X measures with these kernels (profiles/r2_gemm_pingpong: 1.3-1.5 PF/s bf16 at
8192^3; profiles/r2_gemm_fp8: 2.5-3.0 PF/s fp8; profiles/r1_hbm: 6.2 TB/s copy).
"""
from __future__ import annotations

import time
from dataclasses import dataclass

PENDING, PASSED, FAILED = "pending", "passed", "failed"


@dataclass
class BurnInResult:
    ok: bool
    tflops: float = 0.0
    fp8_tflops: float = 0.0
    hbm_gbps: float = 0.0
    vadd_err: float = 0.0
    mfma_rel_err: float = 0.0
    fp8_rel_err: float = 0.0
    seconds: float = 0.0
    reason: str = ""


class BurnIn:
    def __init__(self, min_tflops=700.0, min_hbm_gbps=3000.0, max_rel_err=1e-2, gemm_size=8192, gemm_iters=10,
                 hbm_bytes=1 << 30, hbm_iters=20, vadd_n=50000, min_fp8_tflops=1400.0, fp8=True):
        self.min_tflops = min_tflops
        self.min_fp8_tflops = min_fp8_tflops
        self.fp8 = fp8
        self.min_hbm_gbps = min_hbm_gbps
        self.max_rel_err = max_rel_err
        self.gemm_size = gemm_size
        self.gemm_iters = gemm_iters
        self.hbm_bytes = hbm_bytes
        self.hbm_iters = hbm_iters
        self.vadd_n = vadd_n

    def run(self, hip_index: int) -> BurnInResult:
        """Blocking; call from a worker thread (the HIP calls release the GIL)."""
        from ..ops import hip_kernels as hk
        t0 = time.monotonic()
        r = BurnInResult(ok=False)
        try:
            r.vadd_err = hk.diag_vector_add(hip_index, self.vadd_n)
            m = hk.diag_mfma(hip_index, self.gemm_size, self.gemm_iters)
            r.tflops, r.mfma_rel_err = m["tflops"], m["max_rel_err"]
            if self.fp8:
                m8 = hk.diag_mfma_fp8(hip_index, self.gemm_size, self.gemm_iters)
                r.fp8_tflops, r.fp8_rel_err = m8["tflops"], m8["max_rel_err"]
            r.hbm_gbps = hk.diag_hbm(hip_index, self.hbm_bytes, self.hbm_iters)["GBps"]
        except Exception as e:  # noqa: BLE001 - a HIP error is a failed device
            r.reason = f"HIP error: {e}"
            r.seconds = time.monotonic() - t0
            return r
        r.seconds = time.monotonic() - t0
        r.reason = self.judge(r)
        r.ok = not r.reason
        return r

    def judge(self, r: BurnInResult) -> str:
        if r.vadd_err != 0.0:
            return f"vector_add max error {r.vadd_err:g} (want exact)"
        if not (r.mfma_rel_err <= self.max_rel_err):
            return f"MFMA GEMM relative error {r.mfma_rel_err:.3g} > {self.max_rel_err:g}"
        if self.min_tflops and r.tflops < self.min_tflops:
            return f"MFMA GEMM {r.tflops:.0f} TFLOP/s < {self.min_tflops:.0f}"
        if self.fp8:
            if not (r.fp8_rel_err <= self.max_rel_err):
                return f"fp8 MFMA GEMM relative error {r.fp8_rel_err:.3g} > {self.max_rel_err:g}"
            if self.min_fp8_tflops and r.fp8_tflops < self.min_fp8_tflops:
                return f"fp8 MFMA GEMM {r.fp8_tflops:.0f} TFLOP/s < {self.min_fp8_tflops:.0f}"
        if self.min_hbm_gbps and r.hbm_gbps < self.min_hbm_gbps:
            return f"HBM copy {r.hbm_gbps:.0f} GB/s < {self.min_hbm_gbps:.0f}"
        return ""
