"""ctypes binding for `libkamd_hip.so` (native/hip/kamd_hip.hip, gfx950).

  vector_add(a, b)             -> a + b          (GPU e2e workload kernel)
  gemm_bf16_nt(a, b, out_fp32) -> a @ b.T        (MFMA 16x16x32 bf16, LDS-tiled)
  gemm_fp8_nt(a, b, out_fp32)  -> a @ b.T        (OCP fp8 e4m3, block-scaled MFMA 16x16x128)
  diag_mfma / diag_hbm / diag_vector_add         (device-plugin burn-in diagnostics)
  Payload(dev)                                    (warm per-GPU payload for GPU pods)

The extension is REQUIRED on a GPU host: every entry point raises if the library is missing
rather than silently falling back to a PyTorch implementation.
"""
from __future__ import annotations

import ctypes
import os

from ..native import LIB_DIR

_lib = None


class HIPError(RuntimeError):
    pass


def lib_path():
    return os.path.join(LIB_DIR, "libkamd_hip.so")


def load():
    global _lib
    if _lib is None:
        p = lib_path()
        if not os.path.exists(p):
            raise HIPError(f"{p} is not built (python -m kubernetes_amd.native.build); no fallback exists")
        L = ctypes.CDLL(p)
        vp, i, f, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
        L.kamd_hip_last_error.restype = ctypes.c_char_p
        L.kamd_vector_add_launch.argtypes = [vp, vp, vp, i, vp]
        L.kamd_gemm_bf16_nt_launch.argtypes = [vp, vp, vp, i, i, i, i, f, i, vp]
        L.kamd_gemm_fp8_nt_launch.argtypes = [vp, vp, vp, i, i, i, i, f, i, vp]
        L.kamd_hbm_copy_launch.argtypes = [vp, vp, sz, vp]
        L.kamd_diag_vector_add.argtypes = [i, i, ctypes.POINTER(ctypes.c_float)]
        L.kamd_diag_mfma.argtypes = [i, i, i, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        L.kamd_diag_mfma_fp8.argtypes = [i, i, i, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        L.kamd_diag_hbm.argtypes = [i, sz, i, ctypes.POINTER(ctypes.c_double)]
        L.kamd_payload_create.argtypes = [i, i]
        L.kamd_payload_create.restype = vp
        L.kamd_payload_run.argtypes = [vp]
        L.kamd_payload_run_batch.argtypes = [vp, i, ctypes.POINTER(ctypes.c_int)]
        L.kamd_payload_destroy.argtypes = [vp]
        L.kamd_hip_device_arch.argtypes = [i, ctypes.c_char_p, i]
        L.kamd_gemm_set_path.argtypes = [i]
        L.kamd_gemm_set_group.argtypes = [i]
        L.kamd_hbm_copy_config.argtypes = [i, i]
        _lib = L
    return _lib


def _raise(rc, what):
    if rc != 0:
        raise HIPError(f"{what}: {load().kamd_hip_last_error().decode(errors='replace')}")


def _stream(t):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def device_count() -> int:
    return load().kamd_hip_device_count()


def device_arch(dev=0) -> str:
    buf = ctypes.create_string_buffer(64)
    _raise(load().kamd_hip_device_arch(dev, buf, 64), "device_arch")
    return buf.value.decode()


def vector_add(a, b):
    import torch
    assert a.is_cuda and a.dtype == torch.float32 and a.shape == b.shape and a.is_contiguous() and b.is_contiguous()
    out = torch.empty_like(a)
    _raise(load().kamd_vector_add_launch(a.data_ptr(), b.data_ptr(), out.data_ptr(), a.numel(), _stream(a)), "vector_add")
    return out


def gemm_bf16_nt(a, b, out_fp32=True, alpha=1.0):
    """C = alpha * a @ b.T with a: [M, K] bf16, b: [N, K] bf16 (both row-major, K % 8 == 0)."""
    import torch
    assert a.is_cuda and b.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16
    assert a.dim() == 2 and b.dim() == 2 and a.shape[1] == b.shape[1], (a.shape, b.shape)
    a, b = a.contiguous(), b.contiguous()
    M, K = a.shape
    N = b.shape[0]
    if K % 8:
        raise ValueError(f"K={K} must be a multiple of 8")
    out = torch.empty((M, N), device=a.device, dtype=torch.float32 if out_fp32 else torch.bfloat16)
    _raise(load().kamd_gemm_bf16_nt_launch(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, N, float(alpha),
                                           1 if out_fp32 else 0, _stream(a)), "gemm_bf16_nt")
    return out


def gemm_fp8_nt(a, b, out_fp32=True, alpha=1.0):
    """C = alpha * a @ b.T with a: [M, K], b: [N, K] OCP fp8 e4m3 (torch.float8_e4m3fn), fp32
    accumulate, on the block-scaled MFMA (v_mfma_scale_f32_16x16x128_f8f6f4, unit scales).
    M, N must be multiples of 256 and K of 128."""
    import torch
    assert a.is_cuda and b.is_cuda and a.dtype == torch.float8_e4m3fn and b.dtype == torch.float8_e4m3fn
    assert a.dim() == 2 and b.dim() == 2 and a.shape[1] == b.shape[1], (a.shape, b.shape)
    a, b = a.contiguous(), b.contiguous()
    M, K = a.shape
    N = b.shape[0]
    if M % 256 or N % 256 or K % 128:
        raise ValueError(f"gemm_fp8_nt needs M, N % 256 == 0 and K % 128 == 0, got {M}x{N}x{K}")
    out = torch.empty((M, N), device=a.device, dtype=torch.float32 if out_fp32 else torch.bfloat16)
    _raise(load().kamd_gemm_fp8_nt_launch(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, N, float(alpha),
                                          1 if out_fp32 else 0, _stream(a)), "gemm_fp8_nt")
    return out


def set_gemm_group(group: int):
    """M-tiles per group of the ping-pong GEMM's L2-friendly tile order (default 4)."""
    load().kamd_gemm_set_group(int(group))


def set_gemm_path(path: int):
    """0 = auto (the ping-pong 256x256 global_load_lds kernel — wave groups staggered by one
    barrier — when M, N % 256 == 0 and K % 64 == 0, else the 128x128 kernel), 1 = always the
    128x128 register-staged kernel, 2 = the 2-barrier 256x256 kernel, 3 = ping-pong, 4-6 =
    ping-pong variants (LDS epilogue / static priority / both), 7 = the 8-phase 256x256 kernel."""
    load().kamd_gemm_set_path(int(path))


def hbm_copy_config(variant: int = 0, blocks: int = 0):
    """variant 0: flat, one 16-B element per lane (default, ~6.2 TB/s); 1: grid-stride;
    2: 4 non-temporal loads in flight per lane; 3: the same without the hints."""
    load().kamd_hbm_copy_config(int(variant), int(blocks))


def hbm_copy(src, dst):
    assert src.is_cuda and dst.is_cuda and src.numel() * src.element_size() == dst.numel() * dst.element_size()
    nbytes = src.numel() * src.element_size()
    assert nbytes % 16 == 0
    _raise(load().kamd_hbm_copy_launch(src.data_ptr(), dst.data_ptr(), nbytes, _stream(src)), "hbm_copy")


def diag_vector_add(dev=0, n=50000) -> float:
    e = ctypes.c_float()
    _raise(load().kamd_diag_vector_add(dev, n, ctypes.byref(e)), "diag_vector_add")
    return e.value


def diag_mfma(dev=0, size=4096, iters=20):
    tf, err = ctypes.c_double(), ctypes.c_double()
    _raise(load().kamd_diag_mfma(dev, size, iters, ctypes.byref(tf), ctypes.byref(err)), "diag_mfma")
    return {"tflops": tf.value, "max_rel_err": err.value, "size": size, "iters": iters}


def diag_mfma_fp8(dev=0, size=8192, iters=10):
    tf, err = ctypes.c_double(), ctypes.c_double()
    _raise(load().kamd_diag_mfma_fp8(dev, size, iters, ctypes.byref(tf), ctypes.byref(err)), "diag_mfma_fp8")
    return {"tflops": tf.value, "max_rel_err": err.value, "size": size, "iters": iters}


def diag_hbm(dev=0, nbytes=1 << 30, iters=20):
    g = ctypes.c_double()
    _raise(load().kamd_diag_hbm(dev, nbytes, iters, ctypes.byref(g)), "diag_hbm")
    return {"GBps": g.value, "bytes": nbytes, "iters": iters}


class Payload:
    """Warm per-GPU context: `run()` launches vector_add on the device and verifies it."""

    def __init__(self, dev=0, n=50000):
        self.h = load().kamd_payload_create(dev, n)
        if not self.h:
            raise HIPError(f"payload create on device {dev} failed")
        self.dev = dev

    MAX_BATCH = 256   # PAYLOAD_SLOTS in native/hip/kamd_hip.hip

    def run(self) -> bool:
        return load().kamd_payload_run(self.h) == 0

    def run_batch(self, k: int) -> list:
        """k container starts at once: k vector_add launches, one verify kernel, one sync.
        Returns one pass/fail per start. Thread-safe for a single caller thread at a time."""
        out = []
        while k > 0:
            m = min(k, self.MAX_BATCH)
            ok = (ctypes.c_int * m)()
            rc = load().kamd_payload_run_batch(self.h, m, ok)
            out += [False] * m if rc < 0 else [bool(x) for x in ok]
            k -= m
        return out

    def close(self):
        if self.h:
            load().kamd_payload_destroy(self.h)
            self.h = None
