// kamd_hip — HIP/CDNA4 (gfx950) kernels used by the orchestrator's GPU paths.
//
//  * vector_add        — the GPU e2e workload. MI355X-native replacement for the reference's
//                        cuda-vector-add test image (test/images/cuda-vector-add/Dockerfile,
//                        used by test/e2e/scheduling/nvidia-gpus.go:51-113): 1-D grid of
//                        ceil(N/256) blocks x 256 threads, N = 50000 floats by default.
//  * gemm_bf16_nt      — MFMA (v_mfma_f32_16x16x32_bf16) LDS-tiled GEMM, C = A · Bᵀ (default: the
//                        ping-pong 256x256 kernel, 0.87-0.89x hipBLASLt on MI355X), used by the
//                        device-plugin burn-in diagnostic (matrix-core health + throughput, the
//                        role DCGM diag plays in the NVIDIA stack) and by the workload payload.
//  * hbm_copy          — 16 B/lane streaming copy: HBM3E bandwidth health probe.
//
// Everything is exported through a C ABI (extern "C") so the Python side binds with ctypes
// and passes torch tensor pointers + the current HIP stream.
#include <hip/hip_runtime.h>
#include <type_traits>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

static thread_local char g_err[256];
static int g_pp_group = 4;     // ping-pong GEMM: M-tiles per group of the L2-friendly tile order
static int g_gemm_path = 0;   // 0 auto (ping-pong 256-tile kernel when the shape allows), 1 force the 128-tile
                              // kernel, 2 the 2-barrier 256-tile glds kernel, 3-6 ping-pong variants, 7 the 8-phase
                              // 256-tile kernel

static int check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    snprintf(g_err, sizeof g_err, "%s: %s", what, hipGetErrorString(e));
    return -1;
  }
  return 0;
}
#define HC(x)                              \
  do {                                     \
    if (check((x), #x) != 0) return -1;    \
  } while (0)

// ---------------------------------------------------------------------------
// vector_add
__global__ void __launch_bounds__(256) vector_add_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                          float* __restrict__ c, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) c[i] = a[i] + b[i];
}

// ---------------------------------------------------------------------------
// MFMA GEMM: C[M,N] = A[M,K] · B[N,K]ᵀ   (A, B bf16 row-major; C fp32 or bf16)
//
// Block tile 128x128, BK = 64, 256 threads = 4 waves in a 2x2 grid; each wave owns a 64x64
// sub-tile = 4x4 MFMA 16x16 tiles (16 f32x4 accumulators). LDS holds one A and one B tile
// (128 rows x 64 bf16 = 128 B per row) per stage, double buffered (64 KiB). Rows are stored
// with the 16-byte chunk index XOR-swizzled by ((row >> 1) & 7) so that the 16 lanes of each
// ds_read_b128 group (16 consecutive rows, same k chunk) cover all 64 banks exactly once.
// Global->LDS is register-staged (prefetch tile t+1 into VGPRs while computing tile t).
// The block id is remapped so blocks sharing an XCD (bid % 8) take consecutive tiles (T1).
namespace gemm {
constexpr int BM = 128, BN = 128, BK = 64, THREADS = 256;
constexpr int ROW_BYTES = BK * 2;                // 128 B
constexpr int TILE_BYTES = BM * ROW_BYTES;       // 16 KiB
constexpr int CHUNKS = TILE_BYTES / 16;          // 1024 16-B chunks per tile
constexpr int LOADS = CHUNKS / THREADS;          // 4 per thread per operand

__device__ __forceinline__ int swz(int row, int chunk) { return row * ROW_BYTES + ((chunk ^ ((row >> 1) & 7)) << 4); }

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  // bijective: blocks with the same (bid % 8) — the same XCD under round-robin dispatch —
  // get a contiguous range of tile ids (shared A rows stay in that XCD's L2)
  int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

template <typename OutT>
__device__ __forceinline__ void store_out(OutT* p, float v);
template <>
__device__ __forceinline__ void store_out<float>(float* p, float v) { *p = v; }
template <>
__device__ __forceinline__ void store_out<__bf16>(__bf16* p, float v) { *p = (__bf16)v; }

template <typename OutT>
__global__ void __launch_bounds__(THREADS, 2)
gemm_bf16_nt_kernel(const u16* __restrict__ A, const u16* __restrict__ B, OutT* __restrict__ C,
                    int M, int N, int K, int ldc, float alpha) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];  // [2 stages][A|B] tiles
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int t = xcd_remap(blockIdx.x, nwg);
  // group 8 tile-rows together (L2 reuse of B columns across consecutive tiles)
  const int GROUP = 8;
  const int group_id = t / (GROUP * tiles_n);
  const int first_m = group_id * GROUP;
  const int gsz = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (t % (GROUP * tiles_n)) % gsz;
  const int tn = (t % (GROUP * tiles_n)) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[LOADS], rb[LOADS];
  const int ktiles = (K + BK - 1) / BK;

  auto gload = [&](int kt) {
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const int c = tid + i * THREADS;           // chunk id within the tile
      const int row = c >> 3, ch = c & 7;
      const int kk = k0 + ch * 8;
      const int ga = m0 + row, gb = n0 + row;
      uint4 z = {0u, 0u, 0u, 0u};
      ra[i] = (ga < M && kk < K) ? *reinterpret_cast<const uint4*>(A + (size_t)ga * K + kk) : z;
      rb[i] = (gb < N && kk < K) ? *reinterpret_cast<const uint4*>(B + (size_t)gb * K + kk) : z;
    }
  };
  auto sstore = [&](int stage) {
    unsigned char* la = lds + stage * 2 * TILE_BYTES;
    unsigned char* lb = la + TILE_BYTES;
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const int c = tid + i * THREADS;
      const int row = c >> 3, ch = c & 7;
      *reinterpret_cast<uint4*>(la + swz(row, ch)) = ra[i];
      *reinterpret_cast<uint4*>(lb + swz(row, ch)) = rb[i];
    }
  };

  gload(0);
  sstore(0);
  __syncthreads();
  const int frow = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < ktiles; ++kt) {
    const int stage = kt & 1;
    if (kt + 1 < ktiles) gload(kt + 1);  // prefetch next tile into VGPRs
    const unsigned char* la = lds + stage * 2 * TILE_BYTES;
    const unsigned char* lb = la + TILE_BYTES;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 af[4], bfr[4];
      const int ch = ks * 4 + fq;  // 16-B chunk holding k = ks*32 + 8*fq .. +7
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bf16x8*>(la + swz(wm + i * 16 + frow, ch));
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(lb + swz(wn + j * 16 + frow, ch));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < ktiles) sstore(stage ^ 1);
    __syncthreads();
  }
  // epilogue: C/D layout col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + wn + j * 16 + frow;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + i * 16 + fq * 4 + r;
        if (row < M && col < N) store_out<OutT>(C + (size_t)row * ldc + col, alpha * acc[i][j][r]);
      }
    }
}
}  // namespace gemm

// ---------------------------------------------------------------------------
// Large-tile path (M, N multiples of 256, K multiple of 64): 256x256x64 tiles, 8 waves (2 M x 4 N),
// each wave a 128x64 output patch = 8x4 MFMA 16x16x32 tiles (128 accumulator VGPRs).
// Operands are staged HBM -> LDS with global_load_lds (16 B / lane, no VGPR round trip) into two
// LDS buffers (128 KiB, ONE __shared__ array): the loads for K-tile t+1 are in flight while the
// MFMAs consume K-tile t. The LDS image is lane-linear per wave instruction, so the bank swizzle
// is applied to the per-lane GLOBAL address: 16-B slot s of LDS row r holds k-chunk s ^ ((r>>1)&7),
// which makes each 16-lane ds_read_b128 group (16 consecutive rows, same chunk) conflict-free.
namespace gemm256 {
using gemm::xcd_remap;
using gemm::store_out;
constexpr int BM = 256, BN = 256, BK = 64, THREADS = 512;
constexpr int TILE_BYTES = BM * BK * 2;        // one operand tile: 256 rows x 128 B
constexpr int STAGE_BYTES = 2 * TILE_BYTES;    // A | B
constexpr int LDS_BYTES = 2 * STAGE_BYTES;     // double buffered: 128 KiB
constexpr int GLDS_PER_OPERAND = TILE_BYTES / (THREADS * 16);  // 4

typedef __attribute__((address_space(3))) void lds_void;

template <typename OutT>
__global__ void __launch_bounds__(THREADS, 1)
gemm_bf16_nt_256_kernel(const u16* __restrict__ A, const u16* __restrict__ B, OutT* __restrict__ C,
                        int M, int N, int K, int ldc, float alpha) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_m = M / BM, tiles_n = N / BN, nwg = tiles_m * tiles_n;
  const int t = xcd_remap(blockIdx.x, nwg);
  // groups of 4 tile-rows walk the tile-columns together: B panels are re-read from L2
  const int GROUP = 4;
  const int group_id = t / (GROUP * tiles_n);
  const int first_m = group_id * GROUP;
  const int gsz = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (t % (GROUP * tiles_n)) % gsz;
  const int tn = (t % (GROUP * tiles_n)) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  // per-thread global source offsets (elements) of its 4 A and 4 B staging chunks
  size_t a_off[GLDS_PER_OPERAND], b_off[GLDS_PER_OPERAND];
#pragma unroll
  for (int j = 0; j < GLDS_PER_OPERAND; ++j) {
    const int q = j * THREADS + tid;             // 16-B chunk index in the LDS image
    const int row = q >> 3, slot = q & 7;
    const int kc = slot ^ ((row >> 1) & 7);      // logical k-chunk stored in this slot
    a_off[j] = (size_t)(m0 + row) * K + kc * 8;
    b_off[j] = (size_t)(n0 + row) * K + kc * 8;
  }
  auto stage = [&](int buf, int kt) {
    unsigned char* base = lds + buf * STAGE_BYTES + wid * 1024;   // wave-uniform; lane adds 16*lane
    const size_t k0 = (size_t)kt * BK;
#pragma unroll
    for (int j = 0; j < GLDS_PER_OPERAND; ++j) {
      __builtin_amdgcn_global_load_lds((const void*)(A + a_off[j] + k0), (lds_void*)(base + j * THREADS * 16), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(B + b_off[j] + k0), (lds_void*)(base + TILE_BYTES + j * THREADS * 16), 16, 0, 0);
    }
  };

  const int wr = wid >> 2, wc = wid & 3;         // wave's 128x64 patch
  const int frow = lane & 15, fq = lane >> 4;
  const int lsw = (frow >> 1) & 7;               // rows i*16+frow all have swizzle (frow>>1)&7
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nt = K / BK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nt) stage(cur ^ 1, kt + 1);
    const unsigned char* la = lds + cur * STAGE_BYTES + (wr * 128 + frow) * 128;
    const unsigned char* lb = lds + cur * STAGE_BYTES + TILE_BYTES + (wc * 64 + frow) * 128;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      const int off = ((ks * 4 + fq) ^ lsw) << 4;
      bf16x8 af[8], bfr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(lb + j * 16 * 128 + off);
#pragma unroll
      for (int i = 0; i < 8; ++i) af[i] = *reinterpret_cast<const bf16x8*>(la + i * 16 * 128 + off);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // epilogue: C/D layout col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + wc * 64 + j * 16 + frow;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wr * 128 + i * 16 + fq * 4 + r;
        store_out<OutT>(C + (size_t)row * ldc + col, alpha * acc[i][j][r]);
      }
    }
}
}  // namespace gemm256

// ---------------------------------------------------------------------------
// 8-phase 256x256 path (the default when M, N % 256 == 0, K % 64 == 0, K/64 >= 2).
// Same tile/wave geometry as gemm256 (8 waves 2M x 4N, 128x64 output per wave), but the K-loop is
// split into 4 phases per K-tile, one per C-quadrant of the wave (64 rows x 32 cols = 16 MFMAs):
//   wait(vmcnt) + s_barrier -> ds_read this phase's fragments -> issue ONE half-tile prefetch
//   (2 x global_load_lds, 16 KiB) -> s_barrier -> lgkmcnt(0) -> setprio(1) MFMAs setprio(0)
// LDS holds 2 K-tiles x 4 half-tiles, each half holding the rows ONE phase consumes (see below),
// 128 KiB in ONE dynamic array. A half-tile's slot is refilled for K-tile t+2 as soon as its only
// ds_read (phase 0/2/0/1 for h0/h1/h2/h3) is behind a barrier, so ~5 half-tiles (10 glds per
// thread) stay in flight and the waits are counted (vmcnt(10)), never vmcnt(0) in steady state.
namespace gemm8 {
using gemm::xcd_remap;
using gemm::store_out;
constexpr int BM = 256, BN = 256, BK = 64, THREADS = 512;
constexpr int HALF_BYTES = 128 * BK * 2;          // 16 KiB: 128 rows x 64 bf16
constexpr int TILE_BYTES = 4 * HALF_BYTES;        // A0 A1 B0 B1
constexpr int LDS_BYTES = 2 * TILE_BYTES;         // 128 KiB
typedef __attribute__((address_space(3))) void lds_void;

#define KAMD_WAIT_VM(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")
#define KAMD_WAIT_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
#define KAMD_BARRIER()                          \
  do {                                          \
    asm volatile("" ::: "memory");              \
    __builtin_amdgcn_s_barrier();               \
    asm volatile("" ::: "memory");              \
  } while (0)

template <typename OutT>
__global__ void __launch_bounds__(THREADS, 1)
gemm_bf16_nt_8ph_kernel(const u16* __restrict__ A, const u16* __restrict__ B, OutT* __restrict__ C,
                        int M, int N, int K, int ldc, float alpha) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_m = M / BM, tiles_n = N / BN, nwg = tiles_m * tiles_n;
  const int t = xcd_remap(blockIdx.x, nwg);
  const int GROUP = 4;
  const int group_id = t / (GROUP * tiles_n);
  const int first_m = group_id * GROUP;
  const int gsz = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (t % (GROUP * tiles_n)) % gsz;
  const int tn = (t % (GROUP * tiles_n)) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  // Half-tiles are split by the PHASE that first reads them, not by contiguous rows:
  //   h0 = A rows {wr*128 + 0..63}   (quadrant row mq = 0 of both wave rows)   read in phase 0
  //   h1 = A rows {wr*128 + 64..127} (mq = 1)                                 read in phase 2
  //   h2 = B rows {wc*64 + 0..31}    (quadrant col nq = 0 of all 4 wave cols) read in phase 0
  //   h3 = B rows {wc*64 + 32..63}   (nq = 1)                                 read in phase 1
  // Local row r of a half sits at r*128 B with 16-B slot s holding k-chunk s ^ ((r >> 1) & 7).
  // Half h of K-tile kt lives in slot ((kt & 1) * 4 + h); each thread stages 2 chunks per half.
  size_t offA[2], offB[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int q = j * THREADS + tid, r = q >> 3, slot = q & 7;
    const int kc = slot ^ ((r >> 1) & 7);
    offA[j] = (size_t)((r >> 6) * 128 + (r & 63)) * K + (kc << 3);
    offB[j] = (size_t)((r >> 5) * 64 + (r & 31)) * K + (kc << 3);
  }
  const u16* half_src[4] = {A + (size_t)m0 * K, A + (size_t)(m0 + 64) * K, B + (size_t)n0 * K,
                            B + (size_t)(n0 + 32) * K};
  auto stage = [&](int kt, int h) {
    unsigned char* dst = lds + ((kt & 1) * 4 + h) * HALF_BYTES + wid * 1024;
    const u16* src = half_src[h] + (size_t)kt * BK;
    const size_t* off = h < 2 ? offA : offB;
    __builtin_amdgcn_global_load_lds((const void*)(src + off[0]), (lds_void*)dst, 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(src + off[1]), (lds_void*)(dst + THREADS * 16), 16, 0, 0);
  };

  const int wr = wid >> 2, wc = wid & 3;
  const int frow = lane & 15, fq = lane >> 4, lsw = (frow >> 1) & 7;
  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fragment registers, one set per quadrant row / column: af[mq][ks][i], bfr[nq][ks][j]
  bf16x8 af[2][2][4], bfr[2][2][2];

  auto read_a = [&](int kt, int mq) {
    const unsigned char* base = lds + ((kt & 1) * 4 + mq) * HALF_BYTES + (wr * 64 + frow) * 128;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[mq][ks][i] = *reinterpret_cast<const bf16x8*>(base + i * 16 * 128 + (((ks * 4 + fq) ^ lsw) << 4));
  };
  auto read_b = [&](int kt, int nq) {
    const unsigned char* base = lds + ((kt & 1) * 4 + 2 + nq) * HALF_BYTES + (wc * 32 + frow) * 128;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bfr[nq][ks][j] = *reinterpret_cast<const bf16x8*>(base + j * 16 * 128 + (((ks * 4 + fq) ^ lsw) << 4));
  };
  auto mma = [&](int mq, int nq) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mq][nq][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mq][ks][i], bfr[nq][ks][j], acc[mq][nq][i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // Software pipeline: each phase ds_reads the fragments the NEXT phase needs while its MFMAs run
  // on registers loaded one phase earlier (h3 at p0, h1 at p1, next tile's h0 at p2 and h2 at p3).
  // Every phase starts with lgkmcnt(0) (the previous phase's reads landed) + counted vmcnt + one
  // barrier, which both publishes the glds data (RAW) and frees the slots read so far (WAR).
  // Tile u+2's halves are issued one per phase (h0 h2 h3 h1 at p0..p3) into tile u's slots.
  const int nt = K / BK;   // >= 2 (checked by the launcher)
  stage(0, 0); stage(0, 2); stage(0, 3); stage(0, 1);
  stage(1, 0); stage(1, 2); stage(1, 3); stage(1, 1);
  KAMD_WAIT_VM(12);                    // h0(0), h2(0) landed (6 half-tiles may still fly)
  KAMD_BARRIER();
  read_a(0, 0);
  read_b(0, 0);
  for (int kt = 0; kt < nt; ++kt) {
    const bool far = kt + 2 < nt, near = kt + 1 < nt;
    // p0: MFMA (0,0); read h3(kt) -> b1; issue h0(kt+2)
    KAMD_WAIT_LGKM0();
    if (near) KAMD_WAIT_VM(10); else KAMD_WAIT_VM(0);
    KAMD_BARRIER();
    read_b(kt, 1);
    if (far) stage(kt + 2, 0);
    mma(0, 0);
    // p1: MFMA (0,1); read h1(kt) -> a1; issue h2(kt+2)
    KAMD_WAIT_LGKM0();
    if (far) KAMD_WAIT_VM(10); else KAMD_WAIT_VM(0);
    KAMD_BARRIER();
    read_a(kt, 1);
    if (far) stage(kt + 2, 2);
    mma(0, 1);
    // p2: MFMA (1,0); read h0(kt+1) -> a0; issue h3(kt+2)
    KAMD_WAIT_LGKM0();
    if (far) KAMD_WAIT_VM(10); else KAMD_WAIT_VM(0);
    KAMD_BARRIER();
    if (near) read_a(kt + 1, 0);
    if (far) stage(kt + 2, 3);
    mma(1, 0);
    // p3: MFMA (1,1); read h2(kt+1) -> b0; issue h1(kt+2)
    KAMD_WAIT_LGKM0();
    if (far) KAMD_WAIT_VM(10); else KAMD_WAIT_VM(0);
    KAMD_BARRIER();
    if (near) read_b(kt + 1, 0);
    if (far) stage(kt + 2, 1);
    mma(1, 1);
  }
  // epilogue: C/D layout col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
  for (int mq = 0; mq < 2; ++mq)
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int col = n0 + wc * 64 + nq * 32 + j * 16 + frow;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = m0 + wr * 128 + mq * 64 + i * 16 + fq * 4 + r;
            store_out<OutT>(C + (size_t)row * ldc + col, alpha * acc[mq][nq][i][j][r]);
          }
        }
}
#undef KAMD_WAIT_VM
#undef KAMD_WAIT_LGKM0
#undef KAMD_BARRIER
}  // namespace gemm8

// ---------------------------------------------------------------------------
// Ping-pong 256x256 path (cdna_hip_programming.md "The 256² 8-phase template": wave groups
// staggered by one barrier). Same tile / wave geometry as gemm8 (8 waves = 2 groups (wave rows)
// x 4 wave columns, 128x64 output per wave, 4 C-quadrants of 16 MFMA 16x16x32 per K-tile), but
// every phase is   [ds_read this quadrant's fragments, stage glds] BARRIER [lgkmcnt(0), MFMAs] BARRIER
// and group 1 runs ONE barrier behind group 0: between any two barriers one group's MFMA segment
// sits beside the other group's load segment on every SIMD (each SIMD holds one wave of each
// group), so the matrix pipe is fed while the partner wave waits on LDS and barriers.
//   LDS: 2 K-tile parities x {A half 0 = rows 0..127 (group 0), A half 1 (group 1), B half 0 =
//   cols 0..127, B half 1} x 16 KiB = 128 KiB; rows of 128 B with the conflict-free slot swizzle
//   s ^ ((r >> 1) & 7) applied on the global side of global_load_lds.
//   K-tile kt+1 is staged into the other parity during K-tile kt: A halves in phase 0, B halves
//   in phase 1 (4 glds per thread); phase 3's load segment retires them (vmcnt(0)) before the
//   barrier that precedes the first read of kt+1 (WAR on that parity: its last reads, K-tile
//   kt-1 phase 2, were retired by lgkmcnt(0) one full segment before the first restage).
namespace gemmpp {
using gemm::xcd_remap;
using gemm::store_out;
constexpr int BM = 256, BN = 256, BK = 64, THREADS = 512;
constexpr int HALF_BYTES = 128 * BK * 2;          // 16 KiB
constexpr int TILE_BYTES = 4 * HALF_BYTES;        // A0 A1 B0 B1 of one K-tile
constexpr int LDS_BYTES = 2 * TILE_BYTES;         // 128 KiB
typedef __attribute__((address_space(3))) void lds_void;

#define KAMD_PP_BARRIER()                       \
  do {                                          \
    asm volatile("" ::: "memory");              \
    __builtin_amdgcn_s_barrier();               \
    asm volatile("" ::: "memory");              \
  } while (0)
#define KAMD_PP_LGKM0()                                   \
  do {                                                    \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");    \
    __builtin_amdgcn_sched_barrier(0);                    \
  } while (0)
#define KAMD_PP_VM0()                                     \
  do {                                                    \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      \
    __builtin_amdgcn_sched_barrier(0);                    \
  } while (0)
#define KAMD_WAIT_VMN(n)                                  \
  do {                                                    \
    asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory"); \
    __builtin_amdgcn_sched_barrier(0);                    \
  } while (0)

constexpr int EPI_STRIDE = 68;                    // fp32 row pitch of the LDS epilogue (bank spread)
constexpr int EPI_BYTES = 8 * 64 * EPI_STRIDE * 4;  // 8 waves x 64 x 68 fp32 = 136 KiB

// VARIANT bit 0: static priority for the second half instead of per-segment setprio flips;
// bit 1: LDS-staged 16-B epilogue.
// FP8: OCP e4m3 operands on the block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 (scales fixed at
// 2^0). A K-tile is still 128 B per row — 64 bf16 or 128 fp8 elements — so staging, LDS layout,
// swizzle and fragment reads are byte-for-byte the bf16 kernel's; the two 16-B fragments a lane
// reads for the bf16 k-steps 0 and 1 become the two halves of its 32-B fp8 operand (A and B use
// the same byte->slot map, so every product still pairs A[i][k] with B[j][k]). One fp8 MFMA
// takes the cycles of two bf16 ones at 4x the K: 2x the FLOPs per K-tile on the same traffic.
template <typename OutT, int VARIANT, bool FP8 = false>
__global__ void __launch_bounds__(THREADS, 1)
gemm_nt_pp_kernel(const void* __restrict__ Av, const void* __restrict__ Bv, OutT* __restrict__ C,
                       int M, int N, int K, int ldc, float alpha, int group) {
  // element type of the operands: addresses below are in elements, as in the bf16 original
  typedef typename std::conditional<FP8, unsigned char, u16>::type elem_t;
  constexpr int EPC = 16 / sizeof(elem_t);           // elements per 16-B chunk (8 bf16, 16 fp8)
  constexpr int BKE = 128 / sizeof(elem_t);          // elements per 128-B K-tile row
  const elem_t* A = static_cast<const elem_t*>(Av);
  const elem_t* B = static_cast<const elem_t*>(Bv);
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_m = M / BM, tiles_n = N / BN, nwg = tiles_m * tiles_n;
  const int t = xcd_remap(blockIdx.x, nwg);
  const int GROUP = group;          // tile-rows per L2 group (swizzled tile order)
  const int group_id = t / (GROUP * tiles_n);
  const int first_m = group_id * GROUP;
  const int gsz = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (t % (GROUP * tiles_n)) % gsz;
  const int tn = (t % (GROUP * tiles_n)) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  // Half-tiles are split by the PHASE that first reads them (as in gemm8), so each phase waits
  // only for its own data with a counted vmcnt and 3 half-tiles stay in flight:
  //   h0 = A rows {g*128 + 0..63}  (mq = 0 of both groups)   read in phase 0
  //   h1 = A rows {g*128 + 64..127} (mq = 1)                read in phase 2
  //   h2 = B rows {wc*64 + 0..31}   (nq = 0, all 4 columns) read in phase 0
  //   h3 = B rows {wc*64 + 32..63}  (nq = 1)                read in phase 1
  // During K-tile kt, phase p stages half ORDER[p] = h0, h2, h3, h1 of K-tile kt+1 (2 glds per
  // thread); the waits: vmcnt(4) after staging in phases 0, 1 and 3 (the half the next read
  // segment needs is then the oldest outstanding one).
  size_t offA[2], offB[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int q = j * THREADS + tid, r = q >> 3, slot = q & 7;
    const int kc = slot ^ ((r >> 1) & 7);
    offA[j] = (size_t)((r >> 6) * 128 + (r & 63)) * K + kc * EPC;
    offB[j] = (size_t)((r >> 5) * 64 + (r & 31)) * K + kc * EPC;
  }
  const elem_t* half_src[4] = {A + (size_t)m0 * K, A + (size_t)(m0 + 64) * K, B + (size_t)n0 * K,
                               B + (size_t)(n0 + 32) * K};
  auto stage = [&](int kt, const int par, int h) {
    unsigned char* dst = lds + (par * 4 + h) * HALF_BYTES + wid * 1024;
    const elem_t* src = half_src[h] + (size_t)kt * BKE;
    const size_t* off = h < 2 ? offA : offB;
    __builtin_amdgcn_global_load_lds((const void*)(src + off[0]), (lds_void*)dst, 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(src + off[1]), (lds_void*)(dst + THREADS * 16), 16, 0, 0);
  };

  const int wr = wid >> 2, wc = wid & 3;           // group = wave row
  const int frow = lane & 15, fq = lane >> 4, lsw = (frow >> 1) & 7;
  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[2][2][4], bfr[2][2][2];
  // fp8: the two 16-B reads land directly in the low / high half of one 8-VGPR operand (no copies)
  i32x8 af8[2][4], bf8[2][2];
  auto read_a = [&](const int par, int mq) {   // half h = mq, local rows wr*64 + ...
    const unsigned char* base = lds + (par * 4 + mq) * HALF_BYTES + (wr * 64 + frow) * 128;
    if constexpr (FP8) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const unsigned char* p = base + i * 16 * 128;
        af8[mq][i] = __builtin_shufflevector(*reinterpret_cast<const i32x4*>(p + ((fq ^ lsw) << 4)),
                                             *reinterpret_cast<const i32x4*>(p + (((4 + fq) ^ lsw) << 4)),
                                             0, 1, 2, 3, 4, 5, 6, 7);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          af[mq][ks][i] = *reinterpret_cast<const bf16x8*>(base + i * 16 * 128 + (((ks * 4 + fq) ^ lsw) << 4));
    }
  };
  auto read_b = [&](const int par, int nq) {   // half h = 2 + nq, local rows wc*32 + ...
    const unsigned char* base = lds + (par * 4 + 2 + nq) * HALF_BYTES + (wc * 32 + frow) * 128;
    if constexpr (FP8) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const unsigned char* p = base + j * 16 * 128;
        bf8[nq][j] = __builtin_shufflevector(*reinterpret_cast<const i32x4*>(p + ((fq ^ lsw) << 4)),
                                             *reinterpret_cast<const i32x4*>(p + (((4 + fq) ^ lsw) << 4)),
                                             0, 1, 2, 3, 4, 5, 6, 7);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bfr[nq][ks][j] = *reinterpret_cast<const bf16x8*>(base + j * 16 * 128 + (((ks * 4 + fq) ^ lsw) << 4));
    }
  };
  auto mma = [&](int mq, int nq) {
    if (!(VARIANT & 1)) __builtin_amdgcn_s_setprio(1);
    if constexpr (FP8) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          // formats A = B = 0 (fp8 e4m3), E8M0 scales 127 = 2^0
          acc[mq][nq][i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af8[mq][i], bf8[nq][j], acc[mq][nq][i][j],
                                                                                0, 0, 0, 127, 0, 127);
      // pin the MFMAs to this phase: without a use here the compiler sinks these pure ops past
      // the barriers (it does for the scaled fp8 form) and the ping-pong collapses
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(acc[mq][nq][i][j]));
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[mq][nq][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mq][ks][i], bfr[nq][ks][j], acc[mq][nq][i][j], 0, 0, 0);
    }
    if (!(VARIANT & 1)) __builtin_amdgcn_s_setprio(0);
  };

  const int nt = K / BKE;
  // TUNED: static priority for the second-dispatched half (MI355X_MICROARCH "Two waves per
  // SIMD" item 4) instead of per-segment flips
  if ((VARIANT & 1) && wr == 1) __builtin_amdgcn_s_setprio(1);
  stage(0, 0, 0); stage(0, 0, 2); stage(0, 0, 3); stage(0, 0, 1);
  KAMD_PP_VM0();
  KAMD_PP_BARRIER();                  // K-tile 0 published to every wave
  if (wr == 1) KAMD_PP_BARRIER();     // group 1 runs one barrier behind group 0
  // one K-tile; `par` = kt & 1 is a literal at each call site (the loop is unrolled by 2), so LDS
  // addresses fold to constants
  auto ktile = [&](int kt, const int par, const bool more) {
    // phase 0: read B nq=0, A mq=0 (h2, h0); stage h0(kt+1); then h3(kt) must land for phase 1
    read_b(par, 0);
    __builtin_amdgcn_sched_barrier(0);
    read_a(par, 0);
    if (more) { stage(kt + 1, par ^ 1, 0); KAMD_WAIT_VMN(4); } else { KAMD_WAIT_VMN(2); }
    KAMD_PP_BARRIER();
    KAMD_PP_LGKM0();
    mma(0, 0);
    KAMD_PP_BARRIER();
    // phase 1: read B nq=1 (h3); stage h2(kt+1); then h1(kt) must land for phase 2
    read_b(par, 1);
    if (more) { stage(kt + 1, par ^ 1, 2); KAMD_WAIT_VMN(4); } else { KAMD_PP_VM0(); }
    KAMD_PP_BARRIER();
    KAMD_PP_LGKM0();
    mma(0, 1);
    KAMD_PP_BARRIER();
    // phase 2: read A mq=1 (h1); stage h3(kt+1)
    read_a(par, 1);
    if (more) stage(kt + 1, par ^ 1, 3);
    KAMD_PP_BARRIER();
    KAMD_PP_LGKM0();
    mma(1, 0);
    KAMD_PP_BARRIER();
    // phase 3: no reads; stage h1(kt+1); then h0, h2 of kt+1 must land for its phase 0
    if (more) { stage(kt + 1, par ^ 1, 1); KAMD_WAIT_VMN(4); }
    KAMD_PP_BARRIER();
    mma(1, 1);
    KAMD_PP_BARRIER();
  };
  int kt = 0;
  for (; kt + 1 < nt; kt += 2) {
    ktile(kt, 0, true);
    ktile(kt + 1, 1, kt + 2 < nt);
  }
  if (kt < nt) ktile(kt, 0, false);
  if (wr == 0) KAMD_PP_BARRIER();     // balance group 1's extra barrier
  if (VARIANT & 2) {
    // epilogue through LDS (free now: every wave is past its last read and glds): each wave
    // transposes a 64x64 fp32 quadrant row to row-major, then writes 16-B vectors (256 B per
    // 16 lanes of a row) instead of 4-B scattered stores
    __builtin_amdgcn_s_setprio(0);
    float* ep = reinterpret_cast<float*>(lds) + wid * (64 * EPI_STRIDE);
#pragma unroll
    for (int mq = 0; mq < 2; ++mq) {
#pragma unroll
      for (int nq = 0; nq < 2; ++nq)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              ep[(i * 16 + fq * 4 + r) * EPI_STRIDE + nq * 32 + j * 16 + frow] = alpha * acc[mq][nq][i][j][r];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      const int c4 = lane & 15;
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int row = it * 4 + (lane >> 4);
        const f32x4 v = *reinterpret_cast<const f32x4*>(ep + row * EPI_STRIDE + c4 * 4);
        OutT* dst = C + (size_t)(m0 + wr * 128 + mq * 64 + row) * ldc + n0 + wc * 64 + c4 * 4;
        if constexpr (sizeof(OutT) == 4) {
          *reinterpret_cast<f32x4*>(dst) = v;
        } else {
          // 4 bf16 (8 B) per lane: 128 B per 16 lanes of a row
          typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
          *reinterpret_cast<bf16x4*>(dst) = bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
    return;
  }
  // epilogue: C/D layout col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
  for (int mq = 0; mq < 2; ++mq)
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int col = n0 + wc * 64 + nq * 32 + j * 16 + frow;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = m0 + wr * 128 + mq * 64 + i * 16 + fq * 4 + r;
            store_out<OutT>(C + (size_t)row * ldc + col, alpha * acc[mq][nq][i][j][r]);
          }
        }
}
#undef KAMD_PP_BARRIER
#undef KAMD_PP_LGKM0
#undef KAMD_PP_VM0
#undef KAMD_WAIT_VMN
}  // namespace gemmpp

// ---------------------------------------------------------------------------
// HBM streaming copy, 16 B per lane, grid-stride
__global__ void __launch_bounds__(256) hbm_copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) dst[i] = src[i];
}

// 4 independent 16-B loads in flight per lane before the stores (64 B/lane/iteration), streaming
// (non-temporal) hints so the copy does not sweep the L2 / Infinity Cache.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) hbm_copy_x4_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    u32x4 a = __builtin_nontemporal_load(src + i);
    u32x4 b = __builtin_nontemporal_load(src + i + stride);
    u32x4 c = __builtin_nontemporal_load(src + i + 2 * stride);
    u32x4 d = __builtin_nontemporal_load(src + i + 3 * stride);
    __builtin_nontemporal_store(a, dst + i);
    __builtin_nontemporal_store(b, dst + i + stride);
    __builtin_nontemporal_store(c, dst + i + 2 * stride);
    __builtin_nontemporal_store(d, dst + i + 3 * stride);
  }
  for (; i < n; i += stride) dst[i] = src[i];
}
// one 16-B element per lane, no loop: a grid of n/256 workgroups
__global__ void __launch_bounds__(256) hbm_copy_flat_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}
// x4 without the non-temporal hints
__global__ void __launch_bounds__(256) hbm_copy_x4p_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    u32x4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n; i += stride) dst[i] = src[i];
}
static int g_copy_variant = 0;   // 0: flat (one element per lane), 1: grid-stride, 2: x4 non-temporal, 3: x4 plain
static int g_copy_blocks = 0;    // 0: default grid

__global__ void fill_bf16_kernel(u16* p, size_t n, uint32_t seed, float scale) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    float f = ((float)(x & 0xFFFFFF) / 16777216.0f * 2.f - 1.f) * scale;  // uniform [-scale, scale)
    __bf16 b = (__bf16)f;
    p[i] = *reinterpret_cast<u16*>(&b);
  }
}

// random OCP e4m3 bytes with exponent field 5..8 (|v| in [0.25, 3.75]): no NaN encodings, and a
// magnitude range where fp32 accumulation of K products stays far from overflow
__global__ void fill_fp8_kernel(unsigned char* p, size_t n, uint32_t seed) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (unsigned char)(((x >> 8) & 0x80) | ((5 + ((x >> 3) & 3)) << 3) | (x & 7));
  }
}

static double fp8_e4m3_to_double(unsigned char b) {
  const int s = b >> 7, e = (b >> 3) & 15, m = b & 7;
  const double v = e == 0 ? m / 8.0 * ldexp(1.0, -6) : (1.0 + m / 8.0) * ldexp(1.0, e - 7);
  return s ? -v : v;
}

// ---------------------------------------------------------------------------
extern "C" {

const char* kamd_hip_last_error() { return g_err; }

void kamd_gemm_set_path(int path) { g_gemm_path = path; }
void kamd_gemm_set_group(int group) { g_pp_group = group > 0 ? group : 4; }

int kamd_hip_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int kamd_hip_device_arch(int dev, char* out, int len) {
  hipDeviceProp_t p;
  HC(hipGetDeviceProperties(&p, dev));
  snprintf(out, len, "%s", p.gcnArchName);
  return 0;
}

// async launches on a caller stream (torch tensors)
int kamd_vector_add_launch(const float* a, const float* b, float* c, int n, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(vector_add_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, a, b, c, n);
  return check(hipGetLastError(), "vector_add launch");
}

// fp8 (OCP e4m3) GEMM C = alpha * A @ B^T on the ping-pong kernel: A M x K, B N x K row-major
// bytes; M, N multiples of 256, K a multiple of 128 (no other tile path exists for fp8).
int kamd_gemm_fp8_nt_launch(const void* A, const void* B, void* C, int M, int N, int K, int ldc, float alpha,
                            int out_fp32, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (M % gemmpp::BM || N % gemmpp::BN || K % 128) {
    snprintf(g_err, sizeof g_err, "gemm_fp8_nt: need M, N %% 256 == 0 and K %% 128 == 0 (got %d x %d x %d)", M, N, K);
    return -1;
  }
  if ((((uintptr_t)A) | ((uintptr_t)B)) & 15) {
    snprintf(g_err, sizeof g_err, "gemm_fp8_nt: A/B must be 16-byte aligned");
    return -1;
  }
  const int tiles = (M / gemmpp::BM) * (N / gemmpp::BN);
  // LDS-staged vector epilogue: default for bf16 output (+1-3 %), set_gemm_path(4) forces it,
  // any other path forces the register epilogue (A/B experiments)
  const bool lds_epi = g_gemm_path == 4 || (g_gemm_path == 0 && !out_fp32);
  const size_t lds = lds_epi ? gemmpp::EPI_BYTES : gemmpp::LDS_BYTES;
#define KAMD_F8_LAUNCH(T, V)                                                                                 \
  do {                                                                                                       \
    static bool attr = false;                                                                                \
    if (!attr) {                                                                                             \
      HC(hipFuncSetAttribute((const void*)gemmpp::gemm_nt_pp_kernel<T, V, true>,                              \
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));                         \
      attr = true;                                                                                           \
    }                                                                                                        \
    hipLaunchKernelGGL((gemmpp::gemm_nt_pp_kernel<T, V, true>), dim3(tiles), dim3(gemmpp::THREADS), lds,      \
                       stream, A, B, (T*)C, M, N, K, ldc, alpha, g_pp_group);                                \
  } while (0)
  if (out_fp32) {
    if (lds_epi) KAMD_F8_LAUNCH(float, 2); else KAMD_F8_LAUNCH(float, 0);
  } else {
    if (lds_epi) KAMD_F8_LAUNCH(__bf16, 2); else KAMD_F8_LAUNCH(__bf16, 0);
  }
#undef KAMD_F8_LAUNCH
  return check(hipGetLastError(), "gemm fp8 launch");
}

int kamd_gemm_bf16_nt_launch(const void* A, const void* B, void* C, int M, int N, int K, int ldc, float alpha,
                             int out_fp32, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (K % 8 != 0) {
    snprintf(g_err, sizeof g_err, "gemm_bf16_nt: K (%d) must be a multiple of 8", K);
    return -1;
  }
  if ((((uintptr_t)A) | ((uintptr_t)B)) & 15) {
    snprintf(g_err, sizeof g_err, "gemm_bf16_nt: A/B must be 16-byte aligned");
    return -1;
  }
  if ((g_gemm_path == 0 || (g_gemm_path >= 3 && g_gemm_path <= 6)) && M % gemmpp::BM == 0 && N % gemmpp::BN == 0 && K % gemmpp::BK == 0) {
    // path 3: variant 0, 4: LDS epilogue, 5: static priority, 6: both; auto (0) takes the LDS-staged
    // vector epilogue for bf16 output (+1.3-1.8 %, profiles/r2_gemm_fp8/epilogue_ab.txt)
    const int variant = g_gemm_path == 0 ? (out_fp32 ? 0 : 2)
                        : g_gemm_path == 3 ? 0 : g_gemm_path == 4 ? 2 : g_gemm_path == 5 ? 1 : 3;
    const size_t lds = (variant & 2) ? gemmpp::EPI_BYTES : gemmpp::LDS_BYTES;
    const int tiles = (M / gemmpp::BM) * (N / gemmpp::BN);
#define KAMD_PP_LAUNCH(T, V)                                                                                   \
  do {                                                                                                         \
    static bool attr = false;                                                                                  \
    if (!attr) {                                                                                               \
      HC(hipFuncSetAttribute((const void*)gemmpp::gemm_nt_pp_kernel<T, V>,                                \
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));                           \
      attr = true;                                                                                             \
    }                                                                                                          \
    hipLaunchKernelGGL((gemmpp::gemm_nt_pp_kernel<T, V>), dim3(tiles), dim3(gemmpp::THREADS), lds, stream, \
                       A, B, (T*)C, M, N, K, ldc, alpha, g_pp_group);                                          \
  } while (0)
    if (out_fp32) {
      switch (variant) {
        case 0: KAMD_PP_LAUNCH(float, 0); break;
        case 1: KAMD_PP_LAUNCH(float, 1); break;
        case 2: KAMD_PP_LAUNCH(float, 2); break;
        default: KAMD_PP_LAUNCH(float, 3); break;
      }
    } else {
      switch (variant) {
        case 0: KAMD_PP_LAUNCH(__bf16, 0); break;
        case 1: KAMD_PP_LAUNCH(__bf16, 1); break;
        case 2: KAMD_PP_LAUNCH(__bf16, 2); break;
        default: KAMD_PP_LAUNCH(__bf16, 3); break;
      }
    }
#undef KAMD_PP_LAUNCH
    return check(hipGetLastError(), "gemm ping-pong launch");
  }
  if (g_gemm_path == 7 && M % gemm8::BM == 0 && N % gemm8::BN == 0 && K % gemm8::BK == 0 && K / gemm8::BK >= 2) {
    static bool attr8 = false;
    if (!attr8) {
      HC(hipFuncSetAttribute((const void*)gemm8::gemm_bf16_nt_8ph_kernel<float>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, gemm8::LDS_BYTES));
      HC(hipFuncSetAttribute((const void*)gemm8::gemm_bf16_nt_8ph_kernel<__bf16>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, gemm8::LDS_BYTES));
      attr8 = true;
    }
    const int tiles = (M / gemm8::BM) * (N / gemm8::BN);
    if (out_fp32)
      hipLaunchKernelGGL(gemm8::gemm_bf16_nt_8ph_kernel<float>, dim3(tiles), dim3(gemm8::THREADS), gemm8::LDS_BYTES,
                         stream, (const u16*)A, (const u16*)B, (float*)C, M, N, K, ldc, alpha);
    else
      hipLaunchKernelGGL(gemm8::gemm_bf16_nt_8ph_kernel<__bf16>, dim3(tiles), dim3(gemm8::THREADS), gemm8::LDS_BYTES,
                         stream, (const u16*)A, (const u16*)B, (__bf16*)C, M, N, K, ldc, alpha);
    return check(hipGetLastError(), "gemm8 launch");
  }
  if (g_gemm_path != 1 && M % gemm256::BM == 0 && N % gemm256::BN == 0 && K % gemm256::BK == 0) {
    static bool attr_set = false;
    if (!attr_set) {   // > 64 KiB of dynamic LDS must be opted into per kernel
      HC(hipFuncSetAttribute((const void*)gemm256::gemm_bf16_nt_256_kernel<float>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, gemm256::LDS_BYTES));
      HC(hipFuncSetAttribute((const void*)gemm256::gemm_bf16_nt_256_kernel<__bf16>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, gemm256::LDS_BYTES));
      attr_set = true;
    }
    const int tiles256 = (M / gemm256::BM) * (N / gemm256::BN);
    if (out_fp32)
      hipLaunchKernelGGL(gemm256::gemm_bf16_nt_256_kernel<float>, dim3(tiles256), dim3(gemm256::THREADS),
                         gemm256::LDS_BYTES, stream, (const u16*)A, (const u16*)B, (float*)C, M, N, K, ldc, alpha);
    else
      hipLaunchKernelGGL(gemm256::gemm_bf16_nt_256_kernel<__bf16>, dim3(tiles256), dim3(gemm256::THREADS),
                         gemm256::LDS_BYTES, stream, (const u16*)A, (const u16*)B, (__bf16*)C, M, N, K, ldc, alpha);
    return check(hipGetLastError(), "gemm256 launch");
  }
  const int tiles = ((M + gemm::BM - 1) / gemm::BM) * ((N + gemm::BN - 1) / gemm::BN);
  const size_t lds = 2 * 2 * gemm::TILE_BYTES;
  if (out_fp32) {
    hipLaunchKernelGGL(gemm::gemm_bf16_nt_kernel<float>, dim3(tiles), dim3(gemm::THREADS), lds, stream,
                       (const u16*)A, (const u16*)B, (float*)C, M, N, K, ldc, alpha);
  } else {
    hipLaunchKernelGGL(gemm::gemm_bf16_nt_kernel<__bf16>, dim3(tiles), dim3(gemm::THREADS), lds, stream,
                       (const u16*)A, (const u16*)B, (__bf16*)C, M, N, K, ldc, alpha);
  }
  return check(hipGetLastError(), "gemm launch");
}

int kamd_hbm_copy_launch(const void* src, void* dst, size_t bytes, hipStream_t stream) {
  size_t n = bytes / 16;
  // measured on MI355X (profiles/r1_hbm): flat 6.2 TB/s, grid-stride loops 4.7-5.3 TB/s
  if (g_copy_variant == 1) {
    hipLaunchKernelGGL(hbm_copy_kernel, dim3(256 * 8), dim3(256), 0, stream, (const uint4*)src, (uint4*)dst, n);
  } else if (g_copy_variant == 2) {
    const int blocks = g_copy_blocks > 0 ? g_copy_blocks : 256 * 8;   // 8 WGs (32 waves) per CU
    hipLaunchKernelGGL(hbm_copy_x4_kernel, dim3(blocks), dim3(256), 0, stream, (const u32x4*)src, (u32x4*)dst, n);
  } else if (g_copy_variant == 3) {
    const int blocks = g_copy_blocks > 0 ? g_copy_blocks : 256 * 8;
    hipLaunchKernelGGL(hbm_copy_x4p_kernel, dim3(blocks), dim3(256), 0, stream, (const u32x4*)src, (u32x4*)dst, n);
  } else {
    hipLaunchKernelGGL(hbm_copy_flat_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, (const u32x4*)src,
                       (u32x4*)dst, n);
  }
  return check(hipGetLastError(), "hbm_copy launch");
}

void kamd_hbm_copy_config(int variant, int blocks) {
  g_copy_variant = variant;
  g_copy_blocks = blocks;
}

// --- self-contained diagnostics (allocate, run, verify, free) -------------

// vectorAdd sample semantics: returns 0 and prints nothing; *max_err = max |c - (a+b)|.
int kamd_diag_vector_add(int dev, int n, float* max_err) {
  HC(hipSetDevice(dev));
  std::vector<float> ha(n), hb(n), hc(n);
  for (int i = 0; i < n; ++i) {
    ha[i] = (float)((i * 1103515245u + 12345u) % 10007) / 10007.f;
    hb[i] = (float)((i * 2654435761u + 7u) % 10009) / 10009.f;
  }
  float *da = nullptr, *db = nullptr, *dc = nullptr;
  size_t bytes = (size_t)n * sizeof(float);
  HC(hipMalloc(&da, bytes));
  HC(hipMalloc(&db, bytes));
  HC(hipMalloc(&dc, bytes));
  HC(hipMemcpy(da, ha.data(), bytes, hipMemcpyHostToDevice));
  HC(hipMemcpy(db, hb.data(), bytes, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(vector_add_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, da, db, dc, n);
  HC(hipGetLastError());
  HC(hipMemcpy(hc.data(), dc, bytes, hipMemcpyDeviceToHost));
  float e = 0.f;
  for (int i = 0; i < n; ++i) {
    float d = hc[i] - (ha[i] + hb[i]);
    if (d < 0) d = -d;
    if (d > e) e = d;
  }
  *max_err = e;
  hipFree(da);
  hipFree(db);
  hipFree(dc);
  return 0;
}

// fp8 MFMA burn-in: the block-scaled fp8 path (v_mfma_scale_f32_16x16x128_f8f6f4), same protocol
// as kamd_diag_mfma (size must be a multiple of 256).
int kamd_diag_mfma_fp8(int dev, int size, int iters, double* tflops, double* max_rel_err) {
  HC(hipSetDevice(dev));
  const int M = size, N = size, K = size;
  unsigned char *A = nullptr, *B = nullptr;
  float* C = nullptr;
  HC(hipMalloc(&A, (size_t)M * K));
  HC(hipMalloc(&B, (size_t)N * K));
  HC(hipMalloc(&C, (size_t)M * N * 4));
  int rc = -1;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  do {
    hipLaunchKernelGGL(fill_fp8_kernel, dim3(1024), dim3(256), 0, 0, A, (size_t)M * K, 0x1234u);
    hipLaunchKernelGGL(fill_fp8_kernel, dim3(1024), dim3(256), 0, 0, B, (size_t)N * K, 0x9876u);
    if (check(hipGetLastError(), "fill_fp8") != 0) break;
    if (kamd_gemm_fp8_nt_launch(A, B, C, M, N, K, N, 1.f, 1, 0) != 0) break;   // warm-up
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) break;
    hipEventRecord(e0, 0);
    bool ok = true;
    for (int i = 0; i < iters && ok; ++i) ok = kamd_gemm_fp8_nt_launch(A, B, C, M, N, K, N, 1.f, 1, 0) == 0;
    if (!ok) break;
    hipEventRecord(e1, 0);
    if (check(hipEventSynchronize(e1), "diag_mfma_fp8 sync") != 0) break;
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    *tflops = 2.0 * M * N * (double)K * iters / (ms * 1e-3) / 1e12;
    std::vector<unsigned char> ha((size_t)M * K), hb((size_t)N * K);
    std::vector<float> hc((size_t)M * N);
    if (check(hipMemcpy(ha.data(), A, ha.size(), hipMemcpyDeviceToHost), "copy A") != 0) break;
    if (check(hipMemcpy(hb.data(), B, hb.size(), hipMemcpyDeviceToHost), "copy B") != 0) break;
    if (check(hipMemcpy(hc.data(), C, hc.size() * 4, hipMemcpyDeviceToHost), "copy C") != 0) break;
    double worst = 0;
    for (int s = 0; s < 256; ++s) {
      int i = (int)((s * 7919u) % (unsigned)M), j = (int)((s * 104729u + 13u) % (unsigned)N);
      double ref = 0, mag = 0;
      for (int k = 0; k < K; ++k) {
        double pr = fp8_e4m3_to_double(ha[(size_t)i * K + k]) * fp8_e4m3_to_double(hb[(size_t)j * K + k]);
        ref += pr;
        mag += pr < 0 ? -pr : pr;
      }
      double err = hc[(size_t)i * N + j] - ref;
      if (err < 0) err = -err;
      double rel = err / (mag > 1e-30 ? mag : 1.0);
      if (rel > worst) worst = rel;
    }
    *max_rel_err = worst;
    rc = 0;
  } while (0);
  if (e0) hipEventDestroy(e0);
  if (e1) hipEventDestroy(e1);
  hipFree(A);
  hipFree(B);
  hipFree(C);
  return rc;
}

// MFMA burn-in: random bf16 operands, `iters` timed GEMMs of M=N=K=`size`; result checked on
// a sampled set of output elements against an fp64 host dot product.
int kamd_diag_mfma(int dev, int size, int iters, double* tflops, double* max_rel_err) {
  HC(hipSetDevice(dev));
  const int M = size, N = size, K = size;
  u16 *A = nullptr, *B = nullptr;
  float* C = nullptr;
  HC(hipMalloc(&A, (size_t)M * K * 2));
  HC(hipMalloc(&B, (size_t)N * K * 2));
  HC(hipMalloc(&C, (size_t)M * N * 4));
  hipLaunchKernelGGL(fill_bf16_kernel, dim3(1024), dim3(256), 0, 0, A, (size_t)M * K, 0x1234u, 1.f);
  hipLaunchKernelGGL(fill_bf16_kernel, dim3(1024), dim3(256), 0, 0, B, (size_t)N * K, 0x9876u, 1.f);
  HC(hipGetLastError());
  if (kamd_gemm_bf16_nt_launch(A, B, C, M, N, K, N, 1.f, 1, 0) != 0) return -1;  // warm-up
  hipEvent_t e0, e1;
  HC(hipEventCreate(&e0));
  HC(hipEventCreate(&e1));
  HC(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i)
    if (kamd_gemm_bf16_nt_launch(A, B, C, M, N, K, N, 1.f, 1, 0) != 0) return -1;
  HC(hipEventRecord(e1, 0));
  HC(hipEventSynchronize(e1));
  float ms = 0.f;
  HC(hipEventElapsedTime(&ms, e0, e1));
  *tflops = 2.0 * M * N * (double)K * iters / (ms * 1e-3) / 1e12;
  // verify 256 sampled outputs
  std::vector<u16> ha((size_t)M * K), hb((size_t)N * K);
  std::vector<float> hc((size_t)M * N);
  HC(hipMemcpy(ha.data(), A, ha.size() * 2, hipMemcpyDeviceToHost));
  HC(hipMemcpy(hb.data(), B, hb.size() * 2, hipMemcpyDeviceToHost));
  HC(hipMemcpy(hc.data(), C, hc.size() * 4, hipMemcpyDeviceToHost));
  auto bf = [](u16 v) { uint32_t u = (uint32_t)v << 16; float f; memcpy(&f, &u, 4); return (double)f; };
  double worst = 0;
  for (int s = 0; s < 256; ++s) {
    int i = (int)((s * 7919u) % (unsigned)M), j = (int)((s * 104729u + 13u) % (unsigned)N);
    double ref = 0, mag = 0;
    for (int k = 0; k < K; ++k) {
      double p = bf(ha[(size_t)i * K + k]) * bf(hb[(size_t)j * K + k]);
      ref += p;
      mag += p < 0 ? -p : p;
    }
    double err = hc[(size_t)i * N + j] - ref;
    if (err < 0) err = -err;
    double rel = err / (mag > 1e-30 ? mag : 1.0);
    if (rel > worst) worst = rel;
  }
  *max_rel_err = worst;
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipFree(A);
  hipFree(B);
  hipFree(C);
  return 0;
}

int kamd_diag_hbm(int dev, size_t bytes, int iters, double* gbps) {
  HC(hipSetDevice(dev));
  void *s = nullptr, *d = nullptr;
  HC(hipMalloc(&s, bytes));
  HC(hipMalloc(&d, bytes));
  HC(hipMemset(s, 1, bytes));
  kamd_hbm_copy_launch(s, d, bytes, 0);
  hipEvent_t e0, e1;
  HC(hipEventCreate(&e0));
  HC(hipEventCreate(&e1));
  HC(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) kamd_hbm_copy_launch(s, d, bytes, 0);
  HC(hipEventRecord(e1, 0));
  HC(hipEventSynchronize(e1));
  float ms = 0.f;
  HC(hipEventElapsedTime(&ms, e0, e1));
  *gbps = 2.0 * (double)bytes * iters / (ms * 1e-3) / 1e9;  // read + write
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipFree(s);
  hipFree(d);
  return 0;
}

// Persistent per-GPU payload context (warm HIP context + buffers): the stub runtime's
// "container start" for GPU pods runs vector_add on the pod's device and verifies it.
// Container-start payload. One call = one GPU container start = one vector_add launch into its
// own output slot; a batch of k starts (k container starts that reached the rank together) is
// k launches + ONE verify kernel that checks sampled elements of every slot and writes a pass
// flag per start straight into pinned host memory, then ONE stream sync — instead of k
// launch + pageable-memcpy + sync round trips.
constexpr int PAYLOAD_SLOTS = 256;

struct kamd_payload {
  int dev;
  int n;
  float *a, *b, *c;        // c: PAYLOAD_SLOTS output slots of n floats
  float* host;
  int* flags;              // pinned host, PAYLOAD_SLOTS pass flags
  int next;                // next output slot (round robin)
  hipStream_t stream;
};

__device__ __forceinline__ void payload_samples(int n, int* idx) {
  idx[0] = 0;
  idx[1] = n / 3;
  idx[2] = n / 2;
  idx[3] = n - 1;
}

__global__ void __launch_bounds__(256) payload_poison_kernel(float* __restrict__ c, int n, int first, int k) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= k) return;
  float* cs = c + (size_t)((first + j) % PAYLOAD_SLOTS) * n;
  int idx[4];
  payload_samples(n, idx);
#pragma unroll
  for (int q = 0; q < 4; ++q) cs[idx[q]] = -1.f;   // never a valid a + b (both >= 0)
}

__global__ void __launch_bounds__(256) payload_verify_kernel(const float* __restrict__ c, int n, int first, int k,
                                                             int* __restrict__ flags) {
  // one thread per start: 4 sampled elements of its slot must equal a + b = 2 * (i % 1000)
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= k) return;
  const int slot = (first + j) % PAYLOAD_SLOTS;
  const float* cs = c + (size_t)slot * n;
  int idx[4];
  payload_samples(n, idx);
  int ok = 1;
#pragma unroll
  for (int q = 0; q < 4; ++q) ok &= cs[idx[q]] == 2.f * (float)(idx[q] % 1000);
  flags[j] = ok;
}

void* kamd_payload_create(int dev, int n) {
  if (n < 1 || hipSetDevice(dev) != hipSuccess) return nullptr;
  kamd_payload* p = new kamd_payload();
  p->dev = dev;
  p->n = n;
  p->next = 0;
  size_t bytes = (size_t)n * sizeof(float);
  if (hipMalloc(&p->a, bytes) != hipSuccess || hipMalloc(&p->b, bytes) != hipSuccess ||
      hipMalloc(&p->c, bytes * PAYLOAD_SLOTS) != hipSuccess || hipHostMalloc(&p->host, bytes) != hipSuccess ||
      hipHostMalloc(&p->flags, PAYLOAD_SLOTS * sizeof(int)) != hipSuccess ||
      hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess) {
    delete p;
    return nullptr;
  }
  for (int i = 0; i < n; ++i) p->host[i] = (float)(i % 1000);
  hipMemcpy(p->a, p->host, bytes, hipMemcpyHostToDevice);
  hipMemcpy(p->b, p->host, bytes, hipMemcpyHostToDevice);
  return p;
}

// Runs k payloads (1 <= k <= PAYLOAD_SLOTS); ok[j] = 1 if start j computed c == a + b.
// Returns 0 when every start passed, 1 if any failed verification, -1 on a HIP error.
int kamd_payload_run_batch(void* h, int k, int* ok) {
  kamd_payload* p = (kamd_payload*)h;
  if (!p || k < 1 || k > PAYLOAD_SLOTS) return -1;
  if (hipSetDevice(p->dev) != hipSuccess) return -1;
  const int first = p->next;
  // a stale slot must not pass by itself: poison the sampled elements of every slot first
  hipLaunchKernelGGL(payload_poison_kernel, dim3((k + 255) / 256), dim3(256), 0, p->stream, p->c, p->n, first, k);
  for (int j = 0; j < k; ++j) {
    float* cs = p->c + (size_t)((first + j) % PAYLOAD_SLOTS) * p->n;
    hipLaunchKernelGGL(vector_add_kernel, dim3((p->n + 255) / 256), dim3(256), 0, p->stream, p->a, p->b, cs, p->n);
  }
  p->next = (first + k) % PAYLOAD_SLOTS;
  hipLaunchKernelGGL(payload_verify_kernel, dim3((k + 255) / 256), dim3(256), 0, p->stream, p->c, p->n, first, k,
                     p->flags);
  if (hipGetLastError() != hipSuccess || hipStreamSynchronize(p->stream) != hipSuccess) return -1;
  int all = 1;
  for (int j = 0; j < k; ++j) {
    ok[j] = p->flags[j];
    all &= ok[j];
  }
  return all ? 0 : 1;
}

// Runs one payload; returns 0 if c == a + b on sampled elements.
int kamd_payload_run(void* h) {
  int ok = 0;
  return kamd_payload_run_batch(h, 1, &ok);
}

void kamd_payload_destroy(void* h) {
  kamd_payload* p = (kamd_payload*)h;
  if (!p) return;
  hipSetDevice(p->dev);
  hipStreamDestroy(p->stream);
  hipFree(p->a);
  hipFree(p->b);
  hipFree(p->c);
  hipHostFree(p->host);
  hipHostFree(p->flags);
  delete p;
}

}  // extern "C"
