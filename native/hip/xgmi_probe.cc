// xgmi-probe — RCCL all-reduce over the GPUs visible to this process (one RCCL rank per GPU,
// single-process multi-device mode). Reports algorithm and bus bandwidth like rccl-tests:
// busBW = algBW * 2(n-1)/n. Used as (a) a device-plugin/e2e check that an allocated GPU set
// really sits in one fully connected xGMI hive and (b) a link-health probe.
// SURVEY §2.3 "Collective over the GPU fabric".
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

// rank r starts from x[e] = (r + 1) + (e % 8): after the sum every element of every rank must be
// n(n+1)/2 + n*(e % 8) — exact in fp32 for these small integers, and a mis-placed or missing
// chunk shows as a wrong value at its offset
__global__ void init_pattern(float* x, size_t n, int rank) {
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x)
    x[e] = (float)(rank + 1) + (float)(e % 8);
}

__global__ void count_bad(const float* x, size_t n, int ranks, unsigned long long* bad) {
  unsigned long long mine = 0;
  const float base = (float)ranks * (ranks + 1) / 2;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x)
    mine += x[e] != base + (float)ranks * (float)(e % 8);
  if (mine) atomicAdd(bad, mine);
}

#define HIPCHK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
#define NCCLCHK(x) do { ncclResult_t r = (x); if (r != ncclSuccess) { fprintf(stderr, "%s: %s\n", #x, ncclGetErrorString(r)); return 1; } } while (0)

// --p2p [MiB] [iters]: pairwise peer-to-peer copy bandwidth (hipMemcpyPeerAsync, src stream
// timed with events) for every ordered pair of visible GPUs, plus each GPU's local
// device-to-device copy bandwidth; one JSON object. The device plugin turns pairs that are far
// below a healthy xGMI link into missing edges of the published link graph.
static int p2p(size_t mib, int iters) {
  int n = 0;
  HIPCHK(hipGetDeviceCount(&n));
  if (n < 1) { fprintf(stderr, "no devices\n"); return 2; }
  size_t bytes = mib << 20;
  std::vector<void*> a(n), b(n);
  std::vector<hipStream_t> st(n);
  for (int i = 0; i < n; ++i) {
    HIPCHK(hipSetDevice(i));
    HIPCHK(hipMalloc(&a[i], bytes));
    HIPCHK(hipMalloc(&b[i], bytes));
    HIPCHK(hipMemset(a[i], i + 1, bytes));
    HIPCHK(hipStreamCreate(&st[i]));
  }
  auto timed = [&](int dev, auto&& op, double* gbps) -> int {
    hipEvent_t e0, e1;
    HIPCHK(hipSetDevice(dev));
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    if (op()) return 1;                                   // warm-up (maps peer memory)
    HIPCHK(hipStreamSynchronize(st[dev]));
    HIPCHK(hipEventRecord(e0, st[dev]));
    for (int k = 0; k < iters; ++k) if (op()) return 1;
    HIPCHK(hipEventRecord(e1, st[dev]));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    *gbps = (double)bytes * iters / (ms / 1e3) / 1e9;
    HIPCHK(hipEventDestroy(e0));
    HIPCHK(hipEventDestroy(e1));
    return 0;
  };
  printf("{\"mode\": \"p2p\", \"devices\": %d, \"bytes\": %zu, \"local\": [", n, bytes);
  for (int i = 0; i < n; ++i) {
    double g = 0;
    if (timed(i, [&]() -> int { HIPCHK(hipMemcpyAsync(b[i], a[i], bytes, hipMemcpyDeviceToDevice, st[i])); return 0; }, &g)) return 1;
    printf("%s{\"dev\": %d, \"GBps\": %.1f}", i ? ", " : "", i, g);
  }
  printf("], \"pairs\": [");
  bool first = true;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      if (i == j) continue;
      int can = 0;
      HIPCHK(hipDeviceCanAccessPeer(&can, i, j));
      double g = 0;
      if (can) {
        HIPCHK(hipSetDevice(i));
        hipError_t e = hipDeviceEnablePeerAccess(j, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) { fprintf(stderr, "peer %d->%d: %s\n", i, j, hipGetErrorString(e)); return 1; }
        (void)hipGetLastError();
      }
      if (timed(i, [&]() -> int { HIPCHK(hipMemcpyPeerAsync(b[j], j, a[i], i, bytes, st[i])); return 0; }, &g)) return 1;
      printf("%s{\"src\": %d, \"dst\": %d, \"peer\": %s, \"GBps\": %.1f}", first ? "" : ", ", i, j, can ? "true" : "false", g);
      first = false;
    }
  printf("]}\n");
  for (int i = 0; i < n; ++i) { hipSetDevice(i); hipFree(a[i]); hipFree(b[i]); hipStreamDestroy(st[i]); }
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && strcmp(argv[1], "--p2p") == 0)
    return p2p(argc > 2 ? (size_t)atol(argv[2]) : 256, argc > 3 ? atoi(argv[3]) : 10);
  size_t mib = argc > 1 ? (size_t)atol(argv[1]) : 256;
  int iters = argc > 2 ? atoi(argv[2]) : 20;
  int n = 0;
  HIPCHK(hipGetDeviceCount(&n));
  if (n < 1) { fprintf(stderr, "no devices\n"); return 2; }
  if (mib < 1) mib = 1;
  size_t count = mib * (1 << 20) / sizeof(float);
  std::vector<int> devs(n);
  for (int i = 0; i < n; ++i) devs[i] = i;
  std::vector<ncclComm_t> comms(n);
  NCCLCHK(ncclCommInitAll(comms.data(), n, devs.data()));
  std::vector<float*> buf(n);
  std::vector<hipStream_t> st(n);
  const int kBlocks = 1024, kThreads = 256;   // >> 256 CUs, grid-stride over the buffer
  for (int i = 0; i < n; ++i) {
    HIPCHK(hipSetDevice(i));
    HIPCHK(hipMalloc(&buf[i], count * sizeof(float)));
    HIPCHK(hipStreamCreate(&st[i]));
    hipLaunchKernelGGL(init_pattern, dim3(kBlocks), dim3(kThreads), 0, st[i], buf[i], count, i);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(st[i]));
  }
  auto run = [&](int k) -> int {
    for (int it = 0; it < k; ++it) {
      NCCLCHK(ncclGroupStart());
      for (int i = 0; i < n; ++i) NCCLCHK(ncclAllReduce(buf[i], buf[i], count, ncclFloat, ncclSum, comms[i], st[i]));
      NCCLCHK(ncclGroupEnd());
    }
    for (int i = 0; i < n; ++i) { HIPCHK(hipSetDevice(i)); HIPCHK(hipStreamSynchronize(st[i])); }
    return 0;
  };
  if (run(1)) return 1;
  // correctness after one all-reduce: the WHOLE buffer, on EVERY rank
  std::vector<unsigned long long> bad(n, 0);
  unsigned long long total_bad = 0;
  for (int i = 0; i < n; ++i) {
    HIPCHK(hipSetDevice(i));
    unsigned long long* d_bad = nullptr;
    HIPCHK(hipMalloc(&d_bad, sizeof(unsigned long long)));
    HIPCHK(hipMemset(d_bad, 0, sizeof(unsigned long long)));
    hipLaunchKernelGGL(count_bad, dim3(kBlocks), dim3(kThreads), 0, st[i], buf[i], count, n, d_bad);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(st[i]));
    HIPCHK(hipMemcpy(&bad[i], d_bad, sizeof(unsigned long long), hipMemcpyDeviceToHost));
    HIPCHK(hipFree(d_bad));
    total_bad += bad[i];
  }
  bool correct = total_bad == 0;
  // timing on EVERY rank's stream: a slow peer shows up as its own (and everyone's) longer
  // time, not only through the final host sync; the reported time is the slowest rank's
  std::vector<hipEvent_t> e0(n), e1(n);
  for (int i = 0; i < n; ++i) {
    HIPCHK(hipSetDevice(i));
    HIPCHK(hipEventCreate(&e0[i]));
    HIPCHK(hipEventCreate(&e1[i]));
    HIPCHK(hipEventRecord(e0[i], st[i]));
  }
  for (int it = 0; it < iters; ++it) {
    NCCLCHK(ncclGroupStart());
    for (int i = 0; i < n; ++i) NCCLCHK(ncclAllReduce(buf[i], buf[i], count, ncclFloat, ncclSum, comms[i], st[i]));
    NCCLCHK(ncclGroupEnd());
  }
  for (int i = 0; i < n; ++i) {
    HIPCHK(hipSetDevice(i));
    HIPCHK(hipEventRecord(e1[i], st[i]));
  }
  std::vector<double> rank_s(n, 0.0);
  double t = 0, tmin = 1e30;
  for (int i = 0; i < n; ++i) {
    HIPCHK(hipSetDevice(i));
    HIPCHK(hipEventSynchronize(e1[i]));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e0[i], e1[i]));
    rank_s[i] = ms / 1e3 / iters;
    if (rank_s[i] > t) t = rank_s[i];
    if (rank_s[i] < tmin) tmin = rank_s[i];
    HIPCHK(hipEventDestroy(e0[i]));
    HIPCHK(hipEventDestroy(e1[i]));
  }
  double bytes = (double)count * sizeof(float);
  printf("{\"ranks\": %d, \"bytes\": %zu, \"time_us\": %.1f, \"time_us_min_rank\": %.1f, \"rank_time_us\": [",
         n, count * sizeof(float), t * 1e6, tmin * 1e6);
  for (int i = 0; i < n; ++i) printf("%s%.1f", i ? ", " : "", rank_s[i] * 1e6);
  if (n > 1) {
    double algbw = bytes / t / 1e9;
    double busbw = algbw * 2.0 * (n - 1) / n;
    double busbw_fast = bytes / tmin / 1e9 * 2.0 * (n - 1) / n;
    printf("], \"algbw_GBps\": %.2f, \"busbw_GBps\": %.2f, \"busbw_GBps_fastest_rank\": %.2f, ", algbw, busbw, busbw_fast);
  } else {
    // one rank moves nothing over xGMI: RCCL's single-rank all-reduce is a local no-op, so any
    // bandwidth figure would be meaningless (and could be asserted against a floor)
    printf("], \"algbw_GBps\": null, \"busbw_GBps\": null, \"busbw_GBps_fastest_rank\": null, ");
  }
  printf("\"elements_checked_per_rank\": %zu, \"bad_elements\": [", count);
  for (int i = 0; i < n; ++i) printf("%s%llu", i ? ", " : "", bad[i]);
  printf("], \"correct\": %s}\n", correct ? "true" : "false");
  for (int i = 0; i < n; ++i) { ncclCommDestroy(comms[i]); hipSetDevice(i); hipFree(buf[i]); }
  return correct ? 0 : 3;
}
