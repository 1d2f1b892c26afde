// hip-vector-add — GPU e2e test workload (the MI355X analog of cuda-samples vectorAdd used by
// the reference's test/images/cuda-vector-add image, test/e2e/scheduling/nvidia-gpus.go:51-113).
// Runs on the device(s) the runtime exposed to the container (HIP_VISIBLE_DEVICES /
// ROCR_VISIBLE_DEVICES set by the amd.com/gpu device plugin) and prints "Test PASSED".
//   hip-vector-add [N] [--hold-mib M --hold-seconds S]
// --hold-mib keeps M MiB of HBM allocated (and touched) for S seconds after the test, so the
// per-container GPU memory attribution of the kubelet summary API can be checked end to end.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

extern "C" int kamd_diag_vector_add(int dev, int n, float* max_err);
extern "C" const char* kamd_hip_last_error();

int main(int argc, char** argv) {
  int n = 50000;
  long hold_mib = 0, hold_s = 0;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--hold-mib") && i + 1 < argc) hold_mib = atol(argv[++i]);
    else if (!strcmp(argv[i], "--hold-seconds") && i + 1 < argc) hold_s = atol(argv[++i]);
    else n = atoi(argv[i]);
  }
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
    fprintf(stderr, "no HIP device visible\n");
    return 2;
  }
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  printf("[Vector addition of %d elements] on %s (%s), %d visible device(s)\n", n, p.name, p.gcnArchName, count);
  float err = 0;
  if (kamd_diag_vector_add(0, n, &err) != 0) {
    fprintf(stderr, "vector_add failed: %s\n", kamd_hip_last_error());
    return 1;
  }
  if (err > 1e-5f) {
    fprintf(stderr, "Result verification failed (max err %g)\n", err);
    return 1;
  }
  printf("Test PASSED\nDone\n");
  if (hold_mib > 0) {
    void* buf = nullptr;
    size_t bytes = (size_t)hold_mib << 20;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMemset(buf, 1, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
      fprintf(stderr, "could not hold %ld MiB\n", hold_mib);
      return 1;
    }
    printf("HOLDING %ld MiB\n", hold_mib);
    fflush(stdout);
    sleep((unsigned)hold_s);
    hipFree(buf);
  }
  return 0;
}
