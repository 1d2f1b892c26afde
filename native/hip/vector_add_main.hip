// hip-vector-add — GPU e2e test workload (the MI355X analog of cuda-samples vectorAdd used by
// the reference's test/images/cuda-vector-add image, test/e2e/scheduling/nvidia-gpus.go:51-113).
// Runs on the device(s) the runtime exposed to the container (HIP_VISIBLE_DEVICES /
// ROCR_VISIBLE_DEVICES set by the amd.com/gpu device plugin) and prints "Test PASSED".
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

extern "C" int kamd_diag_vector_add(int dev, int n, float* max_err);
extern "C" const char* kamd_hip_last_error();

int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 50000;
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
  return 0;
}
