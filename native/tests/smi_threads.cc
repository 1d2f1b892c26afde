// ThreadSanitizer stress of the AMD SMI shim (native/amdsmi_shim/kamd_smi.cc) on the fake
// backend: the device plugin's health loop, the exporter's scrape handler and the kubelet's
// stats provider all call into one process-wide shim from different threads. Built by
// `python -m kubernetes_amd.native.build --sanitize` with -fsanitize=thread; any report fails it.
//
//   smi_threads FIXTURE.json [threads] [iterations]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <thread>
#include <vector>

#include "../amdsmi_shim/kamd_smi.h"

int main(int argc, char** argv) {
  if (argc < 2) { fprintf(stderr, "usage: smi_threads FIXTURE [threads] [iters]\n"); return 2; }
  const char* fx = argv[1];
  const int nthreads = argc > 2 ? atoi(argv[2]) : 8;
  const int iters = argc > 3 ? atoi(argv[3]) : 2000;
  if (kamd_init(fx) != KAMD_BACKEND_FAKE) { fprintf(stderr, "init: %s\n", kamd_last_error()); return 2; }
  std::atomic<long> calls{0}, bad{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < nthreads; ++t) {
    ts.emplace_back([&, t] {
      for (int i = 0; i < iters; ++i) {
        int n = kamd_device_count();
        if (n <= 0) {   // a concurrent re-init is in progress: allowed to see 0 devices briefly
          (void)kamd_last_error();
          continue;
        }
        int d = (i + t) % n;
        kamd_device_info_t info;
        kamd_metrics_t met;
        kamd_link_t link;
        kamd_proc_t procs[4];
        switch ((i + t) % 6) {
          case 0: if (kamd_device_info(d, &info) == 0 && strncmp(info.arch, "gfx", 3) != 0) bad++; break;
          case 1: (void)kamd_metrics(d, &met); break;
          case 2: (void)kamd_link(d, (d + 1) % n, &link); break;
          case 3: (void)kamd_process_list(d, procs, 4); break;
          case 4: (void)kamd_fake_set_ecc(d, (uint64_t)i); (void)kamd_fake_set_links_up(d, 7); break;
          case 5:
            (void)kamd_backend();
            if (kamd_device_info(-1, &info) == 0) bad++;        // error path: per-thread message
            if (strstr(kamd_last_error(), "bad device index") == nullptr) bad++;
            if (t == 0 && i % 250 == 0) (void)kamd_init(fx);   // re-init while others read
            break;
        }
        calls++;
      }
    });
  }
  for (auto& th : ts) th.join();
  kamd_shutdown();
  if (bad) { fprintf(stderr, "%ld inconsistent results\n", bad.load()); return 1; }
  printf("smi_threads: %d threads x %d iterations, %ld calls: OK\n", nthreads, iters, calls.load());
  return 0;
}
