// kamd_smi — C ABI over AMD SMI for the amd.com/gpu device plugin, the kubelet's
// accelerator stats and the amd-smi Prometheus exporter.
//
// MI355X-native replacement for the reference's cgo NVML shim
// (vendor/github.com/mindprince/gonvml/bindings.go:20-245): libamd_smi.so is dlopen()ed at
// runtime (no link-time dependency, like gonvml's dlopen of libnvidia-ml.so.1 at :120), so
// one binary runs on GPU-less CI hosts. A second, fake backend serves a JSON fixture of a
// node (8 x MI355X, one xGMI hive) so every consumer is testable without a GPU — the role
// the reference's DevicePluginStub plays for the kubelet.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum kamd_backend_t { KAMD_BACKEND_NONE = 0, KAMD_BACKEND_AMDSMI = 1, KAMD_BACKEND_FAKE = 2 };

#define KAMD_STR 128
#define KAMD_MAX_LINKS 8

typedef struct {
  int32_t index;             // enumeration order (HIP/HSA id)
  char uuid[KAMD_STR];
  char bdf[32];              // dddd:bb:dd.f
  char market_name[KAMD_STR];
  char arch[32];             // gfx950
  uint32_t vendor_id;        // 0x1002
  uint64_t device_id;
  uint64_t vram_total_mb;
  uint32_t compute_units;
  int32_t render_minor;      // /dev/dri/renderD<minor>
  int32_t card_minor;        // /dev/dri/card<minor>
  int32_t hsa_id;
  int32_t hip_id;
  uint64_t xgmi_hive_id;
  uint64_t xgmi_node_id;
  int32_t numa_node;
  uint64_t kfd_id;
  int32_t partition_id;      // current compute partition index on the physical GPU
  char compute_partition[32];// SPX / DPX / QPX / CPX
  char serial[KAMD_STR];
  int32_t socket;            // physical package (OAM) index: compute partitions of one GPU share it
  char memory_partition[16]; // NPS1 / NPS2
} kamd_device_info_t;

typedef struct {
  int32_t type;      // 0 unknown, 1 PCIe, 2 xGMI (amdsmi_link_type_t)
  uint64_t hops;
  uint64_t weight;
  int32_t p2p;       // 1 if peer access works
} kamd_link_t;

typedef struct {
  uint32_t gfx_activity;      // %
  uint32_t umc_activity;      // %
  uint64_t vram_used_bytes;
  uint64_t vram_total_bytes;
  uint32_t power_w;
  uint32_t power_limit_w;
  int64_t temp_hotspot_c;
  int64_t temp_mem_c;
  uint64_t ecc_correctable;
  uint64_t ecc_uncorrectable;
  uint32_t xgmi_links_total;
  uint32_t xgmi_links_up;
  uint32_t sclk_mhz;
} kamd_metrics_t;

typedef struct {
  uint32_t pid;
  char name[KAMD_STR];
  uint64_t vram_bytes;
  uint64_t gfx_ns;
  uint32_t cu_occupancy;
} kamd_proc_t;

// init: fixture != NULL -> fake backend from that JSON file; otherwise try libamd_smi.so.
// Returns backend id (>0) or 0 on failure (see kamd_last_error()).
int kamd_init(const char* fixture_path);
int kamd_backend(void);
int kamd_device_count(void);
int kamd_device_info(int idx, kamd_device_info_t* out);
int kamd_link(int src, int dst, kamd_link_t* out);
int kamd_metrics(int idx, kamd_metrics_t* out);
int kamd_process_list(int idx, kamd_proc_t* out, int max_procs);
// Fake backend only: mutate health-relevant state (for device-plugin health tests).
int kamd_fake_set_ecc(int idx, uint64_t uncorrectable);
int kamd_fake_set_links_up(int idx, uint32_t up);
// type: 2 = xGMI, 1 = PCIe (a failed xGMI link between two packages of a hive)
int kamd_fake_set_link(int src, int dst, int type);
// replace the process list of a device (amdsmi_get_gpu_process_list of the fake backend)
int kamd_fake_set_procs(int idx, const kamd_proc_t* procs, int n);
const char* kamd_last_error(void);
void kamd_shutdown(void);

#ifdef __cplusplus
}
#endif
