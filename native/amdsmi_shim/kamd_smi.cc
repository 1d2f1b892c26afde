// kamd_smi implementation: a dlopen()ed AMD SMI backend and a JSON-fixture fake backend.
// See kamd_smi.h. Built as libkamd_smi.so (g++ -O2 -shared -fPIC); depends only on libdl.
#include "kamd_smi.h"

#include <dlfcn.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <fstream>
#include <map>
#include <memory>
#include <atomic>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include <amd_smi/amdsmi.h>

namespace {

std::mutex g_mu;
// errno-style: each thread sees the error of its own last call (kamd_last_error() is read
// without the lock, so a shared string would race with another thread's set_err)
thread_local std::string g_err;
std::atomic<int> g_backend{KAMD_BACKEND_NONE};   // read lock-free by kamd_backend()

void set_err(const std::string& s) { g_err = s; }

// ---------------------------------------------------------------------------
// minimal JSON (objects, arrays, strings, numbers, bools, null) for the fixture
struct JVal {
  enum T { NUL, BOOL, NUM, STR, ARR, OBJ } t = NUL;
  bool b = false;
  double n = 0;
  std::string s;
  std::vector<JVal> a;
  std::map<std::string, JVal> o;
  const JVal* get(const char* k) const {
    auto it = o.find(k);
    return it == o.end() ? nullptr : &it->second;
  }
  double num(const char* k, double d) const {
    const JVal* v = get(k);
    return (v && v->t == NUM) ? v->n : d;
  }
  std::string str(const char* k, const char* d) const {
    const JVal* v = get(k);
    return (v && v->t == STR) ? v->s : std::string(d);
  }
};

struct JParser {
  const char* p;
  const char* end;
  bool ok = true;
  void ws() { while (p < end && isspace((unsigned char)*p)) ++p; }
  bool lit(const char* w) {
    size_t n = strlen(w);
    if ((size_t)(end - p) >= n && strncmp(p, w, n) == 0) { p += n; return true; }
    return false;
  }
  std::string string() {
    std::string out;
    ++p;  // opening quote
    while (p < end && *p != '"') {
      if (*p == '\\' && p + 1 < end) {
        ++p;
        char c = *p;
        if (c == 'n') out += '\n'; else if (c == 't') out += '\t';
        else if (c == 'u' && end - p > 4) { out += '?'; p += 4; }
        else out += c;
        ++p;
      } else {
        out += *p++;
      }
    }
    if (p < end) ++p; else ok = false;
    return out;
  }
  JVal value() {
    JVal v;
    ws();
    if (p >= end) { ok = false; return v; }
    char c = *p;
    if (c == '{') {
      v.t = JVal::OBJ; ++p; ws();
      if (p < end && *p == '}') { ++p; return v; }
      while (ok && p < end) {
        ws();
        if (*p != '"') { ok = false; break; }
        std::string k = string();
        ws();
        if (p >= end || *p != ':') { ok = false; break; }
        ++p;
        v.o[k] = value();
        ws();
        if (p < end && *p == ',') { ++p; continue; }
        if (p < end && *p == '}') { ++p; break; }
        ok = false;
      }
    } else if (c == '[') {
      v.t = JVal::ARR; ++p; ws();
      if (p < end && *p == ']') { ++p; return v; }
      while (ok && p < end) {
        v.a.push_back(value());
        ws();
        if (p < end && *p == ',') { ++p; continue; }
        if (p < end && *p == ']') { ++p; break; }
        ok = false;
      }
    } else if (c == '"') {
      v.t = JVal::STR; v.s = string();
    } else if (lit("true")) { v.t = JVal::BOOL; v.b = true; }
    else if (lit("false")) { v.t = JVal::BOOL; }
    else if (lit("null")) { v.t = JVal::NUL; }
    else {
      char* e = nullptr;
      v.t = JVal::NUM; v.n = strtod(p, &e);
      if (e == p) ok = false;
      p = e;
    }
    return v;
  }
};

// ---------------------------------------------------------------------------
// backend interface
struct Backend {
  virtual ~Backend() {}
  virtual int count() = 0;
  virtual int info(int i, kamd_device_info_t* o) = 0;
  virtual int link(int s, int d, kamd_link_t* o) = 0;
  virtual int metrics(int i, kamd_metrics_t* o) = 0;
  virtual int procs(int i, kamd_proc_t* o, int max) = 0;
};

void copy_str(char* dst, size_t n, const std::string& s) {
  strncpy(dst, s.c_str(), n - 1);
  dst[n - 1] = 0;
}

// ---------------------------------------------------------------------------
struct FakeDev {
  kamd_device_info_t info;
  kamd_metrics_t m;
  std::vector<kamd_proc_t> procs;
};

struct FakeBackend : Backend {
  std::vector<FakeDev> devs;
  std::vector<std::vector<kamd_link_t>> links;

  bool load(const char* path) {
    std::ifstream f(path);
    if (!f) { set_err(std::string("cannot open fixture ") + path); return false; }
    std::stringstream ss; ss << f.rdbuf();
    std::string txt = ss.str();
    JParser jp{txt.data(), txt.data() + txt.size()};
    JVal root = jp.value();
    if (!jp.ok || root.t != JVal::OBJ) { set_err("fixture: malformed JSON"); return false; }
    const JVal* ds = root.get("devices");
    if (!ds || ds->t != JVal::ARR) { set_err("fixture: missing devices[]"); return false; }
    int idx = 0;
    for (const JVal& d : ds->a) {
      FakeDev fd;
      memset(&fd.info, 0, sizeof fd.info);
      memset(&fd.m, 0, sizeof fd.m);
      kamd_device_info_t& in = fd.info;
      in.index = idx;
      copy_str(in.uuid, sizeof in.uuid, d.str("uuid", ""));
      copy_str(in.bdf, sizeof in.bdf, d.str("bdf", ""));
      copy_str(in.market_name, sizeof in.market_name, d.str("market_name", "AMD Instinct MI355X"));
      copy_str(in.arch, sizeof in.arch, d.str("arch", "gfx950"));
      copy_str(in.compute_partition, sizeof in.compute_partition, d.str("partition", "SPX"));
      copy_str(in.serial, sizeof in.serial, d.str("serial", ""));
      in.vendor_id = (uint32_t)d.num("vendor_id", 0x1002);
      in.device_id = (uint64_t)d.num("device_id", 0x75a3);
      in.vram_total_mb = (uint64_t)d.num("vram_total_mb", 294912);
      in.compute_units = (uint32_t)d.num("compute_units", 256);
      in.render_minor = (int32_t)d.num("render_minor", 128 + idx);
      in.card_minor = (int32_t)d.num("card_minor", idx);
      in.hsa_id = (int32_t)d.num("hsa_id", idx);
      in.hip_id = (int32_t)d.num("hip_id", idx);
      in.xgmi_hive_id = (uint64_t)d.num("xgmi_hive_id", 0);
      in.xgmi_node_id = (uint64_t)d.num("xgmi_node_id", idx);
      in.numa_node = (int32_t)d.num("numa_node", idx / 4);
      in.kfd_id = (uint64_t)d.num("kfd_id", 1000 + idx);
      in.partition_id = (int32_t)d.num("partition_id", 0);
      in.socket = (int32_t)d.num("socket", idx);
      copy_str(in.memory_partition, sizeof in.memory_partition, d.str("memory_partition", "NPS1"));
      kamd_metrics_t& m = fd.m;
      m.gfx_activity = (uint32_t)d.num("gfx_activity", 0);
      m.umc_activity = (uint32_t)d.num("umc_activity", 0);
      m.vram_total_bytes = in.vram_total_mb << 20;
      m.vram_used_bytes = ((uint64_t)d.num("vram_used_mb", 0)) << 20;
      m.power_w = (uint32_t)d.num("power_w", 180);
      m.power_limit_w = (uint32_t)d.num("power_limit_w", 1400);
      m.temp_hotspot_c = (int64_t)d.num("temp_c", 38);
      m.temp_mem_c = (int64_t)d.num("temp_mem_c", 36);
      m.ecc_correctable = (uint64_t)d.num("ecc_correctable", 0);
      m.ecc_uncorrectable = (uint64_t)d.num("ecc_uncorrectable", 0);
      m.xgmi_links_total = (uint32_t)d.num("xgmi_links_total", 7);
      m.xgmi_links_up = (uint32_t)d.num("xgmi_links_up", 7);
      m.sclk_mhz = (uint32_t)d.num("sclk_mhz", 2400);
      devs.push_back(fd);
      ++idx;
    }
    int n = (int)devs.size();
    links.assign(n, std::vector<kamd_link_t>(n));
    // default topology: same hive id => xGMI, 1 hop (MI355X UBB: every GPU has a direct link
    // to each of the other 7); different hive => PCIe, 2 hops. Compute partitions of one
    // package (CPX/DPX/QPX) reach each other over the on-package fabric: 0 hops, weight 5.
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        kamd_link_t& l = links[i][j];
        if (i == j) { l.type = 0; l.hops = 0; l.weight = 0; l.p2p = 1; continue; }
        if (devs[i].info.socket == devs[j].info.socket) { l.type = 2; l.hops = 0; l.weight = 5; l.p2p = 1; continue; }
        bool same = devs[i].info.xgmi_hive_id != 0 && devs[i].info.xgmi_hive_id == devs[j].info.xgmi_hive_id;
        l.type = same ? 2 : 1;
        l.hops = same ? 1 : 2;
        l.weight = same ? 15 : 40;
        l.p2p = same ? 1 : 0;
      }
    // explicit overrides: "links": [[src, dst, type, hops, weight], ...]
    const JVal* ls = root.get("links");
    if (ls && ls->t == JVal::ARR) {
      for (const JVal& e : ls->a) {
        if (e.t != JVal::ARR || e.a.size() < 3) continue;
        int s = (int)e.a[0].n, d = (int)e.a[1].n;
        if (s < 0 || d < 0 || s >= n || d >= n) continue;
        links[s][d].type = (int32_t)e.a[2].n;
        if (e.a.size() > 3) links[s][d].hops = (uint64_t)e.a[3].n;
        if (e.a.size() > 4) links[s][d].weight = (uint64_t)e.a[4].n;
        links[s][d].p2p = links[s][d].type == 2;
      }
    }
    return true;
  }
  int count() override { return (int)devs.size(); }
  int info(int i, kamd_device_info_t* o) override { *o = devs[i].info; return 0; }
  int link(int s, int d, kamd_link_t* o) override { *o = links[s][d]; return 0; }
  int metrics(int i, kamd_metrics_t* o) override { *o = devs[i].m; return 0; }
  int procs(int i, kamd_proc_t* o, int max) override {
    int k = 0;
    for (const kamd_proc_t& p : devs[i].procs) {
      if (k >= max) break;
      o[k++] = p;
    }
    return k;
  }
};

// ---------------------------------------------------------------------------
// real backend: AMD SMI via dlopen
#define KAMD_FNS(X)                                                                              \
  X(amdsmi_init, amdsmi_status_t (*)(uint64_t))                                                  \
  X(amdsmi_shut_down, amdsmi_status_t (*)(void))                                                 \
  X(amdsmi_get_socket_handles, amdsmi_status_t (*)(uint32_t*, amdsmi_socket_handle*))            \
  X(amdsmi_get_processor_handles,                                                               \
    amdsmi_status_t (*)(amdsmi_socket_handle, uint32_t*, amdsmi_processor_handle*))              \
  X(amdsmi_get_processor_type, amdsmi_status_t (*)(amdsmi_processor_handle, processor_type_t*))  \
  X(amdsmi_get_gpu_device_uuid, amdsmi_status_t (*)(amdsmi_processor_handle, unsigned int*, char*)) \
  X(amdsmi_get_gpu_device_bdf, amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_bdf_t*))       \
  X(amdsmi_get_gpu_asic_info, amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_asic_info_t*))  \
  X(amdsmi_get_gpu_vram_info, amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_vram_info_t*))  \
  X(amdsmi_get_gpu_kfd_info, amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_kfd_info_t*))    \
  X(amdsmi_get_gpu_enumeration_info,                                                             \
    amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_enumeration_info_t*))                     \
  X(amdsmi_get_xgmi_info, amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_xgmi_info_t*))      \
  X(amdsmi_get_gpu_topo_numa_affinity, amdsmi_status_t (*)(amdsmi_processor_handle, int32_t*))   \
  X(amdsmi_topo_get_link_type, amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_processor_handle, \
                                                    uint64_t*, amdsmi_link_type_t*))               \
  X(amdsmi_topo_get_link_weight,                                                                 \
    amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_processor_handle, uint64_t*))            \
  X(amdsmi_is_P2P_accessible,                                                                    \
    amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_processor_handle, bool*))                \
  X(amdsmi_get_gpu_activity, amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_engine_usage_t*)) \
  X(amdsmi_get_gpu_memory_usage,                                                                 \
    amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_memory_type_t, uint64_t*))               \
  X(amdsmi_get_gpu_memory_total,                                                                 \
    amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_memory_type_t, uint64_t*))               \
  X(amdsmi_get_power_info, amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_power_info_t*))    \
  X(amdsmi_get_temp_metric, amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_temperature_type_t, \
                                                 amdsmi_temperature_metric_t, int64_t*))          \
  X(amdsmi_get_gpu_total_ecc_count,                                                              \
    amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_error_count_t*))                          \
  X(amdsmi_get_gpu_xgmi_link_status,                                                             \
    amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_xgmi_link_status_t*))                     \
  X(amdsmi_get_gpu_compute_partition, amdsmi_status_t (*)(amdsmi_processor_handle, char*, uint32_t)) \
  X(amdsmi_get_gpu_memory_partition, amdsmi_status_t (*)(amdsmi_processor_handle, char*, uint32_t)) \
  X(amdsmi_get_gpu_process_list,                                                                 \
    amdsmi_status_t (*)(amdsmi_processor_handle, uint32_t*, amdsmi_proc_info_t*))                \
  X(amdsmi_get_clock_info, amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_clk_type_t, amdsmi_clk_info_t*)) \
  X(amdsmi_status_code_to_string, amdsmi_status_t (*)(amdsmi_status_t, const char**))

struct SmiFns {
#define DECL(name, type) decltype(&::name) name = nullptr;
  KAMD_FNS(DECL)
#undef DECL
};

struct SmiBackend : Backend {
  void* lib = nullptr;
  SmiFns f;
  std::vector<amdsmi_processor_handle> gpus;
  std::vector<int32_t> socket_of;   // per entry of gpus: index of its amdsmi socket handle

  std::string code(amdsmi_status_t s) {
    const char* msg = nullptr;
    if (f.amdsmi_status_code_to_string && f.amdsmi_status_code_to_string(s, &msg) == AMDSMI_STATUS_SUCCESS && msg)
      return msg;
    return "amdsmi status " + std::to_string((int)s);
  }

  bool open() {
    const char* cands[] = {"libamd_smi.so", "libamd_smi.so.26", "/opt/rocm/lib/libamd_smi.so", nullptr};
    for (int i = 0; cands[i] && !lib; ++i) lib = dlopen(cands[i], RTLD_NOW | RTLD_LOCAL);
    if (!lib) { set_err(std::string("dlopen libamd_smi.so: ") + dlerror()); return false; }
#define LOAD(name, type) f.name = (decltype(&::name))dlsym(lib, #name);
    KAMD_FNS(LOAD)
#undef LOAD
    if (!f.amdsmi_init || !f.amdsmi_get_socket_handles || !f.amdsmi_get_processor_handles) {
      set_err("libamd_smi.so: missing core symbols");
      return false;
    }
    amdsmi_status_t s = f.amdsmi_init(AMDSMI_INIT_AMD_GPUS);
    if (s != AMDSMI_STATUS_SUCCESS) { set_err("amdsmi_init: " + code(s)); return false; }
    uint32_t ns = 0;
    if ((s = f.amdsmi_get_socket_handles(&ns, nullptr)) != AMDSMI_STATUS_SUCCESS) {
      set_err("amdsmi_get_socket_handles: " + code(s)); return false;
    }
    std::vector<amdsmi_socket_handle> socks(ns);
    f.amdsmi_get_socket_handles(&ns, socks.data());
    for (uint32_t i = 0; i < ns; ++i) {
      uint32_t np = 0;
      if (f.amdsmi_get_processor_handles(socks[i], &np, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
      std::vector<amdsmi_processor_handle> ph(np);
      f.amdsmi_get_processor_handles(socks[i], &np, ph.data());
      for (auto h : ph) {
        processor_type_t t;
        if (f.amdsmi_get_processor_type && f.amdsmi_get_processor_type(h, &t) == AMDSMI_STATUS_SUCCESS &&
            t != AMDSMI_PROCESSOR_TYPE_AMD_GPU)
          continue;
        gpus.push_back(h);
        socket_of.push_back((int32_t)i);
      }
    }
    // order by HIP enumeration id when available, so index == HIP device ordinal
    if (f.amdsmi_get_gpu_enumeration_info) {
      struct Ent { uint32_t k; amdsmi_processor_handle h; int32_t sock; };
      std::vector<Ent> ord;
      for (size_t i = 0; i < gpus.size(); ++i) {
        amdsmi_enumeration_info_t e;
        memset(&e, 0, sizeof e);
        uint32_t k = (uint32_t)i;
        if (f.amdsmi_get_gpu_enumeration_info(gpus[i], &e) == AMDSMI_STATUS_SUCCESS) k = e.hip_id;
        ord.push_back({k, gpus[i], socket_of[i]});
      }
      std::stable_sort(ord.begin(), ord.end(), [](const Ent& a, const Ent& b) { return a.k < b.k; });
      for (size_t i = 0; i < ord.size(); ++i) { gpus[i] = ord[i].h; socket_of[i] = ord[i].sock; }
    }
    return true;
  }

  ~SmiBackend() override {
    if (lib && f.amdsmi_shut_down) f.amdsmi_shut_down();
    // keep lib mapped: amdsmi registers atexit handlers
  }

  int count() override { return (int)gpus.size(); }

  int info(int i, kamd_device_info_t* o) override {
    memset(o, 0, sizeof *o);
    amdsmi_processor_handle h = gpus[i];
    o->index = i;
    o->numa_node = -1;
    o->render_minor = -1;
    o->card_minor = -1;
    o->partition_id = -1;
    o->socket = socket_of[i];
    unsigned int ul = sizeof o->uuid;
    if (f.amdsmi_get_gpu_device_uuid) f.amdsmi_get_gpu_device_uuid(h, &ul, o->uuid);
    amdsmi_bdf_t bdf;
    if (f.amdsmi_get_gpu_device_bdf && f.amdsmi_get_gpu_device_bdf(h, &bdf) == AMDSMI_STATUS_SUCCESS)
      snprintf(o->bdf, sizeof o->bdf, "%04llx:%02llx:%02llx.%llx", (unsigned long long)bdf.domain_number,
               (unsigned long long)bdf.bus_number, (unsigned long long)bdf.device_number,
               (unsigned long long)bdf.function_number);
    amdsmi_asic_info_t a;
    memset(&a, 0, sizeof a);
    if (f.amdsmi_get_gpu_asic_info && f.amdsmi_get_gpu_asic_info(h, &a) == AMDSMI_STATUS_SUCCESS) {
      copy_str(o->market_name, sizeof o->market_name, a.market_name);
      copy_str(o->serial, sizeof o->serial, a.asic_serial);
      o->vendor_id = a.vendor_id;
      o->device_id = a.device_id;
      if (a.num_of_compute_units != 0xFFFFFFFFu) o->compute_units = a.num_of_compute_units;
      uint64_t v = a.target_graphics_version;
      if (v != 0xFFFFFFFFFFFFFFFFull && v) {
        // AMD SMI encodes the gfx target as hex digits: 0x950 -> gfx950, 0x942 -> gfx942, 0x90a -> gfx90a
        snprintf(o->arch, sizeof o->arch, "gfx%llx", (unsigned long long)v);
      }
    }
    amdsmi_vram_info_t vi;
    memset(&vi, 0, sizeof vi);
    if (f.amdsmi_get_gpu_vram_info && f.amdsmi_get_gpu_vram_info(h, &vi) == AMDSMI_STATUS_SUCCESS)
      o->vram_total_mb = vi.vram_size;
    if (!o->vram_total_mb && f.amdsmi_get_gpu_memory_total) {
      uint64_t t = 0;
      if (f.amdsmi_get_gpu_memory_total(h, AMDSMI_MEM_TYPE_VRAM, &t) == AMDSMI_STATUS_SUCCESS) o->vram_total_mb = t >> 20;
    }
    amdsmi_enumeration_info_t e;
    memset(&e, 0, sizeof e);
    if (f.amdsmi_get_gpu_enumeration_info && f.amdsmi_get_gpu_enumeration_info(h, &e) == AMDSMI_STATUS_SUCCESS) {
      o->render_minor = (int32_t)e.drm_render;
      o->card_minor = (int32_t)e.drm_card;
      o->hsa_id = (int32_t)e.hsa_id;
      o->hip_id = (int32_t)e.hip_id;
    }
    amdsmi_kfd_info_t k;
    memset(&k, 0, sizeof k);
    if (f.amdsmi_get_gpu_kfd_info && f.amdsmi_get_gpu_kfd_info(h, &k) == AMDSMI_STATUS_SUCCESS) {
      o->kfd_id = k.kfd_id;
      if (k.current_partition_id != 0xFFFFFFFFu) o->partition_id = (int32_t)k.current_partition_id;
    }
    amdsmi_xgmi_info_t x;
    memset(&x, 0, sizeof x);
    if (f.amdsmi_get_xgmi_info && f.amdsmi_get_xgmi_info(h, &x) == AMDSMI_STATUS_SUCCESS) {
      o->xgmi_hive_id = x.xgmi_hive_id;
      o->xgmi_node_id = x.xgmi_node_id;
    }
    int32_t numa = -1;
    if (f.amdsmi_get_gpu_topo_numa_affinity && f.amdsmi_get_gpu_topo_numa_affinity(h, &numa) == AMDSMI_STATUS_SUCCESS)
      o->numa_node = numa;
    if (f.amdsmi_get_gpu_compute_partition)
      f.amdsmi_get_gpu_compute_partition(h, o->compute_partition, sizeof o->compute_partition);
    if (f.amdsmi_get_gpu_memory_partition)
      f.amdsmi_get_gpu_memory_partition(h, o->memory_partition, sizeof o->memory_partition);
    return 0;
  }

  int link(int s, int d, kamd_link_t* o) override {
    memset(o, 0, sizeof *o);
    if (s == d) { o->p2p = 1; return 0; }
    amdsmi_link_type_t t = AMDSMI_LINK_TYPE_UNKNOWN;
    uint64_t hops = 0, w = 0;
    if (f.amdsmi_topo_get_link_type && f.amdsmi_topo_get_link_type(gpus[s], gpus[d], &hops, &t) == AMDSMI_STATUS_SUCCESS) {
      o->type = t == AMDSMI_LINK_TYPE_XGMI ? 2 : (t == AMDSMI_LINK_TYPE_PCIE ? 1 : 0);
      o->hops = hops;
    }
    if (f.amdsmi_topo_get_link_weight && f.amdsmi_topo_get_link_weight(gpus[s], gpus[d], &w) == AMDSMI_STATUS_SUCCESS)
      o->weight = w;
    bool acc = false;
    if (f.amdsmi_is_P2P_accessible && f.amdsmi_is_P2P_accessible(gpus[s], gpus[d], &acc) == AMDSMI_STATUS_SUCCESS)
      o->p2p = acc ? 1 : 0;
    return 0;
  }

  int metrics(int i, kamd_metrics_t* o) override {
    memset(o, 0, sizeof *o);
    amdsmi_processor_handle h = gpus[i];
    amdsmi_engine_usage_t u;
    memset(&u, 0, sizeof u);
    if (f.amdsmi_get_gpu_activity && f.amdsmi_get_gpu_activity(h, &u) == AMDSMI_STATUS_SUCCESS) {
      o->gfx_activity = u.gfx_activity;
      o->umc_activity = u.umc_activity;
    }
    uint64_t v = 0;
    if (f.amdsmi_get_gpu_memory_usage && f.amdsmi_get_gpu_memory_usage(h, AMDSMI_MEM_TYPE_VRAM, &v) == AMDSMI_STATUS_SUCCESS)
      o->vram_used_bytes = v;
    if (f.amdsmi_get_gpu_memory_total && f.amdsmi_get_gpu_memory_total(h, AMDSMI_MEM_TYPE_VRAM, &v) == AMDSMI_STATUS_SUCCESS)
      o->vram_total_bytes = v;
    amdsmi_power_info_t p;
    memset(&p, 0, sizeof p);
    if (f.amdsmi_get_power_info && f.amdsmi_get_power_info(h, &p) == AMDSMI_STATUS_SUCCESS) {
      o->power_w = p.current_socket_power != 0xFFFFFFFFu ? p.current_socket_power : p.average_socket_power;
      // some drivers report the cap in microwatts
      o->power_limit_w = p.power_limit > 100000u ? p.power_limit / 1000000u : p.power_limit;
    }
    int64_t t = 0;
    if (f.amdsmi_get_temp_metric && f.amdsmi_get_temp_metric(h, AMDSMI_TEMPERATURE_TYPE_HOTSPOT, AMDSMI_TEMP_CURRENT, &t) == AMDSMI_STATUS_SUCCESS)
      o->temp_hotspot_c = t;
    if (f.amdsmi_get_temp_metric && f.amdsmi_get_temp_metric(h, AMDSMI_TEMPERATURE_TYPE_VRAM, AMDSMI_TEMP_CURRENT, &t) == AMDSMI_STATUS_SUCCESS)
      o->temp_mem_c = t;
    amdsmi_error_count_t ec;
    memset(&ec, 0, sizeof ec);
    if (f.amdsmi_get_gpu_total_ecc_count && f.amdsmi_get_gpu_total_ecc_count(h, &ec) == AMDSMI_STATUS_SUCCESS) {
      o->ecc_correctable = ec.correctable_count;
      o->ecc_uncorrectable = ec.uncorrectable_count;
    }
    amdsmi_xgmi_link_status_t ls;
    memset(&ls, 0, sizeof ls);
    if (f.amdsmi_get_gpu_xgmi_link_status && f.amdsmi_get_gpu_xgmi_link_status(h, &ls) == AMDSMI_STATUS_SUCCESS) {
      o->xgmi_links_total = ls.total_links;
      for (uint32_t k = 0; k < ls.total_links && k < AMDSMI_MAX_NUM_XGMI_LINKS; ++k)
        if (ls.status[k] == AMDSMI_XGMI_LINK_UP) o->xgmi_links_up++;
    }
    amdsmi_clk_info_t ci;
    memset(&ci, 0, sizeof ci);
    if (f.amdsmi_get_clock_info && f.amdsmi_get_clock_info(h, AMDSMI_CLK_TYPE_GFX, &ci) == AMDSMI_STATUS_SUCCESS)
      o->sclk_mhz = ci.clk;
    return 0;
  }

  int procs(int i, kamd_proc_t* out, int max) override {
    if (!f.amdsmi_get_gpu_process_list) return 0;
    uint32_t n = 0;
    if (f.amdsmi_get_gpu_process_list(gpus[i], &n, nullptr) != AMDSMI_STATUS_SUCCESS || n == 0) return 0;
    std::vector<amdsmi_proc_info_t> v(n);
    if (f.amdsmi_get_gpu_process_list(gpus[i], &n, v.data()) != AMDSMI_STATUS_SUCCESS) return 0;
    int k = 0;
    for (uint32_t j = 0; j < n && k < max; ++j, ++k) {
      out[k].pid = v[j].pid;
      copy_str(out[k].name, sizeof out[k].name, v[j].name);
      out[k].vram_bytes = v[j].memory_usage.vram_mem;
      out[k].gfx_ns = v[j].engine_usage.gfx;
      out[k].cu_occupancy = v[j].cu_occupancy;
    }
    return k;
  }
};

// The backend is deliberately NOT destroyed during static destruction: tearing AMD SMI down
// after the HIP runtime / other libraries have begun unloading crashes the process at exit.
// kamd_shutdown() is the explicit teardown.
struct BackendHolder {
  std::unique_ptr<Backend> p;
  ~BackendHolder() { (void)p.release(); }
};
BackendHolder g_hold;
#define g_b g_hold.p

}  // namespace

extern "C" {

int kamd_init(const char* fixture) {
  std::lock_guard<std::mutex> l(g_mu);
  g_b.reset();
  g_backend = KAMD_BACKEND_NONE;
  if (fixture && *fixture) {
    auto fb = std::make_unique<FakeBackend>();
    if (!fb->load(fixture)) return 0;
    g_b = std::move(fb);
    g_backend = KAMD_BACKEND_FAKE;
    return g_backend;
  }
  auto sb = std::make_unique<SmiBackend>();
  if (!sb->open()) return 0;
  g_b = std::move(sb);
  g_backend = KAMD_BACKEND_AMDSMI;
  return g_backend;
}

int kamd_backend(void) { return g_backend.load(); }

int kamd_device_count(void) {
  std::lock_guard<std::mutex> l(g_mu);
  return g_b ? g_b->count() : -1;
}

static bool valid(int i) { return g_b && i >= 0 && i < g_b->count(); }

int kamd_device_info(int idx, kamd_device_info_t* out) {
  std::lock_guard<std::mutex> l(g_mu);
  if (!valid(idx) || !out) { set_err("bad device index"); return -1; }
  return g_b->info(idx, out);
}

int kamd_link(int s, int d, kamd_link_t* out) {
  std::lock_guard<std::mutex> l(g_mu);
  if (!valid(s) || !valid(d) || !out) { set_err("bad device index"); return -1; }
  return g_b->link(s, d, out);
}

int kamd_metrics(int idx, kamd_metrics_t* out) {
  std::lock_guard<std::mutex> l(g_mu);
  if (!valid(idx) || !out) { set_err("bad device index"); return -1; }
  return g_b->metrics(idx, out);
}

int kamd_process_list(int idx, kamd_proc_t* out, int max) {
  std::lock_guard<std::mutex> l(g_mu);
  if (!valid(idx) || !out || max <= 0) return 0;
  return g_b->procs(idx, out, max);
}

int kamd_fake_set_ecc(int idx, uint64_t unc) {
  std::lock_guard<std::mutex> l(g_mu);
  if (g_backend != KAMD_BACKEND_FAKE || !valid(idx)) return -1;
  static_cast<FakeBackend*>(g_b.get())->devs[idx].m.ecc_uncorrectable = unc;
  return 0;
}

int kamd_fake_set_procs(int idx, const kamd_proc_t* procs, int n) {
  std::lock_guard<std::mutex> l(g_mu);
  if (g_backend != KAMD_BACKEND_FAKE || !valid(idx) || n < 0) return -1;
  auto& v = static_cast<FakeBackend*>(g_b.get())->devs[idx].procs;
  v.assign(procs, procs + n);
  return 0;
}

int kamd_fake_set_link(int s, int d, int type) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_b || g_backend != KAMD_BACKEND_FAKE) return -1;
  auto* fb = static_cast<FakeBackend*>(g_b.get());
  int n = (int)fb->devs.size();
  if (s < 0 || d < 0 || s >= n || d >= n) return -1;
  fb->links[s][d].type = type;
  fb->links[s][d].p2p = type == 2;
  return 0;
}

int kamd_fake_set_links_up(int idx, uint32_t up) {
  std::lock_guard<std::mutex> l(g_mu);
  if (g_backend != KAMD_BACKEND_FAKE || !valid(idx)) return -1;
  static_cast<FakeBackend*>(g_b.get())->devs[idx].m.xgmi_links_up = up;
  return 0;
}

const char* kamd_last_error(void) { return g_err.c_str(); }

void kamd_shutdown(void) {
  std::lock_guard<std::mutex> l(g_mu);
  g_b.reset();
  g_backend = KAMD_BACKEND_NONE;
}

}  // extern "C"
