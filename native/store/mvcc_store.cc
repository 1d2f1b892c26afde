// kamd-etcd — native MVCC key-value store with etcd-v3 semantics, embeddable (C ABI, libkamd_store.so)
// and servable (kamd-etcd binary, unix/TCP socket, binary protocol, watch streams).
//
// What the API server needs from etcd (reference staging/src/k8s.io/apiserver/pkg/storage/etcd3/store.go:128-666):
// one cluster revision; per-key create/mod revision and version; multi-key transactions with
// compare-and-swap (GuaranteedUpdate, conditional delete, and here also the device-claim keys that
// make GPU double-assignment impossible across API server workers); ordered range with limit +
// start key; watch from a revision with a bounded history (compaction -> "compacted" error); WAL.
//
// Resource versions are injected by the store: a put op may name a token (random per API server
// worker, so user data cannot collide with it) whose occurrences in the value are replaced by the
// decimal commit revision, so a worker encodes an object ONCE without knowing the revision
// another worker may take concurrently.
//
// Protocol (little endian). Request frame:  u32 len | u32 id | u8 op | payload
//                           Response frame: u32 len | u32 id | u8 status | payload
//   TXN(1):   u16 ncmp {u8 kind(0 modrev==,1 exists,2 absent,3 value==) u32 klen key i64 arg u32 vlen val}
//             u16 nops {u8 kind(0 put,1 del,2 put+inject,3 del+tombstone) u32 klen key u32 vlen val
//                       [kinds 2,3: u32 tlen token]}
//             -> status 0: i64 rev | status 1 (compare failed): u16 idx of failed compare, kv of that key
//   GET(2):   u32 klen key -> status 0: kv | status 4 not found
//   RANGE(3): u32 plen prefix u32 limit u32 salen start_after -> i64 rev u8 more u32 n {kv}
//   WATCH(4): i64 from_rev u32 plen prefix [u16 nexcl {u32 len excluded_prefix}]
//             -> status 0 i64 rev, then EVENT frames (status 8) on the same id: u8 type(0 put,1 del) kv;
//             status 3 if from_rev is compacted. Keys under an excluded prefix are not sent; instead
//             the watch gets at most one PROGRESS frame (status 10: i64 rev) per event-loop pass, so
//             a client that waits for "my cache has seen revision R" still advances (API server
//             workers exclude the resources they read from the store instead of caching).
//   REV(5):   -> i64 rev
//   COMPACT(6): i64 rev
//   kv = i64 create_rev i64 mod_rev i64 version u32 klen key u32 vlen val
//   A kind-3 delete carries the "tombstone" (final object state) reported in the delete event
//   instead of the last stored value; it is not stored.
//
// Threads (server): ONE store thread owns the engine, the worker connections and their watches
// (epoll loop: read, commit, reply); `--fan-threads N` (1..4) fan-out threads own the Kubernetes
// watch streams handed over by API server workers (SCM_RIGHTS on `<socket>.watch`). Once per loop
// pass the store thread posts that pass's committed events (one shared immutable vector per txn)
// and any newly handed-over watch to each fan-out thread, in commit order, under one mutex +
// eventfd wake. KV values are immutable after commit; the only mutable field, the index-frame
// parse cache `KV::aux[slot]`, is written only by fan-out thread `slot`. kubemark/store_bench.py
// measures the capacity; tests/test_sanitizers.py runs the multi-worker suite on a TSan build.
#include <ctype.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <time.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <string_view>
#include <atomic>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#ifdef KAMD_STORE_SERVER
// protobuf-stored objects are transcoded to JSON for Kubernetes watch streams (schema-driven,
// shared with the API server's codec)
#include "../pbcodec/pb_codec.h"
static pbc::Schema* g_pb_schema = nullptr;
#endif

namespace kamd {

struct KV {
  int64_t create_rev = 0, mod_rev = 0, version = 0;
  std::string value;
  // server-side parse cache of the value's index frame, one slot per watch fan-out thread (each
  // thread only touches its own): a value is immutable, so its header is parsed once per thread —
  // as an event's new state and again as the next event's `prev`
  static constexpr int kAuxSlots = 4;
  mutable std::shared_ptr<void> aux[kAuxSlots];
};

struct Event {
  uint8_t type;  // 0 put, 1 delete
  int64_t rev;
  std::string key;
  std::shared_ptr<KV> kv;    // state after the event (for delete: last value, version 0)
  std::shared_ptr<KV> prev;  // state before the event (null for a create)
};

struct Cmp {
  uint8_t kind;
  std::string key;
  int64_t arg;
  std::string val;
};

struct Op {
  uint8_t kind;  // 0 put, 1 delete, 2 put with RV injection, 3 delete with tombstone + RV injection
  std::string key;
  std::string val;
  std::string token;  // kinds 2/3: every occurrence in val is replaced by the commit revision
};

static void inject(std::string* v, const std::string& token, const std::string& rs) {
  if (token.empty()) return;
  size_t pos = 0;
  while ((pos = v->find(token, pos)) != std::string::npos) {
    v->replace(pos, token.size(), rs);
    pos += rs.size();
  }
}

class Engine {
 public:
  explicit Engine(size_t history_cap = 200000) : cap_(history_cap) {}

  int64_t rev() const { return rev_; }
  int64_t compacted() const { return compact_rev_; }

  bool open_wal(const std::string& path) {
    replay(path);
    wal_ = fopen(path.c_str(), "ab");
    return wal_ != nullptr;
  }
  ~Engine() {
    if (wal_) fclose(wal_);
  }

  const KV* get(const std::string& k) const {
    auto it = data_.find(k);
    return it == data_.end() ? nullptr : it->second.get();
  }

  // returns -1 on success (rev in *rev_out), otherwise index of the failed compare
  int txn(const std::vector<Cmp>& cmps, const std::vector<Op>& ops, int64_t* rev_out, std::vector<Event>* evs) {
    for (size_t i = 0; i < cmps.size(); ++i) {
      const Cmp& c = cmps[i];
      const KV* kv = get(c.key);
      bool ok = false;
      switch (c.kind) {
        case 0: ok = kv ? kv->mod_rev == c.arg : c.arg == 0; break;
        case 1: ok = kv != nullptr; break;
        case 2: ok = kv == nullptr; break;
        case 3: ok = kv != nullptr && kv->value == c.val; break;
      }
      if (!ok) return (int)i;
    }
    int64_t r = rev_ + 1;
    std::string rs = std::to_string(r);
    size_t changes = 0;
    for (size_t oi = 0; oi < ops.size(); ++oi) {
      const Op& o = ops[oi];
      bool last = oi + 1 == ops.size();
      if (o.kind == 0 || o.kind == 2) {
        std::string v = o.val;
        inject(&v, o.token, rs);
        auto& slot = data_[o.key];
        std::shared_ptr<KV> before = slot;
        auto nk = std::make_shared<KV>();
        nk->mod_rev = r;
        nk->value = std::move(v);
        if (slot) {
          nk->create_rev = slot->create_rev;
          nk->version = slot->version + 1;
        } else {
          nk->create_rev = r;
          nk->version = 1;
        }
        slot = nk;
        record(Event{0, r, o.key, nk, before}, evs);
        log_wal(0, last, o.key, nk->value);
        ++changes;
      } else {
        auto it = data_.find(o.key);
        if (it == data_.end()) {
          if (last && changes) log_wal(1, true, o.key, "");  // keep the txn terminated in the WAL
          continue;
        }
        // field by field: `aux` belongs to the watch fan-out thread and is never read here
        auto dk = std::make_shared<KV>();
        dk->create_rev = it->second->create_rev;
        dk->mod_rev = r;
        dk->version = 0;
        if (o.kind == 3) {  // tombstone: final object state reported to watchers, not stored
          dk->value = o.val;
          inject(&dk->value, o.token, rs);
        } else {
          dk->value = it->second->value;
        }
        std::shared_ptr<KV> before = it->second;
        data_.erase(it);
        record(Event{1, r, o.key, dk, before}, evs);
        log_wal(1, last, o.key, "");
        ++changes;
      }
    }
    if (changes) {
      rev_ = r;
      if (wal_) fflush(wal_);
    }
    *rev_out = rev_;
    return -1;
  }

  // range over keys with prefix, optionally strictly after start_after
  int64_t range(const std::string& prefix, uint32_t limit, const std::string& start_after,
                std::vector<std::pair<const std::string*, const KV*>>* out, bool* more) const {
    auto it = start_after.empty() ? data_.lower_bound(prefix) : data_.upper_bound(start_after);
    *more = false;
    for (; it != data_.end(); ++it) {
      if (it->first.compare(0, prefix.size(), prefix) != 0) break;
      if (limit && out->size() >= limit) {
        *more = true;
        break;
      }
      out->push_back({&it->first, it->second.get()});
    }
    return rev_;
  }

  // the keys with `prefix` as they were at revision `at` (etcd Range with `revision`): the current
  // state with every later event undone, newest first — each event keeps the state before it.
  // False when `at` is older than the retained history (compacted).
  bool range_at(const std::string& prefix, int64_t at, uint32_t limit, const std::string& start_after,
                std::vector<std::pair<std::string, std::shared_ptr<KV>>>* out, bool* more) const {
    if (at < compact_rev_) return false;
    std::map<std::string, std::shared_ptr<KV>> st;
    for (auto it = data_.lower_bound(prefix); it != data_.end(); ++it) {
      if (it->first.compare(0, prefix.size(), prefix) != 0) break;
      st.emplace(it->first, it->second);
    }
    for (size_t i = hist_.size(); i-- > 0 && hist_[i].rev > at;) {
      const Event& e = hist_[i];
      if (e.key.compare(0, prefix.size(), prefix) != 0) continue;
      if (e.prev) st[e.key] = e.prev;
      else st.erase(e.key);
    }
    *more = false;
    auto it = start_after.empty() ? st.lower_bound(prefix) : st.upper_bound(start_after);
    for (; it != st.end(); ++it) {
      if (limit && out->size() >= limit) {
        *more = true;
        break;
      }
      out->push_back(*it);
    }
    return true;
  }

  // events with rev > from; false if compacted
  bool since(int64_t from, const std::string& prefix, std::vector<const Event*>* out) const {
    if (from < compact_rev_) return false;
    size_t lo = 0, hi = hist_.size();
    while (lo < hi) {
      size_t mid = (lo + hi) / 2;
      if (hist_[mid].rev <= from) lo = mid + 1; else hi = mid;
    }
    for (size_t i = lo; i < hist_.size(); ++i)
      if (hist_[i].key.compare(0, prefix.size(), prefix) == 0) out->push_back(&hist_[i]);
    return true;
  }

  void compact(int64_t r) {
    while (!hist_.empty() && hist_.front().rev <= r) hist_.pop_front();
    if (r > compact_rev_) compact_rev_ = r;
  }

  size_t size() const { return data_.size(); }

  template <typename F>
  void for_prefix(const std::string& prefix, F f) const {
    for (auto it = data_.lower_bound(prefix); it != data_.end(); ++it) {
      if (it->first.compare(0, prefix.size(), prefix) != 0) break;
      f(it->first, it->second);
    }
  }

 private:
  void record(Event&& e, std::vector<Event>* evs) {
    if (evs) evs->push_back(e);
    hist_.push_back(std::move(e));
    if (hist_.size() > cap_) {
      compact_rev_ = hist_.front().rev;
      hist_.pop_front();
    }
  }
  // WAL record: u8 op | u8 last-op-of-txn | u32 klen | u32 vlen | key | value. Replay regroups
  // records into their transactions so revisions survive a restart exactly; a torn tail (partial
  // record or unterminated transaction) is dropped.
  void log_wal(uint8_t op, bool last, const std::string& k, const std::string& v) {
    if (!wal_) return;
    uint32_t kl = (uint32_t)k.size(), vl = (uint32_t)v.size();
    uint8_t end = last ? 1 : 0;
    fwrite(&op, 1, 1, wal_);
    fwrite(&end, 1, 1, wal_);
    fwrite(&kl, 4, 1, wal_);
    fwrite(&vl, 4, 1, wal_);
    fwrite(k.data(), 1, kl, wal_);
    fwrite(v.data(), 1, vl, wal_);
  }
  void replay(const std::string& path) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return;
    std::vector<Op> ops;
    for (;;) {
      uint8_t op, end;
      uint32_t kl, vl;
      if (fread(&op, 1, 1, f) != 1 || fread(&end, 1, 1, f) != 1 || fread(&kl, 4, 1, f) != 1 ||
          fread(&vl, 4, 1, f) != 1)
        break;
      std::string k(kl, '\0'), v(vl, '\0');
      if ((kl && fread(&k[0], 1, kl, f) != kl) || (vl && fread(&v[0], 1, vl, f) != vl)) break;  // torn tail
      ops.push_back(Op{op, k, v, ""});
      if (end) {
        int64_t r;
        FILE* save = wal_;
        wal_ = nullptr;
        txn({}, ops, &r, nullptr);
        wal_ = save;
        ops.clear();
      }
    }
    fclose(f);
  }

  std::map<std::string, std::shared_ptr<KV>> data_;
  std::deque<Event> hist_;
  size_t cap_;
  int64_t rev_ = 1;  // etcd starts at 1
  int64_t compact_rev_ = 0;
  FILE* wal_ = nullptr;
};

// ---------------------------------------------------------------------------
// wire helpers
// largest request frame a client may send (values are bounded far below this, like etcd's
// 1.5 MiB request limit; a txn carries a handful of them)
static constexpr uint32_t kMaxFrame = 256u << 20;

struct Reader {
  const char* p;
  const char* e;
  bool ok = true;
  template <typename T>
  T get() {
    T v{};
    if (e - p < (long)sizeof(T)) { ok = false; return v; }
    memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  std::string str() {
    uint32_t n = get<uint32_t>();
    if (!ok || e - p < (long)n) { ok = false; return {}; }
    std::string s(p, n);
    p += n;
    return s;
  }
};

struct Writer {
  std::string b;
  template <typename T>
  void put(T v) { b.append(reinterpret_cast<const char*>(&v), sizeof(T)); }
  void str(const std::string& s) { put<uint32_t>((uint32_t)s.size()); b.append(s); }
  void kv(const std::string& k, const KV& v) {
    put<int64_t>(v.create_rev);
    put<int64_t>(v.mod_rev);
    put<int64_t>(v.version);
    str(k);
    str(v.value);
  }
};

bool parse_txn(Reader& r, std::vector<Cmp>* cmps, std::vector<Op>* ops) {
  uint16_t nc = r.get<uint16_t>();
  for (uint16_t i = 0; i < nc && r.ok; ++i) {
    Cmp c;
    c.kind = r.get<uint8_t>();
    c.key = r.str();
    c.arg = r.get<int64_t>();
    c.val = r.str();
    if (c.kind > 3) return false;
    cmps->push_back(std::move(c));
  }
  uint16_t no = r.get<uint16_t>();
  for (uint16_t i = 0; i < no && r.ok; ++i) {
    Op o;
    o.kind = r.get<uint8_t>();
    o.key = r.str();
    o.val = r.str();
    if (o.kind >= 2) o.token = r.str();
    if (o.kind > 3) return false;
    ops->push_back(std::move(o));
  }
  return r.ok;
}

}  // namespace kamd

// ===========================================================================
// C ABI (libkamd_store.so): synchronous engine for in-process use and differential tests.
extern "C" {
struct kamd_store {
  kamd::Engine eng;
  std::string out;  // last result buffer
  explicit kamd_store(size_t cap) : eng(cap) {}
};

kamd_store* kamd_store_open(const char* wal_path, uint64_t history_cap) {
  auto* s = new kamd_store(history_cap ? history_cap : 200000);
  if (wal_path && *wal_path && !s->eng.open_wal(wal_path)) {
    delete s;
    return nullptr;
  }
  return s;
}
void kamd_store_close(kamd_store* s) { delete s; }
int64_t kamd_store_rev(kamd_store* s) { return s->eng.rev(); }
int64_t kamd_store_compacted(kamd_store* s) { return s->eng.compacted(); }
uint64_t kamd_store_size(kamd_store* s) { return s->eng.size(); }

// txn request encoded exactly like the TXN wire payload; returns -1 ok (rev in *rev) or the failed index
int kamd_store_txn(kamd_store* s, const char* req, uint32_t len, int64_t* rev) {
  kamd::Reader r{req, req + len};
  std::vector<kamd::Cmp> cmps;
  std::vector<kamd::Op> ops;
  if (!kamd::parse_txn(r, &cmps, &ops)) return -2;
  return s->eng.txn(cmps, ops, rev, nullptr);
}

// results are written into an internal buffer: *out / *out_len valid until the next call
int kamd_store_get(kamd_store* s, const char* key, uint32_t klen, const char** out, uint32_t* out_len) {
  const kamd::KV* kv = s->eng.get(std::string(key, klen));
  if (!kv) return 0;
  kamd::Writer w;
  w.kv(std::string(key, klen), *kv);
  s->out.swap(w.b);
  *out = s->out.data();
  *out_len = (uint32_t)s->out.size();
  return 1;
}

int kamd_store_range(kamd_store* s, const char* prefix, uint32_t plen, uint32_t limit, const char* start, uint32_t slen,
                     const char** out, uint32_t* out_len) {
  std::vector<std::pair<const std::string*, const kamd::KV*>> res;
  bool more = false;
  int64_t rev = s->eng.range(std::string(prefix, plen), limit, std::string(start ? start : "", slen), &res, &more);
  kamd::Writer w;
  w.put<int64_t>(rev);
  w.put<uint8_t>(more ? 1 : 0);
  w.put<uint32_t>((uint32_t)res.size());
  for (auto& kv : res) w.kv(*kv.first, *kv.second);
  s->out.swap(w.b);
  *out = s->out.data();
  *out_len = (uint32_t)s->out.size();
  return (int)res.size();
}

int kamd_store_since(kamd_store* s, int64_t from, const char* prefix, uint32_t plen, const char** out, uint32_t* out_len) {
  std::vector<const kamd::Event*> evs;
  if (!s->eng.since(from, std::string(prefix, plen), &evs)) return -1;
  kamd::Writer w;
  w.put<uint32_t>((uint32_t)evs.size());
  for (auto* e : evs) {
    w.put<uint8_t>(e->type);
    w.kv(e->key, *e->kv);
  }
  s->out.swap(w.b);
  *out = s->out.data();
  *out_len = (uint32_t)s->out.size();
  return (int)evs.size();
}

void kamd_store_compact(kamd_store* s, int64_t rev) { s->eng.compact(rev); }
}  // extern "C"

// ===========================================================================
// server (kamd-etcd)
#ifdef KAMD_STORE_SERVER
namespace kamd {

// KAMD_ETCD_PROFILE=1: time spent per activity, printed to stderr at shutdown (where the
// store's CPU goes under a given API load; there is no perf on the GPU boxes).
struct Prof {
  bool on = false;
  const char* names[12] = {"read+parse", "txn", "get", "range", "watch", "dispatch(workers)", "fan_dispatch",
                           "flush(conns)", "flush(fan)", "progress", "handoff", "fan writes (#)"};
  double ns[12] = {0};
  uint64_t n[12] = {0};
  static double now() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e9 + ts.tv_nsec;
  }
  void add(int k, double t0) { ns[k] += now() - t0; ++n[k]; }
  void print() const {
    if (!on) return;
    double tot = 0;
    for (double v : ns) tot += v;
    fprintf(stderr, "kamd-etcd profile (ms total / count / us avg):\n");
    for (int k = 0; k < 12; ++k)
      if (n[k]) fprintf(stderr, "  %-18s %10.1f ms %10llu %8.2f us  %5.1f%%\n", names[k], ns[k] / 1e6,
                        (unsigned long long)n[k], ns[k] / 1e3 / n[k], tot ? 100 * ns[k] / tot : 0);
  }
};
static Prof g_prof;
#define KPROF_BEGIN double _kp0 = g_prof.on ? Prof::now() : 0
#define KPROF_END(k) do { if (g_prof.on) g_prof.add((k), _kp0); } while (0)

struct Conn {
  int fd;
  std::string in, out;
  bool want_write = false;
  bool pollout = false;   // EPOLLOUT currently registered (MOD only on a change: one syscall less per flush)
};

struct Watch {
  Conn* conn;
  uint32_t id;
  std::string prefix;
  std::vector<std::string> excl;
  int64_t progress = 0;  // latest excluded revision not yet reported

  bool excluded(const std::string& key) const {
    for (const std::string& x : excl)
      if (key.compare(0, x.size(), x) == 0) return true;
    return false;
  }
};


// ---------------------------------------------------------------------------
// Watch fan-out: Kubernetes watch streams served by the store itself.
//
// An API server worker that accepted `GET /api/v1/pods?watch=1` (and authorized it) hands the
// client's socket to this process over the handoff listener (SCM_RIGHTS) together with the
// watch spec: key prefix, start revision or "send the initial state", timeout and the label /
// field requirements. From then on this single epoll loop writes the HTTP chunked watch stream
// (`{"type":"ADDED","object":{...}}` lines, the reference's cacher.go watch format) straight
// from committed transactions, so the per-event fan-out to hundreds of kubelets, scheduler
// shards and informers costs a header parse and a memcpy per matching watcher here instead of
// Python work in every API server worker (reference: staging/.../apiserver/pkg/storage/cacher.go
// dispatchEvent + indexed watchers). Values must carry the shared-store index frame
// (00 'K' 'H' | u32 len | JSON [fields, labels] | object JSON).
// Field/label maps of a value's index frame as views into the value (decoded copies only for
// strings with JSON escapes, kept in `owned`): no allocation per key in the common case.
typedef std::vector<std::pair<std::string_view, std::string_view>> SVMap;

static const std::string_view* sv_find(const SVMap& m, std::string_view k) {
  for (const auto& kv : m)
    if (kv.first == k) return &kv.second;
  return nullptr;
}

struct Index {
  bool ok = false;
  SVMap fields, labels;
  std::deque<std::string> owned;
  size_t body = 0;  // offset of the object (JSON, or a k8s\0 protobuf envelope) in the value
  // protobuf values: the object's JSON for resourceVersion `json_rv` (transcoded once per
  // fan-out thread and revision; the thread owning this Index is the only one touching it)
  mutable std::string json;
  mutable int64_t json_rv = -1;
  // protobuf watchers: the stored envelope with metadata.resourceVersion = pb_rv
  mutable std::string pbenv;
  mutable int64_t pb_rv = -1;
};

struct JsonCursor {
  const char* p;
  const char* e;
  Index* ix;
  bool ok = true;
  void ws() { while (p < e && (*p == ' ' || *p == '\n' || *p == '\t' || *p == '\r')) ++p; }
  bool eat(char c) { ws(); if (p < e && *p == c) { ++p; return true; } return false; }
  static void utf8(std::string* o, unsigned cp) {
    if (cp < 0x80) o->push_back((char)cp);
    else if (cp < 0x800) { o->push_back((char)(0xC0 | (cp >> 6))); o->push_back((char)(0x80 | (cp & 0x3F))); }
    else { o->push_back((char)(0xE0 | (cp >> 12))); o->push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
           o->push_back((char)(0x80 | (cp & 0x3F))); }
  }
  bool str(std::string_view* out) {
    ws();
    if (p >= e || *p != '"') return ok = false;
    const char* s0 = ++p;
    while (p < e && *p != '"' && *p != '\\') ++p;
    if (p < e && *p == '"') {           // no escapes: a view into the value
      *out = std::string_view(s0, (size_t)(p - s0));
      ++p;
      return true;
    }
    std::string o(s0, (size_t)(p - s0));
    while (p < e && *p != '"') {
      if (*p == '\\') {
        if (++p >= e) return ok = false;
        char c = *p++;
        switch (c) {
          case 'n': o.push_back('\n'); break;
          case 't': o.push_back('\t'); break;
          case 'r': o.push_back('\r'); break;
          case 'b': o.push_back('\b'); break;
          case 'f': o.push_back('\f'); break;
          case 'u': {
            if (e - p < 4) return ok = false;
            unsigned cp = (unsigned)strtoul(std::string(p, 4).c_str(), nullptr, 16);
            p += 4;
            utf8(&o, cp);
            break;
          }
          default: o.push_back(c);
        }
      } else {
        o.push_back(*p++);
      }
    }
    if (p >= e) return ok = false;
    ++p;
    ix->owned.push_back(std::move(o));
    *out = ix->owned.back();
    return true;
  }
  // {"k":"v",...} with string values (anything else fails the parse)
  bool obj(SVMap* m) {
    if (!eat('{')) return ok = false;
    if (eat('}')) return true;
    do {
      std::string_view k, v;
      if (!str(&k) || !eat(':') || !str(&v)) return ok = false;
      bool dup = false;
      for (auto& kv : *m)
        if (kv.first == k) { kv.second = v; dup = true; break; }
      if (!dup) m->emplace_back(k, v);
    } while (eat(','));
    return eat('}') || (ok = false);
  }
};

static void parse_index_into(const std::string& v, Index* ix) {
  if (v.size() < 7 || v[0] != '\0' || v[1] != 'K' || v[2] != 'H') return;
  uint32_t hl;
  memcpy(&hl, v.data() + 3, 4);
  if (7 + (size_t)hl > v.size()) return;
  JsonCursor c{v.data() + 7, v.data() + 7 + hl, ix};
  ix->fields.reserve(8);
  if (!c.eat('[') || !c.obj(&ix->fields) || !c.eat(',') || !c.obj(&ix->labels) || !c.eat(']')) {
    ix->fields.clear();
    ix->labels.clear();
    return;
  }
  ix->body = 7 + hl;
  ix->ok = true;
}

// the parsed index frame of a stored value, cached on the KV in the calling fan-out thread's slot
static const Index& index_of(const KV& kv, int slot) {
  std::shared_ptr<void>& a = kv.aux[slot];
  if (!a) {
    auto ix = std::make_shared<Index>();
    parse_index_into(kv.value, ix.get());
    a = ix;
  }
  return *static_cast<const Index*>(a.get());
}

static const Index& empty_index() {
  static const Index e;
  return e;
}

struct Crc32Table {
  uint32_t t[256];
  Crc32Table() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      t[i] = c;
    }
  }
};

static uint32_t crc32_ieee(std::string_view s) {   // zlib.crc32
  static const Crc32Table tab;   // thread-safe one-time init (several fan-out threads call this)
  const uint32_t* table = tab.t;
  uint32_t c = 0xFFFFFFFFu;
  for (unsigned char ch : s) c = table[(c ^ ch) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

// scheduler-shard selection (kubernetes_amd/api/sharding.py): (crc32("ns/name") + offset label) % n == i
static bool shard_match(const Index& ix, const std::string& offset_label, int64_t n, int64_t i) {
  if (n < 1) return false;
  const std::string_view* ns = sv_find(ix.fields, "metadata.namespace");
  const std::string_view* nm = sv_find(ix.fields, "metadata.name");
  std::string key;
  key.reserve(64);
  if (ns) key.append(ns->data(), ns->size());
  key.push_back('/');
  if (nm) key.append(nm->data(), nm->size());
  int64_t off = 0;
  const std::string_view* ol = sv_find(ix.labels, offset_label);
  if (ol && !ol->empty()) {
    std::string lv(ol->data(), ol->size());
    const char* b = lv.c_str();
    char* e = nullptr;
    errno = 0;
    long long v = strtoll(b, &e, 10);
    bool ok = errno == 0 && e && *e == 0 && !isspace((unsigned char)b[0]) && v >= -(1LL << 31) && v <= (1LL << 31);
    off = ok ? v : 0;
  }
  int64_t h = ((int64_t)crc32_ieee(key) + off) % n;
  if (h < 0) h += n;
  return h == i;
}

struct Requirement {
  uint8_t target;  // 0 label, 1 field
  uint8_t op;      // 0 =, 1 !=, 2 in, 3 notin, 4 exists, 5 !exists, 6 shard (key = offset label, vals = [n, i])
  std::string key;
  std::vector<std::string> vals;
  bool matches(const Index& ix) const {
    if (op == 6)
      return vals.size() == 2 && shard_match(ix, key, atoll(vals[0].c_str()), atoll(vals[1].c_str()));
    const std::string_view* it = sv_find(target == 0 ? ix.labels : ix.fields, key);
    // a field that is absent reads as "" (fields.Set semantics); labels keep presence
    bool has = it != nullptr || target == 1;
    std::string_view v = it ? *it : std::string_view();
    auto in = [&]() {
      for (const std::string& x : vals)
        if (v == x) return true;
      return false;
    };
    switch (op) {
      case 0: case 2: return has && in();
      case 1: case 3: return !has || !in();
      case 4: return it != nullptr;
      case 5: return it == nullptr;
    }
    return false;
  }
};

struct FanWatch {
  int fd = -1;
  bool pb = false;        // protobuf watch frames instead of JSON lines
  std::string prefix;
  int64_t min_rev = 0;
  std::vector<Requirement> reqs;
  std::string out;
  bool dead = false;
  bool queued = false;    // in fan_dirty_
  bool node_indexed = false;
  std::string node_key;   // spec.nodeName=X requirement: the watch lives in fan_by_node_[X]
  double deadline = 0;  // CLOCK_MONOTONIC seconds, 0 = none
  bool pollout = false;
  // set by the store thread at handoff, consumed by the fan-out thread when it adopts the watch
  bool send_initial = false;
  std::vector<std::shared_ptr<KV>> initial;   // snapshot of the prefix (list + watch)
  std::vector<Event> replay;                   // events after the requested resourceVersion
  bool matches(const Index& ix) const {
    if (!ix.ok) return false;
    for (const auto& r : reqs)
      if (!r.matches(ix)) return false;
    return true;
  }
};

static double mono_now() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

// the object JSON of a stored value: the bytes after the index frame, or — for a protobuf
// (k8s\0) value — its JSON transcoding with metadata.resourceVersion = rv, cached on the Index
static std::string_view object_json(const std::string& v, const Index& ix, int64_t rv) {
  size_t body = ix.body;
#ifdef KAMD_STORE_SERVER
  if (g_pb_schema && v.size() >= body + 4 && memcmp(v.data() + body, "k8s\0", 4) == 0) {
    if (ix.json_rv != rv) {
      ix.json.clear();
      char rs[24];
      snprintf(rs, sizeof rs, "%lld", (long long)rv);
      pbc::JsonWriter w(*g_pb_schema);
      if (!w.object((const uint8_t*)v.data() + body, v.size() - body, ix.json, rs)) ix.json = "{}";
      ix.json_rv = rv;
    }
    return ix.json;
  }
#endif
  (void)rv;
  return std::string_view(v).substr(body);
}

// the embedded object of a protobuf watch frame: the envelope with its resourceVersion (cached
// on the Index like the JSON form), or the stored JSON for values that are not protobuf
static std::string_view object_pb(const std::string& v, const Index& ix, int64_t rv) {
  size_t body = ix.body;
#ifdef KAMD_STORE_SERVER
  if (g_pb_schema && v.size() >= body + 4 && memcmp(v.data() + body, "k8s\0", 4) == 0) {
    if (ix.pb_rv != rv) {
      ix.pbenv.clear();
      char rs[24];
      snprintf(rs, sizeof rs, "%lld", (long long)rv);
      if (!pbc::envelope_with_rv(*g_pb_schema, (const uint8_t*)v.data() + body, v.size() - body, rs, ix.pbenv))
        ix.pbenv.assign(v.data() + body, v.size() - body);
      ix.pb_rv = rv;
    }
    return ix.pbenv;
  }
#endif
  (void)rv;
  return std::string_view(v).substr(body);
}

static void chunk_pb(std::string* out, const char* type, std::string_view obj) {
  std::string fr;
#ifdef KAMD_STORE_SERVER
  pbc::watch_event_frame(fr, type, obj.data(), obj.size());
#endif
  char hex[24];
  int hl = snprintf(hex, sizeof hex, "%zx\r\n", fr.size());
  out->append(hex, (size_t)hl);
  out->append(fr);
  out->append("\r\n", 2);
}

// metav1.Status{status: Failure, message, reason, code} in a `k8s\0` envelope (TypeMeta v1/Status;
// field numbers of k8s.io.apimachinery.pkg.apis.meta.v1.Status and runtime.Unknown)
static std::string status_envelope(const char* message, const char* reason, int code) {
  std::string st;
#ifdef KAMD_STORE_SERVER
  pbc::pb_put_ld(st, 1, "", 0);                              // metadata: ListMeta{}
  pbc::pb_put_ld(st, 2, "Failure", 7);
  pbc::pb_put_ld(st, 3, message, strlen(message));
  pbc::pb_put_ld(st, 4, reason, strlen(reason));
  pbc::pb_put_varint(st, (6u << 3) | 0);
  pbc::pb_put_varint(st, (uint64_t)code);
  std::string tm, env("k8s\0", 4);
  pbc::pb_put_ld(tm, 1, "v1", 2);
  pbc::pb_put_ld(tm, 2, "Status", 6);
  pbc::pb_put_ld(env, 1, tm.data(), tm.size());
  pbc::pb_put_ld(env, 2, st.data(), st.size());
  pbc::pb_put_ld(env, 3, "", 0);
  pbc::pb_put_ld(env, 4, "", 0);
  return env;
#else
  (void)message; (void)reason; (void)code;
  return st;
#endif
}

// one event of watch w (JSON line or protobuf frame)
static void emit(FanWatch* w, const char* type, const std::string& v, const Index& ix, int64_t rv);

static void chunk(std::string* out, const char* type, std::string_view obj) {
  // {"type":"X","object":<object JSON>}\n as one HTTP chunk
  static const char pre[] = "{\"type\":\"";
  static const char mid[] = "\",\"object\":";
  size_t n = (sizeof pre - 1) + strlen(type) + (sizeof mid - 1) + obj.size() + 2;
  char hex[24];
  int hl = snprintf(hex, sizeof hex, "%zx\r\n", n);
  out->append(hex, (size_t)hl);
  out->append(pre, sizeof pre - 1);
  out->append(type);
  out->append(mid, sizeof mid - 1);
  out->append(obj.data(), obj.size());
  out->append("}\n\r\n", 4);
}

static void emit(FanWatch* w, const char* type, const std::string& v, const Index& ix, int64_t rv) {
  if (w->pb) chunk_pb(&w->out, type, object_pb(v, ix, rv));
  else chunk(&w->out, type, object_json(v, ix, rv));
}

// Watch fan-out thread. Kubernetes watch streams handed over by the API server workers are
// served here, off the store thread: the store thread commits transactions and answers
// workers, then posts each loop pass's events (one lock per pass) and any newly handed-over
// watch, in commit order; this thread matches them against the watches' selectors (index
// parse cached on the value), formats the chunks and writes the sockets. Ordering: a watch is
// adopted after every event that precedes its snapshot / replay and before every later one, so
// nothing is lost or sent twice. The store thread never touches KV::aux (the parse cache).
class FanOut {
 public:
  explicit FanOut(int slot = 0) : slot_(slot) {}
  ~FanOut() { stop(); }
  int watches() const { return watches_.load(std::memory_order_acquire); }

  void start() {
    ep_ = epoll_create1(EPOLL_CLOEXEC);
    evfd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    epoll_event e{};
    e.events = EPOLLIN;
    e.data.fd = evfd_;
    epoll_ctl(ep_, EPOLL_CTL_ADD, evfd_, &e);
    th_ = std::thread([this] { loop(); });
  }

  void stop() {
    if (!th_.joinable()) return;
    stop_.store(true);
    wake();
    th_.join();
    for (auto& kv : fan_) close(kv.first);
    fan_.clear();
    close(evfd_);
    close(ep_);
  }

  // store thread: queue a committed transaction's events (shared by every fan-out thread) / a
  // new watch (order preserved)
  void post(const std::shared_ptr<const std::vector<Event>>& evs) {
    if (watches_.load(std::memory_order_acquire) == 0) return;   // nobody to tell
    if (pending_.empty() || !pending_.back().evs_only) pending_.emplace_back();
    pending_.back().chunks.push_back(evs);
  }
  void post(std::unique_ptr<FanWatch> w) {
    pending_.emplace_back();
    pending_.back().evs_only = false;
    pending_.back().w = std::move(w);
    watches_.fetch_add(1, std::memory_order_acq_rel);   // before any later event is posted
  }
  // store thread, once per loop pass: hand everything queued to the fan-out thread
  void commit() {
    if (pending_.empty()) return;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (Msg& m : pending_) q_.push_back(std::move(m));
    }
    pending_.clear();
    wake();
  }

 private:
  struct Msg {
    bool evs_only = true;
    std::vector<std::shared_ptr<const std::vector<Event>>> chunks;
    std::unique_ptr<FanWatch> w;
  };

  void wake() {
    uint64_t one = 1;
    ssize_t r = write(evfd_, &one, sizeof one);
    (void)r;
  }

  void loop() {
    epoll_event evs[256];
    std::vector<Msg> work;
    while (!stop_.load()) {
      int n = epoll_wait(ep_, evs, 256, next_timeout_ms());
      for (int i = 0; i < n; ++i) {
        int fd = evs[i].data.fd;
        if (fd == evfd_) {
          uint64_t v;
          ssize_t r = read(evfd_, &v, sizeof v);
          (void)r;
          continue;
        }
        auto fw = fan_.find(fd);
        if (fw == fan_.end()) continue;
        FanWatch* w = fw->second.get();
        if (evs[i].events & (EPOLLHUP | EPOLLERR | EPOLLRDHUP)) { close_fan(w); continue; }
        if (evs[i].events & EPOLLIN) {
          char junk[4096];
          ssize_t r = read(fd, junk, sizeof junk);
          if (r == 0 || (r < 0 && errno != EAGAIN && errno != EWOULDBLOCK)) { close_fan(w); continue; }
        }
        if (evs[i].events & EPOLLOUT) flush_fan(w);
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        work.swap(q_);
      }
      for (Msg& m : work) {
        if (m.w) adopt(std::move(m.w));
        else if (!m.chunks.empty()) {
          KPROF_BEGIN;
          for (const auto& c : m.chunks) fan_dispatch(*c);
          KPROF_END(6);
        }
      }
      work.clear();
      {
        KPROF_BEGIN;
        for (FanWatch* w : fan_dirty_) {
          w->queued = false;
          flush_fan(w);
        }
        fan_dirty_.clear();
        KPROF_END(8);
      }
      expire_fan();
      reap_fan();
    }
  }

  void adopt(std::unique_ptr<FanWatch> w) {
    FanWatch* raw = w.get();
    if (w->send_initial) {
      for (const auto& kv : w->initial) {
        const Index& ix = index_of(*kv, slot_);
        if (w->matches(ix)) emit(raw, "ADDED", kv->value, ix, kv->mod_rev);
      }
    }
    for (const Event& e : w->replay) fan_one(raw, e);
    w->initial.clear();
    w->initial.shrink_to_fit();
    w->replay.clear();
    w->replay.shrink_to_fit();
    epoll_event e{};
    e.events = EPOLLIN | EPOLLRDHUP;
    e.data.fd = raw->fd;
    epoll_ctl(ep_, EPOLL_CTL_ADD, raw->fd, &e);
    if (raw->node_indexed) fan_by_node_[raw->node_key].push_back(raw);
    else fan_other_.push_back(raw);
    fan_[raw->fd] = std::move(w);
    flush_fan(raw);
  }

  int next_timeout_ms() {
    double soonest = 0;
    for (auto& kv : fan_)
      if (kv.second->deadline > 0 && (soonest == 0 || kv.second->deadline < soonest)) soonest = kv.second->deadline;
    if (soonest == 0) return 1000;
    double ms = (soonest - mono_now()) * 1000.0;
    return ms < 0 ? 0 : (ms > 1000 ? 1000 : (int)ms + 1);
  }

  // one event into one watch (cacher.go dispatch rules: a MODIFIED object that stops matching is
  // a DELETED for that watcher, one that starts matching an ADDED)
  void fan_one(FanWatch* w, const Event& ev, const Index* cur = nullptr, const Index* prv = nullptr) {
    if (ev.key.compare(0, w->prefix.size(), w->prefix) != 0 || ev.rev <= w->min_rev) return;
    if (!cur) cur = &index_of(*ev.kv, slot_);
    if (!prv) prv = ev.prev ? &index_of(*ev.prev, slot_) : &empty_index();
    bool now = w->matches(*cur);
    bool was = ev.prev && w->matches(*prv);
    const std::string& v = ev.kv->value;
    if (ev.type == 0) {
      if (now && was) emit(w, "MODIFIED", v, *cur, ev.rev);
      else if (now) emit(w, "ADDED", v, *cur, ev.rev);
      else if (was) emit(w, "DELETED", v, *cur, ev.rev);
      else return;
    } else {
      if (!(now || was) || !cur->ok) return;
      emit(w, "DELETED", v, *cur, ev.rev);
    }
    mark_fan(w);
  }

  // Per event: the unindexed watches, plus the watches of the node the object is on now and
  // was on before (O(matching watchers), not O(all watchers), with one watch per kubelet).
  void fan_dispatch(const std::vector<Event>& evs) {
    if (fan_.empty()) return;
    for (const Event& ev : evs) {
      const Index* cur = nullptr;
      const Index* prv = nullptr;
      auto parse = [&]() {
        if (cur) return;
        cur = &index_of(*ev.kv, slot_);
        prv = ev.prev ? &index_of(*ev.prev, slot_) : &empty_index();
      };
      for (FanWatch* w : fan_other_) {
        if (w->dead || ev.key.compare(0, w->prefix.size(), w->prefix) != 0) continue;
        parse();
        fan_one(w, ev, cur, prv);
      }
      if (fan_by_node_.empty()) continue;
      parse();
      auto node_of = [](const Index& ix) -> std::string_view {
        const std::string_view* it = sv_find(ix.fields, "spec.nodeName");
        return it ? *it : std::string_view();
      };
      std::string_view a = node_of(*cur);
      auto bucket = [&](std::string_view n) {
        auto it = fan_by_node_.find(std::string(n));
        if (it == fan_by_node_.end()) return;
        for (FanWatch* w : it->second)
          if (!w->dead) fan_one(w, ev, cur, prv);
      };
      bucket(a);
      if (ev.prev) {
        std::string_view b = node_of(*prv);
        if (b != a) bucket(b);
      }
    }
    // a superseded value's parse is not needed again (resumed watches re-parse on demand):
    // the cache lives on current values only, so history memory does not grow with it
    for (const Event& ev : evs) {
      if (ev.prev) ev.prev->aux[slot_].reset();
      if (ev.type == 1) ev.kv->aux[slot_].reset();   // a tombstone is never a current value
    }
  }

  void mark_fan(FanWatch* w) {
    if (!w->out.empty() && !w->queued) {
      w->queued = true;
      fan_dirty_.push_back(w);
    }
  }

  void set_pollout(FanWatch* w, bool on) {
    if (w->pollout == on) return;
    w->pollout = on;
    epoll_event e{};
    e.events = EPOLLIN | EPOLLRDHUP | (on ? EPOLLOUT : 0);
    e.data.fd = w->fd;
    epoll_ctl(ep_, EPOLL_CTL_MOD, w->fd, &e);
  }

  void flush_fan(FanWatch* w) {
    while (!w->out.empty()) {
      ssize_t n = write(w->fd, w->out.data(), w->out.size());
      if (g_prof.on) ++g_prof.n[11];   // count of fan-out write() calls
      if (n > 0) { w->out.erase(0, (size_t)n); continue; }
      if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        if (w->out.size() > (64u << 20)) { w->dead = true; w->out.clear(); return; }   // slow watcher
        set_pollout(w, true);
        return;
      }
      w->dead = true;
      w->out.clear();
      return;
    }
    set_pollout(w, false);
  }

  void expire_fan() {
    double now = 0;
    for (auto& kv : fan_) {
      FanWatch* w = kv.second.get();
      if (w->deadline <= 0 || w->dead) continue;
      if (now == 0) now = mono_now();
      if (now >= w->deadline) {
        w->out.append("0\r\n\r\n");   // end of the chunked body: the watch timed out normally
        w->dead = true;
        flush_fan(w);
      }
    }
  }

  void close_fan(FanWatch* w) {
    w->dead = true;
    w->out.clear();
  }

  void reap_fan() {
    for (auto it = fan_.begin(); it != fan_.end();) {
      FanWatch* w = it->second.get();
      if (w->dead && w->out.empty()) {
        fan_dirty_.erase(std::remove(fan_dirty_.begin(), fan_dirty_.end(), w), fan_dirty_.end());
        auto drop = [w](std::vector<FanWatch*>* v) { v->erase(std::remove(v->begin(), v->end(), w), v->end()); };
        if (w->node_indexed) {
          auto b = fan_by_node_.find(w->node_key);
          if (b != fan_by_node_.end()) {
            drop(&b->second);
            if (b->second.empty()) fan_by_node_.erase(b);
          }
        } else {
          drop(&fan_other_);
        }
        epoll_ctl(ep_, EPOLL_CTL_DEL, w->fd, nullptr);
        close(w->fd);
        it = fan_.erase(it);
        watches_.fetch_sub(1, std::memory_order_acq_rel);
      } else {
        ++it;
      }
    }
  }

  const int slot_;                // this thread's KV::aux slot
  // store thread only
  std::vector<Msg> pending_;
  // shared
  std::mutex mu_;
  std::vector<Msg> q_;
  std::atomic<bool> stop_{false};
  std::atomic<int> watches_{0};   // posted and not yet reaped
  std::thread th_;
  int ep_ = -1;
  int evfd_ = -1;
  // fan-out thread only
  std::map<int, std::unique_ptr<FanWatch>> fan_;
  std::vector<FanWatch*> fan_dirty_;
  std::vector<FanWatch*> fan_other_;
  std::unordered_map<std::string, std::vector<FanWatch*>> fan_by_node_;
};

class Server {
 public:
  Server(Engine* e) : eng_(e) {}

  int listen_unix(const char* path) {
    int fd = socket(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    sockaddr_un a{};
    a.sun_family = AF_UNIX;
    snprintf(a.sun_path, sizeof a.sun_path, "%s", path);
    unlink(path);
    if (bind(fd, (sockaddr*)&a, sizeof a) < 0 || listen(fd, 1024) < 0) { perror("bind/listen"); return -1; }
    add_listener(fd);
    return fd;
  }

  int listen_handoff(const char* path) {
    int fd = socket(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    sockaddr_un a{};
    a.sun_family = AF_UNIX;
    snprintf(a.sun_path, sizeof a.sun_path, "%s", path);
    unlink(path);
    if (bind(fd, (sockaddr*)&a, sizeof a) < 0 || listen(fd, 1024) < 0) { perror("bind/listen handoff"); return -1; }
    add_listener(fd);
    handoff_listeners_[fd] = 1;
    return fd;
  }

  int listen_tcp(int port, int* bound) {
    int fd = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    a.sin_port = htons((uint16_t)port);
    if (bind(fd, (sockaddr*)&a, sizeof a) < 0 || listen(fd, 1024) < 0) { perror("bind/listen"); return -1; }
    socklen_t l = sizeof a;
    getsockname(fd, (sockaddr*)&a, &l);
    *bound = ntohs(a.sin_port);
    add_listener(fd);
    return fd;
  }

  // returns when SIGTERM/SIGINT set *stop (a clean exit: destructors run, so leak checkers and
  // the WAL's final fclose see a normal shutdown)
  // watch fan-out threads (1..KV::kAuxSlots); watches are spread over them, events go to all
  void set_fan_threads(int n) {
    n = std::max(1, std::min(n, KV::kAuxSlots));
    fans_.clear();
    for (int i = 0; i < n; ++i) fans_.push_back(std::make_unique<FanOut>(i));
  }

  void run(volatile sig_atomic_t* stop) {
    if (fans_.empty()) set_fan_threads(1);
    for (auto& f : fans_) f->start();
    epoll_event evs[256];
    while (!*stop) {
      int n = epoll_wait(ep_, evs, 256, 1000);
      for (int i = 0; i < n; ++i) {
        int fd = evs[i].data.fd;
        if (handoff_listeners_.count(fd)) { accept_handoffs(fd); continue; }
        if (listeners_.count(fd)) { accept_all(fd); continue; }
        if (handoffs_.count(fd)) { read_handoff(fd); continue; }
        auto it = conns_.find(fd);
        if (it == conns_.end()) continue;
        Conn* c = it->second.get();
        if (evs[i].events & (EPOLLHUP | EPOLLERR)) { close_conn(c); continue; }
        if (evs[i].events & EPOLLIN) {
          if (!read_conn(c)) { close_conn(c); continue; }
        }
        if (evs[i].events & EPOLLOUT) flush(c);
      }
      // this pass's committed events and new watches go to the fan-out threads in one batch each
      for (auto& f : fans_) f->commit();
      if (progress_pending_) {
        KPROF_BEGIN;
        send_progress();
        KPROF_END(9);
      }
      // flush every connection with pending output once per loop (coalesces watch events)
      {
        KPROF_BEGIN;
        for (Conn* c : dirty_) flush(c);
        dirty_.clear();
        KPROF_END(7);
      }
    }
    for (auto& f : fans_) f->stop();
  }

 private:
  void add_listener(int fd) {
    if (ep_ < 0) ep_ = epoll_create1(EPOLL_CLOEXEC);
    epoll_event e{};
    e.events = EPOLLIN;
    e.data.fd = fd;
    epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &e);
    listeners_[fd] = 1;
  }

  void accept_all(int lfd) {
    for (;;) {
      int fd = accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      auto c = std::make_unique<Conn>();
      c->fd = fd;
      epoll_event e{};
      e.events = EPOLLIN | EPOLLRDHUP;
      e.data.fd = fd;
      epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &e);
      conns_[fd] = std::move(c);
    }
  }

  void close_conn(Conn* c) {
    for (size_t i = 0; i < watches_.size();) {
      if (watches_[i].conn == c) { watches_[i] = watches_.back(); watches_.pop_back(); } else ++i;
    }
    epoll_ctl(ep_, EPOLL_CTL_DEL, c->fd, nullptr);
    close(c->fd);
    dirty_.erase(std::remove(dirty_.begin(), dirty_.end(), c), dirty_.end());
    conns_.erase(c->fd);
  }

  bool read_conn(Conn* c) {
    KPROF_BEGIN;
    struct Done {
      double t0;
      ~Done() { if (g_prof.on) g_prof.add(0, t0); }
    } done{_kp0};
    char buf[1 << 16];
    for (;;) {
      ssize_t n = read(c->fd, buf, sizeof buf);
      if (n > 0) { c->in.append(buf, (size_t)n); continue; }
      if (n == 0) return false;
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      return false;
    }
    size_t off = 0;
    while (c->in.size() - off >= 9) {
      uint32_t len;
      memcpy(&len, c->in.data() + off, 4);
      // a frame is id(4) + op(1) + body: shorter is malformed, longer than kMaxFrame would only
      // make this connection buffer without bound — either ends the connection
      if (len < 5 || len > kMaxFrame) return false;
      if (c->in.size() - off - 4 < len) break;
      uint32_t id;
      memcpy(&id, c->in.data() + off + 4, 4);
      uint8_t op = (uint8_t)c->in[off + 8];
      handle(c, id, op, c->in.data() + off + 9, len - 5);
      off += 4 + len;
    }
    c->in.erase(0, off);
    return true;
  }

  void reply(Conn* c, uint32_t id, uint8_t status, const std::string& payload) {
    uint32_t len = (uint32_t)(payload.size() + 5);
    c->out.append(reinterpret_cast<const char*>(&len), 4);
    c->out.append(reinterpret_cast<const char*>(&id), 4);
    c->out.push_back((char)status);
    c->out.append(payload);
    mark(c);
  }

  void mark(Conn* c) {
    if (!c->want_write) {
      c->want_write = true;
      dirty_.push_back(c);
    }
  }

  void set_pollout(Conn* c, bool on) {
    if (c->pollout == on) return;
    c->pollout = on;
    epoll_event e{};
    e.events = EPOLLIN | EPOLLRDHUP | (on ? EPOLLOUT : 0);
    e.data.fd = c->fd;
    epoll_ctl(ep_, EPOLL_CTL_MOD, c->fd, &e);
  }

  void flush(Conn* c) {
    while (!c->out.empty()) {
      ssize_t n = write(c->fd, c->out.data(), c->out.size());
      if (n > 0) { c->out.erase(0, (size_t)n); continue; }
      if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        set_pollout(c, true);
        c->want_write = false;
        return;
      }
      break;
    }
    c->want_write = false;
    set_pollout(c, false);
  }

  void send_progress() {
    progress_pending_ = false;
    for (Watch& w : watches_) {
      if (!w.progress) continue;
      Writer pw;
      pw.put<int64_t>(w.progress);
      w.progress = 0;
      reply(w.conn, w.id, 10, pw.b);
    }
  }

  void dispatch(const std::vector<Event>& evs) {
    if (watches_.empty()) return;
    for (const Event& ev : evs) {
      for (Watch& w : watches_) {
        if (ev.key.compare(0, w.prefix.size(), w.prefix) != 0) continue;
        if (!w.excl.empty() && w.excluded(ev.key)) {
          w.progress = ev.rev;
          progress_pending_ = true;
          continue;
        }
        Writer pw;
        pw.put<uint8_t>(ev.type);
        pw.kv(ev.key, *ev.kv);
        reply(w.conn, w.id, 8, pw.b);
      }
    }
  }

  void handle(Conn* c, uint32_t id, uint8_t op, const char* p, uint32_t n) {
    Reader r{p, p + n};
    Writer w;
    switch (op) {
      case 1: {  // TXN
        KPROF_BEGIN;
        std::vector<Cmp> cmps;
        std::vector<Op> ops;
        if (!parse_txn(r, &cmps, &ops)) { reply(c, id, 9, ""); return; }
        int64_t rev;
        std::vector<Event> evs;
        int failed = eng_->txn(cmps, ops, &rev, &evs);
        KPROF_END(1);
        if (failed < 0) {
          w.put<int64_t>(rev);
          reply(c, id, 0, w.b);
          {
            KPROF_BEGIN;
            dispatch(evs);
            KPROF_END(5);
          }
          post_events(std::move(evs));
        } else {
          w.put<uint16_t>((uint16_t)failed);
          const KV* kv = eng_->get(cmps[failed].key);
          w.put<uint8_t>(kv ? 1 : 0);
          if (kv) w.kv(cmps[failed].key, *kv);
          w.put<int64_t>(eng_->rev());
          reply(c, id, 1, w.b);
        }
        return;
      }
      case 2: {  // GET
        KPROF_BEGIN;
        struct Done {
          double t0;
          ~Done() { if (g_prof.on) g_prof.add(2, t0); }
        } done{_kp0};
        std::string k = r.str();
        const KV* kv = eng_->get(k);
        if (!kv) { w.put<int64_t>(eng_->rev()); reply(c, id, 4, w.b); return; }
        w.kv(k, *kv);
        w.put<int64_t>(eng_->rev());
        reply(c, id, 0, w.b);
        return;
      }
      case 3: {  // RANGE
        KPROF_BEGIN;
        struct Done {
          double t0;
          ~Done() { if (g_prof.on) g_prof.add(3, t0); }
        } done{_kp0};
        std::string prefix = r.str();
        uint32_t limit = r.get<uint32_t>();
        std::string sa = r.str();
        std::vector<std::pair<const std::string*, const KV*>> res;
        bool more;
        int64_t rev = eng_->range(prefix, limit, sa, &res, &more);
        w.put<int64_t>(rev);
        w.put<uint8_t>(more ? 1 : 0);
        w.put<uint32_t>((uint32_t)res.size());
        for (auto& kv : res) w.kv(*kv.first, *kv.second);
        reply(c, id, 0, w.b);
        return;
      }
      case 7: {  // RANGE at a past revision: prefix, limit, start_after, revision
        std::string prefix = r.str();
        uint32_t limit = r.get<uint32_t>();
        std::string sa = r.str();
        int64_t at = r.get<int64_t>();
        if (!r.ok) { reply(c, id, 9, ""); return; }
        if (at > eng_->rev()) { w.put<int64_t>(eng_->rev()); reply(c, id, 9, w.b); return; }   // future
        std::vector<std::pair<std::string, std::shared_ptr<KV>>> res;
        bool more;
        if (!eng_->range_at(prefix, at, limit, sa, &res, &more)) {
          w.put<int64_t>(eng_->compacted());
          reply(c, id, 3, w.b);
          return;
        }
        w.put<int64_t>(at);
        w.put<uint8_t>(more ? 1 : 0);
        w.put<uint32_t>((uint32_t)res.size());
        for (auto& kv : res) w.kv(kv.first, *kv.second);
        reply(c, id, 0, w.b);
        return;
      }
      case 4: {  // WATCH
        int64_t from = r.get<int64_t>();
        std::string prefix = r.str();
        Watch nw{c, id, prefix};
        if (r.p + 2 <= r.e) {
          uint16_t nx = r.get<uint16_t>();
          for (uint16_t i = 0; i < nx && r.ok; ++i) nw.excl.push_back(r.str());
          if (!r.ok) { reply(c, id, 9, ""); return; }
        }
        std::vector<const Event*> evs;
        if (from > 0 && !eng_->since(from, prefix, &evs)) {
          w.put<int64_t>(eng_->compacted());
          reply(c, id, 3, w.b);
          return;
        }
        w.put<int64_t>(eng_->rev());
        reply(c, id, 0, w.b);
        for (const Event* e : evs) {
          if (!nw.excl.empty() && nw.excluded(e->key)) continue;
          Writer pw;
          pw.put<uint8_t>(e->type);
          pw.kv(e->key, *e->kv);
          reply(c, id, 8, pw.b);
        }
        watches_.push_back(std::move(nw));
        return;
      }
      case 5:
        w.put<int64_t>(eng_->rev());
        reply(c, id, 0, w.b);
        return;
      case 6:
        eng_->compact(r.get<int64_t>());
        reply(c, id, 0, "");
        return;
      default:
        reply(c, id, 9, "");
    }
  }


  // -- watch fan-out ---------------------------------------------------------
  struct Handoff {
    std::string buf;
    int client = -1;
  };

  void accept_handoffs(int lfd) {
    for (;;) {
      int fd = accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      epoll_event e{};
      e.events = EPOLLIN | EPOLLRDHUP;
      e.data.fd = fd;
      epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &e);
      handoffs_[fd] = Handoff{};
    }
  }

  void drop_handoff(int fd) {
    auto it = handoffs_.find(fd);
    if (it != handoffs_.end() && it->second.client >= 0) close(it->second.client);
    handoffs_.erase(fd);
    epoll_ctl(ep_, EPOLL_CTL_DEL, fd, nullptr);
    close(fd);
  }

  void read_handoff(int fd) {
    Handoff& h = handoffs_[fd];
    for (;;) {
      char data[8192];
      char ctl[CMSG_SPACE(sizeof(int))];
      iovec iov{data, sizeof data};
      msghdr mh{};
      mh.msg_iov = &iov;
      mh.msg_iovlen = 1;
      mh.msg_control = ctl;
      mh.msg_controllen = sizeof ctl;
      ssize_t n = recvmsg(fd, &mh, MSG_CMSG_CLOEXEC);
      if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) return;   // wait for the rest
      if (n <= 0) { drop_handoff(fd); return; }
      for (cmsghdr* c = CMSG_FIRSTHDR(&mh); c; c = CMSG_NXTHDR(&mh, c)) {
        if (c->cmsg_level == SOL_SOCKET && c->cmsg_type == SCM_RIGHTS) {
          int got;
          memcpy(&got, CMSG_DATA(c), sizeof got);
          if (h.client >= 0) close(got); else h.client = got;
        }
      }
      h.buf.append(data, (size_t)n);
      if (h.buf.size() >= 4) {
        uint32_t len;
        memcpy(&len, h.buf.data(), 4);
        if (len > kMaxFrame) {                  // a watch spec is a few hundred bytes
          if (h.client >= 0) close(h.client);
          h.client = -1;
          drop_handoff(fd);
          return;
        }
        if (h.buf.size() >= 4 + (size_t)len) {
          int client = h.client;
          std::string msg = h.buf.substr(4, len);
          h.client = -1;
          drop_handoff(fd);                     // one watch per handoff connection
          if (client >= 0) start_fan(client, msg);
          return;
        }
      }
    }
  }

  void start_fan(int client, const std::string& msg) {
    Reader r{msg.data(), msg.data() + msg.size()};
    auto w = std::make_unique<FanWatch>();
    w->fd = client;
    uint8_t ver = r.get<uint8_t>();
    uint8_t send_initial = r.get<uint8_t>();
    int64_t from = r.get<int64_t>();
    double timeout = r.get<double>();
    w->prefix = r.str();
    uint16_t nreq = r.get<uint16_t>();
    for (uint16_t i = 0; i < nreq && r.ok; ++i) {
      Requirement q;
      q.target = r.get<uint8_t>();
      q.op = r.get<uint8_t>();
      q.key = r.str();
      uint16_t nv = r.get<uint16_t>();
      for (uint16_t j = 0; j < nv && r.ok; ++j) q.vals.push_back(r.str());
      w->reqs.push_back(std::move(q));
    }
    if (ver == 2) w->pb = r.get<uint8_t>() == 1;   // v2: trailing format byte
    if (!r.ok || (ver != 1 && ver != 2)) { close(client); return; }
    for (const Requirement& q : w->reqs)
      if (q.target == 1 && q.op == 0 && q.vals.size() == 1 && q.key == "spec.nodeName") {
        // kubelets watch their own node's pods (cacher.go's nodeName-indexed watchers)
        w->node_indexed = true;
        w->node_key = q.vals[0];
        break;
      }
    int fl = fcntl(client, F_GETFL);
    fcntl(client, F_SETFL, fl | O_NONBLOCK);
    int one = 1;
    setsockopt(client, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    if (timeout > 0) w->deadline = mono_now() + timeout;
    w->out = std::string("HTTP/1.1 200 OK\r\nContent-Type: ") +
             (w->pb ? "application/vnd.kubernetes.protobuf;stream=watch" : "application/json") +
             "\r\nTransfer-Encoding: chunked\r\nCache-Control: no-cache, private\r\n\r\n";
    if (send_initial) {
      // the snapshot is taken here, in commit order; the fan-out thread parses and formats it
      w->send_initial = true;
      eng_->for_prefix(w->prefix, [&](const std::string&, const std::shared_ptr<KV>& kv) { w->initial.push_back(kv); });
    } else if (from > 0) {
      std::vector<const Event*> evs;
      if (!eng_->since(from, w->prefix, &evs)) {
        char b[512];
        snprintf(b, sizeof b,
                 "{\"type\":\"ERROR\",\"object\":{\"kind\":\"Status\",\"apiVersion\":\"v1\",\"metadata\":{},"
                 "\"status\":\"Failure\",\"message\":\"too old resource version: %lld (%lld)\",\"reason\":\"Expired\","
                 "\"code\":410}}\n", (long long)from, (long long)eng_->compacted());
        if (w->pb) {
          // the metav1.Status as a protobuf envelope (v1/Status), what a protobuf stream
          // decoder expects in an ERROR frame (watch.go:166-226)
          char msg[160];
          snprintf(msg, sizeof msg, "too old resource version: %lld (%lld)", (long long)from,
                   (long long)eng_->compacted());
          chunk_pb(&w->out, "ERROR", status_envelope(msg, "Expired", 410));
          w->out.append("0\r\n\r\n");
        } else {
          char hex[24];
          int hl = snprintf(hex, sizeof hex, "%zx\r\n", strlen(b));
          w->out.append(hex, (size_t)hl).append(b).append("\r\n0\r\n\r\n");
        }
        w->dead = true;   // close once written
      } else {
        w->replay.reserve(evs.size());
        for (const Event* e : evs) w->replay.push_back(*e);
      }
      w->min_rev = from;
    }
    // the least loaded fan-out thread adopts the watch
    FanOut* best = fans_[0].get();
    for (auto& f : fans_)
      if (f->watches() < best->watches()) best = f.get();
    best->post(std::move(w));
  }

  void post_events(std::vector<Event>&& evs) {
    bool any = false;
    for (auto& f : fans_) any |= f->watches() > 0;
    if (!any) return;
    auto sp = std::make_shared<const std::vector<Event>>(std::move(evs));
    for (auto& f : fans_) f->post(sp);
  }

  std::unordered_map<int, int> handoff_listeners_;
  std::unordered_map<int, Handoff> handoffs_;
  std::vector<std::unique_ptr<FanOut>> fans_;

  Engine* eng_;
  int ep_ = -1;
  std::unordered_map<int, int> listeners_;
  std::unordered_map<int, std::unique_ptr<Conn>> conns_;
  std::vector<Watch> watches_;
  bool progress_pending_ = false;
  std::vector<Conn*> dirty_;
};

}  // namespace kamd

static volatile sig_atomic_t g_stop = 0;
static void on_term(int) { g_stop = 1; }

int main(int argc, char** argv) {
  signal(SIGPIPE, SIG_IGN);
  struct sigaction sa{};
  sa.sa_handler = on_term;   // no SA_RESTART: epoll_wait returns EINTR and the loop sees g_stop
  sigaction(SIGTERM, &sa, nullptr);
  sigaction(SIGINT, &sa, nullptr);
  const char* unix_path = nullptr;
  const char* wal = nullptr;
  const char* port_file = nullptr;
  const char* handoff_path = nullptr;
  int tcp_port = -1;
  int fan_threads = 1;
  size_t hist = 500000;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&](void) { return i + 1 < argc ? argv[++i] : ""; };
    if (a == "--listen-unix") unix_path = val();
    else if (a == "--listen-tcp") tcp_port = atoi(val());
    else if (a == "--wal") wal = val();
    else if (a == "--history") hist = (size_t)atol(val());
    else if (a == "--port-file") port_file = val();
    else if (a == "--listen-handoff") handoff_path = val();
    else if (a == "--fan-threads") fan_threads = atoi(val());
    else if (a == "--pb-schema") {
      g_pb_schema = new pbc::Schema();
      if (!g_pb_schema->load(val())) {
        fprintf(stderr, "kamd-etcd: --pb-schema: %s\n", g_pb_schema->error.c_str());
        return 2;
      }
    }
    else { fprintf(stderr, "usage: kamd-etcd [--listen-unix PATH] [--listen-tcp PORT] [--listen-handoff PATH] [--wal FILE] [--history N] [--fan-threads N] [--pb-schema FILE]\n"); return 2; }
  }
  kamd::Engine eng(hist);
  if (wal && !eng.open_wal(wal)) { perror("wal"); return 1; }
  kamd::Server srv(&eng);
  srv.set_fan_threads(fan_threads);
  if (unix_path && srv.listen_unix(unix_path) < 0) return 1;
  if (handoff_path && srv.listen_handoff(handoff_path) < 0) return 1;
  if (tcp_port >= 0) {
    int bound = 0;
    if (srv.listen_tcp(tcp_port, &bound) < 0) return 1;
    if (port_file) {
      FILE* f = fopen(port_file, "w");
      fprintf(f, "%d", bound);
      fclose(f);
    }
  }
  fprintf(stderr, "kamd-etcd: serving (rev %lld, %zu keys)\n", (long long)eng.rev(), eng.size());
  kamd::g_prof.on = getenv("KAMD_ETCD_PROFILE") && *getenv("KAMD_ETCD_PROFILE") == '1';
  srv.run(&g_stop);
  kamd::g_prof.print();
  if (unix_path) unlink(unix_path);
  if (handoff_path) unlink(handoff_path);
  return 0;
}
#endif
