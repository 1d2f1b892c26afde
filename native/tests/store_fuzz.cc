// Differential fuzz of the native MVCC engine (native/store/mvcc_store.cc) against a tiny
// reference model, built with AddressSanitizer + UndefinedBehaviorSanitizer by
// `python -m kubernetes_amd.native.build --sanitize` (race/sanitizer tier, SURVEY §5.2: the
// reference runs Go's -race on unit tests; here the native code gets ASan/UBSan/TSan runs).
//
// Covers: multi-op transactions with mod-rev / exists / absent / value compares, puts with
// resource-version injection, deletes with tombstones, ordered paged ranges, watch history
// (`since`) with compaction, and WAL replay (reopened engine == live engine).
//
//   store_fuzz [iterations] [seed] [wal_path]      exit 0 = no divergence
#include "../store/mvcc_store.cc"

#include <random>

namespace {

struct MKV {
  int64_t create = 0, mod = 0, ver = 0;
  std::string val;
};

struct MEvent {
  uint8_t type;
  int64_t rev;
  std::string key;
};

struct Model {
  std::map<std::string, MKV> data;
  std::vector<MEvent> hist;
  int64_t rev = 1;
};

int g_fail = 0;
#define CHECK(c, ...)                                  \
  do {                                                 \
    if (!(c)) {                                        \
      fprintf(stderr, "DIVERGENCE %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                    \
      fprintf(stderr, "\n");                           \
      if (++g_fail > 20) exit(1);                      \
    }                                                  \
  } while (0)

std::string replace_all(std::string v, const std::string& tok, const std::string& rs) {
  if (tok.empty()) return v;
  size_t p = 0;
  while ((p = v.find(tok, p)) != std::string::npos) {
    v.replace(p, tok.size(), rs);
    p += rs.size();
  }
  return v;
}

// encode a TXN payload exactly as the wire protocol does
std::string encode(const std::vector<kamd::Cmp>& cmps, const std::vector<kamd::Op>& ops) {
  kamd::Writer w;
  w.put<uint16_t>((uint16_t)cmps.size());
  for (auto& c : cmps) {
    w.put<uint8_t>(c.kind);
    w.str(c.key);
    w.put<int64_t>(c.arg);
    w.str(c.val);
  }
  w.put<uint16_t>((uint16_t)ops.size());
  for (auto& o : ops) {
    w.put<uint8_t>(o.kind);
    w.str(o.key);
    w.str(o.val);
    if (o.kind >= 2) w.str(o.token);
  }
  return w.b;
}

int model_txn(Model& m, const std::vector<kamd::Cmp>& cmps, const std::vector<kamd::Op>& ops) {
  for (size_t i = 0; i < cmps.size(); ++i) {
    auto it = m.data.find(cmps[i].key);
    bool ok = false;
    switch (cmps[i].kind) {
      case 0: ok = it != m.data.end() ? it->second.mod == cmps[i].arg : cmps[i].arg == 0; break;
      case 1: ok = it != m.data.end(); break;
      case 2: ok = it == m.data.end(); break;
      case 3: ok = it != m.data.end() && it->second.val == cmps[i].val; break;
    }
    if (!ok) return (int)i;
  }
  int64_t r = m.rev + 1;
  std::string rs = std::to_string(r);
  bool changed = false;
  for (auto& o : ops) {
    if (o.kind == 0 || o.kind == 2) {
      MKV& kv = m.data[o.key];
      if (kv.ver == 0) kv.create = r;
      kv.ver += 1;
      kv.mod = r;
      kv.val = replace_all(o.val, o.kind == 2 ? o.token : "", rs);
      m.hist.push_back({0, r, o.key});
      changed = true;
    } else if (m.data.erase(o.key)) {
      m.hist.push_back({1, r, o.key});
      changed = true;
    }
  }
  if (changed) m.rev = r;
  return -1;
}

void compare_all(kamd_store* s, const Model& m, const char* when) {
  CHECK(kamd_store_rev(s) == m.rev, "%s: rev %lld vs model %lld", when, (long long)kamd_store_rev(s), (long long)m.rev);
  CHECK(kamd_store_size(s) == m.data.size(), "%s: size %llu vs %zu", when, (unsigned long long)kamd_store_size(s),
        m.data.size());
  for (auto& [k, v] : m.data) {
    const char* out;
    uint32_t n;
    int found = kamd_store_get(s, k.data(), (uint32_t)k.size(), &out, &n);
    CHECK(found == 1, "%s: %s missing", when, k.c_str());
    if (found != 1) continue;
    kamd::Reader r{out, out + n};
    int64_t cr = r.get<int64_t>(), mr = r.get<int64_t>(), ver = r.get<int64_t>();
    std::string key = r.str(), val = r.str();
    CHECK(r.ok && key == k && cr == v.create && mr == v.mod && ver == v.ver && val == v.val,
          "%s: kv %s differs (cr %lld/%lld mod %lld/%lld ver %lld/%lld)", when, k.c_str(), (long long)cr,
          (long long)v.create, (long long)mr, (long long)v.mod, (long long)ver, (long long)v.ver);
  }
}

}  // namespace

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  const unsigned seed = argc > 2 ? (unsigned)atoi(argv[2]) : 1;
  const char* wal = argc > 3 ? argv[3] : nullptr;
  if (wal) unlink(wal);
  std::mt19937 rng(seed);
  auto rnd = [&](int n) { return (int)(rng() % (unsigned)n); };
  const size_t HIST = 4096;
  kamd_store* s = kamd_store_open(wal, HIST);
  if (!s) { fprintf(stderr, "open failed\n"); return 2; }
  Model m;
  std::vector<std::string> keys;
  for (int i = 0; i < 24; ++i) keys.push_back("/registry/pods/ns" + std::to_string(i % 3) + "/p" + std::to_string(i));
  for (int i = 0; i < 8; ++i) keys.push_back("/registry/devices/node-0/amd.com/gpu/" + std::to_string(i));
  const std::string tok = "@rv-TOKEN@";
  int64_t compacted = 0;

  for (int it = 0; it < iters; ++it) {
    int what = rnd(100);
    if (what < 70) {  // transaction
      std::vector<kamd::Cmp> cmps;
      std::vector<kamd::Op> ops;
      int nc = rnd(3), no = 1 + rnd(3);
      for (int i = 0; i < nc; ++i) {
        kamd::Cmp c;
        c.kind = (uint8_t)rnd(4);
        c.key = keys[rnd((int)keys.size())];
        auto mk = m.data.find(c.key);
        c.arg = (mk != m.data.end() && rnd(4)) ? mk->second.mod : rnd(3);
        c.val = (mk != m.data.end() && rnd(2)) ? mk->second.val : "x";
        cmps.push_back(c);
      }
      for (int i = 0; i < no; ++i) {
        kamd::Op o;
        o.kind = (uint8_t)rnd(4);
        o.key = keys[rnd((int)keys.size())];
        o.val = "{\"rv\":\"" + tok + "\",\"n\":" + std::to_string(rnd(1000)) + (rnd(2) ? "," + tok : "") + "}";
        o.token = tok;
        ops.push_back(o);
      }
      std::string req = encode(cmps, ops);
      int64_t rev = 0;
      int got = kamd_store_txn(s, req.data(), (uint32_t)req.size(), &rev);
      int want = model_txn(m, cmps, ops);
      CHECK(got == want, "iter %d: txn result %d vs model %d", it, got, want);
      if (got == -1) CHECK(rev == m.rev, "iter %d: txn rev %lld vs %lld", it, (long long)rev, (long long)m.rev);
    } else if (what < 85) {  // paged range
      std::string prefix = rnd(2) ? "/registry/pods/ns" + std::to_string(rnd(3)) + "/" : "/registry/";
      uint32_t limit = (uint32_t)rnd(6);
      std::string after;
      std::vector<std::string> got;
      for (int page = 0; page < 64; ++page) {
        const char* out;
        uint32_t n;
        int cnt = kamd_store_range(s, prefix.data(), (uint32_t)prefix.size(), limit, after.data(),
                                   (uint32_t)after.size(), &out, &n);
        kamd::Reader r{out, out + n};
        int64_t rrev = r.get<int64_t>();
        uint8_t more = r.get<uint8_t>();
        uint32_t k = r.get<uint32_t>();
        CHECK(rrev == m.rev && (int)k == cnt, "range header");
        for (uint32_t i = 0; i < k; ++i) {
          r.get<int64_t>(); r.get<int64_t>(); r.get<int64_t>();
          after = r.str();
          r.str();
          got.push_back(after);
        }
        CHECK(r.ok, "range decode");
        if (!more) break;
      }
      std::vector<std::string> want;
      for (auto& [k, v] : m.data)
        if (k.compare(0, prefix.size(), prefix) == 0) want.push_back(k);
      CHECK(got == want, "iter %d: range %s limit %u: %zu keys vs %zu", it, prefix.c_str(), limit, got.size(), want.size());
    } else if (what < 97) {  // watch history
      int64_t from = m.rev - rnd(64);
      const char* out;
      uint32_t n;
      std::string prefix = "/registry/pods/";
      int cnt = kamd_store_since(s, from, prefix.data(), (uint32_t)prefix.size(), &out, &n);
      int64_t eng_compacted = kamd_store_compacted(s);
      if (from < eng_compacted) {
        CHECK(cnt == -1, "iter %d: since(%lld) below compaction %lld must fail", it, (long long)from, (long long)eng_compacted);
      } else {
        size_t want = 0;
        for (auto& e : m.hist)
          if (e.rev > from && e.key.compare(0, prefix.size(), prefix) == 0) ++want;
        CHECK(cnt == (int)want, "iter %d: since(%lld) %d events vs %zu", it, (long long)from, cnt, want);
        kamd::Reader r{out, out + n};
        uint32_t k = r.get<uint32_t>();
        for (uint32_t i = 0; i < k; ++i) {
          uint8_t t = r.get<uint8_t>();
          r.get<int64_t>();
          int64_t mod = r.get<int64_t>();
          int64_t ver = r.get<int64_t>();
          r.str();
          r.str();
          CHECK(mod > from && (t == 0 || ver == 0), "event fields");
        }
        CHECK(r.ok, "since decode");
      }
    } else {  // compaction
      int64_t to = m.rev - rnd(32);
      if (to > compacted) {
        kamd_store_compact(s, to);
        compacted = to;
        while (!m.hist.empty() && m.hist.front().rev <= to) m.hist.erase(m.hist.begin());
      }
    }
    // the engine also compacts itself when its history is full: mirror that in the model
    while (m.hist.size() > HIST) m.hist.erase(m.hist.begin());
    if (it % 997 == 0) compare_all(s, m, "live");
  }
  compare_all(s, m, "final");
  if (wal) {
    kamd_store* r = kamd_store_open(wal, HIST);
    if (!r) { fprintf(stderr, "reopen failed\n"); return 2; }
    compare_all(r, m, "replayed");
    kamd_store_close(r);
  }
  kamd_store_close(s);
  if (g_fail) { fprintf(stderr, "%d divergences\n", g_fail); return 1; }
  printf("store_fuzz: %d iterations, seed %u, rev %lld, %zu keys: OK\n", iters, seed, (long long)m.rev, m.data.size());
  return 0;
}
