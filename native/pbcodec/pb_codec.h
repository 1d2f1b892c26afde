// pb_codec.h — schema-driven Kubernetes protobuf codec core (header-only, no Python).
//
// Loads the schema table that hack/gen_proto_schema.py generates from the reference's
// generated.proto files (kubernetes_amd/api/generated/k8s_proto_schema.json) and transcodes the
// etcd storage format — `k8s\0` + runtime.Unknown{TypeMeta, raw} (reference
// staging/src/k8s.io/apimachinery/pkg/runtime/serializer/protobuf/protobuf.go:42, runtime/types.go:112-124)
// — to the object's JSON form, injecting metadata.resourceVersion (etcd3 stores objects without
// it and sets it from the key's mod revision on read, staging/src/k8s.io/apiserver/pkg/storage/etcd3/store.go).
// Used by the Python extension (native/pbcodec/kamd_pbcodec.cc) and by kamd-etcd's watch fan-out,
// which streams protobuf-stored objects to JSON watchers without a Python hop.
//
// The JSON form follows api/protobuf.py exactly (tests compare the two): fields in field-number
// order, inline-embedded messages (json:",inline") flattened into their parent, special types
// (meta/v1 Time/MicroTime/Duration, resource.Quantity, intstr.IntOrString,
// runtime.RawExtension, apiextensions JSON / JSONSchemaPropsOr*, ExtraValue/Verbs slices) in
// their custom JSON encodings, bytes as base64, maps in wire (sorted) order.
#pragma once

#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <fstream>
#include <memory>
#include <sstream>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace pbc {

enum Scalar : uint8_t { S_STRING, S_BYTES, S_BOOL, S_INT32, S_INT64, S_UINT32, S_UINT64, S_DOUBLE, S_MSG };
enum Special : uint8_t {
  SP_NONE, SP_TIME, SP_MICROTIME, SP_DURATION, SP_QUANTITY, SP_INTORSTR, SP_RAWEXT, SP_JSONRAW,
  SP_ORBOOL, SP_ORARRAY, SP_ORSTRARRAY, SP_SLICE
};
enum Label : uint8_t { L_OPT, L_REP, L_MAP };

struct Field {
  std::string json;
  uint32_t num = 0;
  Label label = L_OPT;
  Scalar type = S_STRING;
  int msg = -1;          // message index when type == S_MSG
  Special sp = SP_NONE;  // special encoding of that message
  Scalar key = S_STRING; // map key type
  bool inl = false;      // json:",inline"
  uint8_t wt = 2;        // wire type
};

struct Message {
  std::string name;
  std::vector<Field> fields;                        // sorted by number
  std::vector<int16_t> by_num;                      // field number -> index (-1)
  // JSON key -> index of the top-level field it encodes into (an inline field for embedded keys)
  std::unordered_map<std::string, int> by_json;
  std::vector<std::string> inline_keys_of;          // unused placeholder for layout stability
  int metadata = -1;                                // index of the ObjectMeta "metadata" field
};

// ---------------------------------------------------------------------------------------------
// minimal JSON reader for the schema file
struct JV {
  enum T { NUL, BOOL, NUM, STR, ARR, OBJ } t = NUL;
  bool b = false;
  double n = 0;
  std::string s;
  std::vector<JV> a;
  std::vector<std::pair<std::string, JV>> o;
};

struct JReader {
  const char* p;
  const char* e;
  bool ok = true;
  void ws() { while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p; }
  std::string str() {
    std::string out;
    if (p >= e || *p != '"') { ok = false; return out; }
    ++p;
    while (p < e && *p != '"') {
      char c = *p++;
      if (c == '\\' && p < e) {
        char d = *p++;
        switch (d) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          case 'r': out += '\r'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'u': {
            if (e - p < 4) { ok = false; return out; }
            unsigned cp = (unsigned)strtoul(std::string(p, 4).c_str(), nullptr, 16);
            p += 4;
            if (cp < 0x80) out += (char)cp;
            else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
            else { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
            break;
          }
          default: out += d;
        }
      } else {
        out += c;
      }
    }
    if (p >= e) ok = false; else ++p;
    return out;
  }
  JV val(int depth = 0) {
    JV v;
    ws();
    if (p >= e || depth > 64) { ok = false; return v; }
    if (*p == '{') {
      v.t = JV::OBJ; ++p; ws();
      if (p < e && *p == '}') { ++p; return v; }
      while (ok) {
        ws();
        std::string k = str();
        ws();
        if (p >= e || *p != ':') { ok = false; break; }
        ++p;
        v.o.emplace_back(std::move(k), val(depth + 1));
        ws();
        if (p < e && *p == ',') { ++p; continue; }
        if (p < e && *p == '}') { ++p; break; }
        ok = false;
      }
      return v;
    }
    if (*p == '[') {
      v.t = JV::ARR; ++p; ws();
      if (p < e && *p == ']') { ++p; return v; }
      while (ok) {
        v.a.push_back(val(depth + 1));
        ws();
        if (p < e && *p == ',') { ++p; continue; }
        if (p < e && *p == ']') { ++p; break; }
        ok = false;
      }
      return v;
    }
    if (*p == '"') { v.t = JV::STR; v.s = str(); return v; }
    if (e - p >= 4 && !strncmp(p, "true", 4)) { p += 4; v.t = JV::BOOL; v.b = true; return v; }
    if (e - p >= 5 && !strncmp(p, "false", 5)) { p += 5; v.t = JV::BOOL; return v; }
    if (e - p >= 4 && !strncmp(p, "null", 4)) { p += 4; return v; }
    char* end;
    v.n = strtod(p, &end);
    if (end == p) { ok = false; return v; }
    p = end;
    v.t = JV::NUM;
    return v;
  }
};

static const char* const META = "k8s.io.apimachinery.pkg.apis.meta.v1.";
static const char* const AXP = "k8s.io.apiextensions_apiserver.pkg.apis.apiextensions.v1beta1.";

struct Schema {
  std::vector<Message> msgs;
  std::unordered_map<std::string, int> by_name;
  std::unordered_map<std::string, int> kinds;   // "group/version/Kind" (core: "v1/Kind")
  int schema_props = -1;                        // apiextensions JSONSchemaProps
  std::string error;

  static Scalar scalar_of(const std::string& t, bool* is_scalar) {
    *is_scalar = true;
    if (t == "string") return S_STRING;
    if (t == "bytes") return S_BYTES;
    if (t == "bool") return S_BOOL;
    if (t == "int32" || t == "sint32") return S_INT32;
    if (t == "int64" || t == "sint64") return S_INT64;
    if (t == "uint32") return S_UINT32;
    if (t == "uint64") return S_UINT64;
    if (t == "double" || t == "float") return S_DOUBLE;
    *is_scalar = false;
    return S_MSG;
  }

  static Special special_of(const std::string& n) {
    std::string meta = META, ax = AXP;
    if (n == meta + "Time") return SP_TIME;
    if (n == meta + "MicroTime") return SP_MICROTIME;
    if (n == meta + "Duration") return SP_DURATION;
    if (n == "k8s.io.apimachinery.pkg.api.resource.Quantity") return SP_QUANTITY;
    if (n == "k8s.io.apimachinery.pkg.util.intstr.IntOrString") return SP_INTORSTR;
    if (n == "k8s.io.apimachinery.pkg.runtime.RawExtension") return SP_RAWEXT;
    if (n == ax + "JSON") return SP_JSONRAW;
    if (n == ax + "JSONSchemaPropsOrBool") return SP_ORBOOL;
    if (n == ax + "JSONSchemaPropsOrArray") return SP_ORARRAY;
    if (n == ax + "JSONSchemaPropsOrStringArray") return SP_ORSTRARRAY;
    if (n == meta + "Verbs") return SP_SLICE;
    size_t d = n.rfind('.');
    if (d != std::string::npos && n.compare(d + 1, std::string::npos, "ExtraValue") == 0 && n.compare(0, 11, "k8s.io.api.") == 0)
      return SP_SLICE;
    return SP_NONE;
  }

  bool load(const std::string& path) {
    std::ifstream f(path);
    if (!f) { error = "cannot open " + path; return false; }
    std::stringstream ss;
    ss << f.rdbuf();
    std::string txt = ss.str();
    JReader r{txt.data(), txt.data() + txt.size()};
    JV root = r.val();
    if (!r.ok || root.t != JV::OBJ) { error = "malformed schema JSON"; return false; }
    const JV* messages = nullptr;
    const JV* kinds_j = nullptr;
    for (auto& kv : root.o) {
      if (kv.first == "messages") messages = &kv.second;
      if (kv.first == "kinds") kinds_j = &kv.second;
    }
    if (!messages || messages->t != JV::OBJ) { error = "schema has no messages"; return false; }
    for (auto& kv : messages->o) {
      by_name[kv.first] = (int)msgs.size();
      Message m;
      m.name = kv.first;
      msgs.push_back(std::move(m));
    }
    size_t mi = 0;
    for (auto& kv : messages->o) {
      Message& m = msgs[mi++];
      for (const JV& fj : kv.second.a) {
        if (fj.t != JV::ARR || fj.a.size() < 6) { error = "bad field in " + kv.first; return false; }
        Field fd;
        fd.json = fj.a[0].s;
        fd.num = (uint32_t)fj.a[1].n;
        const std::string& label = fj.a[2].s;
        fd.label = label == "rep" ? L_REP : (label == "map" ? L_MAP : L_OPT);
        bool sc;
        fd.type = scalar_of(fj.a[3].s, &sc);
        if (!sc) {
          auto it = by_name.find(fj.a[3].s);
          if (it == by_name.end()) { error = "unknown type " + fj.a[3].s; return false; }
          fd.msg = it->second;
          fd.sp = special_of(fj.a[3].s);
        }
        if (fd.label == L_MAP) {
          bool ks;
          fd.key = scalar_of(fj.a[4].s, &ks);
        }
        fd.inl = fj.a[5].b;
        fd.wt = fd.label == L_MAP ? 2 : (fd.type == S_BOOL || fd.type == S_INT32 || fd.type == S_INT64 ||
                                         fd.type == S_UINT32 || fd.type == S_UINT64) ? 0 : (fd.type == S_DOUBLE ? 1 : 2);
        m.fields.push_back(std::move(fd));
      }
      std::sort(m.fields.begin(), m.fields.end(), [](const Field& a, const Field& b) { return a.num < b.num; });
      uint32_t mx = m.fields.empty() ? 0 : m.fields.back().num;
      m.by_num.assign(mx + 1, -1);
      for (size_t i = 0; i < m.fields.size(); ++i) m.by_num[m.fields[i].num] = (int16_t)i;
    }
    // JSON keys (after every message is known: inline fields pull in their message's keys)
    for (size_t i = 0; i < msgs.size(); ++i) build_json((int)i, 0);
    for (auto& m : msgs)
      for (size_t i = 0; i < m.fields.size(); ++i)
        if (m.fields[i].json == "metadata" && m.fields[i].msg >= 0 && msgs[m.fields[i].msg].name == std::string(META) + "ObjectMeta")
          m.metadata = (int)i;
    auto sp = by_name.find(std::string(AXP) + "JSONSchemaProps");
    schema_props = sp == by_name.end() ? -1 : sp->second;
    if (kinds_j)
      for (auto& kv : kinds_j->o) {
        auto it = by_name.find(kv.second.s);
        if (it != by_name.end()) kinds[kv.first] = it->second;
      }
    static const char* const aliases[][2] = {
        {"policy/v1beta1/PodSecurityPolicy", "extensions/v1beta1/PodSecurityPolicy"},
        {"policy/v1beta1/PodSecurityPolicyList", "extensions/v1beta1/PodSecurityPolicyList"},
        {"storage.k8s.io/v1beta1/VolumeAttachment", "storage.k8s.io/v1alpha1/VolumeAttachment"},
        {"storage.k8s.io/v1beta1/VolumeAttachmentList", "storage.k8s.io/v1alpha1/VolumeAttachmentList"}};
    for (auto& a : aliases) {
      auto it = kinds.find(a[1]);
      if (it != kinds.end() && !kinds.count(a[0])) kinds[a[0]] = it->second;
    }
    return true;
  }

  void build_json(int mi, int depth) {
    Message& m = msgs[mi];
    if (!m.by_json.empty() || depth > 16) return;
    for (size_t i = 0; i < m.fields.size(); ++i) {
      const Field& f = m.fields[i];
      if (f.inl && f.msg >= 0) {
        build_json(f.msg, depth + 1);
        for (auto& kv : msgs[f.msg].by_json) m.by_json.emplace(kv.first, (int)i);
      } else {
        m.by_json.emplace(f.json, (int)i);
      }
    }
  }

  // "v1" + "Pod" -> core/v1 Pod; "apps/v1" + "Deployment"
  int message_for(const std::string& api_version, const std::string& kind) const {
    auto it = kinds.find(api_version + "/" + kind);
    return it == kinds.end() ? -1 : it->second;
  }
};

// ---------------------------------------------------------------------------------------------
// wire reading
struct Reader {
  const uint8_t* p;
  const uint8_t* e;
  bool ok = true;
  bool varint(uint64_t* v) {
    uint64_t r = 0;
    int shift = 0;
    while (p < e) {
      uint8_t b = *p++;
      r |= (uint64_t)(b & 0x7F) << shift;
      if (!(b & 0x80)) { *v = r; return true; }
      shift += 7;
      if (shift > 63) break;
    }
    return ok = false;
  }
  // next field: number, wire type, varint value or [ptr, len)
  bool next(uint32_t* num, uint8_t* wt, uint64_t* v, const uint8_t** ptr, size_t* len) {
    // every output is defined whatever the wire type: a caller that reads [ptr, len) of a varint
    // field, or v of a length-delimited one, sees an empty value, never stale stack memory
    *v = 0;
    *ptr = (const uint8_t*)"";
    *len = 0;
    uint64_t k;
    if (!varint(&k)) return false;
    *num = (uint32_t)(k >> 3);
    *wt = (uint8_t)(k & 7);
    switch (*wt) {
      case 0: return varint(v);
      case 1:
        if (e - p < 8) return ok = false;
        *ptr = p; *len = 8; p += 8; return true;
      case 5:
        if (e - p < 4) return ok = false;
        *ptr = p; *len = 4; p += 4; return true;
      case 2: {
        uint64_t l;
        if (!varint(&l) || (uint64_t)(e - p) < l) return ok = false;
        *ptr = p; *len = (size_t)l; p += l; return true;
      }
    }
    return ok = false;
  }
  bool done() const { return p >= e; }
};

// wire type a scalar (or message) value is encoded with
inline uint8_t wire_of(Scalar t) {
  return (t == S_BOOL || t == S_INT32 || t == S_INT64 || t == S_UINT32 || t == S_UINT64) ? 0 : (t == S_DOUBLE ? 1 : 2);
}

// does an occurrence with wire type `wt` fit field f? A repeated varint/double field may also
// arrive packed (one length-delimited run of values).
inline bool wire_ok(const Field& f, uint8_t wt) {
  if (wt == f.wt) return true;
  return f.label == L_REP && wt == 2 && f.wt != 2;
}

// nesting bound for untrusted input (recursive message types: JSONSchemaProps, ...)
constexpr int kMaxDepth = 100;
struct DepthGuard {
  int& d;
  bool ok;
  explicit DepthGuard(int& depth) : d(depth), ok(++depth <= kMaxDepth) {}
  ~DepthGuard() { --d; }
};

// ---------------------------------------------------------------------------------------------
// text helpers shared by both decoders
inline void json_escape(std::string& out, const char* s, size_t n) {
  out += '"';
  for (size_t i = 0; i < n; ++i) {
    unsigned char c = (unsigned char)s[i];
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          snprintf(buf, sizeof buf, "\\u%04x", c);
          out += buf;
        } else {
          out += (char)c;
        }
    }
  }
  out += '"';
}

inline std::string format_time(int64_t sec, int64_t nanos, bool micro) {
  time_t t = (time_t)sec;
  struct tm tmv;
  gmtime_r(&t, &tmv);
  char buf[64];
  if (micro)
    snprintf(buf, sizeof buf, "%04d-%02d-%02dT%02d:%02d:%02d.%06dZ", tmv.tm_year + 1900, tmv.tm_mon + 1, tmv.tm_mday,
             tmv.tm_hour, tmv.tm_min, tmv.tm_sec, (int)(nanos / 1000));
  else
    snprintf(buf, sizeof buf, "%04d-%02d-%02dT%02d:%02d:%02dZ", tmv.tm_year + 1900, tmv.tm_mon + 1, tmv.tm_mday,
             tmv.tm_hour, tmv.tm_min, tmv.tm_sec);
  return buf;
}

// Go's time.Duration.String()
inline std::string format_duration(int64_t d) {
  char buf[32];
  int w = sizeof buf;
  uint64_t u = d < 0 ? (uint64_t)(-(d + 1)) + 1 : (uint64_t)d;
  bool neg = d < 0;
  auto fmt_frac = [&](uint64_t v, int prec) {
    bool print = false;
    for (int i = 0; i < prec; ++i) {
      int digit = (int)(v % 10);
      print = print || digit != 0;
      if (print) buf[--w] = (char)(digit + '0');
      v /= 10;
    }
    if (print) buf[--w] = '.';
    return v;
  };
  auto fmt_int = [&](uint64_t v) {
    if (v == 0) { buf[--w] = '0'; return; }
    while (v > 0) { buf[--w] = (char)(v % 10 + '0'); v /= 10; }
  };
  if (u < 1000000000ULL) {
    int prec = 0;
    --w;
    buf[w] = 's';
    --w;
    if (u == 0) return "0s";
    if (u < 1000ULL) { prec = 0; buf[w] = 'n'; }
    else if (u < 1000000ULL) {
      prec = 3;
      // "µs": U+00B5 in UTF-8
      --w;
      buf[w + 1] = (char)0xB5;
      buf[w] = (char)0xC2;
    } else { prec = 6; buf[w] = 'm'; }
    u = fmt_frac(u, prec);
    fmt_int(u);
  } else {
    buf[--w] = 's';
    u = fmt_frac(u, 9);
    fmt_int(u % 60);
    u /= 60;
    if (u > 0) {
      buf[--w] = 'm';
      fmt_int(u % 60);
      u /= 60;
      if (u > 0) { buf[--w] = 'h'; fmt_int(u); }
    }
  }
  if (neg) buf[--w] = '-';
  return std::string(buf + w, sizeof buf - w);
}

inline void base64(std::string& out, const uint8_t* p, size_t n) {
  static const char t[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  size_t i = 0;
  for (; i + 2 < n; i += 3) {
    uint32_t v = (uint32_t)p[i] << 16 | (uint32_t)p[i + 1] << 8 | p[i + 2];
    out += t[v >> 18]; out += t[(v >> 12) & 63]; out += t[(v >> 6) & 63]; out += t[v & 63];
  }
  if (i + 1 == n) {
    uint32_t v = (uint32_t)p[i] << 16;
    out += t[v >> 18]; out += t[(v >> 12) & 63]; out += "==";
  } else if (i + 2 == n) {
    uint32_t v = (uint32_t)p[i] << 16 | (uint32_t)p[i + 1] << 8;
    out += t[v >> 18]; out += t[(v >> 12) & 63]; out += t[(v >> 6) & 63]; out += '=';
  }
}

inline std::string format_double(double d) {
  char buf[64];
  for (int prec = 1; prec <= 17; ++prec) {
    snprintf(buf, sizeof buf, "%.*g", prec, d);
    if (strtod(buf, nullptr) == d) break;
  }
  std::string s(buf);
  if (s.find_first_of(".eEn") == std::string::npos) s += ".0";   // Python repr: 1.0
  return s;
}

// ---------------------------------------------------------------------------------------------
// protobuf -> JSON text
class JsonWriter {
 public:
  explicit JsonWriter(const Schema& s) : s_(s) {}

  // body of message mi as a JSON object; inject_rv (non-null) replaces metadata.resourceVersion
  bool message(int mi, const uint8_t* p, size_t n, std::string& out, const char* inject_rv = nullptr) {
    DepthGuard g(depth_);
    if (!g.ok) return false;
    out += '{';
    bool first = true;
    if (!members(mi, p, n, out, first, inject_rv)) return false;
    out += '}';
    return true;
  }

  // the whole `k8s\0` envelope -> {"kind":...,"apiVersion":...,<object fields>}
  // canon: kind -> apiVersion to report (an object stored in another version of its type, e.g.
  // an HPA with v2beta1 metrics, is served in its canonical version)
  bool object(const uint8_t* p, size_t n, std::string& out, const char* inject_rv,
              const std::unordered_map<std::string, std::string>* canon = nullptr) {
    if (n < 4 || memcmp(p, "k8s\0", 4) != 0) return false;
    Reader r{p + 4, p + n};
    std::string av, kind;
    const uint8_t* raw = nullptr;
    size_t raw_n = 0;
    uint32_t num; uint8_t wt; uint64_t v; const uint8_t* q; size_t l;
    while (!r.done()) {
      if (!r.next(&num, &wt, &v, &q, &l)) return false;
      if (num == 1 && wt == 2) {
        Reader t{q, q + l};
        uint32_t n2; uint8_t w2; uint64_t v2; const uint8_t* q2; size_t l2;
        while (!t.done()) {
          if (!t.next(&n2, &w2, &v2, &q2, &l2)) return false;
          if (n2 == 1 && w2 == 2) av.assign((const char*)q2, l2);
          else if (n2 == 2 && w2 == 2) kind.assign((const char*)q2, l2);
        }
      } else if (num == 2 && wt == 2) {
        raw = q;
        raw_n = l;
      }
    }
    int mi = s_.message_for(av, kind);
    if (mi < 0) return false;
    out += "{\"kind\":";
    json_escape(out, kind.data(), kind.size());
    out += ",\"apiVersion\":";
    const std::string* shown = &av;
    if (canon) {
      auto it = canon->find(kind);
      if (it != canon->end()) shown = &it->second;
    }
    json_escape(out, shown->data(), shown->size());
    bool first = false;
    if (!members(mi, raw ? raw : (const uint8_t*)"", raw_n, out, first, inject_rv)) return false;
    out += '}';
    return true;
  }

 private:
  const Schema& s_;
  int depth_ = 0;
  struct Occ { int16_t fi; uint8_t wt; uint64_t v; const uint8_t* p; size_t n; };

  void key(std::string& out, bool& first, const std::string& k) {
    if (!first) out += ',';
    first = false;
    json_escape(out, k.data(), k.size());
    out += ':';
  }

  bool members(int mi, const uint8_t* p, size_t n, std::string& out, bool& first, const char* inject_rv) {
    const Message& m = s_.msgs[mi];
    std::vector<Occ> occ;
    occ.reserve(16);
    Reader r{p, p + n};
    uint32_t num; uint8_t wt; uint64_t v; const uint8_t* q; size_t l;
    while (!r.done()) {
      if (!r.next(&num, &wt, &v, &q, &l)) return false;
      if (num >= m.by_num.size() || m.by_num[num] < 0) continue;   // unknown field: skipped
      if (!wire_ok(m.fields[m.by_num[num]], wt)) return false;     // wrong wire type: corrupt
      occ.push_back(Occ{m.by_num[num], wt, v, q, l});
    }
    std::stable_sort(occ.begin(), occ.end(), [](const Occ& a, const Occ& b) { return a.fi < b.fi; });
    bool rv_done = inject_rv == nullptr || m.metadata >= 0;   // only ObjectMeta injects
    bool in_meta = false;
    (void)in_meta;
    size_t i = 0;
    for (size_t fi = 0; fi < m.fields.size(); ++fi) {
      const Field& f = m.fields[fi];
      size_t j = i;
      while (j < occ.size() && occ[j].fi == (int16_t)fi) ++j;
      bool is_rv_slot = !rv_done && f.json == "resourceVersion";
      if (is_rv_slot) {
        key(out, first, f.json);
        json_escape(out, inject_rv, strlen(inject_rv));
        rv_done = true;
        i = j;
        continue;
      }
      if (j == i) continue;
      if (f.inl) {
        DepthGuard g(depth_);
        if (!g.ok) return false;
        for (size_t k = i; k < j; ++k)
          if (!members(f.msg, occ[k].p, occ[k].n, out, first, nullptr)) return false;
        i = j;
        continue;
      }
      key(out, first, f.json);
      const char* sub_rv = (m.metadata == (int)fi) ? inject_rv : nullptr;
      if (f.label == L_REP) {
        out += '[';
        bool firstel = true;
        for (size_t k = i; k < j; ++k) {
          if (occ[k].wt == 2 && f.wt != 2) {   // packed run of scalars
            if (!packed(f, occ[k], out, firstel)) return false;
            continue;
          }
          if (!firstel) out += ',';
          firstel = false;
          if (!value(f, occ[k], out, nullptr)) return false;
        }
        out += ']';
      } else if (f.label == L_MAP) {
        out += '{';
        for (size_t k = i; k < j; ++k) {
          if (k > i) out += ',';
          if (!map_entry(f, occ[k].p, occ[k].n, out)) return false;
        }
        out += '}';
      } else {
        if (!value(f, occ[j - 1], out, sub_rv)) return false;   // last occurrence wins
      }
      i = j;
    }
    if (!rv_done) {   // ObjectMeta without the field number (never: resourceVersion = 6)
      key(out, first, "resourceVersion");
      json_escape(out, inject_rv, strlen(inject_rv));
    }
    return true;
  }

  bool packed(const Field& f, const Occ& o, std::string& out, bool& first) {
    Reader r{o.p, o.p + o.n};
    while (!r.done()) {
      Occ e{o.fi, f.wt, 0, (const uint8_t*)"", 0};
      if (f.wt == 0) {
        if (!r.varint(&e.v)) return false;
      } else {
        if (r.e - r.p < 8) return false;
        e.p = r.p; e.n = 8; r.p += 8;
      }
      if (!first) out += ',';
      first = false;
      if (!value(f, e, out, nullptr)) return false;
    }
    return true;
  }

  bool map_entry(const Field& f, const uint8_t* p, size_t n, std::string& out) {
    Reader r{p, p + n};
    std::string k;
    const uint8_t kwt = wire_of(f.key), vwt = f.type == S_MSG ? 2 : wire_of(f.type);
    Occ val{0, vwt, 0, (const uint8_t*)"", 0};
    bool have = false;
    uint32_t num; uint8_t wt; uint64_t v; const uint8_t* q; size_t l;
    while (!r.done()) {
      if (!r.next(&num, &wt, &v, &q, &l)) return false;
      if ((num == 1 && wt != kwt) || (num == 2 && wt != vwt)) return false;
      if (num == 1) {
        if (wt == 2) k.assign((const char*)q, l);
        else k = std::to_string(f.key == S_INT32 ? (int64_t)(int32_t)v : (int64_t)v);
      } else if (num == 2) {
        val = Occ{0, wt, v, q, l};
        have = true;
      }
    }
    json_escape(out, k.data(), k.size());
    out += ':';
    if (!have && f.type == S_MSG) { val.p = (const uint8_t*)""; val.n = 0; }
    Field vf = f;
    vf.label = L_OPT;
    return value(vf, val, out, nullptr);
  }

  bool value(const Field& f, const Occ& o, std::string& out, const char* inject_rv) {
    if (o.wt != (f.type == S_MSG ? 2 : wire_of(f.type))) return false;
    switch (f.type) {
      case S_STRING: json_escape(out, (const char*)o.p, o.n); return true;
      case S_BYTES: out += '"'; base64(out, o.p, o.n); out += '"'; return true;
      case S_BOOL: out += o.v ? "true" : "false"; return true;
      case S_INT32: out += std::to_string((int64_t)(int32_t)(uint32_t)o.v); return true;
      case S_INT64: out += std::to_string((int64_t)o.v); return true;
      case S_UINT32: case S_UINT64: out += std::to_string(o.v); return true;
      case S_DOUBLE: {
        if (o.n != 8) return false;
        double d;
        memcpy(&d, o.p, 8);
        out += format_double(d);
        return true;
      }
      case S_MSG: break;
    }
    if (f.sp == SP_NONE) return message(f.msg, o.p, o.n, out, inject_rv);
    return special(f.sp, o.p, o.n, out);
  }

  bool special(Special sp, const uint8_t* p, size_t n, std::string& out) {
    DepthGuard g(depth_);
    if (!g.ok) return false;
    Reader r{p, p + n};
    uint32_t num; uint8_t wt; uint64_t v; const uint8_t* q; size_t l;
    switch (sp) {
      case SP_TIME: case SP_MICROTIME: {
        int64_t sec = 0, nanos = 0;
        while (!r.done()) {
          if (!r.next(&num, &wt, &v, &q, &l)) return false;
          if (num == 1) sec = (int64_t)v;
          else if (num == 2) nanos = (int64_t)v;
        }
        std::string t = format_time(sec, nanos, sp == SP_MICROTIME);
        json_escape(out, t.data(), t.size());
        return true;
      }
      case SP_QUANTITY: {
        std::string s = "0";
        while (!r.done()) {
          if (!r.next(&num, &wt, &v, &q, &l)) return false;
          if (num == 1 && wt == 2) s.assign((const char*)q, l);
        }
        json_escape(out, s.data(), s.size());
        return true;
      }
      case SP_INTORSTR: {
        uint64_t typ = 0;
        int64_t iv = 0;
        std::string sv;
        while (!r.done()) {
          if (!r.next(&num, &wt, &v, &q, &l)) return false;
          if (num == 1) typ = v;
          else if (num == 2) iv = (int64_t)(int32_t)(uint32_t)v;
          else if (num == 3 && wt == 2) sv.assign((const char*)q, l);
        }
        if (typ == 0) out += std::to_string(iv);
        else json_escape(out, sv.data(), sv.size());
        return true;
      }
      case SP_DURATION: {
        int64_t d = 0;
        while (!r.done()) {
          if (!r.next(&num, &wt, &v, &q, &l)) return false;
          if (num == 1) d = (int64_t)v;
        }
        std::string s = format_duration(d);
        json_escape(out, s.data(), s.size());
        return true;
      }
      case SP_RAWEXT: case SP_JSONRAW: {
        const uint8_t* raw = nullptr;
        size_t rn = 0;
        while (!r.done()) {
          if (!r.next(&num, &wt, &v, &q, &l)) return false;
          if (num == 1 && wt == 2) { raw = q; rn = l; }
        }
        if (!raw || rn == 0) out += "null";
        else out.append((const char*)raw, rn);   // stored as JSON text
        return true;
      }
      case SP_SLICE: {
        out += '[';
        bool first = true;
        while (!r.done()) {
          if (!r.next(&num, &wt, &v, &q, &l)) return false;
          if (num == 1 && wt == 2) {
            if (!first) out += ',';
            first = false;
            json_escape(out, (const char*)q, l);
          }
        }
        out += ']';
        return true;
      }
      case SP_ORBOOL: {
        bool allows = false;
        const uint8_t* sch = nullptr;
        size_t sn = 0;
        while (!r.done()) {
          if (!r.next(&num, &wt, &v, &q, &l)) return false;
          if (num == 1) allows = v != 0;
          else if (num == 2 && wt == 2) { sch = q; sn = l; }
        }
        if (sch) return message(s_.schema_props, sch, sn, out);
        out += allows ? "true" : "false";
        return true;
      }
      case SP_ORARRAY: case SP_ORSTRARRAY: {
        const uint8_t* sch = nullptr;
        size_t sn = 0;
        std::vector<std::pair<const uint8_t*, size_t>> arr;
        while (!r.done()) {
          if (!r.next(&num, &wt, &v, &q, &l)) return false;
          if (num == 1 && wt == 2) { sch = q; sn = l; }
          else if (num == 2 && wt == 2) arr.emplace_back(q, l);
        }
        if (sch) return message(s_.schema_props, sch, sn, out);
        out += '[';
        for (size_t k = 0; k < arr.size(); ++k) {
          if (k) out += ',';
          if (sp == SP_ORARRAY) {
            if (!message(s_.schema_props, arr[k].first, arr[k].second, out)) return false;
          } else {
            json_escape(out, (const char*)arr[k].first, arr[k].second);
          }
        }
        out += ']';
        return true;
      }
      case SP_NONE: break;
    }
    return false;
  }
};

// ---------------------------------------------------------------------------------------------
// Protobuf watch streams (`application/vnd.kubernetes.protobuf;stream=watch`): apimachinery's
// RawSerializer + LengthDelimitedFramer (`runtime/serializer/protobuf/protobuf.go:436`,
// `endpoints/handlers/watch.go:166-226`). A frame is a 4-byte big-endian length followed by
// metav1.WatchEvent{1: type, 2: RawExtension{1: raw}}, raw = the object in the embedded
// (`k8s\0` envelope) encoding. etcd3 stores objects without their resourceVersion, so the
// envelope is rewritten with ObjectMeta.resourceVersion (field 6) = the revision.
inline void pb_put_varint(std::string& o, uint64_t v) {
  while (v >= 0x80) {
    o += (char)((v & 0x7F) | 0x80);
    v >>= 7;
  }
  o += (char)v;
}

inline void pb_put_ld(std::string& o, uint32_t num, const void* p, size_t n) {
  pb_put_varint(o, ((uint64_t)num << 3) | 2);
  pb_put_varint(o, n);
  o.append((const char*)p, n);
}

// `k8s\0` envelope -> the same envelope with metadata.resourceVersion = rv. False when the
// value is not an envelope of a kind in the schema.
inline bool envelope_with_rv(const Schema& s, const uint8_t* p, size_t n, const char* rv, std::string& out) {
  if (n < 4 || memcmp(p, "k8s\0", 4) != 0) return false;
  Reader r{p + 4, p + n};
  std::string av, kind;
  const uint8_t *tm = nullptr, *raw = nullptr;
  size_t tm_n = 0, raw_n = 0;
  std::string tail;   // contentEncoding / contentType, kept as they were
  uint32_t num; uint8_t wt; uint64_t v; const uint8_t* q; size_t l;
  while (!r.done()) {
    if (!r.next(&num, &wt, &v, &q, &l)) return false;
    if (num == 1 && wt == 2) {
      tm = q; tm_n = l;
      Reader t{q, q + l};
      uint32_t n2; uint8_t w2; uint64_t v2; const uint8_t* q2; size_t l2;
      while (!t.done()) {
        if (!t.next(&n2, &w2, &v2, &q2, &l2)) return false;
        if (n2 == 1 && w2 == 2) av.assign((const char*)q2, l2);
        else if (n2 == 2 && w2 == 2) kind.assign((const char*)q2, l2);
      }
    } else if (num == 2 && wt == 2) {
      raw = q; raw_n = l;
    } else if (wt == 2) {
      pb_put_ld(tail, num, q, l);
    }
  }
  int mi = s.message_for(av, kind);
  if (mi < 0) return false;
  const Message& m = s.msgs[mi];
  uint32_t meta_num = m.metadata >= 0 ? m.fields[m.metadata].num : 0;
  size_t rvn = strlen(rv);
  std::string body;
  body.reserve(raw_n + rvn + 16);
  bool had_meta = false;
  const uint8_t* rb = raw ? raw : p + n;      // an empty range when the envelope has no raw field
  Reader b{rb, rb + raw_n};
  const uint8_t* last = b.p;
  while (!b.done()) {
    const uint8_t* start = b.p;
    if (!b.next(&num, &wt, &v, &q, &l)) return false;
    if (meta_num && num == meta_num && wt == 2 && !had_meta) {
      body.append((const char*)last, (size_t)(start - last));
      std::string meta;
      meta.reserve(l + rvn + 4);
      Reader mr{q, q + l};
      const uint8_t* mlast = mr.p;
      uint32_t n3; uint8_t w3; uint64_t v3; const uint8_t* q3; size_t l3;
      while (!mr.done()) {
        const uint8_t* ms = mr.p;
        if (!mr.next(&n3, &w3, &v3, &q3, &l3)) return false;
        if (n3 == 6) {               // drop any stored resourceVersion
          meta.append((const char*)mlast, (size_t)(ms - mlast));
          mlast = mr.p;
        }
      }
      meta.append((const char*)mlast, (size_t)(mr.p - mlast));
      pb_put_ld(meta, 6, rv, rvn);
      pb_put_ld(body, meta_num, meta.data(), meta.size());
      had_meta = true;
      last = b.p;
    }
  }
  body.append((const char*)last, (size_t)(b.p - last));
  if (meta_num && !had_meta) {
    std::string meta;
    pb_put_ld(meta, 6, rv, rvn);
    pb_put_ld(body, meta_num, meta.data(), meta.size());
  }
  out.assign("k8s\0", 4);
  if (tm) pb_put_ld(out, 1, tm, tm_n);
  pb_put_ld(out, 2, body.data(), body.size());
  out += tail;
  return true;
}

// one length-delimited WatchEvent frame carrying `raw` (an envelope, or JSON bytes for values
// this schema cannot express — clients decode by the `k8s\0` magic)
inline void watch_event_frame(std::string& out, const char* type, const void* raw, size_t raw_n) {
  std::string ext;
  ext.reserve(raw_n + 8);
  pb_put_ld(ext, 1, raw, raw_n);
  std::string ev;
  ev.reserve(ext.size() + 24);
  pb_put_ld(ev, 1, type, strlen(type));
  pb_put_ld(ev, 2, ext.data(), ext.size());
  uint32_t n = (uint32_t)ev.size();
  char hdr[4] = {(char)(n >> 24), (char)(n >> 16), (char)(n >> 8), (char)n};
  out.append(hdr, 4);
  out += ev;
}

}  // namespace pbc
