// _kamd_pbcodec — CPython extension: the native Kubernetes protobuf codec for the API server's
// etcd storage format (see pb_codec.h and kubernetes_amd/api/protobuf.py, the pure-Python
// reference implementation it must agree with byte for byte).
//
//   c = _kamd_pbcodec.Codec(schema_path, error_class, json_dumps, json_loads)
//   c.encode_object(obj, message) -> bytes         k8s\0 envelope; apiVersion/kind from obj
//   c.decode_object(data) -> dict                   envelope -> JSON-form dict (kind, apiVersion first)
//   c.encode_message(message, obj) / c.decode_message(message, data)
//   c.to_json(data, resource_version=None) -> bytes envelope -> JSON text, metadata.resourceVersion injected
//   c.message_for(api_version, kind) -> str | None
//
// Encoding is lossless or an error: a JSON key that is not a field of the message (or of an
// inline-embedded one) raises error_class("<json path>: field ... is not part of ..."); a value
// of the wrong JSON type raises too. `kind` / `apiVersion` keys are TypeMeta (no protobuf tag in
// Go) and are skipped inside messages.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include "pb_codec.h"

namespace {

using pbc::Field;
using pbc::Message;
using pbc::Schema;

// Decode caches (all touched under the GIL only). Watch streams decode the same few hundred
// short strings (namespaces, node names, phases, condition types, images, quantities) and the
// same timestamps over and over: a hit hands back a new reference to the existing str instead
// of allocating and UTF-8-decoding another one.
struct StrSlot {
  uint64_t h = 0;
  uint32_t n = 0;
  char b[32];
  PyObject* o = nullptr;
};
struct TimeSlot {
  int64_t sec = 0, nanos = -1;
  bool micro = false;
  PyObject* o = nullptr;
};
constexpr size_t kStrSlots = 4096, kTimeSlots = 256;

struct CodecObject {
  PyObject_HEAD
  Schema* schema;
  PyObject* error;   // exception class
  PyObject* dumps;   // json.dumps(obj) -> str (RawExtension / JSON values)
  PyObject* loads;   // json.loads(bytes) -> object
  std::unordered_map<std::string, std::string>* canon;   // kind -> served apiVersion
  std::vector<std::vector<PyObject*>>* keys;              // [message][field] -> interned JSON key
  StrSlot* strs;
  TimeSlot* times;
};

void clear_caches(CodecObject* self) {
  if (self->keys) {
    for (auto& v : *self->keys)
      for (PyObject* o : v) Py_XDECREF(o);
    delete self->keys;
    self->keys = nullptr;
  }
  if (self->strs) {
    for (size_t i = 0; i < kStrSlots; ++i) Py_XDECREF(self->strs[i].o);
    delete[] self->strs;
    self->strs = nullptr;
  }
  if (self->times) {
    for (size_t i = 0; i < kTimeSlots; ++i) Py_XDECREF(self->times[i].o);
    delete[] self->times;
    self->times = nullptr;
  }
}

void init_caches(CodecObject* self) {
  clear_caches(self);
  self->keys = new std::vector<std::vector<PyObject*>>(self->schema->msgs.size());
  for (size_t mi = 0; mi < self->schema->msgs.size(); ++mi) {
    auto& fs = self->schema->msgs[mi].fields;
    auto& ks = (*self->keys)[mi];
    ks.resize(fs.size(), nullptr);
    for (size_t fi = 0; fi < fs.size(); ++fi) {
      PyObject* k = PyUnicode_FromStringAndSize(fs[fi].json.data(), (Py_ssize_t)fs[fi].json.size());
      if (k) PyUnicode_InternInPlace(&k);
      ks[fi] = k;
    }
  }
  self->strs = new StrSlot[kStrSlots];
  self->times = new TimeSlot[kTimeSlots];
}

// ---------------------------------------------------------------------------------------------
// wire writing
inline void put_varint(std::string& o, uint64_t v) {
  while (v >= 0x80) {
    o += (char)((v & 0x7F) | 0x80);
    v >>= 7;
  }
  o += (char)v;
}
inline void put_tag(std::string& o, uint32_t num, uint8_t wt) { put_varint(o, ((uint64_t)num << 3) | wt); }
inline void put_ld(std::string& o, uint32_t num, const char* p, size_t n) {
  put_tag(o, num, 2);
  put_varint(o, n);
  o.append(p, n);
}

// error with a JSON path built while unwinding
struct Err {
  bool set = false;
  std::string path, msg;
  void fail(const std::string& m) {
    if (!set) { set = true; msg = m; }
  }
  void prefix(const std::string& seg) {   // seg like ".spec" or "[3]" or "spec"
    if (path.empty() || path[0] == '[') path = seg + path;
    else path = seg + "." + path;
  }
};

struct Encoder {
  const Schema& s;
  CodecObject* self;
  Err err;

  bool utf8(PyObject* o, const char** p, Py_ssize_t* n) {
    *p = PyUnicode_AsUTF8AndSize(o, n);
    if (!*p) {
      PyErr_Clear();
      err.fail("invalid unicode string");
      return false;
    }
    return true;
  }

  static const char* type_name(PyObject* v) { return Py_TYPE(v)->tp_name; }

  bool integer(PyObject* v, int64_t* out) {
    if (PyBool_Check(v)) { err.fail("expected an integer, got bool"); return false; }
    if (PyLong_Check(v)) {
      int overflow = 0;
      long long x = PyLong_AsLongLongAndOverflow(v, &overflow);
      if (overflow) {
        unsigned long long u = PyLong_AsUnsignedLongLong(v);
        if (PyErr_Occurred()) { PyErr_Clear(); err.fail("integer out of range"); return false; }
        *out = (int64_t)u;
        return true;
      }
      *out = x;
      return true;
    }
    if (PyFloat_Check(v)) {
      double d = PyFloat_AS_DOUBLE(v);
      if (d == (double)(int64_t)d) { *out = (int64_t)d; return true; }
    }
    err.fail(std::string("expected an integer, got ") + type_name(v));
    return false;
  }

  bool scalar(const Field& f, uint32_t num, PyObject* v, std::string& o) {
    switch (f.type) {
      case pbc::S_STRING: {
        if (!PyUnicode_Check(v)) { err.fail(std::string("expected a string, got ") + type_name(v)); return false; }
        const char* p; Py_ssize_t n;
        if (!utf8(v, &p, &n)) return false;
        put_ld(o, num, p, (size_t)n);
        return true;
      }
      case pbc::S_BOOL:
        if (!PyBool_Check(v)) { err.fail(std::string("expected a boolean, got ") + type_name(v)); return false; }
        put_tag(o, num, 0);
        o += (char)(v == Py_True ? 1 : 0);
        return true;
      case pbc::S_INT32: case pbc::S_INT64: case pbc::S_UINT32: case pbc::S_UINT64: {
        int64_t x;
        if (!integer(v, &x)) return false;
        put_tag(o, num, 0);
        put_varint(o, (uint64_t)x);
        return true;
      }
      case pbc::S_DOUBLE: {
        double d;
        if (PyBool_Check(v) || !(PyFloat_Check(v) || PyLong_Check(v))) { err.fail("expected a number"); return false; }
        d = PyFloat_Check(v) ? PyFloat_AS_DOUBLE(v) : PyLong_AsDouble(v);
        put_tag(o, num, 1);
        o.append((const char*)&d, 8);
        return true;
      }
      case pbc::S_BYTES: {
        if (!PyUnicode_Check(v)) { err.fail("expected a base64 string"); return false; }
        const char* p; Py_ssize_t n;
        if (!utf8(v, &p, &n)) return false;
        std::string raw;
        if (!unbase64(p, (size_t)n, raw)) { err.fail("invalid base64"); return false; }
        put_ld(o, num, raw.data(), raw.size());
        return true;
      }
      case pbc::S_MSG: break;
    }
    err.fail("unsupported scalar");
    return false;
  }

  static bool unbase64(const char* p, size_t n, std::string& out) {
    auto val = [](char c) -> int {
      if (c >= 'A' && c <= 'Z') return c - 'A';
      if (c >= 'a' && c <= 'z') return c - 'a' + 26;
      if (c >= '0' && c <= '9') return c - '0' + 52;
      if (c == '+') return 62;
      if (c == '/') return 63;
      return -1;
    };
    if (n % 4) return false;
    for (size_t i = 0; i < n; i += 4) {
      int a = val(p[i]), b = val(p[i + 1]);
      int c = p[i + 2] == '=' ? -2 : val(p[i + 2]);
      int d = p[i + 3] == '=' ? -2 : val(p[i + 3]);
      if (a < 0 || b < 0 || c == -1 || d == -1 || (c == -2 && d != -2) || ((c == -2 || d == -2) && i + 4 != n)) return false;
      uint32_t v = (uint32_t)a << 18 | (uint32_t)b << 12 | (uint32_t)(c < 0 ? 0 : c) << 6 | (uint32_t)(d < 0 ? 0 : d);
      out += (char)(v >> 16);
      if (c >= 0) out += (char)((v >> 8) & 0xFF);
      if (d >= 0) out += (char)(v & 0xFF);
    }
    return true;
  }

  // RFC 3339 -> (seconds, nanos)
  bool parse_time(const char* p, size_t n, int64_t* sec, int64_t* nanos) {
    int y, mo, d, h, mi, se;
    if (n < 20 || sscanf(p, "%4d-%2d-%2d", &y, &mo, &d) != 3 || (p[10] != 'T' && p[10] != 't' && p[10] != ' ') ||
        sscanf(p + 11, "%2d:%2d:%2d", &h, &mi, &se) != 3 || p[4] != '-' || p[7] != '-' || p[13] != ':' || p[16] != ':') {
      err.fail("not an RFC 3339 time");
      return false;
    }
    size_t i = 19;
    int64_t frac = 0;
    int digits = 0;
    if (i < n && p[i] == '.') {
      ++i;
      while (i < n && p[i] >= '0' && p[i] <= '9') {
        if (digits < 9) { frac = frac * 10 + (p[i] - '0'); ++digits; }
        ++i;
      }
      while (digits < 9) { frac *= 10; ++digits; }
    }
    int64_t off = 0;
    if (i < n && (p[i] == 'Z' || p[i] == 'z')) {
      ++i;
    } else if (i + 6 == n && (p[i] == '+' || p[i] == '-')) {
      int oh, om;
      if (sscanf(p + i + 1, "%2d:%2d", &oh, &om) != 2) { err.fail("not an RFC 3339 time"); return false; }
      off = (p[i] == '+' ? 1 : -1) * (oh * 3600 + om * 60);
      i += 6;
    } else {
      err.fail("not an RFC 3339 time");
      return false;
    }
    if (i != n) { err.fail("not an RFC 3339 time"); return false; }
    struct tm tmv;
    memset(&tmv, 0, sizeof tmv);
    tmv.tm_year = y - 1900; tmv.tm_mon = mo - 1; tmv.tm_mday = d;
    tmv.tm_hour = h; tmv.tm_min = mi; tmv.tm_sec = se;
    *sec = (int64_t)timegm(&tmv) - off;
    *nanos = frac;
    return true;
  }

  bool parse_duration(const char* p, size_t n, int64_t* out) {
    std::string s(p, n);
    bool neg = false;
    size_t i = 0;
    if (i < s.size() && (s[i] == '-' || s[i] == '+')) { neg = s[i] == '-'; ++i; }
    if (s.substr(i) == "0") { *out = 0; return true; }
    if (i >= s.size()) { err.fail("not a duration"); return false; }
    long double total = 0;
    while (i < s.size()) {
      size_t j = i;
      while (j < s.size() && ((s[j] >= '0' && s[j] <= '9') || s[j] == '.')) ++j;
      if (j == i) { err.fail("not a duration"); return false; }
      long double num = strtold(s.substr(i, j - i).c_str(), nullptr);
      size_t k = j;
      while (k < s.size() && !((s[k] >= '0' && s[k] <= '9') || s[k] == '.')) ++k;
      std::string unit = s.substr(j, k - j);
      long double mult;
      if (unit == "ns") mult = 1;
      else if (unit == "us" || unit == "\xc2\xb5s") mult = 1e3;
      else if (unit == "ms") mult = 1e6;
      else if (unit == "s") mult = 1e9;
      else if (unit == "m") mult = 60e9;
      else if (unit == "h") mult = 3600e9;
      else { err.fail("not a duration"); return false; }
      total += num * mult;
      i = k;
    }
    *out = (int64_t)(neg ? -total : total + 0.5L) ;
    if (neg) *out = -(int64_t)(total + 0.5L);
    return true;
  }

  bool special(pbc::Special sp, PyObject* v, std::string& body) {
    switch (sp) {
      case pbc::SP_TIME: case pbc::SP_MICROTIME: {
        if (!PyUnicode_Check(v)) { err.fail("expected an RFC 3339 time string"); return false; }
        const char* p; Py_ssize_t n;
        if (!utf8(v, &p, &n)) return false;
        int64_t sec, nanos;
        if (!parse_time(p, (size_t)n, &sec, &nanos)) return false;
        if (sp == pbc::SP_TIME) nanos = 0;   // metav1.Time is second precision in JSON
        put_tag(body, 1, 0);
        put_varint(body, (uint64_t)sec);
        if (nanos) { put_tag(body, 2, 0); put_varint(body, (uint64_t)nanos); }
        return true;
      }
      case pbc::SP_QUANTITY: {
        PyObject* sv = nullptr;
        if (PyUnicode_Check(v)) { Py_INCREF(v); sv = v; }
        else if (PyBool_Check(v)) { err.fail("expected a quantity, got bool"); return false; }
        else if (PyLong_Check(v)) sv = PyObject_Str(v);
        else if (PyFloat_Check(v)) {
          double d = PyFloat_AS_DOUBLE(v);
          if (d == (double)(int64_t)d) {
            PyObject* iv = PyLong_FromLongLong((long long)d);
            sv = PyObject_Str(iv);
            Py_DECREF(iv);
          } else {
            sv = PyObject_Repr(v);
          }
        } else { err.fail(std::string("expected a quantity, got ") + type_name(v)); return false; }
        if (!sv) { PyErr_Clear(); err.fail("bad quantity"); return false; }
        const char* p; Py_ssize_t n;
        bool ok = utf8(sv, &p, &n);
        if (ok) put_ld(body, 1, p, (size_t)n);
        Py_DECREF(sv);
        return ok;
      }
      case pbc::SP_INTORSTR: {
        if (PyUnicode_Check(v)) {
          const char* p; Py_ssize_t n;
          if (!utf8(v, &p, &n)) return false;
          put_tag(body, 1, 0); put_varint(body, 1);
          put_tag(body, 2, 0); put_varint(body, 0);
          put_ld(body, 3, p, (size_t)n);
          return true;
        }
        if (PyLong_Check(v) && !PyBool_Check(v)) {
          int64_t x;
          if (!integer(v, &x)) return false;
          put_tag(body, 1, 0); put_varint(body, 0);
          put_tag(body, 2, 0); put_varint(body, (uint64_t)x);
          put_ld(body, 3, "", 0);
          return true;
        }
        err.fail(std::string("expected an int or a string, got ") + type_name(v));
        return false;
      }
      case pbc::SP_DURATION: {
        if (!PyUnicode_Check(v)) { err.fail("expected a duration string"); return false; }
        const char* p; Py_ssize_t n;
        if (!utf8(v, &p, &n)) return false;
        int64_t d;
        if (!parse_duration(p, (size_t)n, &d)) return false;
        put_tag(body, 1, 0);
        put_varint(body, (uint64_t)d);
        return true;
      }
      case pbc::SP_RAWEXT: case pbc::SP_JSONRAW: {
        PyObject* s = PyObject_CallFunctionObjArgs(self->dumps, v, nullptr);
        if (!s) { PyErr_Clear(); err.fail("value is not JSON-serializable"); return false; }
        const char* p; Py_ssize_t n;
        bool ok = utf8(s, &p, &n);
        if (ok) put_ld(body, 1, p, (size_t)n);
        Py_DECREF(s);
        return ok;
      }
      case pbc::SP_SLICE: {
        if (!PyList_Check(v)) { err.fail("expected a list of strings"); return false; }
        for (Py_ssize_t i = 0; i < PyList_GET_SIZE(v); ++i) {
          PyObject* x = PyList_GET_ITEM(v, i);
          if (!PyUnicode_Check(x)) { err.fail("expected a list of strings"); return false; }
          const char* p; Py_ssize_t n;
          if (!utf8(x, &p, &n)) return false;
          put_ld(body, 1, p, (size_t)n);
        }
        return true;
      }
      case pbc::SP_ORBOOL: {
        if (PyBool_Check(v)) { put_tag(body, 1, 0); body += (char)(v == Py_True); return true; }
        std::string sub;
        if (!message(s.schema_props, v, sub)) return false;
        put_tag(body, 1, 0); body += (char)1;
        put_ld(body, 2, sub.data(), sub.size());
        return true;
      }
      case pbc::SP_ORARRAY: case pbc::SP_ORSTRARRAY: {
        if (PyList_Check(v)) {
          for (Py_ssize_t i = 0; i < PyList_GET_SIZE(v); ++i) {
            PyObject* x = PyList_GET_ITEM(v, i);
            if (sp == pbc::SP_ORARRAY) {
              std::string sub;
              if (!message(s.schema_props, x, sub)) { err.prefix("[" + std::to_string(i) + "]"); return false; }
              put_ld(body, 2, sub.data(), sub.size());
            } else {
              PyObject* sx = PyObject_Str(x);
              const char* p; Py_ssize_t n;
              bool ok = sx && utf8(sx, &p, &n);
              if (ok) put_ld(body, 2, p, (size_t)n);
              Py_XDECREF(sx);
              if (!ok) return false;
            }
          }
          return true;
        }
        std::string sub;
        if (!message(s.schema_props, v, sub)) return false;
        put_ld(body, 1, sub.data(), sub.size());
        return true;
      }
      case pbc::SP_NONE: break;
    }
    err.fail("unsupported special type");
    return false;
  }

  bool value(const Field& f, uint32_t num, PyObject* v, std::string& o) {
    if (f.type != pbc::S_MSG) return scalar(f, num, v, o);
    std::string body;
    if (f.sp != pbc::SP_NONE) {
      if (!special(f.sp, v, body)) return false;
    } else {
      if (!PyDict_Check(v)) { err.fail(std::string("expected an object, got ") + type_name(v)); return false; }
      if (!message(f.msg, v, body)) return false;
    }
    put_ld(o, num, body.data(), body.size());
    return true;
  }

  bool map_entry(const Field& f, PyObject* k, PyObject* v, std::string& o) {
    std::string body;
    Field kf;
    kf.type = f.key;
    if (f.key == pbc::S_STRING) {
      if (!scalar(kf, 1, k, body)) return false;
    } else {
      PyObject* iv = PyNumber_Long(k);
      if (!iv) { PyErr_Clear(); err.fail("map key is not an integer"); return false; }
      bool ok = scalar(kf, 1, iv, body);
      Py_DECREF(iv);
      if (!ok) return false;
    }
    Field vf = f;
    vf.label = pbc::L_OPT;
    if (!value(vf, 2, v, body)) return false;
    put_ld(o, f.num, body.data(), body.size());
    return true;
  }

  // obj (dict) -> message body
  bool message(int mi, PyObject* obj, std::string& o) {
    if (mi < 0) { err.fail("no schema message"); return false; }
    if (!PyDict_Check(obj)) { err.fail(std::string("expected an object, got ") + type_name(obj)); return false; }
    const Message& m = s.msgs[mi];
    // field index -> value; inline fields collect their keys in a sub-dict
    struct Slot { int fi; PyObject* v; };
    Slot slots[64];
    std::vector<Slot> more;
    int ns = 0;
    std::vector<std::pair<int, PyObject*>> inl;   // (field index, owned dict)
    PyObject *k, *v;
    Py_ssize_t pos = 0;
    bool ok = true;
    while (PyDict_Next(obj, &pos, &k, &v)) {
      if (v == Py_None) continue;
      const char* kp; Py_ssize_t kn;
      if (!PyUnicode_Check(k) || !(kp = PyUnicode_AsUTF8AndSize(k, &kn))) {
        PyErr_Clear();
        err.fail("non-string key");
        ok = false;
        break;
      }
      auto it = m.by_json.find(std::string(kp, (size_t)kn));
      if (it == m.by_json.end()) {
        if ((kn == 4 && !memcmp(kp, "kind", 4)) || (kn == 10 && !memcmp(kp, "apiVersion", 10))) continue;
        std::string short_name = m.name.substr(m.name.rfind('.') + 1);
        err.fail("field '" + std::string(kp, (size_t)kn) + "' is not part of " + short_name + " in the API schema");
        err.path = std::string(kp, (size_t)kn);
        ok = false;
        break;
      }
      int fi = it->second;
      const Field& f = m.fields[fi];
      if (f.inl) {
        PyObject* d = nullptr;
        for (auto& x : inl)
          if (x.first == fi) d = x.second;
        if (!d) { d = PyDict_New(); inl.emplace_back(fi, d); }
        PyDict_SetItem(d, k, v);
        continue;
      }
      if (ns < 64) slots[ns++] = Slot{fi, v};
      else more.push_back(Slot{fi, v});
    }
    for (int i = 0; i < ns; ++i) more.push_back(slots[i]);
    for (auto& x : inl) more.push_back(Slot{x.first, x.second});
    std::sort(more.begin(), more.end(), [](const Slot& a, const Slot& b) { return a.fi < b.fi; });
    for (size_t si = 0; ok && si < more.size(); ++si) {
      const Field& f = m.fields[more[si].fi];
      PyObject* val = more[si].v;
      if (f.inl) {
        std::string sub;
        if (!message(f.msg, val, sub)) { ok = false; break; }
        put_ld(o, f.num, sub.data(), sub.size());
        continue;
      }
      if (f.label == pbc::L_REP) {
        if (!PyList_Check(val) && !PyTuple_Check(val)) {
          err.fail(std::string("expected a list, got ") + type_name(val));
          err.prefix(f.json);
          ok = false;
          break;
        }
        PyObject* seq = PySequence_Fast(val, "list");
        Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
        for (Py_ssize_t i = 0; i < n; ++i) {
          PyObject* x = PySequence_Fast_GET_ITEM(seq, i);
          if (x == Py_None) { err.fail("null list element"); }
          if (x == Py_None || !value(f, f.num, x, o)) {
            err.prefix("[" + std::to_string(i) + "]");
            err.prefix(f.json);
            ok = false;
            break;
          }
        }
        Py_DECREF(seq);
      } else if (f.label == pbc::L_MAP) {
        if (!PyDict_Check(val)) {
          err.fail(std::string("expected a map, got ") + type_name(val));
          err.prefix(f.json);
          ok = false;
          break;
        }
        std::vector<std::pair<std::string, std::pair<PyObject*, PyObject*>>> ents;
        PyObject *mk, *mv;
        Py_ssize_t mp = 0;
        while (PyDict_Next(val, &mp, &mk, &mv)) {
          const char* kp; Py_ssize_t kn;
          PyObject* ks = PyUnicode_Check(mk) ? (Py_INCREF(mk), mk) : PyObject_Str(mk);
          if (!ks || !(kp = PyUnicode_AsUTF8AndSize(ks, &kn))) { PyErr_Clear(); Py_XDECREF(ks); err.fail("bad map key"); ok = false; break; }
          ents.emplace_back(std::string(kp, (size_t)kn), std::make_pair(mk, mv));
          Py_DECREF(ks);
        }
        if (!ok) { err.prefix(f.json); break; }
        std::sort(ents.begin(), ents.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
        for (auto& e : ents) {
          if (e.second.second == Py_None) { err.fail("null map value"); }
          if (e.second.second == Py_None || !map_entry(f, e.second.first, e.second.second, o)) {
            err.prefix("[" + e.first + "]");
            err.prefix(f.json);
            ok = false;
            break;
          }
        }
      } else if (!value(f, f.num, val, o)) {
        err.prefix(f.json);
        ok = false;
      }
    }
    for (auto& x : inl) Py_DECREF(x.second);
    return ok;
  }
};

// ---------------------------------------------------------------------------------------------
// decode to Python objects
struct Decoder {
  const Schema& s;
  CodecObject* self;
  std::string err;
  int depth = 0;

  PyObject* str(const uint8_t* p, size_t n) {
    if (n == 0 || n > sizeof(StrSlot::b) || !self->strs)
      return PyUnicode_DecodeUTF8((const char*)p, (Py_ssize_t)n, "replace");
    uint64_t h = 1469598103934665603ull;           // FNV-1a
    for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
    StrSlot& e = self->strs[h & (kStrSlots - 1)];
    if (e.o && e.h == h && e.n == n && memcmp(e.b, p, n) == 0) {
      Py_INCREF(e.o);
      return e.o;
    }
    PyObject* o = PyUnicode_DecodeUTF8((const char*)p, (Py_ssize_t)n, "replace");
    if (!o) return nullptr;
    Py_XDECREF(e.o);
    Py_INCREF(o);
    e.o = o; e.h = h; e.n = (uint32_t)n;
    memcpy(e.b, p, n);
    return o;
  }

  PyObject* time_str(int64_t sec, int64_t nanos, bool micro) {
    if (!self->times) {
      std::string t = pbc::format_time(sec, nanos, micro);
      return PyUnicode_FromStringAndSize(t.data(), (Py_ssize_t)t.size());
    }
    uint64_t h = ((uint64_t)sec * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)nanos * 31) ^ (micro ? 1 : 0);
    TimeSlot& e = self->times[(h >> 7) & (kTimeSlots - 1)];
    if (e.o && e.sec == sec && e.nanos == nanos && e.micro == micro) {
      Py_INCREF(e.o);
      return e.o;
    }
    std::string t = pbc::format_time(sec, nanos, micro);
    PyObject* o = PyUnicode_FromStringAndSize(t.data(), (Py_ssize_t)t.size());
    if (!o) return nullptr;
    Py_XDECREF(e.o);
    Py_INCREF(o);
    e.o = o; e.sec = sec; e.nanos = nanos; e.micro = micro;
    return o;
  }

  PyObject* key_of(int mi, int fi, const Field& f) {
    if (self->keys) {
      PyObject* k = (*self->keys)[mi][fi];
      if (k) { Py_INCREF(k); return k; }
    }
    return PyUnicode_FromStringAndSize(f.json.data(), (Py_ssize_t)f.json.size());
  }

  PyObject* value(const Field& f, uint8_t wt, uint64_t v, const uint8_t* p, size_t n) {
    if (wt != (f.type == pbc::S_MSG ? 2 : pbc::wire_of(f.type))) {
      err = "wire type " + std::to_string(wt) + " does not match the field's type";
      return nullptr;
    }
    switch (f.type) {
      case pbc::S_STRING: return str(p, n);
      case pbc::S_BYTES: { std::string b; pbc::base64(b, p, n); return PyUnicode_FromStringAndSize(b.data(), (Py_ssize_t)b.size()); }
      case pbc::S_BOOL: return PyBool_FromLong(v != 0);
      case pbc::S_INT32: return PyLong_FromLongLong((long long)(int32_t)(uint32_t)v);
      case pbc::S_INT64: return PyLong_FromLongLong((long long)(int64_t)v);
      case pbc::S_UINT32: case pbc::S_UINT64: return PyLong_FromUnsignedLongLong(v);
      case pbc::S_DOUBLE: { double d = 0; if (n == 8) memcpy(&d, p, 8); return PyFloat_FromDouble(d); }
      case pbc::S_MSG: break;
    }
    if (f.sp == pbc::SP_NONE) {
      PyObject* d = PyDict_New();
      if (!message(f.msg, p, n, d)) { Py_DECREF(d); return nullptr; }
      return d;
    }
    return special(f.sp, p, n);
  }

  PyObject* special(pbc::Special sp, const uint8_t* p, size_t n) {
    pbc::DepthGuard g(depth);
    if (!g.ok) { err = "protobuf nesting too deep"; return nullptr; }
    // the JSON writer renders special types exactly as api/protobuf.py; reuse it, then parse the
    // (tiny) JSON text for the container-typed ones
    pbc::Reader r{p, p + n};
    uint32_t num; uint8_t wt; uint64_t v; const uint8_t* q; size_t l;
    switch (sp) {
      case pbc::SP_QUANTITY: {
        const uint8_t* sp_ = (const uint8_t*)"0";
        size_t sl = 1;
        while (!r.done()) {
          if (!r.next(&num, &wt, &v, &q, &l)) { err = "truncated"; return nullptr; }
          if (num == 1 && wt == 2) { sp_ = q; sl = l; }
        }
        return str(sp_, sl);
      }
      case pbc::SP_INTORSTR: {
        uint64_t typ = 0;
        int64_t iv = 0;
        const uint8_t* sv = (const uint8_t*)"";
        size_t sl = 0;
        while (!r.done()) {
          if (!r.next(&num, &wt, &v, &q, &l)) { err = "truncated"; return nullptr; }
          if (num == 1) typ = v;
          else if (num == 2) iv = (int64_t)(int32_t)(uint32_t)v;
          else if (num == 3 && wt == 2) { sv = q; sl = l; }
        }
        return typ == 0 ? PyLong_FromLongLong(iv) : str(sv, sl);
      }
      case pbc::SP_TIME: case pbc::SP_MICROTIME: {
        int64_t sec = 0, nanos = 0;
        while (!r.done()) {
          if (!r.next(&num, &wt, &v, &q, &l)) { err = "truncated"; return nullptr; }
          if (num == 1) sec = (int64_t)v;
          else if (num == 2) nanos = (int64_t)v;
        }
        return time_str(sec, nanos, sp == pbc::SP_MICROTIME);
      }
      case pbc::SP_DURATION: {
        int64_t d = 0;
        while (!r.done()) {
          if (!r.next(&num, &wt, &v, &q, &l)) { err = "truncated"; return nullptr; }
          if (num == 1) d = (int64_t)v;
        }
        std::string t = pbc::format_duration(d);
        return PyUnicode_FromStringAndSize(t.data(), (Py_ssize_t)t.size());
      }
      case pbc::SP_SLICE: {
        PyObject* lst = PyList_New(0);
        while (!r.done()) {
          if (!r.next(&num, &wt, &v, &q, &l)) { Py_DECREF(lst); err = "truncated"; return nullptr; }
          if (num == 1 && wt == 2) {
            PyObject* x = str(q, l);
            PyList_Append(lst, x);
            Py_DECREF(x);
          }
        }
        return lst;
      }
      default: {
        // RawExtension / JSON / JSONSchemaPropsOr*: rendered as JSON text, then json.loads
        std::string text;
        if (!render_special(sp, p, n, text)) { err = "bad special value"; return nullptr; }
        PyObject* b = PyBytes_FromStringAndSize(text.data(), (Py_ssize_t)text.size());
        PyObject* o = PyObject_CallFunctionObjArgs(self->loads, b, nullptr);
        Py_DECREF(b);
        if (!o) { PyErr_Clear(); err = "stored JSON value does not parse"; }
        return o;
      }
    }
  }

  bool render_special(pbc::Special sp, const uint8_t* p, size_t n, std::string& out) {
    pbc::Reader r{p, p + n};
    uint32_t num; uint8_t wt; uint64_t v; const uint8_t* q; size_t l;
    pbc::JsonWriter jw(s);
    switch (sp) {
      case pbc::SP_RAWEXT: case pbc::SP_JSONRAW: {
        const uint8_t* raw = nullptr;
        size_t rn = 0;
        while (!r.done()) {
          if (!r.next(&num, &wt, &v, &q, &l)) return false;
          if (num == 1 && wt == 2) { raw = q; rn = l; }
        }
        if (!raw || rn == 0) out = "null";
        else out.assign((const char*)raw, rn);
        return true;
      }
      case pbc::SP_ORBOOL: {
        bool allows = false;
        const uint8_t* sch = nullptr;
        size_t sn = 0;
        while (!r.done()) {
          if (!r.next(&num, &wt, &v, &q, &l)) return false;
          if (num == 1) allows = v != 0;
          else if (num == 2 && wt == 2) { sch = q; sn = l; }
        }
        if (sch) return jw.message(s.schema_props, sch, sn, out);
        out = allows ? "true" : "false";
        return true;
      }
      case pbc::SP_ORARRAY: case pbc::SP_ORSTRARRAY: {
        const uint8_t* sch = nullptr;
        size_t sn = 0;
        std::vector<std::pair<const uint8_t*, size_t>> arr;
        while (!r.done()) {
          if (!r.next(&num, &wt, &v, &q, &l)) return false;
          if (num == 1 && wt == 2) { sch = q; sn = l; }
          else if (num == 2 && wt == 2) arr.emplace_back(q, l);
        }
        if (sch) return jw.message(s.schema_props, sch, sn, out);
        out = "[";
        for (size_t k = 0; k < arr.size(); ++k) {
          if (k) out += ',';
          if (sp == pbc::SP_ORARRAY) {
            if (!jw.message(s.schema_props, arr[k].first, arr[k].second, out)) return false;
          } else {
            pbc::json_escape(out, (const char*)arr[k].first, arr[k].second);
          }
        }
        out += ']';
        return true;
      }
      default: return false;
    }
  }

  // a packed run of repeated varint / double scalars
  bool packed(const Field& f, const uint8_t* q, size_t l, PyObject* lst) {
    pbc::Reader pr{q, q + l};
    while (!pr.done()) {
      uint64_t x = 0;
      const uint8_t* xp = (const uint8_t*)"";
      size_t xn = 0;
      if (f.wt == 0) {
        if (!pr.varint(&x)) { err = "truncated packed field"; return false; }
      } else {
        if (pr.e - pr.p < 8) { err = "truncated packed field"; return false; }
        xp = pr.p; xn = 8; pr.p += 8;
      }
      PyObject* o = value(f, f.wt, x, xp, xn);
      if (!o) return false;
      PyList_Append(lst, o);
      Py_DECREF(o);
    }
    return true;
  }

  bool message(int mi, const uint8_t* p, size_t n, PyObject* out) {
    pbc::DepthGuard g(depth);
    if (!g.ok) { err = "protobuf nesting too deep"; return false; }
    const Message& m = s.msgs[mi];
    pbc::Reader r{p, p + n};
    uint32_t num; uint8_t wt; uint64_t v; const uint8_t* q; size_t l;
    while (!r.done()) {
      if (!r.next(&num, &wt, &v, &q, &l)) { err = "truncated protobuf"; return false; }
      if (num >= m.by_num.size() || m.by_num[num] < 0) continue;
      const int fi = m.by_num[num];
      const Field& f = m.fields[fi];
      if (!pbc::wire_ok(f, wt)) {
        err = "field " + f.json + ": wire type " + std::to_string(wt) + " does not match its type";
        return false;
      }
      if (f.inl) {
        if (!message(f.msg, q, l, out)) return false;
        continue;
      }
      PyObject* key = key_of(mi, fi, f);
      if (f.label == pbc::L_REP) {
        PyObject* lst = PyDict_GetItem(out, key);
        if (!lst) {
          lst = PyList_New(0);
          PyDict_SetItem(out, key, lst);
          Py_DECREF(lst);
        }
        if (wt == 2 && f.wt != 2) {
          if (!packed(f, q, l, lst)) { Py_DECREF(key); return false; }
        } else {
          PyObject* x = value(f, wt, v, q, l);
          if (!x) { Py_DECREF(key); return false; }
          PyList_Append(lst, x);
          Py_DECREF(x);
        }
      } else if (f.label == pbc::L_MAP) {
        PyObject* d = PyDict_GetItem(out, key);
        if (!d) {
          d = PyDict_New();
          PyDict_SetItem(out, key, d);
          Py_DECREF(d);
        }
        pbc::Reader e{q, q + l};
        PyObject* mk = nullptr;
        const uint8_t kwt = pbc::wire_of(f.key), ewt = f.type == pbc::S_MSG ? 2 : pbc::wire_of(f.type);
        uint8_t vwt = ewt;
        uint64_t vv = 0;
        const uint8_t* vp = (const uint8_t*)"";
        size_t vl = 0;
        uint32_t n2; uint8_t w2; uint64_t v2; const uint8_t* q2; size_t l2;
        while (!e.done()) {
          if (!e.next(&n2, &w2, &v2, &q2, &l2)) { Py_XDECREF(mk); Py_DECREF(key); err = "truncated map entry"; return false; }
          if ((n2 == 1 && w2 != kwt) || (n2 == 2 && w2 != ewt)) {
            Py_XDECREF(mk); Py_DECREF(key); err = "map entry " + f.json + ": wrong wire type"; return false;
          }
          if (n2 == 1) {
            Py_XDECREF(mk);
            if (w2 == 2) mk = str(q2, l2);
            else {
              std::string ks = std::to_string(f.key == pbc::S_INT32 ? (int64_t)(int32_t)v2 : (int64_t)v2);
              mk = PyUnicode_FromStringAndSize(ks.data(), (Py_ssize_t)ks.size());
            }
          } else if (n2 == 2) {
            vwt = w2; vv = v2; vp = q2; vl = l2;
          }
        }
        if (!mk) mk = PyUnicode_FromStringAndSize("", 0);
        Field vf = f;
        vf.label = pbc::L_OPT;
        PyObject* x = value(vf, vwt, vv, vp, vl);
        if (!x) { Py_DECREF(mk); Py_DECREF(key); return false; }
        PyDict_SetItem(d, mk, x);
        Py_DECREF(mk);
        Py_DECREF(x);
      } else {
        PyObject* x = value(f, wt, v, q, l);
        if (!x) { Py_DECREF(key); return false; }
        PyDict_SetItem(out, key, x);
        Py_DECREF(x);
      }
      Py_DECREF(key);
    }
    return true;
  }
};

// ---------------------------------------------------------------------------------------------
// envelope helpers
bool read_envelope(const uint8_t* p, size_t n, std::string* av, std::string* kind, const uint8_t** raw, size_t* raw_n) {
  if (n < 4 || memcmp(p, "k8s\0", 4) != 0) return false;
  pbc::Reader r{p + 4, p + n};
  *raw = (const uint8_t*)"";
  *raw_n = 0;
  uint32_t num; uint8_t wt; uint64_t v; const uint8_t* q; size_t l;
  while (!r.done()) {
    if (!r.next(&num, &wt, &v, &q, &l)) return false;
    if (num == 1 && wt == 2) {
      pbc::Reader t{q, q + l};
      uint32_t n2; uint8_t w2; uint64_t v2; const uint8_t* q2; size_t l2;
      while (!t.done()) {
        if (!t.next(&n2, &w2, &v2, &q2, &l2)) return false;
        if (n2 == 1 && w2 == 2) av->assign((const char*)q2, l2);
        else if (n2 == 2 && w2 == 2) kind->assign((const char*)q2, l2);
      }
    } else if (num == 2 && wt == 2) {
      *raw = q;
      *raw_n = l;
    }
  }
  return true;
}

void write_envelope(std::string& out, const std::string& av, const std::string& kind, const std::string& raw) {
  out.append("k8s\0", 4);
  std::string tm;
  put_ld(tm, 1, av.data(), av.size());
  put_ld(tm, 2, kind.data(), kind.size());
  put_ld(out, 1, tm.data(), tm.size());
  put_ld(out, 2, raw.data(), raw.size());
  put_ld(out, 3, "", 0);
  put_ld(out, 4, "", 0);
}

PyObject* raise_err(CodecObject* self, const std::string& path, const std::string& msg) {
  std::string text = path.empty() ? msg : path + ": " + msg;
  PyObject* args = Py_BuildValue("(ss)", msg.c_str(), path.c_str());
  if (args) {
    PyErr_SetObject(self->error, args);
    Py_DECREF(args);
  } else {
    PyErr_SetString(PyExc_ValueError, text.c_str());
  }
  return nullptr;
}

int lookup_msg(CodecObject* self, PyObject* name) {
  const char* p = PyUnicode_AsUTF8(name);
  if (!p) return -1;
  auto it = self->schema->by_name.find(p);
  return it == self->schema->by_name.end() ? -1 : it->second;
}

std::string get_str(PyObject* d, const char* k, const char* dflt) {
  PyObject* v = PyDict_GetItemString(d, k);
  if (!v || !PyUnicode_Check(v)) return dflt;
  const char* p = PyUnicode_AsUTF8(v);
  return p ? p : dflt;
}

// ---------------------------------------------------------------------------------------------
// methods
PyObject* c_encode_message(CodecObject* self, PyObject* args) {
  PyObject *name, *obj;
  if (!PyArg_ParseTuple(args, "UO", &name, &obj)) return nullptr;
  int mi = lookup_msg(self, name);
  if (mi < 0) return raise_err(self, "", std::string("no protobuf message ") + PyUnicode_AsUTF8(name));
  Encoder e{*self->schema, self, {}};
  std::string out;
  if (!e.message(mi, obj, out)) return raise_err(self, e.err.path, e.err.msg);
  return PyBytes_FromStringAndSize(out.data(), (Py_ssize_t)out.size());
}

PyObject* c_encode_object(CodecObject* self, PyObject* args) {
  PyObject *obj, *name;
  if (!PyArg_ParseTuple(args, "O!U", &PyDict_Type, &obj, &name)) return nullptr;
  int mi = lookup_msg(self, name);
  if (mi < 0) return raise_err(self, "", "no protobuf message");
  Encoder e{*self->schema, self, {}};
  std::string raw;
  raw.reserve(512);
  if (!e.message(mi, obj, raw)) return raise_err(self, e.err.path, e.err.msg);
  std::string out;
  out.reserve(raw.size() + 64);
  write_envelope(out, get_str(obj, "apiVersion", "v1"), get_str(obj, "kind", ""), raw);
  return PyBytes_FromStringAndSize(out.data(), (Py_ssize_t)out.size());
}

PyObject* c_decode_message(CodecObject* self, PyObject* args) {
  PyObject* name;
  Py_buffer buf;
  if (!PyArg_ParseTuple(args, "Uy*", &name, &buf)) return nullptr;
  int mi = lookup_msg(self, name);
  if (mi < 0) { PyBuffer_Release(&buf); return raise_err(self, "", "no protobuf message"); }
  Decoder d{*self->schema, self, {}};
  PyObject* out = PyDict_New();
  bool ok = d.message(mi, (const uint8_t*)buf.buf, (size_t)buf.len, out);
  PyBuffer_Release(&buf);
  if (!ok) {
    Py_DECREF(out);
    if (PyErr_Occurred()) return nullptr;
    return raise_err(self, "", d.err);
  }
  return out;
}

PyObject* c_decode_object(CodecObject* self, PyObject* args) {
  Py_buffer buf;
  if (!PyArg_ParseTuple(args, "y*", &buf)) return nullptr;
  std::string av, kind;
  const uint8_t* raw;
  size_t rn;
  if (!read_envelope((const uint8_t*)buf.buf, (size_t)buf.len, &av, &kind, &raw, &rn)) {
    PyBuffer_Release(&buf);
    return raise_err(self, "", "missing k8s protobuf magic or malformed envelope");
  }
  int mi = self->schema->message_for(av, kind);
  if (mi < 0) { PyBuffer_Release(&buf); return raise_err(self, "", "no protobuf message for " + av + "/" + kind); }
  PyObject* out = PyDict_New();
  PyObject* k = PyUnicode_FromStringAndSize(kind.data(), (Py_ssize_t)kind.size());
  PyObject* a = PyUnicode_FromStringAndSize(av.data(), (Py_ssize_t)av.size());
  PyDict_SetItemString(out, "kind", k);
  PyDict_SetItemString(out, "apiVersion", a);
  Py_DECREF(k);
  Py_DECREF(a);
  Decoder d{*self->schema, self, {}};
  bool ok = d.message(mi, raw, rn, out);
  PyBuffer_Release(&buf);
  if (!ok) {
    Py_DECREF(out);
    if (PyErr_Occurred()) return nullptr;
    return raise_err(self, "", d.err);
  }
  return out;
}

PyObject* c_to_json(CodecObject* self, PyObject* args) {
  Py_buffer buf;
  const char* rv = nullptr;
  if (!PyArg_ParseTuple(args, "y*|z", &buf, &rv)) return nullptr;
  pbc::JsonWriter w(*self->schema);
  std::string out;
  out.reserve((size_t)buf.len * 2 + 64);
  bool ok = w.object((const uint8_t*)buf.buf, (size_t)buf.len, out, rv, self->canon);
  PyBuffer_Release(&buf);
  if (!ok) return raise_err(self, "", "not a protobuf object of a known kind");
  return PyBytes_FromStringAndSize(out.data(), (Py_ssize_t)out.size());
}

// watch_frame(type, value, rv=None) -> one length-delimited protobuf WatchEvent frame
PyObject* c_watch_frame(CodecObject* self, PyObject* args) {
  const char* type;
  Py_buffer buf;
  const char* rv = nullptr;
  if (!PyArg_ParseTuple(args, "sy*|z", &type, &buf, &rv)) return nullptr;
  std::string env, out;
  const uint8_t* p = (const uint8_t*)buf.buf;
  size_t n = (size_t)buf.len;
  if (rv && pbc::envelope_with_rv(*self->schema, p, n, rv, env))
    pbc::watch_event_frame(out, type, env.data(), env.size());
  else
    pbc::watch_event_frame(out, type, p, n);
  PyBuffer_Release(&buf);
  return PyBytes_FromStringAndSize(out.data(), (Py_ssize_t)out.size());
}

// with_rv(envelope, rv) -> the envelope with metadata.resourceVersion = rv, or None
PyObject* c_with_rv(CodecObject* self, PyObject* args) {
  Py_buffer buf;
  const char* rv;
  if (!PyArg_ParseTuple(args, "y*s", &buf, &rv)) return nullptr;
  std::string out;
  bool ok = pbc::envelope_with_rv(*self->schema, (const uint8_t*)buf.buf, (size_t)buf.len, rv, out);
  PyBuffer_Release(&buf);
  if (!ok) Py_RETURN_NONE;
  return PyBytes_FromStringAndSize(out.data(), (Py_ssize_t)out.size());
}

// decode_watch_frames(buffer) -> (events [(type, object)], bytes consumed). Objects are decoded
// from their envelope (JSON raw values through json.loads).
PyObject* c_decode_watch_frames(CodecObject* self, PyObject* args) {
  Py_buffer buf;
  if (!PyArg_ParseTuple(args, "y*", &buf)) return nullptr;
  const uint8_t* p = (const uint8_t*)buf.buf;
  size_t n = (size_t)buf.len, pos = 0;
  PyObject* lst = PyList_New(0);
  std::string err;
  while (n - pos >= 4) {
    uint32_t fl = ((uint32_t)p[pos] << 24) | ((uint32_t)p[pos + 1] << 16) | ((uint32_t)p[pos + 2] << 8) | p[pos + 3];
    if (fl > (64u << 20)) { err = "watch frame too large"; break; }
    if (n - pos - 4 < fl) break;
    const uint8_t* f = p + pos + 4;
    pbc::Reader r{f, f + fl};
    const uint8_t *tp = nullptr, *raw = nullptr;
    size_t tn = 0, rn = 0;
    uint32_t num; uint8_t wt; uint64_t v; const uint8_t* q; size_t l;
    bool bad = false;
    while (!r.done()) {
      if (!r.next(&num, &wt, &v, &q, &l)) { bad = true; break; }
      if (num == 1 && wt == 2) { tp = q; tn = l; }
      else if (num == 2 && wt == 2) {
        pbc::Reader e{q, q + l};
        uint32_t n2; uint8_t w2; uint64_t v2; const uint8_t* q2; size_t l2;
        while (!e.done()) {
          if (!e.next(&n2, &w2, &v2, &q2, &l2)) { bad = true; break; }
          if (n2 == 1 && w2 == 2) { raw = q2; rn = l2; }
        }
      }
    }
    if (bad || !tp) { err = "malformed watch frame"; break; }
    PyObject* obj = nullptr;
    if (raw && rn >= 4 && memcmp(raw, "k8s\0", 4) == 0) {
      std::string av, kind;
      const uint8_t* body;
      size_t bn;
      if (!read_envelope(raw, rn, &av, &kind, &body, &bn)) { err = "malformed envelope in watch frame"; break; }
      int mi = self->schema->message_for(av, kind);
      if (mi < 0) { err = "no protobuf message for " + av + "/" + kind; break; }
      obj = PyDict_New();
      auto cit = self->canon ? self->canon->find(kind) : decltype(self->canon->end()){};
      const std::string& shown = (self->canon && cit != self->canon->end()) ? cit->second : av;
      PyObject* k = PyUnicode_FromStringAndSize(kind.data(), (Py_ssize_t)kind.size());
      PyObject* a = PyUnicode_FromStringAndSize(shown.data(), (Py_ssize_t)shown.size());
      PyDict_SetItemString(obj, "kind", k);
      PyDict_SetItemString(obj, "apiVersion", a);
      Py_DECREF(k);
      Py_DECREF(a);
      Decoder d{*self->schema, self, {}};
      if (!d.message(mi, body, bn, obj)) {
        Py_DECREF(obj);
        if (PyErr_Occurred()) { Py_DECREF(lst); PyBuffer_Release(&buf); return nullptr; }
        err = d.err;
        obj = nullptr;
        break;
      }
    } else {
      PyObject* b = PyBytes_FromStringAndSize((const char*)(raw ? raw : (const uint8_t*)""), (Py_ssize_t)rn);
      obj = PyObject_CallFunctionObjArgs(self->loads, b, nullptr);
      Py_DECREF(b);
      if (!obj) { Py_DECREF(lst); PyBuffer_Release(&buf); return nullptr; }
    }
    PyObject* t = PyUnicode_FromStringAndSize((const char*)tp, (Py_ssize_t)tn);
    PyObject* tup = PyTuple_Pack(2, t, obj);
    Py_DECREF(t);
    Py_DECREF(obj);
    PyList_Append(lst, tup);
    Py_DECREF(tup);
    pos += 4 + fl;
  }
  PyBuffer_Release(&buf);
  if (!err.empty()) {
    Py_DECREF(lst);
    return raise_err(self, "", err);
  }
  PyObject* consumed = PyLong_FromSize_t(pos);
  PyObject* res = PyTuple_Pack(2, lst, consumed);
  Py_DECREF(lst);
  Py_DECREF(consumed);
  return res;
}

PyObject* c_set_canonical(CodecObject* self, PyObject* args) {
  PyObject* d;
  if (!PyArg_ParseTuple(args, "O!", &PyDict_Type, &d)) return nullptr;
  auto* m = new std::unordered_map<std::string, std::string>();
  PyObject *k, *v;
  Py_ssize_t pos = 0;
  while (PyDict_Next(d, &pos, &k, &v)) {
    const char* ks = PyUnicode_AsUTF8(k);
    const char* vs = PyUnicode_AsUTF8(v);
    if (!ks || !vs) { delete m; return nullptr; }
    (*m)[ks] = vs;
  }
  delete self->canon;
  self->canon = m;
  Py_RETURN_NONE;
}

PyObject* c_message_for(CodecObject* self, PyObject* args) {
  const char *av, *kind;
  if (!PyArg_ParseTuple(args, "ss", &av, &kind)) return nullptr;
  int mi = self->schema->message_for(av, kind);
  if (mi < 0) Py_RETURN_NONE;
  return PyUnicode_FromString(self->schema->msgs[mi].name.c_str());
}

int codec_init(CodecObject* self, PyObject* args, PyObject*) {
  const char* path;
  PyObject *err, *dumps, *loads;
  if (!PyArg_ParseTuple(args, "sOOO", &path, &err, &dumps, &loads)) return -1;
  auto* s = new Schema();
  if (!s->load(path)) {
    PyErr_Format(PyExc_ValueError, "pbcodec schema: %s", s->error.c_str());
    delete s;
    return -1;
  }
  delete self->schema;
  self->schema = s;
  init_caches(self);
  Py_XINCREF(err); Py_XDECREF(self->error); self->error = err;
  Py_XINCREF(dumps); Py_XDECREF(self->dumps); self->dumps = dumps;
  Py_XINCREF(loads); Py_XDECREF(self->loads); self->loads = loads;
  return 0;
}

void codec_dealloc(CodecObject* self) {
  clear_caches(self);
  delete self->schema;
  delete self->canon;
  Py_XDECREF(self->error);
  Py_XDECREF(self->dumps);
  Py_XDECREF(self->loads);
  Py_TYPE(self)->tp_free((PyObject*)self);
}

PyMethodDef codec_methods[] = {
    {"encode_message", (PyCFunction)c_encode_message, METH_VARARGS, "message body bytes"},
    {"encode_object", (PyCFunction)c_encode_object, METH_VARARGS, "k8s\\0 envelope bytes"},
    {"decode_message", (PyCFunction)c_decode_message, METH_VARARGS, "dict"},
    {"decode_object", (PyCFunction)c_decode_object, METH_VARARGS, "dict"},
    {"to_json", (PyCFunction)c_to_json, METH_VARARGS, "JSON bytes with metadata.resourceVersion injected"},
    {"message_for", (PyCFunction)c_message_for, METH_VARARGS, "message name or None"},
    {"set_canonical", (PyCFunction)c_set_canonical, METH_VARARGS, "kind -> apiVersion reported by to_json"},
    {"with_rv", (PyCFunction)c_with_rv, METH_VARARGS, "envelope with metadata.resourceVersion set, or None"},
    {"watch_frame", (PyCFunction)c_watch_frame, METH_VARARGS, "length-delimited protobuf WatchEvent frame"},
    {"decode_watch_frames", (PyCFunction)c_decode_watch_frames, METH_VARARGS,
     "(events [(type, object)], bytes consumed) from a buffer of watch frames"},
    {nullptr, nullptr, 0, nullptr}};

PyTypeObject CodecType = {PyVarObject_HEAD_INIT(nullptr, 0)};

PyModuleDef module_def = {PyModuleDef_HEAD_INIT, "_kamd_pbcodec", "native Kubernetes protobuf codec", -1, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__kamd_pbcodec(void) {
  CodecType.tp_name = "_kamd_pbcodec.Codec";
  CodecType.tp_basicsize = sizeof(CodecObject);
  CodecType.tp_flags = Py_TPFLAGS_DEFAULT;
  CodecType.tp_new = PyType_GenericNew;
  CodecType.tp_init = (initproc)codec_init;
  CodecType.tp_dealloc = (destructor)codec_dealloc;
  CodecType.tp_methods = codec_methods;
  if (PyType_Ready(&CodecType) < 0) return nullptr;
  PyObject* m = PyModule_Create(&module_def);
  if (!m) return nullptr;
  Py_INCREF(&CodecType);
  PyModule_AddObject(m, "Codec", (PyObject*)&CodecType);
  return m;
}
