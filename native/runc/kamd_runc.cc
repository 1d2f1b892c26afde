// kamd-runc — the process runtime's OCI executor: runs one container from an OCI bundle with
// enforced device isolation.
//
//   kamd-runc features                         JSON: which isolation primitives work here
//   kamd-runc run --bundle DIR [--ready-fd N]  run DIR/config.json in the foreground
//   kamd-runc exec --pid PID [--cwd D] [--user U:G] [--landlock DIR:NODE,...] -- argv
//                                              enter a running container
//
// Parity target: what dockershim + docker/runc gave the reference's GPU pods
// (`pkg/kubelet/dockershim/docker_container.go:164-172` maps the device plugin's DeviceSpecs
// into HostConfig.Resources.Devices; `test/e2e_node/gpu_device_plugin.go:46-143` asserts pods
// get distinct GPUs). On MI355X the allocation is `/dev/kfd` + `/dev/dri/renderD<minor>`; a
// container must see ONLY its render nodes, whatever HIP_VISIBLE_DEVICES says.
//
// Process tree of `run` (one per container):
//   P  host pid the kubelet tracks. Applies host-side settings (cpuset, OOM score, cgroup join,
//      device cgroup), enters/creates namespaces, forks C, forwards signals to C, removes the
//      cgroups it created, exits with C's status.
//   C  first process of the new pid namespace (pid 1). Builds the mount namespace: private
//      propagation, optional pivot_root into the rootfs, /proc, a private tmpfs /dev holding
//      only the default nodes plus the spec's linux.devices (bind mounts of the host nodes —
//      a user namespace cannot mknod), spec mounts, masked / read-only paths, hostname; then
//      identity (groups, gid, uid), capability bounding set, no_new_privs. With a pid namespace
//      C stays as a minimal init (reaps, forwards signals) and forks G, the entrypoint;
//      without one C execs the entrypoint itself.
// Device cgroup: cgroup v2 -> a BPF_PROG_TYPE_CGROUP_DEVICE program generated from
// linux.resources.devices, attached to the container cgroup; cgroup v1 -> devices.deny /
// devices.allow in the devices hierarchy. Unprivileged (no CAP_SYS_ADMIN): a user namespace
// maps the container uid onto the caller's uid.
// Landlock tier (an unprivileged host without user namespaces, e.g. the MI355X CI pool): no
// namespaces at all, but before exec the container process restricts itself with a Landlock
// ruleset under no_new_privs — opening anything under /dev/dri other than its allocated render
// node(s) fails with EACCES, while the rest of the filesystem keeps its normal permissions.
// When no tier works `features` says so and the kubelet reports the node condition
// IsolationUnavailable instead of degrading silently.
#include <errno.h>
#include <fcntl.h>
#include <grp.h>
#include <limits.h>
#include <linux/bpf.h>
#include <linux/capability.h>
#include <linux/landlock.h>
#include <dirent.h>
#include <sched.h>
#include <signal.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mount.h>
#include <sys/prctl.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <sys/statfs.h>
#include <sys/statvfs.h>
#include <sys/syscall.h>
#include <sys/sysmacros.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <string>
#include <utility>
#include <vector>

extern char** environ;

namespace {

// ---------------------------------------------------------------------------------------------
// errors
[[noreturn]] void die(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  fputs("kamd-runc: ", stderr);
  vfprintf(stderr, fmt, ap);
  fputc('\n', stderr);
  va_end(ap);
  _exit(code);
}

void warn(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  fputs("kamd-runc: warning: ", stderr);
  vfprintf(stderr, fmt, ap);
  fputc('\n', stderr);
  va_end(ap);
}

// ---------------------------------------------------------------------------------------------
// a small JSON reader (the bundle's config.json is written by runtime/oci.py)
struct J {
  enum T { NUL, BOOL, NUM, STR, ARR, OBJ } t = NUL;
  bool b = false;
  double n = 0;
  std::string s;
  std::vector<J> a;
  std::vector<std::pair<std::string, J>> o;

  const J& operator[](const char* k) const {
    static const J nul;
    if (t == OBJ)
      for (auto& kv : o)
        if (kv.first == k) return kv.second;
    return nul;
  }
  bool has(const char* k) const { return (*this)[k].t != NUL; }
  std::string str(const char* d = "") const { return t == STR ? s : std::string(d); }
  long long num(long long d = 0) const { return t == NUM ? (long long)n : d; }
  bool boolean(bool d = false) const { return t == BOOL ? b : d; }
};

struct JParser {
  const char* p;
  const char* e;
  void ws() {
    while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  [[noreturn]] void fail() { die(126, "config.json: malformed JSON at offset %ld", (long)(e - p)); }
  static void utf8(std::string& out, unsigned cp) {
    if (cp < 0x80) {
      out += (char)cp;
    } else if (cp < 0x800) {
      out += (char)(0xC0 | (cp >> 6));
      out += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    } else {
      out += (char)(0xF0 | (cp >> 18));
      out += (char)(0x80 | ((cp >> 12) & 0x3F));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    }
  }
  unsigned hex4() {
    if (e - p < 4) fail();
    unsigned v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail();
    }
    return v;
  }
  std::string string() {
    if (p >= e || *p != '"') fail();
    ++p;
    std::string out;
    while (p < e && *p != '"') {
      char c = *p++;
      if (c != '\\') {
        out += c;
        continue;
      }
      if (p >= e) fail();
      c = *p++;
      switch (c) {
        case '"': case '\\': case '/': out += c; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          unsigned cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            p += 2;
            unsigned lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          utf8(out, cp);
          break;
        }
        default: fail();
      }
    }
    if (p >= e) fail();
    ++p;
    return out;
  }
  J value(int depth = 0) {
    if (depth > 64) fail();
    ws();
    if (p >= e) fail();
    J v;
    if (*p == '{') {
      v.t = J::OBJ;
      ++p;
      ws();
      if (p < e && *p == '}') { ++p; return v; }
      for (;;) {
        ws();
        std::string k = string();
        ws();
        if (p >= e || *p != ':') fail();
        ++p;
        v.o.emplace_back(std::move(k), value(depth + 1));
        ws();
        if (p < e && *p == ',') { ++p; continue; }
        if (p < e && *p == '}') { ++p; return v; }
        fail();
      }
    }
    if (*p == '[') {
      v.t = J::ARR;
      ++p;
      ws();
      if (p < e && *p == ']') { ++p; return v; }
      for (;;) {
        v.a.push_back(value(depth + 1));
        ws();
        if (p < e && *p == ',') { ++p; continue; }
        if (p < e && *p == ']') { ++p; return v; }
        fail();
      }
    }
    if (*p == '"') {
      v.t = J::STR;
      v.s = string();
      return v;
    }
    if (e - p >= 4 && !strncmp(p, "true", 4)) { p += 4; v.t = J::BOOL; v.b = true; return v; }
    if (e - p >= 5 && !strncmp(p, "false", 5)) { p += 5; v.t = J::BOOL; return v; }
    if (e - p >= 4 && !strncmp(p, "null", 4)) { p += 4; return v; }
    char* end;
    std::string num;
    while (p < e && strchr("+-0123456789.eE", *p)) num += *p++;
    v.n = strtod(num.c_str(), &end);
    if (num.empty() || *end) fail();
    v.t = J::NUM;
    return v;
  }
};

J read_json(const std::string& path) {
  int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) die(126, "open %s: %s", path.c_str(), strerror(errno));
  std::string buf;
  char tmp[65536];
  ssize_t r;
  while ((r = read(fd, tmp, sizeof tmp)) > 0) buf.append(tmp, (size_t)r);
  close(fd);
  JParser jp{buf.data(), buf.data() + buf.size()};
  J v = jp.value();
  return v;
}

// ---------------------------------------------------------------------------------------------
// small helpers
bool write_file(const std::string& path, const std::string& val, int flags = 0) {
  int fd = open(path.c_str(), O_WRONLY | O_CLOEXEC | flags, 0644);
  if (fd < 0) return false;
  bool ok = write(fd, val.data(), val.size()) == (ssize_t)val.size();
  close(fd);
  return ok;
}

std::string read_small(const std::string& path) {
  int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return "";
  char buf[8192];
  ssize_t r = read(fd, buf, sizeof buf - 1);
  close(fd);
  return r > 0 ? std::string(buf, (size_t)r) : "";
}

void mkdirs(const std::string& path, mode_t mode = 0755) {
  std::string cur;
  size_t i = 0;
  while (i <= path.size()) {
    size_t j = path.find('/', i);
    if (j == std::string::npos) j = path.size();
    cur = path.substr(0, j);
    if (!cur.empty()) mkdir(cur.c_str(), mode);
    i = j + 1;
  }
}

void touch(const std::string& path) {
  size_t s = path.rfind('/');
  if (s != std::string::npos && s > 0) mkdirs(path.substr(0, s));
  int fd = open(path.c_str(), O_CREAT | O_WRONLY | O_CLOEXEC, 0644);
  if (fd >= 0) close(fd);
}

std::vector<std::string> split_path(const std::string& p) {
  std::vector<std::string> out;
  size_t i = 0;
  while (i <= p.size()) {
    size_t j = p.find('/', i);
    if (j == std::string::npos) j = p.size();
    if (j > i) out.push_back(p.substr(i, j - i));
    i = j + 1;
  }
  return out;
}

// `unsafe` resolved under `root` the way a chroot would see it (runc's securejoin): every
// symlink met on the way is read and its target re-rooted at `root` (an absolute target starts
// over at root, `..` never climbs above it). Mount destinations, /dev nodes and masked paths
// come from the image and the spec, and an image may hold `dev -> /usr/bin` or
// `data -> /etc`: without this the runtime (often root) would create, unlink and mount over
// HOST paths before pivot_root. Components that do not exist yet are taken literally.
std::string secure_join(const std::string& root, const std::string& unsafe) {
  if (root.empty() || root == "/") return unsafe.empty() || unsafe[0] != '/' ? "/" + unsafe : unsafe;
  std::vector<std::string> todo = split_path(unsafe), done;
  std::reverse(todo.begin(), todo.end());   // a stack: back() is the next component
  int links = 0;
  auto cur_path = [&](const std::string& extra) {
    std::string c = root;
    for (auto& d : done) c += "/" + d;
    return extra.empty() ? c : c + "/" + extra;
  };
  while (!todo.empty()) {
    std::string c = todo.back();
    todo.pop_back();
    if (c.empty() || c == ".") continue;
    if (c == "..") {
      if (!done.empty()) done.pop_back();
      continue;
    }
    std::string cur = cur_path(c);
    struct stat st;
    if (lstat(cur.c_str(), &st) != 0 || !S_ISLNK(st.st_mode)) {
      done.push_back(c);
      continue;
    }
    if (++links > 255) die(126, "too many levels of symbolic links resolving %s", unsafe.c_str());
    char buf[PATH_MAX];
    ssize_t n = readlink(cur.c_str(), buf, sizeof buf - 1);
    if (n < 0) die(126, "readlink %s: %s", cur.c_str(), strerror(errno));
    std::string t(buf, (size_t)n);
    if (!t.empty() && t[0] == '/') done.clear();
    std::vector<std::string> more = split_path(t);
    for (auto it = more.rbegin(); it != more.rend(); ++it) todo.push_back(*it);
  }
  return cur_path("");
}

// a mountpoint created under root, opened without following a final symlink and checked to be
// inside root; mounts go through /proc/self/fd/<fd> so the checked inode is the one mounted on
struct Pinned {
  int fd = -1;
  std::string proc;
  Pinned() = default;
  Pinned(const Pinned&) = delete;
  Pinned& operator=(const Pinned&) = delete;
  ~Pinned() {
    if (fd >= 0) close(fd);
  }
  const char* c_str() const { return proc.c_str(); }
};

std::string g_root_real;   // realpath of the rootfs ("" = the host root: nothing to check)

// Landlock tier: the errno shim preloaded into the container (libkamd_devshim.so, next to this
// binary's bin/ in ../lib/). Landlock refuses DRM nodes with EACCES, which ROCr's thunk treats as
// fatal where the device cgroup's EPERM means "skip this GPU"; the shim reports EPERM instead.
// "" = not preloaded (no shim built, or the spec opted out with kamd.io/devshim: "false").
std::string g_devshim;
std::string g_devshim_dir;

std::string devshim_path() {
  char exe[PATH_MAX];
  ssize_t n = readlink("/proc/self/exe", exe, sizeof exe - 1);
  if (n <= 0) return "";
  exe[n] = 0;
  std::string d(exe);
  size_t s = d.rfind('/');
  if (s == std::string::npos) return "";
  d.resize(s);                               // .../bin
  s = d.rfind('/');
  if (s == std::string::npos) return "";
  std::string lib = d.substr(0, s) + "/lib/libkamd_devshim.so";
  return access(lib.c_str(), R_OK) == 0 ? lib : "";
}

// LD_PRELOAD with the shim first (an existing preload list is kept after it)
std::string with_devshim(const char* current) {
  if (g_devshim.empty()) return current ? current : "";
  if (current == nullptr || !*current) return g_devshim;
  if (strstr(current, g_devshim.c_str()) != nullptr) return current;
  return g_devshim + ":" + current;
}

void pin(Pinned& p, const std::string& path) {
  p.fd = open(path.c_str(), O_PATH | O_NOFOLLOW | O_CLOEXEC);
  if (p.fd < 0) die(126, "open mountpoint %s: %s", path.c_str(), strerror(errno));
  char link[64];
  snprintf(link, sizeof link, "/proc/self/fd/%d", p.fd);
  p.proc = link;
  if (g_root_real.empty()) return;
  char real[PATH_MAX];
  ssize_t n = readlink(link, real, sizeof real - 1);
  if (n < 0) die(126, "readlink %s: %s", link, strerror(errno));
  std::string r(real, (size_t)n);
  if (r != g_root_real && r.compare(0, g_root_real.size() + 1, g_root_real + "/") != 0)
    die(126, "mountpoint %s resolves to %s, outside the rootfs", path.c_str(), r.c_str());
}

int parse_cpus(const char* s, cpu_set_t* set) {
  CPU_ZERO(set);
  int n = 0;
  while (*s) {
    char* end;
    long a = strtol(s, &end, 10);
    if (end == s || a < 0 || a >= CPU_SETSIZE) return -1;
    long b = a;
    s = end;
    if (*s == '-') {
      b = strtol(s + 1, &end, 10);
      if (end == s + 1 || b < a || b >= CPU_SETSIZE) return -1;
      s = end;
    }
    for (long i = a; i <= b; ++i, ++n) CPU_SET(i, set);
    if (*s == ',') ++s;
    else if (*s) return -1;
  }
  return n;
}

bool has_cap(int cap) {
  struct __user_cap_header_struct h = {_LINUX_CAPABILITY_VERSION_3, 0};
  struct __user_cap_data_struct d[2] = {};
  if (syscall(SYS_capget, &h, d) != 0) return false;
  return (d[cap / 32].effective >> (cap % 32)) & 1;
}

const char* const CAP_NAMES[] = {
    "CAP_CHOWN", "CAP_DAC_OVERRIDE", "CAP_DAC_READ_SEARCH", "CAP_FOWNER", "CAP_FSETID", "CAP_KILL", "CAP_SETGID",
    "CAP_SETUID", "CAP_SETPCAP", "CAP_LINUX_IMMUTABLE", "CAP_NET_BIND_SERVICE", "CAP_NET_BROADCAST",
    "CAP_NET_ADMIN", "CAP_NET_RAW", "CAP_IPC_LOCK", "CAP_IPC_OWNER", "CAP_SYS_MODULE", "CAP_SYS_RAWIO",
    "CAP_SYS_CHROOT", "CAP_SYS_PTRACE", "CAP_SYS_PACCT", "CAP_SYS_ADMIN", "CAP_SYS_BOOT", "CAP_SYS_NICE",
    "CAP_SYS_RESOURCE", "CAP_SYS_TIME", "CAP_SYS_TTY_CONFIG", "CAP_MKNOD", "CAP_LEASE", "CAP_AUDIT_WRITE",
    "CAP_AUDIT_CONTROL", "CAP_SETFCAP", "CAP_MAC_OVERRIDE", "CAP_MAC_ADMIN", "CAP_SYSLOG", "CAP_WAKE_ALARM",
    "CAP_BLOCK_SUSPEND", "CAP_AUDIT_READ", "CAP_PERFMON", "CAP_BPF", "CAP_CHECKPOINT_RESTORE"};
constexpr int NCAPS = sizeof CAP_NAMES / sizeof CAP_NAMES[0];

int cap_last() {
  std::string s = read_small("/proc/sys/kernel/cap_last_cap");
  int v = s.empty() ? NCAPS - 1 : atoi(s.c_str());
  return v;
}

// true when this process holds no permitted capability (an unprivileged runtime)
bool no_permitted_caps() {
  std::string st = read_small("/proc/self/status");
  size_t p = st.find("CapPrm:");
  if (p == std::string::npos) return false;
  return strtoull(st.c_str() + p + 7, nullptr, 16) == 0;
}

// keep only `keep` (a bitmask over cap numbers) in the bounding set: an exec'd root process then
// gets at most these capabilities (permitted' = bounding & file-permitted(all for root)).
// An unprivileged runtime (no CAP_SETPCAP, nothing permitted) cannot narrow the bounding set; its
// container holds no capability either, and no_new_privs then keeps setuid/file-capability
// binaries from granting any on exec — the same ceiling, reached the other way.
void restrict_bounding(const std::vector<bool>& keep, bool drop_mknod) {
  int last = cap_last();
  for (int c = 0; c <= last; ++c) {
    bool k = c < (int)keep.size() && keep[c] && !(drop_mknod && c == CAP_MKNOD);
    if (!k && prctl(PR_CAPBSET_READ, c, 0, 0, 0) == 1 && prctl(PR_CAPBSET_DROP, c, 0, 0, 0) != 0) {
      if (errno == EPERM && no_permitted_caps()) {
        if (prctl(PR_SET_NO_NEW_PRIVS, 1, 0, 0, 0) != 0)
          die(126, "no_new_privs (unprivileged runtime): %s", strerror(errno));
        return;
      }
      die(126, "dropping capability %d: %s", c, strerror(errno));
    }
  }
}

std::vector<bool> caps_from(const J& list) {
  std::vector<bool> keep(64, false);
  for (auto& v : list.a)
    for (int i = 0; i < NCAPS; ++i)
      if (v.s == CAP_NAMES[i]) keep[i] = true;
  return keep;
}

// ---------------------------------------------------------------------------------------------
// device cgroup
struct DevRule {
  bool allow = true;
  char type = 'a';  // 'a' | 'c' | 'b'
  long long major = -1, minor = -1;
  int access = 7;   // BPF_DEVCG_ACC_{MKNOD=1,READ=2,WRITE=4}
};

int access_bits(const std::string& s) {
  int a = 0;
  for (char c : s) a |= c == 'm' ? 1 : c == 'r' ? 2 : c == 'w' ? 4 : 0;
  return a ? a : 7;
}

std::vector<DevRule> dev_rules(const J& spec) {
  std::vector<DevRule> out;
  for (auto& r : spec["linux"]["resources"]["devices"].a) {
    DevRule d;
    d.allow = r["allow"].boolean(false);
    std::string t = r["type"].str("a");
    d.type = t.empty() ? 'a' : t[0];
    d.major = r.has("major") ? r["major"].num(-1) : -1;
    d.minor = r.has("minor") ? r["minor"].num(-1) : -1;
    d.access = access_bits(r["access"].str("rwm"));
    out.push_back(d);
  }
  return out;
}

// default nodes every container gets (runc's default allow list): null, zero, full, random,
// urandom, tty, ptmx + /dev/pts/*
std::vector<DevRule> default_rules() {
  std::vector<DevRule> v;
  const long long m[][2] = {{1, 3}, {1, 5}, {1, 7}, {1, 8}, {1, 9}, {5, 0}, {5, 2}, {136, -1}};
  for (auto& x : m) {
    DevRule d;
    d.type = 'c';
    d.major = x[0];
    d.minor = x[1];
    d.access = 7;
    v.push_back(d);
  }
  return v;
}

struct Insn {
  uint8_t code;
  uint8_t regs;  // dst | src << 4
  int16_t off;
  int32_t imm;
};

Insn I(uint8_t code, int dst, int src, int16_t off, int32_t imm) {
  return Insn{code, (uint8_t)((dst & 0xf) | ((src & 0xf) << 4)), off, imm};
}

// BPF_PROG_TYPE_CGROUP_DEVICE program: rules are OCI-ordered (later entries override earlier),
// so they are tested last-to-first and the first match decides; no match denies.
std::vector<Insn> device_program(const std::vector<DevRule>& rules) {
  std::vector<Insn> p;
  p.push_back(I(BPF_LDX | BPF_MEM | BPF_W, 2, 1, 0, 0));   // r2 = ctx->access_type
  p.push_back(I(BPF_ALU | BPF_MOV | BPF_X, 3, 2, 0, 0));   // w3 = w2
  p.push_back(I(BPF_ALU | BPF_AND | BPF_K, 3, 0, 0, 0xffff));  // w3 = dev type
  p.push_back(I(BPF_ALU | BPF_MOV | BPF_X, 4, 2, 0, 0));   // w4 = w2
  p.push_back(I(BPF_ALU | BPF_RSH | BPF_K, 4, 0, 0, 16));  // w4 = requested access
  p.push_back(I(BPF_LDX | BPF_MEM | BPF_W, 5, 1, 4, 0));   // r5 = major
  p.push_back(I(BPF_LDX | BPF_MEM | BPF_W, 6, 1, 8, 0));   // r6 = minor
  for (size_t k = rules.size(); k-- > 0;) {
    const DevRule& r = rules[k];
    std::vector<size_t> jumps;
    if (r.type == 'c' || r.type == 'b') {
      jumps.push_back(p.size());
      p.push_back(I(BPF_JMP | BPF_JNE | BPF_K, 3, 0, 0, r.type == 'c' ? BPF_DEVCG_DEV_CHAR : BPF_DEVCG_DEV_BLOCK));
    }
    if ((r.access & 7) != 7) {
      p.push_back(I(BPF_ALU | BPF_MOV | BPF_X, 7, 4, 0, 0));
      p.push_back(I(BPF_ALU | BPF_AND | BPF_K, 7, 0, 0, ~r.access & 7));
      jumps.push_back(p.size());
      p.push_back(I(BPF_JMP | BPF_JNE | BPF_K, 7, 0, 0, 0));  // asks for more than allowed
    }
    if (r.major >= 0) {
      jumps.push_back(p.size());
      p.push_back(I(BPF_JMP | BPF_JNE | BPF_K, 5, 0, 0, (int32_t)r.major));
    }
    if (r.minor >= 0) {
      jumps.push_back(p.size());
      p.push_back(I(BPF_JMP | BPF_JNE | BPF_K, 6, 0, 0, (int32_t)r.minor));
    }
    p.push_back(I(BPF_ALU64 | BPF_MOV | BPF_K, 0, 0, 0, r.allow ? 1 : 0));
    p.push_back(I(BPF_JMP | BPF_EXIT, 0, 0, 0, 0));
    for (size_t j : jumps) p[j].off = (int16_t)(p.size() - (j + 1));
    if (jumps.empty()) return p;  // matches everything: the earlier rules are unreachable
  }
  p.push_back(I(BPF_ALU64 | BPF_MOV | BPF_K, 0, 0, 0, 0));
  p.push_back(I(BPF_JMP | BPF_EXIT, 0, 0, 0, 0));
  return p;
}

int bpf_load_device_prog(const std::vector<DevRule>& rules, std::string* log_out) {
  std::vector<Insn> prog = device_program(rules);
  static char log[16384];
  log[0] = 0;
  union bpf_attr attr;
  memset(&attr, 0, sizeof attr);
  attr.prog_type = BPF_PROG_TYPE_CGROUP_DEVICE;
  attr.insns = (uint64_t)(uintptr_t)prog.data();
  attr.insn_cnt = (uint32_t)prog.size();
  attr.license = (uint64_t)(uintptr_t) "GPL";
  attr.log_buf = (uint64_t)(uintptr_t)log;
  attr.log_size = sizeof log;
  attr.log_level = 1;
  int fd = (int)syscall(SYS_bpf, BPF_PROG_LOAD, &attr, sizeof attr);
  if (fd < 0 && log_out) *log_out = log;
  return fd;
}

bool is_cgroup2(const std::string& path) {
  struct statfs s;
  return statfs(path.c_str(), &s) == 0 && (unsigned long)s.f_type == 0x63677270UL;  // CGROUP2_SUPER_MAGIC
}

bool is_cgroup1(const std::string& path) {
  struct statfs s;
  return statfs(path.c_str(), &s) == 0 && (unsigned long)s.f_type == 0x27e0ebUL;  // CGROUP_SUPER_MAGIC
}

const char* V1_DEVICES = "/sys/fs/cgroup/devices";

struct CgroupState {
  std::string leaf;         // cgroup we created (removed on exit)
  std::string v1_devices;   // v1 devices cgroup we created
  std::string mode = "none";  // device enforcement: bpf | v1 | none
  std::string error;
};

// Join the container cgroup (creating it) and install the device filter. Runs in P, in the host
// namespaces, before anything else: the children inherit the membership.
void setup_cgroups(const J& spec, const std::string& cid, CgroupState& cg) {
  std::string path = spec["linux"]["cgroupsPath"].str();
  std::vector<DevRule> rules = default_rules();
  std::vector<DevRule> extra = dev_rules(spec);
  bool want_filter = !extra.empty();
  rules.insert(rules.begin(), extra.begin(), extra.end());
  // spec order first ({allow:false, rwm} deny-all then allows), then defaults: later wins
  std::string pid = std::to_string(getpid());
  if (!path.empty()) {
    struct stat st;
    if (stat(path.c_str(), &st) != 0) {
      mkdirs(path);
      if (stat(path.c_str(), &st) == 0) cg.leaf = path;
    }
    if (!write_file(path + "/cgroup.procs", pid, O_CREAT)) warn("joining cgroup %s: %s", path.c_str(), strerror(errno));
  }
  if (!want_filter) return;
  if (!path.empty() && is_cgroup2(path)) {
    std::string log;
    int pfd = bpf_load_device_prog(rules, &log);
    if (pfd < 0) {
      cg.error = std::string("BPF_PROG_LOAD: ") + strerror(errno) + " " + log.substr(0, 512);
    } else {
      int cfd = open(path.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
      union bpf_attr attr;
      memset(&attr, 0, sizeof attr);
      attr.target_fd = (uint32_t)cfd;
      attr.attach_bpf_fd = (uint32_t)pfd;
      attr.attach_type = BPF_CGROUP_DEVICE;
      attr.attach_flags = BPF_F_ALLOW_MULTI;
      if (cfd >= 0 && syscall(SYS_bpf, BPF_PROG_ATTACH, &attr, sizeof attr) == 0) cg.mode = "bpf";
      else cg.error = std::string("BPF_PROG_ATTACH: ") + strerror(errno);
      if (cfd >= 0) close(cfd);
      close(pfd);
    }
  }
  if (cg.mode == "none" && is_cgroup1(V1_DEVICES) && access((std::string(V1_DEVICES) + "/devices.allow").c_str(), W_OK) == 0) {
    std::string d = std::string(V1_DEVICES) + "/kamd/" + cid;
    mkdirs(d);
    bool ok = write_file(d + "/devices.deny", "a");
    for (auto& r : rules) {
      if (!r.allow || !ok) continue;  // deny-all already written; v1 cannot express a deny after allows
      char line[96];
      std::string acc;
      if (r.access & 2) acc += 'r';
      if (r.access & 4) acc += 'w';
      if (r.access & 1) acc += 'm';
      std::string maj = r.major < 0 ? "*" : std::to_string(r.major), min = r.minor < 0 ? "*" : std::to_string(r.minor);
      snprintf(line, sizeof line, "%c %s:%s %s", r.type, maj.c_str(), min.c_str(), acc.c_str());
      ok = write_file(d + "/devices.allow", line);
    }
    if (ok && write_file(d + "/cgroup.procs", pid)) {
      cg.mode = "v1";
      cg.v1_devices = d;
    } else {
      cg.error += std::string(cg.error.empty() ? "" : "; ") + "v1 devices cgroup: " + strerror(errno);
      rmdir(d.c_str());
    }
  }
}

void cleanup_cgroups(const CgroupState& cg) {
  // P itself is still a member: move it out first (to the parent) so rmdir can succeed
  if (!cg.v1_devices.empty()) {
    write_file(std::string(V1_DEVICES) + "/cgroup.procs", std::to_string(getpid()));
    rmdir(cg.v1_devices.c_str());
  }
  if (!cg.leaf.empty()) {
    std::string parent = cg.leaf.substr(0, cg.leaf.rfind('/'));
    write_file(parent + "/cgroup.procs", std::to_string(getpid()));
    rmdir(cg.leaf.c_str());
  }
}

// ---------------------------------------------------------------------------------------------
// mounts
struct MountFlag {
  const char* name;
  bool clear;
  unsigned long flag;
};
const MountFlag MOUNT_FLAGS[] = {
    {"ro", false, MS_RDONLY}, {"rw", true, MS_RDONLY}, {"nosuid", false, MS_NOSUID}, {"suid", true, MS_NOSUID},
    {"nodev", false, MS_NODEV}, {"dev", true, MS_NODEV}, {"noexec", false, MS_NOEXEC}, {"exec", true, MS_NOEXEC},
    {"noatime", false, MS_NOATIME}, {"relatime", false, MS_RELATIME}, {"strictatime", false, MS_STRICTATIME},
    {"nodiratime", false, MS_NODIRATIME}, {"bind", false, MS_BIND}, {"rbind", false, MS_BIND | MS_REC},
    {"sync", false, MS_SYNCHRONOUS}, {"dirsync", false, MS_DIRSYNC}};

void parse_options(const J& opts, unsigned long* flags, std::string* data) {
  for (auto& o : opts.a) {
    bool known = false;
    for (auto& f : MOUNT_FLAGS)
      if (o.s == f.name) {
        known = true;
        if (f.clear) *flags &= ~f.flag;
        else *flags |= f.flag;
      }
    if (!known && o.s != "private" && o.s != "rprivate" && o.s != "slave" && o.s != "rslave") {
      if (!data->empty()) *data += ',';
      *data += o.s;
    }
  }
}

// flags a remount inside a user namespace must keep (the kernel refuses to clear locked ones)
unsigned long locked_flags(const std::string& path) {
  struct statvfs s;
  unsigned long f = 0;
  if (statvfs(path.c_str(), &s) != 0) return 0;
  if (s.f_flag & ST_NOSUID) f |= MS_NOSUID;
  if (s.f_flag & ST_NODEV) f |= MS_NODEV;
  if (s.f_flag & ST_NOEXEC) f |= MS_NOEXEC;
  if (s.f_flag & ST_RDONLY) f |= MS_RDONLY;
  return f;
}

void bind_remount(const std::string& target, unsigned long extra) {
  unsigned long f = MS_BIND | MS_REMOUNT | extra | locked_flags(target);
  if (mount(nullptr, target.c_str(), nullptr, f, nullptr) != 0)
    die(126, "remount %s: %s", target.c_str(), strerror(errno));
}

struct HostNode {
  std::string path;  // in the container
  int fd = -1;       // O_PATH fd of the host node, opened before /dev is replaced
  unsigned maj = 0, min = 0;
};

// ---------------------------------------------------------------------------------------------
// Landlock (unprivileged device confinement)
int landlock_abi() {
  long r = syscall(__NR_landlock_create_ruleset, nullptr, 0, LANDLOCK_CREATE_RULESET_VERSION);
  return r < 0 ? 0 : (int)r;
}

// Restrict this process (and its future children) so that files under `dir` can be opened for
// reading or writing only when they are in `allowed`; everywhere else opens behave as before.
// Landlock rules only ever ALLOW, so the ruleset allows every sibling on the way from / down to
// `dir` and, inside `dir`, just the allowed entries. What is not an open (readdir, stat, exec,
// mkdir, ...) is not handled by the ruleset and stays unrestricted. Returns "" or an error.
std::string landlock_restrict(const std::string& dir_in, const std::vector<std::string>& allowed, int* nrules) {
  const uint64_t rights = LANDLOCK_ACCESS_FS_READ_FILE | LANDLOCK_ACCESS_FS_WRITE_FILE;
  char real[PATH_MAX];
  if (!realpath(dir_in.c_str(), real)) return "realpath " + dir_in + ": " + strerror(errno);
  std::string dir = real;
  if (dir == "/") return "refusing to restrict /";
  struct landlock_ruleset_attr ra;
  memset(&ra, 0, sizeof ra);
  ra.handled_access_fs = rights;
  int rs = (int)syscall(__NR_landlock_create_ruleset, &ra, sizeof ra, 0);
  if (rs < 0) return std::string("landlock_create_ruleset: ") + strerror(errno);
  int n = 0;
  std::string err;
  // required: an allowed device node must get its rule; the siblings along the way are best
  // effort (a pipe or socket behind /dev/stderr: nothing to open there anyway). A sibling that
  // is a symlink is skipped, never followed: it may point back at `dir` or one of its ancestors
  // (pytest's `pytest-current`, a distro's /var/run -> /run), and a rule on its target would
  // allow the whole tree. Its target needs no rule of its own — a real path leaves the chain
  // to `dir` at some real sibling, which has one.
  auto allow = [&](const std::string& path, bool required) {
    int fd = open(path.c_str(), O_PATH | O_CLOEXEC | (required ? 0 : O_NOFOLLOW));
    if (fd < 0) {
      if (required && err.empty()) err = "open " + path + ": " + strerror(errno);
      return;
    }
    struct stat st;
    bool fsobj = fstat(fd, &st) == 0 && (S_ISDIR(st.st_mode) || S_ISREG(st.st_mode) || S_ISCHR(st.st_mode) ||
                                         S_ISBLK(st.st_mode) || S_ISFIFO(st.st_mode));
    struct landlock_path_beneath_attr pb;
    memset(&pb, 0, sizeof pb);
    pb.allowed_access = rights;              // file rights: valid on files and directories
    pb.parent_fd = fd;
    if (fsobj && syscall(__NR_landlock_add_rule, rs, LANDLOCK_RULE_PATH_BENEATH, &pb, 0) == 0) ++n;
    else if (required && err.empty()) err = "landlock_add_rule " + path + ": " + strerror(errno);
    close(fd);
  };
  std::vector<std::string> comps = split_path(dir);
  std::string level = "/";
  for (size_t k = 0; k < comps.size(); ++k) {
    DIR* d = opendir(level.c_str());
    if (!d) { close(rs); return "opendir " + level + ": " + strerror(errno); }
    while (struct dirent* e = readdir(d)) {
      std::string name = e->d_name;
      if (name == "." || name == ".." || name == comps[k]) continue;
      allow((level == "/" ? "/" : level + "/") + name, false);
    }
    closedir(d);
    level = (level == "/" ? "/" : level + "/") + comps[k];
  }
  std::vector<std::string> inside;
  for (auto& a : allowed) {
    char ar[PATH_MAX];
    if (!realpath(a.c_str(), ar)) continue;
    std::string r = ar;
    if (r.compare(0, dir.size() + 1, dir + "/") == 0) {
      allow(r, true);
      inside.push_back(r);
    }
  }
  if (!err.empty()) { close(rs); return err; }
  // restrict_self needs no_new_privs (or CAP_SYS_ADMIN): set it either way — a setuid binary in
  // the container could otherwise regain what the ruleset takes away
  if (prctl(PR_SET_NO_NEW_PRIVS, 1, 0, 0, 0) != 0) { close(rs); return std::string("no_new_privs: ") + strerror(errno); }
  if (syscall(__NR_landlock_restrict_self, rs, 0) != 0) {
    std::string e = std::string("landlock_restrict_self: ") + strerror(errno);
    close(rs);
    return e;
  }
  close(rs);
  if (nrules) *nrules = n;
  return "";
}

struct Report {
  std::string tier = "none";               // namespaces | landlock | none
  int landlock_rules = 0;
  bool devshim = false;                    // Landlock tier: EACCES->EPERM errno shim preloaded
  bool user_ns = false, mount_ns = false, pid_ns = false, ipc_ns = false, uts_ns = false;
  std::string proc = "host", dev = "host", sys = "host";
  std::vector<std::string> devices;
  std::vector<std::string> notes;
};

// device nodes to expose: the defaults + linux.devices. A spec device names its node inside the
// container; the host node is found at the same path (the device plugin's pathOnHost is recorded
// in the kamd.io/host-path field when it differs) and must carry the spec's major:minor.
std::vector<HostNode> open_host_nodes(const J& spec) {
  std::vector<HostNode> out;
  const char* defaults[] = {"/dev/null", "/dev/zero", "/dev/full", "/dev/random", "/dev/urandom", "/dev/tty"};
  for (const char* d : defaults) {
    HostNode h;
    h.path = d;
    h.fd = open(d, O_PATH | O_CLOEXEC);
    if (h.fd >= 0) out.push_back(h);
  }
  for (auto& d : spec["linux"]["devices"].a) {
    HostNode h;
    h.path = d["path"].str();
    std::string host = d["kamd.io/host-path"].str(h.path.c_str());
    h.fd = open(host.c_str(), O_PATH | O_CLOEXEC);
    if (h.fd < 0) die(126, "device %s: %s", host.c_str(), strerror(errno));
    struct stat st;
    if (fstat(h.fd, &st) != 0 || !(S_ISCHR(st.st_mode) || S_ISBLK(st.st_mode)))
      die(126, "device %s is not a device node", host.c_str());
    h.maj = major(st.st_rdev);
    h.min = minor(st.st_rdev);
    if (d.has("major") && (d["major"].num() != h.maj || d["minor"].num() != h.min))
      die(126, "device %s is %u:%u, the spec says %lld:%lld", host.c_str(), h.maj, h.min, d["major"].num(),
          d["minor"].num());
    out.push_back(h);
  }
  return out;
}

void bind_fd(int fd, const std::string& target) {
  char src[64];
  snprintf(src, sizeof src, "/proc/self/fd/%d", fd);
  touch(target);
  Pinned t;
  pin(t, target);
  if (mount(src, t.c_str(), nullptr, MS_BIND, nullptr) != 0)
    die(126, "bind %s: %s", target.c_str(), strerror(errno));
}

void setup_dev(const std::string& rootfs, const std::string& target, const std::string& data,
               std::vector<HostNode>& nodes, Report& rep) {
  // nodev: a node created here by mknod is dead; only the bind-mounted host nodes work
  {
    Pinned t;
    pin(t, target);
    if (mount("tmpfs", t.c_str(), "tmpfs", MS_NOSUID | MS_NODEV | MS_STRICTATIME,
              data.empty() ? "mode=755,size=65536k" : data.c_str()) != 0)
      die(126, "mount tmpfs %s: %s", target.c_str(), strerror(errno));
  }
  rep.dev = "private";
  // nodes live on the fresh tmpfs at `target` (the image's own /dev, symlink or not, is gone)
  auto in_dev = [&](const std::string& p) {
    std::string rel = p.compare(0, 5, "/dev/") == 0 ? p.substr(5) : p;
    return secure_join(target, rel);
  };
  for (auto& h : nodes) {
    bind_fd(h.fd, in_dev(h.path));
    close(h.fd);
    h.fd = -1;
    rep.devices.push_back(h.path);
  }
  const char* links[][2] = {{"/proc/self/fd", "/dev/fd"}, {"/proc/self/fd/0", "/dev/stdin"},
                             {"/proc/self/fd/1", "/dev/stdout"}, {"/proc/self/fd/2", "/dev/stderr"}};
  for (auto& l : links)
    if (symlink(l[0], in_dev(l[1]).c_str()) != 0) warn("symlink %s: %s", l[1], strerror(errno));
}

void do_mounts(const J& spec, const std::string& rootfs, std::vector<HostNode>& nodes, Report& rep) {
  bool dev_done = false;
  // every bind source is opened before the first mount: a private /dev (or any earlier mount)
  // may cover a source such as a memory-backed emptyDir under /dev/shm; the bind then goes
  // through /proc/self/fd/<fd>, the inode opened here
  std::vector<int> src_fd(spec["mounts"].a.size(), -1);
  for (size_t i = 0; i < spec["mounts"].a.size(); ++i) {
    const J& m = spec["mounts"].a[i];
    unsigned long f0 = 0;
    std::string d0;
    parse_options(m["options"], &f0, &d0);
    if (m["type"].str() == "bind" || (f0 & MS_BIND)) {
      std::string src = m["source"].str();
      src_fd[i] = open(src.c_str(), O_PATH | O_CLOEXEC);
      if (src_fd[i] < 0) die(126, "bind source %s: %s", src.c_str(), strerror(errno));
    }
  }
  size_t mi = 0;
  for (auto& m : spec["mounts"].a) {
    int sfd = src_fd[mi++];
    std::string dst = m["destination"].str(), type = m["type"].str(), src = m["source"].str();
    std::string target = secure_join(rootfs, dst);
    unsigned long flags = 0;
    std::string data;
    parse_options(m["options"], &flags, &data);
    if (type == "bind" || (flags & MS_BIND)) {
      struct stat st;
      if (fstat(sfd, &st) != 0) die(126, "bind source %s: %s", src.c_str(), strerror(errno));
      char sproc[64];
      snprintf(sproc, sizeof sproc, "/proc/self/fd/%d", sfd);
      struct stat tst;
      if (rootfs == "/" && stat(target.c_str(), &tst) != 0) {
        // the container's root is the host's own: creating the mountpoint would write to the
        // host filesystem, so the volume stays reachable at its host path only
        rep.notes.push_back("bind " + dst + ": no mountpoint on the host root");
        close(sfd);
        continue;
      }
      if (S_ISDIR(st.st_mode)) mkdirs(target);
      else touch(target);
      {
        Pinned t;
        pin(t, target);
        if (mount(sproc, t.c_str(), nullptr, MS_BIND | (flags & MS_REC), nullptr) != 0)
          die(126, "bind %s -> %s: %s", src.c_str(), target.c_str(), strerror(errno));
      }
      close(sfd);
      unsigned long extra = flags & (MS_RDONLY | MS_NOSUID | MS_NODEV | MS_NOEXEC);
      if (extra) bind_remount(target, extra);
      continue;
    }
    mkdirs(target);
    Pinned tp;
    if (!(type == "tmpfs" && dst == "/dev")) pin(tp, target);   // setup_dev pins its own
    if (type == "proc") {
      if (rep.pid_ns && mount("proc", tp.c_str(), "proc", MS_NOSUID | MS_NODEV | MS_NOEXEC, nullptr) == 0) {
        rep.proc = "private";
      } else {
        // no pid namespace (or /proc overmounted by the host): keep the host's /proc
        rep.notes.push_back(std::string("proc: host view (") + (rep.pid_ns ? strerror(errno) : "no pid namespace") + ")");
        if (rootfs != "/" && mount("/proc", tp.c_str(), nullptr, MS_BIND | MS_REC, nullptr) != 0)
          die(126, "bind /proc: %s", strerror(errno));
      }
    } else if (type == "tmpfs" && dst == "/dev") {
      setup_dev(rootfs, target, data, nodes, rep);
      dev_done = true;
    } else if (type == "devpts") {
      std::string d = data.empty() ? "newinstance,ptmxmode=0666,mode=0620" : data;
      if (mount("devpts", tp.c_str(), "devpts", MS_NOSUID | MS_NOEXEC, d.c_str()) == 0) {
        std::string ptmx = secure_join(rootfs, "/dev/ptmx");
        unlink(ptmx.c_str());
        if (symlink("pts/ptmx", ptmx.c_str()) != 0) warn("/dev/ptmx: %s", strerror(errno));
      } else {
        rep.notes.push_back(std::string("devpts: ") + strerror(errno));
      }
    } else if (type == "sysfs") {
      if (mount("sysfs", tp.c_str(), "sysfs", flags | MS_NOSUID | MS_NODEV | MS_NOEXEC, nullptr) == 0) {
        rep.sys = "private";
      } else if (rootfs != "/") {
        // a user namespace without its own network namespace may not mount sysfs: bind the
        // host's read-only (HIP reads the KFD topology from /sys/class/kfd)
        if (mount("/sys", tp.c_str(), nullptr, MS_BIND | MS_REC, nullptr) != 0)
          die(126, "bind /sys: %s", strerror(errno));
        bind_remount(target, MS_RDONLY);
        rep.sys = "host-ro";
      }
    } else {
      if (mount(src.empty() ? type.c_str() : src.c_str(), tp.c_str(), type.c_str(), flags, data.empty() ? nullptr : data.c_str()) != 0)
        rep.notes.push_back("mount " + type + " " + dst + ": " + strerror(errno));
    }
  }
  if (!dev_done && !nodes.empty()) {
    // the spec did not ask for a private /dev: expose the host's, but never silently
    rep.notes.push_back("/dev: host view (no tmpfs /dev mount in the spec)");
    for (auto& h : nodes) {
      close(h.fd);
      h.fd = -1;
    }
  }
}

void mask_paths(const J& spec, const std::string& rootfs) {
  for (auto& p : spec["linux"]["maskedPaths"].a) {
    std::string t = secure_join(rootfs, p.s);
    struct stat st;
    if (lstat(t.c_str(), &st) != 0) continue;
    Pinned tp;
    pin(tp, t);
    if (S_ISDIR(st.st_mode)) mount("tmpfs", tp.c_str(), "tmpfs", MS_RDONLY, "size=0");
    else mount("/dev/null", tp.c_str(), nullptr, MS_BIND, nullptr);
  }
  for (auto& p : spec["linux"]["readonlyPaths"].a) {
    std::string t = secure_join(rootfs, p.s);
    if (access(t.c_str(), F_OK) != 0) continue;
    Pinned tp;
    pin(tp, t);
    if (mount(tp.c_str(), tp.c_str(), nullptr, MS_BIND | MS_REC, nullptr) == 0) {
      unsigned long f = MS_BIND | MS_REMOUNT | MS_RDONLY | locked_flags(t);
      mount(nullptr, t.c_str(), nullptr, f, nullptr);
    }
  }
}

void pivot(const std::string& rootfs) {
  if (chdir(rootfs.c_str()) != 0) die(126, "chdir %s: %s", rootfs.c_str(), strerror(errno));
  if (syscall(SYS_pivot_root, ".", ".") != 0) die(126, "pivot_root: %s", strerror(errno));
  if (umount2(".", MNT_DETACH) != 0) die(126, "detaching the old root: %s", strerror(errno));
  if (chdir("/") != 0) die(126, "chdir /: %s", strerror(errno));
}

// ---------------------------------------------------------------------------------------------
// identity
struct Identity {
  uid_t uid = 0;
  gid_t gid = 0;
  std::vector<gid_t> groups;
  bool set = false;
};

Identity identity_of(const J& spec) {
  Identity id;
  const J& u = spec["process"]["user"];
  id.set = u.has("uid");
  id.uid = (uid_t)u["uid"].num(geteuid());
  id.gid = (gid_t)u["gid"].num(getegid());
  for (auto& g : u["additionalGids"].a) id.groups.push_back((gid_t)g.num());
  return id;
}

void apply_identity(const Identity& id, bool user_ns) {
  if (!user_ns) {
    if (geteuid() == 0) {
      if (setgroups(id.groups.size(), id.groups.data()) != 0) die(126, "setgroups: %s", strerror(errno));
    } else if (!id.groups.empty()) {
      warn("not root: supplementary groups left unchanged");
    }
  }
  if (getegid() != id.gid && setgid(id.gid) != 0) die(126, "setgid %u: %s", id.gid, strerror(errno));
  if (geteuid() != id.uid && setuid(id.uid) != 0) die(126, "setuid %u: %s", id.uid, strerror(errno));
}

// ---------------------------------------------------------------------------------------------
// signals
volatile pid_t g_child = -1;

void forward(int sig) {
  if (g_child > 0) kill(g_child, sig);
}

void install_forwarding() {
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_handler = forward;
  sigemptyset(&sa.sa_mask);
  sa.sa_flags = SA_RESTART;
  for (int s : {SIGTERM, SIGINT, SIGHUP, SIGQUIT, SIGUSR1, SIGUSR2, SIGWINCH, SIGCONT})
    sigaction(s, &sa, nullptr);
}

int status_code(int st) {
  if (WIFEXITED(st)) return WEXITSTATUS(st);
  if (WIFSIGNALED(st)) return 128 + WTERMSIG(st);
  return 255;
}

// wait for `child`, reaping anything else (an init reaps orphans), return its exit code
int wait_child(pid_t child) {
  for (;;) {
    int st;
    pid_t w = waitpid(-1, &st, 0);
    if (w < 0) {
      if (errno == EINTR) continue;
      return 255;
    }
    if (w == child) return status_code(st);
  }
}

void exec_entrypoint(const J& spec) {
  const J& proc = spec["process"];
  std::vector<std::string> args, env;
  for (auto& a : proc["args"].a) args.push_back(a.s);
  bool preload_set = false;
  for (auto& e : proc["env"].a) {
    if (!g_devshim.empty() && e.s.compare(0, 11, "LD_PRELOAD=") == 0) {
      env.push_back("LD_PRELOAD=" + with_devshim(e.s.c_str() + 11));
      preload_set = true;
    } else {
      env.push_back(e.s);
    }
  }
  if (!g_devshim.empty() && !preload_set) env.push_back("LD_PRELOAD=" + g_devshim);
  if (!g_devshim.empty()) env.push_back("KAMD_DEVSHIM_DIR=" + g_devshim_dir);
  if (args.empty()) die(126, "process.args is empty");
  std::vector<char*> argv, envp;
  for (auto& a : args) argv.push_back(const_cast<char*>(a.c_str()));
  argv.push_back(nullptr);
  for (auto& e : env) envp.push_back(const_cast<char*>(e.c_str()));
  envp.push_back(nullptr);
  std::string cwd = proc["cwd"].str("/");
  if (chdir(cwd.c_str()) != 0) die(126, "chdir %s: %s", cwd.c_str(), strerror(errno));
  // PATH lookup uses the container's PATH
  for (auto& e : env)
    if (e.compare(0, 5, "PATH=") == 0) setenv("PATH", e.c_str() + 5, 1);
  environ = envp.data();
  execvp(argv[0], argv.data());
  fprintf(stderr, "kamd-runc: exec %s: %s\n", argv[0], strerror(errno));
  _exit(127);
}

std::string json_str(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    if ((unsigned char)c < 0x20) {
      char b[8];
      snprintf(b, sizeof b, "\\u%04x", c);
      o += b;
      continue;
    }
    o += c;
  }
  return o + "\"";
}

std::string report_json(const Report& r, const CgroupState& cg) {
  std::string o = "{";
  auto b = [&](const char* k, bool v) { o += std::string("\"") + k + "\":" + (v ? "true" : "false") + ","; };
  b("user_ns", r.user_ns);
  b("mount_ns", r.mount_ns);
  b("pid_ns", r.pid_ns);
  b("ipc_ns", r.ipc_ns);
  b("uts_ns", r.uts_ns);
  o += "\"tier\":" + json_str(r.tier) + ",";
  if (r.tier == "landlock") o += "\"landlock_rules\":" + std::to_string(r.landlock_rules) + ",";
  if (r.tier == "landlock") b("devshim", r.devshim);
  o += "\"proc\":" + json_str(r.proc) + ",\"dev\":" + json_str(r.dev) + ",\"sys\":" + json_str(r.sys);
  o += ",\"device_cgroup\":" + json_str(cg.mode);
  if (!cg.error.empty()) o += ",\"device_cgroup_error\":" + json_str(cg.error);
  o += ",\"devices\":[";
  for (size_t i = 0; i < r.devices.size(); ++i) o += (i ? "," : "") + json_str(r.devices[i]);
  o += "],\"notes\":[";
  for (size_t i = 0; i < r.notes.size(); ++i) o += (i ? "," : "") + json_str(r.notes[i]);
  return o + "]}";
}

int ns_flag(const std::string& t) {
  if (t == "mount") return CLONE_NEWNS;
  if (t == "pid") return CLONE_NEWPID;
  if (t == "ipc") return CLONE_NEWIPC;
  if (t == "uts") return CLONE_NEWUTS;
  if (t == "network") return CLONE_NEWNET;
  if (t == "user") return CLONE_NEWUSER;
  if (t == "cgroup") return CLONE_NEWCGROUP;
  return 0;
}

bool privileged() { return geteuid() == 0 && has_cap(CAP_SYS_ADMIN); }

void write_id_maps(uid_t inside_uid, gid_t inside_gid, uid_t outside_uid, gid_t outside_gid) {
  char buf[64];
  write_file("/proc/self/setgroups", "deny");
  snprintf(buf, sizeof buf, "%u %u 1\n", inside_uid, outside_uid);
  if (!write_file("/proc/self/uid_map", buf)) die(126, "uid_map: %s", strerror(errno));
  snprintf(buf, sizeof buf, "%u %u 1\n", inside_gid, outside_gid);
  if (!write_file("/proc/self/gid_map", buf)) die(126, "gid_map: %s", strerror(errno));
}

// ---------------------------------------------------------------------------------------------
int cmd_run(const std::string& bundle, int ready_fd) {
  J spec = read_json(bundle + "/config.json");
  std::string root = spec["root"]["path"].str("/");
  if (root.empty()) root = "/";
  if (root[0] != '/') root = bundle + "/" + root;
  // the v1 devices cgroup is named after the bundle: leaf name + a hash of the full bundle path,
  // so two runtimes (different roots) numbering their containers alike never share one
  std::string cid = bundle.substr(bundle.rfind('/') + 1);
  {
    unsigned long long h = 1469598103934665603ULL;        // FNV-1a over the absolute bundle path
    for (unsigned char ch : bundle) { h ^= ch; h *= 1099511628211ULL; }
    char tag[24];
    snprintf(tag, sizeof tag, "-%012llx", h & 0xffffffffffffULL);
    cid += tag;
  }
  const J& proc = spec["process"];
  const J& lin = spec["linux"];

  // -- host-side settings (P) ------------------------------------------------------------------
  std::string cpus = lin["resources"]["cpu"]["cpus"].str();
  if (!cpus.empty()) {
    cpu_set_t set;
    if (parse_cpus(cpus.c_str(), &set) <= 0) die(126, "bad cpuset %s", cpus.c_str());
    if (sched_setaffinity(0, sizeof set, &set) != 0) die(126, "sched_setaffinity: %s", strerror(errno));
  }
  if (proc.has("oomScoreAdj")) write_file("/proc/self/oom_score_adj", std::to_string(proc["oomScoreAdj"].num()));
  for (auto& rl : proc["rlimits"].a) {
    static const std::pair<const char*, int> names[] = {{"RLIMIT_NOFILE", RLIMIT_NOFILE}, {"RLIMIT_NPROC", RLIMIT_NPROC},
                                                        {"RLIMIT_CORE", RLIMIT_CORE}, {"RLIMIT_MEMLOCK", RLIMIT_MEMLOCK},
                                                        {"RLIMIT_STACK", RLIMIT_STACK}};
    for (auto& n : names)
      if (rl["type"].s == n.first) {
        struct rlimit r = {(rlim_t)rl["soft"].num(), (rlim_t)rl["hard"].num()};
        if (setrlimit(n.second, &r) != 0) warn("%s: %s", n.first, strerror(errno));
      }
  }
  CgroupState cg;
  setup_cgroups(spec, cid, cg);
  Identity id = identity_of(spec);

  // -- namespaces --------------------------------------------------------------------------------
  Report rep;
  int flags = 0;
  std::vector<std::pair<int, std::string>> join_ns;  // (flag, path)
  for (auto& n : lin["namespaces"].a) {
    int f = ns_flag(n["type"].str());
    if (!f) continue;
    if (n.has("path")) join_ns.emplace_back(f, n["path"].str());
    else flags |= f;
  }
  uid_t out_uid = geteuid();
  gid_t out_gid = getegid();
  bool priv = privileged();
  bool joined_user = false;
  // user namespace first: joining one grants the rights to join the rest
  for (auto& j : join_ns)
    if (j.first == CLONE_NEWUSER) {
      int fd = open(j.second.c_str(), O_RDONLY | O_CLOEXEC);
      if (fd < 0 || setns(fd, CLONE_NEWUSER) != 0) die(126, "joining user namespace %s: %s", j.second.c_str(), strerror(errno));
      close(fd);
      joined_user = true;
    }
  for (auto& j : join_ns) {
    if (j.first == CLONE_NEWUSER) continue;
    int fd = open(j.second.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0 || setns(fd, j.first) != 0) die(126, "joining namespace %s: %s", j.second.c_str(), strerror(errno));
    close(fd);
  }
  bool new_user = (flags & CLONE_NEWUSER) || (!priv && !joined_user && (flags & ~CLONE_NEWUSER));
  if (new_user) flags |= CLONE_NEWUSER;
  if (flags && unshare(flags) != 0) die(126, "unshare: %s", strerror(errno));
  if (new_user) {
    // the container's uid/gid map onto the caller's: nothing outside gains a privilege
    write_id_maps(id.uid, id.gid, out_uid, out_gid);
  }
  rep.user_ns = new_user || joined_user;
  rep.mount_ns = flags & CLONE_NEWNS;
  rep.pid_ns = flags & CLONE_NEWPID;
  rep.ipc_ns = flags & CLONE_NEWIPC;
  rep.uts_ns = flags & CLONE_NEWUTS;
  for (auto& j : join_ns) {
    if (j.first == CLONE_NEWIPC) rep.ipc_ns = true;
    if (j.first == CLONE_NEWUTS) rep.uts_ns = true;
  }

  // sync pipe C -> P: "ok" after setup, or an error message
  int sync[2];
  if (pipe2(sync, O_CLOEXEC) != 0) die(126, "pipe: %s", strerror(errno));
  std::vector<HostNode> nodes = rep.mount_ns ? open_host_nodes(spec) : std::vector<HostNode>{};
  pid_t parent = getpid();
  pid_t c = fork();
  if (c < 0) die(126, "fork: %s", strerror(errno));
  if (c == 0) {
    close(sync[0]);
    if (ready_fd >= 0) close(ready_fd);  // P's alone: the kubelet reads it to EOF
    // die with P (P is what the kubelet signals / kills)
    prctl(PR_SET_PDEATHSIG, SIGKILL);
    // (in a new pid namespace the parent is outside it and getppid() reads 0)
    if (!rep.pid_ns && getppid() != parent) _exit(137);
    setpgid(0, 0);
    if (rep.mount_ns) {
      if (mount(nullptr, "/", nullptr, MS_REC | MS_PRIVATE, nullptr) != 0) die(126, "making / private: %s", strerror(errno));
      const J& ann = spec["annotations"];
      if (root != "/" && ann.has("kamd.io/rootfs-lower")) {
        // image rootfs: a copy-on-write overlay of the unpacked image (read-only lower) and the
        // container's own upper layer, mounted only inside this mount namespace
        std::string opts = "lowerdir=" + ann["kamd.io/rootfs-lower"].str() + ",upperdir=" +
                           ann["kamd.io/rootfs-upper"].str() + ",workdir=" + ann["kamd.io/rootfs-work"].str();
        if (mount("overlay", root.c_str(), "overlay", 0, opts.c_str()) != 0)
          die(126, "overlay rootfs %s: %s", root.c_str(), strerror(errno));
      } else if (root != "/") {
        if (mount(root.c_str(), root.c_str(), nullptr, MS_BIND | MS_REC, nullptr) != 0)
          die(126, "bind rootfs %s: %s", root.c_str(), strerror(errno));
      }
      if (root != "/") {
        char real[PATH_MAX];
        if (!realpath(root.c_str(), real)) die(126, "realpath %s: %s", root.c_str(), strerror(errno));
        g_root_real = real;
      }
      do_mounts(spec, root, nodes, rep);
      mask_paths(spec, root);
      if (root != "/") pivot(root);
      if (spec["root"]["readonly"].boolean()) bind_remount("/", MS_RDONLY);
    }
    if (rep.uts_ns && spec.has("hostname")) {
      std::string h = spec["hostname"].str();
      if (sethostname(h.c_str(), h.size()) != 0) warn("sethostname: %s", strerror(errno));
    }
    if (rep.mount_ns && rep.dev == "private") rep.tier = "namespaces";
    const J& ann2 = spec["annotations"];
    if (!rep.mount_ns && ann2["kamd.io/isolation-tier"].str() == "landlock") {
      // Landlock tier: the spec's device nodes under the restricted directory are the only
      // ones there this container may open
      std::string dir = ann2["kamd.io/landlock-dir"].str("/dev/dri");
      std::vector<std::string> allowed;
      for (auto& d : spec["linux"]["devices"].a) {
        allowed.push_back(d["kamd.io/host-path"].str(d["path"].str().c_str()));
        rep.devices.push_back(d["path"].str());
      }
      std::string e = landlock_restrict(dir, allowed, &rep.landlock_rules);
      if (!e.empty()) die(126, "landlock: %s", e.c_str());
      rep.tier = "landlock";
      rep.dev = "host (landlock: " + dir + " limited to the allocated nodes)";
      if (ann2["kamd.io/devshim"].str("true") != "false") {
        g_devshim = devshim_path();
        g_devshim_dir = dir;
        if (g_devshim.empty()) rep.notes.push_back("devshim: libkamd_devshim.so not found; denied GPU nodes read EACCES");
      }
      rep.devshim = !g_devshim.empty();
    }
    // the bundle path may be gone after pivot_root: the report goes to P over the sync pipe
    std::string report = report_json(rep, cg);
    // bounding set first: dropping needs CAP_SETPCAP, which a setuid away from root loses
    const J& caps = proc["capabilities"];
    if (caps.has("bounding")) restrict_bounding(caps_from(caps["bounding"]), cg.mode == "none");
    apply_identity(id, rep.user_ns);
    if (proc["noNewPrivileges"].boolean()) prctl(PR_SET_NO_NEW_PRIVS, 1, 0, 0, 0);
    prctl(PR_SET_PDEATHSIG, SIGKILL);  // identity changes cleared it
    std::string msg = "ok " + report + "\n";
    if (write(sync[1], msg.data(), msg.size()) < 0) _exit(126);
    close(sync[1]);
    if (!rep.pid_ns) exec_entrypoint(spec);
    // pid 1 of the container: fork the entrypoint, reap, forward signals
    pid_t g = fork();
    if (g < 0) die(126, "fork: %s", strerror(errno));
    if (g == 0) {
      signal(SIGCHLD, SIG_DFL);
      exec_entrypoint(spec);
    }
    g_child = g;
    install_forwarding();
    _exit(wait_child(g));
  }
  close(sync[1]);
  for (auto& h : nodes)
    if (h.fd >= 0) close(h.fd);
  g_child = c;
  install_forwarding();
  // read C's setup result (an error text arrives on C's stderr and as EOF without "ok")
  std::string got;
  char buf[4096];
  ssize_t r;
  while ((r = read(sync[0], buf, sizeof buf)) != 0) {
    if (r < 0) {
      if (errno == EINTR) continue;
      break;
    }
    got.append(buf, (size_t)r);
  }
  close(sync[0]);
  if (got.compare(0, 3, "ok ") == 0) {
    std::string report = got.substr(3);
    while (!report.empty() && report.back() == '\n') report.pop_back();
    write_file(bundle + "/isolation.json", report + "\n", O_CREAT | O_TRUNC);
    if (ready_fd >= 0) {
      std::string line = std::to_string(c) + " " + report + "\n";
      if (write(ready_fd, line.data(), line.size()) < 0) warn("ready fd: %s", strerror(errno));
    }
  }
  if (ready_fd >= 0) close(ready_fd);
  int code = wait_child(c);
  cleanup_cgroups(cg);
  return code;
}

// enter a running container (CRI ExecSync / streaming exec): its user namespace first (when it
// has one of its own), then ipc, uts, net, pid and mount; fork so the pid namespace applies.
int cmd_exec(pid_t target, const std::string& cwd, const std::string& user, const std::string& landlock,
             char** argv) {
  const char* order[] = {"user", "ipc", "uts", "net", "pid", "mnt"};
  const int flags[] = {CLONE_NEWUSER, CLONE_NEWIPC, CLONE_NEWUTS, CLONE_NEWNET, CLONE_NEWPID, CLONE_NEWNS};
  int fds[6];
  for (int i = 0; i < 6; ++i) {
    char p[64], q[64];
    snprintf(p, sizeof p, "/proc/%d/ns/%s", (int)target, order[i]);
    snprintf(q, sizeof q, "/proc/self/ns/%s", order[i]);
    struct stat a, b;
    fds[i] = -1;
    if (stat(p, &a) != 0) die(126, "container %d: %s", (int)target, strerror(errno));
    if (stat(q, &b) == 0 && a.st_ino == b.st_ino && a.st_dev == b.st_dev) continue;  // shared with us
    fds[i] = open(p, O_RDONLY | O_CLOEXEC);
    if (fds[i] < 0) die(126, "open %s: %s", p, strerror(errno));
  }
  // capability bounding set of the container's init: the exec'd process gets no more
  std::string status = read_small("/proc/" + std::to_string(target) + "/status");
  unsigned long long bnd = ~0ULL;
  size_t at = status.find("CapBnd:");
  if (at != std::string::npos) bnd = strtoull(status.c_str() + at + 7, nullptr, 16);
  bool user_ns = fds[0] >= 0;
  for (int i = 0; i < 6; ++i)
    if (fds[i] >= 0) {
      if (setns(fds[i], flags[i]) != 0) die(126, "setns %s: %s", order[i], strerror(errno));
      close(fds[i]);
    }
  pid_t c = fork();
  if (c < 0) die(126, "fork: %s", strerror(errno));
  if (c == 0) {
    prctl(PR_SET_PDEATHSIG, SIGKILL);
    std::vector<bool> keep(64, false);
    for (int k = 0; k < 64; ++k) keep[k] = (bnd >> k) & 1;
    restrict_bounding(keep, false);
    if (!user.empty()) {
      Identity id;
      id.uid = (uid_t)strtoul(user.c_str(), nullptr, 10);
      size_t colon = user.find(':');
      id.gid = colon == std::string::npos ? getegid() : (gid_t)strtoul(user.c_str() + colon + 1, nullptr, 10);
      apply_identity(id, user_ns);
    }

    prctl(PR_SET_NO_NEW_PRIVS, 1, 0, 0, 0);
    if (!landlock.empty()) {
      // a Landlock-tier container: the exec'd process gets the container's ruleset
      size_t c2 = landlock.find(':');
      std::string dir = landlock.substr(0, c2);
      std::vector<std::string> allowed;
      if (c2 != std::string::npos) {
        std::string rest = landlock.substr(c2 + 1);
        size_t i = 0;
        while (i <= rest.size()) {
          size_t j = rest.find(',', i);
          if (j == std::string::npos) j = rest.size();
          if (j > i) allowed.push_back(rest.substr(i, j - i));
          i = j + 1;
        }
      }
      std::string e = landlock_restrict(dir, allowed, nullptr);
      if (!e.empty()) die(126, "landlock: %s", e.c_str());
      g_devshim = devshim_path();
      if (!g_devshim.empty()) {
        setenv("LD_PRELOAD", with_devshim(getenv("LD_PRELOAD")).c_str(), 1);
        setenv("KAMD_DEVSHIM_DIR", dir.c_str(), 1);
      }
    }
    if (chdir(cwd.empty() ? "/" : cwd.c_str()) != 0) die(126, "chdir %s: %s", cwd.c_str(), strerror(errno));
    execvp(argv[0], argv);
    fprintf(stderr, "kamd-runc: exec %s: %s\n", argv[0], strerror(errno));
    _exit(127);
  }
  g_child = c;
  install_forwarding();
  return wait_child(c);
}

// what this host lets the runtime enforce, probed in a throwaway child
int cmd_features(const std::string& cgroup_dir) {
  bool priv = privileged();
  int p[2];
  if (pipe(p) != 0) return 1;
  pid_t c = fork();
  if (c == 0) {
    close(p[0]);
    std::string out;
    uid_t u = geteuid();
    gid_t g = getegid();
    int flags = CLONE_NEWNS | CLONE_NEWPID | CLONE_NEWIPC | CLONE_NEWUTS | (priv ? 0 : CLONE_NEWUSER);
    bool ns = unshare(flags) == 0;
    std::string err = ns ? "" : strerror(errno);
    if (ns && !priv) write_id_maps(u, g, u, g);
    bool tmpfs = false;
    if (ns) {
      mount(nullptr, "/", nullptr, MS_REC | MS_PRIVATE, nullptr);
      tmpfs = mount("tmpfs", "/tmp", "tmpfs", MS_NODEV, "size=4k") == 0;
      if (!tmpfs) err = std::string("tmpfs: ") + strerror(errno);
    }
    out = std::string(ns ? "1" : "0") + (tmpfs ? "1" : "0") + " " + err;
    if (write(p[1], out.data(), out.size()) < 0) _exit(1);
    _exit(0);
  }
  close(p[1]);
  char buf[512] = {0};
  ssize_t r = read(p[0], buf, sizeof buf - 1);
  (void)r;
  close(p[0]);
  int st;
  waitpid(c, &st, 0);
  bool ns = buf[0] == '1', tmpfs = buf[1] == '1';
  std::string err = strlen(buf) > 3 ? std::string(buf + 3) : "";
  // device cgroup: BPF on cgroup v2 (program load needs CAP_SYS_ADMIN / CAP_BPF), else v1 devices
  std::string dc = "none", dc_err;
  std::vector<DevRule> rules = default_rules();
  if (!cgroup_dir.empty() && is_cgroup2(cgroup_dir)) {
    std::string log;
    int fd = bpf_load_device_prog(rules, &log);
    if (fd >= 0) {
      dc = access(cgroup_dir.c_str(), W_OK) == 0 ? "bpf" : "none";
      if (dc == "none") dc_err = "cgroup " + cgroup_dir + " not writable";
      close(fd);
    } else {
      dc_err = std::string("BPF_PROG_LOAD: ") + strerror(errno);
    }
  }
  if (dc == "none" && is_cgroup1(V1_DEVICES) && access((std::string(V1_DEVICES) + "/devices.allow").c_str(), W_OK) == 0)
    dc = "v1";
  else if (dc == "none" && dc_err.empty())
    dc_err = "no writable device cgroup (v2 BPF or v1 devices)";
  printf("{\"privileged\":%s,\"user_ns\":%s,\"mount_ns\":%s,\"private_dev\":%s,\"device_cgroup\":%s",
         priv ? "true" : "false", (!priv && ns) ? "true" : "false", ns ? "true" : "false", tmpfs ? "true" : "false",
         json_str(dc).c_str());
  if (!err.empty()) printf(",\"namespace_error\":%s", json_str(err).c_str());
  if (!dc_err.empty()) printf(",\"device_cgroup_error\":%s", json_str(dc_err).c_str());
  // Landlock is probed in the same throwaway way: a ruleset restricting a scratch directory is
  // created and enforced in a child (no_new_privs, nothing else) — a kernel that lists the LSM
  // but refuses restrict_self (seccomp, old ABI) reads as unavailable
  int abi = landlock_abi();
  std::string ll_err;
  if (abi > 0) {
    int q[2];
    if (pipe(q) == 0) {
      pid_t lc = fork();
      if (lc == 0) {
        close(q[0]);
        std::string e = landlock_restrict("/dev", {}, nullptr);
        if (write(q[1], e.data(), e.size()) < 0) _exit(1);
        _exit(0);
      }
      close(q[1]);
      char eb[256] = {0};
      ssize_t er = read(q[0], eb, sizeof eb - 1);
      (void)er;
      close(q[0]);
      int lst;
      waitpid(lc, &lst, 0);
      ll_err = eb;
      if (!ll_err.empty()) abi = 0;
    }
  } else {
    ll_err = "landlock_create_ruleset: not supported by this kernel";
  }
  printf(",\"landlock\":%d", abi);
  if (!ll_err.empty()) printf(",\"landlock_error\":%s", json_str(ll_err).c_str());
  const char* tier = (ns && tmpfs) ? "namespaces" : abi > 0 ? "landlock" : "none";
  printf(",\"tier\":\"%s\",\"isolation\":%s}\n", tier, (ns && tmpfs) ? "true" : "false");
  return 0;
}

void usage() {
  fprintf(stderr,
          "usage: kamd-runc features [--cgroup DIR]\n"
          "       kamd-runc run --bundle DIR [--ready-fd N]\n"
          "       kamd-runc exec --pid PID [--cwd DIR] [--user UID[:GID]] [--landlock DIR:NODE,...] -- argv...\n");
  _exit(126);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) usage();
  std::string cmd = argv[1];
  if (cmd == "features") {
    std::string cg;
    for (int i = 2; i + 1 < argc; ++i)
      if (!strcmp(argv[i], "--cgroup")) cg = argv[++i];
    return cmd_features(cg);
  }
  if (cmd == "run") {
    std::string bundle;
    int ready = -1;
    for (int i = 2; i < argc; ++i) {
      if (!strcmp(argv[i], "--bundle") && i + 1 < argc) bundle = argv[++i];
      else if (!strcmp(argv[i], "--ready-fd") && i + 1 < argc) ready = atoi(argv[++i]);
      else usage();
    }
    if (bundle.empty()) usage();
    char abs[PATH_MAX];
    if (!realpath(bundle.c_str(), abs)) die(126, "bundle %s: %s", bundle.c_str(), strerror(errno));
    return cmd_run(abs, ready);
  }
  if (cmd == "exec") {
    pid_t pid = 0;
    std::string cwd, user, landlock;
    int i = 2;
    for (; i < argc; ++i) {
      if (!strcmp(argv[i], "--")) { ++i; break; }
      if (i + 1 >= argc) usage();
      if (!strcmp(argv[i], "--pid")) pid = (pid_t)atoi(argv[++i]);
      else if (!strcmp(argv[i], "--cwd")) cwd = argv[++i];
      else if (!strcmp(argv[i], "--user")) user = argv[++i];
      else if (!strcmp(argv[i], "--landlock")) landlock = argv[++i];
      else usage();
    }
    if (pid <= 0 || i >= argc) usage();
    return cmd_exec(pid, cwd, user, landlock, argv + i);
  }
  usage();
}
