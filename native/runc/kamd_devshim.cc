// libkamd_devshim.so — preloaded into Landlock-tier containers by kamd-runc.
//
// Why: the MI355X user-space stack (libhsakmt inside ROCr) enumerates every GPU in the KFD
// topology and opens each one's /dev/dri/renderD* node. A node it may not open is skipped when
// the open fails with ENOENT (node absent: a private /dev) or EPERM (device cgroup denial: the
// namespaces tier, Docker, the reference's device plugin), but any other errno aborts HSA
// initialisation with HSA_STATUS_ERROR_OUT_OF_RESOURCES (measured on the MI355X pool:
// profiles/r5_gpu/README.md, test_isolation.py::test_rocr_start_under_landlock_denial).
// Landlock denies with EACCES. So in the Landlock tier — no namespaces, no cgroup device
// control — a container confined to GPU k would fail HIP init because its sibling GPUs' nodes
// are EACCES.
//
// What: an open of a node under the restricted directory (/dev/dri; kamd-runc passes it in
// KAMD_DEVSHIM_DIR) that fails with EACCES is reported as EPERM,
// exactly what the same container would see under device-cgroup confinement. Nothing else
// changes: the kernel (Landlock) still refuses the open, every other path and errno passes
// through untouched, and a successful open is returned as is.
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <stdarg.h>
#include <stdlib.h>
#include <string.h>
#include <sys/types.h>

#include <string>

namespace {

// the Landlock-restricted directory, from kamd-runc (KAMD_DEVSHIM_DIR, default /dev/dri),
// read once before main() — the container may change its own environment later
std::string& restricted_dir() {
  static std::string dir = [] {
    const char* d = getenv("KAMD_DEVSHIM_DIR");
    std::string s = d && *d ? d : "/dev/dri";
    if (s.back() != '/') s += '/';
    return s;
  }();
  return dir;
}

__attribute__((constructor)) void init_dir() { restricted_dir(); }

bool is_drm_node(const char* p) {
  const std::string& d = restricted_dir();
  return p != nullptr && strncmp(p, d.c_str(), d.size()) == 0;
}

int translate(int rc, const char* path) {
  if (rc < 0 && errno == EACCES && is_drm_node(path)) errno = EPERM;
  return rc;
}

template <typename F>
F next(const char* name) {
  return reinterpret_cast<F>(dlsym(RTLD_NEXT, name));
}

bool wants_mode(int flags) {
#ifdef O_TMPFILE
  if ((flags & O_TMPFILE) == O_TMPFILE) return true;
#endif
  return (flags & O_CREAT) != 0;
}

using open_fn = int (*)(const char*, int, ...);
using openat_fn = int (*)(int, const char*, int, ...);
using open2_fn = int (*)(const char*, int);
using openat2_fn = int (*)(int, const char*, int);

}  // namespace

extern "C" {

#define KAMD_OPEN(NAME)                                                     \
  int NAME(const char* path, int flags, ...) {                              \
    static open_fn real = next<open_fn>(#NAME);                             \
    mode_t mode = 0;                                                        \
    if (wants_mode(flags)) {                                                \
      va_list ap;                                                           \
      va_start(ap, flags);                                                  \
      mode = va_arg(ap, mode_t);                                            \
      va_end(ap);                                                           \
    }                                                                       \
    if (real == nullptr) {                                                  \
      errno = ENOSYS;                                                       \
      return -1;                                                            \
    }                                                                       \
    return translate(real(path, flags, mode), path);                        \
  }

#define KAMD_OPENAT(NAME)                                                   \
  int NAME(int dirfd, const char* path, int flags, ...) {                   \
    static openat_fn real = next<openat_fn>(#NAME);                         \
    mode_t mode = 0;                                                        \
    if (wants_mode(flags)) {                                                \
      va_list ap;                                                           \
      va_start(ap, flags);                                                  \
      mode = va_arg(ap, mode_t);                                            \
      va_end(ap);                                                           \
    }                                                                       \
    if (real == nullptr) {                                                  \
      errno = ENOSYS;                                                       \
      return -1;                                                            \
    }                                                                       \
    return translate(real(dirfd, path, flags, mode), path);                 \
  }

// _FORTIFY_SOURCE entry points (`open(path, flags)` compiled with fortification)
#define KAMD_OPEN2(NAME)                                                    \
  int NAME(const char* path, int flags) {                                   \
    static open2_fn real = next<open2_fn>(#NAME);                           \
    if (real == nullptr) {                                                  \
      errno = ENOSYS;                                                       \
      return -1;                                                            \
    }                                                                       \
    return translate(real(path, flags), path);                              \
  }

#define KAMD_OPENAT2(NAME)                                                  \
  int NAME(int dirfd, const char* path, int flags) {                        \
    static openat2_fn real = next<openat2_fn>(#NAME);                       \
    if (real == nullptr) {                                                  \
      errno = ENOSYS;                                                       \
      return -1;                                                            \
    }                                                                       \
    return translate(real(dirfd, path, flags), path);                       \
  }

KAMD_OPEN(open)
KAMD_OPEN(open64)
KAMD_OPENAT(openat)
KAMD_OPENAT(openat64)
KAMD_OPEN2(__open_2)
KAMD_OPEN2(__open64_2)
KAMD_OPENAT2(__openat_2)
KAMD_OPENAT2(__openat64_2)

}  // extern "C"
