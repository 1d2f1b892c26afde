// oci_devices — device-injection helper for the container runtime hook.
//
// Given the host device nodes the amd.com/gpu plugin assigned to a container (always the
// shared /dev/kfd plus one /dev/dri/renderD<minor> per GPU, optionally /dev/dri/card<n>),
// stat() each node and emit the OCI runtime-spec fragments a runtime needs:
//   "devices":   [{"path","type","major","minor","fileMode","uid","gid"}]   (linux.devices)
//   "allow":     [{"allow":true,"type":"c","major":226,"minor":128,"access":"rwm"}] (cgroup rules)
// This is what nvidia-container-runtime's prestart hook did for /dev/nvidia* (char major 195,
// reference vendor/github.com/google/cadvisor/accelerators/nvidia.go:198); on MI355X there is
// no vendor runtime: DRM render nodes are char major 226 and /dev/kfd has a dynamic major.
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>
#include <sys/sysmacros.h>

#include <string>

static void append_json_str(std::string& o, const char* s) {
  o += '"';
  for (; *s; ++s) {
    if (*s == '"' || *s == '\\') o += '\\';
    o += *s;
  }
  o += '"';
}

extern "C" {

// paths: newline-separated list. access: cgroup access string ("rwm", "rw").
// Writes a JSON object into out (NUL-terminated). Returns bytes written (excluding NUL),
// -1 if out is too small, or -(100+i) if the i-th path could not be stat()ed / is not a device.
int kamd_oci_devices(const char* paths, const char* access, char* out, int len) {
  std::string devs = "[", allow = "[";
  int i = 0;
  const char* p = paths;
  bool first = true;
  while (p && *p) {
    const char* nl = strchr(p, '\n');
    std::string path = nl ? std::string(p, nl - p) : std::string(p);
    p = nl ? nl + 1 : nullptr;
    if (path.empty()) continue;
    struct stat st;
    if (stat(path.c_str(), &st) != 0) return -(100 + i);
    char type;
    if (S_ISCHR(st.st_mode)) type = 'c';
    else if (S_ISBLK(st.st_mode)) type = 'b';
    else return -(100 + i);
    char buf[256];
    if (!first) { devs += ','; allow += ','; }
    first = false;
    devs += "{\"path\":";
    append_json_str(devs, path.c_str());
    snprintf(buf, sizeof buf, ",\"type\":\"%c\",\"major\":%u,\"minor\":%u,\"fileMode\":%u,\"uid\":%u,\"gid\":%u}", type,
             major(st.st_rdev), minor(st.st_rdev), (unsigned)(st.st_mode & 07777), (unsigned)st.st_uid, (unsigned)st.st_gid);
    devs += buf;
    snprintf(buf, sizeof buf, "{\"allow\":true,\"type\":\"%c\",\"major\":%u,\"minor\":%u,\"access\":", type,
             major(st.st_rdev), minor(st.st_rdev));
    allow += buf;
    append_json_str(allow, access && *access ? access : "rwm");
    allow += '}';
    ++i;
  }
  std::string o = "{\"devices\":" + devs + "],\"allow\":" + allow + "]}";
  if ((int)o.size() + 1 > len) return -1;
  memcpy(out, o.c_str(), o.size() + 1);
  return (int)o.size();
}

}  // extern "C"
