// container-init — applies a container's process attributes, then execs its entrypoint.
//
// The process runtime's counterpart of an OCI runtime's init step (runc init): the kubelet's
// process runtime starts every container through this helper instead of running a Python
// pre-exec hook in the forked child, so the kubelet can spawn with vfork/posix_spawn (a
// pre-exec hook forces a full fork of the kubelet's address space, ~5x the spawn CPU).
//
//   container-init [-c CPULIST] [-o OOM_SCORE_ADJ] [-g CGROUP_DIR] [-u UID] [-G GID] [-S G1,G2]
//                  -- argv...
//
// CPULIST is a cpuset list ("0-3,8"); pinning failures are fatal (the cpu manager promised
// those CPUs), OOM score and cgroup failures are not (an unprivileged kubelet may only raise
// oom_score_adj and may not own a cgroup subtree). CGROUP_DIR is the container's own cgroup
// (a leaf under the pod cgroup, created here): cgroup v2 forbids processes in the pod cgroup
// itself once it delegates controllers to children. -S sets the supplemental groups (the pod's
// fsGroup + supplementalGroups, kuberuntime/security_context.go:58-66); a non-root caller that
// cannot change them keeps its own and warns instead of failing. A uid/gid equal to the current
// one needs no privilege. Exit 127 when the entrypoint cannot be executed, like a shell.
#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <grp.h>
#include <sys/stat.h>
#include <unistd.h>

static int parse_cpus(const char* s, cpu_set_t* set) {
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

static void write_file(const char* path, const char* val, int extra_flags) {
  int fd = open(path, O_WRONLY | O_CLOEXEC | extra_flags, 0644);
  if (fd < 0) return;
  ssize_t r = write(fd, val, strlen(val));
  (void)r;
  close(fd);
}

int main(int argc, char** argv) {
  const char* cpus = nullptr;
  const char* oom = nullptr;
  const char* cgroup = nullptr;
  const char* uid = nullptr;   // securityContext.runAsUser
  const char* gid = nullptr;   // primary group (runAsGroup)
  const char* groups = nullptr;  // supplemental groups
  int i = 1;
  for (; i < argc; ++i) {
    if (strcmp(argv[i], "--") == 0) { ++i; break; }
    if (i + 1 >= argc) { fprintf(stderr, "container-init: %s needs a value\n", argv[i]); return 126; }
    if (strcmp(argv[i], "-c") == 0) cpus = argv[++i];
    else if (strcmp(argv[i], "-o") == 0) oom = argv[++i];
    else if (strcmp(argv[i], "-g") == 0) cgroup = argv[++i];
    else if (strcmp(argv[i], "-u") == 0) uid = argv[++i];
    else if (strcmp(argv[i], "-G") == 0) gid = argv[++i];
    else if (strcmp(argv[i], "-S") == 0) groups = argv[++i];
    else { fprintf(stderr, "container-init: unknown option %s\n", argv[i]); return 126; }
  }
  if (i >= argc) { fprintf(stderr, "container-init: no command\n"); return 126; }
  if (cpus && *cpus) {
    cpu_set_t set;
    if (parse_cpus(cpus, &set) <= 0) { fprintf(stderr, "container-init: bad cpuset %s\n", cpus); return 126; }
    if (sched_setaffinity(0, sizeof set, &set) != 0) { perror("container-init: sched_setaffinity"); return 126; }
  }
  if (oom && *oom) write_file("/proc/self/oom_score_adj", oom, 0);
  if (cgroup && *cgroup) {
    mkdir(cgroup, 0755);
    char path[4096];
    if (snprintf(path, sizeof path, "%s/cgroup.procs", cgroup) < (int)sizeof path) write_file(path, "0", O_CREAT | O_TRUNC);
  }
  // identity last: the cgroup / OOM writes above may need the kubelet's privileges. Groups before
  // gid before uid (setuid drops the right to change the others).
  gid_t want[64];
  int nwant = 0;
  if (groups) {
    for (const char* p = groups; *p && nwant < 64;) {
      char* end;
      unsigned long g = strtoul(p, &end, 10);
      if (end == p) { fprintf(stderr, "container-init: bad group list %s\n", groups); return 126; }
      want[nwant++] = (gid_t)g;
      p = *end == ',' ? end + 1 : end;
    }
  }
  if (groups || (gid && *gid) || (uid && *uid)) {
    if (geteuid() == 0) {
      if (setgroups(nwant, want) != 0) { perror("container-init: setgroups"); return 126; }
    } else if (nwant) {
      gid_t have[256];
      int n = getgroups(256, have);
      for (int k = 0; k < nwant; ++k) {
        bool found = want[k] == getegid();
        for (int j = 0; j < n && !found; ++j) found = have[j] == want[k];
        if (!found) fprintf(stderr, "container-init: warning: not root, supplemental group %u not added\n", want[k]);
      }
    }
  }
  if (gid && *gid) {
    gid_t g = (gid_t)strtoul(gid, nullptr, 10);
    if (g != getegid() && setgid(g) != 0) {
      perror("container-init: setgid");
      return 126;
    }
  }
  if (uid && *uid) {
    uid_t u = (uid_t)strtoul(uid, nullptr, 10);
    if (u != geteuid() && setuid(u) != 0) {
      perror("container-init: setuid");
      return 126;
    }
  }
  execvp(argv[i], argv + i);
  fprintf(stderr, "container-init: exec %s: %s\n", argv[i], strerror(errno));
  return 127;
}
