// orphan — test helper (reference build/pause/orphan.c:22-36): forks a child that outlives
// its parent, so the child is re-parented to the sandbox's PID 1 and must be reaped by it.
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

int main(int argc, char** argv) {
  unsigned delay = argc > 1 ? (unsigned)atoi(argv[1]) : 1;
  pid_t pid = fork();
  if (pid < 0) return 1;
  if (pid == 0) {
    sleep(delay);  // child keeps running after the parent exits
    printf("orphan child %d exiting\n", getpid());
    return 0;
  }
  printf("parent %d exiting, child %d orphaned\n", getpid(), pid);
  return 0;
}
