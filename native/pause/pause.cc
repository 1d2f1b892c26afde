// pause — PID 1 of every pod sandbox.
//
// Same contract as the reference's build/pause/pause.c:24-51: SIGINT/SIGTERM exit(0),
// SIGCHLD reaps every exited child (so orphans re-parented to the sandbox never become
// zombies), and otherwise the process sleeps forever. Built static (-static -Os).
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <unistd.h>

static void on_term(int sig) {
  (void)sig;
  _exit(0);
}

static void on_chld(int sig) {
  (void)sig;
  while (waitpid(-1, nullptr, WNOHANG) > 0) {
  }
}

int main(int argc, char** argv) {
  if (argc > 1 && strcmp(argv[1], "-v") == 0) {
    printf("pause.cc (kubernetes-amd) 1.0\n");
    return 0;
  }
  if (getpid() != 1) fprintf(stderr, "Warning: pause should be the first process\n");
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_handler = on_term;
  if (sigaction(SIGINT, &sa, nullptr) < 0 || sigaction(SIGTERM, &sa, nullptr) < 0) return 1;
  sa.sa_handler = on_chld;
  sa.sa_flags = SA_NOCLDSTOP;
  if (sigaction(SIGCHLD, &sa, nullptr) < 0) return 2;
  for (;;) pause();
  return 42;
}
