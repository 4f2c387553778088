/* Native backtrace on SIGSEGV for diagnosing host faults inside the HIP runtime (the round-5
 * graph-replay fault): prints every frame as module + offset (dladdr), then hands
 * the signal to the handler installed before it (Python's faulthandler, which prints the
 * Python stack).  Debug tooling only, not part of liboflow.
 *   gcc -O1 -g -shared -fPIC tools/crash_bt.c -o tools/libcrashbt.so -ldl
 * tests/conftest.py loads it when OFLOW_NATIVE_BT=1. */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <sys/resource.h>
#include <unistd.h>

static struct sigaction g_prev;

static void on_segv(int sig, siginfo_t* si, void* uc) {
  void* fr[64];
  int n = backtrace(fr, 64);
  char line[512];
  int len = snprintf(line, sizeof line, "\n[crash_bt] signal %d at address %p, %d frames\n", sig,
                     si ? si->si_addr : 0, n);
  write(2, line, len);
  for (int i = 0; i < n; ++i) {
    Dl_info d;
    memset(&d, 0, sizeof d);
    if (dladdr(fr[i], &d) && d.dli_fname) {
      len = snprintf(line, sizeof line, "[crash_bt] #%02d %s +0x%lx (%s)\n", i, d.dli_fname,
                     (unsigned long)((char*)fr[i] - (char*)d.dli_fbase),
                     d.dli_sname ? d.dli_sname : "?");
    } else {
      len = snprintf(line, sizeof line, "[crash_bt] #%02d %p\n", i, fr[i]);
    }
    write(2, line, len);
  }
  struct rlimit rl;
  if (getrlimit(RLIMIT_STACK, &rl) == 0) {
    len = snprintf(line, sizeof line, "[crash_bt] stack limit %ld KiB, fault %ld KiB below this "
                   "frame\n", (long)(rl.rlim_cur / 1024),
                   (long)(((char*)&rl - (char*)(si ? si->si_addr : 0)) / 1024));
    write(2, line, len);
  }
  sigaction(SIGSEGV, &g_prev, NULL);       /* the previous handler runs on the re-fault */
  (void)uc;
}

int crash_bt_install(void) {
  /* an alternate signal stack: a fault that is a stack overflow still gets its backtrace */
  static char altstack[1 << 20];
  stack_t ss;
  memset(&ss, 0, sizeof ss);
  ss.ss_sp = altstack;
  ss.ss_size = sizeof altstack;
  if (sigaltstack(&ss, NULL) != 0) return -1;
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = on_segv;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigemptyset(&sa.sa_mask);
  return sigaction(SIGSEGV, &sa, &g_prev);
}
