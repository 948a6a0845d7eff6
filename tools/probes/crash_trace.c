/* crash_trace.c — diagnostic only (bench.py loads it when FME_CRASH_TRACE is set): on SIGSEGV /
 * SIGBUS / SIGABRT print the native stack (backtrace_symbols_fd, plus the shared object and offset
 * of each frame from dladdr) to stderr, then re-raise with the default action.  Used to name the
 * static destructor behind the exit-time SIGSEGV in __cxa_finalize under rocprofv3
 * --memory-copy-trace (What's weak 4).  Never loaded by the product path. */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

static void on_fault(int sig, siginfo_t* si, void* uc) {
  (void)uc;
  void* frames[64];
  int n = backtrace(frames, 64);
  char line[512];
  int len = snprintf(line, sizeof line, "\n[crash_trace] signal %d at address %p, %d frames:\n", sig,
                     si ? si->si_addr : 0, n);
  write(2, line, (size_t)len);
  for (int i = 0; i < n; i++) {
    Dl_info info;
    memset(&info, 0, sizeof info);
    if (dladdr(frames[i], &info) && info.dli_fname) {
      len = snprintf(line, sizeof line, "  #%02d %p %s+0x%lx (%s)\n", i, frames[i], info.dli_fname,
                     (unsigned long)((char*)frames[i] - (char*)info.dli_fbase),
                     info.dli_sname ? info.dli_sname : "?");
    } else {
      len = snprintf(line, sizeof line, "  #%02d %p ?\n", i, frames[i]);
    }
    write(2, line, (size_t)len);
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

__attribute__((constructor)) static void install(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = on_fault;
  sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
  sigaction(SIGSEGV, &sa, 0);
  sigaction(SIGBUS, &sa, 0);
  sigaction(SIGABRT, &sa, 0);
}

/* re-install (after a library that set its own handler): callable from ctypes */
void crash_trace_install(void) { install(); }
