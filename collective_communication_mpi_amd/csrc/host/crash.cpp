// Native crash reporter: on SIGSEGV / SIGBUS / SIGILL / SIGFPE / SIGABRT print the
// signal, the faulting address and a symbolised native backtrace (library + offset
// for stripped libraries such as the HIP runtime) to a file descriptor, then hand
// the signal to the handler that was installed before (Python's faulthandler, which
// prints the Python stacks and re-raises).  Python's faulthandler alone only shows
// where in Python a native crash happened (e.g. "CUDAGraph.replay"); this shows in
// which native function.  Async-signal-safe: write(2), backtrace_symbols_fd and
// dladdr only (backtrace() is primed once at install so it does not allocate later).
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>

namespace ccmpi {
namespace {

int g_fd = 2;
struct sigaction g_prev[32];
bool g_installed = false;
const int kSignals[] = {SIGSEGV, SIGBUS, SIGILL, SIGFPE, SIGABRT};

void put(const char* s) {
  ssize_t r = write(g_fd, s, strlen(s));
  (void)r;
}

void put_hex(unsigned long v) {
  char buf[2 + 16 + 1];
  buf[0] = '0';
  buf[1] = 'x';
  for (int i = 0; i < 16; ++i) buf[2 + i] = "0123456789abcdef"[(v >> (60 - 4 * i)) & 0xf];
  buf[18] = 0;
  put(buf);
}

void on_signal(int sig, siginfo_t* info, void* uctx) {
  put("\n[ccmpi crash] signal ");
  char num[8];
  snprintf(num, sizeof(num), "%d", sig);
  put(num);
  put(" fault address ");
  put_hex(reinterpret_cast<unsigned long>(info ? info->si_addr : nullptr));
  put(" pid ");
  snprintf(num, sizeof(num), "%d", (int)getpid() % 10000000);
  put(num);
  put("\n[ccmpi crash] native backtrace (frame: object(symbol+off) [pc] | object base):\n");
  void* frames[64];
  int n = backtrace(frames, 64);
  for (int i = 0; i < n; ++i) {
    backtrace_symbols_fd(&frames[i], 1, g_fd);
    Dl_info dl;
    if (dladdr(frames[i], &dl) && dl.dli_fbase) {
      put("    base ");
      put_hex(reinterpret_cast<unsigned long>(dl.dli_fbase));
      put(" offset ");
      put_hex(reinterpret_cast<unsigned long>(frames[i]) - reinterpret_cast<unsigned long>(dl.dli_fbase));
      put("\n");
    }
  }
  put("[ccmpi crash] end of native backtrace\n");
  // chain: the previous handler (faulthandler) prints Python stacks and re-raises
  struct sigaction& prev = g_prev[sig];
  if (prev.sa_flags & SA_SIGINFO) {
    if (prev.sa_sigaction) {
      prev.sa_sigaction(sig, info, uctx);
      return;
    }
  } else if (prev.sa_handler != SIG_DFL && prev.sa_handler != SIG_IGN && prev.sa_handler) {
    prev.sa_handler(sig);
    return;
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

}  // namespace

// Install once per process.  Returns the number of signals hooked.
int install_crash_handler(int fd) {
  if (g_installed) return 0;
  g_fd = fd;
  void* prime[2];
  backtrace(prime, 2);  // loads libgcc's unwinder now, not inside the handler
  static char altstack[1 << 16];
  stack_t ss;
  ss.ss_sp = altstack;
  ss.ss_size = sizeof(altstack);
  ss.ss_flags = 0;
  sigaltstack(&ss, nullptr);
  int hooked = 0;
  for (int sig : kSignals) {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = on_signal;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK | SA_NODEFER;
    sigemptyset(&sa.sa_mask);
    if (sigaction(sig, &sa, &g_prev[sig]) == 0) ++hooked;
  }
  g_installed = true;
  return hooked;
}

}  // namespace ccmpi
