/* Host-only crash reporter for repro scripts: on SIGSEGV/SIGABRT print the native backtrace (glibc execinfo) to
   stderr, then re-raise with the default action. Loaded with ctypes.CDLL by scripts/r6_drop_repro.py. */
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void on_fault(int sig) {
    void *frames[96];
    int n = backtrace(frames, 96);
    const char msg[] = "\n[segv_bt] native backtrace:\n";
    write(2, msg, sizeof(msg) - 1);
    backtrace_symbols_fd(frames, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

__attribute__((constructor)) static void install(void) {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_handler = on_fault;
    sigaction(SIGSEGV, &sa, 0);
    sigaction(SIGABRT, &sa, 0);
}
