/* Diagnostics only (never loaded by the product, the tests or bench.py): a
 * SIGSEGV handler that writes the faulting address, each frame's library +
 * offset + nearest dynamic symbol (dladdr) and the process's executable
 * mappings to stderr, then hands the signal to the handler it replaced. Used
 * to name the library of the rocprofv3 --pmc crash (tools/crash_diag.py). */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <ucontext.h>
#include <unistd.h>

static struct sigaction g_old;

static void put(const char* s) { (void)!write(2, s, strlen(s)); }

static void frame(void* p) {
    char buf[768];
    Dl_info d;
    if (p && dladdr(p, &d) && d.dli_fname) {
        snprintf(buf, sizeof buf, "crashmaps:   %p %s+0x%lx (%s+0x%lx)\n", p, d.dli_fname,
                 (unsigned long)((char*)p - (char*)d.dli_fbase), d.dli_sname ? d.dli_sname : "?",
                 d.dli_saddr ? (unsigned long)((char*)p - (char*)d.dli_saddr) : 0ul);
    } else {
        snprintf(buf, sizeof buf, "crashmaps:   %p (no mapping)\n", p);
    }
    put(buf);
}

static void handler(int sig, siginfo_t* si, void* ucv) {
    char buf[256];
    ucontext_t* uc = (ucontext_t*)ucv;
    void* pc = (void*)uc->uc_mcontext.gregs[REG_RIP];
    snprintf(buf, sizeof buf, "crashmaps: signal %d, fault address %p, pc:\n", sig, si->si_addr);
    put(buf);
    frame(pc);
    put("crashmaps: frames:\n");
    void* pcs[64];
    const int n = backtrace(pcs, 64);
    for (int i = 0; i < n; ++i) frame(pcs[i]);
    put("crashmaps: mappings (r-x, and the one holding the fault address):\n");
    const int fd = open("/proc/self/maps", O_RDONLY);
    if (fd >= 0) {
        char line[1024];
        int len = 0;
        char c;
        while (read(fd, &c, 1) == 1) {
            if (len < (int)sizeof line - 2) line[len++] = c;
            if (c != '\n') continue;
            line[len] = 0;
            unsigned long lo = 0, hi = 0;
            char perm[8] = {0};
            if (sscanf(line, "%lx-%lx %7s", &lo, &hi, perm) == 3 &&
                (perm[2] == 'x' || ((unsigned long)si->si_addr >= lo && (unsigned long)si->si_addr < hi) ||
                 ((unsigned long)si->si_addr >= lo - 0x200000 && (unsigned long)si->si_addr < hi + 0x200000)))
                put(line);
            len = 0;
        }
        close(fd);
    }
    sigaction(SIGSEGV, &g_old, NULL);  /* the fault repeats on return, into the previous handler */
}

void crashmaps_install(void) {
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGSEGV, &sa, &g_old);
}
