/* Developer tool (not shipped): a minimal sampling profiler for the host
 * code on a CPU-only machine.  LD_PRELOAD it; every 1 ms of process CPU time
 * (ITIMER_PROF) the interrupted thread's program counter is recorded; at exit
 * the samples are resolved to <object> + offset and written to
 * $SPROF_OUT (default /tmp/sprof.txt) as "count object offset" lines, for
 * tools/hostbench/sprof_report.py to symbolize with addr2line. */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>
#include <ucontext.h>

#define MAXS (1 << 22)
static unsigned long samples[MAXS];
static volatile long nsamp;

static void on_prof(int sig, siginfo_t* si, void* ctx) {
  (void)sig;
  (void)si;
  const long k = __atomic_fetch_add(&nsamp, 1, __ATOMIC_RELAXED);
  if (k < MAXS) samples[k] = (unsigned long)((ucontext_t*)ctx)->uc_mcontext.gregs[REG_RIP];
}

static int cmp(const void* a, const void* b) {
  const unsigned long x = *(const unsigned long*)a, y = *(const unsigned long*)b;
  return x < y ? -1 : x > y;
}

static void dump(void) {
  struct itimerval off = {{0, 0}, {0, 0}};
  setitimer(ITIMER_PROF, &off, NULL);
  long n = nsamp < MAXS ? nsamp : MAXS;
  qsort(samples, n, sizeof samples[0], cmp);
  const char* path = getenv("SPROF_OUT");
  FILE* f = fopen(path ? path : "/tmp/sprof.txt", "w");
  if (!f) return;
  for (long i = 0; i < n;) {
    long j = i;
    while (j < n && samples[j] == samples[i]) ++j;
    Dl_info di;
    if (dladdr((void*)samples[i], &di) && di.dli_fname)
      fprintf(f, "%ld %s %lx\n", j - i, di.dli_fname, samples[i] - (unsigned long)di.dli_fbase);
    else
      fprintf(f, "%ld ? %lx\n", j - i, samples[i]);
    i = j;
  }
  fclose(f);
}

__attribute__((constructor)) static void start(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigaction(SIGPROF, &sa, NULL);
  struct itimerval it = {{0, 1000}, {0, 1000}};
  setitimer(ITIMER_PROF, &it, NULL);
  atexit(dump);
}
