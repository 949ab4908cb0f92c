/* tools/sampler.c -- a minimal SIGPROF sampling profiler for host-side code (no perf in the
 * image).  LD_PRELOAD it into a program: every 100 us of CPU time it records the interrupted PC
 * and the return addresses of up to 3 frame-pointer frames; at exit it writes them, with
 * /proc/self/maps, to $NTC_SAMPLER_OUT (default /tmp/ntc_samples.txt).  tools/sampler_report.py
 * turns the file into a flat profile (self) and an inclusive one (self + callers).
 *
 * build: gcc -O2 -shared -fPIC -o /tmp/libsampler.so tools/sampler.c -lrt
 */
#define _GNU_SOURCE
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>
#include <time.h>
#include <ucontext.h>

#define MAXS (1 << 21)
#define DEPTH 4
static uintptr_t g_pc[MAXS][DEPTH];
static volatile long g_n = 0;
/* NTC_SAMPLER_GATED=1: record only between ntc_sampler_enable(1) and ntc_sampler_enable(0), which
 * a program under study looks up with dlsym(RTLD_DEFAULT, ...) around its timed region */
static volatile int g_on = 1;
static void start_timer(void);
static int g_started = 0;
/* gated: the timer itself starts at the first enable, so no signal lands in the program's start-up
 * (a GPU runtime's initialisation does not tolerate interrupted system calls everywhere) */
void ntc_sampler_enable(int on)
{
  if (on && !g_started) start_timer();
  g_on = on;
}
static uintptr_t g_stk_lo = 0, g_stk_hi = 0;
static timer_t g_timer;
static int g_have_timer = 0;   /* main thread stack: frames are walked only inside */

static void on_prof(int sig, siginfo_t* si, void* uc_)
{
  (void)sig; (void)si;
  ucontext_t* uc = (ucontext_t*)uc_;
  long n = g_n;
  if (n >= MAXS || !g_on) return;
  g_pc[n][0] = (uintptr_t)uc->uc_mcontext.gregs[REG_RIP];
  uintptr_t* fp = (uintptr_t*)uc->uc_mcontext.gregs[REG_RBP];
  for (int d = 1; d < DEPTH; ++d) {
    if (((uintptr_t)fp & 7) || (uintptr_t)fp < g_stk_lo || (uintptr_t)fp + 16 > g_stk_hi) {
      for (int e = d; e < DEPTH; ++e) g_pc[n][e] = 0;
      break;
    }
    uintptr_t ret = fp[1];
    uintptr_t* nfp = (uintptr_t*)fp[0];
    g_pc[n][d] = ret;
    if (nfp <= fp) { for (int e = d + 1; e < DEPTH; ++e) g_pc[n][e] = 0; break; }
    fp = nfp;
  }
  g_n = n + 1;
}

__attribute__((constructor)) static void start(void)
{
  if (getenv("NTC_SAMPLER_GATED") && atoi(getenv("NTC_SAMPLER_GATED"))) g_on = 0;
  FILE* m = fopen("/proc/self/maps", "r");
  char line[4096];
  while (m && fgets(line, sizeof line, m))
    if (strstr(line, "[stack]")) {
      unsigned long lo, hi;
      if (sscanf(line, "%lx-%lx", &lo, &hi) == 2) { g_stk_lo = lo; g_stk_hi = hi; }
    }
  if (m) fclose(m);
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigaction(SIGPROF, &sa, NULL);
  if (g_on) start_timer();
}

static void start_timer(void)
{
  g_started = 1;
  /* a wall-clock POSIX timer (hrtimer): CPU-time timers tick at the kernel HZ here (a few ms);
   * profile a single busy thread */
  struct sigevent sev;
  memset(&sev, 0, sizeof sev);
  sev.sigev_notify = SIGEV_SIGNAL;
  sev.sigev_signo = SIGPROF;
  if (timer_create(CLOCK_MONOTONIC, &sev, &g_timer) == 0) {
    struct itimerspec its = {{0, 100000}, {0, 100000}};
    timer_settime(g_timer, 0, &its, NULL);
    g_have_timer = 1;
  } else {
    struct itimerval it = {{0, 100}, {0, 100}};
    setitimer(ITIMER_PROF, &it, NULL);
  }
}

__attribute__((destructor)) static void stop(void)
{
  if (g_have_timer) timer_delete(g_timer);
  struct itimerval it = {{0, 0}, {0, 0}};
  setitimer(ITIMER_PROF, &it, NULL);
  const char* path = getenv("NTC_SAMPLER_OUT");
  FILE* f = fopen(path ? path : "/tmp/ntc_samples.txt", "w");
  if (!f) return;
  FILE* m = fopen("/proc/self/maps", "r");
  char line[4096];
  while (m && fgets(line, sizeof line, m)) fprintf(f, "M %s", line);
  if (m) fclose(m);
  for (long i = 0; i < g_n; ++i) {
    fprintf(f, "S");
    for (int d = 0; d < DEPTH; ++d) fprintf(f, " %lx", (unsigned long)g_pc[i][d]);
    fprintf(f, "\n");
  }
  fclose(f);
}
