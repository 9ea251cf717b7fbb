/* tools/dropin_threads.c -- (b1) drop-in throughput and latency from N POSIX
 * threads at once, with no interpreter in the way (tools/service_interference.py
 * drives the calls from Python threads, whose own locking caps the rate).
 * Each thread calls in_cksum_hdr on the SURVEY.md 8(a) KAT header (0x61B8)
 * in a loop for the given seconds and times every call (CLOCK_MONOTONIC).
 * One JSON line per thread count.
 *
 *   gcc -O2 -pthread tools/dropin_threads.c -Llibunsod_amd/lib -lmicksum \
 *       -Wl,-rpath,$PWD/libunsod_amd/lib -o tools/dropin_threads
 *   tools/dropin_threads 1,2,4,8,16 2.0
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

unsigned int in_cksum_hdr(const void *ip);

static const uint8_t kHdr[20] = {0x45, 0x00, 0x00, 0x73, 0x00, 0x00, 0x40, 0x00, 0x40, 0x11,
                                 0x00, 0x00, 0xc0, 0xa8, 0x00, 0x01, 0xc0, 0xa8, 0x00, 0xc7};
enum { kMaxSamples = 1 << 20 };

struct Arg {
  double seconds;
  pthread_barrier_t *bar;
  float *lat;  /* us */
  long n, bad;
};

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

static void *worker(void *p) {
  struct Arg *a = p;
  uint8_t buf[128] __attribute__((aligned(64)));
  memcpy(buf + 2, kHdr, 20); /* 2 mod 4, as behind a 14-byte Ethernet header */
  if (in_cksum_hdr(buf + 2) != 0x61B8) a->bad++;
  pthread_barrier_wait(a->bar);
  const double end = now() + a->seconds;
  for (;;) {
    const double t0 = now();
    if (in_cksum_hdr(buf + 2) != 0x61B8) a->bad++;
    const double t1 = now();
    if (a->n < kMaxSamples) a->lat[a->n] = (float)((t1 - t0) * 1e6);
    a->n++;
    if (t1 > end) break;
  }
  return NULL;
}

static int cmpf(const void *x, const void *y) {
  const float a = *(const float *)x, b = *(const float *)y;
  return (a > b) - (a < b);
}

int main(int argc, char **argv) {
  const char *list = argc > 1 ? argv[1] : "1,2,4,8,16";
  const double seconds = argc > 2 ? atof(argv[2]) : 2.0;
  char *dup = strdup(list);
  char *save = NULL;
  for (char *tok = strtok_r(dup, ",", &save); tok; tok = strtok_r(NULL, ",", &save)) {
    const int n = atoi(tok);
    pthread_t th[64];
    struct Arg args[64];
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)n);
    for (int i = 0; i < n; ++i) {
      args[i] = (struct Arg){seconds, &bar, malloc(sizeof(float) * kMaxSamples), 0, 0};
      pthread_create(&th[i], NULL, worker, &args[i]);
    }
    long total = 0, bad = 0, kept = 0;
    for (int i = 0; i < n; ++i) {
      pthread_join(th[i], NULL);
      total += args[i].n;
      bad += args[i].bad;
      kept += args[i].n < kMaxSamples ? args[i].n : kMaxSamples;
    }
    float *all = malloc(sizeof(float) * (size_t)kept);
    long k = 0;
    for (int i = 0; i < n; ++i) {
      const long m = args[i].n < kMaxSamples ? args[i].n : kMaxSamples;
      memcpy(all + k, args[i].lat, sizeof(float) * (size_t)m);
      k += m;
      free(args[i].lat);
    }
    qsort(all, (size_t)kept, sizeof(float), cmpf);
    printf("{\"threads\": %d, \"calls_per_s\": %.0f, \"call_us_p50\": %.2f, \"call_us_p99\": %.2f, \"wrong\": %ld}\n", n,
           total / seconds, all[kept / 2], all[(long)(kept * 0.99)], bad);
    fflush(stdout);
    free(all);
    pthread_barrier_destroy(&bar);
  }
  free(dup);
  return 0;
}
