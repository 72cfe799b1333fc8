/* Experiment (not shipped): single-file call latency from a C host (no Python):
 * open+read+close alone, sdgpu_generate_cas_id, sdgpu_file_checksum on a 4 KiB
 * and a 1 MiB file; median of 2000 calls each.
 * Build: gcc -O2 -Iinclude scripts/exp/exp_single_latency.c -Lspacedrive_amd -lsdgpu
 *        -Wl,-rpath,$PWD/spacedrive_amd -o build/exp_single_latency */
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "sdgpu.h"

static double now_us(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec / 1e3;
}
static int cmp(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}
#define N 2000
static double ts[N];
#define MEDIAN(expr)                              \
  ({                                              \
    for (int i = 0; i < 50; ++i) (void)(expr);    \
    for (int i = 0; i < N; ++i) {                 \
      const double t0 = now_us();                 \
      (void)(expr);                               \
      ts[i] = now_us() - t0;                      \
    }                                             \
    qsort(ts, N, sizeof(double), cmp);            \
    ts[N / 2];                                    \
  })

static int read_all(const char* p, unsigned char* buf, size_t cap) {
  const int fd = open(p, O_RDONLY);
  const ssize_t r = read(fd, buf, cap);
  close(fd);
  return (int)r;
}

int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : "/tmp";
  sdgpu_ctx* c = NULL;
  if (sdgpu_open(0, &c)) return 1;
  static unsigned char buf[1 << 20];
  for (int i = 0; i < (1 << 20); ++i) buf[i] = (unsigned char)(i * 13 + 7);
  const size_t sizes[2] = {4096, 1 << 20};
  for (int k = 0; k < 2; ++k) {
    char p[512];
    snprintf(p, sizeof p, "%s/lat_%zu.bin", dir, sizes[k]);
    FILE* f = fopen(p, "wb");
    fwrite(buf, 1, sizes[k], f);
    fclose(f);
    char hex[17], hex64[65];
    static unsigned char rb[1 << 20];
    printf("%7zu B: read %6.1f us  generate_cas_id %6.1f us  file_checksum %6.1f us\n", sizes[k],
           MEDIAN(read_all(p, rb, sizeof rb)), MEDIAN(sdgpu_generate_cas_id(c, p, sizes[k], hex)),
           MEDIAN(sdgpu_file_checksum(c, p, hex64)));
    /* kernel time alone (HIP events around the latency kernel) */
    for (int pass = 0; pass < 2; ++pass) {
      sdgpu_set_timing(c, 1);
      sdgpu_timing_reset(c);
      for (int i = 0; i < 200; ++i) {
        if (pass == 0) sdgpu_generate_cas_id(c, p, sizes[k], hex);
        else sdgpu_file_checksum(c, p, hex64);
      }
      char name[32];
      double ms;
      uint64_t cnt;
      for (uint32_t i = 0; sdgpu_timing_read(c, i, name, &ms, &cnt) == 0; ++i)
        printf("    %s: %s %.1f us per launch (%llu)\n", pass ? "file_checksum" : "generate_cas_id",
               name, 1e3 * ms / (double)cnt, (unsigned long long)cnt);
      sdgpu_set_timing(c, 0);
    }
  }
  sdgpu_close(c);
  return 0;
}
