/*
 * ranks_demo.c -- the sharded grouping from a plain C host with one process
 * per rank (no torch, no HIP headers), the way a Rust host with one process
 * per GPU would drive libsdgpu: the parent forks W children BEFORE anything
 * touches the GPU; each child opens a context, joins the communicator
 * (sdgpu_comm_init_host here: the ranks share the test box's one GPU, which
 * RCCL refuses; the calls below are the ones made under RCCL), puts its share
 * of the rows on the device and runs the write-set exchange
 * (sdgpu_group_link_sharded_device) three times -- counted (B unknown),
 * then padded twice back to back, the second resolving the first -- then
 * sdgpu_comm_wait and writes its lists to <dir>/rank<r>.bin:
 *   u32 entries, u32 who[entries], u32 obj[entries]
 * tests/test_c_abi.py checks the union of the ranks' lists against the
 * oracle's write set of all rows.  Rows: row i has key splitmix64(seed, i %
 * distinct) (so ~distinct/total duplicates), has_key = (i % 997 != 0), global
 * rank i; rank r holds rows [r n / W, (r + 1) n / W).
 * Usage: ranks_demo <world> <total_rows> <distinct> <dir>   exit 0 = all ranks ok
 */
#define _POSIX_C_SOURCE 200809L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <unistd.h>

#include "sdgpu.h"

static uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

#define TRY(expr)                                                               \
  do {                                                                          \
    const int rc_ = (expr);                                                     \
    if (rc_ != 0) {                                                             \
      fprintf(stderr, "rank %d: %s -> %d (%s)\n", rank, #expr, rc_, sdgpu_strerror(rc_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

static int run_rank(int world, int rank, uint64_t total, uint64_t distinct, const char* dir) {
  const uint64_t lo = total * (uint64_t)rank / (uint64_t)world;
  const uint64_t hi = total * (uint64_t)(rank + 1) / (uint64_t)world;
  const uint64_t n = hi - lo, cap = total + n;
  uint64_t* key = malloc(8 * (n ? n : 1));
  uint8_t* has = malloc(n ? n : 1);
  uint32_t* grank = malloc(4 * (n ? n : 1));
  uint32_t* who = malloc(4 * cap);
  uint32_t* obj = malloc(4 * cap);
  if (!key || !has || !grank || !who || !obj) return 1;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t g = lo + i;
    key[i] = splitmix64(0x5D00 + g % distinct);
    has[i] = g % 997 != 0;
    grank[i] = (uint32_t)g;
  }
  sdgpu_ctx* ctx = NULL;
  TRY(sdgpu_open(0, &ctx));
  char path[4096];
  snprintf(path, sizeof path, "%s/comm", dir);
  sdgpu_comm* comm = NULL;
  TRY(sdgpu_comm_init_host(ctx, world, rank, path, 16 * (total + 4096), 60000, &comm));
  void *d_key, *d_has, *d_rank, *d_who, *d_obj, *d_counts;
  TRY(sdgpu_alloc_device(ctx, 8 * (n ? n : 1), &d_key));
  TRY(sdgpu_alloc_device(ctx, n ? n : 1, &d_has));
  TRY(sdgpu_alloc_device(ctx, 4 * (n ? n : 1), &d_rank));
  TRY(sdgpu_alloc_device(ctx, 4 * cap, &d_who));
  TRY(sdgpu_alloc_device(ctx, 4 * cap, &d_obj));
  TRY(sdgpu_alloc_device(ctx, 16, &d_counts));
  void* s = sdgpu_stream(ctx);
  TRY(sdgpu_memcpy_async(ctx, d_key, key, 8 * n, s));
  TRY(sdgpu_memcpy_async(ctx, d_has, has, n, s));
  TRY(sdgpu_memcpy_async(ctx, d_rank, grank, 4 * n, s));
  TRY(sdgpu_sync(ctx));
  for (int call = 0; call < 3; ++call)
    TRY(sdgpu_group_link_sharded_device(ctx, comm, d_key, d_has, NULL, d_rank, n, 100, d_who,
                                        d_obj, cap, d_counts, s));
  TRY(sdgpu_comm_wait(comm, s));
  sdgpu_comm_stats_t st;
  TRY(sdgpu_comm_stats(comm, &st));
  uint32_t counts[3];
  TRY(sdgpu_memcpy_async(ctx, counts, d_counts, 12, s));
  TRY(sdgpu_sync(ctx));
  const uint32_t e = counts[2];
  if (e > cap) return 1;
  TRY(sdgpu_memcpy_async(ctx, who, d_who, 4ull * e, s));
  TRY(sdgpu_memcpy_async(ctx, obj, d_obj, 4ull * e, s));
  TRY(sdgpu_sync(ctx));
  snprintf(path, sizeof path, "%s/rank%d.bin", dir, rank);
  FILE* f = fopen(path, "wb");
  if (!f || fwrite(&e, 4, 1, f) != 1 || fwrite(who, 4, e, f) != e || fwrite(obj, 4, e, f) != e)
    return 1;
  fclose(f);
  printf("rank %d: rows %llu entries %u calls %llu padded %llu reruns %llu\n", rank,
         (unsigned long long)n, e, (unsigned long long)st.calls,
         (unsigned long long)st.padded_calls, (unsigned long long)st.overflow_reruns);
  TRY(sdgpu_comm_destroy(comm));
  sdgpu_free_device(ctx, d_key);
  sdgpu_free_device(ctx, d_has);
  sdgpu_free_device(ctx, d_rank);
  sdgpu_free_device(ctx, d_who);
  sdgpu_free_device(ctx, d_obj);
  sdgpu_free_device(ctx, d_counts);
  TRY(sdgpu_close(ctx));
  free(key);
  free(has);
  free(grank);
  free(who);
  free(obj);
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: ranks_demo <world> <total_rows> <distinct> <dir>\n");
    return 2;
  }
  const int world = atoi(argv[1]);
  const uint64_t total = strtoull(argv[2], NULL, 10), distinct = strtoull(argv[3], NULL, 10);
  if (world < 1 || world > 16 || distinct == 0) return 2;
  fflush(stdout);
  pid_t pids[16];
  for (int r = 0; r < world; ++r) {  /* fork before any process touches the GPU */
    pids[r] = fork();
    if (pids[r] < 0) return 1;
    if (pids[r] == 0) {
      const int rc = run_rank(world, r, total, distinct, argv[4]);
      fflush(stdout);
      _exit(rc);
    }
  }
  int bad = 0;
  for (int r = 0; r < world; ++r) {
    int status = 0;
    if (waitpid(pids[r], &status, 0) < 0 || !WIFEXITED(status) || WEXITSTATUS(status) != 0) ++bad;
  }
  if (bad == 0) printf("c ranks ok\n");
  return bad ? 1 : 0;
}
