/*
 * abi_demo.c -- a plain C host of libsdgpu.so (no torch, no HIP headers): the
 * shape of the FFI a Rust `sdgpu-sys` crate binds.  Checks
 * the C ABI end to end against golden vectors that tests/test_gpu_c_abi.py
 * passes in a text file ("<len> <blake3 hex>" lines for the input
 * byte i = i % 251, from tests/golden/golden.json):
 *   - sdgpu_checksum (host buffer)      == golden digest
 *   - sdgpu_cas_batch (host arena)      == first 16 hex chars of the digest
 *   - sdgpu_generate_cas_id(path, size) == sdgpu_cas_batch of size_le || file
 *   - sdgpu_file_checksum(path)         == golden digest
 *   - sdgpu_dedup                       == the canonical grouping rule
 * Exit 0 = all equal.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sdgpu.h"

static int fails = 0;
#define CHECK(c, ...)               \
  do {                              \
    if (!(c)) {                     \
      fprintf(stderr, __VA_ARGS__); \
      fputc('\n', stderr);          \
      ++fails;                      \
    }                               \
  } while (0)

static void hex(const uint8_t* d, int n, char* out) {
  for (int i = 0; i < n; ++i) sprintf(out + 2 * i, "%02x", d[i]);
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: abi_demo <vectors.txt> <tmpdir>\n");
    return 2;
  }
  sdgpu_ctx* ctx = NULL;
  int rc = sdgpu_open(0, &ctx);
  if (rc) {
    fprintf(stderr, "sdgpu_open: %s\n", sdgpu_strerror(rc));
    return 1;
  }
  FILE* f = fopen(argv[1], "r");
  if (!f) return 2;
  size_t len;
  char want[65];
  int vectors = 0;
  while (fscanf(f, "%zu %64s", &len, want) == 2) {
    uint8_t* buf = malloc(len + 16);
    for (size_t i = 0; i < len; ++i) buf[i] = (uint8_t)(i % 251);
    uint8_t d[32];
    char h[65];
    CHECK(sdgpu_checksum(ctx, buf, len, d) == 0, "sdgpu_checksum failed");
    hex(d, 32, h);
    CHECK(strcmp(h, want) == 0, "checksum(%zu) %s != %s", len, h, want);
    if (len <= SDGPU_CAS_MAX_MSG_LEN) {
      const uint64_t off = 0;
      const uint32_t l32 = (uint32_t)len;
      uint8_t out8[1][8];
      int32_t st = 1;
      CHECK(sdgpu_cas_batch(ctx, buf, &off, &l32, 1, out8, &st) == 0 && st == 0, "cas_batch");
      hex(out8[0], 8, h);
      CHECK(strncmp(h, want, 16) == 0, "cas(%zu) %s != %.16s", len, h, want);
    }
    /* the same bytes as a file: file_checksum and generate_cas_id */
    char path[4096];
    snprintf(path, sizeof path, "%s/v%zu.bin", argv[2], len);
    FILE* o = fopen(path, "wb");
    if (len) fwrite(buf, 1, len, o);
    fclose(o);
    char fh[65];
    CHECK(sdgpu_file_checksum(ctx, path, fh) == 0 && strcmp(fh, want) == 0,
          "file_checksum(%zu)", len);
    if (len && len <= 100 * 1024) {
      uint8_t* m = malloc(8 + len);
      for (int i = 0; i < 8; ++i) m[i] = (uint8_t)((uint64_t)len >> (8 * i));
      memcpy(m + 8, buf, len);
      const uint64_t off = 0;
      const uint32_t l32 = (uint32_t)(8 + len);
      uint8_t out8[1][8];
      CHECK(sdgpu_cas_batch(ctx, m, &off, &l32, 1, out8, NULL) == 0, "cas_batch msg");
      char c1[17], c2[17];
      hex(out8[0], 8, c1);
      CHECK(sdgpu_generate_cas_id(ctx, path, len, c2) == 0 && strcmp(c1, c2) == 0,
            "generate_cas_id(%zu) %s != %s", len, c2, c1);
      free(m);
    }
    free(buf);
    ++vectors;
  }
  fclose(f);

  /* grouping: keys cycle with period 7 over 1000 rows, chunks of 100 */
  enum { N = 1000 };
  uint64_t key[N];
  uint8_t has[N];
  uint32_t rep[N];
  for (uint32_t r = 0; r < N; ++r) {
    key[r] = 0x9E3779B97F4A7C15ull * (r % 7 + 1);
    has[r] = r % 97 != 5;
  }
  CHECK(sdgpu_dedup(ctx, key, has, N, 100, rep) == 0, "sdgpu_dedup");
  for (uint32_t r = 0; r < N; ++r) {
    uint32_t first = r;
    if (has[r])
      for (uint32_t q = 0; q < r; ++q)
        if (has[q] && key[q] == key[r]) {
          first = q;
          break;
        }
    const uint32_t expect = (!has[r] || first / 100 == r / 100) ? r : first;
    CHECK(rep[r] == expect, "rep[%u] = %u, expected %u", r, rep[r], expect);
  }
  sdgpu_close(ctx);
  if (fails) {
    fprintf(stderr, "%d failures\n", fails);
    return 1;
  }
  printf("c abi ok: %d vectors\n", vectors);
  return 0;
}
