/*
 * sanitize_main.c -- TEST INFRASTRUCTURE: drives the C oracle under
 * AddressSanitizer + UndefinedBehaviorSanitizer (tests/test_sanitizers.py
 * builds `gcc -fsanitize=address,undefined sd_oracle.c sanitize_main.c`).
 * Exercises every tree shape up to 5 chunks + 1 byte, the incremental hasher,
 * the threaded tree, the cas message builder and the grouping rule, and checks
 * the formulations against each other.  Exit status 0 = clean and consistent.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void orc_blake3(const uint8_t *in, size_t len, uint8_t out32[32]);
void orc_blake3_mt(const uint8_t *in, size_t len, int threads, uint8_t out32[32]);
void orc_blake3_incremental(const uint8_t *in, size_t len, size_t piece, uint8_t out32[32]);
void orc_blake3_derive_key(const char *context, size_t context_len, const uint8_t *material,
                           size_t material_len, uint8_t out32[32]);
uint32_t orc_synth_cas_message(uint64_t size, uint64_t seed, uint8_t *out);
void orc_cas_id_of_message(const uint8_t *msg, size_t len, char out_hex[17]);
int orc_group_reps(const uint64_t *key, const uint8_t *has_key, uint32_t n, uint32_t chunk_rows,
                   uint32_t *rep);
void orc_cas_batch(const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint64_t n,
                   uint8_t *out8, int threads);
void orc_cas_batch_simd(const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                        uint64_t n, uint8_t *out8, int threads);

static int fails = 0;
#define CHECK(c, ...)                 \
  do {                                \
    if (!(c)) {                       \
      fprintf(stderr, __VA_ARGS__);   \
      fputc('\n', stderr);            \
      ++fails;                        \
    }                                 \
  } while (0)

int main(void) {
  /* derive_b3 KAT: crates/crypto/src/keys/hashing.rs:210-213,324-327 */
  static const uint8_t kat[32] = {27,  34,  251, 101, 201, 89, 78,  90,  20,  175, 62,
                                  206, 200, 153, 166, 103, 118, 179, 194, 44,  216, 26,
                                  48,  120, 137, 157, 60,  234, 234, 53,  46,  60};
  const char *ctx = "spacedrive 2023-02-09 17:44:14 test key derivation";
  uint8_t material[48];
  memset(material, 0x23, 32);
  memset(material + 32, 0xFF, 16);
  uint8_t d[32], e[32];
  orc_blake3_derive_key(ctx, strlen(ctx), material, sizeof material, d);
  CHECK(memcmp(d, kat, 32) == 0, "derive_key KAT mismatch");

  const size_t max = 5 * 1024 + 1;
  uint8_t *buf = malloc(max);
  for (size_t i = 0; i < max; ++i) buf[i] = (uint8_t)(i * 131 + 7);
  for (size_t n = 0; n <= max; n += (n < 2100 ? 1 : 61)) {
    orc_blake3(buf, n, d);
    orc_blake3_incremental(buf, n, 1 + n % 97, e);
    CHECK(memcmp(d, e, 32) == 0, "recursive vs incremental differ at %zu", n);
  }
  free(buf);

  const size_t big = (size_t)9 << 20;
  uint8_t *b2 = malloc(big);
  for (size_t i = 0; i < big; ++i) b2[i] = (uint8_t)(i ^ (i >> 9));
  orc_blake3(b2, big, d);
  orc_blake3_mt(b2, big, 4, e);
  CHECK(memcmp(d, e, 32) == 0, "threaded tree differs");
  free(b2);

  uint8_t *msg = malloc(8 + 102400 + 64);
  const uint64_t sizes[] = {0, 1, 1024, 102400, 102401, 1 << 20, ((uint64_t)1 << 32) + 1};
  for (size_t i = 0; i < sizeof sizes / sizeof *sizes; ++i) {
    const uint32_t len = orc_synth_cas_message(sizes[i], 99 + i, msg);
    char hex[17];
    orc_cas_id_of_message(msg, len, hex);
    orc_blake3_incremental(msg, len, 8192, d);
    char hex2[17];
    for (int k = 0; k < 8; ++k) snprintf(hex2 + 2 * k, 3, "%02x", d[k]);
    CHECK(strcmp(hex, hex2) == 0, "cas id formulations differ for size %llu",
          (unsigned long long)sizes[i]);
  }
  free(msg);

  /* AVX2 8-way baseline == scalar on every chunk count 1..101 with ragged tails */
  {
    enum { M = 101 * 3 };
    uint64_t off[M];
    uint32_t len[M];
    uint64_t pos = 0;
    for (int i = 0; i < M; ++i) {
      len[i] = (uint32_t)((i / 3 + 1) * 1024 - (i % 3 == 0 ? 0 : (i % 3 == 1 ? 1 : 1000)));
      off[i] = pos;
      pos += (len[i] + 127) / 128 * 128;
    }
    uint8_t *arena = malloc(pos + 64);
    for (uint64_t i = 0; i < pos + 64; ++i) arena[i] = (uint8_t)(i * 2654435761u >> 13);
    uint8_t a[M][8], b[M][8];
    orc_cas_batch(arena, off, len, M, &a[0][0], 2);
    orc_cas_batch_simd(arena, off, len, M, &b[0][0], 2);
    CHECK(memcmp(a, b, sizeof a) == 0, "simd baseline differs from scalar");
    free(arena);
  }

  const uint32_t n = 50000;
  uint64_t *key = malloc(n * sizeof *key);
  uint8_t *has = malloc(n);
  uint32_t *rep = malloc(n * sizeof *rep);
  uint64_t x = 88172645463325252ull;
  for (uint32_t r = 0; r < n; ++r) {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    key[r] = x % 20000;
    has[r] = (x >> 40) % 50 != 0;
  }
  CHECK(orc_group_reps(key, has, n, 100, rep) == 0, "group_reps failed");
  for (uint32_t r = 0; r < n; ++r) {
    CHECK(rep[r] <= r, "rep after row %u", r);
    CHECK(rep[rep[r]] == rep[r], "rep not a fixed point at %u", r);
    if (!has[r]) CHECK(rep[r] == r, "keyless row %u linked", r);
    if (rep[r] != r) CHECK(key[rep[r]] == key[r] && rep[r] / 100 != r / 100, "bad link %u", r);
  }
  free(key);
  free(has);
  free(rep);
  if (fails) fprintf(stderr, "%d failures\n", fails);
  else printf("sanitized oracle: ok\n");
  return fails ? 1 : 0;
}
