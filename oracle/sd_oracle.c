/*
 * sd_oracle.c -- CPU ORACLE for the Spacedrive content-identification hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (spacedrive_amd/,
 * libsdgpu.so) links, loads or calls this file.  Only tests/, the smoke() check
 * in __graft_entry__.py and bench.py's cpu_baseline leg use it, and only as the
 * checker / the timed CPU baseline, never as the thing measured on the GPU.
 *
 * What it restates (plain C, scalar, written from the specs below):
 *
 *  - BLAKE3 (third-party crate `blake3` 1.4.1, /root/reference/Cargo.lock:620-631;
 *    NOT vendored under /root/reference).  Restated from the published BLAKE3
 *    specification: SHA-256 IV, 7 rounds, G rotations 16/12/8/7, message
 *    permutation [2,6,3,10,7,0,4,13,1,11,12,5,9,14,15,8], 1 KiB chunks of 16
 *    64-byte blocks, flags CHUNK_START=1 CHUNK_END=2 PARENT=4 ROOT=8
 *    KEYED_HASH=16 DERIVE_KEY_CONTEXT=32 DERIVE_KEY_MATERIAL=64, left-complete
 *    binary tree of chunk chaining values.
 *    The tree here is built RECURSIVELY (split at the largest power of two
 *    strictly below the chunk count), deliberately unlike the incremental
 *    CV-stack formulation of oracle/blake3_py.py, so the two restatements
 *    cross-check each other's tree shape.
 *    Pinned by the reference's BLAKE3 known-answer tests in
 *    /root/reference/crates/crypto/src/keys/hashing.rs: derive_b3 (:324-327,
 *    expected bytes :210-213, inputs :121,132-141, concatenation order
 *    /root/reference/crates/crypto/src/types.rs:163-170; derive-key mode) and
 *    the six Balloon-BLAKE3 vectors (:180-208, tests :269-321), which run
 *    BLAKE3 in HASH mode -- the mode of cas.rs / hash.rs -- over ~2.7-11 M
 *    messages of 24-74 bytes each (orc_balloon_blake3 below); and by the
 *    spec's hash of the empty input.
 *
 *  - generate_cas_id  (/root/reference/core/src/object/cas.rs:23-62), incl. the
 *    exact file-I/O pattern (open, read_exact header, 4 x {read_exact 10 KiB,
 *    seek}, seek End(-8192), read_exact footer) for the CPU baseline.
 *
 *  - file_checksum    (/root/reference/core/src/object/validation/hash.rs:10-24),
 *    1 MiB reads, stop at the first short read.
 *
 *  - the cas_id -> Object grouping rule of identifier_job_step
 *    (/root/reference/core/src/object/file_identifier/mod.rs:167-333) over
 *    CHUNK_SIZE=100 chunks (mod.rs:36, file_identifier_job.rs:286-309), in the
 *    canonical form fixed in SURVEY.md §8(a) row a6.
 *
 *  - the synthetic corpus content function shared with the device generator
 *    (spacedrive_amd/csrc/synth.hip); see DESIGN.md "Synthetic corpora".
 *
 *  - (end of file) an AVX2 8-way chunk/parent hasher used ONLY as bench.py's
 *    timed CPU baseline (the crate hashes chunks with SIMD too), checked
 *    bit-exact against the scalar restatement above.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

/* ------------------------------------------------------------------------- */
/* BLAKE3 core                                                               */
/* ------------------------------------------------------------------------- */

enum {
  B3_CHUNK_START = 1,
  B3_CHUNK_END = 2,
  B3_PARENT = 4,
  B3_ROOT = 8,
  B3_KEYED_HASH = 16,
  B3_DERIVE_KEY_CONTEXT = 32,
  B3_DERIVE_KEY_MATERIAL = 64,
};

#define B3_BLOCK 64u
#define B3_CHUNK 1024u

static const uint32_t B3_IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u,
                                  0xA54FF53Au, 0x510E527Fu, 0x9B05688Cu,
                                  0x1F83D9ABu, 0x5BE0CD19u};

static const uint8_t B3_PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13,
                                    1, 11, 12, 5, 9, 14, 15, 8};

static inline uint32_t rotr32(uint32_t x, int n) {
  return (x >> n) | (x << (32 - n));
}

static inline uint32_t load32le(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
         ((uint32_t)p[3] << 24);
}

static inline void store32le(uint8_t *p, uint32_t w) {
  p[0] = (uint8_t)w;
  p[1] = (uint8_t)(w >> 8);
  p[2] = (uint8_t)(w >> 16);
  p[3] = (uint8_t)(w >> 24);
}

static inline void b3_g(uint32_t *s, int a, int b, int c, int d, uint32_t x,
                        uint32_t y) {
  s[a] = s[a] + s[b] + x;
  s[d] = rotr32(s[d] ^ s[a], 16);
  s[c] = s[c] + s[d];
  s[b] = rotr32(s[b] ^ s[c], 12);
  s[a] = s[a] + s[b] + y;
  s[d] = rotr32(s[d] ^ s[a], 8);
  s[c] = s[c] + s[d];
  s[b] = rotr32(s[b] ^ s[c], 7);
}

/* Full compression; writes the 16-word output (first 8 words = new CV). */
static void b3_compress(const uint32_t cv[8], const uint8_t block[64],
                        uint64_t counter, uint32_t block_len, uint32_t flags,
                        uint32_t out[16]) {
  uint32_t m[16], t[16], s[16];
  for (int i = 0; i < 16; i++) m[i] = load32le(block + 4 * i);
  for (int i = 0; i < 8; i++) s[i] = cv[i];
  s[8] = B3_IV[0];
  s[9] = B3_IV[1];
  s[10] = B3_IV[2];
  s[11] = B3_IV[3];
  s[12] = (uint32_t)counter;
  s[13] = (uint32_t)(counter >> 32);
  s[14] = block_len;
  s[15] = flags;
  for (int r = 0; r < 7; r++) {
    b3_g(s, 0, 4, 8, 12, m[0], m[1]);
    b3_g(s, 1, 5, 9, 13, m[2], m[3]);
    b3_g(s, 2, 6, 10, 14, m[4], m[5]);
    b3_g(s, 3, 7, 11, 15, m[6], m[7]);
    b3_g(s, 0, 5, 10, 15, m[8], m[9]);
    b3_g(s, 1, 6, 11, 12, m[10], m[11]);
    b3_g(s, 2, 7, 8, 13, m[12], m[13]);
    b3_g(s, 3, 4, 9, 14, m[14], m[15]);
    if (r < 6) {
      for (int i = 0; i < 16; i++) t[i] = m[B3_PERM[i]];
      memcpy(m, t, sizeof m);
    }
  }
  for (int i = 0; i < 8; i++) {
    out[i] = s[i] ^ s[i + 8];
    out[i + 8] = s[i + 8] ^ cv[i];
  }
}

/* Output of a node: either a chunk's last block or a parent block, kept
 * un-compressed so the caller decides between CV and ROOT output. */
typedef struct {
  uint32_t cv[8];
  uint8_t block[64];
  uint64_t counter;
  uint32_t block_len;
  uint32_t flags;
} b3_output;

static void b3_output_cv(const b3_output *o, uint32_t cv[8]) {
  uint32_t w[16];
  b3_compress(o->cv, o->block, o->counter, o->block_len, o->flags, w);
  memcpy(cv, w, 32);
}

static void b3_output_root(const b3_output *o, uint8_t out32[32]) {
  uint32_t w[16];
  /* root output block 0: counter 0, ROOT flag added */
  b3_compress(o->cv, o->block, 0, o->block_len, o->flags | B3_ROOT, w);
  for (int i = 0; i < 8; i++) store32le(out32 + 4 * i, w[i]);
}

/* Chunk `chunk_index` holding `len` (0..1024) bytes at `in`. */
static void b3_chunk_output(const uint32_t key[8], uint32_t base_flags,
                            const uint8_t *in, size_t len,
                            uint64_t chunk_index, b3_output *o) {
  uint32_t cv[8];
  memcpy(cv, key, 32);
  size_t nblocks = len == 0 ? 1 : (len + B3_BLOCK - 1) / B3_BLOCK;
  for (size_t b = 0; b < nblocks; b++) {
    uint8_t blk[64];
    size_t off = b * B3_BLOCK;
    size_t bl = len - off < B3_BLOCK ? len - off : B3_BLOCK;
    if (len == 0) bl = 0;
    memset(blk, 0, sizeof blk);
    if (bl) memcpy(blk, in + off, bl);
    uint32_t flags = base_flags;
    if (b == 0) flags |= B3_CHUNK_START;
    if (b == nblocks - 1) {
      flags |= B3_CHUNK_END;
      memcpy(o->cv, cv, 32);
      memcpy(o->block, blk, 64);
      o->counter = chunk_index;
      o->block_len = (uint32_t)bl;
      o->flags = flags;
      return;
    }
    uint32_t w[16];
    b3_compress(cv, blk, chunk_index, (uint32_t)bl, flags, w);
    memcpy(cv, w, 32);
  }
}

static void b3_parent_output(const uint32_t key[8], uint32_t base_flags,
                             const uint32_t l[8], const uint32_t r[8],
                             b3_output *o) {
  memcpy(o->cv, key, 32);
  for (int i = 0; i < 8; i++) {
    store32le(o->block + 4 * i, l[i]);
    store32le(o->block + 32 + 4 * i, r[i]);
  }
  o->counter = 0;
  o->block_len = 64;
  o->flags = base_flags | B3_PARENT;
}

static uint64_t largest_pow2_below(uint64_t n) { /* n >= 2 */
  uint64_t p = 1;
  while (p * 2 < n) p *= 2;
  return p;
}

/* Recursive subtree over chunks [first_chunk, first_chunk + n_chunks). */
static void b3_subtree_output(const uint32_t key[8], uint32_t base_flags,
                              const uint8_t *in, size_t len,
                              uint64_t first_chunk, b3_output *o) {
  uint64_t n_chunks = len <= B3_CHUNK ? 1 : (len + B3_CHUNK - 1) / B3_CHUNK;
  if (n_chunks == 1) {
    b3_chunk_output(key, base_flags, in, len, first_chunk, o);
    return;
  }
  uint64_t left_chunks = largest_pow2_below(n_chunks);
  size_t left_len = (size_t)(left_chunks * B3_CHUNK);
  b3_output lo, ro;
  uint32_t lcv[8], rcv[8];
  b3_subtree_output(key, base_flags, in, left_len, first_chunk, &lo);
  b3_subtree_output(key, base_flags, in + left_len, len - left_len,
                    first_chunk + left_chunks, &ro);
  b3_output_cv(&lo, lcv);
  b3_output_cv(&ro, rcv);
  b3_parent_output(key, base_flags, lcv, rcv, o);
}

static void b3_hash_keyed_flags(const uint32_t key[8], uint32_t flags,
                                const uint8_t *in, size_t len,
                                uint8_t out32[32]) {
  b3_output o;
  b3_subtree_output(key, flags, in, len, 0, &o);
  b3_output_root(&o, out32);
}

/* BLAKE3 hash mode (key = IV, flags 0) -- blake3::Hasher::new / hash. */
void orc_blake3(const uint8_t *in, size_t len, uint8_t out32[32]) {
  b3_hash_keyed_flags(B3_IV, 0, in, len, out32);
}

/* blake3::derive_key(context, material). */
void orc_blake3_derive_key(const char *context, size_t context_len,
                           const uint8_t *material, size_t material_len,
                           uint8_t out32[32]) {
  uint8_t ck[32];
  uint32_t ckw[8];
  b3_hash_keyed_flags(B3_IV, B3_DERIVE_KEY_CONTEXT, (const uint8_t *)context,
                      context_len, ck);
  for (int i = 0; i < 8; i++) ckw[i] = load32le(ck + 4 * i);
  b3_hash_keyed_flags(ckw, B3_DERIVE_KEY_MATERIAL, material, material_len,
                      out32);
}

/* blake3::keyed_hash(key, input). */
void orc_blake3_keyed(const uint8_t key32[32], const uint8_t *in, size_t len,
                      uint8_t out32[32]) {
  uint32_t kw[8];
  for (int i = 0; i < 8; i++) kw[i] = load32le(key32 + 4 * i);
  b3_hash_keyed_flags(kw, B3_KEYED_HASH, in, len, out32);
}

/* ------------------------------------------------------------------------- */
/* Balloon hashing over BLAKE3 hash mode: the reference's only known-answer  */
/* tests that run BLAKE3 in hash mode (the mode cas.rs and hash.rs use).     */
/* ------------------------------------------------------------------------- */
/*
 * Restates `Algorithm::Balloon` of the third-party crate balloon-hash 0.4.0
 * (/root/reference/Cargo.lock:492-500; not vendored) as the reference calls
 * it: Balloon::<blake3::Hasher>::new(Algorithm::Balloon, params, Some(secret))
 * .hash_into(password, salt, key) (crates/crypto/src/keys/hashing.rs:95-114;
 * params (s_cost, t_cost, p_cost) = (131072|262144|524288, 2, 1), :58-63;
 * with no secret the crate still receives Some(&[]), :101).  The algorithm is
 * Boneh, Corrigan-Gibbs and Schechter's Balloon (eprint 2016/027 §3.1) with
 * delta = 3, every hash H = BLAKE3 of the concatenation of its arguments:
 *   cnt = 0
 *   buf[0] = H(cnt++ u64le, pwd, salt, secret)
 *   buf[m] = H(cnt++, buf[m-1])                          m = 1 .. s-1
 *   for t < t_cost, m < s:
 *     buf[m] = H(cnt++, buf[(m-1) mod s], buf[m])
 *     for i < 3:
 *       idx   = H(t u64le, m u64le, i u64le)
 *       other = H(cnt++, salt, secret, idx) as a 256-bit LE integer mod s
 *       buf[m] = H(cnt++, buf[m], buf[other])
 *   key = buf[s-1]
 * Pinned by the six HASH_B3BALLOON_* vectors (hashing.rs:180-208, tests
 * :269-321; password :130, salt :138-141, secret :143-146). */
/* Optional transcript: every stride-th hashed message (<= 128 B kept) and its
 * digest, so a test can replay the KAT's own messages through another hasher. */
typedef struct {
  uint64_t stride, seen, kept, cap;
  uint8_t *msg;  /* [cap][128] */
  uint32_t *len; /* [cap] */
  uint8_t *dig;  /* [cap][32] */
} bal_trace;

static void b3_cat(bal_trace *tr, uint8_t out32[32], int nparts,
                   const uint8_t *const *p, const size_t *l) {
  uint8_t msg[1024];
  size_t n = 0;
  for (int i = 0; i < nparts; i++) {
    memcpy(msg + n, p[i], l[i]);
    n += l[i];
  }
  orc_blake3(msg, n, out32);
  if (tr && tr->seen++ % tr->stride == 0 && tr->kept < tr->cap && n <= 128) {
    memcpy(tr->msg + 128 * tr->kept, msg, n);
    tr->len[tr->kept] = (uint32_t)n;
    memcpy(tr->dig + 32 * tr->kept, out32, 32);
    tr->kept++;
  }
}

static void le64(uint8_t b[8], uint64_t x) {
  for (int i = 0; i < 8; i++) b[i] = (uint8_t)(x >> (8 * i));
}

static int balloon_run(bal_trace *tr, const uint8_t *pwd, size_t pwd_len,
                       const uint8_t *salt, size_t salt_len, const uint8_t *secret,
                       size_t secret_len, uint32_t s_cost, uint32_t t_cost,
                       uint8_t out32[32]) {
  if (s_cost == 0 || t_cost == 0 || pwd_len + salt_len + secret_len > 900 ||
      salt_len + secret_len > 900)
    return -EINVAL;
  uint8_t (*buf)[32] = malloc((size_t)32 * s_cost);
  if (!buf) return -ENOMEM;
  uint64_t cnt = 0;
  uint8_t c8[8], t8[8], m8[8], i8[8], idx[32], oth[32];
  le64(c8, cnt++);
  {
    const uint8_t *p[4] = {c8, pwd, salt, secret};
    const size_t l[4] = {8, pwd_len, salt_len, secret_len};
    b3_cat(tr, buf[0], 4, p, l);
  }
  for (uint32_t m = 1; m < s_cost; m++) {
    le64(c8, cnt++);
    const uint8_t *p[2] = {c8, buf[m - 1]};
    const size_t l[2] = {8, 32};
    b3_cat(tr, buf[m], 2, p, l);
  }
  for (uint64_t t = 0; t < t_cost; t++) {
    for (uint32_t m = 0; m < s_cost; m++) {
      const uint8_t *prev = buf[m == 0 ? s_cost - 1 : m - 1];
      le64(c8, cnt++);
      {
        const uint8_t *p[3] = {c8, prev, buf[m]};
        const size_t l[3] = {8, 32, 32};
        b3_cat(tr, buf[m], 3, p, l);
      }
      for (uint64_t i = 0; i < 3; i++) {
        le64(t8, t);
        le64(m8, m);
        le64(i8, i);
        {
          const uint8_t *p[3] = {t8, m8, i8};
          const size_t l[3] = {8, 8, 8};
          b3_cat(tr, idx, 3, p, l);
        }
        le64(c8, cnt++);
        {
          const uint8_t *p[4] = {c8, salt, secret, idx};
          const size_t l[4] = {8, salt_len, secret_len, 32};
          b3_cat(tr, oth, 4, p, l);
        }
        uint64_t r = 0; /* (digest as little-endian 256-bit integer) mod s_cost */
        for (int k = 31; k >= 0; k--) r = ((r << 8) | oth[k]) % s_cost;
        le64(c8, cnt++);
        {
          const uint8_t *p[3] = {c8, buf[m], buf[r]};
          const size_t l[3] = {8, 32, 32};
          b3_cat(tr, buf[m], 3, p, l);
        }
      }
    }
  }
  memcpy(out32, buf[s_cost - 1], 32);
  free(buf);
  return 0;
}

int orc_balloon_blake3(const uint8_t *pwd, size_t pwd_len, const uint8_t *salt,
                       size_t salt_len, const uint8_t *secret, size_t secret_len,
                       uint32_t s_cost, uint32_t t_cost, uint8_t out32[32]) {
  return balloon_run(NULL, pwd, pwd_len, salt, salt_len, secret, secret_len, s_cost,
                     t_cost, out32);
}

/* Same, recording every `stride`-th hashed message: msg [cap][128], len [cap],
 * dig [cap][32]; returns the number kept (or -errno). */
int64_t orc_balloon_blake3_trace(const uint8_t *pwd, size_t pwd_len, const uint8_t *salt,
                                 size_t salt_len, const uint8_t *secret,
                                 size_t secret_len, uint32_t s_cost, uint32_t t_cost,
                                 uint8_t out32[32], uint64_t stride, uint64_t cap,
                                 uint8_t *msg, uint32_t *len, uint8_t *dig) {
  bal_trace tr = {stride ? stride : 1, 0, 0, cap, msg, len, dig};
  const int rc = balloon_run(&tr, pwd, pwd_len, salt, salt_len, secret, secret_len,
                             s_cost, t_cost, out32);
  return rc ? rc : (int64_t)tr.kept;
}

/* ------------------------------------------------------------------------- */
/* Multi-threaded full-input hash (for multi-GiB parity checks and the CPU   */
/* baseline of the validator).  Splits the input at the top levels of the    */
/* BLAKE3 tree: the subtrees are hashed in parallel, the top is recombined     */
/* with the same recursive rule, so the result equals orc_blake3().           */
/* ------------------------------------------------------------------------- */

typedef struct {
  const uint8_t *in;
  size_t len;
  uint64_t first;
  int threads;
  b3_output out;
} mt_job;

static void mt_subtree_output(const uint8_t *in, size_t len,
                              uint64_t first_chunk, int threads,
                              b3_output *o);

static void *mt_worker(void *arg) {
  mt_job *j = (mt_job *)arg;
  mt_subtree_output(j->in, j->len, j->first, j->threads, &j->out);
  return NULL;
}

/* Output of the subtree over [first_chunk, +len) using up to `threads`
 * threads: the left (power-of-two) subtree runs on a new thread, the right
 * one on this thread, then the parent is formed exactly as the recursive
 * single-thread rule does. */
static void mt_subtree_output(const uint8_t *in, size_t len,
                              uint64_t first_chunk, int threads,
                              b3_output *o) {
  uint64_t n_chunks = len <= B3_CHUNK ? 1 : (len + B3_CHUNK - 1) / B3_CHUNK;
  if (threads <= 1 || n_chunks < 64) {
    b3_subtree_output(B3_IV, 0, in, len, first_chunk, o);
    return;
  }
  uint64_t left_chunks = largest_pow2_below(n_chunks);
  size_t left_len = (size_t)(left_chunks * B3_CHUNK);
  int lt = threads / 2, rt = threads - lt;
  mt_job jl = {in, left_len, first_chunk, lt, {{0}, {0}, 0, 0, 0}};
  b3_output ro;
  uint32_t lcv[8], rcv[8];
  pthread_t th;
  int spawned = pthread_create(&th, NULL, mt_worker, &jl) == 0;
  if (!spawned) mt_worker(&jl);
  mt_subtree_output(in + left_len, len - left_len, first_chunk + left_chunks,
                    rt, &ro);
  if (spawned) pthread_join(th, NULL);
  b3_output_cv(&jl.out, lcv);
  b3_output_cv(&ro, rcv);
  b3_parent_output(B3_IV, 0, lcv, rcv, o);
}

void orc_blake3_mt(const uint8_t *in, size_t len, int threads,
                   uint8_t out32[32]) {
  b3_output o;
  mt_subtree_output(in, len, 0, threads, &o);
  b3_output_root(&o, out32);
}

/* ------------------------------------------------------------------------- */
/* Incremental hasher with the reference crate's update()/finalize() shape.   */
/* Used by the path-based restatements below (bytes arrive in reads).        */
/* ------------------------------------------------------------------------- */

typedef struct {
  uint32_t cv_stack[64][8];
  int stack_len;
  uint32_t chunk_cv[8];
  uint64_t chunk_counter;
  uint8_t buf[64];
  uint32_t buf_len;
  uint32_t blocks_compressed;
} orc_hasher;

static void h_init(orc_hasher *h) {
  memset(h, 0, sizeof *h);
  memcpy(h->chunk_cv, B3_IV, 32);
}

static void h_push_cv(orc_hasher *h, const uint32_t cv_in[8],
                      uint64_t total_chunks) {
  uint32_t cv[8];
  memcpy(cv, cv_in, 32);
  while ((total_chunks & 1) == 0) {
    b3_output o;
    h->stack_len--;
    b3_parent_output(B3_IV, 0, h->cv_stack[h->stack_len], cv, &o);
    b3_output_cv(&o, cv);
    total_chunks >>= 1;
  }
  memcpy(h->cv_stack[h->stack_len++], cv, 32);
}

static void h_update(orc_hasher *h, const uint8_t *in, size_t len) {
  while (len) {
    /* a full chunk is finished only when more input arrives */
    if (h->blocks_compressed == 15 && h->buf_len == 64) {
      b3_output o;
      memcpy(o.cv, h->chunk_cv, 32);
      memcpy(o.block, h->buf, 64);
      o.counter = h->chunk_counter;
      o.block_len = 64;
      o.flags = B3_CHUNK_END | (h->blocks_compressed == 0 ? B3_CHUNK_START : 0);
      uint32_t cv[8];
      b3_output_cv(&o, cv);
      h->chunk_counter++;
      h_push_cv(h, cv, h->chunk_counter);
      memcpy(h->chunk_cv, B3_IV, 32);
      h->buf_len = 0;
      h->blocks_compressed = 0;
    }
    if (h->buf_len == 64) {
      uint32_t w[16];
      uint32_t flags = h->blocks_compressed == 0 ? B3_CHUNK_START : 0;
      b3_compress(h->chunk_cv, h->buf, h->chunk_counter, 64, flags, w);
      memcpy(h->chunk_cv, w, 32);
      h->blocks_compressed++;
      h->buf_len = 0;
    }
    size_t take = 64 - h->buf_len;
    if (take > len) take = len;
    memcpy(h->buf + h->buf_len, in, take);
    h->buf_len += (uint32_t)take;
    in += take;
    len -= take;
  }
}

static void h_finalize(orc_hasher *h, uint8_t out32[32]) {
  b3_output o;
  memcpy(o.cv, h->chunk_cv, 32);
  memset(o.block, 0, 64);
  memcpy(o.block, h->buf, h->buf_len);
  o.counter = h->chunk_counter;
  o.block_len = h->buf_len;
  o.flags = B3_CHUNK_END | (h->blocks_compressed == 0 ? B3_CHUNK_START : 0);
  for (int i = h->stack_len - 1; i >= 0; i--) {
    uint32_t cv[8];
    b3_output_cv(&o, cv);
    b3_parent_output(B3_IV, 0, h->cv_stack[i], cv, &o);
  }
  b3_output_root(&o, out32);
}

/* ------------------------------------------------------------------------- */
/* generate_cas_id  -- /root/reference/core/src/object/cas.rs:10-62          */
/* ------------------------------------------------------------------------- */

#define CAS_SAMPLE_COUNT 4u              /* cas.rs:10 */
#define CAS_SAMPLE_SIZE (1024u * 10u)    /* cas.rs:11 */
#define CAS_HEADER_OR_FOOTER (1024u * 8u) /* cas.rs:12 */
#define CAS_MINIMUM_FILE_SIZE (1024u * 100u) /* cas.rs:15 */
#define CAS_LARGE_MSG_LEN (8u + 2u * CAS_HEADER_OR_FOOTER + CAS_SAMPLE_COUNT * CAS_SAMPLE_SIZE)

static const char HEXD[] = "0123456789abcdef";

static void hex_of(const uint8_t *d, int n, char *out) {
  for (int i = 0; i < n; i++) {
    out[2 * i] = HEXD[d[i] >> 4];
    out[2 * i + 1] = HEXD[d[i] & 15];
  }
  out[2 * n] = 0;
}

/* Length of the cas message M for a file whose stat size is `size` and whose
 * content length is `size` (the synthetic / consistent case). */
uint32_t orc_cas_msg_len(uint64_t size) {
  return size <= CAS_MINIMUM_FILE_SIZE ? (uint32_t)(8 + size) : CAS_LARGE_MSG_LEN;
}

/* Builds M from the full file bytes `file[0..file_len)` and the `size`
 * argument passed to generate_cas_id, following cas.rs:24-58 exactly:
 *  - size <= 100 KiB: the whole file as read (cas.rs:29);
 *  - else header file[0,8192) (:35-38), samples at 8192 + k*seek_jump
 *    with seek_jump = (size - 16384)/4 computed from `size` (:41-51),
 *    footer = last 8192 bytes of the ACTUAL file (SeekFrom::End, :54-58).
 * Returns the message length, or -1 where the reference's read_exact fails
 * (UnexpectedEof).  `out` must hold max(8 + file_len, 57352) bytes. */
int64_t orc_cas_build_message(const uint8_t *file, uint64_t file_len,
                              uint64_t size, uint8_t *out) {
  for (int i = 0; i < 8; i++) out[i] = (uint8_t)(size >> (8 * i));
  if (size <= CAS_MINIMUM_FILE_SIZE) {
    memcpy(out + 8, file, file_len);
    return (int64_t)(8 + file_len);
  }
  uint8_t *p = out + 8;
  if (file_len < CAS_HEADER_OR_FOOTER) return -1;
  memcpy(p, file, CAS_HEADER_OR_FOOTER);
  p += CAS_HEADER_OR_FOOTER;
  uint64_t current_pos = CAS_HEADER_OR_FOOTER; /* read_exact returns 8192 */
  uint64_t seek_jump = (size - CAS_HEADER_OR_FOOTER * 2) / CAS_SAMPLE_COUNT;
  uint64_t file_pos = CAS_HEADER_OR_FOOTER; /* cursor after the header read */
  for (;;) {
    if (file_pos + CAS_SAMPLE_SIZE > file_len) return -1;
    memcpy(p, file + file_pos, CAS_SAMPLE_SIZE);
    p += CAS_SAMPLE_SIZE;
    if (current_pos >= CAS_HEADER_OR_FOOTER + seek_jump * (CAS_SAMPLE_COUNT - 1))
      break;
    current_pos = current_pos + seek_jump; /* seek(Start(..)) returns it */
    file_pos = current_pos;
  }
  if (file_len < CAS_HEADER_OR_FOOTER) return -1;
  memcpy(p, file + file_len - CAS_HEADER_OR_FOOTER, CAS_HEADER_OR_FOOTER);
  p += CAS_HEADER_OR_FOOTER;
  return (int64_t)(p - out);
}

/* cas_id hex (16 chars) of an already-built message. */
void orc_cas_id_of_message(const uint8_t *msg, size_t len, char out_hex[17]) {
  uint8_t h[32];
  orc_blake3(msg, len, h);
  hex_of(h, 8, out_hex); /* to_hex()[..16], cas.rs:61 */
}

static int read_exact_fd(int fd, uint8_t *buf, size_t n) {
  size_t got = 0;
  while (got < n) {
    ssize_t r = read(fd, buf + got, n - got);
    if (r < 0) {
      if (errno == EINTR) continue;
      return -errno;
    }
    if (r == 0) return -ENODATA; /* io::ErrorKind::UnexpectedEof */
    got += (size_t)r;
  }
  return 0;
}

/* Path-based restatement with the reference's I/O pattern (cas.rs:23-62).
 * Returns 0, or -errno (-ENODATA stands for UnexpectedEof). */
int orc_cas_id_path(const char *path, uint64_t size, char out_hex[17]) {
  orc_hasher h;
  h_init(&h);
  uint8_t sz[8];
  for (int i = 0; i < 8; i++) sz[i] = (uint8_t)(size >> (8 * i));
  h_update(&h, sz, 8);
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -errno;
  int rc = 0;
  if (size <= CAS_MINIMUM_FILE_SIZE) {
    /* fs::read: read the whole file whatever its current length */
    uint8_t buf[65536];
    for (;;) {
      ssize_t r = read(fd, buf, sizeof buf);
      if (r < 0) {
        if (errno == EINTR) continue;
        rc = -errno;
        break;
      }
      if (r == 0) break;
      h_update(&h, buf, (size_t)r);
    }
  } else {
    uint8_t buf[CAS_SAMPLE_SIZE];
    rc = read_exact_fd(fd, buf, CAS_HEADER_OR_FOOTER);
    if (!rc) {
      uint64_t current_pos = CAS_HEADER_OR_FOOTER;
      h_update(&h, buf, CAS_HEADER_OR_FOOTER);
      uint64_t seek_jump = (size - CAS_HEADER_OR_FOOTER * 2) / CAS_SAMPLE_COUNT;
      for (;;) {
        rc = read_exact_fd(fd, buf, CAS_SAMPLE_SIZE);
        if (rc) break;
        h_update(&h, buf, CAS_SAMPLE_SIZE);
        if (current_pos >=
            CAS_HEADER_OR_FOOTER + seek_jump * (CAS_SAMPLE_COUNT - 1))
          break;
        off_t np = lseek(fd, (off_t)(current_pos + seek_jump), SEEK_SET);
        if (np < 0) {
          rc = -errno;
          break;
        }
        current_pos = (uint64_t)np;
      }
      if (!rc) {
        if (lseek(fd, -(off_t)CAS_HEADER_OR_FOOTER, SEEK_END) < 0) rc = -errno;
        if (!rc) rc = read_exact_fd(fd, buf, CAS_HEADER_OR_FOOTER);
        if (!rc) h_update(&h, buf, CAS_HEADER_OR_FOOTER);
      }
    }
  }
  close(fd);
  if (rc) return rc;
  uint8_t out[32];
  h_finalize(&h, out);
  hex_of(out, 8, out_hex);
  return 0;
}

/* file_checksum -- validation/hash.rs:8-24: 1 MiB reads, stop on the first
 * read shorter than 1 MiB, full 64-char hex. */
int orc_file_checksum_path(const char *path, char out_hex[65]) {
  enum { BLOCK_LEN = 1048576 };
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -errno;
  uint8_t *buf = (uint8_t *)malloc(BLOCK_LEN);
  if (!buf) {
    close(fd);
    return -ENOMEM;
  }
  orc_hasher h;
  h_init(&h);
  int rc = 0;
  for (;;) {
    /* tokio File::read on a regular file returns min(len, its buffer cap);
     * modelled as a full read of up to BLOCK_LEN (open
     * assumption): loop read() until BLOCK_LEN or EOF. */
    size_t got = 0;
    while (got < BLOCK_LEN) {
      ssize_t r = read(fd, buf + got, BLOCK_LEN - got);
      if (r < 0) {
        if (errno == EINTR) continue;
        rc = -errno;
        break;
      }
      if (r == 0) break;
      got += (size_t)r;
    }
    if (rc) break;
    h_update(&h, buf, got);
    if (got != BLOCK_LEN) break;
  }
  free(buf);
  close(fd);
  if (rc) return rc;
  uint8_t out[32];
  h_finalize(&h, out);
  hex_of(out, 32, out_hex);
  return 0;
}

/* Streaming-shape hash of an in-memory buffer through the incremental hasher
 * fed in `piece`-byte updates (cross-checks the recursive tree). */
void orc_blake3_incremental(const uint8_t *in, size_t len, size_t piece,
                            uint8_t out32[32]) {
  orc_hasher h;
  h_init(&h);
  if (piece == 0) piece = 1;
  for (size_t off = 0; off < len; off += piece) {
    size_t n = len - off < piece ? len - off : piece;
    h_update(&h, in + off, n);
  }
  h_finalize(&h, out32);
}

/* ------------------------------------------------------------------------- */
/* Batched in-memory cas (CPU baseline, threads over files)                  */
/* ------------------------------------------------------------------------- */

typedef struct {
  const uint8_t *arena;
  const uint64_t *off;
  const uint32_t *len;
  uint8_t *out8;
  uint64_t begin, end;
} cas_job;

static void *cas_worker(void *arg) {
  cas_job *j = (cas_job *)arg;
  for (uint64_t i = j->begin; i < j->end; i++) {
    uint8_t h[32];
    orc_blake3(j->arena + j->off[i], j->len[i], h);
    memcpy(j->out8 + 8 * i, h, 8);
  }
  return NULL;
}

void orc_cas_batch(const uint8_t *arena, const uint64_t *off,
                   const uint32_t *len, uint64_t n, uint8_t *out8,
                   int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  cas_job jobs[256];
  for (int t = 0; t < threads; t++) {
    jobs[t].arena = arena;
    jobs[t].off = off;
    jobs[t].len = len;
    jobs[t].out8 = out8;
    jobs[t].begin = n * (uint64_t)t / (uint64_t)threads;
    jobs[t].end = n * (uint64_t)(t + 1) / (uint64_t)threads;
    pthread_create(&th[t], NULL, cas_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}

/* ------------------------------------------------------------------------- */
/* Synthetic corpus content (shared definition with csrc/synth.hip)          */
/* ------------------------------------------------------------------------- */

static inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* Byte at offset `o` of the synthetic file with content seed `seed`. */
static inline uint8_t synth_byte(uint64_t seed, uint64_t o) {
  uint64_t w = mix64(seed + (o >> 3) * 0x9E3779B97F4A7C15ull);
  return (uint8_t)(w >> (8 * (o & 7)));
}

void orc_synth_file_bytes(uint64_t seed, uint64_t offset, uint64_t n,
                          uint8_t *out) {
  for (uint64_t i = 0; i < n; i++) out[i] = synth_byte(seed, offset + i);
}

/* cas message of a synthetic file (size, seed); returns its length. */
uint32_t orc_synth_cas_message(uint64_t size, uint64_t seed, uint8_t *out) {
  for (int i = 0; i < 8; i++) out[i] = (uint8_t)(size >> (8 * i));
  if (size <= CAS_MINIMUM_FILE_SIZE) {
    orc_synth_file_bytes(seed, 0, size, out + 8);
    return (uint32_t)(8 + size);
  }
  uint8_t *p = out + 8;
  uint64_t jump = (size - 2 * CAS_HEADER_OR_FOOTER) / CAS_SAMPLE_COUNT;
  orc_synth_file_bytes(seed, 0, CAS_HEADER_OR_FOOTER, p);
  p += CAS_HEADER_OR_FOOTER;
  for (uint32_t k = 0; k < CAS_SAMPLE_COUNT; k++) {
    orc_synth_file_bytes(seed, CAS_HEADER_OR_FOOTER + k * jump,
                         CAS_SAMPLE_SIZE, p);
    p += CAS_SAMPLE_SIZE;
  }
  orc_synth_file_bytes(seed, size - CAS_HEADER_OR_FOOTER, CAS_HEADER_OR_FOOTER,
                       p);
  return CAS_LARGE_MSG_LEN;
}

/* Synthetic cas arena for n files, packed at 128-byte aligned offsets
 * (the same packing rule as the device generator).  Returns total bytes. */
uint64_t orc_synth_arena_layout(const uint64_t *sizes, uint64_t n,
                                uint64_t *off, uint32_t *len) {
  uint64_t pos = 0;
  for (uint64_t i = 0; i < n; i++) {
    len[i] = orc_cas_msg_len(sizes[i]);
    off[i] = pos;
    pos += ((uint64_t)len[i] + 127u) & ~(uint64_t)127u;
  }
  return pos;
}

typedef struct {
  const uint64_t *sizes, *seeds, *off;
  uint8_t *arena;
  uint64_t begin, end;
} synth_job;

static void *synth_worker(void *arg) {
  synth_job *j = (synth_job *)arg;
  for (uint64_t i = j->begin; i < j->end; i++)
    orc_synth_cas_message(j->sizes[i], j->seeds[i], j->arena + j->off[i]);
  return NULL;
}

void orc_synth_arena_fill(const uint64_t *sizes, const uint64_t *seeds,
                          const uint64_t *off, uint64_t n, uint8_t *arena,
                          int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  synth_job jobs[256];
  for (int t = 0; t < threads; t++) {
    jobs[t].sizes = sizes;
    jobs[t].seeds = seeds;
    jobs[t].off = off;
    jobs[t].arena = arena;
    jobs[t].begin = n * (uint64_t)t / (uint64_t)threads;
    jobs[t].end = n * (uint64_t)(t + 1) / (uint64_t)threads;
    pthread_create(&th[t], NULL, synth_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}

/* Dedup corpus rows (same definition as csrc/synth.hip k_synth_dedup). */
static uint64_t orc_perm(uint64_t x, uint64_t T, uint64_t seed) {
  uint32_t bits = 2;
  while ((1ull << bits) < T) bits += 2;
  uint32_t h = bits / 2;
  uint64_t mask = (1ull << h) - 1;
  do {
    uint64_t L = x >> h, R = x & mask;
    for (uint32_t r = 0; r < 4; r++) {
      uint64_t F = mix64(R ^ (seed + 0x632BE59BD9B4E019ull * (r + 1))) & mask;
      uint64_t nl = R;
      R = L ^ F;
      L = nl;
    }
    x = (L << h) | R;
  } while (x >= T);
  return x;
}

void orc_synth_dedup_rows(uint64_t seed, uint64_t total, uint64_t distinct,
                          uint64_t first, uint64_t n, uint64_t *key,
                          uint8_t *has_key, uint32_t *rank) {
  for (uint64_t i = 0; i < n; i++) {
    uint64_t g = first + i;
    uint64_t u = orc_perm(g, total, seed);
    uint64_t item =
        u < distinct ? u : mix64(u ^ seed ^ 0xD6E8FEB86659FD93ull) % distinct;
    key[i] = mix64(seed * 0x9E3779B97F4A7C15ull + item + 1);
    has_key[i] = (mix64(g ^ (seed << 1) ^ 0xA0761D6478BD642Full) % 1000) != 0;
    rank[i] = (uint32_t)g;
  }
}

/* ------------------------------------------------------------------------- */
/* cas_id -> Object grouping (identifier_job_step, canonical form)           */
/* ------------------------------------------------------------------------- */
/*
 * Rows are the orphan file_paths in ascending id; rank r = position.  The job
 * processes chunks of `chunk_rows` (=CHUNK_SIZE 100, mod.rs:36).  Within the
 * chunk that first contains cas key X every row with X becomes its own new
 * Object (mod.rs:233-297, nothing links them because the Object rows did not
 * exist when find_many ran, :168-175); rows with X in later chunks link to an
 * existing Object (:189-225) -- canonically the one of the lowest-rank row of
 * X.  Rows without a key (empty files, cas_id None, mod.rs:80-88) are
 * singletons (:238-239).  rep[r] = rank of the row whose Object r ends up in.
 */
typedef struct {
  uint64_t key;
  uint32_t rank;
} kr_pair;

static int kr_cmp(const void *a, const void *b) {
  const kr_pair *x = (const kr_pair *)a, *y = (const kr_pair *)b;
  if (x->key != y->key) return x->key < y->key ? -1 : 1;
  return x->rank < y->rank ? -1 : (x->rank > y->rank);
}

int orc_group_reps(const uint64_t *key, const uint8_t *has_key, uint32_t n,
                   uint32_t chunk_rows, uint32_t *rep) {
  if (chunk_rows == 0) return -EINVAL;
  kr_pair *v = (kr_pair *)malloc((size_t)n * sizeof *v + 1);
  if (!v) return -ENOMEM;
  uint32_t m = 0;
  for (uint32_t r = 0; r < n; r++) {
    rep[r] = r;
    if (has_key[r]) {
      v[m].key = key[r];
      v[m].rank = r;
      m++;
    }
  }
  qsort(v, m, sizeof *v, kr_cmp);
  for (uint32_t i = 0; i < m;) {
    uint32_t j = i;
    while (j < m && v[j].key == v[i].key) j++;
    uint32_t first = v[i].rank; /* lowest rank of the segment */
    uint32_t c0 = first / chunk_rows;
    for (uint32_t k = i; k < j; k++)
      rep[v[k].rank] = (v[k].rank / chunk_rows == c0) ? v[k].rank : first;
    i = j;
  }
  free(v);
  return 0;
}

/* ------------------------------------------------------------------------- */
/* AVX2 8-way chunk hashing (CPU BASELINE ONLY: bench.py cpu_baseline leg).  */
/* ------------------------------------------------------------------------- */
/*
 * The reference's blake3 1.4.1 crate hashes a message's full chunks several at
 * a time with SIMD (hash_many; AVX2 = 8 lanes).  This is the same idea written
 * from the spec: 8 chunks' states live transposed in 16 __m256i registers,
 * their message blocks are transposed 8x8 on load, and the parent levels are
 * hashed 8 at a time the same way (a parent block = two adjacent CVs).  The
 * tree is folded level by level, odd node carried up (BLAKE3's left-complete
 * tree).  tests/test_oracle.py checks it bit-exact against the scalar oracle.
 */
#include <immintrin.h>

typedef __m256i v8u;

static inline v8u v_add(v8u a, v8u b) { return _mm256_add_epi32(a, b); }
static inline v8u v_xor(v8u a, v8u b) { return _mm256_xor_si256(a, b); }
static inline v8u v_set1(uint32_t x) { return _mm256_set1_epi32((int)x); }
static inline v8u v_rot16(v8u x) {
  const v8u m = _mm256_setr_epi8(2, 3, 0, 1, 6, 7, 4, 5, 10, 11, 8, 9, 14, 15, 12, 13, 2, 3, 0,
                                 1, 6, 7, 4, 5, 10, 11, 8, 9, 14, 15, 12, 13);
  return _mm256_shuffle_epi8(x, m);
}
static inline v8u v_rot8(v8u x) {
  const v8u m = _mm256_setr_epi8(1, 2, 3, 0, 5, 6, 7, 4, 9, 10, 11, 8, 13, 14, 15, 12, 1, 2, 3,
                                 0, 5, 6, 7, 4, 9, 10, 11, 8, 13, 14, 15, 12);
  return _mm256_shuffle_epi8(x, m);
}
static inline v8u v_rot12(v8u x) {
  return _mm256_or_si256(_mm256_srli_epi32(x, 12), _mm256_slli_epi32(x, 20));
}
static inline v8u v_rot7(v8u x) {
  return _mm256_or_si256(_mm256_srli_epi32(x, 7), _mm256_slli_epi32(x, 25));
}

#define VG(a, b, c, d, x, y)      \
  do {                            \
    a = v_add(v_add(a, b), x);    \
    d = v_rot16(v_xor(d, a));     \
    c = v_add(c, d);              \
    b = v_rot12(v_xor(b, c));     \
    a = v_add(v_add(a, b), y);    \
    d = v_rot8(v_xor(d, a));      \
    c = v_add(c, d);              \
    b = v_rot7(v_xor(b, c));      \
  } while (0)

/* 8 compressions: h[8] in/out (transposed CVs), m[16] transposed words. */
static inline void v_compress(v8u h[8], const v8u m[16], v8u ctr_lo, v8u ctr_hi, uint32_t blen,
                              uint32_t flags) {
  static const uint8_t S[7][16] = {
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
      {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8},
      {3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1},
      {10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6},
      {12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4},
      {9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7},
      {11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13}};
  v8u v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3], v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
  v8u v8 = v_set1(B3_IV[0]), v9 = v_set1(B3_IV[1]), v10 = v_set1(B3_IV[2]),
      v11 = v_set1(B3_IV[3]);
  v8u v12 = ctr_lo, v13 = ctr_hi, v14 = v_set1(blen), v15 = v_set1(flags);
  for (int r = 0; r < 7; ++r) {
    const uint8_t *s = S[r];
    VG(v0, v4, v8, v12, m[s[0]], m[s[1]]);
    VG(v1, v5, v9, v13, m[s[2]], m[s[3]]);
    VG(v2, v6, v10, v14, m[s[4]], m[s[5]]);
    VG(v3, v7, v11, v15, m[s[6]], m[s[7]]);
    VG(v0, v5, v10, v15, m[s[8]], m[s[9]]);
    VG(v1, v6, v11, v12, m[s[10]], m[s[11]]);
    VG(v2, v7, v8, v13, m[s[12]], m[s[13]]);
    VG(v3, v4, v9, v14, m[s[14]], m[s[15]]);
  }
  h[0] = v_xor(v0, v8);
  h[1] = v_xor(v1, v9);
  h[2] = v_xor(v2, v10);
  h[3] = v_xor(v3, v11);
  h[4] = v_xor(v4, v12);
  h[5] = v_xor(v5, v13);
  h[6] = v_xor(v6, v14);
  h[7] = v_xor(v7, v15);
}

/* r[j] = 8 words (32 B) of lane j -> out[w] = word w of every lane. */
static inline void v_transpose8(const v8u r[8], v8u out[8]) {
  const v8u t0 = _mm256_unpacklo_epi32(r[0], r[1]), t1 = _mm256_unpackhi_epi32(r[0], r[1]);
  const v8u t2 = _mm256_unpacklo_epi32(r[2], r[3]), t3 = _mm256_unpackhi_epi32(r[2], r[3]);
  const v8u t4 = _mm256_unpacklo_epi32(r[4], r[5]), t5 = _mm256_unpackhi_epi32(r[4], r[5]);
  const v8u t6 = _mm256_unpacklo_epi32(r[6], r[7]), t7 = _mm256_unpackhi_epi32(r[6], r[7]);
  const v8u u0 = _mm256_unpacklo_epi64(t0, t2), u1 = _mm256_unpackhi_epi64(t0, t2);
  const v8u u2 = _mm256_unpacklo_epi64(t1, t3), u3 = _mm256_unpackhi_epi64(t1, t3);
  const v8u u4 = _mm256_unpacklo_epi64(t4, t6), u5 = _mm256_unpackhi_epi64(t4, t6);
  const v8u u6 = _mm256_unpacklo_epi64(t5, t7), u7 = _mm256_unpackhi_epi64(t5, t7);
  out[0] = _mm256_permute2x128_si256(u0, u4, 0x20);
  out[1] = _mm256_permute2x128_si256(u1, u5, 0x20);
  out[2] = _mm256_permute2x128_si256(u2, u6, 0x20);
  out[3] = _mm256_permute2x128_si256(u3, u7, 0x20);
  out[4] = _mm256_permute2x128_si256(u0, u4, 0x31);
  out[5] = _mm256_permute2x128_si256(u1, u5, 0x31);
  out[6] = _mm256_permute2x128_si256(u2, u6, 0x31);
  out[7] = _mm256_permute2x128_si256(u3, u7, 0x31);
}

/* Words of 64-byte block b of the 8 inputs p[j] (+ 64 b), transposed. */
static inline void v_load_block(const uint8_t *const p[8], size_t boff, v8u m[16]) {
  v8u r[8];
  for (int j = 0; j < 8; ++j) r[j] = _mm256_loadu_si256((const v8u *)(p[j] + boff));
  v_transpose8(r, m);
  for (int j = 0; j < 8; ++j) r[j] = _mm256_loadu_si256((const v8u *)(p[j] + boff + 32));
  v_transpose8(r, m + 8);
}

static inline void v_store_cvs(const v8u h[8], uint32_t *out[8]) {
  v8u t[8];
  v_transpose8(h, t); /* t[j] = CV of lane j (the transpose is an involution) */
  for (int j = 0; j < 8; ++j) _mm256_storeu_si256((v8u *)out[j], t[j]);
}

/* CVs of 8 FULL non-root chunks p[j] with chunk counters ctr0 + j. */
static void v_chunks8(const uint8_t *const p[8], uint64_t ctr0, uint32_t *out[8]) {
  v8u h[8], m[16];
  for (int w = 0; w < 8; ++w) h[w] = v_set1(B3_IV[w]);
  uint32_t lo[8], hi[8];
  for (int j = 0; j < 8; ++j) {
    lo[j] = (uint32_t)(ctr0 + j);
    hi[j] = (uint32_t)((ctr0 + j) >> 32);
  }
  const v8u clo = _mm256_loadu_si256((const v8u *)lo), chi = _mm256_loadu_si256((const v8u *)hi);
  for (int b = 0; b < 16; ++b) {
    v_load_block(p, (size_t)64 * b, m);
    v_compress(h, m, clo, chi, 64, (b == 0 ? B3_CHUNK_START : 0) | (b == 15 ? B3_CHUNK_END : 0));
  }
  v_store_cvs(h, out);
}

/* 8 parents: out[j] = P(cvs[2k], cvs[2k+1]) for pair k = k0 + j (8 words each). */
static void v_parents8(const uint32_t *pairs[8], uint32_t *out[8]) {
  v8u h[8], m[16];
  for (int w = 0; w < 8; ++w) h[w] = v_set1(B3_IV[w]);
  const uint8_t *p[8];
  for (int j = 0; j < 8; ++j) p[j] = (const uint8_t *)pairs[j];
  v_load_block(p, 0, m);
  const v8u z = _mm256_setzero_si256();
  v_compress(h, m, z, z, 64, B3_PARENT);
  v_store_cvs(h, out);
}

static void s_chunk_cv(const uint8_t *p, size_t clen, uint64_t ctr, uint32_t cv[8]) {
  b3_output o;
  b3_chunk_output(B3_IV, 0, p, clen, ctr, &o);
  b3_output_cv(&o, cv);
}

static void s_parent_cv(const uint32_t l[8], const uint32_t r[8], uint32_t flags,
                        uint32_t cv[8]) {
  b3_output o;
  b3_parent_output(B3_IV, 0, l, r, &o);
  uint32_t w[16];
  b3_compress(o.cv, o.block, 0, 64, o.flags | flags, w);
  memcpy(cv, w, 32);
}

/* ------------------------------------------------------------------------- */
/* AVX-512 16-way (CPU BASELINE ONLY), used when the host has AVX-512F/VL:    */
/* the blake3 crate's hash_many takes 16 inputs at a time there, so an AVX2   */
/* baseline would understate the reference on such a host.  Same scheme as   */
/* above with 16 lanes: native 32-bit rotates (vprord), a 16 x 16 word        */
/* transpose per 64-byte block.                                               */
/* ------------------------------------------------------------------------- */
#define T512 __attribute__((target("avx512f,avx512vl")))
typedef __m512i v16u;

#define WG(a, b, c, d, x, y)                          \
  do {                                                \
    a = _mm512_add_epi32(_mm512_add_epi32(a, b), x);  \
    d = _mm512_ror_epi32(_mm512_xor_si512(d, a), 16); \
    c = _mm512_add_epi32(c, d);                       \
    b = _mm512_ror_epi32(_mm512_xor_si512(b, c), 12); \
    a = _mm512_add_epi32(_mm512_add_epi32(a, b), y);  \
    d = _mm512_ror_epi32(_mm512_xor_si512(d, a), 8);  \
    c = _mm512_add_epi32(c, d);                       \
    b = _mm512_ror_epi32(_mm512_xor_si512(b, c), 7);  \
  } while (0)

T512 static inline void w_compress(v16u h[8], const v16u m[16], v16u ctr_lo, v16u ctr_hi,
                                   uint32_t blen, uint32_t flags) {
  static const uint8_t S[7][16] = {
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
      {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8},
      {3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1},
      {10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6},
      {12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4},
      {9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7},
      {11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13}};
  v16u v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3], v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
  v16u v8 = _mm512_set1_epi32((int)B3_IV[0]), v9 = _mm512_set1_epi32((int)B3_IV[1]),
       v10 = _mm512_set1_epi32((int)B3_IV[2]), v11 = _mm512_set1_epi32((int)B3_IV[3]);
  v16u v12 = ctr_lo, v13 = ctr_hi, v14 = _mm512_set1_epi32((int)blen),
       v15 = _mm512_set1_epi32((int)flags);
  for (int r = 0; r < 7; ++r) {
    const uint8_t *sg = S[r];
    WG(v0, v4, v8, v12, m[sg[0]], m[sg[1]]);
    WG(v1, v5, v9, v13, m[sg[2]], m[sg[3]]);
    WG(v2, v6, v10, v14, m[sg[4]], m[sg[5]]);
    WG(v3, v7, v11, v15, m[sg[6]], m[sg[7]]);
    WG(v0, v5, v10, v15, m[sg[8]], m[sg[9]]);
    WG(v1, v6, v11, v12, m[sg[10]], m[sg[11]]);
    WG(v2, v7, v8, v13, m[sg[12]], m[sg[13]]);
    WG(v3, v4, v9, v14, m[sg[14]], m[sg[15]]);
  }
  h[0] = _mm512_xor_si512(v0, v8);
  h[1] = _mm512_xor_si512(v1, v9);
  h[2] = _mm512_xor_si512(v2, v10);
  h[3] = _mm512_xor_si512(v3, v11);
  h[4] = _mm512_xor_si512(v4, v12);
  h[5] = _mm512_xor_si512(v5, v13);
  h[6] = _mm512_xor_si512(v6, v14);
  h[7] = _mm512_xor_si512(v7, v15);
}

/* r[j] = the 16 words of lane j -> m[w] = word w of every lane.  32-bit then
 * 64-bit unpacks inside 128-bit lanes, then two 128-bit lane shuffles. */
T512 static inline void w_transpose16(const v16u r[16], v16u m[16]) {
  v16u t[16], u[16];
  for (int i = 0; i < 8; ++i) {
    t[2 * i] = _mm512_unpacklo_epi32(r[2 * i], r[2 * i + 1]);
    t[2 * i + 1] = _mm512_unpackhi_epi32(r[2 * i], r[2 * i + 1]);
  }
  for (int i = 0; i < 4; ++i) {  /* u[4i + k], 128-bit lane L: rows 4i..4i+3 of word 4L + k */
    u[4 * i + 0] = _mm512_unpacklo_epi64(t[4 * i + 0], t[4 * i + 2]);
    u[4 * i + 1] = _mm512_unpackhi_epi64(t[4 * i + 0], t[4 * i + 2]);
    u[4 * i + 2] = _mm512_unpacklo_epi64(t[4 * i + 1], t[4 * i + 3]);
    u[4 * i + 3] = _mm512_unpackhi_epi64(t[4 * i + 1], t[4 * i + 3]);
  }
  for (int k = 0; k < 4; ++k) {
    const v16u x0 = _mm512_shuffle_i32x4(u[k], u[4 + k], 0x44);
    const v16u x1 = _mm512_shuffle_i32x4(u[8 + k], u[12 + k], 0x44);
    const v16u x2 = _mm512_shuffle_i32x4(u[k], u[4 + k], 0xEE);
    const v16u x3 = _mm512_shuffle_i32x4(u[8 + k], u[12 + k], 0xEE);
    m[k] = _mm512_shuffle_i32x4(x0, x1, 0x88);
    m[4 + k] = _mm512_shuffle_i32x4(x0, x1, 0xDD);
    m[8 + k] = _mm512_shuffle_i32x4(x2, x3, 0x88);
    m[12 + k] = _mm512_shuffle_i32x4(x2, x3, 0xDD);
  }
}

T512 static inline void w_store_cvs(const v16u h[8], uint32_t *out[16]) {
  uint32_t t[8][16] __attribute__((aligned(64)));
  for (int w = 0; w < 8; ++w) _mm512_store_si512((void *)t[w], h[w]);
  for (int j = 0; j < 16; ++j)
    for (int w = 0; w < 8; ++w) out[j][w] = t[w][j];
}

/* CVs of 16 FULL non-root chunks p[j] with chunk counters ctr0 + j. */
T512 static void w_chunks16(const uint8_t *const p[16], uint64_t ctr0, uint32_t *out[16]) {
  v16u h[8], m[16], r[16];
  for (int w = 0; w < 8; ++w) h[w] = _mm512_set1_epi32((int)B3_IV[w]);
  uint32_t lo[16], hi[16];
  for (int j = 0; j < 16; ++j) {
    lo[j] = (uint32_t)(ctr0 + j);
    hi[j] = (uint32_t)((ctr0 + j) >> 32);
  }
  const v16u clo = _mm512_loadu_si512(lo), chi = _mm512_loadu_si512(hi);
  for (int b = 0; b < 16; ++b) {
    for (int j = 0; j < 16; ++j) r[j] = _mm512_loadu_si512(p[j] + 64 * b);
    w_transpose16(r, m);
    w_compress(h, m, clo, chi, 64, (b == 0 ? B3_CHUNK_START : 0) | (b == 15 ? B3_CHUNK_END : 0));
  }
  w_store_cvs(h, out);
}

/* 16 parents: out[j] = P(pairs[j][0..8), pairs[j][8..16)). */
T512 static void w_parents16(const uint32_t *pairs[16], uint32_t *out[16]) {
  v16u h[8], m[16], r[16];
  for (int w = 0; w < 8; ++w) h[w] = _mm512_set1_epi32((int)B3_IV[w]);
  for (int j = 0; j < 16; ++j) r[j] = _mm512_loadu_si512(pairs[j]);
  w_transpose16(r, m);
  const v16u z = _mm512_setzero_si512();
  w_compress(h, m, z, z, 64, B3_PARENT);
  w_store_cvs(h, out);
}

/* 16 when the host has AVX-512F/VL (the crate's hash_many width there), else 8. */
int orc_simd_width(void) {
  static int w = 0;
  if (!w) {
    __builtin_cpu_init();
    w = (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl")) ? 16 : 8;
    const char *e = getenv("ORC_SIMD_WIDTH"); /* "8": the AVX2 path on any host (A/B) */
    if (e && e[0] == '8') w = 8;
  }
  return w;
}

/* CVs of `count` consecutive FULL non-root chunks at p (counters ctr0..),
 * 16 / 8 at a time, the rest one by one. */
static void chunks_batch(const uint8_t *p, size_t count, uint64_t ctr0, uint32_t (*out)[8]) {
  size_t c = 0;
  if (orc_simd_width() == 16)
    for (; c + 16 <= count; c += 16) {
      const uint8_t *pp[16];
      uint32_t *o[16];
      for (int j = 0; j < 16; ++j) {
        pp[j] = p + (c + j) * B3_CHUNK;
        o[j] = out[c + j];
      }
      w_chunks16(pp, ctr0 + c, o);
    }
  for (; c + 8 <= count; c += 8) {
    const uint8_t *pp[8];
    uint32_t *o[8];
    for (int j = 0; j < 8; ++j) {
      pp[j] = p + (c + j) * B3_CHUNK;
      o[j] = out[c + j];
    }
    v_chunks8(pp, ctr0 + c, o);
  }
  for (; c < count; ++c) s_chunk_cv(p + c * B3_CHUNK, B3_CHUNK, ctr0 + c, out[c]);
}

/* One tree level in place: cvs[k] = P(cvs[2k], cvs[2k+1]) for k < half. */
static void parents_batch(uint32_t (*cvs)[8], size_t half) {
  size_t k = 0;
  if (orc_simd_width() == 16)
    for (; k + 16 <= half; k += 16) {
      const uint32_t *pr[16];
      uint32_t *o[16];
      uint32_t tmp[16][8];
      for (int j = 0; j < 16; ++j) {
        pr[j] = cvs[2 * (k + j)];
        o[j] = tmp[j];
      }
      w_parents16(pr, o);
      for (int j = 0; j < 16; ++j) memcpy(cvs[k + j], tmp[j], 32);
    }
  for (; k + 8 <= half; k += 8) {
    const uint32_t *pr[8];
    uint32_t *o[8];
    uint32_t tmp[8][8] __attribute__((aligned(32)));
    for (int j = 0; j < 8; ++j) {
      pr[j] = cvs[2 * (k + j)];
      o[j] = tmp[j];
    }
    v_parents8(pr, o);
    for (int j = 0; j < 8; ++j) memcpy(cvs[k + j], tmp[j], 32);
  }
  for (; k < half; ++k) {
    uint32_t t[8];
    s_parent_cv(cvs[2 * k], cvs[2 * k + 1], 0, t);
    memcpy(cvs[k], t, 32);
  }
}

/* BLAKE3 (hash mode, first 8 digest bytes) of one message <= 128 chunks. */
static void simd_hash8(const uint8_t *msg, size_t len, uint8_t out8[8]) {
  const size_t nch = len <= B3_CHUNK ? 1 : (len + B3_CHUNK - 1) / B3_CHUNK;
  if (nch == 1 || nch > 128) {
    uint8_t d[32];
    orc_blake3(msg, len, d);
    memcpy(out8, d, 8);
    return;
  }
  uint32_t cvs[128][8] __attribute__((aligned(32)));
  /* full chunks 16 / 8 at a time (the last chunk is never ROOT here: nch >= 2) */
  const size_t full = len / B3_CHUNK;
  chunks_batch(msg, full, 0, cvs);
  for (size_t c = full; c < nch; ++c) {
    const size_t clen = len - c * B3_CHUNK < B3_CHUNK ? len - c * B3_CHUNK : B3_CHUNK;
    s_chunk_cv(msg + c * B3_CHUNK, clen, c, cvs[c]);
  }
  size_t cnt = nch;
  while (cnt > 2) {
    const size_t half = cnt / 2;
    parents_batch(cvs, half);
    if (cnt & 1) memcpy(cvs[half], cvs[cnt - 1], 32);
    cnt = half + (cnt & 1);
  }
  uint32_t root[8];
  s_parent_cv(cvs[0], cvs[1], B3_ROOT, root);
  for (int i = 0; i < 2; ++i) store32le(out8 + 4 * i, root[i]);
}

typedef struct {
  const uint8_t *arena;
  const uint64_t *off;
  const uint32_t *len;
  uint8_t *out8;
  uint64_t begin, end;
} simd_job;

static void *simd_worker(void *arg) {
  simd_job *j = (simd_job *)arg;
  for (uint64_t i = j->begin; i < j->end; i++)
    simd_hash8(j->arena + j->off[i], j->len[i], j->out8 + 8 * i);
  return NULL;
}

/* cas bytes of n messages, AVX2 8-way per message, `threads` threads. */
void orc_cas_batch_simd(const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                        uint64_t n, uint8_t *out8, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  simd_job jobs[256];
  for (int t = 0; t < threads; t++) {
    jobs[t] = (simd_job){arena, off, len, out8, n * (uint64_t)t / (uint64_t)threads,
                         n * (uint64_t)(t + 1) / (uint64_t)threads};
    pthread_create(&th[t], NULL, simd_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}

/* ------------------------------------------------------------------------- */
/* file_checksum's hashing with AVX2 (CPU BASELINE ONLY: bench.py's config-3 */
/* leg): the crate hashes a file's chunks 8/16 at a time (hash_many); here   */
/* aligned 1024-chunk subtrees go through v_chunks8 / v_parents8 and are     */
/* pushed on the incremental hasher's CV stack; the tail (>= 1 byte, so the  */
/* last chunk stays in the chunk state for ROOT) through h_update.           */
/* ------------------------------------------------------------------------- */

/* CV (non-root) of the aligned subtree of 1024 full chunks at chunk ctr0. */
static void simd_subtree1024(const uint8_t *p, uint64_t ctr0, uint32_t cv[8]) {
  uint32_t cvs[1024][8] __attribute__((aligned(32)));
  chunks_batch(p, 1024, ctr0, cvs);
  for (size_t cnt = 1024; cnt > 2; cnt /= 2) parents_batch(cvs, cnt / 2);
  s_parent_cv(cvs[0], cvs[1], 0, cv);
}

void orc_blake3_simd(const uint8_t *in, size_t len, uint8_t out32[32]) {
  orc_hasher h;
  h_init(&h);
  const size_t S = (size_t)1024 * B3_CHUNK;
  size_t off = 0;
  while (len - off > S) {
    uint32_t cv[8];
    simd_subtree1024(in + off, off / B3_CHUNK, cv);
    off += S;
    h_push_cv(&h, cv, (off / B3_CHUNK) >> 10); /* totals in units of subtrees */
  }
  h.chunk_counter = off / B3_CHUNK;
  h_update(&h, in + off, len - off);
  h_finalize(&h, out32);
}

typedef struct {
  const uint8_t *in;
  size_t len;
  int reps;
  uint8_t out32[32];
} ck_job;

static void *ck_worker(void *arg) {
  ck_job *j = (ck_job *)arg;
  for (int r = 0; r < j->reps; ++r) orc_blake3_simd(j->in, j->len, j->out32);
  return NULL;
}

/* `threads` threads, each hashing the buffer `reps` times (one file per
 * thread, as N validator jobs would); out32 = the digest of thread 0. */
void orc_checksum_simd_mt(const uint8_t *in, size_t len, int threads, int reps,
                          uint8_t out32[32]) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  ck_job jobs[256];
  for (int t = 0; t < threads; t++) {
    jobs[t].in = in;
    jobs[t].len = len;
    jobs[t].reps = reps;
    pthread_create(&th[t], NULL, ck_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  memcpy(out32, jobs[0].out32, 32);
}

/* ------------------------------------------------------------------------- */
/* generate_cas_id over real files with the reference's I/O pattern and the  */
/* AVX2 hasher (CPU BASELINE ONLY: bench.py's config-1 leg).                 */
/* ------------------------------------------------------------------------- */

/* The bytes orc_cas_id_path feeds its hasher, read the same way (cas.rs:23-62:
 * fs::read for <= 100 KiB, else open, read_exact header, 4 x {read_exact
 * sample, seek}, seek End(-8192), read_exact footer) into a growable buffer;
 * returns its length or -errno. */
static int64_t cas_read_message(const char *path, uint64_t size, uint8_t **buf,
                                size_t *cap) {
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -errno;
  size_t len = 8;
  int rc = 0;
  if (*cap < 8 + CAS_MINIMUM_FILE_SIZE + 4096) {
    free(*buf);
    *cap = 8 + CAS_MINIMUM_FILE_SIZE + 4096;
    *buf = (uint8_t *)malloc(*cap);
    if (!*buf) {
      close(fd);
      return -ENOMEM;
    }
  }
  for (int i = 0; i < 8; i++) (*buf)[i] = (uint8_t)(size >> (8 * i));
  if (size <= CAS_MINIMUM_FILE_SIZE) {
    for (;;) {
      if (len == *cap) {
        uint8_t *nb = (uint8_t *)realloc(*buf, *cap * 2);
        if (!nb) {
          rc = -ENOMEM;
          break;
        }
        *buf = nb;
        *cap *= 2;
      }
      ssize_t r = read(fd, *buf + len, *cap - len);
      if (r < 0) {
        if (errno == EINTR) continue;
        rc = -errno;
        break;
      }
      if (r == 0) break;
      len += (size_t)r;
    }
  } else {
    uint8_t *p = *buf;
    rc = read_exact_fd(fd, p + len, CAS_HEADER_OR_FOOTER);
    len += CAS_HEADER_OR_FOOTER;
    uint64_t current_pos = CAS_HEADER_OR_FOOTER;
    uint64_t seek_jump = (size - CAS_HEADER_OR_FOOTER * 2) / CAS_SAMPLE_COUNT;
    while (!rc) {
      rc = read_exact_fd(fd, p + len, CAS_SAMPLE_SIZE);
      if (rc) break;
      len += CAS_SAMPLE_SIZE;
      if (current_pos >= CAS_HEADER_OR_FOOTER + seek_jump * (CAS_SAMPLE_COUNT - 1)) break;
      off_t np = lseek(fd, (off_t)(current_pos + seek_jump), SEEK_SET);
      if (np < 0) rc = -errno;
      else current_pos = (uint64_t)np;
    }
    if (!rc) {
      if (lseek(fd, -(off_t)CAS_HEADER_OR_FOOTER, SEEK_END) < 0) rc = -errno;
      if (!rc) rc = read_exact_fd(fd, p + len, CAS_HEADER_OR_FOOTER);
      len += CAS_HEADER_OR_FOOTER;
    }
  }
  close(fd);
  return rc ? rc : (int64_t)len;
}

typedef struct {
  const char *const *paths;
  const uint64_t *sizes;
  uint64_t n;
  uint8_t *out8;
  int32_t *status;
  uint64_t *next; /* shared work counter (atomic) */
} path_job;

static void *path_worker(void *arg) {
  path_job *j = (path_job *)arg;
  uint8_t *buf = NULL;
  size_t cap = 0;
  for (;;) {
    uint64_t i0 = __atomic_fetch_add(j->next, 64, __ATOMIC_RELAXED);
    if (i0 >= j->n) break;
    uint64_t i1 = i0 + 64 < j->n ? i0 + 64 : j->n;
    for (uint64_t i = i0; i < i1; i++) {
      int64_t len = cas_read_message(j->paths[i], j->sizes[i], &buf, &cap);
      j->status[i] = len < 0 ? (int32_t)len : 0;
      if (len < 0) {
        memset(j->out8 + 8 * i, 0, 8);
      } else if ((uint64_t)len <= 128u * B3_CHUNK) {
        simd_hash8(buf, (size_t)len, j->out8 + 8 * i);
      } else {
        uint8_t d[32];
        orc_blake3(buf, (size_t)len, d);
        memcpy(j->out8 + 8 * i, d, 8);
      }
    }
  }
  free(buf);
  return NULL;
}

/* cas bytes of n files (paths, stat sizes), `threads` threads pulling 64
 * files at a time: the reference's reads per file + AVX2 hashing. */
void orc_cas_paths_simd(const char *const *paths, const uint64_t *sizes, uint64_t n,
                        uint8_t *out8, int32_t *status, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  uint64_t next = 0;
  pthread_t th[256];
  path_job job = {paths, sizes, n, out8, status, &next};
  for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, path_worker, &job);
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}
