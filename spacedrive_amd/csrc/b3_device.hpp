// BLAKE3 compression for gfx950 (CDNA4), one message block per lane.
//
// Replaces the arithmetic of the third-party `blake3` crate 1.4.1 that
// generate_cas_id (/root/reference/core/src/object/cas.rs:24-61) and
// file_checksum (/root/reference/core/src/object/validation/hash.rs:12-21) call.
//
// Pure 32-bit integer VALU work (add / xor / rotate): no MFMA.  The state and
// the 16 message words live in VGPRs; the 7 rounds are fully unrolled with the
// message schedule resolved at compile time, so each G is
//   v_add3_u32, v_xor_b32, v_alignbit_b32, v_add_u32, v_xor_b32, v_alignbit_b32,
//   v_add3_u32, v_xor_b32, v_alignbit_b32, v_add_u32, v_xor_b32, v_alignbit_b32
// = 12 VALU instructions; 7 x 8 x 12 + 8 output xors = 680 per compression.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sdgpu {

enum : uint32_t {
  B3_CHUNK_START = 1u,
  B3_CHUNK_END = 2u,
  B3_PARENT = 4u,
  B3_ROOT = 8u,
};

constexpr uint32_t B3_BLOCK_LEN = 64u;
constexpr uint32_t B3_CHUNK_LEN = 1024u;

constexpr uint32_t IV0 = 0x6A09E667u, IV1 = 0xBB67AE85u, IV2 = 0x3C6EF372u,
                   IV3 = 0xA54FF53Au, IV4 = 0x510E527Fu, IV5 = 0x9B05688Cu,
                   IV6 = 0x1F83D9ABu, IV7 = 0x5BE0CD19u;

__device__ __forceinline__ uint32_t rotr32(uint32_t x, uint32_t n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}

#define SDGPU_G(a, b, c, d, x, y)    \
  do {                               \
    a = a + b + (x);                 \
    d = rotr32(d ^ a, 16);           \
    c = c + d;                       \
    b = rotr32(b ^ c, 12);           \
    a = a + b + (y);                 \
    d = rotr32(d ^ a, 8);            \
    c = c + d;                       \
    b = rotr32(b ^ c, 7);            \
  } while (0)

// Round with message words picked by the round's schedule (compile time).
#define SDGPU_ROUND(M, s0, s1, s2, s3, s4, s5, s6, s7, s8, s9, s10, s11, s12, s13, s14, s15) \
  do {                                                                                     \
    SDGPU_G(v0, v4, v8, v12, M[s0], M[s1]);                                                \
    SDGPU_G(v1, v5, v9, v13, M[s2], M[s3]);                                                \
    SDGPU_G(v2, v6, v10, v14, M[s4], M[s5]);                                               \
    SDGPU_G(v3, v7, v11, v15, M[s6], M[s7]);                                               \
    SDGPU_G(v0, v5, v10, v15, M[s8], M[s9]);                                               \
    SDGPU_G(v1, v6, v11, v12, M[s10], M[s11]);                                             \
    SDGPU_G(v2, v7, v8, v13, M[s12], M[s13]);                                              \
    SDGPU_G(v3, v4, v9, v14, M[s14], M[s15]);                                              \
  } while (0)

// cv <- first 8 output words of compress(cv, m, counter, block_len, flags).
// For a ROOT compression this is the first 32 bytes of the digest.
__device__ __forceinline__ void b3_compress(uint32_t cv[8], const uint32_t m[16],
                                            uint32_t counter_lo, uint32_t counter_hi,
                                            uint32_t block_len, uint32_t flags) {
  uint32_t v0 = cv[0], v1 = cv[1], v2 = cv[2], v3 = cv[3];
  uint32_t v4 = cv[4], v5 = cv[5], v6 = cv[6], v7 = cv[7];
  uint32_t v8 = IV0, v9 = IV1, v10 = IV2, v11 = IV3;
  uint32_t v12 = counter_lo, v13 = counter_hi, v14 = block_len, v15 = flags;
  // schedules: sigma_{r+1}[i] = sigma_r[PERM[i]], PERM = [2,6,3,10,7,0,4,13,1,11,12,5,9,14,15,8]
  SDGPU_ROUND(m, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
  SDGPU_ROUND(m, 2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8);
  SDGPU_ROUND(m, 3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1);
  SDGPU_ROUND(m, 10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6);
  SDGPU_ROUND(m, 12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4);
  SDGPU_ROUND(m, 9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7);
  SDGPU_ROUND(m, 11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13);
  cv[0] = v0 ^ v8;
  cv[1] = v1 ^ v9;
  cv[2] = v2 ^ v10;
  cv[3] = v3 ^ v11;
  cv[4] = v4 ^ v12;
  cv[5] = v5 ^ v13;
  cv[6] = v6 ^ v14;
  cv[7] = v7 ^ v15;
}

__device__ __forceinline__ void b3_iv(uint32_t cv[8]) {
  cv[0] = IV0; cv[1] = IV1; cv[2] = IV2; cv[3] = IV3;
  cv[4] = IV4; cv[5] = IV5; cv[6] = IV6; cv[7] = IV7;
}

// Parent node: cv <- compress(IV, left || right, 0, 64, PARENT | extra).
__device__ __forceinline__ void b3_parent(uint32_t out[8], const uint32_t l[8],
                                          const uint32_t r[8], uint32_t extra_flags) {
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    m[i] = l[i];
    m[8 + i] = r[i];
  }
  b3_iv(out);
  b3_compress(out, m, 0u, 0u, B3_BLOCK_LEN, B3_PARENT | extra_flags);
}

// 64 bytes at a 16-byte aligned address -> 16 little-endian words.
__device__ __forceinline__ void b3_load_block(const uint8_t* __restrict__ p, uint32_t m[16]) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  const uint4 a = q[0], b = q[1], c = q[2], d = q[3];
  m[0] = a.x; m[1] = a.y; m[2] = a.z; m[3] = a.w;
  m[4] = b.x; m[5] = b.y; m[6] = b.z; m[7] = b.w;
  m[8] = c.x; m[9] = c.y; m[10] = c.z; m[11] = c.w;
  m[12] = d.x; m[13] = d.y; m[14] = d.z; m[15] = d.w;
}

// First `n` (0..64) bytes at a 4-byte aligned address, zero padded.  Never
// touches a byte at or beyond p + n (no over-read past a message end).
__device__ __forceinline__ void b3_load_block_partial(const uint8_t* __restrict__ p, uint32_t n,
                                                      uint32_t m[16]) {
  if (n == 64u) {
    if ((reinterpret_cast<uintptr_t>(p) & 15u) == 0) {
      b3_load_block(p, m);
      return;
    }
  }
#pragma unroll
  for (uint32_t w = 0; w < 16; ++w) {
    const uint32_t lo = 4u * w;
    uint32_t v = 0;
    if (lo + 4u <= n) {
      v = *reinterpret_cast<const uint32_t*>(p + lo);
    } else if (lo < n) {
      for (uint32_t k = lo; k < n; ++k) v |= static_cast<uint32_t>(p[k]) << (8u * (k - lo));
    }
    m[w] = v;
  }
}

// Chaining value (or, with ROOT in `root_flag`, the digest words) of one chunk
// of `clen` (0..1024) bytes at 16-byte aligned `p`, chunk counter `ctr`.
__device__ __forceinline__ void b3_chunk(const uint8_t* __restrict__ p, uint32_t clen,
                                         uint64_t ctr, uint32_t root_flag, uint32_t cv[8]) {
  b3_iv(cv);
  const uint32_t nb = clen == 0 ? 1u : (clen + 63u) >> 6;
  const uint32_t lo = static_cast<uint32_t>(ctr), hi = static_cast<uint32_t>(ctr >> 32);
  uint32_t m[16];
  uint32_t b = 0;
  for (; b + 1 < nb; ++b) {
    b3_load_block(p + 64u * b, m);
    b3_compress(cv, m, lo, hi, B3_BLOCK_LEN, b == 0 ? B3_CHUNK_START : 0u);
  }
  const uint32_t last = clen - 64u * b;
  b3_load_block_partial(p + 64u * b, last, m);
  b3_compress(cv, m, root_flag ? 0u : lo, root_flag ? 0u : hi, last,
              B3_CHUNK_END | (nb == 1 ? B3_CHUNK_START : 0u) | root_flag);
}

// A FULL 1024-byte chunk (16 blocks) at 16-byte aligned `p`, non-root.  Loads
// one 128-byte line per lane (two blocks, 8 x dwordx4) per step: measured on
// MI355X with lanes 4 KiB apart in HBM, 128-B steps sustain ~54.5 G
// compressions/s against ~50.5 G for 64-B steps (scripts/exp_units.hip; the
// register-only roof is ~56.4 G).
__device__ __forceinline__ void b3_chunk_full(const uint8_t* __restrict__ p, uint64_t ctr,
                                              uint32_t cv[8]) {
  b3_iv(cv);
  const uint32_t lo = static_cast<uint32_t>(ctr), hi = static_cast<uint32_t>(ctr >> 32);
  for (uint32_t b = 0; b < 16; b += 2) {
    uint32_t m0[16], m1[16];
    const uint4* q = reinterpret_cast<const uint4*>(p + 64u * b);
    uint4 x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = q[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      m0[4 * k] = x[k].x; m0[4 * k + 1] = x[k].y; m0[4 * k + 2] = x[k].z; m0[4 * k + 3] = x[k].w;
      m1[4 * k] = x[k + 4].x; m1[4 * k + 1] = x[k + 4].y; m1[4 * k + 2] = x[k + 4].z;
      m1[4 * k + 3] = x[k + 4].w;
    }
    b3_compress(cv, m0, lo, hi, B3_BLOCK_LEN, b == 0 ? B3_CHUNK_START : 0u);
    b3_compress(cv, m1, lo, hi, B3_BLOCK_LEN, b == 14 ? B3_CHUNK_END : 0u);
  }
}

// Same as b3_chunk, software-pipelined: the next block's 64 bytes are loaded
// before the current block is compressed, so one wave keeps a load in flight
// under every compression.
__device__ __forceinline__ void b3_chunk_pipelined(const uint8_t* __restrict__ p, uint32_t clen,
                                                   uint64_t ctr, uint32_t root_flag,
                                                   uint32_t cv[8]) {
  b3_iv(cv);
  const uint32_t nb = clen == 0 ? 1u : (clen + 63u) >> 6;
  const uint32_t last = clen - 64u * (nb - 1);
  const uint32_t lo = static_cast<uint32_t>(ctr), hi = static_cast<uint32_t>(ctr >> 32);
  uint32_t m[16], mn[16];
  if (nb > 1) b3_load_block(p, m);
  else b3_load_block_partial(p, last, m);
  for (uint32_t b = 0; b + 1 < nb; ++b) {
    if (b + 2 < nb) b3_load_block(p + 64u * (b + 1), mn);
    else b3_load_block_partial(p + 64u * (b + 1), last, mn);
    b3_compress(cv, m, lo, hi, B3_BLOCK_LEN, b == 0 ? B3_CHUNK_START : 0u);
#pragma unroll
    for (int w = 0; w < 16; ++w) m[w] = mn[w];
  }
  b3_compress(cv, m, root_flag ? 0u : lo, root_flag ? 0u : hi, last,
              B3_CHUNK_END | (nb == 1 ? B3_CHUNK_START : 0u) | root_flag);
}

}  // namespace sdgpu
