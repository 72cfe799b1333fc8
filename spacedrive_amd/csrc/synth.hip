// Synthetic corpora generated directly in HBM (bench / tests only; never on the
// identification path).  The content function is the one the CPU oracle uses
// (oracle/sd_oracle.c: synth_byte / orc_synth_cas_message), so device and CPU
// agree byte for byte:
//   byte(seed, o) = byte (o & 7) of mix64(seed + (o >> 3) * 0x9E3779B97F4A7C15)
// A cas message for a file (size, seed) is laid out as generate_cas_id reads it
// (/root/reference/core/src/object/cas.rs:24-58): size_le || whole file (size <=
// 100 KiB) or size_le || header || 4 samples at 8192 + k*((size-16384)/4) || footer.
#include "b3_device.hpp"
#include "internal.hpp"

namespace sdgpu {

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t synth_byte(uint64_t seed, uint64_t o) {
  const uint64_t w = mix64(seed + (o >> 3) * 0x9E3779B97F4A7C15ull);
  return static_cast<uint32_t>(w >> (8 * (o & 7))) & 0xFFu;
}

// 4 message bytes starting at message position p (p % 4 == 0, p >= 8); a
// 4-byte group never straddles a window boundary (all boundaries are at
// multiples of 8 in M).
__device__ __forceinline__ uint32_t msg_word(uint64_t size, uint64_t seed, uint32_t p) {
  const uint32_t q = p - 8u;
  uint64_t fo;
  if (size <= 102400u) {
    fo = q;
  } else if (q < 8192u) {
    fo = q;
  } else if (q < 8192u + 4u * 10240u) {
    const uint64_t jump = (size - 16384u) / 4u;
    const uint32_t k = (q - 8192u) / 10240u, r = (q - 8192u) % 10240u;
    fo = 8192u + k * jump + r;
  } else {
    fo = size - 8192u + (q - 8192u - 40960u);
  }
  uint32_t v = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) v |= synth_byte(seed, fo + b) << (8 * b);
  return v;
}

// One block per file: fills arena[off[i] .. off[i] + msg_len) with M_i.
__global__ __launch_bounds__(kThreads) void k_synth_cas(const uint64_t* __restrict__ sizes,
                                                        const uint64_t* __restrict__ seeds,
                                                        const uint64_t* __restrict__ off,
                                                        uint32_t n, uint8_t* __restrict__ arena) {
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint64_t size = sizes[i], seed = seeds[i];
    const uint32_t len = size <= 102400u ? static_cast<uint32_t>(8 + size) : 57352u;
    uint8_t* m = arena + off[i];
    for (uint32_t p = threadIdx.x * 4; p < len; p += kThreads * 4) {
      uint32_t v;
      if (p < 8) {
        v = static_cast<uint32_t>(size >> (8 * p));  // p is 0 or 4
      } else {
        v = msg_word(size, seed, p);
      }
      if (p + 4 <= len) {
        *reinterpret_cast<uint32_t*>(m + p) = v;
      } else {
        for (uint32_t b = 0; p + b < len; ++b) m[p + b] = static_cast<uint8_t>(v >> (8 * b));
      }
    }
  }
}

// out[0..len) = bytes [offset, offset+len) of the synthetic file `seed`
// (offset % 8 == 0; out 16-B aligned).  Two words per thread per step.
__global__ __launch_bounds__(kThreads) void k_synth_file(uint64_t seed, uint64_t offset,
                                                         uint64_t len, uint8_t* __restrict__ out) {
  const uint64_t nwords = len / 8;
  const uint64_t w0 = offset / 8;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x; i * 2 < nwords;
       i += stride) {
    const uint64_t a = mix64(seed + (w0 + 2 * i) * 0x9E3779B97F4A7C15ull);
    if (2 * i + 1 < nwords) {
      const uint64_t b = mix64(seed + (w0 + 2 * i + 1) * 0x9E3779B97F4A7C15ull);
      reinterpret_cast<ulonglong2*>(out)[i] = make_ulonglong2(a, b);
    } else {
      reinterpret_cast<uint64_t*>(out)[2 * i] = a;
    }
  }
  // tail bytes
  if (blockIdx.x == 0 && threadIdx.x < (len & 7)) {
    const uint64_t o = nwords * 8 + threadIdx.x;
    out[o] = static_cast<uint8_t>(synth_byte(seed, offset + o));
  }
}

// Bijective pseudo-random permutation of [0, T) (4-round Feistel on 2h bits
// with cycle-walking); identical to orc_perm in oracle/sd_oracle.c.
__device__ __forceinline__ uint64_t perm_index(uint64_t x, uint64_t T, uint64_t seed) {
  uint32_t bits = 2;
  while ((1ull << bits) < T) bits += 2;
  const uint32_t h = bits / 2;
  const uint64_t mask = (1ull << h) - 1;
  do {
    uint64_t L = x >> h, R = x & mask;
    for (uint32_t r = 0; r < 4; ++r) {
      const uint64_t F = mix64(R ^ (seed + 0x632BE59BD9B4E019ull * (r + 1))) & mask;
      const uint64_t nl = R;
      R = L ^ F;
      L = nl;
    }
    x = (L << h) | R;
  } while (x >= T);
  return x;
}

// Row with global rank g: u = perm(g); u < distinct -> key of distinct item u;
// else a duplicate of distinct item (mix(u) % distinct).  1 row in 1000 has no key.
__global__ __launch_bounds__(kThreads) void k_synth_dedup(uint64_t seed, uint64_t total,
                                                          uint64_t distinct, uint64_t first,
                                                          uint64_t n, uint64_t* __restrict__ key,
                                                          uint8_t* __restrict__ has_key,
                                                          uint32_t* __restrict__ rank) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x; i < n;
       i += stride) {
    const uint64_t g = first + i;
    const uint64_t u = perm_index(g, total, seed);
    const uint64_t item = u < distinct ? u : mix64(u ^ seed ^ 0xD6E8FEB86659FD93ull) % distinct;
    key[i] = mix64(seed * 0x9E3779B97F4A7C15ull + item + 1);
    has_key[i] = (mix64(g ^ (seed << 1) ^ 0xA0761D6478BD642Full) % 1000) != 0;
    rank[i] = static_cast<uint32_t>(g);
  }
}

// 8 independent G-like chains per lane: v_add3_u32 / v_xor_b32 /
// v_alignbit_b32 in BLAKE3's mix, to measure the integer VALU issue rate.
__global__ __launch_bounds__(256) void k_valu_probe(uint32_t* __restrict__ sink, uint32_t iters) {
  uint32_t a[8], b[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a[k] = threadIdx.x * 0x9E3779B9u + k;
    b[k] = blockIdx.x * 0x85EBCA6Bu + 3 * k;
  }
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      a[k] = a[k] + b[k] + it;                                  // v_add3_u32
      b[k] = __builtin_amdgcn_alignbit(b[k] ^ a[k], b[k] ^ a[k], 16);  // xor + alignbit
      a[k] = a[k] + b[k] + 7u;
      b[k] = __builtin_amdgcn_alignbit(b[k] ^ a[k], b[k] ^ a[k], 7);
    }
  }
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) x ^= a[k] ^ b[k];
  if (x == 0x12345678u) sink[blockIdx.x] = x;
}

// One instruction class only, forced by inline asm (8 independent chains per
// lane, 6 instructions per chain per iteration): prices VOP2 vs VOP3 issue.
template <int kKind>
__global__ __launch_bounds__(256) void k_valu_class(uint32_t* __restrict__ sink, uint32_t iters) {
  uint32_t a[8];
  const uint32_t b = blockIdx.x * 0x85EBCA6Bu, c = threadIdx.x * 0x9E3779B9u;
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = c + k;
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 6; ++r) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (kKind == 1) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a[k]) : "v"(b));
        if (kKind == 2) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(b), "v"(c));
        if (kKind == 3) asm volatile("v_alignbit_b32 %0, %0, %0, 16" : "+v"(a[k]));
        if (kKind == 4) asm volatile("v_add_u32 %0, %1, %0" : "+v"(a[k]) : "v"(b));
      }
    }
  }
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) x ^= a[k];
  if (x == 0x12345678u) sink[blockIdx.x] = x;
}

}  // namespace

// BLAKE3 compressions with everything in registers (no memory): the
// attainable roof of the exact instruction stream K1/K2 issue (680 VALU per
// compression, BLAKE3's add3/xor/alignbit mix).
__global__ __launch_bounds__(256) void k_compress_probe(uint32_t* __restrict__ sink,
                                                        uint32_t iters) {
  uint32_t cv[8], m[16];
  b3_iv(cv);
#pragma unroll
  for (int i = 0; i < 16; ++i) m[i] = threadIdx.x * 0x9E3779B9u + blockIdx.x * 7u + i;
  for (uint32_t it = 0; it < iters; ++it) {
    b3_compress(cv, m, it, 0u, 64u, 0u);
    m[it & 15] ^= cv[it & 7];
  }
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) x ^= cv[i];
  if (x == 0x12345u) sink[blockIdx.x] = x;
}

// Config-5 run: the files of step `step` are the pool's files with new content
// for the rows marked vary[i] -- a new content gives a new cas key, emulated as
// key' = mix64(key ^ step * phi) (a bijection, so distinct files stay distinct
// and duplicates stay duplicates); unmarked rows keep their key (files seen in
// every step: they link to the Objects of the first).
__global__ __launch_bounds__(kThreads) void k_vary_keys(uint64_t* __restrict__ key,
                                                        const uint8_t* __restrict__ vary,
                                                        uint64_t n, uint64_t step) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (i < n && vary[i]) key[i] = mix64(key[i] ^ (step * 0x9E3779B97F4A7C15ull));
}

hipError_t vary_keys_launch(uint64_t* key, const uint8_t* vary, uint64_t n, uint64_t step,
                            hipStream_t s) {
  if (n && step)
    k_vary_keys<<<static_cast<uint32_t>((n + kThreads - 1) / kThreads), kThreads, 0, s>>>(
        key, vary, n, step);
  return hipGetLastError();
}

hipError_t valu_probe_launch(int kind, uint32_t* sink, uint32_t iters, uint32_t blocks,
                             hipStream_t s) {
  switch (kind) {
    case 5: k_compress_probe<<<blocks, 256, 0, s>>>(sink, iters); break;
    case 1: k_valu_class<1><<<blocks, 256, 0, s>>>(sink, iters); break;
    case 2: k_valu_class<2><<<blocks, 256, 0, s>>>(sink, iters); break;
    case 3: k_valu_class<3><<<blocks, 256, 0, s>>>(sink, iters); break;
    case 4: k_valu_class<4><<<blocks, 256, 0, s>>>(sink, iters); break;
    default: k_valu_probe<<<blocks, 256, 0, s>>>(sink, iters); break;
  }
  return hipGetLastError();
}

hipError_t synth_dedup_rows_launch(uint64_t seed, uint64_t total_rows, uint64_t distinct,
                                   uint64_t first_rank, uint64_t n, uint64_t* key,
                                   uint8_t* has_key, uint32_t* rank, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t want = (n + kThreads - 1) / kThreads;
  const uint32_t grid = static_cast<uint32_t>(want < 16384 ? want : 16384);
  k_synth_dedup<<<grid, kThreads, 0, s>>>(seed, total_rows, distinct, first_rank, n, key, has_key,
                                          rank);
  return hipGetLastError();
}

hipError_t synth_cas_arena_launch(const uint64_t* sizes, const uint64_t* seeds,
                                  const uint64_t* off, uint32_t n, uint8_t* arena, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint32_t grid = n < 65536 ? n : 65536;
  k_synth_cas<<<grid, kThreads, 0, s>>>(sizes, seeds, off, n, arena);
  return hipGetLastError();
}

hipError_t synth_file_launch(uint64_t seed, uint64_t offset, uint64_t len, uint8_t* out,
                             hipStream_t s) {
  if (len == 0) return hipSuccess;
  if (offset % 8 != 0) return hipErrorInvalidValue;
  const uint64_t pairs = (len / 8 + 1) / 2;
  uint64_t want = (pairs + kThreads - 1) / kThreads;
  const uint32_t grid = static_cast<uint32_t>(want < 16384 ? (want ? want : 1) : 16384);
  k_synth_file<<<grid, kThreads, 0, s>>>(seed, offset, len, out);
  return hipGetLastError();
}

}  // namespace sdgpu
