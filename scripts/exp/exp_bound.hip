// Experiment (round 3): what bounds each kernel of the
// 12.5 M-row one-level grouping?  Each variant removes one ingredient of a
// product kernel and is timed alone (HIP events, median of reps):
//   hist:    H0 product | H1 cheap bijective hash (x ^ x >> 32) * odd |
//            H2 loads only (no hash, no LDS atomics) | H3 raw key bits as digit
//   scatter: S0 product k_part_scatter_ws | S1 no record stores | S2 no rep
//            init | S3 cheap hash | S4 raw key bits as digit
//   group:   G0 product k_bucket_group12_pk | G1 no rep writes | G2 loads only
// Only H0/S0/G0 produce the product's result (checked); the others are
// timing probes.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_bound.hip -o build/exp_bound
#include "../../spacedrive_amd/csrc/dedup.hip"

#include <stdio.h>

#include <algorithm>
#include <functional>
#include <vector>

using namespace sdgpu;

namespace {

constexpr uint32_t kNb = 1u << kStageBits;

__global__ void k_rows(uint64_t* key, uint8_t* has, uint64_t n, uint64_t distinct) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint64_t j = (i * 0x9E3779B1ull) % n;
    key[i] = row_hash((j % distinct) * 0x2545F4914F6CDD1Dull + 7);
    has[i] = (row_hash(i ^ 0x55ull) % 1000) != 0;
  }
}

// 0: splitmix64 (product), 1: one 64-bit multiply of x ^ x >> 32, 2: none
template <int kH>
__device__ __forceinline__ uint64_t hmode(uint64_t k) {
  if constexpr (kH == 0) return row_hash(k);
  else if constexpr (kH == 1) return (k ^ (k >> 32)) * 0x9E3779B97F4A7C15ull;
  else return k;
}

// hist: the product's pair-load path with a hash mode; kH = 3: loads only
template <int kH>
__global__ __launch_bounds__(kPartThreads) void k_hist_var(const uint64_t* __restrict__ key,
                                                           const uint8_t* __restrict__ valid,
                                                           uint64_t n, uint32_t* __restrict__ hist,
                                                           uint32_t* __restrict__ sink) {
  __shared__ uint32_t cnt[kNb];
  for (uint32_t b = threadIdx.x; b < kNb; b += kPartThreads) cnt[b] = 0;
  __syncthreads();
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  const uint64_t p0 = (t0 + 1) / 2, p1 = t1 / 2;
  const uint4* __restrict__ k4 = reinterpret_cast<const uint4*>(key);
  const uint16_t* __restrict__ v2 = reinterpret_cast<const uint16_t*>(valid);
  constexpr int kP = kUnroll / 2;
  uint32_t acc = 0;
  for (uint64_t q0 = p0 + threadIdx.x; q0 < p1; q0 += kP * kPartThreads) {
    uint4 kk[kP];
    uint32_t vv[kP];
#pragma unroll
    for (int u = 0; u < kP; ++u) {
      const uint64_t q = q0 + static_cast<uint64_t>(u) * kPartThreads;
      kk[u] = k4[q < p1 ? q : q0];
      vv[u] = v2[q < p1 ? q : q0];
    }
#pragma unroll
    for (int u = 0; u < kP; ++u) {
      if (q0 + static_cast<uint64_t>(u) * kPartThreads >= p1) continue;
      if constexpr (kH == 3) {
        acc += kk[u].x ^ kk[u].y ^ kk[u].z ^ kk[u].w ^ vv[u];
      } else {
        const uint64_t a = (static_cast<uint64_t>(kk[u].y) << 32) | kk[u].x;
        const uint64_t b = (static_cast<uint64_t>(kk[u].w) << 32) | kk[u].z;
        if (vv[u] & 0xFFu) atomicAdd(&cnt[digit_of(hmode<kH>(a), kShardBits, kStageBits)], 1u);
        if (vv[u] >> 8) atomicAdd(&cnt[digit_of(hmode<kH>(b), kShardBits, kStageBits)], 1u);
      }
    }
  }
  if constexpr (kH == 3) {
    if (acc == 0x12345678u) sink[0] = acc;
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < kNb; b += kPartThreads)
    hist[static_cast<uint64_t>(part_block()) * kNb + b] = cnt[b];
}

// k_part_scatter_ws with ingredients removable
template <bool kStore, bool kRep, int kH>
__global__ __launch_bounds__(kPartThreads) void k_ws_var(RowsIn in, uint64_t n, uint32_t skip,
                                                         const uint32_t* __restrict__ offs,
                                                         const uint32_t* __restrict__ ftot,
                                                         uint3* __restrict__ out,
                                                         uint32_t* __restrict__ rep,
                                                         uint32_t* __restrict__ fbase) {
  constexpr uint32_t nbins = kNb;
  constexpr uint32_t kRound = kWsProd * kWsRows;
  __shared__ uint3 stage[nbins][2];
  __shared__ uint32_t fill[nbins], cur[nbins];
  __shared__ uint3 ovf[kRound];
  __shared__ uint32_t ovf_n;
  constexpr uint32_t kPerT = nbins / kPartThreads;
  const uint32_t t = threadIdx.x, lane = __lane_id();
  uint32_t v[kPerT], sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPerT; ++k) {
    v[k] = ftot[t * kPerT + k];
    sum += v[k];
  }
  uint32_t inc = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d);
    if (lane >= static_cast<uint32_t>(d)) inc += o;
  }
  if (lane == 63) fill[t >> 6] = inc;
  __syncthreads();
  uint32_t base = inc - sum, total = 0;
  for (uint32_t w = 0; w < kPartThreads / 64; ++w) {
    if (w < (t >> 6)) base += fill[w];
    total += fill[w];
  }
  __syncthreads();
  const uint32_t j = part_block();
#pragma unroll
  for (uint32_t k = 0; k < kPerT; ++k) {
    const uint32_t b = t * kPerT + k;
    cur[b] = base + offs[static_cast<uint64_t>(j) * nbins + b];
    fill[b] = 0;
    if (j == 0) fbase[b] = base;
    base += v[k];
  }
  if (j == 0 && t == 0) fbase[nbins] = total;
  if (t == 0) ovf_n = 0;
  __syncthreads();
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  const uint32_t rounds = t1 > t0 ? static_cast<uint32_t>((t1 - t0 + kRound - 1) / kRound) : 0u;
  if (t < kWsProd) {
    RowBatch<kWsRows> qa, qb;
    in.template load_many<kWsRows>(t0 + t, kWsProd, t1, t0, qa);
    in.template load_many<kWsRows>(t0 + kRound + t, kWsProd, t1, t0, qb);
    auto stage_round = [&](const RowBatch<kWsRows>& q) {
#pragma unroll
      for (int u = 0; u < kWsRows; ++u) {
        if (!in.valid_of(q, u)) continue;
        const uint64_t h = hmode<kH>(in.key_of(q, u));
        const uint32_t b = digit_of(h, skip, kStageBits);
        const uint3 rq = make_uint3(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32),
                                    in.row_of(q, u));
        const uint32_t sl = atomicAdd(&fill[b], 1u);
        if (sl < 2)
          stage[b][sl] = rq;
        else
          ovf[atomicAdd(&ovf_n, 1u)] = rq;
      }
    };
    for (uint32_t r = 0; r < rounds; r += 2) {
      stage_round(qa);
      lds_barrier();
      in.template load_many<kWsRows>(t0 + (r + 2) * static_cast<uint64_t>(kRound) + t, kWsProd, t1,
                                     t0, qa);
      lds_barrier();
      lds_barrier();
      if (r + 1 >= rounds) break;
      stage_round(qb);
      lds_barrier();
      in.template load_many<kWsRows>(t0 + (r + 3) * static_cast<uint64_t>(kRound) + t, kWsProd, t1,
                                     t0, qb);
      lds_barrier();
      lds_barrier();
    }
  } else {
    const uint32_t c = t - kWsProd;
    uint32_t junk = 0;
    for (uint32_t r = 0; r < rounds; ++r) {
      lds_barrier();
      if constexpr (kRep) {
        const uint64_t r0 = t0 + static_cast<uint64_t>(r) * kRound;
#pragma unroll
        for (uint32_t u = 0; u < kRound / kWsProd; ++u) {
          const uint64_t i = r0 + c + u * kWsProd;
          if (i < t1) rep[i] = in.rank_base + static_cast<uint32_t>(i);
        }
      }
#pragma unroll
      for (uint32_t k = 0; k < nbins / kWsProd; ++k) {
        const uint32_t b = c + k * kWsProd;
        if (fill[b] >= 2) {
          const uint32_t p = cur[b];
          const uint3 x0 = stage[b][0], x1 = stage[b][1];
          if constexpr (kStore) {
            out[p] = x0;
            out[p + 1] = x1;
          } else {
            junk += x0.x ^ x1.y;
          }
          cur[b] = p + 2;
          fill[b] = 0;
        }
      }
      const uint32_t no = ovf_n;
      lds_barrier();
      for (uint32_t o = c; o < no; o += kWsProd) {
        const uint3 rq = ovf[o];
        const uint32_t p = atomicAdd(&cur[digit_of((static_cast<uint64_t>(rq.y) << 32) | rq.x, skip,
                                                   kStageBits)], 1u);
        if constexpr (kStore) out[p] = rq;
        else junk += rq.z ^ p;
      }
      if (c == 0) ovf_n = 0;
      lds_barrier();
    }
    if (!kStore && junk == 0x12345678u) out[0] = make_uint3(junk, 0, 0);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads)
    for (uint32_t k = 0; k < fill[b]; ++k) out[cur[b] + k] = stage[b][k];
}

// Producer row loads issued by inline asm and waited for with a COUNTED
// vmcnt: the compiler's own waits (vmcnt(0) at the ping-pong loop head, i.e.
// the prefetch of round r + 2 drained before round r is staged) are gone.
// Producers issue no other vector-memory instruction in the loop, so each
// round's 8 loads (4 keys, 4 valid bytes) are the only entries of vmcnt: the
// batch of round r is complete at vmcnt(8) (round r + 1's 8 in flight).
struct AsmBatch {
  uint64_t k[kWsRows];
  uint32_t b[kWsRows];
};
__device__ __forceinline__ void asm_load_batch(const uint64_t* key, const uint8_t* valid,
                                               uint64_t i0, uint64_t end, uint64_t safe,
                                               AsmBatch& q) {
#pragma unroll
  for (int u = 0; u < kWsRows; ++u) {
    const uint64_t i = i0 + static_cast<uint64_t>(u) * kWsProd;
    const uint64_t r = i < end ? i : safe;
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(q.k[u]) : "v"(key + r) : "memory");
  }
#pragma unroll
  for (int u = 0; u < kWsRows; ++u) {
    const uint64_t i = i0 + static_cast<uint64_t>(u) * kWsProd;
    const uint64_t r = i < end ? i : safe;
    asm volatile("global_load_ubyte %0, %1, off" : "=v"(q.b[u]) : "v"(valid + r) : "memory");
  }
}
template <int kLeft>
__device__ __forceinline__ void asm_wait_batch(AsmBatch& q) {
  asm volatile("s_waitcnt vmcnt(%c8)"
               : "+v"(q.k[0]), "+v"(q.k[1]), "+v"(q.k[2]), "+v"(q.k[3]), "+v"(q.b[0]),
                 "+v"(q.b[1]), "+v"(q.b[2]), "+v"(q.b[3])
               : "i"(kLeft)
               : "memory");
}

template <bool kStore>
__global__ __launch_bounds__(kPartThreads) void k_ws_asm(RowsIn in, uint64_t n, uint32_t skip,
                                                         const uint32_t* __restrict__ offs,
                                                         const uint32_t* __restrict__ ftot,
                                                         uint3* __restrict__ out,
                                                         uint32_t* __restrict__ rep,
                                                         uint32_t* __restrict__ fbase) {
  constexpr uint32_t nbins = kNb;
  constexpr uint32_t kRound = kWsProd * kWsRows;
  __shared__ uint3 stage[nbins][2];
  __shared__ uint32_t fill[nbins], cur[nbins];
  __shared__ uint3 ovf[kRound];
  __shared__ uint32_t ovf_n;
  constexpr uint32_t kPerT = nbins / kPartThreads;
  const uint32_t t = threadIdx.x, lane = __lane_id();
  uint32_t v[kPerT], sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPerT; ++k) {
    v[k] = ftot[t * kPerT + k];
    sum += v[k];
  }
  uint32_t inc = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d);
    if (lane >= static_cast<uint32_t>(d)) inc += o;
  }
  if (lane == 63) fill[t >> 6] = inc;
  __syncthreads();
  uint32_t base = inc - sum, total = 0;
  for (uint32_t w = 0; w < kPartThreads / 64; ++w) {
    if (w < (t >> 6)) base += fill[w];
    total += fill[w];
  }
  __syncthreads();
  const uint32_t j = part_block();
#pragma unroll
  for (uint32_t k = 0; k < kPerT; ++k) {
    const uint32_t b = t * kPerT + k;
    cur[b] = base + offs[static_cast<uint64_t>(j) * nbins + b];
    fill[b] = 0;
    if (j == 0) fbase[b] = base;
    base += v[k];
  }
  if (j == 0 && t == 0) fbase[nbins] = total;
  if (t == 0) ovf_n = 0;
  __syncthreads();
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  const uint32_t rounds = t1 > t0 ? static_cast<uint32_t>((t1 - t0 + kRound - 1) / kRound) : 0u;
  if (t < kWsProd) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing of the prologue in flight
    AsmBatch qa, qb;
    asm_load_batch(in.key, in.valid, t0 + t, t1, t0, qa);
    asm_load_batch(in.key, in.valid, t0 + kRound + t, t1, t0, qb);
    auto stage_round = [&](const AsmBatch& q, uint64_t i0) {
#pragma unroll
      for (int u = 0; u < kWsRows; ++u) {
        const uint64_t i = i0 + t + static_cast<uint64_t>(u) * kWsProd;
        if (i >= t1 || (q.b[u] & 0xFFu) == 0) continue;
        const uint64_t h = row_hash(q.k[u]);
        const uint32_t b = digit_of(h, skip, kStageBits);
        const uint3 rq = make_uint3(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32),
                                    static_cast<uint32_t>(i));
        const uint32_t sl = atomicAdd(&fill[b], 1u);
        if (sl < 2)
          stage[b][sl] = rq;
        else
          ovf[atomicAdd(&ovf_n, 1u)] = rq;
      }
    };
    for (uint32_t r = 0; r < rounds; r += 2) {
      asm_wait_batch<8>(qa);
      stage_round(qa, t0 + static_cast<uint64_t>(r) * kRound);
      lds_barrier();
      asm_load_batch(in.key, in.valid, t0 + (r + 2) * static_cast<uint64_t>(kRound) + t, t1, t0, qa);
      lds_barrier();
      lds_barrier();
      if (r + 1 >= rounds) break;
      asm_wait_batch<8>(qb);
      stage_round(qb, t0 + static_cast<uint64_t>(r + 1) * kRound);
      lds_barrier();
      asm_load_batch(in.key, in.valid, t0 + (r + 3) * static_cast<uint64_t>(kRound) + t, t1, t0, qb);
      lds_barrier();
      lds_barrier();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the last prefetches
  } else {
    const uint32_t c = t - kWsProd;
    uint32_t junk = 0;
    for (uint32_t r = 0; r < rounds; ++r) {
      lds_barrier();
      {
        const uint64_t r0 = t0 + static_cast<uint64_t>(r) * kRound;
#pragma unroll
        for (uint32_t u = 0; u < kRound / kWsProd; ++u) {
          const uint64_t i = r0 + c + u * kWsProd;
          if (i < t1) rep[i] = in.rank_base + static_cast<uint32_t>(i);
        }
      }
#pragma unroll
      for (uint32_t k = 0; k < nbins / kWsProd; ++k) {
        const uint32_t b = c + k * kWsProd;
        if (fill[b] >= 2) {
          const uint32_t p = cur[b];
          const uint3 x0 = stage[b][0], x1 = stage[b][1];
          if constexpr (kStore) {
            out[p] = x0;
            out[p + 1] = x1;
          } else {
            junk += x0.x ^ x1.y;
          }
          cur[b] = p + 2;
          fill[b] = 0;
        }
      }
      const uint32_t no = ovf_n;
      lds_barrier();
      for (uint32_t o = c; o < no; o += kWsProd) {
        const uint3 rq = ovf[o];
        const uint32_t p = atomicAdd(&cur[digit_of((static_cast<uint64_t>(rq.y) << 32) | rq.x, skip,
                                                   kStageBits)], 1u);
        if constexpr (kStore) out[p] = rq;
        else junk += rq.z ^ p;
      }
      if (c == 0) ovf_n = 0;
      lds_barrier();
    }
    if (!kStore && junk == 0x12345678u) out[0] = make_uint3(junk, 0, 0);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads)
    for (uint32_t k = 0; k < fill[b]; ++k) out[cur[b] + k] = stage[b][k];
}

// Batched LDS round trips: the producer issues its 4 rows' fill atomics back
// to back (one LDS latency, not four) and reserves its overflow entries with
// one atomic; the consumer reads its 8 buckets' fills at once, then the
// flushed buckets' cursors and slots at once, then stores.
template <bool kStore>
__global__ __launch_bounds__(kPartThreads) void k_ws_batched(RowsIn in, uint64_t n, uint32_t skip,
                                                             const uint32_t* __restrict__ offs,
                                                             const uint32_t* __restrict__ ftot,
                                                             uint3* __restrict__ out,
                                                             uint32_t* __restrict__ rep,
                                                             uint32_t* __restrict__ fbase) {
  constexpr uint32_t nbins = kNb;
  constexpr uint32_t kRound = kWsProd * kWsRows;
  constexpr uint32_t kPerC = nbins / kWsProd;  // buckets per consumer thread
  __shared__ uint3 stage[nbins][2];
  __shared__ uint32_t fill[nbins], cur[nbins];
  __shared__ uint3 ovf[kRound];
  __shared__ uint32_t ovf_n;
  constexpr uint32_t kPerT = nbins / kPartThreads;
  const uint32_t t = threadIdx.x, lane = __lane_id();
  uint32_t v[kPerT], sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPerT; ++k) {
    v[k] = ftot[t * kPerT + k];
    sum += v[k];
  }
  uint32_t inc = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d);
    if (lane >= static_cast<uint32_t>(d)) inc += o;
  }
  if (lane == 63) fill[t >> 6] = inc;
  __syncthreads();
  uint32_t base = inc - sum, total = 0;
  for (uint32_t w = 0; w < kPartThreads / 64; ++w) {
    if (w < (t >> 6)) base += fill[w];
    total += fill[w];
  }
  __syncthreads();
  const uint32_t j = part_block();
#pragma unroll
  for (uint32_t k = 0; k < kPerT; ++k) {
    const uint32_t b = t * kPerT + k;
    cur[b] = base + offs[static_cast<uint64_t>(j) * nbins + b];
    fill[b] = 0;
    if (j == 0) fbase[b] = base;
    base += v[k];
  }
  if (j == 0 && t == 0) fbase[nbins] = total;
  if (t == 0) ovf_n = 0;
  __syncthreads();
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  const uint32_t rounds = t1 > t0 ? static_cast<uint32_t>((t1 - t0 + kRound - 1) / kRound) : 0u;
  if (t < kWsProd) {
    RowBatch<kWsRows> qa, qb;
    in.template load_many<kWsRows>(t0 + t, kWsProd, t1, t0, qa);
    in.template load_many<kWsRows>(t0 + kRound + t, kWsProd, t1, t0, qb);
    auto stage_round = [&](const RowBatch<kWsRows>& q) {
      uint32_t bk[kWsRows], sl[kWsRows];
      uint3 rq[kWsRows];
      bool ok[kWsRows];
#pragma unroll
      for (int u = 0; u < kWsRows; ++u) {
        ok[u] = in.valid_of(q, u);
        const uint64_t h = row_hash(in.key_of(q, u));
        bk[u] = digit_of(h, skip, kStageBits);
        rq[u] = make_uint3(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32), in.row_of(q, u));
      }
#pragma unroll
      for (int u = 0; u < kWsRows; ++u) sl[u] = ok[u] ? atomicAdd(&fill[bk[u]], 1u) : 2u;
      uint32_t nov = 0;
#pragma unroll
      for (int u = 0; u < kWsRows; ++u) {
        if (ok[u] && sl[u] < 2) stage[bk[u]][sl[u]] = rq[u];
        nov += (ok[u] && sl[u] >= 2) ? 1u : 0u;
      }
      if (nov) {
        uint32_t o = atomicAdd(&ovf_n, nov);
#pragma unroll
        for (int u = 0; u < kWsRows; ++u)
          if (ok[u] && sl[u] >= 2) ovf[o++] = rq[u];
      }
    };
    for (uint32_t r = 0; r < rounds; r += 2) {
      stage_round(qa);
      lds_barrier();
      in.template load_many<kWsRows>(t0 + (r + 2) * static_cast<uint64_t>(kRound) + t, kWsProd, t1,
                                     t0, qa);
      lds_barrier();
      lds_barrier();
      if (r + 1 >= rounds) break;
      stage_round(qb);
      lds_barrier();
      in.template load_many<kWsRows>(t0 + (r + 3) * static_cast<uint64_t>(kRound) + t, kWsProd, t1,
                                     t0, qb);
      lds_barrier();
      lds_barrier();
    }
  } else {
    const uint32_t c = t - kWsProd;
    uint32_t junk = 0;
    for (uint32_t r = 0; r < rounds; ++r) {
      lds_barrier();
      {
        const uint64_t r0 = t0 + static_cast<uint64_t>(r) * kRound;
#pragma unroll
        for (uint32_t u = 0; u < kRound / kWsProd; ++u) {
          const uint64_t i = r0 + c + u * kWsProd;
          if (i < t1) rep[i] = in.rank_base + static_cast<uint32_t>(i);
        }
      }
      uint32_t f[kPerC], p[kPerC];
      uint3 x0[kPerC], x1[kPerC];
#pragma unroll
      for (uint32_t k = 0; k < kPerC; ++k) f[k] = fill[c + k * kWsProd];
      // unconditional reads (no branch between them: one LDS latency); a
      // wave executes every bucket's branch anyway, some lane's is full
#pragma unroll
      for (uint32_t k = 0; k < kPerC; ++k) {
        const uint32_t b = c + k * kWsProd;
        p[k] = cur[b];
        x0[k] = stage[b][0];
        x1[k] = stage[b][1];
      }
      // keep the reads here (the compiler sinks them into the branches below
      // and waits for each bucket's in turn)
#pragma unroll
      for (uint32_t k = 0; k < kPerC; ++k)
        asm volatile("" ::"v"(p[k]), "v"(x0[k].x), "v"(x0[k].y), "v"(x0[k].z), "v"(x1[k].x),
                     "v"(x1[k].y), "v"(x1[k].z));
      const uint32_t no = ovf_n;
#pragma unroll
      for (uint32_t k = 0; k < kPerC; ++k) {
        const uint32_t b = c + k * kWsProd;
        if (f[k] >= 2) {
          if constexpr (kStore) {
            out[p[k]] = x0[k];
            out[p[k] + 1] = x1[k];
          } else {
            junk += x0[k].x ^ x1[k].y;
          }
          cur[b] = p[k] + 2;
          fill[b] = 0;
        }
      }
      lds_barrier();  // M: fills, cursors and ovf_n read by every consumer
      for (uint32_t o = c; o < no; o += kWsProd) {
        const uint3 rq = ovf[o];
        const uint32_t q = atomicAdd(&cur[digit_of((static_cast<uint64_t>(rq.y) << 32) | rq.x, skip,
                                                   kStageBits)], 1u);
        if constexpr (kStore) out[q] = rq;
        else junk += rq.z ^ q;
      }
      if (c == 0) ovf_n = 0;
      lds_barrier();
    }
    if (!kStore && junk == 0x12345678u) out[0] = make_uint3(junk, 0, 0);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads)
    for (uint32_t k = 0; k < fill[b]; ++k) out[cur[b] + k] = stage[b][k];
}

// k_part_scatter_ws generalised to 2^kBits buckets with kSlots-record staging
// (kSlots x 2^kBits x 12 B = 96 KiB): fewer, longer runs per flush.
template <uint32_t kBits, uint32_t kSlots, bool kStore>
__global__ __launch_bounds__(kPartThreads) void k_ws_gen(RowsIn in, uint64_t n, uint32_t skip,
                                                         const uint32_t* __restrict__ offs,
                                                         const uint32_t* __restrict__ ftot,
                                                         uint3* __restrict__ out,
                                                         uint32_t* __restrict__ rep,
                                                         uint32_t* __restrict__ fbase) {
  constexpr uint32_t nbins = 1u << kBits;
  constexpr uint32_t kRound = kWsProd * kWsRows;
  __shared__ uint3 stage[nbins][kSlots];
  __shared__ uint32_t fill[nbins], cur[nbins];
  __shared__ uint3 ovf[kRound];
  __shared__ uint32_t ovf_n;
  __shared__ uint32_t wsum[kPartThreads / 64];
  constexpr uint32_t kPerT = nbins >= kPartThreads ? nbins / kPartThreads : 1u;
  const uint32_t t = threadIdx.x, lane = __lane_id();
  uint32_t v[kPerT], sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPerT; ++k) {
    const uint32_t b = t * kPerT + k;
    v[k] = b < nbins ? ftot[b] : 0u;
    sum += v[k];
  }
  uint32_t inc = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d);
    if (lane >= static_cast<uint32_t>(d)) inc += o;
  }
  if (lane == 63) wsum[t >> 6] = inc;
  __syncthreads();
  uint32_t base = inc - sum, total = 0;
  for (uint32_t w = 0; w < kPartThreads / 64; ++w) {
    if (w < (t >> 6)) base += wsum[w];
    total += wsum[w];
  }
  const uint32_t j = part_block();
#pragma unroll
  for (uint32_t k = 0; k < kPerT; ++k) {
    const uint32_t b = t * kPerT + k;
    if (b < nbins) {
      cur[b] = base + offs[static_cast<uint64_t>(j) * nbins + b];
      fill[b] = 0;
      if (j == 0) fbase[b] = base;
    }
    base += v[k];
  }
  if (j == 0 && t == 0) fbase[nbins] = total;
  if (t == 0) ovf_n = 0;
  __syncthreads();
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  const uint32_t rounds = t1 > t0 ? static_cast<uint32_t>((t1 - t0 + kRound - 1) / kRound) : 0u;
  if (t < kWsProd) {
    RowBatch<kWsRows> qa, qb;
    in.template load_many<kWsRows>(t0 + t, kWsProd, t1, t0, qa);
    in.template load_many<kWsRows>(t0 + kRound + t, kWsProd, t1, t0, qb);
    auto stage_round = [&](const RowBatch<kWsRows>& q) {
#pragma unroll
      for (int u = 0; u < kWsRows; ++u) {
        if (!in.valid_of(q, u)) continue;
        const uint64_t h = row_hash(in.key_of(q, u));
        const uint32_t b = digit_of(h, skip, kBits);
        const uint3 rq = make_uint3(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32),
                                    in.row_of(q, u));
        const uint32_t sl = atomicAdd(&fill[b], 1u);
        if (sl < kSlots)
          stage[b][sl] = rq;
        else
          ovf[atomicAdd(&ovf_n, 1u)] = rq;
      }
    };
    for (uint32_t r = 0; r < rounds; r += 2) {
      stage_round(qa);
      lds_barrier();
      in.template load_many<kWsRows>(t0 + (r + 2) * static_cast<uint64_t>(kRound) + t, kWsProd, t1,
                                     t0, qa);
      lds_barrier();
      lds_barrier();
      if (r + 1 >= rounds) break;
      stage_round(qb);
      lds_barrier();
      in.template load_many<kWsRows>(t0 + (r + 3) * static_cast<uint64_t>(kRound) + t, kWsProd, t1,
                                     t0, qb);
      lds_barrier();
      lds_barrier();
    }
  } else {
    const uint32_t c = t - kWsProd;
    uint32_t junk = 0;
    for (uint32_t r = 0; r < rounds; ++r) {
      lds_barrier();
      {
        const uint64_t r0 = t0 + static_cast<uint64_t>(r) * kRound;
#pragma unroll
        for (uint32_t u = 0; u < kRound / kWsProd; ++u) {
          const uint64_t i = r0 + c + u * kWsProd;
          if (i < t1) rep[i] = in.rank_base + static_cast<uint32_t>(i);
        }
      }
#pragma unroll
      for (uint32_t k = 0; k < (nbins + kWsProd - 1) / kWsProd; ++k) {
        const uint32_t b = c + k * kWsProd;
        if (b < nbins && fill[b] >= kSlots) {
          const uint32_t p = cur[b];
#pragma unroll
          for (uint32_t e = 0; e < kSlots; ++e) {
            const uint3 x = stage[b][e];
            if constexpr (kStore) out[p + e] = x;
            else junk += x.x;
          }
          cur[b] = p + kSlots;
          fill[b] = 0;
        }
      }
      const uint32_t no = ovf_n;
      lds_barrier();
      for (uint32_t o = c; o < no; o += kWsProd) {
        const uint3 rq = ovf[o];
        const uint32_t p = atomicAdd(&cur[digit_of((static_cast<uint64_t>(rq.y) << 32) | rq.x, skip,
                                                   kBits)], 1u);
        if constexpr (kStore) out[p] = rq;
        else junk += rq.z ^ p;
      }
      if (c == 0) ovf_n = 0;
      lds_barrier();
    }
    if (!kStore && junk == 0x12345678u) out[0] = make_uint3(junk, 0, 0);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads)
    for (uint32_t k = 0; k < fill[b]; ++k) out[cur[b] + k] = stage[b][k];
}

// Cooperative flush: a producer whose row fills a bucket's kSlots slots
// appends the bucket to an LDS list; the consumers then write each listed
// bucket's kSlots records with kSlots ADJACENT lanes (one contiguous run per
// lane group: the stores of a wave-instruction touch 64 / kSlots runs, not 64),
// lane 0 of the group advancing the cursor.
template <uint32_t kBits, uint32_t kSlots, bool kStore>
__global__ __launch_bounds__(kPartThreads) void k_ws_coop(RowsIn in, uint64_t n, uint32_t skip,
                                                          const uint32_t* __restrict__ offs,
                                                          const uint32_t* __restrict__ ftot,
                                                          uint3* __restrict__ out,
                                                          uint32_t* __restrict__ rep,
                                                          uint32_t* __restrict__ fbase) {
  constexpr uint32_t nbins = 1u << kBits;
  constexpr uint32_t kRound = kWsProd * kWsRows;
  static_assert(64 % kSlots == 0, "runs do not straddle waves");
  __shared__ uint3 stage[nbins][kSlots];
  __shared__ uint32_t fill[nbins], cur[nbins];
  __shared__ uint16_t full[nbins];
  __shared__ uint3 ovf[kRound - 1];  // >= 1 row of a round takes a slot
  __shared__ uint32_t ovf_n, full_n;
  uint32_t* wsum = reinterpret_cast<uint32_t*>(full);  // prologue scratch (LDS is full)
  constexpr uint32_t kPerT = nbins >= kPartThreads ? nbins / kPartThreads : 1u;
  const uint32_t t = threadIdx.x, lane = __lane_id();
  uint32_t v[kPerT], sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPerT; ++k) {
    const uint32_t b = t * kPerT + k;
    v[k] = b < nbins ? ftot[b] : 0u;
    sum += v[k];
  }
  uint32_t inc = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d);
    if (lane >= static_cast<uint32_t>(d)) inc += o;
  }
  if (lane == 63) wsum[t >> 6] = inc;
  __syncthreads();
  uint32_t base = inc - sum, total = 0;
  for (uint32_t w = 0; w < kPartThreads / 64; ++w) {
    if (w < (t >> 6)) base += wsum[w];
    total += wsum[w];
  }
  __syncthreads();  // wsum (= full) read by every wave
  const uint32_t j = part_block();
#pragma unroll
  for (uint32_t k = 0; k < kPerT; ++k) {
    const uint32_t b = t * kPerT + k;
    if (b < nbins) {
      cur[b] = base + offs[static_cast<uint64_t>(j) * nbins + b];
      fill[b] = 0;
      if (j == 0) fbase[b] = base;
    }
    base += v[k];
  }
  if (j == 0 && t == 0) fbase[nbins] = total;
  if (t == 0) {
    ovf_n = 0;
    full_n = 0;
  }
  __syncthreads();
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  const uint32_t rounds = t1 > t0 ? static_cast<uint32_t>((t1 - t0 + kRound - 1) / kRound) : 0u;
  if (t < kWsProd) {
    RowBatch<kWsRows> qa, qb;
    in.template load_many<kWsRows>(t0 + t, kWsProd, t1, t0, qa);
    in.template load_many<kWsRows>(t0 + kRound + t, kWsProd, t1, t0, qb);
    auto stage_round = [&](const RowBatch<kWsRows>& q) {
#pragma unroll
      for (int u = 0; u < kWsRows; ++u) {
        if (!in.valid_of(q, u)) continue;
        const uint64_t h = row_hash(in.key_of(q, u));
        const uint32_t b = digit_of(h, skip, kBits);
        const uint3 rq = make_uint3(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32),
                                    in.row_of(q, u));
        const uint32_t sl = atomicAdd(&fill[b], 1u);
        if (sl < kSlots) {
          stage[b][sl] = rq;
          if (sl == kSlots - 1) full[atomicAdd(&full_n, 1u)] = static_cast<uint16_t>(b);
        } else {
          ovf[atomicAdd(&ovf_n, 1u)] = rq;
        }
      }
    };
    for (uint32_t r = 0; r < rounds; r += 2) {
      stage_round(qa);
      lds_barrier();
      in.template load_many<kWsRows>(t0 + (r + 2) * static_cast<uint64_t>(kRound) + t, kWsProd, t1,
                                     t0, qa);
      lds_barrier();
      lds_barrier();
      if (r + 1 >= rounds) break;
      stage_round(qb);
      lds_barrier();
      in.template load_many<kWsRows>(t0 + (r + 3) * static_cast<uint64_t>(kRound) + t, kWsProd, t1,
                                     t0, qb);
      lds_barrier();
      lds_barrier();
    }
  } else {
    const uint32_t c = t - kWsProd;
    uint32_t junk = 0;
    for (uint32_t r = 0; r < rounds; ++r) {
      lds_barrier();  // A
      {
        const uint64_t r0 = t0 + static_cast<uint64_t>(r) * kRound;
#pragma unroll
        for (uint32_t u = 0; u < kRound / kWsProd; ++u) {
          const uint64_t i = r0 + c + u * kWsProd;
          if (i < t1) rep[i] = in.rank_base + static_cast<uint32_t>(i);
        }
      }
      const uint32_t nf = full_n, no = ovf_n;
      for (uint32_t x = c; x < nf * kSlots; x += kWsProd) {
        const uint32_t e = x / kSlots, k = x % kSlots;
        const uint32_t b = full[e];
        const uint32_t p = cur[b];
        const uint3 rec = stage[b][k];
        if constexpr (kStore) out[p + k] = rec;
        else junk += rec.x ^ p;
        if (k == 0) {
          cur[b] = p + kSlots;  // after every lane of the group read it (same wave)
          fill[b] = 0;
        }
      }
      lds_barrier();  // M: cursors advanced, counts read
      for (uint32_t o = c; o < no; o += kWsProd) {
        const uint3 rq = ovf[o];
        const uint32_t p = atomicAdd(&cur[digit_of((static_cast<uint64_t>(rq.y) << 32) | rq.x, skip,
                                                   kBits)], 1u);
        if constexpr (kStore) out[p] = rq;
        else junk += rq.z ^ p;
      }
      if (c == 0) {
        ovf_n = 0;
        full_n = 0;
      }
      lds_barrier();  // B
    }
    if (!kStore && junk == 0x12345678u) out[0] = make_uint3(junk, 0, 0);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads)
    for (uint32_t k = 0; k < fill[b]; ++k) out[cur[b] + k] = stage[b][k];
}

// Two barriers per round: a row that meets a full bucket is written straight
// away by its producer (cursor taken by an LDS atomic in the producers' phase,
// before the consumers flush), so there is no overflow list and no middle
// barrier; kRows rows per producer thread per round.
template <uint32_t kBits, uint32_t kSlots, int kRows, bool kStore>
__global__ __launch_bounds__(kPartThreads) void k_ws_coop2(RowsIn in, uint64_t n, uint32_t skip,
                                                           const uint32_t* __restrict__ offs,
                                                           const uint32_t* __restrict__ ftot,
                                                           uint3* __restrict__ out,
                                                           uint32_t* __restrict__ rep,
                                                           uint32_t* __restrict__ fbase) {
  constexpr uint32_t nbins = 1u << kBits;
  constexpr uint32_t kRound = kWsProd * kRows;
  static_assert(64 % kSlots == 0, "runs do not straddle waves");
  __shared__ uint3 stage[nbins][kSlots];
  __shared__ uint32_t fill[nbins], cur[nbins];
  __shared__ uint16_t full[nbins];
  __shared__ uint32_t full_n[2];  // by round parity: reset a round ahead, no extra barrier
  __shared__ uint32_t wsum[kPartThreads / 64];
  constexpr uint32_t kPerT = nbins >= kPartThreads ? nbins / kPartThreads : 1u;
  const uint32_t t = threadIdx.x, lane = __lane_id();
  uint32_t v[kPerT], sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPerT; ++k) {
    const uint32_t b = t * kPerT + k;
    v[k] = b < nbins ? ftot[b] : 0u;
    sum += v[k];
  }
  uint32_t inc = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d);
    if (lane >= static_cast<uint32_t>(d)) inc += o;
  }
  if (lane == 63) wsum[t >> 6] = inc;
  __syncthreads();
  uint32_t base = inc - sum, total = 0;
  for (uint32_t w = 0; w < kPartThreads / 64; ++w) {
    if (w < (t >> 6)) base += wsum[w];
    total += wsum[w];
  }
  const uint32_t j = part_block();
#pragma unroll
  for (uint32_t k = 0; k < kPerT; ++k) {
    const uint32_t b = t * kPerT + k;
    if (b < nbins) {
      cur[b] = base + offs[static_cast<uint64_t>(j) * nbins + b];
      fill[b] = 0;
      if (j == 0) fbase[b] = base;
    }
    base += v[k];
  }
  if (j == 0 && t == 0) fbase[nbins] = total;
  if (t == 0) full_n[0] = full_n[1] = 0;
  __syncthreads();
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  const uint32_t rounds = t1 > t0 ? static_cast<uint32_t>((t1 - t0 + kRound - 1) / kRound) : 0u;
  if (t < kWsProd) {
    RowBatch<kRows> qa, qb;
    in.template load_many<kRows>(t0 + t, kWsProd, t1, t0, qa);
    in.template load_many<kRows>(t0 + kRound + t, kWsProd, t1, t0, qb);
    auto stage_round = [&](const RowBatch<kRows>& q, uint32_t par) {
#pragma unroll
      for (int u = 0; u < kRows; ++u) {
        if (!in.valid_of(q, u)) continue;
        const uint64_t h = row_hash(in.key_of(q, u));
        const uint32_t b = digit_of(h, skip, kBits);
        const uint3 rq = make_uint3(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32),
                                    in.row_of(q, u));
        const uint32_t sl = atomicAdd(&fill[b], 1u);
        if (sl < kSlots) {
          stage[b][sl] = rq;
          if (sl == kSlots - 1) full[atomicAdd(&full_n[par], 1u)] = static_cast<uint16_t>(b);
        } else {
          const uint32_t p = atomicAdd(&cur[b], 1u);
          if constexpr (kStore) out[p] = rq;
        }
      }
    };
    for (uint32_t r = 0; r < rounds; r += 2) {
      stage_round(qa, r & 1u);
      lds_barrier();  // A
      in.template load_many<kRows>(t0 + (r + 2) * static_cast<uint64_t>(kRound) + t, kWsProd, t1,
                                   t0, qa);
      lds_barrier();  // B
      if (r + 1 >= rounds) break;
      stage_round(qb, (r + 1) & 1u);
      lds_barrier();  // A
      in.template load_many<kRows>(t0 + (r + 3) * static_cast<uint64_t>(kRound) + t, kWsProd, t1,
                                   t0, qb);
      lds_barrier();  // B
    }
  } else {
    const uint32_t c = t - kWsProd;
    uint32_t junk = 0;
    for (uint32_t r = 0; r < rounds; ++r) {
      lds_barrier();  // A
      {
        const uint64_t r0 = t0 + static_cast<uint64_t>(r) * kRound;
#pragma unroll
        for (uint32_t u = 0; u < kRound / kWsProd; ++u) {
          const uint64_t i = r0 + c + u * kWsProd;
          if (i < t1) rep[i] = in.rank_base + static_cast<uint32_t>(i);
        }
      }
      const uint32_t nf = full_n[r & 1u];
      if (c == 0) full_n[(r + 1) & 1u] = 0;  // last read in round r - 1
      for (uint32_t x = c; x < nf * kSlots; x += kWsProd) {
        const uint32_t e = x / kSlots, k = x % kSlots;
        const uint32_t b = full[e];
        const uint32_t p = cur[b];
        const uint3 rec = stage[b][k];
        if constexpr (kStore) out[p + k] = rec;
        else junk += rec.x ^ p;
        if (k == 0) {
          cur[b] = p + kSlots;
          fill[b] = 0;
        }
      }
      lds_barrier();  // B
    }
    if (!kStore && junk == 0x12345678u) out[0] = make_uint3(junk, 0, 0);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads)
    for (uint32_t k = 0; k < fill[b]; ++k) out[cur[b] + k] = stage[b][k];
}

// Group-by of 11-bit buckets (~6.1 k rows) in ONE workgroup, as two 12-bit
// sub-buckets (the next hash bit) grouped one after the other in the same
// packed 7680-slot LDS table (76 KiB: two workgroups per CU).  A record's
// state between the passes is 3 registers: mine = {h without its 12 digit
// bits, index in its sub-bucket + 1} and its row.  Slot = h bits [0, 32)
// scaled, probe step from h bits [32, 42) (both outside the digit bits).
constexpr int kG2Per = 7;                          // records per thread
// the global-table path out of line: inlined twice it set the kernel's
// register allocation (spills)
__device__ __attribute__((noinline)) void group11_global(const uint3* rec, uint32_t rank_base,
                                                         uint32_t start, uint32_t end,
                                                         ChunkOf chunk_of, uint64_t* gkey,
                                                         uint32_t* gmin, uint32_t* rep,
                                                         uint32_t* special_min) {
  group_bucket_global(Rec12Src{rec, rank_base}, start, end, chunk_of, gkey, gmin, rep, *special_min);
}
constexpr uint32_t kG2Cap = kG2Per * kGroupThreads;  // larger buckets: global table
__global__ __launch_bounds__(kGroupThreads, 8) void k_group11(const uint3* __restrict__ rec,
                                                              uint32_t rank_base,
                                                              const uint32_t* __restrict__ offs,
                                                              ChunkOf chunk_of,
                                                              uint64_t* __restrict__ gkey,
                                                              uint32_t* __restrict__ gmin,
                                                              uint32_t* __restrict__ rep) {
  __shared__ uint64_t tab[kPkSlots];
  __shared__ uint32_t lmin[kPkCap + 1];
  __shared__ uint32_t scnt[2];
  __shared__ uint32_t special_min;
  const uint32_t start = offs[blockIdx.x], end = offs[blockIdx.x + 1];
  const uint32_t m = end - start;
  if (m == 0) return;
  if (m > kG2Cap) {
    group_bucket_global(Rec12Src{rec, rank_base}, start, end, chunk_of, gkey, gmin, rep, special_min);
    return;
  }
  if (threadIdx.x < 2) scnt[threadIdx.x] = 0;
  uint3 q[kG2Per];
#pragma unroll
  for (int j = 0; j < kG2Per; ++j) q[j] = rec[min(start + threadIdx.x + j * kGroupThreads, end - 1)];
#pragma unroll
  for (int j = 0; j < kG2Per; ++j)
    if (start + threadIdx.x + j * kGroupThreads >= end) q[j] = make_uint3(0, 0, kPadRow);
  __syncthreads();  // scnt
  uint64_t mine[kG2Per];
  uint32_t row[kG2Per], sub1 = 0, live = 0;
#pragma unroll
  for (int j = 0; j < kG2Per; ++j) {
    const uint64_t h = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
    row[j] = q[j].z;
    const uint32_t sb = digit_of(h, kShardBits + 11, 1);
    uint32_t idx = 0;
    if (row[j] != kPadRow) {
      live |= 1u << j;
      sub1 |= sb << j;
      idx = atomicAdd(&scnt[sb], 1u);
    }
    mine[j] = (key_rest(h, 12) << 12) | ((idx + 1) & 0xFFFu);
  }
  for (uint32_t s = threadIdx.x; s < kPkSlots; s += kGroupThreads) tab[s] = 0ull;
  for (uint32_t s = threadIdx.x; s <= kPkCap; s += kGroupThreads) lmin[s] = 0xFFFFFFFFu;
  __syncthreads();  // table clear; scnt final
  if (scnt[0] > kPkCap || scnt[1] > kPkCap) {  // a sub-bucket beyond 12-bit indices
    group_bucket_global(Rec12Src{rec, rank_base}, start, end, chunk_of, gkey, gmin, rep, special_min);
    return;
  }
#pragma unroll 1
  for (uint32_t sp = 0; sp < 2; ++sp) {
    if (sp == 1) {
      __syncthreads();  // pass 0's lookups done
      for (uint32_t s = threadIdx.x; s < kPkSlots; s += kGroupThreads) tab[s] = 0ull;
      for (uint32_t s = threadIdx.x; s <= kPkCap; s += kGroupThreads) lmin[s] = 0xFFFFFFFFu;
      __syncthreads();
    }
    const uint32_t act = live & (sp ? sub1 : ~sub1);
    // slot[j]: the probe slot while record j probes, then its owner's index
    // (the step is recomputed from mine on a collision: registers are the
    // occupancy limit here)
    uint32_t slot[kG2Per];
#pragma unroll
    for (int j = 0; j < kG2Per; ++j)
      slot[j] = static_cast<uint32_t>((static_cast<uint64_t>(static_cast<uint32_t>(mine[j] >> 12)) * kPkSlots) >> 32);
    uint32_t pend = act;
    while (pend) {
      uint64_t prev[kG2Per];
#pragma unroll
      for (int j = 0; j < kG2Per; ++j)
        prev[j] = (pend >> j & 1u)
                      ? atomicCAS(reinterpret_cast<unsigned long long*>(&tab[slot[j]]), 0ull,
                                  static_cast<unsigned long long>(mine[j]))
                      : 0ull;
#pragma unroll
      for (int j = 0; j < kG2Per; ++j) {
        if (!(pend >> j & 1u)) continue;
        if (prev[j] == 0ull) {
          slot[j] = static_cast<uint32_t>(mine[j] & 0xFFFu) - 1;  // placed: owns its key
          pend &= ~(1u << j);
        } else if ((prev[j] >> 12) == (mine[j] >> 12)) {
          slot[j] = static_cast<uint32_t>(prev[j] & 0xFFFu) - 1;
          pend &= ~(1u << j);
        } else {
          uint32_t st = 1u + 2u * static_cast<uint32_t>((mine[j] >> 44) & 1023u);  // h bits [32, 42)
          st += (st % 3u == 0) ? 2u : 0u;
          st += (st % 5u == 0) ? 2u : 0u;
          st += (st % 3u == 0) ? 2u : 0u;
          const uint32_t sn = slot[j] + st;
          slot[j] = sn >= kPkSlots ? sn - kPkSlots : sn;
        }
      }
    }
    uint32_t* owner = slot;
#pragma unroll
    for (int j = 0; j < kG2Per; ++j)
      if (act >> j & 1u) atomicMin(&lmin[owner[j]], rank_base + row[j]);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kG2Per; ++j) {
      if (!(act >> j & 1u)) continue;
      const uint32_t r = rank_base + row[j], f = lmin[owner[j]];
      if (chunk_of(r) != chunk_of(f)) rep[row[j]] = f;
    }
  }
}

// The same grouping with BOTH sub-buckets' tables in LDS at once (152 KiB:
// one workgroup per CU, 128 registers): one probe pass over the 7 records.
__global__ __launch_bounds__(kGroupThreads, 4) void k_group11b(const uint3* __restrict__ rec,
                                                               uint32_t rank_base,
                                                               const uint32_t* __restrict__ offs,
                                                               ChunkOf chunk_of,
                                                               uint64_t* __restrict__ gkey,
                                                               uint32_t* __restrict__ gmin,
                                                               uint32_t* __restrict__ rep) {
  __shared__ uint64_t tab[2][kPkSlots];
  __shared__ uint32_t lmin[2][kPkCap + 1];
  __shared__ uint32_t scnt[2];
  __shared__ uint32_t special_min;
  const uint32_t start = offs[blockIdx.x], end = offs[blockIdx.x + 1];
  const uint32_t m = end - start;
  if (m == 0) return;
  if (m > kG2Cap) {
    group_bucket_global(Rec12Src{rec, rank_base}, start, end, chunk_of, gkey, gmin, rep, special_min);
    return;
  }
  if (threadIdx.x < 2) scnt[threadIdx.x] = 0;
  uint3 q[kG2Per];
#pragma unroll
  for (int j = 0; j < kG2Per; ++j) q[j] = rec[min(start + threadIdx.x + j * kGroupThreads, end - 1)];
#pragma unroll
  for (int j = 0; j < kG2Per; ++j)
    if (start + threadIdx.x + j * kGroupThreads >= end) q[j] = make_uint3(0, 0, kPadRow);
  for (uint32_t s = threadIdx.x; s < 2 * kPkSlots; s += kGroupThreads) (&tab[0][0])[s] = 0ull;
  for (uint32_t s = threadIdx.x; s < 2 * (kPkCap + 1); s += kGroupThreads) (&lmin[0][0])[s] = 0xFFFFFFFFu;
  __syncthreads();  // scnt, tables
  uint64_t mine[kG2Per];
  uint32_t slot[kG2Per], sub1 = 0, live = 0;
#pragma unroll
  for (int j = 0; j < kG2Per; ++j) {
    const uint64_t h = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
    const uint32_t sb = digit_of(h, kShardBits + 11, 1);
    uint32_t idx = 0;
    if (q[j].z != kPadRow) {
      live |= 1u << j;
      sub1 |= sb << j;
      idx = atomicAdd(&scnt[sb], 1u);
    }
    mine[j] = (key_rest(h, 12) << 12) | ((idx + 1) & 0xFFFu);
    slot[j] = static_cast<uint32_t>((static_cast<uint64_t>(q[j].x) * kPkSlots) >> 32);
  }
  __syncthreads();  // scnt final
  if (scnt[0] > kPkCap || scnt[1] > kPkCap) {
    group_bucket_global(Rec12Src{rec, rank_base}, start, end, chunk_of, gkey, gmin, rep, special_min);
    return;
  }
  uint32_t pend = live;
  while (pend) {
    uint64_t prev[kG2Per];
#pragma unroll
    for (int j = 0; j < kG2Per; ++j)
      prev[j] = (pend >> j & 1u)
                    ? atomicCAS(reinterpret_cast<unsigned long long*>(&tab[sub1 >> j & 1u][slot[j]]),
                                0ull, static_cast<unsigned long long>(mine[j]))
                    : 0ull;
#pragma unroll
    for (int j = 0; j < kG2Per; ++j) {
      if (!(pend >> j & 1u)) continue;
      if (prev[j] == 0ull) {
        slot[j] = static_cast<uint32_t>(mine[j] & 0xFFFu) - 1;
        pend &= ~(1u << j);
      } else if ((prev[j] >> 12) == (mine[j] >> 12)) {
        slot[j] = static_cast<uint32_t>(prev[j] & 0xFFFu) - 1;
        pend &= ~(1u << j);
      } else {
        uint32_t st = 1u + 2u * static_cast<uint32_t>((mine[j] >> 44) & 1023u);
        st += (st % 3u == 0) ? 2u : 0u;
        st += (st % 5u == 0) ? 2u : 0u;
        st += (st % 3u == 0) ? 2u : 0u;
        const uint32_t sn = slot[j] + st;
        slot[j] = sn >= kPkSlots ? sn - kPkSlots : sn;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < kG2Per; ++j)
    if (live >> j & 1u) atomicMin(&lmin[sub1 >> j & 1u][slot[j]], rank_base + q[j].z);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kG2Per; ++j) {
    if (!(live >> j & 1u)) continue;
    const uint32_t r = rank_base + q[j].z, f = lmin[sub1 >> j & 1u][slot[j]];
    if (chunk_of(r) != chunk_of(f)) rep[q[j].z] = f;
  }
}

// Persistent packed-table group: kWg workgroups (2 per CU) walk the buckets;
// the table is cleared ONCE, and after each bucket every record that placed
// a key clears the slot it placed it in and its lmin entry (about 2.5 k of the
// 7680 + 4096 words a full clear writes).  kPrefetch: the next bucket's
// records are loaded while the current one is grouped.
template <bool kPrefetch>
__global__ __launch_bounds__(kGroupThreads, 8) void k_group_pers(const uint3* __restrict__ rec,
                                                                 uint32_t rank_base,
                                                                 const uint32_t* __restrict__ offs,
                                                                 uint32_t nb, ChunkOf chunk_of,
                                                                 uint64_t* __restrict__ gkey,
                                                                 uint32_t* __restrict__ gmin,
                                                                 uint32_t* __restrict__ rep) {
  __shared__ uint64_t tab[kPkSlots];
  __shared__ uint32_t lmin[kPkCap + 1];
  __shared__ uint32_t special_min;
  constexpr int kP = (kPkCap + kGroupThreads) / kGroupThreads;  // 4
  for (uint32_t s = threadIdx.x; s < kPkSlots; s += kGroupThreads) tab[s] = 0ull;
  for (uint32_t s = threadIdx.x; s <= kPkCap; s += kGroupThreads) lmin[s] = 0xFFFFFFFFu;
  const Rec12Src src{rec, rank_base};
  uint3 nq[kP];
  auto load = [&](uint32_t b, uint3 (&q)[kP]) {
    const uint32_t st = offs[b], en = offs[b + 1];
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      const uint32_t i = st + threadIdx.x + j * kGroupThreads;
      q[j] = (i < en && en - st <= kPkCap) ? rec[i] : make_uint3(0, 0, kPadRow);
    }
  };
  if (kPrefetch && blockIdx.x < nb) load(blockIdx.x, nq);
  __syncthreads();
  for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const uint32_t start = offs[b], end = offs[b + 1];
    if (end - start > kPkCap) {  // uniform: the global table (LDS untouched)
      group_bucket_global(src, start, end, chunk_of, gkey, gmin, rep, special_min);
      if (kPrefetch && b + gridDim.x < nb) load(b + gridDim.x, nq);
      __syncthreads();
      continue;
    }
    uint3 q[kP];
    if constexpr (kPrefetch) {
#pragma unroll
      for (int j = 0; j < kP; ++j) q[j] = nq[j];
      if (b + gridDim.x < nb) load(b + gridDim.x, nq);
    } else {
      load(b, q);
    }
    uint32_t slot[kP], owner[kP];
    uint64_t mine[kP];
    uint32_t pend = 0;
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      const uint64_t h = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
      const uint32_t idx = threadIdx.x + j * kGroupThreads;
      mine[j] = (key_rest(h, kStageBits) << 12) | (idx + 1);
      slot[j] = static_cast<uint32_t>((static_cast<uint64_t>(q[j].x) * kPkSlots) >> 32);
      owner[j] = idx;
      if (q[j].z != kPadRow) pend |= 1u << j;
    }
    const uint32_t live = pend;
    while (pend) {
      uint64_t prev[kP];
#pragma unroll
      for (int j = 0; j < kP; ++j)
        prev[j] = (pend >> j & 1u)
                      ? atomicCAS(reinterpret_cast<unsigned long long*>(&tab[slot[j]]), 0ull,
                                  static_cast<unsigned long long>(mine[j]))
                      : 0ull;
#pragma unroll
      for (int j = 0; j < kP; ++j) {
        if (!(pend >> j & 1u)) continue;
        if (prev[j] == 0ull) {
          pend &= ~(1u << j);
        } else if ((prev[j] >> 12) == (mine[j] >> 12)) {
          owner[j] = static_cast<uint32_t>(prev[j] & 0xFFFu) - 1;
          pend &= ~(1u << j);
        } else {
          const uint64_t h = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
          uint32_t st = 1u + 2u * static_cast<uint32_t>((h >> 40) & 1023u);
          st += (st % 3u == 0) ? 2u : 0u;
          st += (st % 5u == 0) ? 2u : 0u;
          st += (st % 3u == 0) ? 2u : 0u;
          const uint32_t sn = slot[j] + st;
          slot[j] = sn >= kPkSlots ? sn - kPkSlots : sn;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kP; ++j)
      if (live >> j & 1u) atomicMin(&lmin[owner[j]], rank_base + q[j].z);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      if (!(live >> j & 1u)) continue;
      const uint32_t r = rank_base + q[j].z, f = lmin[owner[j]];
      if (chunk_of(r) != chunk_of(f)) rep[q[j].z] = f;
    }
    __syncthreads();  // every lookup done before the owners clear
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      const uint32_t idx = threadIdx.x + j * kGroupThreads;
      if ((live >> j & 1u) && owner[j] == idx) {  // placed its key at slot[j]
        tab[slot[j]] = 0ull;
        lmin[idx] = 0xFFFFFFFFu;
      }
    }
    __syncthreads();
  }
}

// Asynchronous producer / consumer rounds: no workgroup barrier per round.
// Producers stage round r and, the last of their waves to finish, publish
// pround = r + 1; consumers flush round r's LISTED full buckets (and its
// overflow list) once pround > r, the last of their waves publishing
// cround = r + 1 after clearing round r's list counts.  A producer stages
// round r only after cround >= r - 1 (list buffers by round parity), so the
// producers run up to two rounds ahead instead of alternating with the
// consumers.  A flushed bucket's cursor is taken by an atomic (producers take
// cursors too when the overflow list is full) and its fill reset after its
// slots are read: a row arriving meanwhile saw fill >= 2 and went to the
// overflow list.  Every poll is bounded (kSpinCap): a broken protocol gives
// wrong rows, not a hung device.
constexpr uint32_t kAsyncOvf = 256;
constexpr uint32_t kSpinCap = 1u << 22;
__device__ __forceinline__ void spin_until(const uint32_t* ctr, uint32_t target, uint32_t* err) {
  uint32_t it = 0;
  while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < target) {
    __builtin_amdgcn_s_sleep(1);
    if (++it > kSpinCap) {
      *err = 1u;
      break;
    }
  }
}
template <bool kStore>
__global__ __launch_bounds__(kPartThreads) void k_ws_async(RowsIn in, uint64_t n, uint32_t skip,
                                                           const uint32_t* __restrict__ offs,
                                                           const uint32_t* __restrict__ ftot,
                                                           uint3* __restrict__ out,
                                                           uint32_t* __restrict__ rep,
                                                           uint32_t* __restrict__ fbase,
                                                           uint32_t* __restrict__ err) {
  constexpr uint32_t nbins = kNb;
  constexpr uint32_t kRound = kWsProd * kWsRows;
  constexpr uint32_t kPW = kWsProd / 64;  // producer waves
  __shared__ uint3 stage[nbins][2];
  __shared__ uint32_t fill[nbins], cur[nbins];
  __shared__ uint16_t flist[2][nbins];
  __shared__ uint3 ovf[2][kAsyncOvf];
  __shared__ uint32_t fn[2], on[2], pc[2], cc[2], pround, cround;
  constexpr uint32_t kPerT = nbins / kPartThreads;
  const uint32_t t = threadIdx.x, lane = __lane_id();
  uint32_t* wsum = reinterpret_cast<uint32_t*>(&flist[0][0]);  // prologue scratch
  uint32_t v[kPerT], sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPerT; ++k) {
    v[k] = ftot[t * kPerT + k];
    sum += v[k];
  }
  uint32_t inc = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d);
    if (lane >= static_cast<uint32_t>(d)) inc += o;
  }
  if (lane == 63) wsum[t >> 6] = inc;
  __syncthreads();
  uint32_t base = inc - sum, total = 0;
  for (uint32_t w = 0; w < kPartThreads / 64; ++w) {
    if (w < (t >> 6)) base += wsum[w];
    total += wsum[w];
  }
  __syncthreads();
  const uint32_t j = part_block();
#pragma unroll
  for (uint32_t k = 0; k < kPerT; ++k) {
    const uint32_t b = t * kPerT + k;
    cur[b] = base + offs[static_cast<uint64_t>(j) * nbins + b];
    fill[b] = 0;
    if (j == 0) fbase[b] = base;
    base += v[k];
  }
  if (j == 0 && t == 0) fbase[nbins] = total;
  if (t == 0) {
    fn[0] = fn[1] = on[0] = on[1] = 0;
    pc[0] = pc[1] = cc[0] = cc[1] = 0;
    pround = cround = 0;
  }
  __syncthreads();
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  const uint32_t rounds = t1 > t0 ? static_cast<uint32_t>((t1 - t0 + kRound - 1) / kRound) : 0u;
  if (t < kWsProd) {
    RowBatch<kWsRows> qa, qb;
    in.template load_many<kWsRows>(t0 + t, kWsProd, t1, t0, qa);
    in.template load_many<kWsRows>(t0 + kRound + t, kWsProd, t1, t0, qb);
    auto stage_round = [&](const RowBatch<kWsRows>& q, uint32_t r) {
      const uint32_t par = r & 1u;
      if (r >= 2) spin_until(&cround, r - 1, err);  // round r - 2's lists consumed
#pragma unroll
      for (int u = 0; u < kWsRows; ++u) {
        if (!in.valid_of(q, u)) continue;
        const uint64_t h = row_hash(in.key_of(q, u));
        const uint32_t b = digit_of(h, skip, kStageBits);
        const uint3 rq = make_uint3(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32),
                                    in.row_of(q, u));
        const uint32_t sl = atomicAdd(&fill[b], 1u);
        if (sl < 2) {
          stage[b][sl] = rq;
          if (sl == 1) flist[par][atomicAdd(&fn[par], 1u)] = static_cast<uint16_t>(b);
        } else {
          const uint32_t o = atomicAdd(&on[par], 1u);
          if (o < kAsyncOvf) {
            ovf[par][o] = rq;
          } else {
            const uint32_t p = atomicAdd(&cur[b], 1u);
            if constexpr (kStore) out[p] = rq;
          }
        }
      }
      // publish: every LDS write of this wave done, then one arrival per wave
      // on the round's (parity) counter; its last arriver resets the counter
      // and advances pround (atomic max: waves may be a round apart)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) {
        const uint32_t a = __hip_atomic_fetch_add(&pc[par], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (a == kPW - 1) {
          pc[par] = 0;
          __hip_atomic_fetch_max(&pround, r + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    };
    for (uint32_t r = 0; r < rounds; r += 2) {
      stage_round(qa, r);
      in.template load_many<kWsRows>(t0 + (r + 2) * static_cast<uint64_t>(kRound) + t, kWsProd, t1,
                                     t0, qa);
      if (r + 1 >= rounds) break;
      stage_round(qb, r + 1);
      in.template load_many<kWsRows>(t0 + (r + 3) * static_cast<uint64_t>(kRound) + t, kWsProd, t1,
                                     t0, qb);
    }
  } else {
    const uint32_t c = t - kWsProd;
    constexpr uint32_t kCW = (kPartThreads - kWsProd) / 64;
    for (uint32_t r = 0; r < rounds; ++r) {
      const uint32_t par = r & 1u;
      {
        const uint64_t r0 = t0 + static_cast<uint64_t>(r) * kRound;
#pragma unroll
        for (uint32_t u = 0; u < kRound / kWsProd; ++u) {
          const uint64_t i = r0 + c + u * kWsProd;
          if (i < t1) rep[i] = in.rank_base + static_cast<uint32_t>(i);
        }
      }
      spin_until(&pround, r + 1, err);
      const uint32_t nf = fn[par], no = min(on[par], kAsyncOvf);
      for (uint32_t e = c; e < nf; e += kWsProd) {
        const uint32_t b = flist[par][e];
        const uint3 x0 = stage[b][0], x1 = stage[b][1];
        const uint32_t p = atomicAdd(&cur[b], 2u);
        fill[b] = 0;  // after the slots were read (same wave, in order)
        if constexpr (kStore) {
          out[p] = x0;
          out[p + 1] = x1;
        }
      }
      for (uint32_t o = c; o < no; o += kWsProd) {
        const uint3 rq = ovf[par][o];
        const uint32_t p = atomicAdd(&cur[digit_of((static_cast<uint64_t>(rq.y) << 32) | rq.x, skip,
                                                   kStageBits)], 1u);
        if constexpr (kStore) out[p] = rq;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) {
        const uint32_t a = __hip_atomic_fetch_add(&cc[par], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (a == kCW - 1) {  // the round's last consumer wave: clear its lists
          cc[par] = 0;
          fn[par] = 0;
          on[par] = 0;
          __hip_atomic_fetch_max(&cround, r + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    }
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads)
    for (uint32_t k = 0; k < min(fill[b], 2u); ++k) out[cur[b] + k] = stage[b][k];
}

// kB buckets per workgroup: every bucket's records loaded up front (one
// memory latency for all of them), then the buckets grouped one after the
// other through the same table.  kLminInit: each record writes its own rank
// into lmin[its index] instead of the 4096-entry clear (only owners' entries
// are read).
template <int kB, bool kLminInit>
__global__ __launch_bounds__(kGroupThreads, 8) void k_group_multi(const uint3* __restrict__ rec,
                                                                  uint32_t rank_base,
                                                                  const uint32_t* __restrict__ offs,
                                                                  ChunkOf chunk_of,
                                                                  uint64_t* __restrict__ gkey,
                                                                  uint32_t* __restrict__ gmin,
                                                                  uint32_t* __restrict__ rep) {
  __shared__ uint64_t tab[kPkSlots];
  __shared__ uint32_t lmin[kPkCap + 1];
  __shared__ uint32_t special_min;
  constexpr int kP = (kPkCap + kGroupThreads) / kGroupThreads;  // 4
  uint3 q[kB][kP];
  uint32_t st[kB], en[kB];
#pragma unroll
  for (int bb = 0; bb < kB; ++bb) {
    const uint32_t b = blockIdx.x * kB + bb;
    st[bb] = offs[b];
    en[bb] = offs[b + 1];
  }
#pragma unroll
  for (int bb = 0; bb < kB; ++bb)
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      const uint32_t i = st[bb] + threadIdx.x + j * kGroupThreads;
      q[bb][j] = rec[min(i, max(en[bb], st[bb] + 1) - 1)];
    }
#pragma unroll
  for (int bb = 0; bb < kB; ++bb) {
    const uint32_t start = st[bb], end = en[bb];
    if (end - start > kPkCap) {  // uniform
      if (bb) __syncthreads();
      group_bucket_global(Rec12Src{rec, rank_base}, start, end, chunk_of, gkey, gmin, rep, special_min);
      continue;
    }
    if (bb) __syncthreads();  // the previous bucket's lookups done
    for (uint32_t s = threadIdx.x; s < kPkSlots; s += kGroupThreads) tab[s] = 0ull;
    if constexpr (!kLminInit)
      for (uint32_t s = threadIdx.x; s <= kPkCap; s += kGroupThreads) lmin[s] = 0xFFFFFFFFu;
    uint32_t slot[kP], owner[kP];
    uint64_t mine[kP];
    uint32_t pend = 0;
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      const uint3 v = q[bb][j];
      const uint64_t h = (static_cast<uint64_t>(v.y) << 32) | v.x;
      const uint32_t idx = threadIdx.x + j * kGroupThreads;
      mine[j] = (key_rest(h, kStageBits) << 12) | (idx + 1);
      slot[j] = static_cast<uint32_t>((static_cast<uint64_t>(v.x) * kPkSlots) >> 32);
      owner[j] = idx;
      if (start + idx < end) {
        pend |= 1u << j;
        if constexpr (kLminInit) lmin[idx] = rank_base + v.z;
      }
    }
    __syncthreads();
    const uint32_t live = pend;
    while (pend) {
      uint64_t prev[kP];
#pragma unroll
      for (int j = 0; j < kP; ++j)
        prev[j] = (pend >> j & 1u)
                      ? atomicCAS(reinterpret_cast<unsigned long long*>(&tab[slot[j]]), 0ull,
                                  static_cast<unsigned long long>(mine[j]))
                      : 0ull;
#pragma unroll
      for (int j = 0; j < kP; ++j) {
        if (!(pend >> j & 1u)) continue;
        if (prev[j] == 0ull) {
          pend &= ~(1u << j);
        } else if ((prev[j] >> 12) == (mine[j] >> 12)) {
          owner[j] = static_cast<uint32_t>(prev[j] & 0xFFFu) - 1;
          pend &= ~(1u << j);
        } else {
          const uint3 v = q[bb][j];
          const uint64_t h = (static_cast<uint64_t>(v.y) << 32) | v.x;
          uint32_t stp = 1u + 2u * static_cast<uint32_t>((h >> 40) & 1023u);
          stp += (stp % 3u == 0) ? 2u : 0u;
          stp += (stp % 5u == 0) ? 2u : 0u;
          stp += (stp % 3u == 0) ? 2u : 0u;
          const uint32_t sn = slot[j] + stp;
          slot[j] = sn >= kPkSlots ? sn - kPkSlots : sn;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kP; ++j)
      if ((live >> j & 1u) && (!kLminInit || owner[j] != threadIdx.x + j * kGroupThreads))
        atomicMin(&lmin[owner[j]], rank_base + q[bb][j].z);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      if (!(live >> j & 1u)) continue;
      const uint32_t r = rank_base + q[bb][j].z, f = lmin[owner[j]];
      if (chunk_of(r) != chunk_of(f)) rep[q[bb][j].z] = f;
    }
  }
}

// 11-bit buckets grouped as two 12-bit sub-buckets at TWO workgroups per CU:
// the 7 records per thread are loaded, then REDISTRIBUTED through LDS (the
// table's memory, not yet in use) into per-sub-bucket lists, and read back
// so that each thread holds at most 4 records of each sub-bucket; the two
// sub-buckets are then grouped one after the other exactly as the 12-bit
// kernel groups a bucket.
constexpr int kC4 = 4;  // records per thread per sub-bucket (4096 capacity)
struct SubRec {
  uint32_t lo, hi, row;  // h, row (h's low word first)
};
__global__ __launch_bounds__(kGroupThreads, 8) void k_group11c(const uint3* __restrict__ rec,
                                                               uint32_t rank_base,
                                                               const uint32_t* __restrict__ offs,
                                                               ChunkOf chunk_of,
                                                               uint64_t* __restrict__ gkey,
                                                               uint32_t* __restrict__ gmin,
                                                               uint32_t* __restrict__ rep) {
  __shared__ uint64_t tab[kPkSlots];    // 61440 B
  __shared__ uint32_t lmin[kPkCap + 1];  // 16384 B
  __shared__ uint32_t scnt[2];
  __shared__ uint32_t special_min;
  const uint32_t start = offs[blockIdx.x], end = offs[blockIdx.x + 1];
  const uint32_t m = end - start;
  if (m == 0) return;
  if (m > kG2Cap) {
    group_bucket_global(Rec12Src{rec, rank_base}, start, end, chunk_of, gkey, gmin, rep, special_min);
    return;
  }
  // scratch lists in the table's memory: sub-bucket s's records at
  // lst + s * 4096 (12 B each: 2 x 4096 x 12 = 96 KiB > 76 KiB, so the
  // capacity per sub-bucket here is (76 KiB / 2) / 12 B = 3276 records;
  // larger sub-buckets take the global table)
  constexpr uint32_t kLst = (sizeof(tab) + sizeof(lmin)) / 2 / sizeof(SubRec);  // 3276
  SubRec* lst = reinterpret_cast<SubRec*>(tab);
  if (threadIdx.x < 2) scnt[threadIdx.x] = 0;
  uint3 q[kG2Per];
#pragma unroll
  for (int j = 0; j < kG2Per; ++j) q[j] = rec[min(start + threadIdx.x + j * kGroupThreads, end - 1)];
  __syncthreads();  // scnt
#pragma unroll
  for (int j = 0; j < kG2Per; ++j) {
    if (start + threadIdx.x + j * kGroupThreads >= end) continue;
    const uint64_t h = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
    const uint32_t sb = digit_of(h, kShardBits + 11, 1);
    const uint32_t idx = atomicAdd(&scnt[sb], 1u);
    if (idx < kLst) lst[sb * kLst + idx] = SubRec{q[j].x, q[j].y, q[j].z};
  }
  __syncthreads();
  const uint32_t n0 = scnt[0], n1 = scnt[1];
  if (n0 > kLst || n1 > kLst) {  // uniform
    group_bucket_global(Rec12Src{rec, rank_base}, start, end, chunk_of, gkey, gmin, rep, special_min);
    return;
  }
  SubRec r2[2][kC4];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int j = 0; j < kC4; ++j) {
      const uint32_t i = threadIdx.x + j * kGroupThreads;
      r2[s2][j] = lst[s2 * kLst + min(i, kLst - 1)];
    }
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const uint32_t cnt = s2 ? n1 : n0;
    __syncthreads();  // the lists read (s2 = 0) / the previous lookups done
    for (uint32_t s = threadIdx.x; s < kPkSlots; s += kGroupThreads) tab[s] = 0ull;
    for (uint32_t s = threadIdx.x; s <= kPkCap; s += kGroupThreads) lmin[s] = 0xFFFFFFFFu;
    __syncthreads();
    uint32_t slot[kC4], owner[kC4];
    uint64_t mine[kC4];
    uint32_t pend = 0;
#pragma unroll
    for (int j = 0; j < kC4; ++j) {
      const uint64_t h = (static_cast<uint64_t>(r2[s2][j].hi) << 32) | r2[s2][j].lo;
      const uint32_t idx = threadIdx.x + j * kGroupThreads;
      mine[j] = (key_rest(h, 12) << 12) | ((idx + 1) & 0xFFFu);
      slot[j] = static_cast<uint32_t>((static_cast<uint64_t>(r2[s2][j].lo) * kPkSlots) >> 32);
      owner[j] = idx;
      if (idx < cnt) pend |= 1u << j;
    }
    const uint32_t live = pend;
    while (pend) {
      uint64_t prev[kC4];
#pragma unroll
      for (int j = 0; j < kC4; ++j)
        prev[j] = (pend >> j & 1u)
                      ? atomicCAS(reinterpret_cast<unsigned long long*>(&tab[slot[j]]), 0ull,
                                  static_cast<unsigned long long>(mine[j]))
                      : 0ull;
#pragma unroll
      for (int j = 0; j < kC4; ++j) {
        if (!(pend >> j & 1u)) continue;
        if (prev[j] == 0ull) {
          pend &= ~(1u << j);
        } else if ((prev[j] >> 12) == (mine[j] >> 12)) {
          owner[j] = static_cast<uint32_t>(prev[j] & 0xFFFu) - 1;
          pend &= ~(1u << j);
        } else {
          uint32_t st = 1u + 2u * static_cast<uint32_t>((r2[s2][j].hi >> 8) & 1023u);  // h bits [40, 50)
          st += (st % 3u == 0) ? 2u : 0u;
          st += (st % 5u == 0) ? 2u : 0u;
          st += (st % 3u == 0) ? 2u : 0u;
          const uint32_t sn = slot[j] + st;
          slot[j] = sn >= kPkSlots ? sn - kPkSlots : sn;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kC4; ++j)
      if (live >> j & 1u) atomicMin(&lmin[owner[j]], rank_base + r2[s2][j].row);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kC4; ++j) {
      if (!(live >> j & 1u)) continue;
      const uint32_t r = rank_base + r2[s2][j].row, f = lmin[owner[j]];
      if (chunk_of(r) != chunk_of(f)) rep[r2[s2][j].row] = f;
    }
  }
}

// group: kMode 0 product, 1 no rep writes, 2 loads only (records summed)
template <int kMode>
__global__ __launch_bounds__(kGroupThreads, 8) void k_group_var(const uint3* __restrict__ rec,
                                                                const uint32_t* __restrict__ offs,
                                                                ChunkOf chunk_of,
                                                                uint32_t* __restrict__ rep) {
  __shared__ uint64_t tab[kPkSlots];
  __shared__ uint32_t lmin[kPkCap + 1];
  constexpr int kP = (kPkCap + kGroupThreads) / kGroupThreads;
  const uint32_t start = offs[blockIdx.x], end = offs[blockIdx.x + 1];
  uint4 q[kP];
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const uint32_t i = start + threadIdx.x + j * kGroupThreads;
    if (i < end) {
      const uint3 v = rec[i];
      q[j] = make_uint4(v.x, v.y, v.z, v.z);
    } else {
      q[j] = make_uint4(0, 0, kPadRow, kPadRow);
    }
  }
  if constexpr (kMode == 2) {
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < kP; ++j) acc ^= q[j].x ^ q[j].y ^ q[j].z;
    if (acc == 0x12345678u) rep[0] = acc;
    return;
  }
  if constexpr (kMode != 3) {  // 3: timing probe without the table clear (wrong results)
    for (uint32_t s = threadIdx.x; s < kPkSlots; s += kGroupThreads) tab[s] = 0ull;
    for (uint32_t s = threadIdx.x; s <= kPkCap; s += kGroupThreads) lmin[s] = 0xFFFFFFFFu;
  }
  __syncthreads();
  uint32_t slot[kP], step[kP], owner[kP];
  uint64_t mine[kP];
  uint32_t pend = 0;
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const uint64_t h = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
    const uint32_t idx = threadIdx.x + j * kGroupThreads;
    mine[j] = (key_rest(h, kStageBits) << 12) | (idx + 1);
    slot[j] = static_cast<uint32_t>((static_cast<uint64_t>(static_cast<uint32_t>(h)) * kPkSlots) >> 32);
    // kMode 4: the probe step from h bits [32, 42) (bits 44-55 are the digit,
    // constant in a bucket: (h >> 40) & 1023 varies in 4 bits only)
    uint32_t st = 1u + 2u * static_cast<uint32_t>((h >> (kMode == 4 ? 32 : 40)) & 1023u);
    st += (st % 3u == 0) ? 2u : 0u;
    st += (st % 5u == 0) ? 2u : 0u;
    st += (st % 3u == 0) ? 2u : 0u;
    step[j] = st;
    owner[j] = idx;
    if (q[j].w != kPadRow) pend |= 1u << j;
  }
  const uint32_t live = pend;
  while (pend) {
    uint64_t prev[kP];
#pragma unroll
    for (int j = 0; j < kP; ++j)
      prev[j] = (pend >> j & 1u)
                    ? atomicCAS(reinterpret_cast<unsigned long long*>(&tab[slot[j]]), 0ull,
                                static_cast<unsigned long long>(mine[j]))
                    : 0ull;
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      if (!(pend >> j & 1u)) continue;
      if (prev[j] == 0ull) {
        pend &= ~(1u << j);
      } else if ((prev[j] >> 12) == (mine[j] >> 12)) {
        owner[j] = static_cast<uint32_t>(prev[j] & 0xFFFu) - 1;
        pend &= ~(1u << j);
      } else {
        const uint32_t sn = slot[j] + step[j];
        slot[j] = sn >= kPkSlots ? sn - kPkSlots : sn;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < kP; ++j)
    if (live >> j & 1u) atomicMin(&lmin[owner[j]], q[j].z);
  __syncthreads();
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    if (!(live >> j & 1u)) continue;
    const uint32_t r = q[j].z, f = lmin[owner[j]];
    if (chunk_of(r) != chunk_of(f)) {
      if constexpr (kMode == 0 || kMode == 4) rep[q[j].w] = f;
      else acc += f;
    }
  }
  if (kMode == 1 && acc == 0x12345678u) rep[0] = acc;
}

template <typename F>
float time_ms(F f, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  f();
  std::vector<float> v;
  for (int r = 0; r < reps; ++r) {
    (void)hipEventRecord(a, 0);
    f();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    v.push_back(ms);
  }
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

}  // namespace

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 12500000ull;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const GroupLayout L = group_layout(n);
  if (L.bits != kStageBits || L.cbits) {
    printf("n %llu: not the one-level 12-bit path\n", (unsigned long long)n);
    return 2;
  }
  uint64_t* key;
  uint8_t* has;
  uint32_t *rep0, *rep1, *sink;
  (void)hipMalloc(&key, 8 * n);
  (void)hipMalloc(&has, n);
  (void)hipMalloc(&rep0, 4 * n);
  (void)hipMalloc(&rep1, 4 * n);
  (void)hipMalloc(&sink, 64);
  k_rows<<<4096, 256>>>(key, has, n, n * 4 / 5);
  void* ws;
  (void)hipMalloc(&ws, L.total);
  uint8_t* w = static_cast<uint8_t*>(ws);
  uint3* rec = reinterpret_cast<uint3*>(w + L.rec);
  uint64_t* gkey = reinterpret_cast<uint64_t*>(w + L.gkey);
  uint32_t* gmin = reinterpret_cast<uint32_t*>(w + L.gmin);
  uint32_t* fine = reinterpret_cast<uint32_t*>(w + L.fine);
  uint32_t* fE = reinterpret_cast<uint32_t*>(w + L.fE);
  uint32_t* ftot = reinterpret_cast<uint32_t*>(w + L.ftot);
  uint32_t* fbase = reinterpret_cast<uint32_t*>(w + L.fbase);
  uint32_t* ovf = reinterpret_cast<uint32_t*>(w + L.ovf);
  const uint32_t P = kPartBlocks;
  const RowsIn in{key, has, nullptr, 0};
  const ChunkOf c = ChunkOf::make(100);
  GroupInput gi;
  gi.key = key;
  gi.valid = has;
  gi.n = n;
  (void)dedup_local_launch(gi, 100, rep0, true, ws, 0, nullptr);
  (void)hipDeviceSynchronize();
  std::vector<uint32_t> a(n), b(n);
  (void)hipMemcpy(a.data(), rep0, 4 * n, hipMemcpyDeviceToHost);

  auto scan = [&] { k_fine_scan<kPartBlocks, 1><<<kNb / 64, 1024>>>(fine, kNb, fE, ftot, ovf); };
  auto h0 = [&] {
    k_part_hist<RowsIn><<<P, kPartThreads, sizeof(uint32_t) * kNb>>>(in, n, kShardBits, kStageBits,
                                                                     0, fine, nullptr, true);
  };
  auto h1 = [&] { k_hist_var<1><<<P, kPartThreads>>>(key, has, n, fine, sink); };
  auto h2 = [&] { k_hist_var<3><<<P, kPartThreads>>>(key, has, n, fine, sink); };
  auto h3 = [&] { k_hist_var<2><<<P, kPartThreads>>>(key, has, n, fine, sink); };
  auto hv = [&] { k_hist_var<0><<<P, kPartThreads>>>(key, has, n, fine, sink); };
  auto s0 = [&] {
    k_part_scatter_ws<true><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase);
  };
  auto s1 = [&] {
    k_ws_var<false, true, 0><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase);
  };
  auto s2 = [&] {
    k_ws_var<true, false, 0><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase);
  };
  auto s3 = [&] {
    k_ws_var<true, true, 1><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase);
  };
  auto s4 = [&] {
    k_ws_var<true, true, 2><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase);
  };
  auto sv = [&] {
    k_ws_var<true, true, 0><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase);
  };
  auto s6 = [&] {
    k_ws_asm<true><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase);
  };
  auto s7 = [&] {
    k_ws_asm<false><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase);
  };
  auto s8 = [&] {
    k_ws_batched<true><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase);
  };
  auto s9 = [&] {
    k_ws_batched<false><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase);
  };
  auto hb = [&](uint32_t bits) {
    k_part_hist<RowsIn><<<P, kPartThreads, sizeof(uint32_t) << bits>>>(in, n, kShardBits, bits, 0,
                                                                      fine, nullptr, true);
    k_fine_scan<kPartBlocks, 1><<<(1u << bits) / 64, 1024>>>(fine, 1u << bits, fE, ftot, ovf);
  };
  auto g11 = [&] { k_ws_gen<11, 4, true><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase); };
  auto g11n = [&] { k_ws_gen<11, 4, false><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase); };
  auto g10 = [&] { k_ws_gen<10, 8, true><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase); };
  auto g10n = [&] { k_ws_gen<10, 8, false><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase); };
  auto g12 = [&] { k_ws_gen<12, 2, true><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase); };
  auto c12 = [&] { k_ws_coop<12, 2, true><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase); };
  auto c11 = [&] { k_ws_coop<11, 4, true><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase); };
  auto c11n = [&] { k_ws_coop<11, 4, false><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase); };
  auto c10 = [&] { k_ws_coop<10, 8, true><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase); };
  auto c10n = [&] { k_ws_coop<10, 8, false><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase); };
  auto d11 = [&] { k_ws_coop2<11, 4, 4, true><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase); };
  auto d11n = [&] { k_ws_coop2<11, 4, 4, false><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase); };
  auto d11r8 = [&] { k_ws_coop2<11, 4, 8, true><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase); };
  auto d12 = [&] { k_ws_coop2<12, 2, 4, true><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase); };
  auto d12r8 = [&] { k_ws_coop2<12, 2, 8, true><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase); };
  auto gr11 = [&] {
    k_group11<<<2048, kGroupThreads>>>(rec, 0, fbase, c, gkey, gmin, rep1);
  };
  auto gr11b = [&] {
    k_group11b<<<2048, kGroupThreads>>>(rec, 0, fbase, c, gkey, gmin, rep1);
  };
  auto gp0 = [&] { k_group_pers<false><<<512, kGroupThreads>>>(rec, 0, fbase, kNb, c, gkey, gmin, rep1); };
  auto gp1 = [&] { k_group_pers<true><<<512, kGroupThreads>>>(rec, 0, fbase, kNb, c, gkey, gmin, rep1); };
  uint32_t* d_err;
  (void)hipMalloc(&d_err, 4);
  (void)hipMemset(d_err, 0, 4);
  auto sa = [&] {
    k_ws_async<true><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase, d_err);
  };
  auto san = [&] {
    k_ws_async<false><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase, d_err);
  };
  auto gm1 = [&] { k_group_multi<1, true><<<kNb, kGroupThreads>>>(rec, 0, fbase, c, gkey, gmin, rep1); };
  auto gm2 = [&] { k_group_multi<2, false><<<kNb / 2, kGroupThreads>>>(rec, 0, fbase, c, gkey, gmin, rep1); };
  auto gm2i = [&] { k_group_multi<2, true><<<kNb / 2, kGroupThreads>>>(rec, 0, fbase, c, gkey, gmin, rep1); };
  auto gr11c = [&] {
    k_group11c<<<2048, kGroupThreads>>>(rec, 0, fbase, c, gkey, gmin, rep1);
  };
  auto g0 = [&] {
    k_bucket_group12_pk<<<kNb, kGroupThreads>>>(rec, 0, fbase, kStageBits, c, gkey, gmin, rep1);
  };
  auto g0v = [&] { k_group_var<0><<<kNb, kGroupThreads>>>(rec, fbase, c, rep1); };
  auto g1 = [&] { k_group_var<1><<<kNb, kGroupThreads>>>(rec, fbase, c, rep1); };
  auto g2 = [&] { k_group_var<2><<<kNb, kGroupThreads>>>(rec, fbase, c, rep1); };
  auto g4 = [&] { k_group_var<4><<<kNb, kGroupThreads>>>(rec, fbase, c, rep1); };


  // correctness of the product-equivalent copies (hv, sv, g0v)
  {
    (void)hipMemset(rep1, 0xFF, 4 * n);
    hv();
    scan();
    sv();
    g0v();
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(b.data(), rep1, 4 * n, hipMemcpyDeviceToHost);
    uint64_t bad = 0;
    for (uint64_t i = 0; i < n; ++i) bad += a[i] != b[i];
    printf("copies (hist/ws/group) vs product: %llu mismatches (%s)\n", (unsigned long long)bad,
           hipGetErrorString(hipGetLastError()));
    (void)hipMemset(rep1, 0xFF, 4 * n);
    h0();
    scan();
    s6();
    g0v();
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(b.data(), rep1, 4 * n, hipMemcpyDeviceToHost);
    bad = 0;
    for (uint64_t i = 0; i < n; ++i) bad += a[i] != b[i];
    printf("S6 asm-load scatter + group vs product: %llu mismatches (%s)\n", (unsigned long long)bad,
           hipGetErrorString(hipGetLastError()));
    (void)hipMemset(rep1, 0xFF, 4 * n);
    h0();
    scan();
    s8();
    g0v();
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(b.data(), rep1, 4 * n, hipMemcpyDeviceToHost);
    bad = 0;
    for (uint64_t i = 0; i < n; ++i) bad += a[i] != b[i];
    printf("S8 batched scatter + group vs product: %llu mismatches (%s)\n", (unsigned long long)bad,
           hipGetErrorString(hipGetLastError()));
    (void)hipMemset(rep1, 0xFF, 4 * n);
    h0();
    scan();
    k_ws_coop<12, 2, true><<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase);
    g0v();
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(b.data(), rep1, 4 * n, hipMemcpyDeviceToHost);
    bad = 0;
    for (uint64_t i = 0; i < n; ++i) bad += a[i] != b[i];
    printf("SC12 coop scatter + group vs product: %llu mismatches (%s)\n", (unsigned long long)bad,
           hipGetErrorString(hipGetLastError()));
    {
      // the 11-bit pipeline: hist (11 bits) + fine scan, 2-barrier scatter, k_group11
      (void)hipMemset(rep1, 0xFF, 4 * n);
      hb(11);
      d11();
      gr11();
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(b.data(), rep1, 4 * n, hipMemcpyDeviceToHost);
      bad = 0;
      for (uint64_t i = 0; i < n; ++i) bad += a[i] != b[i];
      printf("P11 11-bit pipeline vs product: %llu mismatches (%s)\n", (unsigned long long)bad,
             hipGetErrorString(hipGetLastError()));
      (void)hipMemset(rep1, 0xFF, 4 * n);
      hb(11);
      d11();
      gr11b();
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(b.data(), rep1, 4 * n, hipMemcpyDeviceToHost);
      bad = 0;
      for (uint64_t i = 0; i < n; ++i) bad += a[i] != b[i];
      printf("P11b 11-bit pipeline (two tables) vs product: %llu mismatches (%s)\n",
             (unsigned long long)bad, hipGetErrorString(hipGetLastError()));
      (void)hipMemset(rep1, 0xFF, 4 * n);
      hb(11);
      d11();
      gr11c();
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(b.data(), rep1, 4 * n, hipMemcpyDeviceToHost);
      bad = 0;
      for (uint64_t i = 0; i < n; ++i) bad += a[i] != b[i];
      printf("P11c 11-bit pipeline (LDS redistribution) vs product: %llu mismatches (%s)\n",
             (unsigned long long)bad, hipGetErrorString(hipGetLastError()));
    }
    {
      (void)hipMemset(rep1, 0xFF, 4 * n);
      h0();
      scan();
      sa();
      g0v();
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(b.data(), rep1, 4 * n, hipMemcpyDeviceToHost);
      bad = 0;
      for (uint64_t i = 0; i < n; ++i) bad += a[i] != b[i];
      uint32_t e = 0;
      (void)hipMemcpy(&e, d_err, 4, hipMemcpyDeviceToHost);
      printf("SA async scatter + group vs product: %llu mismatches, spin cap hit %u (%s)\n",
             (unsigned long long)bad, e, hipGetErrorString(hipGetLastError()));
    }
    for (int gg = 0; gg < 6; ++gg) {
      (void)hipMemset(rep1, 0xFF, 4 * n);
      h0();
      scan();
      s0();
      if (gg == 0) gp0(); else if (gg == 1) gp1(); else if (gg == 2) gm1(); else if (gg == 3) gm2(); else if (gg == 4) gm2i(); else g4();
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(b.data(), rep1, 4 * n, hipMemcpyDeviceToHost);
      bad = 0;
      for (uint64_t i = 0; i < n; ++i) bad += a[i] != b[i];
      printf("G%s group vs product: %llu mismatches (%s)\n",
             gg == 0 ? "P0" : gg == 1 ? "P1" : gg == 2 ? "M1" : gg == 3 ? "M2" : gg == 4 ? "M2i" : "4 (step bits)", (unsigned long long)bad,
             hipGetErrorString(hipGetLastError()));
    }
    for (int rr = 0; rr < 2; ++rr) {
      (void)hipMemset(rep1, 0xFF, 4 * n);
      h0();
      scan();
      if (rr == 0) d12(); else d12r8();
      g0v();
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(b.data(), rep1, 4 * n, hipMemcpyDeviceToHost);
      bad = 0;
      for (uint64_t i = 0; i < n; ++i) bad += a[i] != b[i];
      printf("SD12%s 2-barrier scatter + group vs product: %llu mismatches (%s)\n", rr ? "r8" : "",
             (unsigned long long)bad, hipGetErrorString(hipGetLastError()));
    }
  }
  struct V {
    const char* name;
    std::function<void()> f;
  };
  for (int r = 0; r < 2; ++r) {
    std::vector<V> hs = {{"H0 hist product", h0}, {"Hv hist copy (mix64)", hv},
                         {"H1 hist cheap hash", h1}, {"H3 hist raw digit", h3},
                         {"H2 hist loads only", h2}};
    for (auto& v : hs) printf("%-32s %.4f ms\n", v.name, time_ms(v.f, reps));
    // every scatter runs on the offsets of its own digit mode (a record
    // outside its bucket's counted region would write past the array)
    struct SV {
      const char* name;
      std::function<void()> hist, f;
    };
    std::vector<SV> ss = {{"S0 ws product", h0, s0},       {"Sv ws copy", h0, sv},
                          {"S1 ws no record stores", h0, s1}, {"S2 ws no rep init", h0, s2},
                          {"S3 ws cheap hash", h1, s3},     {"S4 ws raw digit", h3, s4},
                          {"S6 ws asm loads, counted waits", h0, s6},
                          {"S7 ws asm loads, no rec stores", h0, s7},
                          {"S8 ws batched LDS trips", h0, s8},
                          {"S9 ws batched, no rec stores", h0, s9},
                          {"SA ws async rounds", h0, sa},
                          {"SAn ws async, no rec stores", h0, san}};
    for (auto& v : ss) {
      v.hist();
      scan();
      printf("%-32s %.4f ms\n", v.name, time_ms(v.f, reps));
    }
    {
      struct GV {
        const char* name;
        uint32_t bits;
        std::function<void()> f;
      };
      std::vector<GV> gv = {{"SG12 generic 12 bits / 2 slots", 12, g12},
                            {"SG11 11 bits / 4 slots", 11, g11},
                            {"SG11n 11 bits / 4 slots, no stores", 11, g11n},
                            {"SG10 10 bits / 8 slots", 10, g10},
                            {"SG10n 10 bits / 8 slots, no stores", 10, g10n},
                            {"SC12 coop 12 bits / 2 slots", 12, c12},
                            {"SC11 coop 11 bits / 4 slots", 11, c11},
                            {"SC11n coop 11/4, no stores", 11, c11n},
                            {"SC10 coop 10 bits / 8 slots", 10, c10},
                            {"SC10n coop 10/8, no stores", 10, c10n},
                            {"SD11 2-barrier 11/4, 4 rows", 11, d11},
                            {"SD11n 2-barrier 11/4, no stores", 11, d11n},
                            {"SD11r8 2-barrier 11/4, 8 rows", 11, d11r8},
                            {"SD12 2-barrier 12/2, 4 rows", 12, d12},
                            {"SD12r8 2-barrier 12/2, 8 rows", 12, d12r8}};
      for (auto& v : gv) {
        hb(v.bits);
        printf("%-32s %.4f ms\n", v.name, time_ms(v.f, reps));
      }
    }
    hb(11);
    d11();
    printf("%-32s %.4f ms\n", "G11 group 11-bit buckets", time_ms(gr11, reps));
    printf("%-32s %.4f ms\n", "G11b group 11-bit, two tables", time_ms(gr11b, reps));
    printf("%-32s %.4f ms\n", "G11c group 11-bit, redistributed", time_ms(gr11c, reps));
    printf("%-32s %.4f ms\n", "P11c whole 11-bit (redistributed)",
           time_ms([&] { hb(11); d11(); gr11c(); }, reps));
    printf("%-32s %.4f ms\n", "P11b whole 11-bit (two tables)",
           time_ms([&] { hb(11); d11(); gr11b(); }, reps));
    printf("%-32s %.4f ms\n", "P11 whole 11-bit pipeline",
           time_ms([&] { hb(11); d11(); gr11(); }, reps));
    printf("%-32s %.4f ms\n", "P12 whole product pipeline",
           time_ms([&] { (void)dedup_local_launch(gi, 100, rep0, true, ws, 0, nullptr); }, reps));
    h0();
    scan();
    s0();
    std::vector<V> gs = {{"G0 group product", g0}, {"Gv group copy", g0v},
                         {"G1 group no rep writes", g1}, {"G2 group loads only", g2},
                         {"G4 group, step from h bits 32-41", g4},
                         {"GM1 1 bucket, lmin by records", gm1},
                         {"GM2 2 buckets per workgroup", gm2},
                         {"GM2i 2 buckets, lmin by records", gm2i},
                         {"GP0 persistent, targeted clear", gp0},
                         {"GP1 persistent + prefetch", gp1}};
    for (auto& v : gs) printf("%-32s %.4f ms\n", v.name, time_ms(v.f, reps));
  }
  printf("%s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
