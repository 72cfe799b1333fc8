// Experiment: the one-level bucket scatter with ALIGNED
// 32-byte pair writes.
//
// Finding that motivates it (profiles/r3/exp_xcd_scatter): sharing one run
// per (XCD, bucket) -- ~4096 open lines per XCD, well inside its L2 -- wrote
// as many bytes as the product (444 vs 389 MB), so the L2 does not merge a
// run's partial writes into whole lines; what counts is how many 32-B sectors
// each store touches.  The product's 24-B pairs of 12-B records at any
// 4-B alignment touch 1.5 sectors on average (391 MB for 200 MB), the 16-B
// path's 32-B pairs at 16-B alignment the same (1.4x).
// Here records are 16 B {h lo, h hi, rank, row} and every (block, bucket)
// region is padded to an even record count and starts at an even record
// index (k_fine_scan over counts rounded up to 2), so a flushed pair is ONE
// aligned 32-B sector, written by two adjacent lanes (coalesced).  A record
// arriving at a full slot goes to the BACK of its region (descending), so the
// pairs at the front stay aligned; the last staged record and a pad record
// (row ~0, skipped by the group kernel) close the region.
//   P0  product: 12-B records, staged 24-B pairs, k_bucket_group12
//   PK  product scatter + the packed-table group kernel (12-B records)
//   A2  aligned 16-B pairs + packed-table group kernel over 16-B records
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_scatter_align.hip -o build/exp_scatter_align
#include "../../spacedrive_amd/csrc/dedup.hip"

#include <stdio.h>

#include <algorithm>
#include <functional>
#include <vector>

using namespace sdgpu;

namespace {

constexpr uint32_t kNb = 1u << kStageBits;
constexpr uint32_t kPkCap = 4095;  // record index + 1 in 12 bits, 0 = empty slot
constexpr uint32_t kPad = 0xFFFFFFFFu;

__global__ void k_rows(uint64_t* key, uint8_t* has, uint64_t n, uint64_t distinct) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint64_t j = (i * 0x9E3779B1ull) % n;
    key[i] = row_hash((j % distinct) * 0x2545F4914F6CDD1Dull + 7);
    has[i] = (row_hash(i ^ 0x55ull) % 1000) != 0;
  }
}

// k_fine_scan over counts rounded up to even (one-level: kR = 1).
__global__ __launch_bounds__(1024) void k_fine_scan_pad2(const uint32_t* __restrict__ fine,
                                                         uint32_t nfine, uint32_t* __restrict__ E,
                                                         uint32_t* __restrict__ tot) {
  constexpr uint32_t kJ = kPartBlocks / 16;
  __shared__ uint32_t part[16][64];
  const uint32_t bi = threadIdx.x & 63u, jg = threadIdx.x >> 6;
  const uint32_t b = blockIdx.x * 64 + bi;
  uint32_t sj[kJ], local = 0;
#pragma unroll
  for (uint32_t k = 0; k < kJ; ++k) {
    const uint64_t j = jg * kJ + k;
    const uint32_t v = b < nfine ? (fine[j * nfine + b] + 1u) & ~1u : 0u;
    sj[k] = v;
    local += v;
  }
  part[jg][bi] = local;
  __syncthreads();
  uint32_t pre = 0, all = 0;
#pragma unroll
  for (uint32_t g = 0; g < 16; ++g) {
    const uint32_t v = part[g][bi];
    pre += g < jg ? v : 0u;
    all += v;
  }
  if (b >= nfine) return;
#pragma unroll
  for (uint32_t k = 0; k < kJ; ++k) {
    E[static_cast<uint64_t>(jg * kJ + k) * nfine + b] = pre;
    pre += sj[k];
  }
  if (jg == 0) tot[b] = all;
}

// Aligned-pair bucket scatter (rows in rank order: rank = rank_base + row).
__global__ __launch_bounds__(kPartThreads) void k_scatter_aligned(
    RowsIn in, uint64_t n, uint32_t skip, const uint32_t* __restrict__ fine,
    const uint32_t* __restrict__ E, const uint32_t* __restrict__ ftot, uint4* __restrict__ out,
    uint32_t* __restrict__ rep, uint32_t* __restrict__ fbase) {
  constexpr uint32_t nbins = kNb;
  __shared__ uint3 stage[nbins][2];
  __shared__ uint32_t front[nbins], back[nbins], fill[nbins];
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
    const uint32_t f0 = base + E[static_cast<uint64_t>(j) * nbins + b];
    front[b] = f0;
    back[b] = f0 + ((fine[static_cast<uint64_t>(j) * nbins + b] + 1u) & ~1u);
    fill[b] = 0;
    if (j == 0) fbase[b] = base;
    base += v[k];
  }
  if (j == 0 && t == 0) fbase[nbins] = total;
  __syncthreads();
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  constexpr int U = 2;
  constexpr uint64_t kStep = static_cast<uint64_t>(U) * kPartThreads;
  const uint32_t rb = in.rank_base;
  auto round = [&](const RowBatch<U>& q, uint64_t i0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = i0 + threadIdx.x + static_cast<uint64_t>(u) * kPartThreads;
      if (!q.in[u]) continue;
      rep[i] = in.rank_of(q, u);
      if (!in.valid_of(q, u)) continue;
      const uint64_t h = row_hash(in.key_of(q, u));
      const uint32_t b = digit_of(h, skip, kStageBits);
      const uint32_t row = in.row_of(q, u);
      const uint32_t sl = atomicAdd(&fill[b], 1u);
      if (sl < 2) {
        stage[b][sl] = make_uint3(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32), row);
      } else {  // slot full: the back of the region
        out[atomicSub(&back[b], 1u) - 1u] =
            make_uint4(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32), rb + row, row);
      }
    }
    lds_barrier();
    // flush: lanes 2m, 2m+1 write slot 0 / 1 of one bucket -> one aligned 32-B sector
    const uint32_t slot = threadIdx.x & 1u;
#pragma unroll
    for (uint32_t k = 0; k < 2 * nbins / kPartThreads; ++k) {
      const uint32_t b = (threadIdx.x >> 1) + k * (kPartThreads / 2);
      if (fill[b] >= 2) {
        const uint32_t p = front[b];
        const uint3 r = stage[b][slot];
        out[p + slot] = make_uint4(r.x, r.y, rb + r.z, r.z);
        if (slot == 0) {
          front[b] = p + 2;
          fill[b] = 0;
        }
      }
    }
    lds_barrier();
  };
  if (t0 < t1) {
    RowBatch<U> qa, qb;
    in.template load_many<U>(t0 + threadIdx.x, kPartThreads, t1, t0, qa);
    for (uint64_t i0 = t0;; i0 += 2 * kStep) {
      in.template load_many<U>(i0 + kStep + threadIdx.x, kPartThreads, t1, t0, qb);
      round(qa, i0);
      if (i0 + kStep >= t1) break;
      in.template load_many<U>(i0 + 2 * kStep + threadIdx.x, kPartThreads, t1, t0, qa);
      round(qb, i0 + kStep);
      if (i0 + 2 * kStep >= t1) break;
    }
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads) {
    uint32_t p = front[b];
    if (fill[b] == 1) {
      const uint3 r = stage[b][0];
      out[p++] = make_uint4(r.x, r.y, rb + r.z, r.z);
    }
    if (p < back[b]) out[p] = make_uint4(0u, 0u, kPad, kPad);  // pad to the even size
  }
}

// U0: the product's staged 12-B scatter with a FIXED number of store
// instructions per round (every store unconditional; lanes with nothing to
// store write a per-thread dummy slot behind the records).  Hypothesis: the
// product's conditional stores make the compiler wait for them (vmcnt counts
// loads and stores in order) before it may use the next round's prefetched
// rows, so each round waits out the store latency.
__global__ __launch_bounds__(kPartThreads) void k_scatter_fixed_stores(
    RowsIn in, uint64_t n, uint32_t skip, const uint32_t* __restrict__ offs,
    const uint32_t* __restrict__ ftot, uint3* __restrict__ out, uint32_t* __restrict__ rep,
    uint32_t* __restrict__ fbase, uint3* __restrict__ dummy, uint32_t* __restrict__ dummy_rep) {
  constexpr uint32_t nbins = kNb;
  __shared__ uint3 stage[nbins][2];
  __shared__ uint32_t fill[nbins], cur[nbins];
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
  __syncthreads();
  uint3* __restrict__ my_dummy = dummy + (static_cast<uint64_t>(blockIdx.x) * kPartThreads + t) * 2;
  uint32_t* __restrict__ my_dummy_rep = dummy_rep + static_cast<uint64_t>(blockIdx.x) * kPartThreads + t;
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  constexpr int U = 2;
  constexpr uint64_t kStep = static_cast<uint64_t>(U) * kPartThreads;
  auto round = [&](const RowBatch<U>& q, uint64_t i0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = i0 + threadIdx.x + static_cast<uint64_t>(u) * kPartThreads;
      const bool inr = q.in[u];
      const bool val = in.valid_of(q, u);  // implies inr
      *(inr ? rep + i : my_dummy_rep) = in.rank_of(q, u);
      const uint64_t h = row_hash(in.key_of(q, u));
      const uint32_t b = digit_of(h, skip, kStageBits);
      const uint3 rq = make_uint3(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32), in.row_of(q, u));
      uint32_t sl = 2, p = 0;
      if (val) {
        sl = atomicAdd(&fill[b], 1u);
        if (sl < 2) stage[b][sl] = rq;
        else p = atomicAdd(&cur[b], 1u);
      }
      *(val && sl >= 2 ? out + p : my_dummy) = rq;
    }
    lds_barrier();
#pragma unroll
    for (uint32_t k = 0; k < nbins / kPartThreads; ++k) {
      const uint32_t b = threadIdx.x + k * kPartThreads;
      const bool f = fill[b] >= 2;
      const uint32_t p = cur[b];
      uint3* dst = f ? out + p : my_dummy;
      dst[0] = stage[b][0];
      dst[1] = stage[b][1];
      if (f) {
        cur[b] = p + 2;
        fill[b] = 0;
      }
    }
    lds_barrier();
  };
  if (t0 < t1) {
    RowBatch<U> qa, qb;
    in.template load_many<U>(t0 + threadIdx.x, kPartThreads, t1, t0, qa);
    for (uint64_t i0 = t0;; i0 += 2 * kStep) {
      in.template load_many<U>(i0 + kStep + threadIdx.x, kPartThreads, t1, t0, qb);
      round(qa, i0);
      if (i0 + kStep >= t1) break;
      in.template load_many<U>(i0 + 2 * kStep + threadIdx.x, kPartThreads, t1, t0, qa);
      round(qb, i0 + kStep);
      if (i0 + 2 * kStep >= t1) break;
    }
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads)
    for (uint32_t k = 0; k < fill[b]; ++k) out[cur[b] + k] = stage[b][k];
}

// W: warp-specialised staged scatter (implicit rank).  Waves 0-7 only LOAD and
// stage (their next rows are prefetched two rounds ahead and they never
// store, so their waits cover loads only); waves 8-15 only STORE: the full
// pairs, the rows that met a full slot (an LDS overflow list) and rep = rank
// of the round's rows (computed, no load).  Two barriers per round.
constexpr uint32_t kWProd = 512;  // producer threads
constexpr int kWU = 4;            // rows per producer thread per round
__global__ __launch_bounds__(kPartThreads) void k_scatter_warpspec(
    RowsIn in, uint64_t n, uint32_t skip, const uint32_t* __restrict__ offs,
    const uint32_t* __restrict__ ftot, uint3* __restrict__ out, uint32_t* __restrict__ rep,
    uint32_t* __restrict__ fbase) {
  constexpr uint32_t nbins = kNb;
  constexpr uint32_t kRound = kWProd * kWU;  // 2048 rows
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
  if (t < kWProd) {
    // producers
    RowBatch<kWU> qa, qb;
    in.template load_many<kWU>(t0 + t, kWProd, t1, t0, qa);
    in.template load_many<kWU>(t0 + kRound + t, kWProd, t1, t0, qb);
    auto stage_round = [&](const RowBatch<kWU>& q) {
#pragma unroll
      for (int u = 0; u < kWU; ++u) {
        if (!in.valid_of(q, u)) continue;
        const uint64_t h = row_hash(in.key_of(q, u));
        const uint32_t b = digit_of(h, skip, kStageBits);
        const uint3 rq = make_uint3(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32), in.row_of(q, u));
        const uint32_t sl = atomicAdd(&fill[b], 1u);
        if (sl < 2) stage[b][sl] = rq;
        else ovf[atomicAdd(&ovf_n, 1u)] = rq;
      }
    };
    // per round exactly the consumers' three barriers: A (staged), M, B (flushed)
    for (uint32_t r = 0; r < rounds; r += 2) {
      stage_round(qa);
      lds_barrier();  // A
      in.template load_many<kWU>(t0 + (r + 2) * static_cast<uint64_t>(kRound) + t, kWProd, t1, t0, qa);
      lds_barrier();  // M
      lds_barrier();  // B
      if (r + 1 >= rounds) break;
      stage_round(qb);
      lds_barrier();  // A
      in.template load_many<kWU>(t0 + (r + 3) * static_cast<uint64_t>(kRound) + t, kWProd, t1, t0, qb);
      lds_barrier();  // M
      lds_barrier();  // B
    }
  } else {
    // consumers
    const uint32_t c = t - kWProd;
    for (uint32_t r = 0; r < rounds; ++r) {
      lds_barrier();  // A
      const uint64_t r0 = t0 + static_cast<uint64_t>(r) * kRound;
#pragma unroll
      for (uint32_t u = 0; u < kRound / kWProd; ++u) {  // rep = rank of the round's rows
        const uint64_t i = r0 + c + u * kWProd;
        if (i < t1) rep[i] = in.rank_base + static_cast<uint32_t>(i);
      }
#pragma unroll
      for (uint32_t k = 0; k < nbins / kWProd; ++k) {
        const uint32_t b = c + k * kWProd;
        if (fill[b] >= 2) {
          const uint32_t p = cur[b];
          out[p] = stage[b][0];
          out[p + 1] = stage[b][1];
          cur[b] = p + 2;
          fill[b] = 0;
        }
      }
      const uint32_t no = ovf_n;
      lds_barrier();  // M: every consumer read ovf_n and the fills; overflow rows next
      for (uint32_t o = c; o < no; o += kWProd) {
        const uint3 rq = ovf[o];
        const uint32_t b = digit_of((static_cast<uint64_t>(rq.y) << 32) | rq.x, skip, kStageBits);
        out[atomicAdd(&cur[b], 1u)] = rq;
      }
      if (c == 0) ovf_n = 0;
      lds_barrier();  // B
    }
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads)
    for (uint32_t k = 0; k < fill[b]; ++k) out[cur[b] + k] = stage[b][k];
}

// AW: warp-specialised AND aligned: 16-B records in even-padded (block,
// bucket) regions, pairs flushed by two adjacent consumer lanes as one aligned
// 32-B sector, rows that met a full slot to the back of their region (through
// a 1024-entry LDS list; a producer writes directly only when the list is
// full -- rare, so its loads' waits stay store-free in the usual round).
constexpr uint32_t kAwOvf = 1024;
__global__ __launch_bounds__(kPartThreads) void k_scatter_aw(
    RowsIn in, uint64_t n, uint32_t skip, const uint32_t* __restrict__ fine,
    const uint32_t* __restrict__ E, const uint32_t* __restrict__ ftot, uint4* __restrict__ out,
    uint32_t* __restrict__ rep, uint32_t* __restrict__ fbase) {
  constexpr uint32_t nbins = kNb;
  constexpr uint32_t kRound = kWProd * kWU;  // 2048 rows
  __shared__ uint3 stage[nbins][2];
  __shared__ uint32_t fill[nbins], front[nbins], back[nbins];
  __shared__ uint3 ovf[kAwOvf];
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
    const uint32_t f0 = base + E[static_cast<uint64_t>(j) * nbins + b];
    front[b] = f0;
    back[b] = f0 + ((fine[static_cast<uint64_t>(j) * nbins + b] + 1u) & ~1u);
    fill[b] = 0;
    if (j == 0) fbase[b] = base;
    base += v[k];
  }
  if (j == 0 && t == 0) fbase[nbins] = total;
  if (t == 0) ovf_n = 0;
  __syncthreads();
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  const uint32_t rb = in.rank_base;
  const uint32_t rounds = t1 > t0 ? static_cast<uint32_t>((t1 - t0 + kRound - 1) / kRound) : 0u;
  if (t < kWProd) {
    RowBatch<kWU> qa, qb;
    in.template load_many<kWU>(t0 + t, kWProd, t1, t0, qa);
    in.template load_many<kWU>(t0 + kRound + t, kWProd, t1, t0, qb);
    auto stage_round = [&](const RowBatch<kWU>& q) {
#pragma unroll
      for (int u = 0; u < kWU; ++u) {
        if (!in.valid_of(q, u)) continue;
        const uint64_t h = row_hash(in.key_of(q, u));
        const uint32_t b = digit_of(h, skip, kStageBits);
        const uint32_t row = in.row_of(q, u);
        const uint32_t sl = atomicAdd(&fill[b], 1u);
        if (sl < 2) {
          stage[b][sl] = make_uint3(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32), row);
        } else {
          const uint32_t o = atomicAdd(&ovf_n, 1u);
          if (o < kAwOvf)
            ovf[o] = make_uint3(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32), row);
          else  // list full (many rows of one key in a round): directly
            out[atomicSub(&back[b], 1u) - 1u] =
                make_uint4(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32), rb + row, row);
        }
      }
    };
    for (uint32_t r = 0; r < rounds; r += 2) {
      stage_round(qa);
      lds_barrier();  // A
      in.template load_many<kWU>(t0 + (r + 2) * static_cast<uint64_t>(kRound) + t, kWProd, t1, t0, qa);
      lds_barrier();  // M
      lds_barrier();  // B
      if (r + 1 >= rounds) break;
      stage_round(qb);
      lds_barrier();  // A
      in.template load_many<kWU>(t0 + (r + 3) * static_cast<uint64_t>(kRound) + t, kWProd, t1, t0, qb);
      lds_barrier();  // M
      lds_barrier();  // B
    }
  } else {
    const uint32_t c = t - kWProd, slot = c & 1u;
    for (uint32_t r = 0; r < rounds; ++r) {
      lds_barrier();  // A
      const uint64_t r0 = t0 + static_cast<uint64_t>(r) * kRound;
#pragma unroll
      for (uint32_t u = 0; u < kRound / kWProd; ++u) {
        const uint64_t i = r0 + c + u * kWProd;
        if (i < t1) rep[i] = rb + static_cast<uint32_t>(i);
      }
      // lanes 2m, 2m+1: slot 0 / 1 of one bucket -> one aligned 32-B sector
#pragma unroll
      for (uint32_t k = 0; k < 2 * nbins / kWProd; ++k) {
        const uint32_t b = (c >> 1) + k * (kWProd / 2);
        if (fill[b] >= 2) {
          const uint32_t p = front[b];
          const uint3 rr = stage[b][slot];
          out[p + slot] = make_uint4(rr.x, rr.y, rb + rr.z, rr.z);
        }
      }
      const uint32_t no = min(ovf_n, kAwOvf);
      lds_barrier();  // M: every consumer has read the fills, front and ovf_n
#pragma unroll
      for (uint32_t k = 0; k < nbins / kWProd; ++k) {
        const uint32_t b = c + k * kWProd;
        if (fill[b] >= 2) {
          front[b] += 2;
          fill[b] = 0;
        }
      }
      for (uint32_t o = c; o < no; o += kWProd) {
        const uint3 rr = ovf[o];
        const uint32_t b = digit_of((static_cast<uint64_t>(rr.y) << 32) | rr.x, skip, kStageBits);
        out[atomicSub(&back[b], 1u) - 1u] = make_uint4(rr.x, rr.y, rb + rr.z, rr.z);
      }
      if (c == 0) ovf_n = 0;
      lds_barrier();  // B
    }
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads) {
    uint32_t p = front[b];
    if (fill[b] == 1) {
      const uint3 rr = stage[b][0];
      out[p++] = make_uint4(rr.x, rr.y, rb + rr.z, rr.z);
    }
    if (p < back[b]) out[p] = make_uint4(0u, 0u, kPad, kPad);
  }
}

// h without its `bits` digit bits [56 - bits, 56): 64 - bits bits
__device__ __forceinline__ uint64_t key_rest(uint64_t h, uint32_t bits) {
  const uint32_t lo = 56 - bits;
  return (h & ((1ull << lo) - 1)) | ((h >> 56) << lo);
}

// Group-by with the packed 8-B LDS table (see exp_group_packed); RecT = uint3
// {h lo, h hi, row} (rank = rank_base + row) or uint4 {h lo, h hi, rank, row}
// with pad records (row ~0) skipped.  Buckets above 4095 records: global table.
template <typename RecT, uint32_t kSlots>
__global__ __launch_bounds__(kGroupThreads, 8) void k_group_packed(
    const RecT* __restrict__ rec, uint32_t rank_base, const uint32_t* __restrict__ offs,
    uint32_t bits, ChunkOf chunk_of, uint64_t* __restrict__ gkey, uint32_t* __restrict__ gmin,
    uint32_t* __restrict__ rep) {
  constexpr bool k16 = std::is_same<RecT, uint4>::value;
  __shared__ uint64_t tab[kSlots];
  __shared__ uint32_t lmin[kPkCap + 1];
  constexpr int kP = (kPkCap + kGroupThreads) / kGroupThreads;
  const uint32_t b = blockIdx.x;
  const uint32_t start = offs[b], end = offs[b + 1], m = end - start;
  auto get = [&](uint32_t i) -> uint4 {
    if constexpr (k16) {
      return rec[i];
    } else {
      const uint3 v = rec[i];
      return make_uint4(v.x, v.y, rank_base + v.z, v.z);
    }
  };
  if (m > kPkCap) {
    __shared__ uint32_t special_min;
    uint64_t tsize = 1;
    while (tsize * 2 <= 4ull * m) tsize *= 2;
    uint64_t* tk = gkey + 4ull * start;
    uint32_t* tm = gmin + 4ull * start;
    for (uint64_t s = threadIdx.x; s < tsize; s += kGroupThreads) {
      tk[s] = kEmpty;
      tm[s] = 0xFFFFFFFFu;
    }
    if (threadIdx.x == 0) special_min = 0xFFFFFFFFu;
    __syncthreads();
    for (uint32_t i = start + threadIdx.x; i < end; i += kGroupThreads) {
      const uint4 qq = get(i);
      if (qq.w == kPad) continue;
      const uint64_t k = (static_cast<uint64_t>(qq.y) << 32) | qq.x;
      if (k == kEmpty) {
        atomicMin(&special_min, qq.z);
        continue;
      }
      uint64_t h = k & (tsize - 1);
      for (;;) {
        const uint64_t prev = atomicCAS(reinterpret_cast<unsigned long long*>(&tk[h]),
                                        static_cast<unsigned long long>(kEmpty),
                                        static_cast<unsigned long long>(k));
        if (prev == kEmpty || prev == k) {
          atomicMin(&tm[h], qq.z);
          break;
        }
        h = (h + 1) & (tsize - 1);
      }
    }
    __syncthreads();
    for (uint32_t i = start + threadIdx.x; i < end; i += kGroupThreads) {
      const uint4 qq = get(i);
      if (qq.w == kPad) continue;
      const uint64_t k = (static_cast<uint64_t>(qq.y) << 32) | qq.x;
      uint32_t f;
      if (k == kEmpty) {
        f = special_min;
      } else {
        uint64_t h = k & (tsize - 1);
        while (__hip_atomic_load(&tk[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != k)
          h = (h + 1) & (tsize - 1);
        f = __hip_atomic_load(&tm[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (chunk_of(qq.z) != chunk_of(f)) rep[qq.w] = f;
    }
    return;
  }
  uint4 q[kP];
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const uint32_t i = start + threadIdx.x + j * kGroupThreads;
    q[j] = i < end ? get(i) : make_uint4(0, 0, kPad, kPad);
  }
  for (uint32_t s = threadIdx.x; s < kSlots; s += kGroupThreads) tab[s] = 0ull;
  for (uint32_t s = threadIdx.x; s <= kPkCap; s += kGroupThreads) lmin[s] = 0xFFFFFFFFu;
  __syncthreads();
  uint32_t slot[kP], step[kP], owner[kP];
  uint64_t mine[kP];
  uint32_t pend = 0;
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const uint64_t h = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
    const uint32_t idx = threadIdx.x + j * kGroupThreads;
    mine[j] = (key_rest(h, bits) << 12) | (idx + 1);
    slot[j] = static_cast<uint32_t>((static_cast<uint64_t>(static_cast<uint32_t>(h)) * kSlots) >> 32);
    uint32_t st = 1u + 2u * static_cast<uint32_t>((h >> 40) & 1023u);
    while (st % 3u == 0 || st % 5u == 0) st += 2;
    step[j] = st % kSlots;
    owner[j] = idx;
    if (q[j].w != kPad) pend |= 1u << j;
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
        const uint32_t s = slot[j] + step[j];
        slot[j] = s >= kSlots ? s - kSlots : s;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < kP; ++j)
    if (live >> j & 1u) atomicMin(&lmin[owner[j]], q[j].z);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    if (!(live >> j & 1u)) continue;
    const uint32_t r = q[j].z, f = lmin[owner[j]];
    if (chunk_of(r) != chunk_of(f)) rep[q[j].w] = f;
  }
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
  uint32_t *rep0, *rep1;
  uint4* rec16;
  (void)hipMalloc(&key, 8 * n);
  (void)hipMalloc(&has, n);
  (void)hipMalloc(&rep0, 4 * n);
  (void)hipMalloc(&rep1, 4 * n);
  (void)hipMalloc(&rec16, 16 * (n + 2ull * kNb * kPartBlocks));
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
  const size_t lds = sizeof(uint32_t) << kStageBits;
  GroupInput gi;
  gi.key = key;
  gi.valid = has;
  gi.n = n;
  (void)dedup_local_launch(gi, 100, rep0, true, ws, 0, nullptr);
  (void)hipDeviceSynchronize();
  std::vector<uint32_t> a(n), b(n);
  (void)hipMemcpy(a.data(), rep0, 4 * n, hipMemcpyDeviceToHost);
  auto hist = [&] {
    k_part_hist<RowsIn><<<P, kPartThreads, lds>>>(in, n, kShardBits, kStageBits, 0, fine, nullptr, true);
  };
  auto p0_scan = [&] { k_fine_scan<kPartBlocks, 1><<<kNb / 64, 1024>>>(fine, kNb, fE, ftot, ovf); };
  auto p0_scatter = [&] {
    k_part_scatter_rec_staged<RowsIn, true, kStageBits, 2, 2, true><<<P, kPartThreads>>>(
        in, n, kShardBits, fE, reinterpret_cast<uint4*>(rec), rep1, nullptr, 0, ftot, fbase);
  };
  auto p0_group = [&] { k_bucket_group12<<<kNb, kGroupThreads>>>(rec, 0, fbase, c, gkey, gmin, rep1); };
  auto pk_group = [&] {
    k_group_packed<uint3, 7680><<<kNb, kGroupThreads>>>(rec, 0, fbase, kStageBits, c, gkey, gmin, rep1);
  };
  auto a2_scan = [&] { k_fine_scan_pad2<<<kNb / 64, 1024>>>(fine, kNb, fE, ftot); };
  auto a2_scatter = [&] {
    k_scatter_aligned<<<P, kPartThreads>>>(in, n, kShardBits, fine, fE, ftot, rec16, rep1, fbase);
  };
  auto a2_group = [&] {
    k_group_packed<uint4, 7680><<<kNb, kGroupThreads>>>(rec16, 0, fbase, kStageBits, c, gkey, gmin, rep1);
  };
  uint3* dummy;
  uint32_t* dummy_rep;
  (void)hipMalloc(&dummy, 12ull * 2 * kPartThreads * P);
  (void)hipMalloc(&dummy_rep, 4ull * kPartThreads * P);
  auto u0_scatter = [&] {
    k_scatter_fixed_stores<<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase, dummy,
                                                dummy_rep);
  };
  auto aw_scatter = [&] {
    k_scatter_aw<<<P, kPartThreads>>>(in, n, kShardBits, fine, fE, ftot, rec16, rep1, fbase);
  };
  auto w_scatter = [&] {
    k_scatter_warpspec<<<P, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1, fbase);
  };
  struct V {
    const char* name;
    std::function<void()> scan, scatter, group;
  };
  std::vector<V> vs = {{"P0 product 12-B pairs + group12", p0_scan, p0_scatter, p0_group},
                       {"PK product scatter + packed group", p0_scan, p0_scatter, pk_group},
                       {"A2 aligned 16-B pairs + packed group", a2_scan, a2_scatter, a2_group},
                       {"U0 fixed-count stores + group12", p0_scan, u0_scatter, p0_group},
                       {"W  warp-specialised + group12", p0_scan, w_scatter, p0_group},
                       {"WP warp-specialised + packed group", p0_scan, w_scatter, pk_group},
                       {"AW aligned warp-spec. + packed group", a2_scan, aw_scatter, a2_group}};
  for (auto& v : vs) {
    (void)hipMemset(rep1, 0xFF, 4 * n);
    hist();
    v.scan();
    v.scatter();
    v.group();
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(b.data(), rep1, 4 * n, hipMemcpyDeviceToHost);
    uint64_t bad = 0;
    for (uint64_t i = 0; i < n; ++i) bad += a[i] != b[i];
    printf("%-40s mismatches vs product: %llu (%s)\n", v.name, (unsigned long long)bad,
           hipGetErrorString(hipGetLastError()));
  }
  for (int r = 0; r < 2; ++r)
    for (auto& v : vs) {
      const float whole = time_ms([&] { hist(); v.scan(); v.scatter(); v.group(); }, reps);
      hist();
      v.scan();
      const float sc = time_ms(v.scatter, reps);
      const float gr = time_ms(v.group, reps);
      printf("%-40s whole %.4f ms  scatter %.4f ms  group %.4f ms\n", v.name, whole, sc, gr);
    }
  return 0;
}
