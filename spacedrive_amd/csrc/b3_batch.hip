// K1: batched BLAKE3 over many short messages -- the sampled cas_id path.
//
// Replaces generate_cas_id's hashing (/root/reference/core/src/object/cas.rs:24-61)
// as run for every orphan file_path by identifier_job_step
// (/root/reference/core/src/object/file_identifier/mod.rs:107-134), where the
// reference hashes <=100 files per step, one after another, on one CPU thread.
//
// Input: a device arena of cas messages M_i = size_le(8 B) || windows
// (<= 102 408 B each, 16-B aligned offsets), packed by the host or the synthetic
// generator.  Decomposition (DESIGN.md "K1"):
//   plan   : n_chunks per message, exclusive scan -> chunk_base, chunk -> message map
//   chunks : ONE LANE PER 1 KiB CHUNK over the flattened chunk list of the whole
//            batch (full 64-lane utilisation whatever the file sizes are); a
//            single-chunk message finishes here with the ROOT flag
//   parents: ONE LANE PER MESSAGE folds that message's chunk CVs pairwise
//            (left-complete tree = BLAKE3 tree), ROOT on the last parent.
// Every compression is done by exactly one lane: no log-depth idle tree phase.
#include <errno.h>
#include <stdlib.h>

#include <algorithm>

#include "b3_device.hpp"
#include "internal.hpp"
#include "scan_device.hpp"

namespace sdgpu {

namespace {

constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void k_plan(const uint64_t* __restrict__ off,
                                                   const uint32_t* __restrict__ len, uint32_t n,
                                                   uint32_t max_len,
                                                   uint32_t* __restrict__ n_chunks,
                                                   int32_t* __restrict__ status,
                                                   uint32_t out_words, uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const uint32_t l = len[i];
  const bool ok = l <= max_len && (off[i] & 15u) == 0;
  n_chunks[i] = ok ? (l <= B3_CHUNK_LEN ? 1u : (l + B3_CHUNK_LEN - 1) / B3_CHUNK_LEN) : 0u;
  if (status) status[i] = ok ? 0 : -EINVAL;
  if (!ok)
    for (uint32_t w = 0; w < out_words; ++w) out[i * out_words + w] = 0u;
}

// chunk -> message map; one wave per message, lanes stride its chunks.
__global__ __launch_bounds__(kThreads) void k_fill_map(const uint32_t* __restrict__ n_chunks,
                                                       const uint32_t* __restrict__ chunk_base,
                                                       uint32_t n,
                                                       uint32_t* __restrict__ chunk_msg) {
  const uint32_t wave = (blockIdx.x * kThreads + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63u;
  if (wave >= n) return;
  const uint32_t b = chunk_base[wave], c = n_chunks[wave];
  for (uint32_t j = lane; j < c; j += 64) chunk_msg[b + j] = wave;
}

// One lane per chunk (grid-stride over the flattened chunk list).
// K1 variant for A/B runs in one process.  SDGPU_K1_VARIANT unset or 3: the
// persistent longest-first queue (default; 5 waves/SIMD, 4: the same pinned
// to 6 waves/SIMD with a few bytes of spill); 2: unit/message lanes over a
// fixed grid; 0: chunk-lane + parent-lane scheme; 1: the same with
// software-pipelined block loads.
int k1_variant() {
  const char* v = getenv("SDGPU_K1_VARIANT");
  return v ? atoi(v) : 3;
}

template <bool kPipelined>
__global__ __launch_bounds__(kThreads) void k_chunks(
    const uint8_t* __restrict__ arena, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, const uint32_t* __restrict__ chunk_msg,
    const uint32_t* __restrict__ chunk_base, const uint32_t* __restrict__ d_total,
    uint32_t* __restrict__ cvs, uint32_t out_words, uint32_t* __restrict__ out) {
  const uint32_t total = *d_total;
  const uint32_t stride = gridDim.x * kThreads;
  for (uint32_t t = blockIdx.x * kThreads + threadIdx.x; t < total; t += stride) {
    const uint32_t m = chunk_msg[t];
    const uint32_t j = t - chunk_base[m];
    const uint32_t l = len[m];
    const bool single = l <= B3_CHUNK_LEN;
    const uint32_t clen = min(B3_CHUNK_LEN, l - j * B3_CHUNK_LEN);
    uint32_t cv[8];
    if (kPipelined)
      b3_chunk_pipelined(arena + off[m] + static_cast<uint64_t>(j) * B3_CHUNK_LEN, clen,
                                j, single ? B3_ROOT : 0u, cv);
    else
      b3_chunk(arena + off[m] + static_cast<uint64_t>(j) * B3_CHUNK_LEN, clen, j,
                      single ? B3_ROOT : 0u, cv);
    if (single) {
      for (uint32_t w = 0; w < out_words; ++w) out[m * out_words + w] = cv[w];
    } else {
      uint4* dst = reinterpret_cast<uint4*>(cvs + static_cast<uint64_t>(t) * 8);
      dst[0] = make_uint4(cv[0], cv[1], cv[2], cv[3]);
      dst[1] = make_uint4(cv[4], cv[5], cv[6], cv[7]);
    }
  }
}

__device__ __forceinline__ void load_cv(const uint32_t* p, uint32_t cv[8]) {
  const uint4 a = reinterpret_cast<const uint4*>(p)[0];
  const uint4 b = reinterpret_cast<const uint4*>(p)[1];
  cv[0] = a.x; cv[1] = a.y; cv[2] = a.z; cv[3] = a.w;
  cv[4] = b.x; cv[5] = b.y; cv[6] = b.z; cv[7] = b.w;
}

__device__ __forceinline__ void store_cv(uint32_t* p, const uint32_t cv[8]) {
  reinterpret_cast<uint4*>(p)[0] = make_uint4(cv[0], cv[1], cv[2], cv[3]);
  reinterpret_cast<uint4*>(p)[1] = make_uint4(cv[4], cv[5], cv[6], cv[7]);
}

// Parent lanes are ordered by chunk count (descending) so that the 64 lanes of
// a wave fold equally long trees: bin = 127 - min(n_chunks, 127), messages
// with fewer than 2 chunks are left out.  Block-aggregated counting sort.
constexpr uint32_t kBins = 128;

__device__ __forceinline__ uint32_t parent_bin(uint32_t nch) {
  return kBins - 1 - min(nch, kBins - 1);
}

__global__ __launch_bounds__(kThreads) void k_bin_hist(const uint32_t* __restrict__ n_chunks,
                                                       uint32_t n, uint32_t* __restrict__ bins) {
  __shared__ uint32_t h[kBins];
  if (threadIdx.x < kBins) h[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads) {
    const uint32_t c = n_chunks[i];
    if (c >= 2) atomicAdd(&h[parent_bin(c)], 1u);
  }
  __syncthreads();
  if (threadIdx.x < kBins && h[threadIdx.x]) atomicAdd(&bins[threadIdx.x], h[threadIdx.x]);
}

// bins[0..kBins) -> exclusive offsets (used as cursors), bins[kBins] = total.
__global__ void k_bin_scan(uint32_t* __restrict__ bins) {
  if (threadIdx.x != 0) return;
  uint32_t run = 0;
  for (uint32_t b = 0; b < kBins; ++b) {
    const uint32_t v = bins[b];
    bins[b] = run;
    run += v;
  }
  bins[kBins] = run;
}

__global__ __launch_bounds__(kThreads) void k_bin_scatter(const uint32_t* __restrict__ n_chunks,
                                                          uint32_t n, uint32_t* __restrict__ bins,
                                                          uint32_t* __restrict__ order) {
  __shared__ uint32_t h[kBins], base[kBins];
  for (uint32_t i0 = blockIdx.x * kThreads; i0 < n; i0 += gridDim.x * kThreads) {
    if (threadIdx.x < kBins) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t i = i0 + threadIdx.x;
    const uint32_t c = i < n ? n_chunks[i] : 0u;
    uint32_t local = 0, b = 0;
    if (c >= 2) {
      b = parent_bin(c);
      local = atomicAdd(&h[b], 1u);
    }
    __syncthreads();
    if (threadIdx.x < kBins && h[threadIdx.x])
      base[threadIdx.x] = atomicAdd(&bins[threadIdx.x], h[threadIdx.x]);
    __syncthreads();
    if (c >= 2) order[base[b] + local] = i;
    __syncthreads();
  }
}

// One lane per multi-chunk message: pairwise fold of its chunk CVs, in place.
// Pairwise merging with the odd node carried up builds exactly BLAKE3's
// left-complete tree; the last merge (two nodes left) carries ROOT.  The next
// pair is loaded before the current one is compressed.
__global__ __launch_bounds__(kThreads) void k_parents(const uint32_t* __restrict__ n_chunks,
                                                      const uint32_t* __restrict__ chunk_base,
                                                      const uint32_t* __restrict__ order,
                                                      const uint32_t* __restrict__ bins,
                                                      uint32_t n, uint32_t* __restrict__ cvs,
                                                      uint32_t out_words,
                                                      uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= bins[kBins]) return;
  const uint32_t m = order[i];
  uint32_t cnt = n_chunks[m];
  uint32_t* c = cvs + static_cast<uint64_t>(chunk_base[m]) * 8;
  uint32_t l[8], r[8], p[8], ln[8], rn[8];
  while (cnt > 2) {
    const uint32_t half = cnt >> 1;
    load_cv(c, l);
    load_cv(c + 8, r);
    for (uint32_t k = 0; k < half; ++k) {
      if (k + 1 < half) {
        load_cv(c + 16 * (k + 1), ln);
        load_cv(c + 16 * (k + 1) + 8, rn);
      }
      b3_parent(p, l, r, 0u);
      store_cv(c + 8 * k, p);
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        l[w] = ln[w];
        r[w] = rn[w];
      }
    }
    if (cnt & 1u) {
      load_cv(c + 8 * (cnt - 1), l);
      store_cv(c + 8 * half, l);
    }
    cnt = half + (cnt & 1u);
  }
  load_cv(c, l);
  load_cv(c + 8, r);
  b3_parent(p, l, r, B3_ROOT);
  for (uint32_t w = 0; w < out_words; ++w) out[m * out_words + w] = p[w];
}

// ============================================================================
// K1 v2: 4-chunk units + one lane per message for the ragged rest.
//
// A message of n > 4 chunks has q = floor(full_chunks / 4) aligned units of 4
// FULL chunks.  UNIT lanes (grid-stride over all units of the batch) hash the
// 4 chunks and merge them in-lane: P(P(c0,c1), P(c2,c3)) -- 67 compressions,
// identical for every lane, no ragged chunk anywhere.  A unit is a complete
// level-2 subtree of BLAKE3's tree.  MESSAGE lanes (one per message, ordered
// by remaining work so waves are uniform) hash the 0..4 remaining chunks
// [4q, n) into one level-2 node and fold the q + 1 level-2 nodes pairwise
// (ROOT on the last compression).  Messages of <= 4 chunks are done entirely
// by their message lane.  For a sampled cas message (56 full chunks + 8 bytes)
// that is 14 unit lanes and 15 compressions on the message lane instead of
// 56 serial parents.
// ============================================================================

__device__ __forceinline__ uint32_t n_chunks_of(uint32_t len) {
  return len <= B3_CHUNK_LEN ? 1u : (len + B3_CHUNK_LEN - 1) / B3_CHUNK_LEN;
}

__device__ __forceinline__ uint32_t units_of(uint32_t len) {
  return n_chunks_of(len) > 4 ? (len / B3_CHUNK_LEN) / 4 : 0u;
}

// Remaining work of a message lane, in compressions (for ordering only).
__device__ __forceinline__ uint32_t msg_work(uint32_t len) {
  const uint32_t nch = n_chunks_of(len), q = units_of(len);
  const uint32_t first = 4 * q * B3_CHUNK_LEN;
  const uint32_t rem_bytes = len - first;
  const uint32_t rem_blocks = rem_bytes == 0 ? (q ? 0u : 1u) : (rem_bytes + 63) / 64;
  const uint32_t rem = nch - 4 * q;
  return 1 + rem_blocks + (rem > 1 ? rem - 1 : 0) + (q ? q + (rem ? 1 : 0) - 1 : 0);
}

__global__ __launch_bounds__(kThreads) void k_plan2(const uint64_t* __restrict__ off,
                                                    const uint32_t* __restrict__ len, uint32_t n,
                                                    uint32_t max_len,
                                                    uint32_t* __restrict__ units,
                                                    uint32_t* __restrict__ slots,
                                                    uint32_t* __restrict__ work,
                                                    int32_t* __restrict__ status,
                                                    uint32_t out_words, uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const uint32_t l = len[i];
  const bool ok = l <= max_len && (off[i] & 15u) == 0;
  const uint32_t q = ok ? units_of(l) : 0u;
  units[i] = q;
  slots[i] = q ? q + 1 : 0u;
  work[i] = ok ? msg_work(l) : 0u;
  if (status) status[i] = ok ? 0 : -EINVAL;
  if (!ok)
    for (uint32_t w = 0; w < out_words; ++w) out[i * out_words + w] = 0u;
}

__global__ __launch_bounds__(kThreads) void k_units(
    const uint8_t* __restrict__ arena, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ unit_msg, const uint32_t* __restrict__ unit_base,
    const uint32_t* __restrict__ slot_base, const uint32_t* __restrict__ d_total,
    uint32_t* __restrict__ cvs) {
  const uint32_t total = *d_total;
  const uint32_t stride = gridDim.x * kThreads;
  for (uint32_t u = blockIdx.x * kThreads + threadIdx.x; u < total; u += stride) {
    const uint32_t m = unit_msg[u];
    const uint32_t g = u - unit_base[m];
    const uint32_t j0 = 4 * g;
    const uint8_t* p = arena + off[m] + static_cast<uint64_t>(j0) * B3_CHUNK_LEN;
    uint32_t a[8], b[8];
    b3_chunk_full(p, j0, a);
    b3_chunk_full(p + 1024, j0 + 1, b);
    b3_parent(a, a, b, 0u);
    b3_chunk_full(p + 2048, j0 + 2, b);
    uint32_t c[8];
    b3_chunk_full(p + 3072, j0 + 3, c);
    b3_parent(b, b, c, 0u);
    b3_parent(c, a, b, 0u);
    store_cv(cvs + static_cast<uint64_t>(slot_base[m] + g) * 8, c);
  }
}

// In-place pairwise fold of cnt >= 2 CVs at c; ROOT on the last merge.
__device__ __forceinline__ void fold_root(uint32_t* c, uint32_t cnt, uint32_t p[8]) {
  uint32_t l[8], r[8], ln[8], rn[8];
  while (cnt > 2) {
    const uint32_t half = cnt >> 1;
    load_cv(c, l);
    load_cv(c + 8, r);
    for (uint32_t k = 0; k < half; ++k) {
      if (k + 1 < half) {
        load_cv(c + 16 * (k + 1), ln);
        load_cv(c + 16 * (k + 1) + 8, rn);
      }
      b3_parent(p, l, r, 0u);
      store_cv(c + 8 * k, p);
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        l[w] = ln[w];
        r[w] = rn[w];
      }
    }
    if (cnt & 1u) {
      load_cv(c + 8 * (cnt - 1), l);
      store_cv(c + 8 * half, l);
    }
    cnt = half + (cnt & 1u);
  }
  load_cv(c, l);
  load_cv(c + 8, r);
  b3_parent(p, l, r, B3_ROOT);
}

__global__ __launch_bounds__(kThreads) void k_msgs(
    const uint8_t* __restrict__ arena, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, const uint32_t* __restrict__ slot_base,
    const uint32_t* __restrict__ order, const uint32_t* __restrict__ bins,
    uint32_t* __restrict__ cvs, uint32_t out_words, uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= bins[kBins]) return;
  const uint32_t m = order[i];
  const uint32_t l = len[m];
  const uint32_t nch = n_chunks_of(l), q = units_of(l);
  const uint32_t rem = nch - 4 * q;  // 0..4 (1..4 when q == 0)
  const uint8_t* p = arena + off[m];
  const uint32_t rootf = q == 0 ? B3_ROOT : 0u;
  // level-2 node of the remaining chunks [4q, nch): pairwise fold of <= 4
  // chunk CVs with a 2-entry register stack (s0, s1).
  uint32_t cv[8], s0[8], s1[8];
  uint32_t sp = 0;
  for (uint32_t k = 0; k < rem; ++k) {
    const uint32_t j = 4 * q + k;
    const uint32_t clen = min(B3_CHUNK_LEN, l - j * B3_CHUNK_LEN);
    b3_chunk(p + static_cast<uint64_t>(j) * B3_CHUNK_LEN, clen, j, rem == 1 ? rootf : 0u, cv);
    if (k + 1 == rem) break;
    if (((k + 1) & 1u) == 0) {  // two nodes of the pair are complete: merge
      uint32_t t[8];
#pragma unroll
      for (int w = 0; w < 8; ++w) t[w] = sp == 2 ? s1[w] : s0[w];
      b3_parent(cv, t, cv, 0u);
      --sp;
    }
    if (sp == 0) {
#pragma unroll
      for (int w = 0; w < 8; ++w) s0[w] = cv[w];
    } else {
#pragma unroll
      for (int w = 0; w < 8; ++w) s1[w] = cv[w];
    }
    ++sp;
  }
  while (sp > 0) {
    uint32_t t[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) t[w] = sp == 2 ? s1[w] : s0[w];
    b3_parent(cv, t, cv, sp == 1 ? rootf : 0u);
    --sp;
  }
  if (q == 0) {
    for (uint32_t w = 0; w < out_words; ++w) out[m * out_words + w] = cv[w];
    return;
  }
  uint32_t* c = cvs + static_cast<uint64_t>(slot_base[m]) * 8;
  if (rem) store_cv(c + 8 * q, cv);
  uint32_t r[8];
  fold_root(c, q + (rem ? 1u : 0u), r);
  for (uint32_t w = 0; w < out_words; ++w) out[m * out_words + w] = r[w];
}

// order = messages with key >= kmin sorted by descending key (capped at 127).
__global__ __launch_bounds__(kThreads) void k_kbin_hist(const uint32_t* __restrict__ key,
                                                        uint32_t n, uint32_t kmin,
                                                        uint32_t* __restrict__ bins) {
  __shared__ uint32_t h[kBins];
  if (threadIdx.x < kBins) h[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads) {
    const uint32_t c = key[i];
    if (c >= kmin) atomicAdd(&h[parent_bin(c)], 1u);
  }
  __syncthreads();
  if (threadIdx.x < kBins && h[threadIdx.x]) atomicAdd(&bins[threadIdx.x], h[threadIdx.x]);
}

__global__ __launch_bounds__(kThreads) void k_kbin_scatter(const uint32_t* __restrict__ key,
                                                           uint32_t n, uint32_t kmin,
                                                           uint32_t* __restrict__ bins,
                                                           uint32_t* __restrict__ order) {
  __shared__ uint32_t h[kBins], base[kBins];
  for (uint32_t i0 = blockIdx.x * kThreads; i0 < n; i0 += gridDim.x * kThreads) {
    if (threadIdx.x < kBins) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t i = i0 + threadIdx.x;
    const uint32_t c = i < n ? key[i] : 0u;
    uint32_t local = 0, b = 0;
    if (c >= kmin) {
      b = parent_bin(c);
      local = atomicAdd(&h[b], 1u);
    }
    __syncthreads();
    if (threadIdx.x < kBins && h[threadIdx.x])
      base[threadIdx.x] = atomicAdd(&bins[threadIdx.x], h[threadIdx.x]);
    __syncthreads();
    if (c >= kmin) order[base[b] + local] = i;
    __syncthreads();
  }
}

hipError_t batch_hash_launch_v2(const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                                uint32_t n, uint32_t max_len, uint32_t out_words, uint8_t* out,
                                int32_t* status, const BatchWork& w, hipStream_t s,
                                KTimer* timer) {
  const uint32_t blocks = (n + kThreads - 1) / kThreads;
  uint32_t* o = reinterpret_cast<uint32_t*>(out);
  // n_chunks <- units per message; the per-message work estimate is parked in
  // the head of the CV buffer, which k_units only writes after the sort.
  uint32_t* units = w.n_chunks;
  uint32_t* slots = w.slot_base;
  k_plan2<<<blocks, kThreads, 0, s>>>(off, len, n, max_len, units, slots, w.cvs, status,
                                      out_words, o);
  scan::exclusive(units, n, w.chunk_base, w.block_sums, w.total, s);
  scan::exclusive(slots, n, w.slot_base, w.slot_sums, nullptr, s);
  k_fill_map<<<(n + 3) / 4, kThreads, 0, s>>>(units, w.chunk_base, n, w.chunk_msg);
  // sort message lanes by work (the estimate sits in w.cvs[0..n) until k_units)
  (void)hipMemsetAsync(w.bins, 0, sizeof(uint32_t) * (kBins + 1), s);
  const uint32_t g = blocks < 1024 ? blocks : 1024;
  k_kbin_hist<<<g, kThreads, 0, s>>>(w.cvs, n, 1, w.bins);
  k_bin_scan<<<1, 64, 0, s>>>(w.bins);
  k_kbin_scatter<<<g, kThreads, 0, s>>>(w.cvs, n, 1, w.bins, w.order);
  uint64_t want = (w.max_chunks / 4 + kThreads - 1) / kThreads;
  const uint32_t grid = static_cast<uint32_t>(want < 8192 ? (want ? want : 1) : 8192);
  {
    KScope k(timer, "cas_units", s);
    k_units<<<grid, kThreads, 0, s>>>(arena, off, w.chunk_msg, w.chunk_base, w.slot_base, w.total,
                                      w.cvs);
  }
  {
    KScope k(timer, "cas_msgs", s);
    k_msgs<<<blocks, kThreads, 0, s>>>(arena, off, len, w.slot_base, w.order, w.bins, w.cvs,
                                       out_words, o);
  }
  return hipGetLastError();
}

// ============================================================================
// K1 v3: persistent, longest-first work queue over units and message items.
//
// v2 launched one lane per unit over a fixed grid of 8192 blocks: with 6
// resident blocks per CU that is 5.3 "rounds" of blocks, and the last third of
// a round ran on a third of the machine (~11 % of K1 lost to the tail).  v3:
//   leaves: a grid of exactly the resident capacity; each wave grabs the next
//           64 items from one global counter.  Items are the U units (67
//           compressions each, the heaviest items) followed by the R message
//           items (the 1..4 ragged chunks of each message, or the whole
//           message when it has <= 4 chunks) sorted by descending work, so
//           the queue drains heaviest-first (LPT) and the tail is made of the
//           lightest items.
//   fold  : one lane per unit-bearing message (sorted by node count) folds
//           its q (+1) level-2 nodes pairwise, ROOT on the last parent.
// CV slots: message m owns slots [unit_base[m] + m, + q + 1): its units'
// nodes, then the node of its ragged chunks.  sum(q + 1) <= total chunks.
// Both lane orders come from one counting sort (per-block histograms in
// bin-major order + one exclusive scan: no global atomics on hot bins).
// ============================================================================

constexpr uint32_t kSortBlocks = 256;

// Leaf work of message m (compressions of its message item; 0 = no item).
__device__ __forceinline__ uint32_t leaf_work3(uint32_t len) {
  const uint32_t nch = n_chunks_of(len), q = units_of(len);
  const uint32_t rem = nch - 4 * q;
  if (rem == 0) return 0u;
  const uint32_t rem_bytes = len - 4 * q * B3_CHUNK_LEN;
  const uint32_t rem_blocks = rem_bytes == 0 ? 1u : (rem_bytes + 63) / 64;
  return rem_blocks + (rem - 1);
}

// Sort bins of message (len, ok): key 0 = message item by leaf work, key 1 =
// fold lane by node count.  kBins means "not in this list".
__device__ __forceinline__ void bins3(uint32_t len, bool ok, uint32_t& b0, uint32_t& b1) {
  b0 = b1 = kBins;
  if (!ok) return;
  const uint32_t lw = leaf_work3(len);
  if (lw) b0 = parent_bin(lw);
  const uint32_t q = units_of(len);
  if (q) b1 = parent_bin(q + (n_chunks_of(len) > 4 * q ? 1u : 0u));
}

struct Range3 {
  uint32_t lo, hi;
};
__device__ __forceinline__ Range3 block_range3(uint32_t n) {
  const uint32_t per = (n + gridDim.x - 1) / gridDim.x;
  const uint32_t lo = min(n, blockIdx.x * per);
  return {lo, min(n, lo + per)};
}

// Per message: unit count, status, zeroed output of invalid messages; per
// block: histograms of both sort keys -> hist[(key * kBins + bin) * NB + blk].
__global__ __launch_bounds__(kThreads) void k_plan3(const uint64_t* __restrict__ off,
                                                    const uint32_t* __restrict__ len, uint32_t n,
                                                    uint32_t max_len, uint32_t* __restrict__ units,
                                                    uint32_t* __restrict__ hist,
                                                    uint32_t* __restrict__ grab,
                                                    int32_t* __restrict__ status,
                                                    uint32_t out_words, uint32_t* __restrict__ out) {
  __shared__ uint32_t h[2][kBins];
  for (uint32_t t = threadIdx.x; t < 2 * kBins; t += kThreads) (&h[0][0])[t] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) *grab = 0;
  __syncthreads();
  const Range3 r = block_range3(n);
  for (uint32_t i = r.lo + threadIdx.x; i < r.hi; i += kThreads) {
    const uint32_t l = len[i];
    const bool ok = l <= max_len && (off[i] & 15u) == 0;
    units[i] = ok ? units_of(l) : 0u;
    if (status) status[i] = ok ? 0 : -EINVAL;
    if (!ok)
      for (uint32_t w = 0; w < out_words; ++w) out[i * out_words + w] = 0u;
    uint32_t b0, b1;
    bins3(l, ok, b0, b1);
    if (b0 < kBins) atomicAdd(&h[0][b0], 1u);
    if (b1 < kBins) atomicAdd(&h[1][b1], 1u);
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < 2 * kBins; t += kThreads)
    hist[static_cast<size_t>(t) * gridDim.x + blockIdx.x] = (&h[0][0])[t];
}

// Scatter both lane orders (positions from the scanned histograms: key 0 lands
// in [0, R), key 1 in [R, R + F)) and fill the unit -> message map.
__global__ __launch_bounds__(kThreads) void k_scatter3(const uint64_t* __restrict__ off,
                                                       const uint32_t* __restrict__ len, uint32_t n,
                                                       uint32_t max_len,
                                                       const uint32_t* __restrict__ unit_base,
                                                       const uint32_t* __restrict__ hist_scan,
                                                       uint32_t* __restrict__ order,
                                                       uint32_t* __restrict__ unit_msg) {
  __shared__ uint32_t cur[2][kBins], cnt[2][kBins];
  for (uint32_t t = threadIdx.x; t < 2 * kBins; t += kThreads) {
    (&cur[0][0])[t] = hist_scan[static_cast<size_t>(t) * gridDim.x + blockIdx.x];
    (&cnt[0][0])[t] = 0;
  }
  __syncthreads();
  const Range3 r = block_range3(n);
  for (uint32_t i0 = r.lo; i0 < r.hi; i0 += kThreads) {
    const uint32_t i = i0 + threadIdx.x;
    uint32_t b0 = kBins, b1 = kBins, l0 = 0, l1 = 0;
    if (i < r.hi) {
      const uint32_t l = len[i];
      const bool ok = l <= max_len && (off[i] & 15u) == 0;
      bins3(l, ok, b0, b1);
      if (b0 < kBins) l0 = atomicAdd(&cnt[0][b0], 1u);
      if (b1 < kBins) l1 = atomicAdd(&cnt[1][b1], 1u);
      const uint32_t q = ok ? units_of(l) : 0u;
      const uint32_t ub = unit_base[i];
      for (uint32_t g = 0; g < q; ++g) unit_msg[ub + g] = i;
    }
    __syncthreads();
    if (b0 < kBins) order[cur[0][b0] + l0] = i;
    if (b1 < kBins) order[cur[1][b1] + l1] = i;
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < 2 * kBins; t += kThreads) {
      (&cur[0][0])[t] += (&cnt[0][0])[t];
      (&cnt[0][0])[t] = 0;
    }
    __syncthreads();
  }
}

// One 4-chunk unit: level-2 node of chunks [4g, 4g + 4) of message m.
__device__ __forceinline__ void unit_item(const uint8_t* __restrict__ arena,
                                          const uint64_t* __restrict__ off,
                                          const uint32_t* __restrict__ unit_msg,
                                          const uint32_t* __restrict__ unit_base, uint32_t u,
                                          uint32_t* __restrict__ cvs) {
  const uint32_t m = unit_msg[u];
  const uint32_t ub = unit_base[m];
  const uint32_t g = u - ub;
  const uint32_t j0 = 4 * g;
  const uint8_t* p = arena + off[m] + static_cast<uint64_t>(j0) * B3_CHUNK_LEN;
  uint32_t a[8], b[8], c[8];
  b3_chunk_full(p, j0, a);
  b3_chunk_full(p + 1024, j0 + 1, b);
  b3_parent(a, a, b, 0u);
  b3_chunk_full(p + 2048, j0 + 2, b);
  b3_chunk_full(p + 3072, j0 + 3, c);
  b3_parent(b, b, c, 0u);
  b3_parent(c, a, b, 0u);
  store_cv(cvs + static_cast<uint64_t>(ub + m + g) * 8, c);
}

// Chunk j of a message (full chunks take the 128-byte-line path).
__device__ __forceinline__ void chunk_any(const uint8_t* __restrict__ p, uint32_t l, uint32_t j,
                                          uint32_t root_flag, uint32_t cv[8]) {
  const uint32_t clen = min(B3_CHUNK_LEN, l - j * B3_CHUNK_LEN);
  const uint8_t* cp = p + static_cast<uint64_t>(j) * B3_CHUNK_LEN;
  if (clen == B3_CHUNK_LEN && root_flag == 0)
    b3_chunk_full(cp, j, cv);
  else
    b3_chunk(cp, clen, j, root_flag, cv);
}

// Message item: the node of chunks [4q, nch) (the whole message, with ROOT,
// when q == 0).  1..4 chunks form the left-complete subtree
// c0 | P(c0,c1) | P(P(c0,c1),c2) | P(P(c0,c1),P(c2,c3)), built with the
// same three CV registers as a unit.
__device__ __forceinline__ void msg_item(const uint8_t* __restrict__ arena,
                                         const uint64_t* __restrict__ off,
                                         const uint32_t* __restrict__ len,
                                         const uint32_t* __restrict__ unit_base, uint32_t m,
                                         uint32_t* __restrict__ cvs, uint32_t out_words,
                                         uint32_t* __restrict__ out) {
  const uint32_t l = len[m];
  const uint32_t nch = n_chunks_of(l), q = units_of(l);
  const uint32_t rem = nch - 4 * q;  // 1..4
  const uint8_t* p = arena + off[m];
  const uint32_t rootf = q == 0 ? B3_ROOT : 0u;
  const uint32_t j0 = 4 * q;
  uint32_t a[8], b[8], c[8];
  chunk_any(p, l, j0, rem == 1 ? rootf : 0u, a);
  if (rem >= 2) {
    chunk_any(p, l, j0 + 1, 0u, b);
    b3_parent(a, a, b, rem == 2 ? rootf : 0u);
  }
  if (rem >= 3) {
    chunk_any(p, l, j0 + 2, 0u, b);
    if (rem == 4) {
      chunk_any(p, l, j0 + 3, 0u, c);
      b3_parent(b, b, c, 0u);
    }
    b3_parent(a, a, b, rootf);
  }
  if (q == 0) {
    for (uint32_t w = 0; w < out_words; ++w) out[m * out_words + w] = a[w];
  } else {
    store_cv(cvs + static_cast<uint64_t>(unit_base[m] + m + q) * 8, a);
  }
}

template <int kMinBlocks>
__global__ __launch_bounds__(kThreads, kMinBlocks) void k_leaves3(
    const uint8_t* __restrict__ arena, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, const uint32_t* __restrict__ unit_msg,
    const uint32_t* __restrict__ unit_base, const uint32_t* __restrict__ d_units,
    const uint32_t* __restrict__ order, const uint32_t* __restrict__ d_r,
    uint32_t* __restrict__ grab, uint32_t* __restrict__ cvs, uint32_t out_words,
    uint32_t* __restrict__ out) {
  const uint32_t U = *d_units;
  const uint32_t total = U + *d_r;
  const uint32_t lane = threadIdx.x & 63u;
  for (;;) {
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(grab, 64u);
    base = __builtin_amdgcn_readfirstlane(__shfl(base, 0));
    if (base >= total) break;  // uniform: every wave reaches this exit
    const uint32_t i = base + lane;
    if (i < U)
      unit_item(arena, off, unit_msg, unit_base, i, cvs);
    else if (i < total)
      msg_item(arena, off, len, unit_base, order[i - U], cvs, out_words, out);
  }
}

// Fold lanes keep a CV stack of depth 5 in LDS (lane-minor, conflict-free):
// enough for the <= 26 level-2 nodes of any cas message (<= 100 KiB); longer
// staged messages fall back to the in-place pairwise fold.
constexpr uint32_t kFoldStack = 5;

__global__ __launch_bounds__(kThreads) void k_fold3(const uint32_t* __restrict__ len,
                                                    const uint32_t* __restrict__ unit_base,
                                                    const uint32_t* __restrict__ order,
                                                    const uint32_t* __restrict__ d_r,
                                                    const uint32_t* __restrict__ d_end,
                                                    uint32_t* __restrict__ cvs, uint32_t out_words,
                                                    uint32_t* __restrict__ out) {
  __shared__ uint32_t stk[kFoldStack][8][kThreads];
  const uint32_t R = *d_r;
  const uint32_t i = R + blockIdx.x * kThreads + threadIdx.x;
  if (i >= *d_end) return;
  const uint32_t m = order[i];
  const uint32_t l = len[m];
  const uint32_t q = units_of(l);
  const uint32_t cnt = q + (n_chunks_of(l) > 4 * q ? 1u : 0u);
  uint32_t* c = cvs + static_cast<uint64_t>(unit_base[m] + m) * 8;
  uint32_t r[8];
  if (cnt > (1u << kFoldStack)) {
    fold_root(c, cnt, r);
  } else {
    // BLAKE3's lazy-merge stack over the level-2 nodes: merge while the count
    // of completed nodes is even, never merge the last node before the end.
    uint32_t lf[8], nx[8];
    uint32_t sp = 0;
    load_cv(c, r);
    for (uint32_t k = 0; k + 1 < cnt; ++k) {
      load_cv(c + 8 * (k + 1), nx);  // next node, loaded ahead of the merges
      for (uint32_t tot = k + 1; (tot & 1u) == 0; tot >>= 1) {
        --sp;
#pragma unroll
        for (int w = 0; w < 8; ++w) lf[w] = stk[sp][w][threadIdx.x];
        b3_parent(r, lf, r, 0u);
      }
#pragma unroll
      for (int w = 0; w < 8; ++w) stk[sp][w][threadIdx.x] = r[w];
      ++sp;
#pragma unroll
      for (int w = 0; w < 8; ++w) r[w] = nx[w];
    }
    while (sp > 0) {
      --sp;
#pragma unroll
      for (int w = 0; w < 8; ++w) lf[w] = stk[sp][w][threadIdx.x];
      b3_parent(r, lf, r, sp == 0 ? B3_ROOT : 0u);
    }
  }
  for (uint32_t w = 0; w < out_words; ++w) out[m * out_words + w] = r[w];
}

// Resident-capacity grid of k_leaves3<kMinBlocks> on the current device.
template <int kMinBlocks>
uint32_t leaves3_grid() {
  static int cached_dev = -1;
  static uint32_t cached = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev != cached_dev) {
    int cus = 0, per = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_leaves3<kMinBlocks>, kThreads, 0);
    cached = static_cast<uint32_t>(std::max(1, cus) * std::max(1, per));
    cached_dev = dev;
  }
  return cached;
}

hipError_t batch_hash_launch_v3(const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                                uint32_t n, uint32_t max_len, uint32_t out_words, uint8_t* out,
                                int32_t* status, const BatchWork& w, hipStream_t s,
                                KTimer* timer, bool occ6) {
  uint32_t* o = reinterpret_cast<uint32_t*>(out);
  const uint32_t nb = std::min<uint32_t>(kSortBlocks, (n + kThreads - 1) / kThreads);
  const uint32_t nh = 2 * kBins * nb;
  // hist_scan[kBins * nb] = R (start of the fold list), hist_scan[nh] = R + F
  k_plan3<<<nb, kThreads, 0, s>>>(off, len, n, max_len, w.n_chunks, w.hist, w.grab, status,
                                  out_words, o);
  scan::exclusive(w.n_chunks, n, w.chunk_base, w.block_sums, w.total, s);
  scan::exclusive(w.hist, nh, w.hist, w.hist_sums, nullptr, s);
  k_scatter3<<<nb, kThreads, 0, s>>>(off, len, n, max_len, w.chunk_base, w.hist, w.order,
                                     w.chunk_msg);
  const uint32_t* d_r = w.hist + static_cast<size_t>(kBins) * nb;
  {
    KScope k(timer, "cas_leaves", s);
    if (occ6)
      k_leaves3<6><<<leaves3_grid<6>(), kThreads, 0, s>>>(arena, off, len, w.chunk_msg,
                                                          w.chunk_base, w.total, w.order, d_r,
                                                          w.grab, w.cvs, out_words, o);
    else
      k_leaves3<5><<<leaves3_grid<5>(), kThreads, 0, s>>>(arena, off, len, w.chunk_msg,
                                                          w.chunk_base, w.total, w.order, d_r,
                                                          w.grab, w.cvs, out_words, o);
  }
  {
    KScope k(timer, "cas_fold", s);
    k_fold3<<<(n + kThreads - 1) / kThreads, kThreads, 0, s>>>(len, w.chunk_base, w.order, d_r,
                                                               w.hist + nh, w.cvs, out_words, o);
  }
  return hipGetLastError();
}

// ============================================================================
// Latency path: one workgroup per message of at most 1024 chunks (1 MiB).
// Thread t hashes chunk t (16 compressions), then the CVs are folded level by
// level in LDS (pairwise, odd node carried up: BLAKE3's left-complete tree),
// one compression per level, ROOT on the last.  A 57-chunk cas message is one
// pass of 57 lanes + 6 levels: ~22 compression latencies in ONE launch, for
// the single-file callers (watcher/utils.rs:236,411,467, non_indexed.rs:161)
// where K1's planning launches would dominate.
// ============================================================================

constexpr uint32_t kSmallMaxChunks = 1024;

__global__ __launch_bounds__(1024) void k_small(const uint8_t* __restrict__ arena,
                                                const uint64_t* __restrict__ off,
                                                const uint32_t* __restrict__ len,
                                                uint32_t max_len, uint32_t out_words,
                                                uint32_t* __restrict__ out,
                                                int32_t* __restrict__ status) {
  __shared__ uint32_t cv[8][kSmallMaxChunks];  // word-major: lane-indexed access is conflict-free
  const uint32_t m = blockIdx.x;
  const uint32_t t = threadIdx.x;
  const uint32_t l = len[m];
  const bool ok = l <= max_len && (off[m] & 15u) == 0 && l <= kSmallMaxChunks * B3_CHUNK_LEN;
  if (t == 0 && status) status[m] = ok ? 0 : -EINVAL;
  if (!ok) {
    if (t < out_words) out[m * out_words + t] = 0u;
    return;
  }
  const uint32_t nch = n_chunks_of(l);
  const uint8_t* p = arena + off[m];
  uint32_t c[8];
  if (nch == 1) {
    if (t == 0) {
      b3_chunk(p, l, 0, B3_ROOT, c);
      for (uint32_t w = 0; w < out_words; ++w) out[m * out_words + w] = c[w];
    }
    return;
  }
  if (t < nch) {
    chunk_any(p, l, t, 0u, c);
#pragma unroll
    for (int w = 0; w < 8; ++w) cv[w][t] = c[w];
  }
  __syncthreads();
  uint32_t cnt = nch;
  while (cnt > 2) {
    const uint32_t half = cnt >> 1;
    uint32_t a[8], b[8];
    const bool merge = t < half;
    const bool carry = (cnt & 1u) && t == half;
    if (merge) {
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        a[w] = cv[w][2 * t];
        b[w] = cv[w][2 * t + 1];
      }
      b3_parent(c, a, b, 0u);
    } else if (carry) {
#pragma unroll
      for (int w = 0; w < 8; ++w) c[w] = cv[w][cnt - 1];
    }
    __syncthreads();
    if (merge || carry) {
#pragma unroll
      for (int w = 0; w < 8; ++w) cv[w][t] = c[w];
    }
    __syncthreads();
    cnt = half + (cnt & 1u);
  }
  if (t == 0) {
    uint32_t a[8], b[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      a[w] = cv[w][0];
      b[w] = cv[w][1];
    }
    b3_parent(c, a, b, B3_ROOT);
    for (uint32_t w = 0; w < out_words; ++w) out[m * out_words + w] = c[w];
  }
}

}  // namespace

hipError_t batch_hash_launch(const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                             uint32_t n, uint32_t max_len, uint32_t out_words, uint8_t* out,
                             int32_t* status, const BatchWork& w, hipStream_t s,
                             KTimer* timer) {
  if (n == 0) return hipSuccess;
  const int variant = k1_variant();
  if (variant == 3 || variant == 4)
    return batch_hash_launch_v3(arena, off, len, n, max_len, out_words, out, status, w, s, timer,
                                variant == 4);
  if (k1_variant() == 2)
    return batch_hash_launch_v2(arena, off, len, n, max_len, out_words, out, status, w, s, timer);
  const uint32_t blocks = (n + kThreads - 1) / kThreads;
  uint32_t* o = reinterpret_cast<uint32_t*>(out);
  k_plan<<<blocks, kThreads, 0, s>>>(off, len, n, max_len, w.n_chunks, status, out_words, o);
  scan::exclusive(w.n_chunks, n, w.chunk_base, w.block_sums, w.total, s);
  k_fill_map<<<(n + 3) / 4, kThreads, 0, s>>>(w.n_chunks, w.chunk_base, n, w.chunk_msg);
  // Grid-stride over chunks: enough waves to fill 256 CUs several times over.
  uint64_t want = (w.max_chunks + kThreads - 1) / kThreads;
  const uint32_t grid = static_cast<uint32_t>(want < 8192 ? (want ? want : 1) : 8192);
  {
    KScope k(timer, "cas_chunks", s);
    if (k1_variant() == 1)
      k_chunks<true><<<grid, kThreads, 0, s>>>(arena, off, len, w.chunk_msg, w.chunk_base,
                                               w.total, w.cvs, out_words, o);
    else
      k_chunks<false><<<grid, kThreads, 0, s>>>(arena, off, len, w.chunk_msg, w.chunk_base,
                                                w.total, w.cvs, out_words, o);
  }
  {
    KScope k(timer, "cas_parents", s);
    (void)hipMemsetAsync(w.bins, 0, sizeof(uint32_t) * (kBins + 1), s);
    const uint32_t g = blocks < 1024 ? blocks : 1024;
    k_bin_hist<<<g, kThreads, 0, s>>>(w.n_chunks, n, w.bins);
    k_bin_scan<<<1, 64, 0, s>>>(w.bins);
    k_bin_scatter<<<g, kThreads, 0, s>>>(w.n_chunks, n, w.bins, w.order);
    k_parents<<<blocks, kThreads, 0, s>>>(w.n_chunks, w.chunk_base, w.order, w.bins, n, w.cvs,
                                          out_words, o);
  }
  return hipGetLastError();
}

}  // namespace sdgpu

namespace sdgpu {

// One workgroup per message; max_chunks = the largest chunk count of the batch
// (host-known), which sizes the workgroup.  Messages must be <= 1 MiB.
hipError_t small_hash_launch(const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                             uint32_t n, uint32_t max_len, uint32_t max_chunks,
                             uint32_t out_words, uint8_t* out, int32_t* status, hipStream_t s,
                             KTimer* timer) {
  if (n == 0) return hipSuccess;
  if (max_chunks > kSmallMaxChunks) return hipErrorInvalidValue;
  const uint32_t threads = std::max<uint32_t>(64, (max_chunks + 63) / 64 * 64);
  KScope k(timer, "cas_small", s);
  k_small<<<n, threads, 0, s>>>(arena, off, len, max_len, out_words,
                                reinterpret_cast<uint32_t*>(out), status);
  return hipGetLastError();
}

}  // namespace sdgpu
