// K1: batched BLAKE3 over many short messages -- the sampled cas_id path.
//
// Replaces generate_cas_id's hashing (/root/reference/core/src/object/cas.rs:24-61)
// as run for every orphan file_path by identifier_job_step
// (/root/reference/core/src/object/file_identifier/mod.rs:107-134), where the
// reference hashes <=100 files per step, one after another, on one CPU thread.
//
// Input: a device arena of cas messages M_i = size_le(8 B) || windows
// (<= 102 408 B each, 16-B aligned offsets), packed by the host or the synthetic
// generator.  Decomposition: a persistent, longest-first work queue over
// 4-chunk UNITS and MESSAGE items, then a per-message fold.
//
// A message of n > 4 chunks has q = floor(full_chunks / 4) aligned units of 4
// FULL chunks.  A unit lane hashes the 4 chunks and merges them in-lane,
// P(P(c0,c1), P(c2,c3)) -- 67 compressions, identical for every lane, no ragged
// chunk anywhere: a unit is a complete level-2 subtree of BLAKE3's tree.  The
// message item hashes the 1..4 remaining chunks [4q, n) into one level-2 node
// (the whole message, with ROOT, when q == 0).  For a sampled cas message (56
// full chunks + 8 bytes) that is 14 unit items, one message item and a fold of
// 15 nodes instead of 56 serial parents.
//   leaves: a grid of exactly the resident capacity; each wave grabs the next
//           64 items from one global counter.  Items are the U units (the
//           heaviest, uniform items) followed by the R message items sorted by
//           descending work, so the queue drains heaviest-first (LPT) and the
//           tail is made of the lightest items.  (A fixed 8192-block grid of
//           one lane per unit ran its last round on a third of the machine,
//           ~11 % of K1: DESIGN.md §4.)
//   fold  : one lane per unit-bearing message (sorted by node count) folds
//           its q (+1) level-2 nodes, ROOT on the last parent.
// CV slots: message m owns slots [unit_base[m] + m, + q + 1): its units'
// nodes, then the node of its ragged chunks.  Both lane orders come from one
// counting sort (per-block histograms in bin-major order + one exclusive scan:
// no global atomics on hot bins).
//
// Workspace guard: the host sizes the CV slots and the unit map from the arena
// size (arena_bytes / 1024 + n >= sum(q + 1) for disjoint messages inside the
// arena).  A message that ends past the arena is -EINVAL; if the messages
// overlap so much that U + n exceeds the capacity, every message gets -ENOBUFS
// and nothing is written past the workspace.
#include <errno.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>

#include "b3_device.hpp"
#include "internal.hpp"
#include "scan_device.hpp"

namespace sdgpu {

namespace {

constexpr int kThreads = 256;

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

// Lanes are ordered by work (descending) so that the 64 lanes of a wave do
// equal work: bin = 127 - min(work, 127).
constexpr uint32_t kBins = 128;

__device__ __forceinline__ uint32_t parent_bin(uint32_t nch) {
  return kBins - 1 - min(nch, kBins - 1);
}

__device__ __forceinline__ uint32_t n_chunks_of(uint32_t len) {
  return len <= B3_CHUNK_LEN ? 1u : (len + B3_CHUNK_LEN - 1) / B3_CHUNK_LEN;
}

__device__ __forceinline__ uint32_t units_of(uint32_t len) {
  return n_chunks_of(len) > 4 ? (len / B3_CHUNK_LEN) / 4 : 0u;
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
// A message is hashed when it fits the kernel (len <= max_len), is 16-B aligned
// and lies inside the arena.
__device__ __forceinline__ bool msg_ok(uint64_t o, uint32_t l, uint32_t max_len,
                                       uint64_t arena_bytes) {
  return l <= max_len && (o & 15u) == 0 && o <= arena_bytes && l <= arena_bytes - o;
}

__global__ __launch_bounds__(kThreads) void k_plan3(const uint64_t* __restrict__ off,
                                                    const uint32_t* __restrict__ len, uint32_t n,
                                                    uint32_t max_len, uint64_t arena_bytes,
                                                    uint32_t* __restrict__ units,
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
    const bool ok = msg_ok(off[i], l, max_len, arena_bytes);
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

// The CV slots of the batch (U + n) exceed the workspace: nothing is hashed.
__device__ __forceinline__ bool over_capacity(const uint32_t* d_units, uint32_t n, uint64_t cap) {
  return static_cast<uint64_t>(*d_units) + n > cap;
}

// Scatter both lane orders (positions from the scanned histograms: key 0 lands
// in [0, R), key 1 in [R, R + F)) and fill the unit -> message map.  Over
// capacity, every message is marked -ENOBUFS instead.
__global__ __launch_bounds__(kThreads) void k_scatter3(const uint64_t* __restrict__ off,
                                                       const uint32_t* __restrict__ len, uint32_t n,
                                                       uint32_t max_len, uint64_t arena_bytes,
                                                       uint64_t cap, const uint32_t* __restrict__ d_units,
                                                       int32_t* __restrict__ status,
                                                       uint32_t out_words, uint32_t* __restrict__ out,
                                                       const uint32_t* __restrict__ unit_base,
                                                       const uint32_t* __restrict__ hist_scan,
                                                       uint32_t* __restrict__ order,
                                                       uint32_t* __restrict__ unit_msg) {
  __shared__ uint32_t cur[2][kBins], cnt[2][kBins];
  const Range3 r = block_range3(n);
  if (over_capacity(d_units, n, cap)) {  // uniform over the grid
    for (uint32_t i = r.lo + threadIdx.x; i < r.hi; i += kThreads) {
      if (status) status[i] = -ENOBUFS;
      for (uint32_t w = 0; w < out_words; ++w) out[i * out_words + w] = 0u;
    }
    return;
  }
  for (uint32_t t = threadIdx.x; t < 2 * kBins; t += kThreads) {
    (&cur[0][0])[t] = hist_scan[static_cast<size_t>(t) * gridDim.x + blockIdx.x];
    (&cnt[0][0])[t] = 0;
  }
  __syncthreads();
  for (uint32_t i0 = r.lo; i0 < r.hi; i0 += kThreads) {
    const uint32_t i = i0 + threadIdx.x;
    uint32_t b0 = kBins, b1 = kBins, l0 = 0, l1 = 0;
    if (i < r.hi) {
      const uint32_t l = len[i];
      const bool ok = msg_ok(off[i], l, max_len, arena_bytes);
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

// 5 resident blocks (20 waves) per CU: the 6-block variant needs a few bytes
// of spill and measured no faster.
constexpr int kLeavesMinBlocks = 5;

__global__ __launch_bounds__(kThreads, kLeavesMinBlocks) void k_leaves3(
    const uint8_t* __restrict__ arena, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, const uint32_t* __restrict__ unit_msg,
    const uint32_t* __restrict__ unit_base, const uint32_t* __restrict__ d_units,
    const uint32_t* __restrict__ order, const uint32_t* __restrict__ d_r,
    uint32_t* __restrict__ grab, uint32_t* __restrict__ cvs, uint32_t out_words,
    uint32_t* __restrict__ out, uint32_t n, uint64_t cap) {
  if (over_capacity(d_units, n, cap)) return;
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
                                                    uint32_t* __restrict__ out,
                                                    const uint32_t* __restrict__ d_units, uint32_t n,
                                                    uint64_t cap) {
  __shared__ uint32_t stk[kFoldStack][8][kThreads];
  if (over_capacity(d_units, n, cap)) return;
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

// Resident-capacity grid of k_leaves3 on the current device.
uint32_t leaves3_grid() {
  static int cached_dev = -1;
  static uint32_t cached = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev != cached_dev) {
    int cus = 0, per = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_leaves3, kThreads, 0);
    cached = static_cast<uint32_t>(std::max(1, cus) * std::max(1, per));
    cached_dev = dev;
  }
  return cached;
}

// ============================================================================
// Latency paths, for the single-file callers (watcher/utils.rs:236,411,467,
// non_indexed.rs:161) and small batches, where K1's planning launches would
// dominate: a message's chunks are hashed in parallel, then the CVs folded
// level by level in LDS (pairwise, odd node carried up: BLAKE3's
// left-complete tree), one compression per level, ROOT on the last -- each
// compression spread over a quad of lanes.  k_small_host / k_service: one
// workgroup per message of <= 112 KiB; k_small_split: messages of <= 1 MiB
// (1024 chunks) split into 64 KiB groups, one workgroup each.
// ============================================================================

constexpr uint32_t kSmallMaxChunks = 1024;

// ---- Quad-lane hashing of an LDS-staged message (the latency paths) ---------
// A single message is a chain of dependent compressions (16 per chunk, then
// one per tree level), so its latency is one compression's latency times the
// chain, and one wave64 lane per chunk spends ~2,800 cycles on each (680
// VALU instructions, 4 independent G chains).  Here each compression is spread
// over a QUAD of lanes: lane i holds state column i (a, b, c, d) =
// (v[i], v[4+i], v[8+i], v[12+i]) and computes G_i of the column step, then,
// after DPP quad rotations of rows b, c, d, G_i of the diagonal step -- 30
// instructions per round instead of 96; its 4 message words per round are
// read from LDS at per-lane offsets of the message schedule.  The outputs
// cv[i] = a ^ c and cv[4+i] = b ^ d are exactly the next block's a and b.
// One wave, chained compressions (scripts/exp_chain.hip,
// profiles/r3/latency/r3L_exp_chain.log): ~1,000 cycles (0.42 us) per
// compression against ~2,800-2,950 (1.15-1.23 us) for the lane form.
__device__ __constant__ uint8_t kQuadSched[7][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8},
    {3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1},
    {10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6},
    {12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4},
    {9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7},
    {11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13}};

// DPP quad_perm: lane i of each quad reads lane i+1 / i+2 / i+3 (mod 4)
constexpr int kQuadRot1 = 0x39, kQuadRot2 = 0x4E, kQuadRot3 = 0x93;
template <int kCtrl>
__device__ __forceinline__ uint32_t quad_perm(uint32_t x) {
  return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(x), kCtrl, 0xF, 0xF, false));
}

__device__ __forceinline__ void quad_g(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d,
                                       uint32_t x, uint32_t y) {
  SDGPU_G(a, b, c, d, x, y);
}

// Per-lane state of the quad form: lane i = threadIdx.x & 3.
struct QuadLane {
  uint32_t i;            // column
  uint32_t iv_a, iv_b;   // IV[i], IV[4 + i]
  uint32_t woff[28];     // byte offsets of this lane's message words, round by round
  __device__ __forceinline__ void init() {
    i = threadIdx.x & 3u;
    const uint32_t iva[4] = {IV0, IV1, IV2, IV3}, ivb[4] = {IV4, IV5, IV6, IV7};
    iv_a = i == 0 ? iva[0] : i == 1 ? iva[1] : i == 2 ? iva[2] : iva[3];
    iv_b = i == 0 ? ivb[0] : i == 1 ? ivb[1] : i == 2 ? ivb[2] : ivb[3];
#pragma unroll
    for (int r = 0; r < 7; ++r) {
      woff[4 * r] = 4u * kQuadSched[r][2 * i];
      woff[4 * r + 1] = 4u * kQuadSched[r][2 * i + 1];
      woff[4 * r + 2] = 4u * kQuadSched[r][8 + 2 * i];
      woff[4 * r + 3] = 4u * kQuadSched[r][9 + 2 * i];
    }
  }
  // (h0, h1) = (cv[i], cv[4+i]) <- compress of the 64-byte block at LDS `blk`
  // (4-byte aligned, zero padded); d = this lane's word of {counter lo,
  // counter hi, block length, flags}.
  __device__ __forceinline__ void compress(uint32_t& h0, uint32_t& h1, const uint8_t* blk,
                                           uint32_t d) const {
    uint32_t w[28];
#pragma unroll
    for (int k = 0; k < 28; ++k) w[k] = *reinterpret_cast<const uint32_t*>(blk + woff[k]);
    uint32_t a = h0, b = h1, c = iv_a;
#pragma unroll
    for (int r = 0; r < 7; ++r) {
      quad_g(a, b, c, d, w[4 * r], w[4 * r + 1]);  // column step
      b = quad_perm<kQuadRot1>(b);
      c = quad_perm<kQuadRot2>(c);
      d = quad_perm<kQuadRot3>(d);
      quad_g(a, b, c, d, w[4 * r + 2], w[4 * r + 3]);  // diagonal step
      b = quad_perm<kQuadRot3>(b);
      c = quad_perm<kQuadRot2>(c);
      d = quad_perm<kQuadRot1>(d);
    }
    h0 = a ^ c;
    h1 = b ^ d;
  }
  __device__ __forceinline__ uint32_t dword(uint32_t ctr, uint32_t blen, uint32_t flags) const {
    return i == 0 ? ctr : i == 1 ? 0u : i == 2 ? blen : flags;
  }
};

// Chunk CVs of the glen bytes staged at LDS `msg` (zero padded to a 64-byte
// multiple, at least 64 bytes), chunk counters ctr0, ctr0 + 1, ...: lane i of
// the quad owning chunk j writes cvr[8 j + i] and cvr[8 j + 4 + i] (row-major
// CVs: a parent's 16 message words are its two children's rows, contiguous).
// With `whole` (these bytes are the whole message) and a single chunk, that
// chunk is the ROOT: its output words i and 4 + i are left in (h0, h1) of
// lanes i = 0..3 and nothing is written.  Every thread must call it.
__device__ __forceinline__ void quad_chunks(const QuadLane& L, const uint8_t* msg, uint32_t glen,
                                            uint32_t ctr0, bool whole, uint32_t* cvr, uint32_t& h0,
                                            uint32_t& h1) {
  const uint32_t q = threadIdx.x >> 2, Q = blockDim.x >> 2;
  const uint32_t nch = n_chunks_of(glen);
  const bool root_chunk = whole && nch == 1;
  for (uint32_t c = q; c < nch; c += Q) {
    const uint32_t clen = min(B3_CHUNK_LEN, glen - c * B3_CHUNK_LEN);
    const uint32_t nb = clen == 0 ? 1u : (clen + 63u) >> 6;
    const uint8_t* cp = msg + c * B3_CHUNK_LEN;
    uint32_t a = L.iv_a, b = L.iv_b;
    for (uint32_t j = 0; j < nb; ++j) {
      const bool last = j + 1 == nb;
      const uint32_t flags = (j == 0 ? B3_CHUNK_START : 0u) |
                             (last ? (B3_CHUNK_END | (root_chunk ? B3_ROOT : 0u)) : 0u);
      L.compress(a, b, cp + 64u * j,
                 L.dword(root_chunk ? 0u : ctr0 + c, last ? clen - 64u * j : B3_BLOCK_LEN, flags));
    }
    if (root_chunk) {
      h0 = a;
      h1 = b;
    } else {
      cvr[8 * c + L.i] = a;
      cvr[8 * c + 4 + L.i] = b;
    }
  }
}

// The tree over the cnt >= 1 CVs in cvr (written before a barrier the caller
// placed): level by level, parents of (2p, 2p + 1) one per quad, the odd last
// CV carried; top_flags (ROOT or 0) on the last parent.  cnt == 1: the CV
// itself.  Leaves the result's words i and 4 + i in (h0, h1) of lanes 0..3;
// every thread must call it; needs blockDim.x / 4 >= cnt / 2.
__device__ __forceinline__ void quad_tree(const QuadLane& L, uint32_t* cvr, uint32_t cnt,
                                          uint32_t top_flags, uint32_t& h0, uint32_t& h1) {
  const uint32_t q = threadIdx.x >> 2;
  while (cnt > 2) {
    const uint32_t half = cnt >> 1;
    uint32_t a = 0, b = 0;
    if (q < half) {
      a = L.iv_a;
      b = L.iv_b;
      L.compress(a, b, reinterpret_cast<const uint8_t*>(cvr + 16 * q),
                 L.dword(0u, B3_BLOCK_LEN, B3_PARENT));
    }
    __syncthreads();
    if (q < half) {
      cvr[8 * q + L.i] = a;
      cvr[8 * q + 4 + L.i] = b;
    } else if ((cnt & 1u) && q == half) {
      cvr[8 * half + L.i] = cvr[8 * (cnt - 1) + L.i];
      cvr[8 * half + 4 + L.i] = cvr[8 * (cnt - 1) + 4 + L.i];
    }
    __syncthreads();
    cnt = half + (cnt & 1u);
  }
  if (q == 0) {
    if (cnt == 1) {
      h0 = cvr[L.i];
      h1 = cvr[4 + L.i];
    } else {
      h0 = L.iv_a;
      h1 = L.iv_b;
      L.compress(h0, h1, reinterpret_cast<const uint8_t*>(cvr),
                 L.dword(0u, B3_BLOCK_LEN, B3_PARENT | top_flags));
    }
  }
}

// The BLAKE3 hash of the l-byte message staged at LDS `msg` (zero padded to a
// 64-byte multiple, at least 64 bytes), by the whole workgroup in quads; the
// digest's words i and 4 + i end in lanes i = 0..3 (h0, h1).
__device__ __forceinline__ void quad_hash_staged(const QuadLane& L, const uint8_t* msg, uint32_t l,
                                                 uint32_t* cvr, uint32_t& h0, uint32_t& h1) {
  quad_chunks(L, msg, l, 0u, true, cvr, h0, h1);
  const uint32_t nch = n_chunks_of(l);
  if (nch == 1) return;  // uniform
  __syncthreads();
  quad_tree(L, cvr, nch, B3_ROOT, h0, h1);
}

// Copies the l-byte message at `src` (16-B aligned, readable up to the next 16
// bytes) into LDS `dst`, zeroing the bytes past l up to the 64-byte block end
// (at least one block), as the quad hash reads whole blocks.
__device__ __forceinline__ void stage_message(uint8_t* dst, const uint8_t* __restrict__ src,
                                              uint32_t l) {
  const uint32_t nvec = (l + 15) / 16;
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
  uint4* d4 = reinterpret_cast<uint4*>(dst);
  constexpr int kU = 8;
  for (uint32_t i0 = threadIdx.x; i0 < nvec; i0 += kU * blockDim.x) {
    uint4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const uint32_t i = i0 + u * blockDim.x;
      v[u] = i < nvec ? s4[i] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const uint32_t i = i0 + u * blockDim.x;
      if (i >= nvec) continue;
      if (16 * i + 16 > l) {  // the last vector: bytes past l -> 0
        const uint32_t vb = l - 16 * i;
        uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
          const uint32_t n = vb > 4 * k ? min(vb - 4 * k, 4u) : 0u;
          w[k] &= n >= 4 ? ~0u : (1u << (8 * n)) - 1u;
        }
        v[u] = make_uint4(w[0], w[1], w[2], w[3]);
      }
      d4[i] = v[u];
    }
  }
  const uint32_t end = l == 0 ? 64u : (l + 63u) & ~63u;  // whole blocks
  for (uint32_t i = nvec + threadIdx.x; i < end / 16; i += blockDim.x) d4[i] = make_uint4(0, 0, 0, 0);
}

// Host-staged latency path: a few messages of at most kHostStageMax bytes in
// pinned host memory (the caller's staging slab), one workgroup each, copied
// into LDS by the workgroup (16 B per lane, eight loads in flight per lane: a couple of PCIe
// round trips), hashed there in quads of lanes (quad_hash_staged), and the
// out_words written straight into pinned host memory -- no H2D / D2H copy
// commands around the launch (they are ~2/3 of a 4 KiB single-file call's
// fixed cost, profiles/r2/latency/).
constexpr uint32_t kHostStageChunks = kHostStageMax / B3_CHUNK_LEN;

__global__ __launch_bounds__(1024) void k_small_host(const uint8_t* __restrict__ arena,
                                                     const uint64_t* __restrict__ off,
                                                     const uint32_t* __restrict__ len,
                                                     uint32_t out_words,
                                                     uint32_t* __restrict__ out_all) {
  extern __shared__ __attribute__((aligned(16))) uint8_t stage[];
  __shared__ __attribute__((aligned(16))) uint32_t cvr[8 * kHostStageChunks];
  const uint32_t m = blockIdx.x;
  const uint32_t l = len[m];
  uint32_t* __restrict__ out = out_all + static_cast<uint64_t>(m) * out_words;
  QuadLane L;
  L.init();
  stage_message(stage, arena + off[m], l);
  __syncthreads();
  uint32_t h0 = 0, h1 = 0;
  quad_hash_staged(L, stage, l, cvr, h0, h1);
  if (threadIdx.x < 4) {  // digest words i and 4 + i
    if (L.i < out_words) out[L.i] = h0;
    if (4 + L.i < out_words) out[4 + L.i] = h1;
  }
}

// Messages of up to 1 MiB (SMALL_MAX_BYTES): each split into 64-chunk groups
// (64 KiB subtrees, complete and power-of-two aligned, so their CVs are nodes
// of BLAKE3's tree), one 256-thread workgroup per group staging its bytes in
// LDS and hashing them in quads; the group CVs go to `scratch`, and the
// workgroup that finishes a message's last group (agent-scope counter) folds
// them with ROOT.  A 1 MiB message: 16 workgroups of 16 dependent
// compressions + 6 levels, then 4 levels, instead of one workgroup whose 16
// waves issue 1024 lanes' compressions on one CU (k_small, ~96 us).  The
// source may be device or pinned host memory (16-B aligned offsets, readable
// up to the next 16 bytes).  scratch: small_split_scratch_bytes(), its
// counters zero (every last workgroup resets its counter); <= 64 messages.
constexpr uint32_t kSplitThreads = 256;
constexpr uint32_t kSplitGroupChunks = 64;
constexpr uint32_t kSplitMaxGroups = SMALL_MAX_BYTES / (kSplitGroupChunks * B3_CHUNK_LEN);
constexpr uint32_t kSplitMaxMsgs = 64;  // scratch: kSplitMaxMsgs counters, then the group CVs
static_assert(kSplitThreads / 4 >= kSplitGroupChunks / 2 && kSplitThreads / 4 >= kSplitMaxGroups / 2,
              "one quad per parent of a first tree level");

__global__ __launch_bounds__(kSplitThreads) void k_small_split(
    const uint8_t* __restrict__ arena, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, uint32_t max_len, uint32_t gmax, uint32_t out_words,
    uint32_t* __restrict__ out, int32_t* __restrict__ status, uint32_t* __restrict__ scratch) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[kSplitGroupChunks * B3_CHUNK_LEN];
  __shared__ __attribute__((aligned(16))) uint32_t cvr[8 * kSplitGroupChunks];
  __shared__ uint32_t s_last;
  const uint32_t m = blockIdx.x / gmax, g = blockIdx.x % gmax, t = threadIdx.x;
  const uint32_t l = len[m];
  const bool ok = l <= max_len && (off[m] & 15u) == 0 && l <= SMALL_MAX_BYTES;
  if (g == 0 && t == 0 && status) status[m] = ok ? 0 : -EINVAL;
  uint32_t* __restrict__ o = out + static_cast<uint64_t>(m) * out_words;
  if (!ok) {
    if (g == 0 && t < out_words) o[t] = 0u;
    return;
  }
  const uint32_t nch = n_chunks_of(l);
  const uint32_t G = (nch + kSplitGroupChunks - 1) / kSplitGroupChunks;
  if (g >= G) return;  // uniform per workgroup
  constexpr uint32_t kGroupBytes = kSplitGroupChunks * B3_CHUNK_LEN;
  const uint32_t glen = min(kGroupBytes, l - g * kGroupBytes);
  QuadLane L;
  L.init();
  stage_message(stage, arena + off[m] + static_cast<uint64_t>(g) * kGroupBytes, glen);
  __syncthreads();
  const bool whole = G == 1;
  uint32_t h0 = 0, h1 = 0;
  quad_chunks(L, stage, glen, g * kSplitGroupChunks, whole, cvr, h0, h1);
  const uint32_t k = n_chunks_of(glen);
  if (!(whole && k == 1)) {
    __syncthreads();
    quad_tree(L, cvr, k, whole ? B3_ROOT : 0u, h0, h1);
  }
  if (!whole) {
    // counters first (fixed place whatever n is: each stays zero between uses)
    uint32_t* cnt = scratch;
    uint32_t* cv = scratch + kSplitMaxMsgs + (static_cast<uint64_t>(m) * kSplitMaxGroups + g) * 8;
    if (t < 4) {
      __hip_atomic_store(cv + L.i, h0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(cv + 4 + L.i, h1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (t == 0) {
      const uint32_t done =
          __hip_atomic_fetch_add(cnt + m, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      s_last = done + 1 == G;
      if (s_last) __hip_atomic_store(cnt + m, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!s_last) return;  // uniform
    // the last group of the message: every group CV is published; fold them
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    const uint32_t* all = scratch + kSplitMaxMsgs + static_cast<uint64_t>(m) * kSplitMaxGroups * 8;
    if (t < 8 * G) cvr[t] = __hip_atomic_load(all + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    quad_tree(L, cvr, G, B3_ROOT, h0, h1);
  }
  if (t < 4) {  // digest words i and 4 + i
    if (L.i < out_words) o[L.i] = h0;
    if (4 + L.i < out_words) o[4 + L.i] = h1;
  }
}

// The resident latency service (internal.hpp SvcMailbox).  Thread 0 polls
// the request number with system-scope acquire loads (the message area and
// the mailbox are coherent pinned memory, so every load reads the host's
// current bytes); the workgroup then hashes the message exactly as
// k_small_host (in quads of lanes) and thread 0 publishes the digest words
// (gathered from the first quad by shuffles), then the request
// number (system-scope release).  Every wave reaches the loop's exit: the
// stop request, the idle deadline and the lifetime deadline are decided by
// thread 0 and broadcast through LDS.
constexpr uint32_t kSvcThreads = 256;
static_assert(kSvcThreads / 4 >= kHostStageChunks / 2, "one quad per parent of the first tree level");

// mb and msg carry no const / __restrict__: the host rewrites both between
// requests within one kernel lifetime, so their loads must not be treated as
// invariant (hoisted or merged across loop iterations).
__global__ __launch_bounds__(kSvcThreads) void k_service(SvcMailbox* mb, uint8_t* msg,
                                                         uint32_t last_seq, uint64_t idle_ticks,
                                                         uint64_t life_ticks) {
  extern __shared__ __attribute__((aligned(16))) uint8_t stage[];
  __shared__ __attribute__((aligned(16))) uint32_t cvr[8 * kHostStageChunks];
  __shared__ uint32_t s_go, s_len, s_words;
  const uint32_t t = threadIdx.x;
  QuadLane L;
  L.init();
  const uint64_t t_start = wall_clock64();
  uint64_t t_last = t_start;
  for (;;) {
    if (t == 0) {
      uint32_t go = 0;
      for (;;) {
        const uint32_t seq = __hip_atomic_load(&mb->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (seq != last_seq) {
          const uint32_t op = __hip_atomic_load(&mb->op, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          go = op == kSvcHash ? seq : 0u;
          s_len = __hip_atomic_load(&mb->len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          s_words = __hip_atomic_load(&mb->out_words, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          if (go == 0) last_seq = seq;  // stop
          break;
        }
        const uint64_t now = wall_clock64();
        if (now - t_last > idle_ticks || now - t_start > life_ticks) break;
        __builtin_amdgcn_s_sleep(2);
      }
      s_go = go;
    }
    __syncthreads();
    const uint32_t go = s_go;
    if (go == 0) break;  // uniform: stop, idle or lifetime deadline
    const uint64_t t_seen = wall_clock64();
    const uint32_t l = min(s_len, kHostStageMax), out_words = min(s_words, 16u);
    stage_message(stage, msg, l);
    __syncthreads();
    const uint64_t t_loaded = wall_clock64();
    uint32_t h0 = 0, h1 = 0;
    quad_hash_staged(L, stage, l, cvr, h0, h1);
    if (t < 64) {  // wave 0: thread 0 gathers the digest from lanes 0..3
      uint32_t dg[8];
#pragma unroll
      for (int w = 0; w < 8; ++w) dg[w] = __shfl(w < 4 ? h0 : h1, w & 3);
      if (t == 0) {
        for (uint32_t w = 0; w < out_words; ++w)
          __hip_atomic_store(&mb->digest[w], w < 8 ? dg[w] : 0u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&mb->t_seen, t_seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&mb->t_loaded, t_loaded, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&mb->t_done, wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&mb->done, go, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        last_seq = go;
      }
    }
    t_last = wall_clock64();
    __syncthreads();  // LDS (stage, cvr, s_*) reused by the next request
  }
  if (t == 0) __hip_atomic_store(&mb->state, kSvcExited, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

hipError_t batch_hash_launch(const uint8_t* arena, uint64_t arena_bytes, const uint64_t* off,
                             const uint32_t* len, uint32_t n, uint32_t max_len,
                             uint32_t out_words, uint8_t* out, int32_t* status,
                             const BatchWork& w, hipStream_t s, KTimer* timer) {
  if (n == 0) return hipSuccess;
  uint32_t* o = reinterpret_cast<uint32_t*>(out);
  const uint32_t nb = std::min<uint32_t>(kSortBlocks, (n + kThreads - 1) / kThreads);
  const uint32_t nh = 2 * kBins * nb;
  const uint64_t cap = w.max_chunks;
  // hist_scan[kBins * nb] = R (start of the fold list), hist_scan[nh] = R + F
  k_plan3<<<nb, kThreads, 0, s>>>(off, len, n, max_len, arena_bytes, w.n_chunks, w.hist, w.grab,
                                  status, out_words, o);
  scan::exclusive(w.n_chunks, n, w.chunk_base, w.block_sums, w.total, s);
  scan::exclusive(w.hist, nh, w.hist, w.hist_sums, nullptr, s);
  k_scatter3<<<nb, kThreads, 0, s>>>(off, len, n, max_len, arena_bytes, cap, w.total, status,
                                     out_words, o, w.chunk_base, w.hist, w.order, w.chunk_msg);
  const uint32_t* d_r = w.hist + static_cast<size_t>(kBins) * nb;
  {
    KScope k(timer, "cas_leaves", s);
    k_leaves3<<<leaves3_grid(), kThreads, 0, s>>>(arena, off, len, w.chunk_msg, w.chunk_base,
                                                  w.total, w.order, d_r, w.grab, w.cvs, out_words,
                                                  o, n, cap);
  }
  {
    KScope k(timer, "cas_fold", s);
    k_fold3<<<(n + kThreads - 1) / kThreads, kThreads, 0, s>>>(len, w.chunk_base, w.order, d_r,
                                                               w.hist + nh, w.cvs, out_words, o,
                                                               w.total, n, cap);
  }
  return hipGetLastError();
}

}  // namespace sdgpu

namespace sdgpu {

size_t small_split_scratch_bytes() {
  return (kSplitMaxMsgs + static_cast<size_t>(kSplitMaxMsgs) * kSplitMaxGroups * 8) * 4;
}

hipError_t small_split_launch(const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                              uint32_t n, uint32_t max_len, uint32_t max_chunks,
                              uint32_t out_words, uint8_t* out, int32_t* status, uint32_t* scratch,
                              hipStream_t s, KTimer* timer) {
  if (n == 0) return hipSuccess;
  if (n > kSplitMaxMsgs || max_chunks > kSmallMaxChunks || !scratch) return hipErrorInvalidValue;
  const uint32_t gmax = std::max<uint32_t>(1, (max_chunks + kSplitGroupChunks - 1) / kSplitGroupChunks);
  KScope k(timer, "cas_small_split", s);
  k_small_split<<<n * gmax, kSplitThreads, 0, s>>>(arena, off, len, max_len, gmax, out_words,
                                                   reinterpret_cast<uint32_t*>(out), status, scratch);
  return hipGetLastError();
}

// Messages in pinned host memory (16-B aligned offsets, readable past `len`
// up to the next 16 bytes; off / len host-visible too), digest words written
// to pinned host memory `h_out` (out_words per message).
hipError_t small_host_launch(const uint8_t* h_arena, const uint64_t* h_off, const uint32_t* h_len,
                             uint32_t n, uint32_t max_len, uint32_t out_words, uint8_t* h_out,
                             hipStream_t s, KTimer* timer) {
  if (n == 0) return hipSuccess;
  if (max_len > kHostStageMax || (reinterpret_cast<uintptr_t>(h_arena) & 15u))
    return hipErrorInvalidValue;
  const uint32_t nch = max_len <= B3_CHUNK_LEN ? 1u : (max_len + B3_CHUNK_LEN - 1) / B3_CHUNK_LEN;
  // quads: >= 64 of them, one per parent of the first tree level
  const uint32_t threads = std::max<uint32_t>(256, (2 * nch + 63) / 64 * 64);
  // whole 64-byte blocks (stage_message zero-pads the last one), at least one
  const size_t lds = std::max<size_t>(64, (static_cast<size_t>(max_len) + 63) / 64 * 64);
  // the dynamic-LDS limit is a per-device attribute of the loaded kernel: set
  // once for each device this process launches on
  static std::atomic<uint64_t> attr_set{0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  const uint64_t bit = 1ull << (dev & 63);
  if (!(attr_set.load(std::memory_order_acquire) & bit)) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_small_host),
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             static_cast<int>(kHostStageMax + 16));
    if (e != hipSuccess) return e;
    attr_set.fetch_or(bit, std::memory_order_release);
  }
  KScope k(timer, "cas_small_host", s);
  k_small_host<<<n, threads, lds, s>>>(h_arena, h_off, h_len, out_words,
                                       reinterpret_cast<uint32_t*>(h_out));
  return hipGetLastError();
}

}  // namespace sdgpu

namespace sdgpu {

hipError_t service_launch(SvcMailbox* mb, const uint8_t* msg, uint32_t last_seq,
                          uint64_t idle_ticks, uint64_t life_ticks, hipStream_t s) {
  static std::atomic<uint64_t> attr_set{0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  const uint64_t bit = 1ull << (dev & 63);
  if (!(attr_set.load(std::memory_order_acquire) & bit)) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_service),
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             static_cast<int>(kHostStageMax + 16));
    if (e != hipSuccess) return e;
    attr_set.fetch_or(bit, std::memory_order_release);
  }
  k_service<<<1, kSvcThreads, kHostStageMax + 16, s>>>(mb, const_cast<uint8_t*>(msg), last_seq,
                                                        idle_ticks, life_ticks);
  return hipGetLastError();
}

}  // namespace sdgpu
