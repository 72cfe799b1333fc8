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
// K1 variant for A/B runs in one process (SDGPU_K1_VARIANT: 0 plain, 1 pipelined).
int k1_variant() {
  const char* v = getenv("SDGPU_K1_VARIANT");
  return v ? atoi(v) : 0;
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

}  // namespace

hipError_t batch_hash_launch(const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                             uint32_t n, uint32_t max_len, uint32_t out_words, uint8_t* out,
                             int32_t* status, const BatchWork& w, hipStream_t s,
                             KTimer* timer) {
  if (n == 0) return hipSuccess;
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
