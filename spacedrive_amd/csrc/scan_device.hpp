// Exclusive prefix sum of u32 counts on the device (reduce-then-scan, three
// launches, no host synchronisation).  Used by the K1 planner and the K4/K6
// radix partitions.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sdgpu {
namespace scan {

constexpr int kThreads = 256;
constexpr uint32_t kTile = 1024;  // elements per tile (4 per thread)

inline uint32_t tiles_for(uint64_t n) { return static_cast<uint32_t>((n + kTile - 1) / kTile); }

__global__ __launch_bounds__(kThreads) static void k_tiles(const uint32_t* __restrict__ in,
                                                           uint64_t n, uint32_t* __restrict__ out,
                                                           uint32_t* __restrict__ tile_sums) {
  __shared__ uint32_t wsum[kThreads / 64];
  const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kTile + threadIdx.x * 4;
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint32_t v[4];
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[k] = base + k < n ? in[base + k] : 0u;
    s += v[k];
  }
  // wave shuffles, then the 4 wave totals (one barrier instead of 16)
  uint32_t inc = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d);
    if (lane >= static_cast<uint32_t>(d)) inc += o;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kThreads / 64; ++k) {
    const uint32_t x = wsum[k];
    pre += static_cast<uint32_t>(k) < w ? x : 0u;
    tot += x;
  }
  uint32_t run = pre + inc - s;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (base + k < n) out[base + k] = run;
    run += v[k];
  }
  if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
}

// Single block of kSumThreads: exclusive scan of the tile sums (wave shuffles,
// then the 16 wave totals); writes the grand total to out[n] (if
// out_total_slot) and *total (if non-null).
constexpr int kSumThreads = 1024;
__global__ __launch_bounds__(kSumThreads) static void k_sums(uint32_t* __restrict__ tile_sums,
                                                             uint32_t ntiles,
                                                             uint32_t* __restrict__ out_total_slot,
                                                             uint32_t* __restrict__ total) {
  __shared__ uint32_t wsum[kSumThreads / 64];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint32_t carry = 0;
  for (uint32_t b0 = 0; b0 < ntiles; b0 += kSumThreads) {
    const uint32_t i = b0 + threadIdx.x;
    const uint32_t v = i < ntiles ? tile_sums[i] : 0u;
    uint32_t inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = __shfl_up(inc, d);
      if (lane >= static_cast<uint32_t>(d)) inc += o;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t pre = 0, blk = 0;
    for (uint32_t k = 0; k < kSumThreads / 64; ++k) {
      const uint32_t x = wsum[k];
      pre += k < w ? x : 0u;
      blk += x;
    }
    if (i < ntiles) tile_sums[i] = carry + pre + inc - v;
    carry += blk;
    __syncthreads();  // wsum is rewritten by the next chunk
  }
  if (threadIdx.x == 0) {
    if (out_total_slot) *out_total_slot = carry;
    if (total) *total = carry;
  }
}

__global__ __launch_bounds__(kThreads) static void k_add(uint32_t* __restrict__ out, uint64_t n,
                                                         const uint32_t* __restrict__ tile_sums) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (i < n) out[i] += tile_sums[i / kTile];
}

// out[0..n) = exclusive scan of in[0..n); out[n] = total (out must hold n+1);
// tile_sums must hold tiles_for(n) entries.  in may alias out.
inline void exclusive(const uint32_t* in, uint64_t n, uint32_t* out, uint32_t* tile_sums,
                      uint32_t* total, hipStream_t s) {
  const uint32_t tiles = tiles_for(n);
  if (tiles == 0) {
    (void)hipMemsetAsync(out, 0, sizeof(uint32_t), s);
    if (total) (void)hipMemsetAsync(total, 0, sizeof(uint32_t), s);
    return;
  }
  k_tiles<<<tiles, kThreads, 0, s>>>(in, n, out, tile_sums);
  k_sums<<<1, kSumThreads, 0, s>>>(tile_sums, tiles, out + n, total);
  k_add<<<static_cast<uint32_t>((n + kThreads - 1) / kThreads), kThreads, 0, s>>>(out, n,
                                                                                   tile_sums);
}

}  // namespace scan
}  // namespace sdgpu
