// Downstream consumers of the grouping, on the device.
//
// Orphan remover (/root/reference/core/src/object/orphan_remover.rs:57-90):
// Objects with no file_path pointing at them (`object::file_paths::none`) are
// found 512 at a time and deleted.  Here: one pass marks every Object id that
// some file_path references (a byte per id, plain stores: marking is
// idempotent, so no atomics are needed), a second pass keeps
// the unreferenced ids of the Object list, in list order (4096-id tiles:
// count, one scan of the tile counts, in-tile ballot ranks), ready for the
// caller's delete batches.
//
// Thumbnail shards (/root/reference/core/src/object/media/thumbnail/shard.rs:4-8):
// a thumbnail lives in directory cas_id[0..2], the first digest byte, i.e. the
// low byte of the little-endian cas key.  Here: a batch's rows counting-sorted
// by that byte (256 directories), so a thumbnailer writes each directory's
// files together; counts per directory alongside.
#include "internal.hpp"
#include "scan_device.hpp"

namespace sdgpu {

namespace {

constexpr int kThreads = 256;

uint32_t grid_for(uint64_t n, uint64_t per = kThreads) {
  const uint64_t g = (n + per - 1) / per;
  return static_cast<uint32_t>(g == 0 ? 1 : (g < 65535 ? g : 65535));
}

// mark[o] = 1: some file_path references Object o (negative = NULL object_id).
// Workgroups go to the 8 XCDs round-robin (block b on XCD b % 8), so block b
// marks only the ids of range b % 8 and every XCD's stores stay inside one
// eighth of the map, which its L2 holds (10 M ids: 1.25 MB of 4 MB) until the
// lines leave whole.  Every file_path id is read once per range (8 times in
// all, the repeats from the shared last-level cache): one scattered byte store
// per row into the whole map left each store a partial-line write of its own.
// Fewer ranges (XCDs sharing a range, fewer re-reads of the file_path ids)
// measured slower: 4 / 2 / 1 ranges 0.198 / 0.230 / 0.230 ms per call against
// 0.170 ms with 8 (profiles/r4/consumers_ab/).
constexpr uint32_t kMarkRanges = 8;
__global__ __launch_bounds__(kThreads) void k_mark(const int32_t* __restrict__ fp_obj, uint64_t n,
                                                   uint8_t* __restrict__ mark, uint32_t max_id,
                                                   uint32_t span, uint32_t ranges) {
  const uint32_t r = blockIdx.x % ranges, g = blockIdx.x / ranges;
  const uint32_t lo = r * span;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x / ranges) * kThreads * 4;
  for (uint64_t i0 = static_cast<uint64_t>(g) * kThreads * 4 + threadIdx.x; i0 < n; i0 += stride) {
    int32_t o[4];
    // loads unconditional (clamped), the tail masked after: a guarded load
    // made the compiler wait out each load's latency in turn
#pragma unroll
    for (int u = 0; u < 4; ++u) o[u] = fp_obj[min(i0 + static_cast<uint64_t>(u) * kThreads, n - 1)];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i0 + static_cast<uint64_t>(u) * kThreads >= n) o[u] = -1;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t d = static_cast<uint32_t>(o[u]) - lo;  // negative ids wrap past span
      if (o[u] >= 0 && d < span && static_cast<uint32_t>(o[u]) <= max_id) mark[o[u]] = 1;
    }
  }
}

// Object o is an orphan: no file_path marked it (ids past max_id are never
// marked).  m = mark[o] read beforehand for every id (mark_of), so the kRows
// gathers of a thread are in flight together.
__device__ __forceinline__ bool orphan(int32_t o, uint8_t m, uint32_t max_id) {
  return o >= 0 && (static_cast<uint32_t>(o) > max_id || m == 0);
}
__device__ __forceinline__ uint8_t mark_of(int32_t o, const uint8_t* mark, uint32_t max_id) {
  const uint32_t c = o < 0 ? 0u : min(static_cast<uint32_t>(o), max_id);  // any in-range byte
  return mark[c];
}

// The Object list in tiles of kORows x kThreads ids: id tile + k * kThreads + t
// (coalesced), and (k, t) order is list order, so in-tile ranks from
// per-(k, wave) ballots keep the orphans in list order.
constexpr int kORows = 16;
constexpr uint64_t kOTile = static_cast<uint64_t>(kORows) * kThreads;
constexpr int kOWaves = kThreads / 64;

// the kORows ids of a thread (loads unconditional, tail masked after), then
// their mark bytes
__device__ __forceinline__ void obj_tile(const int32_t* __restrict__ obj, uint64_t n, uint64_t tile,
                                         const uint8_t* __restrict__ bits, uint32_t max_id,
                                         int32_t (&o)[kORows], uint8_t (&m)[kORows]) {
#pragma unroll
  for (int k = 0; k < kORows; ++k) o[k] = obj[min(tile + k * kThreads + threadIdx.x, n - 1)];
#pragma unroll
  for (int k = 0; k < kORows; ++k)
    if (tile + k * kThreads + threadIdx.x >= n) o[k] = -1;
#pragma unroll
  for (int k = 0; k < kORows; ++k) m[k] = mark_of(o[k], bits, max_id);
}

// orphans per tile
__global__ __launch_bounds__(kThreads) void k_orphan_count(const int32_t* __restrict__ obj,
                                                           uint64_t n,
                                                           const uint8_t* __restrict__ bits,
                                                           uint32_t max_id,
                                                           uint32_t* __restrict__ cnt) {
  __shared__ uint32_t sw[kOWaves];
  const uint64_t tile = static_cast<uint64_t>(blockIdx.x) * kOTile;
  int32_t o[kORows];
  uint8_t m[kORows];
  obj_tile(obj, n, tile, bits, max_id, o, m);
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < kORows; ++k) c += orphan(o[k], m[k], max_id) ? 1u : 0u;
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d);
  if (__lane_id() == 0) sw[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < kOWaves; ++w) t += sw[w];
    cnt[blockIdx.x] = t;
  }
}

// stable compaction: tile b writes its orphans from the scanned offset, in order
__global__ __launch_bounds__(kThreads) void k_orphan_write(const int32_t* __restrict__ obj,
                                                           uint64_t n,
                                                           const uint8_t* __restrict__ bits,
                                                           uint32_t max_id,
                                                           const uint32_t* __restrict__ offs,
                                                           int32_t* __restrict__ out) {
  __shared__ uint32_t off[kORows][kOWaves];
  const uint64_t tile = static_cast<uint64_t>(blockIdx.x) * kOTile;
  const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  int32_t o[kORows];
  uint8_t m[kORows];
  uint32_t pre[kORows], f = 0;
  obj_tile(obj, n, tile, bits, max_id, o, m);
#pragma unroll
  for (int k = 0; k < kORows; ++k) {
    const bool is = orphan(o[k], m[k], max_id);
    f |= (is ? 1u : 0u) << k;
    const uint64_t b = __ballot(is);
    pre[k] = __popcll(b & lt);
    if (lane == 0) off[k][w] = __popcll(b);
  }
  __syncthreads();
  static_assert(kORows * kOWaves == 64, "one wave scans the (row step, wave) counts");
  if (threadIdx.x < 64) {  // (k, wave) order -- k-major, the array's order -- is list order
    uint32_t* f = &off[0][0];
    const uint32_t a = f[lane];
    uint32_t inc = a;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t x = __shfl_up(inc, d);
      if (lane >= static_cast<uint32_t>(d)) inc += x;
    }
    f[lane] = offs[blockIdx.x] + inc - a;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kORows; ++k)
    if (f >> k & 1u) out[off[k][w] + pre[k]] = o[k];
}

// ---- thumbnail shards -----------------------------------------------------------
constexpr uint32_t kShardBins = 256;
// 1024 tiles (4 per CU): 256 left one workgroup per CU walking 16 serial
// rounds of its tile (0.11 ms for 1 M rows, r4x trace)
constexpr uint32_t kShardBlocks = 1024;

__device__ __forceinline__ void tile(uint64_t n, uint64_t& t0, uint64_t& t1) {
  const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
  t0 = min<uint64_t>(n, per * blockIdx.x);
  t1 = min<uint64_t>(n, t0 + per);
}

__global__ __launch_bounds__(kThreads) void k_thumb_hist(const uint8_t* __restrict__ cas8,
                                                         const uint8_t* __restrict__ valid,
                                                         uint64_t n, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[kShardBins];
  h[threadIdx.x] = 0;
  __syncthreads();
  uint64_t t0, t1;
  tile(n, t0, t1);
  for (uint64_t i = t0 + threadIdx.x; i < t1; i += kThreads)
    if (!valid || valid[i]) atomicAdd(&h[cas8[8 * i]], 1u);
  __syncthreads();
  hist[static_cast<uint64_t>(threadIdx.x) * gridDim.x + blockIdx.x] = h[threadIdx.x];
}

// Stable within a block's tile: one round of kThreads rows at a time.  A row's
// place in its bin = cursor + rows with the same byte in earlier waves of the
// round + earlier lanes of its own wave with the same byte.  The lanes holding
// the same byte are found with 8 ballots, one per bit of the byte (round 5;
// a ballot per distinct byte in the wave took ~57 passes for random bytes).
__global__ __launch_bounds__(kThreads) void k_thumb_scatter(const uint8_t* __restrict__ cas8,
                                                            const uint8_t* __restrict__ valid,
                                                            uint64_t n,
                                                            const uint32_t* __restrict__ offs,
                                                            uint32_t* __restrict__ order) {
  constexpr uint32_t kWaves = kThreads / 64;
  __shared__ uint32_t cur[kShardBins];
  __shared__ uint32_t wcnt[kWaves][kShardBins];
  static_assert(kShardBins == kThreads, "one cursor per thread");
  cur[threadIdx.x] = offs[static_cast<uint64_t>(threadIdx.x) * gridDim.x + blockIdx.x];
  const uint32_t lane = __lane_id(), wave = threadIdx.x >> 6;
  uint64_t t0, t1;
  tile(n, t0, t1);
  for (uint64_t i0 = t0; i0 < t1; i0 += kThreads) {  // uniform trip count
    const uint64_t i = i0 + threadIdx.x;
    const bool v = i < t1 && (!valid || valid[i]);
    const uint32_t b = i < t1 ? cas8[8 * i] : 0u;
    for (uint32_t k = threadIdx.x; k < kWaves * kShardBins; k += kThreads) (&wcnt[0][0])[k] = 0;
    __syncthreads();
    uint64_t peers = __ballot(v);  // the valid lanes whose byte equals this lane's
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const bool bit = (b >> k) & 1u;
      const uint64_t mk = __ballot(bit);
      peers &= bit ? mk : ~mk;
    }
    const uint32_t rank = static_cast<uint32_t>(__popcll(peers & ((1ull << lane) - 1ull)));
    if (v && rank == 0) wcnt[wave][b] = static_cast<uint32_t>(__popcll(peers));
    __syncthreads();
    if (v) {
      uint32_t p = cur[b] + rank;
      for (uint32_t w = 0; w < wave; ++w) p += wcnt[w][b];
      order[p] = static_cast<uint32_t>(i);
    }
    __syncthreads();
    uint32_t add = 0;
#pragma unroll
    for (uint32_t w = 0; w < kWaves; ++w) add += wcnt[w][threadIdx.x];
    cur[threadIdx.x] += add;
    __syncthreads();
  }
}

__global__ void k_thumb_counts(const uint32_t* __restrict__ offs, uint32_t* __restrict__ counts) {
  const uint32_t b = threadIdx.x;
  counts[b] = offs[static_cast<uint64_t>(b + 1) * kShardBlocks] -
              offs[static_cast<uint64_t>(b) * kShardBlocks];
}

}  // namespace

size_t orphan_workspace_bytes(uint64_t n_obj, uint32_t max_id) {
  const uint64_t map = (static_cast<uint64_t>(max_id) + 1 + 255) / 256 * 256;
  const uint64_t blocks = (n_obj + kOTile - 1) / kOTile;
  return map + 4 * (blocks + 1) + 4 * (scan::tiles_for(blocks) + 1) + 1024;
}

hipError_t orphan_objects_launch(const int32_t* obj, uint64_t n_obj, const int32_t* fp_obj,
                                 uint64_t n_fp, uint32_t max_id, int32_t* out, uint32_t* d_count,
                                 void* ws, hipStream_t s) {
  const uint64_t map = (static_cast<uint64_t>(max_id) + 1 + 255) / 256 * 256;
  const uint64_t blocks = (n_obj + kOTile - 1) / kOTile;
  uint8_t* bits = static_cast<uint8_t*>(ws);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(bits + map);
  uint32_t* tiles = cnt + blocks + 1;
  (void)hipMemsetAsync(bits, 0, map, s);
  if (n_fp) {
    constexpr uint32_t ranges = kMarkRanges;
    const uint32_t span = static_cast<uint32_t>((static_cast<uint64_t>(max_id) + ranges) / ranges);
    const uint64_t per = (n_fp + 4 * kThreads - 1) / (4 * kThreads);  // 1024-row groups
    const uint32_t groups = static_cast<uint32_t>(per < 256 ? per : 256) * (8 / ranges);
    k_mark<<<groups * ranges, kThreads, 0, s>>>(fp_obj, n_fp, bits, max_id, span, ranges);
  }
  if (blocks) {
    k_orphan_count<<<static_cast<uint32_t>(blocks), kThreads, 0, s>>>(obj, n_obj, bits, max_id,
                                                                      cnt);
    scan::exclusive(cnt, blocks, cnt, tiles, d_count, s);
    k_orphan_write<<<static_cast<uint32_t>(blocks), kThreads, 0, s>>>(obj, n_obj, bits, max_id,
                                                                      cnt, out);
  } else {
    (void)hipMemsetAsync(d_count, 0, 4, s);
  }
  return hipGetLastError();
}

size_t thumb_workspace_bytes() {
  const uint64_t nh = static_cast<uint64_t>(kShardBins) * kShardBlocks;
  return 4 * (nh + 1) + 4 * (scan::tiles_for(nh) + 1) + 512;
}

hipError_t thumbnail_shards_launch(const uint8_t* cas8, const uint8_t* valid, uint64_t n,
                                   uint32_t* order, uint32_t* counts, void* ws, hipStream_t s) {
  const uint64_t nh = static_cast<uint64_t>(kShardBins) * kShardBlocks;
  uint32_t* hist = static_cast<uint32_t*>(ws);
  uint32_t* tiles = hist + nh + 1;
  k_thumb_hist<<<kShardBlocks, kThreads, 0, s>>>(cas8, valid, n, hist);
  scan::exclusive(hist, nh, hist, tiles, nullptr, s);
  k_thumb_scatter<<<kShardBlocks, kThreads, 0, s>>>(cas8, valid, n, hist, order);
  k_thumb_counts<<<1, kShardBins, 0, s>>>(hist, counts);
  return hipGetLastError();
}

}  // namespace sdgpu
