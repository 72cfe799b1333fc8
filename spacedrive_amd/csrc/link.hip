// K7: Object link batch -- the write set of identifier_job_step as dense arrays.
//
// Replaces the per-100-row database decisions of
// /root/reference/core/src/object/file_identifier/mod.rs:189-333: every row
// whose cas_id matched an existing Object is connected to it (`file_path`
// update + `object::connect`, mod.rs:189-225) and every other row gets a new
// Object (`object::create_many` + connect, mod.rs:243-333).  Given the grouping
// rep[] (rank of the row whose Object a row joins; rep == own rank = creates),
// one pass compacts the whole batch into
//   create[0..C)            ranks of the rows that create an Object, ascending
//   link_row/link_obj[0..L) (row rank, creator rank) of the rows that connect
// so the host issues one create_many + one batched connect per large batch
// instead of 4-5 queries per 100 rows.  Rows with valid == 0 (metadata or
// hash failed, mod.rs:113,127) are in neither list: they stay orphans.
// HBM-bound: reads 9 B/row twice, writes 4 B per created row and 8 B per
// linked row; three launches + a scan of two counters per 4096-row tile.
#include "internal.hpp"
#include "scan_device.hpp"

namespace sdgpu {

namespace {

// A block takes a tile of kTile rows: row tile + k * kThreads + t for k in
// [0, kRows) -- coalesced loads, and (k, t) order is row order, so in-block
// ranks from per-(k, wave) ballots keep both lists in row order.
constexpr int kThreads = 256;
constexpr int kRows = 16;
constexpr uint32_t kTile = kThreads * kRows;
constexpr int kWaves = kThreads / 64;

struct LinkRow {
  uint32_t r, p;
  bool c, l;  // creates an Object / connects to one
};

// The kRows rows of a thread: every load issued first and unconditionally
// (rows past the end read row n - 1; a null rank / valid array is replaced by
// the rep array, whose lines are loaded anyway), the rows resolved at use.  A
// guarded load -- `i < n`, or a select on the null pointer -- made the
// compiler branch around each load and wait out its latency in turn.
struct LinkRows {
  uint32_t a[kRows], p[kRows], b[kRows];
};

__device__ __forceinline__ void link_load(const uint32_t* __restrict__ rep,
                                          const uint32_t* __restrict__ rank,
                                          const uint8_t* __restrict__ valid, uint64_t n,
                                          uint64_t tile, LinkRows& q) {
  const uint32_t* rs = rank ? rank : rep;
#pragma unroll
  for (int k = 0; k < kRows; ++k) {
    const uint64_t i = tile + k * kThreads + threadIdx.x;
    const uint64_t j = i < n ? i : n - 1;
    q.p[k] = rep[j];
    q.a[k] = rs[j];
    // null valid: a byte of row j's own rep word (rep indexed as bytes by j
    // would read another line, the first quarter of the rep array)
    q.b[k] = *(valid ? valid + j : reinterpret_cast<const uint8_t*>(rep + j));
  }
}

__device__ __forceinline__ LinkRow link_row(const LinkRows& q, int k, const uint32_t* rank,
                                            const uint8_t* valid, uint32_t first_rank, uint64_t n,
                                            uint64_t i) {
  LinkRow x;
  x.r = rank ? q.a[k] : first_rank + static_cast<uint32_t>(i);
  x.p = q.p[k];
  const bool v = i < n && (!valid || (q.b[k] & 0xFFu) != 0);
  x.c = v && x.p == x.r;
  x.l = v && x.p != x.r;
  return x;
}

// Creators and connectors per tile: cnt[blk] and cnt[nb + blk].
__global__ __launch_bounds__(kThreads) void k_link_count(const uint32_t* __restrict__ rep,
                                                         const uint32_t* __restrict__ rank,
                                                         const uint8_t* __restrict__ valid,
                                                         uint32_t first_rank, uint64_t n,
                                                         uint32_t nb, uint32_t* __restrict__ cnt) {
  __shared__ uint32_t sc[kWaves], sl[kWaves];
  const uint64_t tile = static_cast<uint64_t>(blockIdx.x) * kTile;
  uint32_t c = 0, l = 0;
  LinkRows q;
  link_load(rep, rank, valid, n, tile, q);
#pragma unroll
  for (int k = 0; k < kRows; ++k) {
    const LinkRow x = link_row(q, k, rank, valid, first_rank, n, tile + k * kThreads + threadIdx.x);
    c += x.c;
    l += x.l;
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    c += __shfl_xor(c, d);
    l += __shfl_xor(l, d);
  }
  if (__lane_id() == 0) {
    sc[threadIdx.x >> 6] = c;
    sl[threadIdx.x >> 6] = l;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t tc = 0, tl = 0;
    for (int w = 0; w < kWaves; ++w) {
      tc += sc[w];
      tl += sl[w];
    }
    cnt[blockIdx.x] = tc;
    cnt[nb + blockIdx.x] = tl;
  }
}

// cnt = exclusive scan over [C counts | L counts] (cnt[2 nb] = total): tile
// blk writes its creators from cnt[blk], its connectors from cnt[nb + blk] - C.
__global__ __launch_bounds__(kThreads) void k_link_write(
    const uint32_t* __restrict__ rep, const uint32_t* __restrict__ rank,
    const uint8_t* __restrict__ valid, uint32_t first_rank, uint64_t n, uint32_t nb,
    const uint32_t* __restrict__ cnt, uint32_t* __restrict__ create, uint32_t* __restrict__ link_row_out,
    uint32_t* __restrict__ link_obj, uint32_t* __restrict__ d_counts) {
  __shared__ uint32_t oc[kRows][kWaves], ol[kRows][kWaves];
  const uint64_t tile = static_cast<uint64_t>(blockIdx.x) * kTile;
  const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  const uint32_t total_c = cnt[nb];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    d_counts[0] = total_c;
    d_counts[1] = cnt[2 * static_cast<uint64_t>(nb)] - total_c;
  }
  LinkRow x[kRows];
  uint32_t pc[kRows], pl[kRows];
  LinkRows q;
  link_load(rep, rank, valid, n, tile, q);
#pragma unroll
  for (int k = 0; k < kRows; ++k) {
    x[k] = link_row(q, k, rank, valid, first_rank, n, tile + k * kThreads + threadIdx.x);
    const uint64_t bc = __ballot(x[k].c), bl = __ballot(x[k].l);
    pc[k] = __popcll(bc & lt);
    pl[k] = __popcll(bl & lt);
    if (lane == 0) {
      oc[k][w] = __popcll(bc);
      ol[k][w] = __popcll(bl);
    }
  }
  __syncthreads();
  static_assert(kRows * kWaves == 64, "one wave scans the (row step, wave) counts");
  if (threadIdx.x < 64) {  // (k, wave) order -- k-major, the array's order -- is row order
    uint32_t* fc = &oc[0][0];
    uint32_t* fl = &ol[0][0];
    const uint32_t a = fc[lane], b = fl[lane];
    uint32_t ic = a, il = b;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t xc = __shfl_up(ic, d), xl = __shfl_up(il, d);
      if (lane >= static_cast<uint32_t>(d)) {
        ic += xc;
        il += xl;
      }
    }
    fc[lane] = cnt[blockIdx.x] + ic - a;
    fl[lane] = cnt[nb + blockIdx.x] - total_c + il - b;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kRows; ++k) {
    if (x[k].c) create[oc[k][w] + pc[k]] = x[k].r;
    if (x[k].l) {
      const uint32_t q = ol[k][w] + pl[k];
      link_row_out[q] = x[k].r;
      link_obj[q] = x[k].p;
    }
  }
}

inline uint32_t link_tiles(uint64_t n) { return static_cast<uint32_t>((n + kTile - 1) / kTile); }

// Keyless creators of the fused grouping (sdgpu_group_link_device): rows with
// no cas_id that are valid (empty files: their own Object, mod.rs:238-239) are
// not in the bucket records, so they are listed here, in row order, after the
// keyed entries: who[K + t] = rank of the t-th such row, K = counts[2] (the
// keyed total the group kernel stored).  A thread takes 16 consecutive rows
// (one 16-B load of has_key and of valid); 4096-row tiles, counted, scanned,
// written.
constexpr int kKlRows = 16;
constexpr uint32_t kKlTile = kThreads * kKlRows;

__device__ __forceinline__ uint32_t keyless_mask(const uint8_t* __restrict__ has,
                                                 const uint8_t* __restrict__ valid, uint64_t n,
                                                 uint64_t i0) {
  uint32_t m = 0;
  const bool aligned = (reinterpret_cast<uintptr_t>(has) & 15u) == 0 &&
                       (reinterpret_cast<uintptr_t>(valid) & 15u) == 0;
  if (aligned && i0 + kKlRows <= n) {
    const uint4 h = *reinterpret_cast<const uint4*>(has + i0);
    const uint4 v = valid ? *reinterpret_cast<const uint4*>(valid + i0) : make_uint4(~0u, ~0u, ~0u, ~0u);
    const uint32_t hw[4] = {h.x, h.y, h.z, h.w}, vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < kKlRows; ++k) {
      const uint32_t hb = (hw[k >> 2] >> (8 * (k & 3))) & 0xFFu;
      const uint32_t vb = (vw[k >> 2] >> (8 * (k & 3))) & 0xFFu;
      m |= static_cast<uint32_t>(hb == 0 && vb != 0) << k;
    }
  } else {
    for (int k = 0; k < kKlRows && i0 + k < n; ++k)
      m |= static_cast<uint32_t>(has[i0 + k] == 0 && (!valid || valid[i0 + k] != 0)) << k;
  }
  return m;
}

__global__ __launch_bounds__(kThreads) void k_keyless_count(const uint8_t* __restrict__ has,
                                                            const uint8_t* __restrict__ valid,
                                                            uint64_t n, uint32_t* __restrict__ cnt) {
  __shared__ uint32_t sc[kWaves];
  const uint64_t i0 = static_cast<uint64_t>(blockIdx.x) * kKlTile + threadIdx.x * kKlRows;
  uint32_t c = __popc(keyless_mask(has, valid, n, i0));
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d);
  if (__lane_id() == 0) sc[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < kWaves; ++w) t += sc[w];
    cnt[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(kThreads) void k_keyless_write(
    const uint8_t* __restrict__ has, const uint8_t* __restrict__ valid, const uint32_t* __restrict__ rank,
    uint32_t first_rank, uint64_t n, uint32_t nb, const uint32_t* __restrict__ cnt,
    uint32_t* __restrict__ who, uint32_t* __restrict__ counts) {
  __shared__ uint32_t sw[kWaves];
  const uint64_t i0 = static_cast<uint64_t>(blockIdx.x) * kKlTile + threadIdx.x * kKlRows;
  const uint32_t K = counts[2];
  uint32_t m = keyless_mask(has, valid, n, i0);
  const uint32_t c = __popc(m);
  uint32_t inc = c;
  const uint32_t lane = __lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d);
    if (lane >= static_cast<uint32_t>(d)) inc += o;
  }
  if (lane == 63) sw[threadIdx.x >> 6] = inc;
  __syncthreads();
  uint32_t pos = K + cnt[blockIdx.x] + inc - c;
  for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w) pos += sw[w];
  while (m) {
    const int k = __ffs(m) - 1;
    m &= m - 1;
    const uint64_t i = i0 + k;
    who[pos++] = rank ? rank[i] : first_rank + static_cast<uint32_t>(i);
  }
  if (blockIdx.x == nb - 1 && threadIdx.x == 0) {
    const uint32_t total = cnt[nb];
    counts[0] += total;
    counts[2] = K + total;
  }
}

}  // namespace

size_t keyless_workspace_bytes(uint64_t n) {
  const uint64_t m = (n + kKlTile - 1) / kKlTile;
  return ((m + 1) * 4 + 255) / 256 * 256 + ((scan::tiles_for(m) + 1) * 4 + 255) / 256 * 256;
}

hipError_t keyless_list_launch(const uint8_t* has, const uint8_t* valid, const uint32_t* rank,
                               uint32_t first_rank, uint64_t n, uint32_t* who, uint32_t* counts,
                               void* ws, hipStream_t s, KTimer* timer) {
  if (n == 0 || !has) return hipSuccess;  // every row keyed: nothing to add
  const uint32_t nb = static_cast<uint32_t>((n + kKlTile - 1) / kKlTile);
  uint8_t* b = static_cast<uint8_t*>(ws);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(b);
  uint32_t* tiles = reinterpret_cast<uint32_t*>(b + ((nb + 1) * 4ull + 255) / 256 * 256);
  KScope k(timer, "keyless_list", s);
  k_keyless_count<<<nb, kThreads, 0, s>>>(has, valid, n, cnt);
  scan::exclusive(cnt, nb, cnt, tiles, nullptr, s);
  k_keyless_write<<<nb, kThreads, 0, s>>>(has, valid, rank, first_rank, n, nb, cnt, who, counts);
  return hipGetLastError();
}

size_t link_workspace_bytes(uint64_t n) {
  const uint64_t m = 2ull * link_tiles(n);
  return ((m + 1) * 4 + 255) / 256 * 256 + ((scan::tiles_for(m) + 1) * 4 + 255) / 256 * 256;
}

// Two passes over the rows (count per tile, then rank and write), one scan of
// the 2 x tiles counts in between: ~18 B read per row plus the lists written.
hipError_t link_batch_launch(const uint32_t* rep, const uint32_t* rank, const uint8_t* valid,
                             uint32_t first_rank, uint64_t n, uint32_t* create, uint32_t* link_row,
                             uint32_t* link_obj, uint32_t* d_counts, void* ws, hipStream_t s,
                             KTimer* timer) {
  if (n == 0) return hipMemsetAsync(d_counts, 0, 2 * sizeof(uint32_t), s);
  const uint32_t nb = link_tiles(n);
  const uint64_t m = 2ull * nb;
  uint8_t* b = static_cast<uint8_t*>(ws);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(b);
  uint32_t* tiles = reinterpret_cast<uint32_t*>(b + ((m + 1) * 4 + 255) / 256 * 256);
  KScope k(timer, "link_batch", s);
  k_link_count<<<nb, kThreads, 0, s>>>(rep, rank, valid, first_rank, n, nb, cnt);
  scan::exclusive(cnt, m, cnt, tiles, nullptr, s);
  k_link_write<<<nb, kThreads, 0, s>>>(rep, rank, valid, first_rank, n, nb, cnt, create, link_row,
                                       link_obj, d_counts);
  return hipGetLastError();
}

}  // namespace sdgpu
