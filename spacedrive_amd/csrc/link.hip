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

// Entries of the fused write set that are not in the bucket records
// (sdgpu_group_link_device), appended in row order after the keyed entries
// (who[K + t], K = counts[2], the keyed total the group kernel stored):
//   * valid rows without a cas_id (empty files: their own Objects,
//     mod.rs:238-239): who = rank;
//   * with an Object index, the keyed rows the probe decided (grouped[i] == 0:
//     their cas_id belongs to an Object that existed before the batch,
//     mod.rs:189-225): who = rank | SDGPU_LINKED, obj = the probe's rep -- or
//     who = rank when the probe kept the row's own Object (same chunk).
// A thread takes 16 consecutive rows (16-B loads of has_key / valid /
// grouped); 4096-row tiles.  Three launches: k_extra_count (entries and
// linked entries per segment of tiles), k_extra_scan (ONE block: the
// segments' offsets, and
// counts[] settled from the totals -- no same-address atomics, which
// serialised at ~5 ns each over 24 k tiles at 100 M rows), k_extra_write.
constexpr int kKlRows = 16;
constexpr uint32_t kKlTile = kThreads * kKlRows;
constexpr uint32_t kLinkedBit = 0x80000000u;  // SDGPU_LINKED

__device__ __forceinline__ uint32_t bytes16_mask(const uint8_t* __restrict__ p, uint64_t n,
                                                 uint64_t i0, bool aligned, uint32_t absent) {
  if (!p) return absent;
  uint32_t m = 0;
  if (aligned && i0 + kKlRows <= n) {
    const uint4 h = *reinterpret_cast<const uint4*>(p + i0);
    const uint32_t hw[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
    for (int k = 0; k < kKlRows; ++k)
      m |= static_cast<uint32_t>(((hw[k >> 2] >> (8 * (k & 3))) & 0xFFu) != 0) << k;
  } else {
    for (int k = 0; k < kKlRows && i0 + k < n; ++k) m |= static_cast<uint32_t>(p[i0 + k] != 0) << k;
  }
  return m;
}

// bit k: row i0 + k is an extra entry; h: bit k = row i0 + k is keyed
__device__ __forceinline__ uint32_t extra_mask(const uint8_t* __restrict__ has,
                                               const uint8_t* __restrict__ valid,
                                               const uint8_t* __restrict__ grouped, uint64_t n,
                                               uint64_t i0, uint32_t& h) {
  const bool aligned = ((reinterpret_cast<uintptr_t>(has) | reinterpret_cast<uintptr_t>(valid) |
                         reinterpret_cast<uintptr_t>(grouped)) & 15u) == 0;
  const uint32_t in_range = i0 >= n ? 0u : (i0 + kKlRows <= n ? 0xFFFFu : (1u << (n - i0)) - 1u);
  h = bytes16_mask(has, n, i0, aligned, 0xFFFFu);
  const uint32_t v = bytes16_mask(valid, n, i0, aligned, 0xFFFFu);
  const uint32_t g = bytes16_mask(grouped, n, i0, aligned, 0xFFFFu);
  // keyless and valid, or keyed and decided by the probe
  return in_range & ((~h & v) | (grouped ? (h & ~g) : 0u));
}

// the entry of extra row i: who (rank, | LINKED when the probe's rep is
// another row's), obj (the probe's rep when linked)
__device__ __forceinline__ bool extra_linked(bool keyed, const uint32_t* __restrict__ hitrep,
                                             uint64_t i, uint32_t r, uint32_t& o) {
  if (!keyed) return false;
  o = hitrep[i];
  return o != r;
}

__device__ __forceinline__ uint32_t rank_of(const uint32_t* __restrict__ rank, uint32_t first_rank,
                                            uint64_t i) {
  return rank ? rank[i] : first_rank + static_cast<uint32_t>(i);
}

// Blocks work on SEGMENTS of whole tiles (at most kExtraSegs of them, so the
// one-block scan reads a few values per thread: with one tile per block its
// 24 k-tile loop at 100 M rows was serial load latency, 0.09 ms).
constexpr uint32_t kExtraSegs = 2048;
struct ExtraSegs {
  uint32_t nseg, tps;  // segments, tiles per segment
  uint64_t tiles;
};
__device__ __forceinline__ uint64_t seg_tile0(const ExtraSegs& g, uint32_t seg) {
  return static_cast<uint64_t>(seg) * g.tps;
}
__device__ __forceinline__ uint64_t seg_tile1(const ExtraSegs& g, uint32_t seg) {
  return min(g.tiles, static_cast<uint64_t>(seg + 1) * g.tps);
}

// per segment: cnt[s] = extra entries, lk[s] = the linked ones among them
__global__ __launch_bounds__(kThreads) void k_extra_count(
    const uint8_t* __restrict__ has, const uint8_t* __restrict__ valid,
    const uint8_t* __restrict__ grouped, const uint32_t* __restrict__ hitrep,
    const uint32_t* __restrict__ rank, uint32_t first_rank, uint64_t n, ExtraSegs g,
    uint32_t* __restrict__ cnt, uint32_t* __restrict__ lk) {
  __shared__ uint32_t sc[kWaves], sl[kWaves];
  uint32_t c = 0, l = 0;
  for (uint64_t t = seg_tile0(g, blockIdx.x); t < seg_tile1(g, blockIdx.x); ++t) {
    const uint64_t i0 = t * kKlTile + threadIdx.x * kKlRows;
    uint32_t h;
    const uint32_t m = extra_mask(has, valid, grouped, n, i0, h);
    c += __popc(m);
    // linked entries exist only among probe-decided keyed rows (an index)
    uint32_t d = grouped ? (m & h) : 0u;
    while (d) {
      const int k = __ffs(d) - 1;
      d &= d - 1;
      uint32_t o;
      l += extra_linked(true, hitrep, i0 + k, rank_of(rank, first_rank, i0 + k), o) ? 1u : 0u;
    }
  }
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) {
    c += __shfl_xor(c, s);
    l += __shfl_xor(l, s);
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
    lk[blockIdx.x] = tl;
  }
}

// ONE block: cnt[] -> exclusive tile offsets; kx[0] = K (the keyed entries,
// counts[2] as the group kernel left it, for k_extra_write); counts[0..2] +=
// the extra creators / linked / entries
constexpr int kScanThreads = 1024;
__global__ __launch_bounds__(kScanThreads) void k_extra_scan(uint32_t* __restrict__ cnt,
                                                             const uint32_t* __restrict__ lk,
                                                             uint32_t nb, uint32_t* __restrict__ kx,
                                                             uint32_t* __restrict__ counts,
                                                             uint32_t cap,
                                                             uint32_t* __restrict__ nospc) {
  __shared__ uint32_t sw[kScanThreads / 64], slk[kScanThreads / 64];
  const uint32_t per = (nb + kScanThreads - 1) / kScanThreads;
  const uint32_t b0 = threadIdx.x * per, b1 = min(nb, b0 + per);
  uint32_t t = 0, l = 0;
  for (uint32_t b = b0; b < b1; ++b) {
    t += cnt[b];
    l += lk[b];
  }
  // block-wide exclusive scan of t (wave scan + wave totals)
  const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
  uint32_t inc = t;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d);
    if (lane >= static_cast<uint32_t>(d)) inc += o;
  }
  uint32_t lw = l;
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) lw += __shfl_xor(lw, d);
  if (lane == 63) sw[w] = inc;
  if (lane == 0) slk[w] = lw;
  __syncthreads();
  uint32_t base = inc - t, tot = 0, ltot = 0;
  for (uint32_t v = 0; v < kScanThreads / 64; ++v) {
    if (v < w) base += sw[v];
    tot += sw[v];
    ltot += slk[v];
  }
  for (uint32_t b = b0; b < b1; ++b) {
    const uint32_t c = cnt[b];
    cnt[b] = base;
    base += c;
  }
  if (threadIdx.x == 0) {
    const uint32_t K = counts[2];
    kx[0] = K;
    counts[0] += tot - ltot;
    counts[1] += ltot;
    counts[2] = K + tot;
    // the caller's capacity (the sharded write set): k_extra_write skips
    // entries past it and the call fails with -ENOSPC
    if (nospc && static_cast<uint64_t>(K) + tot > cap) *nospc = 1u;
  }
}

__global__ __launch_bounds__(kThreads) void k_extra_write(
    const uint8_t* __restrict__ has, const uint8_t* __restrict__ valid,
    const uint8_t* __restrict__ grouped, const uint32_t* __restrict__ hitrep,
    const uint32_t* __restrict__ rank, uint32_t first_rank, uint64_t n, ExtraSegs g,
    const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ kx, uint32_t* __restrict__ who,
    uint32_t* __restrict__ obj, uint32_t cap) {
  __shared__ uint32_t sw[kWaves];
  const uint32_t lane = __lane_id(), wv = threadIdx.x >> 6;
  uint32_t base = kx[0] + cnt[blockIdx.x];  // this segment's first entry
  for (uint64_t t = seg_tile0(g, blockIdx.x); t < seg_tile1(g, blockIdx.x); ++t) {
    const uint64_t i0 = t * kKlTile + threadIdx.x * kKlRows;
    uint32_t hm;
    uint32_t m = extra_mask(has, valid, grouped, n, i0, hm);
    const uint32_t c = __popc(m);
    uint32_t inc = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = __shfl_up(inc, d);
      if (lane >= static_cast<uint32_t>(d)) inc += o;
    }
    if (lane == 63) sw[wv] = inc;
    __syncthreads();
    uint32_t pos = base + inc - c, tile_total = 0;
    for (uint32_t w = 0; w < kWaves; ++w) {
      if (w < wv) pos += sw[w];
      tile_total += sw[w];
    }
    __syncthreads();  // sw is rewritten by the next tile
    base += tile_total;
    while (m) {
      const int k = __ffs(m) - 1;
      m &= m - 1;
      const uint64_t i = i0 + k;
      const uint32_t r = rank_of(rank, first_rank, i);
      uint32_t o, w = r;
      const bool room = pos < cap;
      if (extra_linked((hm >> k) & 1u, hitrep, i, r, o)) {  // keyed: decided by the probe
        w = r | kLinkedBit;
        if (room) obj[pos] = o;
      }
      if (room) who[pos] = w;
      ++pos;
    }
  }
}

}  // namespace

namespace {
ExtraSegs extra_segs(uint64_t n) {
  ExtraSegs g;
  g.tiles = (n + kKlTile - 1) / kKlTile;
  g.nseg = static_cast<uint32_t>(std::min<uint64_t>(g.tiles, kExtraSegs));
  g.tps = static_cast<uint32_t>((g.tiles + g.nseg - 1) / g.nseg);
  g.nseg = static_cast<uint32_t>((g.tiles + g.tps - 1) / g.tps);  // no empty segment
  return g;
}
}  // namespace

size_t extra_workspace_bytes(uint64_t) {
  return 2 * (((kExtraSegs + 1) * 4 + 255) / 256 * 256) + 256;
}

hipError_t extra_list_launch(const uint8_t* has, const uint8_t* valid, const uint8_t* grouped,
                             const uint32_t* hitrep, const uint32_t* rank, uint32_t first_rank,
                             uint64_t n, uint32_t* who, uint32_t* obj, uint32_t* counts, void* ws,
                             hipStream_t s, KTimer* timer, uint32_t cap, uint32_t* nospc) {
  if (n == 0 || (!has && !grouped)) return hipSuccess;  // every row keyed, no probe: nothing extra
  const ExtraSegs g = extra_segs(n);
  uint8_t* b = static_cast<uint8_t*>(ws);
  const size_t cb = ((kExtraSegs + 1) * 4ull + 255) / 256 * 256;
  uint32_t* cnt = reinterpret_cast<uint32_t*>(b);
  uint32_t* lk = reinterpret_cast<uint32_t*>(b + cb);
  uint32_t* kx = reinterpret_cast<uint32_t*>(b + 2 * cb);
  KScope k(timer, "extra_list", s);
  k_extra_count<<<g.nseg, kThreads, 0, s>>>(has, valid, grouped, hitrep, rank, first_rank, n, g,
                                            cnt, lk);
  k_extra_scan<<<1, kScanThreads, 0, s>>>(cnt, lk, g.nseg, kx, counts, cap, nospc);
  k_extra_write<<<g.nseg, kThreads, 0, s>>>(has, valid, grouped, hitrep, rank, first_rank, n, g,
                                            cnt, kx, who, obj, nospc ? cap : 0xFFFFFFFFu);
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
