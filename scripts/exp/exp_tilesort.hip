// Experiment: the 12-bit grouping WITHOUT the 4096-way
// scatter.  The product partitions 12.5 M rows by a histogram pass, a block
// offsets scan and a 4096-way LDS-staged scatter whose record stores are pairs
// (0.05 ms of the scatter's 0.12 ms is those pair stores, profiles/r3/exp_stores/).
// Here instead:
//   TS  k_tile_sort: each block counting-sorts 8192-row tiles by the 12-bit
//       digit in LDS and writes every tile back to ITS OWN row range, one
//       contiguous coalesced chunk, plus the tile's 4096 digit ends (u16);
//   TT  k_ends_transpose: the [tile][digit] ends table -> [digit][tile];
//   TG  k_group_tiles: bucket b's records are its run in every tile (~2 rows
//       each): the bucket's runs are scanned in LDS, each record located by a
//       binary search of the run prefix, then grouped exactly as the product's
//       packed-table group kernel.
// No histogram pass and no cross-block offsets; the scattered accesses move from
// pair STORES in the partition to short-run LOADS in the group kernel.
// Records / reps must equal the product's (dedup_local_launch).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_tilesort.hip -o build/exp_tilesort
#include "../../spacedrive_amd/csrc/dedup.hip"

#include <stdio.h>

#include <algorithm>
#include <functional>
#include <vector>

using namespace sdgpu;

namespace {

constexpr uint32_t kNb = 1u << kStageBits;  // 4096 buckets
constexpr uint32_t kT = 8192;               // rows per tile
constexpr uint32_t kTsThreads = 512;        // tile-sort threads (256 VGPRs each)
constexpr int kTU = kT / kTsThreads;        // 16 consecutive rows per thread
constexpr uint32_t kMaxTiles = 2048;        // tiles: 2 per group-kernel thread

__global__ void k_rows(uint64_t* key, uint8_t* has, uint64_t n, uint64_t distinct) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint64_t j = (i * 0x9E3779B1ull) % n;
    key[i] = row_hash((j % distinct) * 0x2545F4914F6CDD1Dull + 7);
    has[i] = (row_hash(i ^ 0x55ull) % 1000) != 0;
  }
}

// A tile's rows for one thread: kTU CONSECUTIVE rows (16-B key pair loads,
// one 8-B load of the validity bytes); rank = row.  Tails (n % 8 != 0, the
// last tile) take the row-by-row path.
struct TileRows {
  uint64_t k[kTU];
  uint4 v;
};

template <bool kInitRep>
__global__ __launch_bounds__(kTsThreads) void k_tile_sort(const uint64_t* __restrict__ key,
                                                            const uint8_t* __restrict__ valid,
                                                            uint64_t n, uint32_t skip,
                                                            uint32_t ntiles, uint3* __restrict__ out,
                                                            uint16_t* __restrict__ ends,
                                                            uint32_t* __restrict__ rep) {
  static_assert(kTU == 16, "16 consecutive rows per thread");
  __shared__ uint3 buf[kT];             // 96 KiB
  __shared__ __attribute__((aligned(16))) uint32_t cnt[2][kNb];  // 32 KiB: a tile's counts, then its starts
  __shared__ uint32_t wsum[kTsThreads / 64];
  const uint32_t t = threadIdx.x, lane = __lane_id(), w = t >> 6;
  for (uint32_t k = t; k < 2 * kNb; k += kTsThreads) (&cnt[0][0])[k] = 0;
  __syncthreads();
  const uint64_t n8 = n & ~15ull;  // rows in whole groups of 16
  auto load = [&](uint32_t tl, TileRows& q) {
    const uint64_t i0 = static_cast<uint64_t>(tl) * kT + 16ull * t;
    if (i0 + 16 <= n8) {
      const uint4* kp = reinterpret_cast<const uint4*>(key + i0);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint4 x = kp[u];
        q.k[2 * u] = (static_cast<uint64_t>(x.y) << 32) | x.x;
        q.k[2 * u + 1] = (static_cast<uint64_t>(x.w) << 32) | x.z;
      }
      q.v = *reinterpret_cast<const uint4*>(valid + i0);
    } else {
      uint32_t vv[4] = {0, 0, 0, 0};
#pragma unroll
      for (int u = 0; u < kTU; ++u) {
        const uint64_t i = i0 + u;
        const bool in = i < n;
        q.k[u] = in ? key[i] : 0ull;
        vv[u >> 2] |= (in && valid[i] ? 1u : 0u) << (8 * (u & 3));
      }
      q.v = make_uint4(vv[0], vv[1], vv[2], vv[3]);
    }
  };
  auto process = [&](const TileRows& q, uint32_t tl, uint32_t par) {
    uint32_t* __restrict__ c = cnt[par];
    const uint64_t t0 = static_cast<uint64_t>(tl) * kT;
    uint32_t lr[kTU], keyed = 0;
    const uint64_t i0 = t0 + 16ull * t;
    if (kInitRep) {
      if (i0 + 16 <= n) {
        uint4* rp = reinterpret_cast<uint4*>(rep + i0);
        const uint32_t r0 = static_cast<uint32_t>(i0);
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u) rp[u] = make_uint4(r0 + 4 * u, r0 + 4 * u + 1, r0 + 4 * u + 2, r0 + 4 * u + 3);
      } else {
        for (uint64_t i = i0; i < n && i < i0 + 16; ++i) rep[i] = static_cast<uint32_t>(i);
      }
    }
    const uint32_t vw[4] = {q.v.x, q.v.y, q.v.z, q.v.w};
#pragma unroll
    for (int u = 0; u < kTU; ++u) {
      const uint32_t vb = (vw[u >> 2] >> (8 * (u & 3))) & 0xFFu;
      if (vb == 0 || i0 + u >= n) continue;
      keyed |= 1u << u;
      lr[u] = atomicAdd(&c[digit_of(row_hash(q.k[u]), skip, kStageBits)], 1u);
    }
    lds_barrier();  // counts complete
    // thread t owns digits 8t .. 8t + 7
    const uint4 va = reinterpret_cast<const uint4*>(c)[2 * t], vb = reinterpret_cast<const uint4*>(c)[2 * t + 1];
    const uint32_t s1 = va.x, s2 = s1 + va.y, s3 = s2 + va.z, s4 = s3 + va.w;
    const uint32_t s5 = s4 + vb.x, s6 = s5 + vb.y, s7 = s6 + vb.z, s8 = s7 + vb.w;
    uint32_t inc = s8;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = __shfl_up(inc, d);
      if (lane >= static_cast<uint32_t>(d)) inc += o;
    }
    if (lane == 63) wsum[w] = inc;
    lds_barrier();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (uint32_t x = 0; x < kTsThreads / 64; ++x) {
      const uint32_t ws = wsum[x];
      before += x < w ? ws : 0u;
      total += ws;
    }
    const uint32_t ex = before + inc - s8;
    // the tile's digit ends (inclusive), u16: one 16-byte store per thread
    reinterpret_cast<uint4*>(ends + static_cast<uint64_t>(tl) * kNb)[t] =
        make_uint4((ex + s1) | ((ex + s2) << 16), (ex + s3) | ((ex + s4) << 16),
                   (ex + s5) | ((ex + s6) << 16), (ex + s7) | ((ex + s8) << 16));
    reinterpret_cast<uint4*>(c)[2 * t] = make_uint4(ex, ex + s1, ex + s2, ex + s3);
    reinterpret_cast<uint4*>(c)[2 * t + 1] = make_uint4(ex + s4, ex + s5, ex + s6, ex + s7);
    lds_barrier();  // starts published
#pragma unroll
    for (int u = 0; u < kTU; ++u) {
      if (!(keyed >> u & 1u)) continue;
      const uint64_t h = row_hash(q.k[u]);
      buf[c[digit_of(h, skip, kStageBits)] + lr[u]] =
          make_uint3(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32),
                     static_cast<uint32_t>(i0 + u));
    }
    lds_barrier();  // tile sorted in LDS
    reinterpret_cast<uint4*>(c)[2 * t] = make_uint4(0, 0, 0, 0);  // reused two tiles later
    reinterpret_cast<uint4*>(c)[2 * t + 1] = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < kTU; ++u) {
      const uint32_t k = t + u * kTsThreads;
      if (k < total) out[t0 + k] = buf[k];
    }
  };
  const uint32_t G = gridDim.x;
  uint32_t tl = blockIdx.x;
  if (tl >= ntiles) return;
  TileRows qa, qb;
  load(tl, qa);
  uint32_t par = 0;
  for (;;) {  // the next tile's rows are loaded while the current one is sorted
    load(tl + G, qb);
    process(qa, tl, par);
    par ^= 1u;
    tl += G;
    if (tl >= ntiles) break;
    load(tl + G, qa);
    process(qb, tl, par);
    par ^= 1u;
    tl += G;
    if (tl >= ntiles) break;
  }
}

// ends[tile][digit] -> endsT[digit][tile] (tiles padded to ntp, pads 0).
__global__ __launch_bounds__(256) void k_ends_transpose(const uint16_t* __restrict__ ends,
                                                        uint32_t ntiles, uint32_t ntp,
                                                        uint16_t* __restrict__ endsT) {
  __shared__ uint16_t tileb[64][66];
  const uint32_t d0 = blockIdx.x * 64, r0 = blockIdx.y * 64;
  const uint32_t tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (uint32_t y = ty; y < 64; y += 4) {
    const uint32_t r = r0 + y;
    tileb[y][tx] = r < ntiles ? ends[static_cast<uint64_t>(r) * kNb + d0 + tx] : 0;
  }
  __syncthreads();
  for (uint32_t y = ty; y < 64; y += 4) {
    const uint32_t r = r0 + tx;
    if (r < ntp) endsT[static_cast<uint64_t>(d0 + y) * ntp + r] = tileb[tx][y];
  }
}

__global__ __launch_bounds__(kGroupThreads, 8) void k_group_tiles(
    const uint3* __restrict__ rec, uint32_t rank_base, const uint16_t* __restrict__ endsT,
    uint32_t ntp, uint32_t bits, ChunkOf chunk_of, uint32_t* __restrict__ rep,
    uint32_t* __restrict__ big) {
  __shared__ uint64_t tab[kPkSlots];
  __shared__ uint32_t lmin[kPkCap + 1];  // first: the run prefix (2048 u32) + run starts (2048 u16)
  __shared__ uint32_t wsum[kGroupThreads / 64];
  constexpr int kP = (kPkCap + kGroupThreads) / kGroupThreads;  // 4
  static_assert(kMaxTiles * 6 <= (kPkCap + 1) * 4, "run lists fit the lmin area");
  uint32_t* runpos = lmin;
  uint16_t* sst = reinterpret_cast<uint16_t*>(lmin + kMaxTiles);
  const uint32_t b = blockIdx.x, t = threadIdx.x, lane = __lane_id(), w = t >> 6;
  uint32_t e = 0, s = 0;
  if (2 * t < ntp) {
    e = *reinterpret_cast<const uint32_t*>(endsT + static_cast<uint64_t>(b) * ntp + 2 * t);
    if (b) s = *reinterpret_cast<const uint32_t*>(endsT + static_cast<uint64_t>(b - 1) * ntp + 2 * t);
  }
  const uint32_t s0 = s & 0xFFFFu, s1 = s >> 16;
  const uint32_t l0 = (e & 0xFFFFu) - s0, l1 = (e >> 16) - s1, sum = l0 + l1;
  uint32_t inc = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d);
    if (lane >= static_cast<uint32_t>(d)) inc += o;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t before = 0, m = 0;
#pragma unroll
  for (uint32_t x = 0; x < kGroupThreads / 64; ++x) {
    const uint32_t ws = wsum[x];
    before += x < w ? ws : 0u;
    m += ws;
  }
  const uint32_t p0 = before + inc - sum;
  // every entry up to kMaxTiles written: past the last tile the prefix is m
  runpos[2 * t] = p0;
  runpos[2 * t + 1] = p0 + l0;
  sst[2 * t] = static_cast<uint16_t>(s0);
  sst[2 * t + 1] = static_cast<uint16_t>(s1);
  lds_barrier();
  if (m == 0) return;
  if (m > kPkCap) {  // experiment: counted, not grouped
    if (t == 0) atomicAdd(big, 1u);
    return;
  }
  uint4 q[kP];
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const uint32_t k = min(t + j * kGroupThreads, m - 1);
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t st = kMaxTiles / 2; st >= 1; st >>= 1)
      if (runpos[pos + st] <= k) pos += st;
    const uint3 v = rec[static_cast<uint64_t>(pos) * kT + sst[pos] + (k - runpos[pos])];
    q[j] = make_uint4(v.x, v.y, rank_base + v.z, v.z);
  }
#pragma unroll
  for (int j = 0; j < kP; ++j)
    if (t + j * kGroupThreads >= m) q[j] = make_uint4(0, 0, kPadRow, kPadRow);
  lds_barrier();  // run lists read: lmin free
  for (uint32_t x = t; x < kPkSlots; x += kGroupThreads) tab[x] = 0ull;
  for (uint32_t x = t; x <= kPkCap; x += kGroupThreads) lmin[x] = 0xFFFFFFFFu;
  __syncthreads();
  uint32_t slot[kP], step[kP], owner[kP];
  uint64_t mine[kP];
  uint32_t pend = 0;
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const uint64_t h = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
    const uint32_t idx = t + j * kGroupThreads;
    mine[j] = (key_rest(h, bits) << 12) | (idx + 1);
    slot[j] = static_cast<uint32_t>((static_cast<uint64_t>(static_cast<uint32_t>(h)) * kPkSlots) >> 32);
    uint32_t st = 1u + 2u * static_cast<uint32_t>((h >> 40) & 1023u);
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
  const uint32_t ntiles = static_cast<uint32_t>((n + kT - 1) / kT);
  const uint32_t ntp = (ntiles + 1) & ~1u;
  if (L.bits != kStageBits || L.cbits || ntiles > kMaxTiles) {
    printf("n %llu: not the one-level 12-bit path\n", (unsigned long long)n);
    return 2;
  }
  uint64_t* key;
  uint8_t* has;
  uint32_t *rep0, *rep1, *big;
  uint3* rec2;
  uint16_t *ends, *endsT;
  (void)hipMalloc(&key, 8 * n);
  (void)hipMalloc(&has, n);
  (void)hipMalloc(&rep0, 4 * n);
  (void)hipMalloc(&rep1, 4 * n);
  (void)hipMalloc(&big, 4);
  (void)hipMalloc(&rec2, 12 * n + 64);
  (void)hipMalloc(&ends, 2ull * ntiles * kNb);
  (void)hipMalloc(&endsT, 2ull * ntp * kNb);
  k_rows<<<4096, 256>>>(key, has, n, n * 4 / 5);
  void* ws;
  (void)hipMalloc(&ws, L.total);
  const ChunkOf c = ChunkOf::make(100);
  GroupInput gi;
  gi.key = key;
  gi.valid = has;
  gi.n = n;
  (void)dedup_local_launch(gi, 100, rep0, true, ws, 0, nullptr);
  (void)hipMemset(big, 0, 4);
  auto ts = [&] { k_tile_sort<true><<<256, kTsThreads>>>(key, has, n, kShardBits, ntiles, rec2, ends, rep1); };
  auto tt = [&] { k_ends_transpose<<<dim3(kNb / 64, (ntp + 63) / 64), 256>>>(ends, ntiles, ntp, endsT); };
  auto tg = [&] {
    k_group_tiles<<<kNb, kGroupThreads>>>(rec2, 0, endsT, ntp, kStageBits, c, rep1, big);
  };
  ts();
  tt();
  tg();
  (void)hipDeviceSynchronize();
  printf("n %llu tiles %u (%s)\n", (unsigned long long)n, ntiles, hipGetErrorString(hipGetLastError()));
  std::vector<uint32_t> a(n), b(n);
  (void)hipMemcpy(a.data(), rep0, 4 * n, hipMemcpyDeviceToHost);
  (void)hipMemcpy(b.data(), rep1, 4 * n, hipMemcpyDeviceToHost);
  uint32_t nbig = 0;
  (void)hipMemcpy(&nbig, big, 4, hipMemcpyDeviceToHost);
  uint64_t bad = 0, linked = 0;
  for (uint64_t i = 0; i < n; ++i) {
    bad += a[i] != b[i];
    linked += a[i] != i;
  }
  printf("tile path mismatches vs product: %llu (linked rows %llu, oversized buckets %u)\n",
         (unsigned long long)bad, (unsigned long long)linked, nbig);
  struct V {
    const char* name;
    std::function<void()> f;
  };
  std::vector<V> vs = {
      {"product dedup_local_launch", [&] { (void)dedup_local_launch(gi, 100, rep0, true, ws, 0, nullptr); }},
      {"TS tile sort", ts},
      {"TT ends transpose", tt},
      {"TG group from tiles", tg},
      {"TS+TT+TG", [&] { ts(); tt(); tg(); }}};
  for (int r = 0; r < 2; ++r)
    for (auto& v : vs) printf("%-30s %.4f ms\n", v.name, time_ms(v.f, reps));
  return 0;
}
