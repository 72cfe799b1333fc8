// Experiment (round 4): the 12-bit warp-specialised
// scatter with THREE LDS slots per bucket instead of two.
// The product (k_part_scatter_ws) stages 2 x 12-B records per bucket in LDS
// (4096 x 2 x 12 B = 96 KiB) and writes full pairs: 24-B runs, and the store
// pattern, not the bytes, sets its time (scripts/exp/exp_stores.hip: runs of
// 2 cost ~4x runs of 16).  Three slots do not fit beside 32-bit fills,
// cursors and the overflow list, so here:
//   * 4096 x 3 x 12 B of slots (144 KiB),
//   * 16-bit fill counts and 16-bit BLOCK-RELATIVE cursors, two per word
//     (8 + 8 KiB; a block writes <= its tile of ~49 k rows to one bucket),
//   * no overflow list: a row meeting a full bucket is stored directly at
//     the bucket's cursor (the block's absolute base per bucket is kept in
//     the consumer's registers and, for those direct stores, in a global
//     per-block table written in the prologue),
//   * two barriers per round instead of three (no overflow phase).
// 160 KiB of LDS exactly.  The records must group exactly as the product's:
// the product's group kernel runs on both record arrays and the reps are
// compared.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_scatter3.hip -o build/exp_scatter3
#include "../../spacedrive_amd/csrc/dedup.hip"

#include <stdio.h>

#include <algorithm>
#include <functional>
#include <vector>

using namespace sdgpu;

namespace {

__global__ void k_rows(uint64_t* key, uint8_t* has, uint64_t n, uint64_t distinct) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint64_t j = (i * 0x9E3779B1ull) % n;
    key[i] = row_hash((j % distinct) * 0x2545F4914F6CDD1Dull + 7);
    has[i] = (row_hash(i ^ 0x55ull) % 1000) != 0;
  }
}

constexpr uint32_t kNb = 1u << kStageBits;

__device__ __forceinline__ uint32_t half_of(uint32_t w, uint32_t b) {
  return (w >> ((b & 1u) << 4)) & 0xFFFFu;
}

template <bool kInitRep>
__global__ __launch_bounds__(kPartThreads) void k_part_scatter_ws3(
    RowsIn in, uint64_t n, uint32_t skip, const uint32_t* __restrict__ offs,
    const uint32_t* __restrict__ ftot, uint3* __restrict__ out, uint32_t* __restrict__ rep,
    uint32_t* __restrict__ fbase, uint32_t* __restrict__ blkbase) {
  constexpr uint32_t nbins = kNb;
  constexpr uint32_t kRound = kWsProd * kWsRows;  // 2048 rows
  __shared__ uint3 stage[nbins][3];
  __shared__ uint32_t fill2[nbins / 2], cur2[nbins / 2];
  constexpr uint32_t kPerT = nbins / kPartThreads;  // 4
  const uint32_t t = threadIdx.x, lane = __lane_id();
  const uint32_t j = part_block();
  uint32_t v[kPerT], ov[kPerT], sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPerT; ++k) {
    v[k] = ftot[t * kPerT + k];
    ov[k] = offs[static_cast<uint64_t>(j) * nbins + t * kPerT + k];
  }
#pragma unroll
  for (uint32_t k = 0; k < kPerT; ++k) sum += v[k];
  uint32_t inc = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d);
    if (lane >= static_cast<uint32_t>(d)) inc += o;
  }
  uint32_t* wsum = fill2;  // scratch before the fills are cleared
  if (lane == 63) wsum[t >> 6] = inc;
  __syncthreads();
  uint32_t base = inc - sum, total = 0;
  for (uint32_t w = 0; w < kPartThreads / 64; ++w) {
    if (w < (t >> 6)) base += wsum[w];
    total += wsum[w];
  }
  __syncthreads();
  uint32_t* bb = blkbase + static_cast<uint64_t>(j) * nbins;
#pragma unroll
  for (uint32_t k = 0; k < kPerT; ++k) {
    const uint32_t b = t * kPerT + k;
    bb[b] = base + ov[k];  // this block's first position in bucket b
    if (j == 0) fbase[b] = base;
    base += v[k];
  }
  if (j == 0 && t == 0) fbase[nbins] = total;
  for (uint32_t w = t; w < nbins / 2; w += kPartThreads) {
    fill2[w] = 0;
    cur2[w] = 0;
  }
  __syncthreads();  // also makes bb visible to the block (direct stores)
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
        const uint32_t b = digit_of(h, skip, kStageBits);
        const uint3 rq = make_uint3(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32),
                                    in.row_of(q, u));
        const uint32_t sh = (b & 1u) << 4;
        const uint32_t sl = (atomicAdd(&fill2[b >> 1], 1u << sh) >> sh) & 0xFFFFu;
        if (sl < 3) {
          stage[b][sl] = rq;
        } else {  // full bucket: straight to its cursor
          const uint32_t rel = (atomicAdd(&cur2[b >> 1], 1u << sh) >> sh) & 0xFFFFu;
          out[bb[b] + rel] = rq;
        }
      }
    };
    for (uint32_t r = 0; r < rounds; r += 2) {
      stage_round(qa);
      lds_barrier();  // A
      in.template load_many<kWsRows>(t0 + (r + 2) * static_cast<uint64_t>(kRound) + t, kWsProd, t1,
                                     t0, qa);
      lds_barrier();  // B
      if (r + 1 >= rounds) break;
      stage_round(qb);
      lds_barrier();  // A
      in.template load_many<kWsRows>(t0 + (r + 3) * static_cast<uint64_t>(kRound) + t, kWsProd, t1,
                                     t0, qb);
      lds_barrier();  // B
    }
  } else {
    const uint32_t c = t - kWsProd;
    uint32_t mybase[nbins / kWsProd];
#pragma unroll
    for (uint32_t k = 0; k < nbins / kWsProd; ++k) mybase[k] = bb[c + k * kWsProd];
    for (uint32_t r = 0; r < rounds; ++r) {
      lds_barrier();  // A
      if constexpr (kInitRep) {
        const uint64_t r0 = t0 + static_cast<uint64_t>(r) * kRound;
#pragma unroll
        for (uint32_t u = 0; u < kRound / kWsProd; ++u) {
          const uint64_t i = r0 + c + u * kWsProd;
          if (i < t1) rep[i] = in.rank_base + static_cast<uint32_t>(i);
        }
      }
#pragma unroll
      for (uint32_t k = 0; k < nbins / kWsProd; ++k) {
        const uint32_t b = c + k * kWsProd, sh = (b & 1u) << 4;
        if (half_of(fill2[b >> 1], b) >= 3) {
          // the producers' direct stores of this round already advanced the
          // cursor; the triple takes the next three positions
          const uint32_t rel = (atomicAdd(&cur2[b >> 1], 3u << sh) >> sh) & 0xFFFFu;
          const uint32_t p = mybase[k] + rel;
          out[p] = stage[b][0];
          out[p + 1] = stage[b][1];
          out[p + 2] = stage[b][2];
          atomicAnd(&fill2[b >> 1], 0xFFFF0000u >> sh);
        }
      }
      lds_barrier();  // B
    }
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads) {
    const uint32_t f = half_of(fill2[b >> 1], b);
    const uint32_t rel = half_of(cur2[b >> 1], b);
    for (uint32_t k = 0; k < min(f, 3u); ++k) out[bb[b] + rel + k] = stage[b][k];
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
  uint32_t *rep0, *rep1, *blkbase;
  (void)hipMalloc(&key, 8 * n);
  (void)hipMalloc(&has, n);
  (void)hipMalloc(&rep0, 4 * n);
  (void)hipMalloc(&rep1, 4 * n);
  (void)hipMalloc(&blkbase, 4ull * kPartBlocks * kNb);
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
  const RowsIn in{key, has, nullptr, 0};
  const ChunkOf c = ChunkOf::make(100);
  GroupInput gi;
  gi.key = key;
  gi.valid = has;
  gi.n = n;
  (void)dedup_local_launch(gi, 100, rep0, true, ws, 0, nullptr);  // product reps
  (void)hipDeviceSynchronize();
  const size_t lds = sizeof(uint32_t) << kStageBits;
  auto hist = [&] {
    k_part_hist<RowsIn><<<kPartBlocks, kPartThreads, lds>>>(in, n, kShardBits, kStageBits, 0, fine,
                                                            nullptr, true);
    k_fine_scan<kPartBlocks, 1><<<kNb / 64, 1024>>>(fine, kNb, fE, ftot, ovf);
  };
  auto ws2 = [&] {
    k_part_scatter_ws<true><<<kPartBlocks, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1,
                                                           fbase);
  };
  auto ws3 = [&] {
    k_part_scatter_ws3<true><<<kPartBlocks, kPartThreads>>>(in, n, kShardBits, fE, ftot, rec, rep1,
                                                            fbase, blkbase);
  };
  auto group = [&] {
    k_bucket_group12_pk<RepOut><<<kNb, kGroupThreads>>>(rec, 0, fbase, kStageBits, c, gkey, gmin,
                                                        RepOut{rep1});
  };
  std::vector<uint32_t> a(n), b(n);
  (void)hipMemcpy(a.data(), rep0, 4 * n, hipMemcpyDeviceToHost);
  for (int variant = 0; variant < 2; ++variant) {
    hist();
    if (variant == 0) ws2(); else ws3();
    group();
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(b.data(), rep1, 4 * n, hipMemcpyDeviceToHost);
    uint64_t bad = 0;
    for (uint64_t i = 0; i < n; ++i) bad += a[i] != b[i];
    printf("%s: reps vs product grouping mismatches %llu (%s)\n",
           variant == 0 ? "WS2 product" : "WS3 three slots", (unsigned long long)bad,
           hipGetErrorString(hipGetLastError()));
  }
  for (int r = 0; r < 2; ++r) {
    printf("hist + fine scan         %.4f ms\n", time_ms(hist, reps));
    printf("WS2 scatter (product)    %.4f ms\n", time_ms(ws2, reps));
    printf("WS3 scatter (3 slots)    %.4f ms\n", time_ms(ws3, reps));
    printf("whole WS2 grouping       %.4f ms\n", time_ms([&] { hist(); ws2(); group(); }, reps));
    printf("whole WS3 grouping       %.4f ms\n", time_ms([&] { hist(); ws3(); group(); }, reps));
  }
  return 0;
}
