// Experiment: the 12-bit bucket scatter of the one-level
// grouping (12.5 M rows, rows in rank order: 12-byte records) with the
// per-(block, bucket) runs replaced by per-(XCD, bucket) runs.
//
// Why: every block of the product's staged scatter owns a run in every bucket
// and writes it pair by pair over the kernel's lifetime; an XCD's 32 blocks x
// 4096 buckets keep ~131 k partially written lines open, far more than its
// 4 MiB L2 holds, so lines leave the L2 half written (PMC: 391 MB written
// for 200 MB of records + reps).  Here the blocks of one XCD share ONE run per
// bucket: a position is reserved with an agent-scope atomicAdd on that run's
// cursor (8 x 4096 cursors; the blocks of XCD x are the logical blocks
// [x P/8, (x+1) P/8), so the run starts are k_fine_scan's E rows x P/8), and
// the open lines per XCD drop to ~4096 -- they can be completed in L2.
//   P0  product: hist -> fine scan -> staged scatter (2 slots) -> group12
//   X2  hist -> fine scan -> cursor init -> XCD-run scatter, 2 LDS slots per
//       bucket, one global atomic per flushed pair -> group12
//   X4  X2 with 4 rows per thread per round
//   X1  same without LDS staging: one global atomic per row
// Every variant's reps must equal the product's.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_xcd_scatter.hip -o build/exp_xcd_scatter
#include "../../spacedrive_amd/csrc/dedup.hip"

#include <stdio.h>

#include <algorithm>
#include <functional>
#include <vector>

using namespace sdgpu;

namespace {

constexpr uint32_t kNb = 1u << kStageBits;

__global__ void k_rows(uint64_t* key, uint8_t* has, uint64_t n, uint64_t distinct) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint64_t j = (i * 0x9E3779B1ull) % n;
    key[i] = row_hash((j % distinct) * 0x2545F4914F6CDD1Dull + 7);
    has[i] = (row_hash(i ^ 0x55ull) % 1000) != 0;
  }
}

// gcur[x][b] = E[x * P/8][b]: the start of XCD x's run inside bucket b.
__global__ void k_init_cur(const uint32_t* __restrict__ E, uint32_t P, uint32_t* __restrict__ gcur) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t >= 8 * kNb) return;
  const uint32_t x = t / kNb, b = t % kNb;
  gcur[t] = E[static_cast<uint64_t>(x) * (P / 8) * kNb + b];
}

template <uint32_t kSlots, int kRows>
__global__ __launch_bounds__(kPartThreads) void k_scatter_xcd(RowsIn in, uint64_t n, uint32_t skip,
                                                             const uint32_t* __restrict__ ftot,
                                                             uint32_t* __restrict__ gcur,
                                                             uint3* __restrict__ out,
                                                             uint32_t* __restrict__ rep,
                                                             uint32_t* __restrict__ fbase) {
  constexpr uint32_t nbins = kNb;
  constexpr uint32_t kS = kSlots ? kSlots : 1;
  __shared__ uint3 stage[nbins][kS];
  __shared__ uint32_t fill[nbins];
  __shared__ uint32_t bst[nbins];
  // bucket starts: exclusive scan of the bucket sizes (4 per thread)
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
    bst[b] = base;
    fill[b] = 0;
    if (j == 0) fbase[b] = base;
    base += v[k];
  }
  if (j == 0 && t == 0) fbase[nbins] = total;
  __syncthreads();
  uint32_t* __restrict__ gc = gcur + (blockIdx.x & 7u) * nbins;
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  constexpr int U = kRows;
  constexpr uint64_t kStep = static_cast<uint64_t>(U) * kPartThreads;
  auto round = [&](const RowBatch<U>& q, uint64_t i0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = i0 + threadIdx.x + static_cast<uint64_t>(u) * kPartThreads;
      if (!q.in[u]) continue;
      rep[i] = in.rank_of(q, u);
      if (!in.valid_of(q, u)) continue;
      const uint64_t h = row_hash(in.key_of(q, u));
      const uint32_t b = digit_of(h, skip, kStageBits);
      const uint3 rq = make_uint3(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32), in.row_of(q, u));
      if constexpr (kSlots > 0) {
        const uint32_t sl = atomicAdd(&fill[b], 1u);
        if (sl < kSlots) {
          stage[b][sl] = rq;
          continue;
        }
      }
      out[bst[b] + atomicAdd(&gc[b], 1u)] = rq;
    }
    if constexpr (kSlots > 0) {
      lds_barrier();
#pragma unroll
      for (uint32_t k = 0; k < nbins / kPartThreads; ++k) {
        const uint32_t b = threadIdx.x + k * kPartThreads;
        if (fill[b] >= kSlots) {
          const uint32_t p = bst[b] + atomicAdd(&gc[b], kSlots);
#pragma unroll
          for (uint32_t s = 0; s < kSlots; ++s) out[p + s] = stage[b][s];
          fill[b] = 0;
        }
      }
      lds_barrier();
    }
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
  if constexpr (kSlots > 0) {
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads) {
      const uint32_t f = fill[b];
      if (f) {
        const uint32_t p = bst[b] + atomicAdd(&gc[b], f);
        for (uint32_t s = 0; s < f; ++s) out[p + s] = stage[b][s];
      }
    }
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
  uint32_t *rep0, *rep1, *gcur;
  (void)hipMalloc(&key, 8 * n);
  (void)hipMalloc(&has, n);
  (void)hipMalloc(&rep0, 4 * n);
  (void)hipMalloc(&rep1, 4 * n);
  (void)hipMalloc(&gcur, 4 * 8 * kNb);
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
  auto prep = [&] {
    k_part_hist<RowsIn><<<P, kPartThreads, lds>>>(in, n, kShardBits, kStageBits, 0, fine, nullptr, true);
    k_fine_scan<kPartBlocks, 1><<<kNb / 64, 1024>>>(fine, kNb, fE, ftot, ovf);
  };
  auto p0_scatter = [&] {
    k_part_scatter_rec_staged<RowsIn, true, kStageBits, 2, 2, true><<<P, kPartThreads>>>(
        in, n, kShardBits, fE, reinterpret_cast<uint4*>(rec), rep1, nullptr, 0, ftot, fbase);
  };
  auto init = [&] { k_init_cur<<<8 * kNb / 256, 256>>>(fE, P, gcur); };
  auto x2_scatter = [&] {
    k_scatter_xcd<2, 2><<<P, kPartThreads>>>(in, n, kShardBits, ftot, gcur, rec, rep1, fbase);
  };
  auto x1_scatter = [&] {
    k_scatter_xcd<0, 2><<<P, kPartThreads>>>(in, n, kShardBits, ftot, gcur, rec, rep1, fbase);
  };
  auto x4_scatter = [&] {
    k_scatter_xcd<2, 4><<<P, kPartThreads>>>(in, n, kShardBits, ftot, gcur, rec, rep1, fbase);
  };
  auto group = [&] {
    k_bucket_group12<<<kNb, kGroupThreads>>>(rec, 0, fbase, c, gkey, gmin, rep1);
  };
  // reference reps: the product call
  (void)dedup_local_launch(gi, 100, rep0, true, ws, 0, nullptr);
  (void)hipDeviceSynchronize();
  std::vector<uint32_t> a(n), b(n);
  (void)hipMemcpy(a.data(), rep0, 4 * n, hipMemcpyDeviceToHost);
  uint64_t linked = 0;
  for (uint64_t i = 0; i < n; ++i) linked += a[i] != i;
  printf("n %llu buckets %u linked %llu\n", (unsigned long long)n, kNb, (unsigned long long)linked);
  struct V {
    const char* name;
    std::function<void()> scatter;
    bool xcd;
  };
  std::vector<V> vs = {{"P0 product staged", p0_scatter, false},
                       {"X2 xcd runs, 2 slots", x2_scatter, true},
                       {"X4 xcd runs, 2 slots, 4 rows/round", x4_scatter, true},
                       {"X1 xcd runs, no staging", x1_scatter, true}};
  for (auto& v : vs) {
    (void)hipMemset(rep1, 0xFF, 4 * n);
    prep();
    if (v.xcd) init();
    v.scatter();
    group();
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(b.data(), rep1, 4 * n, hipMemcpyDeviceToHost);
    uint64_t bad = 0;
    for (uint64_t i = 0; i < n; ++i) bad += a[i] != b[i];
    printf("%-36s mismatches vs product: %llu\n", v.name, (unsigned long long)bad);
  }
  for (int r = 0; r < 2; ++r) {
    for (auto& v : vs) {
      const float whole = time_ms([&] {
        prep();
        if (v.xcd) init();
        v.scatter();
        group();
      }, reps);
      prep();
      const float sc = time_ms([&] {
        if (v.xcd) init();
        v.scatter();
      }, reps);
      printf("%-36s whole %.4f ms   scatter (+init) %.4f ms\n", v.name, whole, sc);
    }
  }
  return 0;
}
