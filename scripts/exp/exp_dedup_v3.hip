// Experiment (not shipped): the one-level grouping of 12.5 M config-4-shaped
// rows without the 3-launch offset scan.
//   V0  product: hist -> scan (k_tiles, k_sums, k_add) -> staged scatter -> group
//   V1  memset(tot) -> hist that reserves each block's within-digit offset with
//       one device atomicAdd per (digit, block) -> staged scatter that scans the
//       4096 digit totals in LDS itself (block 0 also writes the bucket starts)
//       -> group reading the bucket starts (stride 1).  Record order inside a
//       bucket then depends on atomic order; the grouping does not.
// plus hist-only variants: H0 product, H1 2 blocks per CU (P = 512), H2 16 rows
// per thread per batch, H3 no LDS atomics (load floor).
// Result (profiles/r2/exp_dedup_v3_r2C.log): V1 0.311-0.314 vs V0 0.316-0.322 ms
// -- the device atomics and the memset cost about what the scan did; not
// adopted.  The histogram alone runs 0.027 ms (4.2 TB/s), at its load floor.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_dedup_v3.hip -o build/exp_dedup_v3
#include "../../spacedrive_amd/csrc/dedup.hip"

#include <stdio.h>

#include <vector>

using namespace sdgpu;

namespace {

__global__ void k_rows(uint64_t* key, uint32_t* rank, uint8_t* has, uint64_t n, uint64_t distinct) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint64_t j = (i * 0x9E3779B1ull) % n;
    key[i] = row_hash((j % distinct) * 0x2545F4914F6CDD1Dull + 7);
    rank[i] = static_cast<uint32_t>((i * 0x9E3779B1ull) % n);
    has[i] = (row_hash(i ^ 0x55ull) % 1000) != 0;
  }
}

template <typename In, int U, bool kAtomics>
__global__ __launch_bounds__(kPartThreads) void k_hist_var(In in, uint64_t n, uint32_t skip,
                                                           uint32_t bits, uint32_t* __restrict__ tot,
                                                           uint32_t* __restrict__ within) {
  extern __shared__ __attribute__((aligned(16))) uint32_t cnt[];
  const uint32_t nbins = 1u << bits;
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads) cnt[b] = 0;
  __syncthreads();
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  uint32_t acc = 0;
  for (uint64_t i0 = t0 + threadIdx.x; i0 < t1; i0 += U * kPartThreads) {
    RowBatch<U> q;
    in.template load_many<U>(i0, kPartThreads, t1, i0, q);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!in.valid_of(q, u)) continue;
      const uint32_t d = digit_of(in_hash<In>(in.key_of(q, u)), skip, bits);
      if (kAtomics) atomicAdd(&cnt[d], 1u);
      else acc += d;
    }
  }
  if (!kAtomics && acc == 0x12345u) cnt[0] = acc;
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads) {
    const uint32_t c = cnt[b];
    within[static_cast<uint64_t>(b) * gridDim.x + part_block()] =
        tot ? (c ? atomicAdd(&tot[b], c) : 0u) : c;
  }
}

// Exclusive scan of v[0..4096) in place by 1024 threads (4 per thread);
// wsum: 16 words of scratch.  Returns the total.
__device__ uint32_t block_scan4096(uint32_t* v, uint32_t* wsum) {
  const uint32_t t = threadIdx.x, lane = __lane_id(), w = t >> 6;
  uint32_t a0 = v[4 * t], a1 = v[4 * t + 1], a2 = v[4 * t + 2], a3 = v[4 * t + 3];
  const uint32_t s = a0 + a1 + a2 + a3;
  uint32_t inc = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d);
    if (lane >= static_cast<uint32_t>(d)) inc += o;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t wbase = 0, total = 0;
  for (uint32_t k = 0; k < 16; ++k) {
    const uint32_t x = wsum[k];
    if (k < w) wbase += x;
    total += x;
  }
  uint32_t e = wbase + inc - s;
  v[4 * t] = e;
  e += a0;
  v[4 * t + 1] = e;
  e += a1;
  v[4 * t + 2] = e;
  e += a2;
  v[4 * t + 3] = e;
  __syncthreads();
  return total;
}

// The product staged scatter (12-bit digits, 2 slots), with the V1 prologue.
template <typename In>
__global__ __launch_bounds__(kPartThreads) void k_scatter_v1(
    In in, uint64_t n, uint32_t skip, const uint32_t* __restrict__ tot,
    const uint32_t* __restrict__ within, uint32_t* __restrict__ bstart, uint4* __restrict__ rec,
    uint32_t* __restrict__ rep) {
  constexpr uint32_t kBits = kStageBits, kSlots = 2;
  constexpr int kRows = 2;
  constexpr uint32_t nbins = 1u << kBits;
  __shared__ uint4 stage[nbins][kSlots];
  __shared__ uint32_t fill[nbins];
  __shared__ uint32_t cur[nbins];
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads) cur[b] = tot[b];
  __syncthreads();
  const uint32_t total = block_scan4096(cur, fill);
  const uint32_t blk = part_block();
  if (blk == 0) {
    for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads) bstart[b] = cur[b];
    if (threadIdx.x == 0) bstart[nbins] = total;
  }
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads) {
    cur[b] += within[static_cast<uint64_t>(b) * gridDim.x + blk];
    fill[b] = 0;
  }
  __syncthreads();
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  constexpr int U = kRows;
  constexpr uint64_t kStep = static_cast<uint64_t>(U) * kPartThreads;
  auto round = [&](const RowBatch<U>& q, uint64_t i0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = i0 + threadIdx.x + static_cast<uint64_t>(u) * kPartThreads;
      if (!q.in[u]) continue;
      const uint32_t r = in.rank_of(q, u);
      rep[i] = r;
      if (!in.valid_of(q, u)) continue;
      const uint64_t h = in_hash<In>(in.key_of(q, u));
      const uint32_t b = digit_of(h, skip, kBits);
      const uint4 rq = make_uint4(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32), r,
                                  in.row_of(q, u));
      const uint32_t sl = atomicAdd(&fill[b], 1u);
      if (sl < kSlots) {
        stage[b][sl] = rq;
      } else {
        rec[atomicAdd(&cur[b], 1u)] = rq;
      }
    }
    lds_barrier();
#pragma unroll
    for (uint32_t j = 0; j < nbins / kPartThreads; ++j) {
      const uint32_t b = threadIdx.x + j * kPartThreads;
      if (fill[b] >= kSlots) {
        const uint32_t p = cur[b];
        cur[b] = p + kSlots;
#pragma unroll
        for (uint32_t k = 0; k < kSlots; ++k) rec[p + k] = stage[b][k];
        fill[b] = 0;
      }
    }
    lds_barrier();
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
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads)
    for (uint32_t k = 0; k < fill[b]; ++k) rec[cur[b] + k] = stage[b][k];
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
  const GroupLayout L = group_layout(n);
  if (L.bits != kStageBits || L.cbits) {
    printf("n %llu: not the one-level 12-bit path\n", (unsigned long long)n);
    return 2;
  }
  uint64_t* key;
  uint32_t *rank, *rep, *rep2;
  uint8_t* has;
  (void)hipMalloc(&key, 8 * n);
  (void)hipMalloc(&rank, 4 * n);
  (void)hipMalloc(&has, n);
  (void)hipMalloc(&rep, 4 * n);
  (void)hipMalloc(&rep2, 4 * n);
  k_rows<<<4096, 256>>>(key, rank, has, n, n * 4 / 5);
  void* ws;
  (void)hipMalloc(&ws, L.total);
  uint32_t *tot, *within, *bstart;
  const uint32_t nb = 1u << L.bits, P = kPartBlocks;
  (void)hipMalloc(&tot, 4 * nb);
  (void)hipMalloc(&within, 4ull * nb * 1024);
  (void)hipMalloc(&bstart, 4 * (nb + 1));
  uint4* rec2;
  (void)hipMalloc(&rec2, 16 * n);
  uint64_t* gkey;
  uint32_t* gmin;
  (void)hipMalloc(&gkey, 8 * 4 * n);
  (void)hipMalloc(&gmin, 4 * 4 * n);
  GroupInput in;
  in.key = key;
  in.rank = rank;
  in.valid = has;
  in.n = n;
  const RowsIn rin{key, has, rank, 0};
  const ChunkOf c = ChunkOf::make(100);
  const size_t lds = 4u << L.bits;
  auto v1 = [&] {
    (void)hipMemsetAsync(tot, 0, 4 * nb, 0);
    k_hist_var<RowsIn, kUnroll, true><<<P, kPartThreads, lds>>>(rin, n, kShardBits, L.bits, tot, within);
    k_scatter_v1<RowsIn><<<P, kPartThreads>>>(rin, n, kShardBits, tot, within, bstart, rec2, rep2);
    k_bucket_group<<<nb, kGroupThreads>>>(rec2, bstart, 1, c, gkey, gmin, rep2);
  };
  (void)dedup_local_launch(in, 100, rep, true, ws, 0, nullptr);
  v1();
  (void)hipDeviceSynchronize();
  std::vector<uint32_t> a(n), b(n);
  (void)hipMemcpy(a.data(), rep, 4 * n, hipMemcpyDeviceToHost);
  (void)hipMemcpy(b.data(), rep2, 4 * n, hipMemcpyDeviceToHost);
  uint64_t bad = 0, linked = 0;
  for (uint64_t i = 0; i < n; ++i) bad += a[i] != b[i];
  std::vector<uint32_t> rk(n);
  (void)hipMemcpy(rk.data(), rank, 4 * n, hipMemcpyDeviceToHost);
  for (uint64_t i = 0; i < n; ++i) linked += a[i] != rk[i];
  printf("n %llu buckets %u linked %llu\n", (unsigned long long)n, nb, (unsigned long long)linked);
  printf("V1 mismatches vs product: %llu\n", (unsigned long long)bad);
  for (int rep_i = 0; rep_i < 2; ++rep_i) {
    printf("V0 product grouping    %.4f ms\n",
           time_ms([&] { (void)dedup_local_launch(in, 100, rep, true, ws, 0, nullptr); }, 15));
    printf("V1 reserve-by-atomics  %.4f ms\n", time_ms(v1, 15));
  }
  printf("  V1 memset+hist       %.4f ms\n", time_ms([&] {
           (void)hipMemsetAsync(tot, 0, 4 * nb, 0);
           k_hist_var<RowsIn, kUnroll, true><<<P, kPartThreads, lds>>>(rin, n, kShardBits, L.bits, tot, within);
         }, 15));
  printf("  V1 scatter           %.4f ms\n", time_ms([&] {
           k_scatter_v1<RowsIn><<<P, kPartThreads>>>(rin, n, kShardBits, tot, within, bstart, rec2, rep2);
         }, 15));
  printf("  V1 group             %.4f ms\n", time_ms([&] {
           k_bucket_group<<<nb, kGroupThreads>>>(rec2, bstart, 1, c, gkey, gmin, rep2);
         }, 15));
  printf("H0 product hist        %.4f ms\n", time_ms([&] {
           k_hist_var<RowsIn, kUnroll, true><<<P, kPartThreads, lds>>>(rin, n, kShardBits, L.bits, nullptr, within);
         }, 15));
  printf("H1 hist P=512          %.4f ms\n", time_ms([&] {
           k_hist_var<RowsIn, kUnroll, true><<<512, kPartThreads, lds>>>(rin, n, kShardBits, L.bits, nullptr, within);
         }, 15));
  printf("H2 hist 16 rows/batch  %.4f ms\n", time_ms([&] {
           k_hist_var<RowsIn, 16, true><<<P, kPartThreads, lds>>>(rin, n, kShardBits, L.bits, nullptr, within);
         }, 15));
  printf("H3 hist no LDS atomics %.4f ms\n", time_ms([&] {
           k_hist_var<RowsIn, kUnroll, false><<<P, kPartThreads, lds>>>(rin, n, kShardBits, L.bits, nullptr, within);
         }, 15));
  printf("H4 hist P=1024         %.4f ms\n", time_ms([&] {
           k_hist_var<RowsIn, kUnroll, true><<<1024, kPartThreads, lds>>>(rin, n, kShardBits, L.bits, nullptr, within);
         }, 15));
  return bad ? 1 : 0;
}
