// Experiment (group phase): K5 with an 8-byte LDS table.
// Inside a bucket the hash bits of the bucket digit are implied, so a key
// needs 64 - bits bits; with the record's index inside its bucket (< 4096,
// 12 bits) beside them a slot is ONE 64-bit word {key rest, index + 1}.  The
// CAS tells a thread the owner's index directly, the group minimum lives per
// owner (lmin[4096]), and the table can be larger for the same LDS: lower
// load, shorter probe chains (the product's waves wait out chains of up to
// ~19 CAS rounds at load 1/2, profiles/r2/exp_group_persist_r2AG.log).
//   G0   product k_bucket_group12: 6144 x 12-B slots, load ~0.5, 2 WG/CU
//   GK   packed, 7680 slots (60 KiB) + lmin 16 KiB, load ~0.4, 2 WG/CU
//   GK16 packed, 16384 slots (128 KiB), load ~0.19, 1 WG/CU
// Records from the product partition (12.5 M config-4-shaped rows, rank order:
// 12-byte records); reps must equal the product's.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_group_packed.hip -o build/exp_group_packed
#include "../../spacedrive_amd/csrc/dedup.hip"

#include <stdio.h>

#include <algorithm>
#include <functional>
#include <vector>

using namespace sdgpu;

namespace {

constexpr uint32_t kNb = 1u << kStageBits;
constexpr uint32_t kPkCap = 4095;  // index + 1 in 12 bits, 0 = empty

__global__ void k_rows(uint64_t* key, uint8_t* has, uint64_t n, uint64_t distinct) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint64_t j = (i * 0x9E3779B1ull) % n;
    key[i] = row_hash((j % distinct) * 0x2545F4914F6CDD1Dull + 7);
    has[i] = (row_hash(i ^ 0x55ull) % 1000) != 0;
  }
}

// h without its `bits` digit bits [56 - bits, 56): 64 - bits bits
__device__ __forceinline__ uint64_t key_rest(uint64_t h, uint32_t bits) {
  const uint32_t lo = 56 - bits;
  return (h & ((1ull << lo) - 1)) | ((h >> 56) << lo);
}

template <uint32_t kSlots, int kMinWaves>
__global__ __launch_bounds__(kGroupThreads, kMinWaves) void k_group_packed(
    const uint3* __restrict__ rec, uint32_t rank_base, const uint32_t* __restrict__ offs,
    uint32_t bits, ChunkOf chunk_of, uint64_t* __restrict__ gkey, uint32_t* __restrict__ gmin,
    uint32_t* __restrict__ rep) {
  __shared__ uint64_t tab[kSlots];
  __shared__ uint32_t lmin[kPkCap + 1];
  constexpr int kP = (kPkCap + kGroupThreads) / kGroupThreads;  // 4
  const uint32_t b = blockIdx.x;
  const uint32_t start = offs[b], end = offs[b + 1], m = end - start;
  if (m > kPkCap) {  // oversized bucket: a private region of the global table
    __shared__ uint32_t special_min;
    const Rec12Src src{rec, rank_base};
    uint64_t tsize = 1;
    while (tsize * 2 <= 4ull * m) tsize *= 2;
    uint64_t* tk = gkey + 4ull * start;
    uint32_t* tm = gmin + 4ull * start;
    for (uint64_t s = threadIdx.x; s < tsize; s += kGroupThreads) {
      tk[s] = kEmpty;
      tm[s] = 0xFFFFFFFFu;
    }
    if (threadIdx.x == 0) special_min = 0xFFFFFFFFu;
    __syncthreads();
    for (uint32_t i = start + threadIdx.x; i < end; i += kGroupThreads) {
      const uint4 qq = src(i);
      const uint64_t k = (static_cast<uint64_t>(qq.y) << 32) | qq.x;
      if (k == kEmpty) {
        atomicMin(&special_min, qq.z);
        continue;
      }
      uint64_t h = k & (tsize - 1);
      for (;;) {
        const uint64_t prev = atomicCAS(reinterpret_cast<unsigned long long*>(&tk[h]),
                                        static_cast<unsigned long long>(kEmpty),
                                        static_cast<unsigned long long>(k));
        if (prev == kEmpty || prev == k) {
          atomicMin(&tm[h], qq.z);
          break;
        }
        h = (h + 1) & (tsize - 1);
      }
    }
    __syncthreads();
    for (uint32_t i = start + threadIdx.x; i < end; i += kGroupThreads) {
      const uint4 qq = src(i);
      const uint64_t k = (static_cast<uint64_t>(qq.y) << 32) | qq.x;
      uint32_t f;
      if (k == kEmpty) {
        f = special_min;
      } else {
        uint64_t h = k & (tsize - 1);
        while (__hip_atomic_load(&tk[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != k)
          h = (h + 1) & (tsize - 1);
        f = __hip_atomic_load(&tm[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (chunk_of(qq.z) != chunk_of(f)) rep[qq.w] = f;
    }
    return;
  }
  uint3 q[kP];
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const uint32_t i = start + threadIdx.x + j * kGroupThreads;
    q[j] = i < end ? rec[i] : make_uint3(0, 0, 0);
  }
  for (uint32_t s = threadIdx.x; s < kSlots; s += kGroupThreads) tab[s] = 0ull;
  for (uint32_t s = threadIdx.x; s <= kPkCap; s += kGroupThreads) lmin[s] = 0xFFFFFFFFu;
  __syncthreads();
  uint32_t slot[kP], step[kP], owner[kP];
  uint64_t mine[kP];
  uint32_t pend = 0;
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const uint64_t h = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
    const uint32_t idx = threadIdx.x + j * kGroupThreads;
    mine[j] = (key_rest(h, bits) << 12) | (idx + 1);
    slot[j] = static_cast<uint32_t>((static_cast<uint64_t>(static_cast<uint32_t>(h)) * kSlots) >> 32);
    // probe step coprime with kSlots (a power of two or 2^k * 15): odd and not a multiple of 3 or 5
    uint32_t st = 1u + 2u * static_cast<uint32_t>((h >> 40) & 1023u);
    while (st % 3u == 0 || st % 5u == 0) st += 2;
    step[j] = st % kSlots;
    owner[j] = idx;
    if (start + idx < end) pend |= 1u << j;
  }
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
        pend &= ~(1u << j);  // owner: itself
      } else if ((prev[j] >> 12) == (mine[j] >> 12)) {
        owner[j] = static_cast<uint32_t>(prev[j] & 0xFFFu) - 1;
        pend &= ~(1u << j);
      } else {
        const uint32_t s = slot[j] + step[j];
        slot[j] = s >= kSlots ? s - kSlots : s;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < kP; ++j)
    if (start + threadIdx.x + j * kGroupThreads < end) atomicMin(&lmin[owner[j]], rank_base + q[j].z);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    if (start + threadIdx.x + j * kGroupThreads >= end) continue;
    const uint32_t r = rank_base + q[j].z, f = lmin[owner[j]];
    if (chunk_of(r) != chunk_of(f)) rep[q[j].z] = f;
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
  uint32_t *rep0, *rep1, *init;
  (void)hipMalloc(&key, 8 * n);
  (void)hipMalloc(&has, n);
  (void)hipMalloc(&rep0, 4 * n);
  (void)hipMalloc(&rep1, 4 * n);
  (void)hipMalloc(&init, 4 * n);
  k_rows<<<4096, 256>>>(key, has, n, n * 4 / 5);
  void* ws;
  (void)hipMalloc(&ws, L.total);
  uint8_t* w = static_cast<uint8_t*>(ws);
  uint3* rec = reinterpret_cast<uint3*>(w + L.rec);
  uint64_t* gkey = reinterpret_cast<uint64_t*>(w + L.gkey);
  uint32_t* gmin = reinterpret_cast<uint32_t*>(w + L.gmin);
  uint32_t* fbase = reinterpret_cast<uint32_t*>(w + L.fbase);
  const ChunkOf c = ChunkOf::make(100);
  GroupInput gi;
  gi.key = key;
  gi.valid = has;
  gi.n = n;
  // the product's partition + group (records and bucket starts stay in ws)
  (void)dedup_local_launch(gi, 100, rep0, true, ws, 0, nullptr);
  (void)hipDeviceSynchronize();
  std::vector<uint32_t> a(n), b(n), rk(n);
  (void)hipMemcpy(a.data(), rep0, 4 * n, hipMemcpyDeviceToHost);
  for (uint64_t i = 0; i < n; ++i) rk[i] = static_cast<uint32_t>(i);
  (void)hipMemcpy(init, rk.data(), 4 * n, hipMemcpyHostToDevice);
  std::vector<uint32_t> sizes(kNb + 1);
  (void)hipMemcpy(sizes.data(), fbase, 4 * (kNb + 1), hipMemcpyDeviceToHost);
  uint32_t mx = 0;
  for (uint32_t i = 0; i < kNb; ++i) mx = std::max(mx, sizes[i + 1] - sizes[i]);
  printf("n %llu buckets %u largest bucket %u\n", (unsigned long long)n, kNb, mx);
  struct V {
    const char* name;
    std::function<void()> f;
  };
  std::vector<V> vs = {
      {"G0 product group12 (6144 x 12 B)",
       [&] { k_bucket_group12<<<kNb, kGroupThreads>>>(rec, 0, fbase, c, gkey, gmin, rep1); }},
      {"GK packed 7680 x 8 B, 2 WG/CU",
       [&] {
         k_group_packed<7680, 8><<<kNb, kGroupThreads>>>(rec, 0, fbase, kStageBits, c, gkey, gmin, rep1);
       }},
      {"GK16 packed 16384 x 8 B, 1 WG/CU",
       [&] {
         k_group_packed<16384, 4><<<kNb, kGroupThreads>>>(rec, 0, fbase, kStageBits, c, gkey, gmin,
                                                          rep1);
       }}};
  for (auto& v : vs) {
    (void)hipMemcpy(rep1, init, 4 * n, hipMemcpyDeviceToDevice);
    v.f();
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(b.data(), rep1, 4 * n, hipMemcpyDeviceToHost);
    uint64_t bad = 0;
    for (uint64_t i = 0; i < n; ++i) bad += a[i] != b[i];
    printf("%-36s mismatches vs product: %llu  (%s)\n", v.name, (unsigned long long)bad,
           hipGetErrorString(hipGetLastError()));
  }
  for (int r = 0; r < 2; ++r)
    for (auto& v : vs) printf("%-36s %.4f ms\n", v.name, time_ms(v.f, reps));
  return 0;
}
