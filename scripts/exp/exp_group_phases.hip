// Experiment (not shipped): phase costs of K5 bucket_group on 12.5 M
// config-4-shaped rows (80 % distinct keys).  The product partition runs once;
// then the group kernel is timed cut after each phase:
//   A  load the bucket's records into registers (checksum only)
//   B  A + LDS table init + barrier
//   C  B + inserts (CAS probe loop + ds_min) + barrier
//   D  C + lookups (checksum, no rep writes)
//   E  D + rep writes (the product kernel)
// plus E with 512 threads per workgroup (same table, 4 workgroups per CU
// impossible at 72 KiB, so 2) to see the per-thread row count effect.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_group_phases.hip -o build/exp_group_phases
#include "../../spacedrive_amd/csrc/dedup.hip"

#include <stdio.h>

#include <vector>

using namespace sdgpu;

namespace {

// linear probing, as the product kernel used before round 2's double hashing
__device__ __forceinline__ uint32_t lin_next(uint32_t h) {
  return h + 1 == kLdsSlots ? 0u : h + 1;
}

__global__ void k_rows(uint64_t* key, uint32_t* rank, uint64_t n, uint64_t distinct) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint64_t j = (i * 0x9E3779B1ull) % n;
    key[i] = row_hash((j % distinct) * 0x2545F4914F6CDD1Dull + 7);
    rank[i] = static_cast<uint32_t>(i);
  }
}

template <int PH, int T>
__global__ __launch_bounds__(T) void gph(const uint4* __restrict__ rec,
                                        const uint32_t* __restrict__ offs, uint32_t P,
                                        ChunkOf chunk_of, uint32_t* __restrict__ rep,
                                        uint32_t* __restrict__ sink) {
  constexpr int kP = (kLdsCap + T - 1) / T;
  __shared__ uint64_t lkey[kLdsSlots];
  __shared__ uint32_t lmin[kLdsSlots];
  const uint32_t b = blockIdx.x;
  const uint32_t start = offs[static_cast<uint64_t>(b) * P];
  const uint32_t end = offs[static_cast<uint64_t>(b + 1) * P];
  if (end - start > kLdsCap) return;
  uint4 q[kP];
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const uint32_t i = start + threadIdx.x + j * T;
    q[j] = i < end ? rec[i] : make_uint4(0, 0, 0, 0);
  }
  uint32_t acc = 0;
  if (PH == 0) {
#pragma unroll
    for (int j = 0; j < kP; ++j) acc += q[j].x ^ q[j].w;
    if (acc == 0x12345678u) sink[0] = acc;
    return;
  }
  for (uint32_t s = threadIdx.x; s < kLdsSlots; s += T) {
    lkey[s] = kEmpty;
    lmin[s] = 0xFFFFFFFFu;
  }
  __syncthreads();
  uint32_t h[kP], pend = 0;
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const uint64_t k = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
    h[j] = lds_slot(k);
    if (start + threadIdx.x + j * T < end) pend |= 1u << j;
  }
  if (PH == 1) {
#pragma unroll
    for (int j = 0; j < kP; ++j) acc += lkey[h[j]] ^ q[j].w;
    if (acc == 0x12345678u) sink[0] = acc;
    return;
  }
  const uint32_t live = pend;
  while (pend) {
    uint64_t prev[kP];
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      const uint64_t k = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
      prev[j] = (pend >> j & 1u) ? atomicCAS(reinterpret_cast<unsigned long long*>(&lkey[h[j]]),
                                             static_cast<unsigned long long>(kEmpty),
                                             static_cast<unsigned long long>(k))
                                 : 0ull;
    }
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      if (!(pend >> j & 1u)) continue;
      const uint64_t k = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
      if (prev[j] == kEmpty || prev[j] == k) {
        atomicMin(&lmin[h[j]], q[j].z);
        pend &= ~(1u << j);
      } else {
        h[j] = lin_next(h[j]);
      }
    }
  }
  __syncthreads();
  if (PH == 2) {
#pragma unroll
    for (int j = 0; j < kP; ++j) acc += h[j] ^ q[j].w;
    if (acc == 0x12345678u) sink[0] = acc;
    return;
  }
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    if (!(live >> j & 1u)) continue;
    const uint32_t r = q[j].z, f = lmin[h[j]];
    if (chunk_of(r) != chunk_of(f)) {
      if (PH == 4) rep[q[j].w] = f;
      else acc += f ^ q[j].w;
    }
  }
  if (PH == 3 && acc == 0x12345678u) sink[0] = acc;
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
  uint64_t* key;
  uint32_t *rank, *rep, *rep2, *sink;
  (void)hipMalloc(&key, 8 * n);
  (void)hipMalloc(&rank, 4 * n);
  (void)hipMalloc(&rep, 4 * n);
  (void)hipMalloc(&rep2, 4 * n);
  (void)hipMalloc(&sink, 64);
  k_rows<<<4096, 256>>>(key, rank, n, n * 4 / 5);
  const GroupLayout L = group_layout(n);
  void* ws;
  (void)hipMalloc(&ws, L.total);
  GroupInput in;
  in.key = key;
  in.rank = rank;
  in.n = n;
  (void)dedup_local_launch(in, 100, rep, true, ws, 0, nullptr);
  (void)hipDeviceSynchronize();
  uint8_t* w = static_cast<uint8_t*>(ws);
  const uint4* rec = reinterpret_cast<const uint4*>(w + L.rec);
  // bucket starts: the fine-count paths (12-bit one-level, two-level) publish
  // them with stride 1 (round 2); narrower partitions use the digit-major scan
  const bool fine = L.cbits || L.bits == kStageBits;
  const uint32_t* hist = reinterpret_cast<const uint32_t*>(w + (fine ? L.fbase : L.hist));
  const uint32_t P = fine ? 1u : bucket_part_blocks(), nb = 1u << L.bits;
  const ChunkOf c = ChunkOf::make(100);
  printf("n %llu buckets %u\n", (unsigned long long)n, nb);
  printf("full grouping          %.4f ms\n",
         time_ms([&] { (void)dedup_local_launch(in, 100, rep, true, ws, 0, nullptr); }, 9));
  printf("A load                 %.4f ms\n", time_ms([&] { gph<0, 1024><<<nb, 1024>>>(rec, hist, P, c, rep2, sink); }, 9));
  printf("B + init               %.4f ms\n", time_ms([&] { gph<1, 1024><<<nb, 1024>>>(rec, hist, P, c, rep2, sink); }, 9));
  printf("C + insert             %.4f ms\n", time_ms([&] { gph<2, 1024><<<nb, 1024>>>(rec, hist, P, c, rep2, sink); }, 9));
  printf("D + lookup             %.4f ms\n", time_ms([&] { gph<3, 1024><<<nb, 1024>>>(rec, hist, P, c, rep2, sink); }, 9));
  printf("E + rep writes         %.4f ms\n", time_ms([&] { gph<4, 1024><<<nb, 1024>>>(rec, hist, P, c, rep2, sink); }, 9));
  printf("E 512 threads          %.4f ms\n", time_ms([&] { gph<4, 512><<<nb, 512>>>(rec, hist, P, c, rep2, sink); }, 9));
  printf("A 512 threads          %.4f ms\n", time_ms([&] { gph<0, 512><<<nb, 512>>>(rec, hist, P, c, rep2, sink); }, 9));
  // correctness of E against the product (rep2 starts from the product's init)
  (void)hipMemcpy(rep2, rank, 4 * n, hipMemcpyDeviceToDevice);
  gph<4, 1024><<<nb, 1024>>>(rec, hist, P, c, rep2, sink);
  (void)hipDeviceSynchronize();
  std::vector<uint32_t> a(n), b(n);
  (void)hipMemcpy(a.data(), rep, 4 * n, hipMemcpyDeviceToHost);
  (void)hipMemcpy(b.data(), rep2, 4 * n, hipMemcpyDeviceToHost);
  uint64_t bad = 0;
  for (uint64_t i = 0; i < n; ++i) bad += a[i] != b[i];
  printf("E mismatches vs product: %llu\n", (unsigned long long)bad);
  return bad ? 1 : 0;
}
