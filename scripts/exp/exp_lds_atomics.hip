// Experiment (not shipped): LDS operation rates on gfx950, to price K5
// bucket_group's insert phase (one ds_cmpst_rtn_b64 per probe + one ds_min_u32
// per keyed row).  Every kernel: 512 blocks x 1024 threads (2 per CU, the
// group kernel's occupancy), a 6144-slot u64 table + a u32 table in LDS (72 KiB,
// as the group kernel), each thread does kIters operations on pseudo-random
// slots (an LCG per thread, independent across iterations so the latencies
// overlap up to kPar in flight).  Reports lane-operations per ns chip-wide and
// per CU per clock at 2.4 GHz.
//   cas64     ds_cmpst_rtn_b64 (compare never matches: pure atomic traffic)
//   min32     ds_min_u32 (no return)
//   read64    ds_read_b64
//   cas64_dep ds_cmpst_rtn_b64 with each result feeding the next address
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_lds_atomics.hip -o build/exp_lds_atomics
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

namespace {

constexpr int kThreads = 1024;
constexpr uint32_t kSlots = 6144;
constexpr int kIters = 256;
constexpr int kPar = 4;

__device__ __forceinline__ uint32_t slot_of(uint32_t x) {
  return static_cast<uint32_t>((static_cast<uint64_t>(x) * kSlots) >> 32);
}

template <int kMode>
__global__ __launch_bounds__(kThreads) void k_lds(uint32_t seed, uint32_t* __restrict__ sink) {
  __shared__ uint64_t tk[kSlots];
  __shared__ uint32_t tm[kSlots];
  for (uint32_t s = threadIdx.x; s < kSlots; s += kThreads) {
    tk[s] = s;
    tm[s] = 0xFFFFFFFFu;
  }
  __syncthreads();
  uint32_t x[kPar];
#pragma unroll
  for (int p = 0; p < kPar; ++p) x[p] = (blockIdx.x * kThreads + threadIdx.x) * 2654435761u + p * 97u + seed;
  uint64_t acc = 0;
  for (int it = 0; it < kIters / kPar; ++it) {
    uint64_t r[kPar];
#pragma unroll
    for (int p = 0; p < kPar; ++p) {
      x[p] = x[p] * 1664525u + 1013904223u;
      const uint32_t s = slot_of(x[p]);
      if (kMode == 0 || kMode == 3) {
        r[p] = atomicCAS(reinterpret_cast<unsigned long long*>(&tk[s]), ~0ull,
                         static_cast<unsigned long long>(x[p]));
      } else if (kMode == 1) {
        atomicMin(&tm[s], x[p]);
        r[p] = 0;
      } else {
        r[p] = tk[s];
      }
    }
#pragma unroll
    for (int p = 0; p < kPar; ++p) {
      acc += r[p];
      if (kMode == 3) x[p] ^= static_cast<uint32_t>(r[p]);  // serialise on the result
    }
  }
  __syncthreads();
  if (acc == 0x123456789ull) sink[0] = tm[threadIdx.x % kSlots];
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

int main() {
  uint32_t* sink;
  (void)hipMalloc(&sink, 64);
  const uint32_t blocks = 512;
  const double ops = static_cast<double>(blocks) * kThreads * kIters;
  auto report = [&](const char* name, float ms) {
    const double per_ns = ops / (ms * 1e6);
    printf("%-10s %8.4f ms  %8.1f lane-ops/ns chip  %6.2f lane-ops/clk/CU at 2.4 GHz\n", name, ms,
           per_ns, per_ns / 256.0 / 2.4);
  };
  report("cas64", time_ms([&] { k_lds<0><<<blocks, kThreads>>>(1, sink); }, 9));
  report("min32", time_ms([&] { k_lds<1><<<blocks, kThreads>>>(1, sink); }, 9));
  report("read64", time_ms([&] { k_lds<2><<<blocks, kThreads>>>(1, sink); }, 9));
  report("cas64_dep", time_ms([&] { k_lds<3><<<blocks, kThreads>>>(1, sink); }, 9));
  return 0;
}
