// Experiment (round 3): the price of the bucket scatter's store pattern alone.
// 2^24 12-byte records (201 MB) are written with no loads and no LDS, as
// runs of R consecutive records at random run positions (a bijection of the
// run index, so every record is written once), by one lane per record
// (adjacent lanes write adjacent records of a run) or one lane per run:
//   W0  coalesced (run = the whole array)          -- the floor
//   W1  runs of 1 (single 12-B stores)
//   W2  runs of 2, one lane writes both (the product's flush)
//   W2L runs of 2, two adjacent lanes
//   W4L runs of 4, four adjacent lanes
//   W8L runs of 8, eight adjacent lanes
//   W16L runs of 16
//   A2L runs of 2 16-byte records (32-B aligned pairs), two lanes
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_stores.hip -o build/exp_stores
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <functional>
#include <vector>

namespace {

constexpr int kThreads = 1024;
constexpr uint32_t kBlocks = 256;

// position of run j among m runs (m a power of two): (j * odd) mod m, a
// bijection (n = 2^24 records, 201 MB, so that m = n / R is a power of two)
__device__ __forceinline__ uint64_t run_pos(uint64_t j, uint64_t m) {
  return (j * 2654435761ull) & (m - 1);
}

template <uint32_t R, bool kLanePerRec>
__global__ __launch_bounds__(kThreads) void k_runs(uint3* __restrict__ out, uint64_t n) {
  const uint64_t m = n / R;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
  if constexpr (kLanePerRec) {
    for (uint64_t i = blockIdx.x * static_cast<uint64_t>(kThreads) + threadIdx.x; i < m * R;
         i += stride) {
      const uint64_t j = i / R, k = i % R;
      const uint64_t p = run_pos(j, m) * R + k;
      out[p] = make_uint3(static_cast<uint32_t>(i), 1u, 2u);
    }
  } else {
    for (uint64_t j = blockIdx.x * static_cast<uint64_t>(kThreads) + threadIdx.x; j < m;
         j += stride) {
      const uint64_t p = run_pos(j, m) * R;
#pragma unroll
      for (uint32_t k = 0; k < R; ++k) out[p + k] = make_uint3(static_cast<uint32_t>(j), k, 2u);
    }
  }
}

__global__ __launch_bounds__(kThreads) void k_coalesced(uint3* __restrict__ out, uint64_t n) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(kThreads) + threadIdx.x; i < n; i += stride)
    out[i] = make_uint3(static_cast<uint32_t>(i), 1u, 2u);
}

__global__ __launch_bounds__(kThreads) void k_pairs16(uint4* __restrict__ out, uint64_t n) {
  const uint64_t m = n / 2;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(kThreads) + threadIdx.x; i < m * 2;
       i += stride) {
    const uint64_t p = run_pos(i / 2, m) * 2 + (i & 1);
    out[p] = make_uint4(static_cast<uint32_t>(i), 1u, 2u, 3u);
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
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1ull << 24);
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  if (n & (n - 1)) {
    printf("n must be a power of two\n");
    return 2;
  }
  uint3* out;
  uint4* out16;
  (void)hipMalloc(&out, 12 * n);
  (void)hipMalloc(&out16, 16 * n);
  // every record written exactly once (W2: bijection check on the host)
  {
    (void)hipMemset(out, 0xFF, 12 * n);
    k_runs<2, true><<<kBlocks, kThreads>>>(out, n);
    std::vector<uint3> h(n);
    (void)hipMemcpy(h.data(), out, 12 * n, hipMemcpyDeviceToHost);
    uint64_t unwritten = 0;
    for (uint64_t i = 0; i < n; ++i) unwritten += h[i].y == 0xFFFFFFFFu;
    printf("W2L unwritten records: %llu of %llu\n", (unsigned long long)unwritten,
           (unsigned long long)n);
  }
  struct V {
    const char* name;
    std::function<void()> f;
  };
  std::vector<V> vs = {
      {"W0  coalesced", [&] { k_coalesced<<<kBlocks, kThreads>>>(out, n); }},
      {"W1  runs of 1", [&] { k_runs<1, true><<<kBlocks, kThreads>>>(out, n); }},
      {"W2  runs of 2, lane per run", [&] { k_runs<2, false><<<kBlocks, kThreads>>>(out, n); }},
      {"W2L runs of 2, lane per record", [&] { k_runs<2, true><<<kBlocks, kThreads>>>(out, n); }},
      {"W4L runs of 4, lane per record", [&] { k_runs<4, true><<<kBlocks, kThreads>>>(out, n); }},
      {"W8L runs of 8, lane per record", [&] { k_runs<8, true><<<kBlocks, kThreads>>>(out, n); }},
      {"W16L runs of 16, lane per record", [&] { k_runs<16, true><<<kBlocks, kThreads>>>(out, n); }},
      {"A2L 16-B pairs (32-B aligned)", [&] { k_pairs16<<<kBlocks, kThreads>>>(out16, n); }},
  };
  for (int r = 0; r < 2; ++r)
    for (auto& v : vs) printf("%-36s %.4f ms\n", v.name, time_ms(v.f, reps));
  printf("%s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
