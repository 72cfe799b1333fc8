// Experiment: the two-level grouping's second pass (k_part2_runs) at 100 M rows,
// its staging run length kS2, blocks per segment kP2 and rows per thread kR2.
// (run r3F: S2 8 / R2 2 / R2 8 all slower, P2 128 faster; run r3G: P2 256 slower;
// run r3I: the flush threshold -- buckets with at least kF2 staged records
// are flushed at every round's end, so fewer arrivals meet a full slot array
// and leave as single-record stores: ~20 % of records at kF2 = 16 by a
// Poisson model, ~2 % at 8.)
// The product stages 16-record runs with 64 blocks per segment at ~106 KiB of
// LDS, so one block per CU: a block's prologue (segment / run-list / bucket
// scans, each behind a global load) overlaps no other block's main loop.
// 8-record runs halve the staging LDS (two blocks per CU) at the cost of
// shorter store runs; more blocks per segment shorten each block.
// Every variant's reps must equal the product's (dedup_local_launch).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_twolevel_s2.hip -o build/exp_twolevel_s2
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
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 100000000ull;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const GroupLayout L = group_layout(n);
  if (!L.cbits) {
    printf("n %llu: not the two-level path\n", (unsigned long long)n);
    return 2;
  }
  uint64_t* key;
  uint8_t* has;
  uint32_t *rep0, *rep1;
  (void)hipMalloc(&key, 8 * n);
  (void)hipMalloc(&has, n);
  (void)hipMalloc(&rep0, 4 * n);
  (void)hipMalloc(&rep1, 4 * n);
  k_rows<<<4096, 256>>>(key, has, n, n * 4 / 5);
  void* ws;
  if (hipMalloc(&ws, L.total) != hipSuccess) {
    printf("workspace %zu B: out of memory\n", L.total);
    return 1;
  }
  GroupInput gi;
  gi.key = key;
  gi.valid = has;
  gi.n = n;
  (void)dedup_local_launch(gi, 100, rep0, true, ws, 0, nullptr);
  (void)hipDeviceSynchronize();
  std::vector<uint32_t> a(n), b(n);
  (void)hipMemcpy(a.data(), rep0, 4 * n, hipMemcpyDeviceToHost);
  const RowsIn in{key, has, nullptr, 0};
  struct V {
    const char* name;
    std::function<void()> f;
  };
  std::vector<V> vs = {
      {"product (S2 16, P2 64, R2 4)",
       [&] { (void)dedup_local_launch(gi, 100, rep1, true, ws, 0, nullptr); }},
      {"S2 16, P2 128, R2 4 (flush at 16)",
       [&] { (void)two_level_launch<RowsIn, 9, 16, 4, 128, true, 16>(in, n, L, 100, rep1, true, ws, 0, nullptr); }},
      {"flush at 12",
       [&] { (void)two_level_launch<RowsIn, 9, 16, 4, 128, true, 12>(in, n, L, 100, rep1, true, ws, 0, nullptr); }},
      {"flush at 10",
       [&] { (void)two_level_launch<RowsIn, 9, 16, 4, 128, true, 10>(in, n, L, 100, rep1, true, ws, 0, nullptr); }},
      {"flush at 8",
       [&] { (void)two_level_launch<RowsIn, 9, 16, 4, 128, true, 8>(in, n, L, 100, rep1, true, ws, 0, nullptr); }},
      {"flush at 6",
       [&] { (void)two_level_launch<RowsIn, 9, 16, 4, 128, true, 6>(in, n, L, 100, rep1, true, ws, 0, nullptr); }},
  };
  for (auto& v : vs) {
    (void)hipMemset(rep1, 0xFF, 4 * n);
    v.f();
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(b.data(), rep1, 4 * n, hipMemcpyDeviceToHost);
    uint64_t bad = 0;
    for (uint64_t i = 0; i < n; ++i) bad += a[i] != b[i];
    printf("%-32s mismatches vs product: %llu  (%s)\n", v.name, (unsigned long long)bad,
           hipGetErrorString(hipGetLastError()));
  }
  for (int r = 0; r < 2; ++r)
    for (auto& v : vs) printf("%-32s %.4f ms\n", v.name, time_ms(v.f, reps));
  return 0;
}
