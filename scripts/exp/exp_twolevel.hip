// Experiment (not shipped): the two-level partition at 100 M rows (2^15
// buckets): digit split and second-pass block count.  The A/B that retired the
// second pass's histogram kernel (hist2 5+10/8 3.40 ms -> fine counts 6+9/16
// 2.94 ms) ran against the removed variant: profiles/r2/exp_twolevel_r2E.log.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_twolevel.hip -o build/exp_twolevel
#include "../../spacedrive_amd/csrc/dedup.hip"

#include <stdio.h>

#include <string>
#include <utility>
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

__global__ void k_fill_key(uint64_t* key, uint64_t m) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < m; i += gridDim.x * 256ull) key[i] = 42;
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

// Synchronous per-kernel event timer (experiment only).
struct EvTimer : KTimer {
  hipEvent_t a{}, b{};
  const char* cur = nullptr;
  std::vector<std::pair<std::string, std::pair<double, int>>> acc;
  EvTimer() {
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
  }
  void begin(const char* name, hipStream_t s) override {
    cur = name;
    (void)hipEventRecord(a, s);
  }
  void end(hipStream_t s) override {
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    for (auto& e : acc)
      if (e.first == cur) {
        e.second.first += ms;
        e.second.second += 1;
        return;
      }
    acc.push_back({cur, {ms, 1}});
  }
};

uint64_t mismatches(const uint32_t* a_d, const uint32_t* b_d, uint64_t n) {
  std::vector<uint32_t> a(n), b(n);
  (void)hipMemcpy(a.data(), a_d, 4 * n, hipMemcpyDeviceToHost);
  (void)hipMemcpy(b.data(), b_d, 4 * n, hipMemcpyDeviceToHost);
  uint64_t bad = 0;
  for (uint64_t i = 0; i < n; ++i) bad += a[i] != b[i];
  return bad;
}

}  // namespace

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 100000000ull;
  uint64_t* key;
  uint32_t *rank, *rep, *rep2;
  uint8_t* has;
  (void)hipMalloc(&key, 8 * n);
  (void)hipMalloc(&rank, 4 * n);
  (void)hipMalloc(&has, n);
  (void)hipMalloc(&rep, 4 * n);
  (void)hipMalloc(&rep2, 4 * n);
  k_rows<<<4096, 256>>>(key, rank, has, n, n * 4 / 5);
  const GroupLayout L10 = group_layout(n, 10), L9 = group_layout(n, 9);
  void* ws;
  (void)hipMalloc(&ws, std::max(L10.total, L9.total));
  const RowsIn rin{key, has, rank, 0};
  printf("n %llu bits %u\n", (unsigned long long)n, L10.bits);
  auto p9 = [&] { (void)two_level_launch<RowsIn, 9, 16, 4, 64>(rin, n, L9, 100, rep, true, ws, 0, nullptr); };
  auto p10 = [&] { (void)two_level_launch<RowsIn, 10, 8, 4, 64>(rin, n, L10, 100, rep2, true, ws, 0, nullptr); };
  auto p9b = [&] { (void)two_level_launch<RowsIn, 9, 16, 4, 32>(rin, n, L9, 100, rep2, true, ws, 0, nullptr); };
  p9();
  p10();
  (void)hipDeviceSynchronize();
  printf("5+10/8 mismatches vs 6+9/16: %llu\n", (unsigned long long)mismatches(rep, rep2, n));
  for (int r = 0; r < 2; ++r) {
    printf("6+9/16 P2 64 (product) %.4f ms\n", time_ms(p9, 9));
    printf("5+10/8 P2 64           %.4f ms\n", time_ms(p10, 9));
    printf("6+9/16 P2 32           %.4f ms\n", time_ms(p9b, 9));
  }
  EvTimer kt;
  for (int r = 0; r < 5; ++r)
    (void)two_level_launch<RowsIn, 9, 16, 4, 64>(rin, n, L9, 100, rep, true, ws, 0, &kt);
  (void)hipDeviceSynchronize();
  printf("6+9/16 kernels:");
  for (auto& e : kt.acc) printf(" %s %.4f", e.first.c_str(), e.second.first / e.second.second);
  printf("\n");
  // forced fine-count overflow: one key on the first 100 k rows (> 64 Ki in
  // the first coarse block's tile) -> k_fine_recount
  k_fill_key<<<64, 256>>>(key, 100000);
  p9();
  p10();
  (void)hipDeviceSynchronize();
  printf("heavy key: 5+10/8 mismatches vs 6+9/16: %llu\n", (unsigned long long)mismatches(rep, rep2, n));
  printf("heavy key: 6+9/16 %.4f ms\n", time_ms(p9, 5));
  return 0;
}
