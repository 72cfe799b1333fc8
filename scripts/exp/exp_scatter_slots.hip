// Experiment (not shipped): the staged bucket scatter at 12.5 M config-4-shaped
// rows with different (digit bits, LDS slots per bucket, rows per thread per
// round): fewer, wider partial-line writes (more slots) against more buckets.
// Each variant: its own histogram + scan once, then the scatter timed alone
// (median of 9); records checked by a per-variant checksum.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_scatter_slots.hip -o build/exp_scatter_slots
#include "../../spacedrive_amd/csrc/dedup.hip"

#include <stdio.h>

#include <vector>

using namespace sdgpu;

namespace {

__global__ void k_rows(uint64_t* key, uint32_t* rank, uint64_t n, uint64_t distinct) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint64_t j = (i * 0x9E3779B1ull) % n;
    key[i] = row_hash((j % distinct) * 0x2545F4914F6CDD1Dull + 7);
    rank[i] = static_cast<uint32_t>((i * 2654435761ull) % n);
  }
}

__global__ void k_check(const uint4* rec, uint64_t n, unsigned long long* sum) {
  unsigned long long s = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
    s += (static_cast<unsigned long long>(rec[i].z) * 0x9E3779B1ull) ^ rec[i].w ^ rec[i].x;
  atomicAdd(sum, s);
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

template <uint32_t kBits, uint32_t kSlots, int kRows>
void variant(RowsIn in, uint64_t n, uint32_t* hist, uint32_t* tiles, uint4* rec, uint32_t* rep,
             unsigned long long* sum) {
  const uint32_t P = kPartBlocks;
  const uint64_t nh = (uint64_t(1) << kBits) * P;
  const size_t lds = 4u << kBits;
  allow_lds(k_part_hist<RowsIn>, lds);
  k_part_hist<RowsIn><<<P, kPartThreads, lds, 0>>>(in, n, kShardBits, kBits, 0, hist);
  scan::exclusive(hist, nh, hist, tiles, nullptr, 0);
  const float t = time_ms(
      [&] {
        k_part_scatter_rec_staged<RowsIn, true, kBits, kSlots, kRows>
            <<<P, kPartThreads, 0, 0>>>(in, n, kShardBits, hist, rec, rep, nullptr, 0);
      },
      9);
  (void)hipMemset(sum, 0, 8);
  k_check<<<1024, 256>>>(rec, n, sum);
  unsigned long long h = 0;
  (void)hipMemcpy(&h, sum, 8, hipMemcpyDeviceToHost);
  printf("bits %2u slots %u rows/round %d : scatter %.4f ms  (%.2f TB/s of 29 B/row)  check %llx\n",
         kBits, kSlots, kRows, t, 29.0 * n / (t * 1e-3) / 1e12, h);
}

}  // namespace

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 12500000ull;
  uint64_t* key;
  uint32_t *rank, *rep, *hist, *tiles;
  uint4* rec;
  unsigned long long* sum;
  (void)hipMalloc(&key, 8 * n);
  (void)hipMalloc(&rank, 4 * n);
  (void)hipMalloc(&rep, 4 * n);
  (void)hipMalloc(&rec, 16 * n);
  (void)hipMalloc(&hist, 4 * ((uint64_t(1) << 12) * kPartBlocks + 1));
  (void)hipMalloc(&tiles, 4 * 65536);
  (void)hipMalloc(&sum, 8);
  k_rows<<<4096, 256>>>(key, rank, n, n * 4 / 5);
  const RowsIn in{key, nullptr, rank, 0};
  for (int rep_i = 0; rep_i < 2; ++rep_i) {
    variant<12, 2, 2>(in, n, hist, tiles, rec, rep, sum);
    variant<12, 2, 1>(in, n, hist, tiles, rec, rep, sum);
    variant<12, 2, 4>(in, n, hist, tiles, rec, rep, sum);
    variant<11, 4, 2>(in, n, hist, tiles, rec, rep, sum);
    variant<11, 4, 4>(in, n, hist, tiles, rec, rep, sum);
    variant<11, 2, 2>(in, n, hist, tiles, rec, rep, sum);
    variant<10, 8, 4>(in, n, hist, tiles, rec, rep, sum);
  }
  return 0;
}
