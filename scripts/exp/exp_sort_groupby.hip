// Experiment: the "radix sort + segmented group-by" formulation of the
// cas_id -> Object grouping, on the config-4 shape of one GPU (12.5 M rows,
// 80 % distinct u64 keys, ranks a permutation), against which the product's
// one-pass radix partition + LDS hash group-by (dedup.hip, 0.47 ms) is judged.
//
//   A: hipcub::DeviceRadixSort::SortPairs over all 64 key bits, value = row
//      index (u32) -- the cheapest sort that can find equal keys;
//   B: the same with value = (rank << 32 | row) (u64), which the group-by needs;
//   C: B + the segmented group-by: one thread per sorted row, the segment's
//      min rank found by walking back/forward over equal keys (segments are
//      ~1.25 rows), rep scattered to the row's original position.
// Each timed over 20 launches with HIP events; prints ms per call and rows/s.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_sort_groupby.hip -o build/exp_sort_groupby
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>
#include <stdio.h>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__device__ inline uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// 80 % distinct keys, 20 % duplicates of them; rank = (i * a + c) mod n, a
// permutation of the row index since the prime a = 2654435761 does not divide n.
__global__ void k_init(uint64_t* key, uint32_t* idx, uint64_t* val, uint32_t* rank, uint64_t n,
                       uint64_t distinct) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint64_t j = i < distinct ? i : mix(i * 0x9E3779B97F4A7C15ull) % distinct;
    key[i] = mix(j * 0x9E3779B97F4A7C15ull + 4);
    const uint32_t r = static_cast<uint32_t>((i * 2654435761ull + 12345) % n);
    rank[i] = r;
    idx[i] = static_cast<uint32_t>(i);
    val[i] = (static_cast<uint64_t>(r) << 32) | i;
  }
}

__global__ void k_segment_group(const uint64_t* __restrict__ skey, const uint64_t* __restrict__ sval,
                                uint64_t n, uint32_t chunk_rows, uint32_t* __restrict__ rep) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint64_t k = skey[i];
    uint32_t f = static_cast<uint32_t>(sval[i] >> 32);
    for (uint64_t j = i; j > 0 && skey[j - 1] == k; --j) f = min(f, static_cast<uint32_t>(sval[j - 1] >> 32));
    for (uint64_t j = i + 1; j < n && skey[j] == k; ++j) f = min(f, static_cast<uint32_t>(sval[j] >> 32));
    const uint32_t r = static_cast<uint32_t>(sval[i] >> 32);
    rep[static_cast<uint32_t>(sval[i])] = (r / chunk_rows == f / chunk_rows) ? r : f;
  }
}

int main() {
  const uint64_t n = 12'500'000, distinct = n * 8 / 10;
  uint64_t *key, *skey, *val, *sval;
  uint32_t *idx, *sidx, *rank, *rep;
  CK(hipMalloc(&key, 8 * n));
  CK(hipMalloc(&skey, 8 * n));
  CK(hipMalloc(&val, 8 * n));
  CK(hipMalloc(&sval, 8 * n));
  CK(hipMalloc(&idx, 4 * n));
  CK(hipMalloc(&sidx, 4 * n));
  CK(hipMalloc(&rank, 4 * n));
  CK(hipMalloc(&rep, 4 * n));
  k_init<<<4096, 256>>>(key, idx, val, rank, n, distinct);
  CK(hipGetLastError());
  size_t ta = 0, tb = 0;
  CK(hipcub::DeviceRadixSort::SortPairs(nullptr, ta, key, skey, idx, sidx, n));
  CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, key, skey, val, sval, n));
  void* tmp;
  CK(hipMalloc(&tmp, ta > tb ? ta : tb));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 20;
  float ms;
  for (int mode = 0; mode < 3; ++mode) {
    for (int w = 0; w < 2 + reps; ++w) {
      if (w == 2) CK(hipEventRecord(e0));
      if (mode == 0) {
        CK(hipcub::DeviceRadixSort::SortPairs(tmp, ta, key, skey, idx, sidx, n));
      } else {
        CK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, key, skey, val, sval, n));
        if (mode == 2) k_segment_group<<<8192, 256>>>(skey, sval, n, 100, rep);
      }
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    const char* name[3] = {"A sort (u64 key, u32 row)", "B sort (u64 key, u64 rank|row)",
                           "C sort B + segmented group-by + rep scatter"};
    printf("%-46s %8.3f ms  %6.2f G rows/s\n", name[mode], ms / reps, n / (ms / reps * 1e-3) / 1e9);
  }
  // sanity: sorted keys ascending
  uint64_t h[2];
  CK(hipMemcpy(h, skey + n / 2, 16, hipMemcpyDeviceToHost));
  printf("sorted check: %s\n", h[0] <= h[1] ? "ok" : "NOT SORTED");
  return 0;
}
