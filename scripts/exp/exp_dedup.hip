// Experiment: where does the bucket scatter time go?  12.5 M random u64 keys,
// 8192 buckets, 256 blocks x 1024 threads (the K6 shape).
//   S0: LDS cursor atomics + scattered 16-B record stores   (the product kernel)
//   S1: LDS cursor atomics only (stores to the thread's own sequential slot)
//   S2: scattered 16-B stores to a hash position, no LDS atomics
//   S3: scattered 4-B stores (rep-like)
// Build: hipcc --offload-arch=gfx950 -O3 scripts/exp/exp_dedup.hip -o build/exp_dedup
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int T = 1024;
constexpr int B = 256;

__global__ void k_init(uint64_t* key, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull + 12345;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    key[i] = z ^ (z >> 31);
  }
}

template <int kMode>
__global__ __launch_bounds__(T) void k_scat(const uint64_t* __restrict__ key, uint64_t n,
                                            uint32_t bits, uint4* __restrict__ rec,
                                            uint32_t* __restrict__ rep) {
  extern __shared__ uint32_t cur[];
  const uint32_t nb = 1u << bits;
  const uint64_t per = (n + B - 1) / B;
  for (uint32_t b = threadIdx.x; b < nb; b += T) cur[b] = b * static_cast<uint32_t>(n / nb);
  __syncthreads();
  const uint64_t t0 = per * blockIdx.x, t1 = min(n, t0 + per);
  for (uint64_t i = t0 + threadIdx.x; i < t1; i += T) {
    const uint64_t k = key[i];
    const uint32_t d = static_cast<uint32_t>(k >> (64 - bits));
    if (kMode == 0) {
      const uint32_t p = atomicAdd(&cur[d], 1u) % static_cast<uint32_t>(n);
      rec[p] = make_uint4(static_cast<uint32_t>(k), static_cast<uint32_t>(k >> 32),
                          static_cast<uint32_t>(i), static_cast<uint32_t>(i));
    } else if (kMode == 1) {
      const uint32_t p = atomicAdd(&cur[d], 1u);
      rec[i] = make_uint4(static_cast<uint32_t>(k), static_cast<uint32_t>(k >> 32), p,
                          static_cast<uint32_t>(i));
    } else if (kMode == 2) {
      const uint32_t p =
          static_cast<uint32_t>((k * 0x9E3779B97F4A7C15ull) >> 40) % static_cast<uint32_t>(n);
      rec[p] = make_uint4(static_cast<uint32_t>(k), static_cast<uint32_t>(k >> 32),
                          static_cast<uint32_t>(i), static_cast<uint32_t>(i));
    } else {
      const uint32_t p =
          static_cast<uint32_t>((k * 0x9E3779B97F4A7C15ull) >> 40) % static_cast<uint32_t>(n);
      rep[p] = static_cast<uint32_t>(i);
    }
  }
}

template <int kMode>
void run(const char* name, const uint64_t* key, uint64_t n, uint4* rec, uint32_t* rep) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const uint32_t bits = 13;
  k_scat<kMode><<<B, T, 4u << bits>>>(key, n, bits, rec, rep);
  (void)hipEventRecord(a);
  for (int r = 0; r < 10; ++r) k_scat<kMode><<<B, T, 4u << bits>>>(key, n, bits, rec, rep);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  printf("%-58s %8.1f us\n", name, ms * 100);
}

int main() {
  const uint64_t n = 12500000;
  uint64_t* key;
  uint4* rec;
  uint32_t* rep;
  (void)hipMalloc(&key, n * 8);
  (void)hipMalloc(&rec, n * 16);
  (void)hipMalloc(&rep, n * 4);
  k_init<<<4096, 256>>>(key, n);
  run<0>("S0 LDS cursor atomics + scattered 16B stores (product)", key, n, rec, rep);
  run<1>("S1 LDS cursor atomics, sequential 16B stores", key, n, rec, rep);
  run<2>("S2 scattered 16B stores, no LDS atomics", key, n, rec, rep);
  run<3>("S3 scattered 4B stores", key, n, rec, rep);
  return 0;
}
