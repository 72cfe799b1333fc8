// Experiment (not shipped): where a single-file call's ~55 us goes.  Median of
// 2000 iterations each: an empty kernel + stream sync; a 4 KiB pinned H2D copy
// + sync; a 32-B D2H copy + sync; H2D + kernel + D2H + sync (the current
// latency path's shape); a kernel reading the 4 KiB pinned buffer directly
// (zero-copy, one 16-B load per lane) and writing 32 B to pinned memory + sync;
// the same with the host spinning on a flag the kernel writes instead of the
// stream sync.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_latency.hip -o build/exp_latency
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <chrono>
#include <vector>

__global__ void k_empty(uint32_t* out) {
  if (threadIdx.x == 1023 && blockIdx.x == 1234567) out[0] = 1;
}

__global__ void k_read(const uint4* __restrict__ in, uint32_t nvec, uint32_t* __restrict__ out) {
  __shared__ uint32_t acc;
  if (threadIdx.x == 0) acc = 0;
  __syncthreads();
  uint32_t x = 0;
  for (uint32_t i = threadIdx.x; i < nvec; i += blockDim.x) {
    const uint4 v = in[i];
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  atomicXor(&acc, x);
  __syncthreads();
  if (threadIdx.x < 8) out[threadIdx.x] = acc + threadIdx.x;
}

__global__ void k_read_flag(const uint4* __restrict__ in, uint32_t nvec, uint32_t* __restrict__ out,
                            volatile uint32_t* flag, uint32_t seq) {
  __shared__ uint32_t acc;
  if (threadIdx.x == 0) acc = 0;
  __syncthreads();
  uint32_t x = 0;
  for (uint32_t i = threadIdx.x; i < nvec; i += blockDim.x) {
    const uint4 v = in[i];
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  atomicXor(&acc, x);
  __syncthreads();
  if (threadIdx.x < 8) out[threadIdx.x] = acc + threadIdx.x;
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) *flag = seq;
}

template <typename F>
double med_us(F f, int n = 2000) {
  std::vector<double> v;
  for (int i = 0; i < 50; ++i) f();
  for (int i = 0; i < n; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    f();
    v.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  uint8_t *h, *d;
  uint32_t *hout, *dout, *hflag;
  (void)hipHostMalloc(&h, 1 << 20, hipHostMallocDefault);
  (void)hipHostMalloc(&hout, 4096, hipHostMallocDefault);
  (void)hipHostMalloc(&hflag, 4096, hipHostMallocDefault);
  (void)hipMalloc(&d, 1 << 20);
  (void)hipMalloc(&dout, 4096);
  for (int i = 0; i < (1 << 20); ++i) h[i] = uint8_t(i * 7);
  uint8_t *hd;
  uint32_t *houtd, *hflagd;
  (void)hipHostGetDevicePointer(reinterpret_cast<void**>(&hd), h, 0);
  (void)hipHostGetDevicePointer(reinterpret_cast<void**>(&houtd), hout, 0);
  (void)hipHostGetDevicePointer(reinterpret_cast<void**>(&hflagd), hflag, 0);
  printf("empty kernel + sync          %7.1f us\n", med_us([&] {
           k_empty<<<1, 1024, 0, s>>>(dout);
           (void)hipStreamSynchronize(s);
         }));
  for (uint32_t bytes : {4096u, 65536u, 1u << 20}) {
    printf("-- %u B\n", bytes);
    printf("H2D + sync                   %7.1f us\n", med_us([&] {
             (void)hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s);
             (void)hipStreamSynchronize(s);
           }));
    printf("D2H 32 B + sync              %7.1f us\n", med_us([&] {
             (void)hipMemcpyAsync(hout, dout, 32, hipMemcpyDeviceToHost, s);
             (void)hipStreamSynchronize(s);
           }));
    printf("H2D + kernel + D2H + sync    %7.1f us\n", med_us([&] {
             (void)hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s);
             k_read<<<1, 1024, 0, s>>>(reinterpret_cast<const uint4*>(d), bytes / 16, dout);
             (void)hipMemcpyAsync(hout, dout, 32, hipMemcpyDeviceToHost, s);
             (void)hipStreamSynchronize(s);
           }));
    printf("zero-copy kernel + sync      %7.1f us\n", med_us([&] {
             k_read<<<1, 1024, 0, s>>>(reinterpret_cast<const uint4*>(hd), bytes / 16, houtd);
             (void)hipStreamSynchronize(s);
           }));
    uint32_t seq = 0;
    printf("zero-copy kernel + flag spin %7.1f us\n", med_us([&] {
             ++seq;
             k_read_flag<<<1, 1024, 0, s>>>(reinterpret_cast<const uint4*>(hd), bytes / 16, houtd,
                                            hflagd, seq);
             while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != seq) {
             }
           }));
    (void)hipStreamSynchronize(s);
  }
  return 0;
}
