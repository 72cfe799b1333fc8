// Experiment: BLAKE3 compressions per second with everything in registers (no
// memory), i.e. the compute roof of the exact instruction stream K1/K2 issue,
// plus the shader clock under that load (s_memtime vs s_memrealtime @100 MHz).
// Build: hipcc --offload-arch=gfx950 -O3 -I spacedrive_amd/csrc scripts/exp/exp_compress.hip -o build/exp_compress
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "b3_device.hpp"

using namespace sdgpu;

template <int kWavesPerSimd>
__global__ __launch_bounds__(256, kWavesPerSimd) void k_comp(uint32_t* sink, uint32_t iters,
                                                            unsigned long long* clk) {
  uint32_t cv[8], m[16];
  b3_iv(cv);
#pragma unroll
  for (int i = 0; i < 16; ++i) m[i] = threadIdx.x * 0x9E3779B9u + blockIdx.x * 7u + i;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    b3_compress(cv, m, it, 0u, 64u, 0u);
    m[it & 15] ^= cv[it & 7];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x < 1024) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) x ^= cv[i];
  if (x == 0x12345u) sink[blockIdx.x] = x;
}

template <int W>
void run(uint32_t* sink, unsigned long long* dclk, unsigned long long* hclk, int blocks) {
  const uint32_t iters = 2000;
  k_comp<W><<<blocks, 256>>>(sink, 10, dclk);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  k_comp<W><<<blocks, 256>>>(sink, iters, dclk);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  hipMemcpy(hclk, dclk, 2 * 1024 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  double ghz = 0;
  int nb = blocks < 1024 ? blocks : 1024;
  for (int b = 0; b < nb; ++b) ghz += double(hclk[2 * b]) / (double(hclk[2 * b + 1]) * 10.0);
  ghz /= nb;
  const double comps = double(blocks) * 256 * iters;
  printf("launch_bounds waves/SIMD>=%d blocks %d: %.3f ms  %.2f G compressions/s  "
         "(x680 = %.1f T instr-lanes/s)  clock %.2f GHz  cycles/wave-compression %.0f\n",
         W, blocks, ms, comps / ms / 1e6, comps * 680 / ms / 1e9, ghz,
         ghz * 1e9 / (comps / ms * 1e3 / 64 / 1024));
}

int main() {
  uint32_t* sink;
  unsigned long long *dclk, *hclk = (unsigned long long*)malloc(2 * 1024 * 8);
  hipMalloc(&sink, 1 << 22);
  hipMalloc(&dclk, 2 * 1024 * 8);
  run<1>(sink, dclk, hclk, 256 * 4 * 1);
  run<2>(sink, dclk, hclk, 256 * 4 * 2);
  run<4>(sink, dclk, hclk, 256 * 4 * 4);
  run<8>(sink, dclk, hclk, 256 * 4 * 8);
  run<8>(sink, dclk, hclk, 256 * 4 * 32);
  return 0;
}
