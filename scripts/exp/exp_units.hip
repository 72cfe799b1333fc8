// Experiment: the K1 unit loop (4 full chunks per lane, 64 compressions +
// 3 parents) reading (a) a 40 GiB HBM buffer (lanes 4 KiB apart, as in K1),
// (b) the same addresses folded into a 256 KiB L2-resident window, and
// (c) no loads at all.  Reports compressions/s and the in-kernel clock.
// Build: hipcc --offload-arch=gfx950 -O3 -I spacedrive_amd/csrc scripts/exp/exp_units.hip -o build/exp_units
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "b3_device.hpp"

using namespace sdgpu;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ntl(const uint4* q) {
  u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(q));
  return make_uint4(v.x, v.y, v.z, v.w);
}

template <int kMode>  // 0 HBM, 1 L2 window, 2 registers only
__global__ __launch_bounds__(256) void k_units(const uint8_t* __restrict__ buf, uint64_t units,
                                               uint64_t mask, uint32_t* __restrict__ out,
                                               unsigned long long* clk) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256;
  uint32_t acc = 0;
  for (uint64_t u = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; u < units; u += stride) {
    const uint8_t* p = buf + ((u * 4096) & mask);
    uint32_t node[3][8];
    for (int c = 0; c < 4; ++c) {
      uint32_t cv[8], m[16];
      b3_iv(cv);
      if (kMode >= 3) {  // 3: 128-B loads, 4: nt 64-B loads, 5: nt 128-B loads
        for (uint32_t b = 0; b < 16; b += 2) {
          uint32_t m2[16];
          const uint4* q = reinterpret_cast<const uint4*>(p + c * 1024 + 64 * b);
          uint4 x[8];
          if (kMode == 4) {
#pragma unroll
            for (int k = 0; k < 4; ++k) x[k] = ntl(q + k);
#pragma unroll
            for (int k = 4; k < 8; ++k) x[k] = ntl(q + k);
          } else if (kMode == 5) {
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = ntl(q + k);
          } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = q[k];
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            m[4 * k] = x[k].x; m[4 * k + 1] = x[k].y; m[4 * k + 2] = x[k].z; m[4 * k + 3] = x[k].w;
            m2[4 * k] = x[k + 4].x; m2[4 * k + 1] = x[k + 4].y; m2[4 * k + 2] = x[k + 4].z;
            m2[4 * k + 3] = x[k + 4].w;
          }
          b3_compress(cv, m, static_cast<uint32_t>(4 * u + c), 0u, 64u,
                      b == 0 ? B3_CHUNK_START : 0u);
          b3_compress(cv, m2, static_cast<uint32_t>(4 * u + c), 0u, 64u,
                      b + 1 == 15 ? B3_CHUNK_END : 0u);
        }
      } else
      for (uint32_t b = 0; b < 16; ++b) {
        if (kMode == 2) {
#pragma unroll
          for (int w = 0; w < 16; ++w) m[w] = static_cast<uint32_t>(u) * 31u + b * 7u + w;
        } else {
          b3_load_block(p + c * 1024 + 64 * b, m);
        }
        b3_compress(cv, m, static_cast<uint32_t>(4 * u + c), 0u, 64u,
                    (b == 0 ? B3_CHUNK_START : 0u) | (b == 15 ? B3_CHUNK_END : 0u));
      }
      if (c == 0) { for (int w = 0; w < 8; ++w) node[0][w] = cv[w]; }
      if (c == 1) b3_parent(node[0], node[0], cv, 0u);
      if (c == 2) { for (int w = 0; w < 8; ++w) node[1][w] = cv[w]; }
      if (c == 3) {
        b3_parent(node[1], node[1], cv, 0u);
        b3_parent(node[2], node[0], node[1], 0u);
      }
    }
    acc ^= node[2][0] ^ node[2][5];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x < 1024) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
  if (acc == 0x9999u) out[blockIdx.x] = acc;
}

template <int M>
void run(const uint8_t* buf, uint64_t units, uint64_t mask, uint32_t* out, unsigned long long* dclk,
         unsigned long long* hclk) {
  const int blocks = 8192;
  k_units<M><<<blocks, 256>>>(buf, units / 16, mask, out, dclk);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  k_units<M><<<blocks, 256>>>(buf, units, mask, out, dclk);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  hipMemcpy(hclk, dclk, 2 * 1024 * 8, hipMemcpyDeviceToHost);
  double ghz = 0;
  for (int b = 0; b < 1024; ++b) ghz += double(hclk[2 * b]) / (double(hclk[2 * b + 1]) * 10.0);
  ghz /= 1024;
  const double comps = double(units) * 67;
  const char* names[] = {"HBM", "L2 window", "no loads", "HBM 128B/lane", "HBM nt", "HBM nt 128B"};
  printf("mode %d (%s): %.3f ms  %.2f G compressions/s  %.2f TB/s read  clock %.2f GHz\n", M,
         names[M], ms, comps / ms / 1e6,
         double(units) * 4096 / ms / 1e9, ghz);
}

int main() {
  const uint64_t bytes = 40ull << 30;
  uint8_t* buf;
  if (hipMalloc(&buf, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
  hipMemset(buf, 0x5a, bytes);
  uint32_t* out;
  unsigned long long *dclk, *hclk = (unsigned long long*)malloc(2 * 1024 * 8);
  hipMalloc(&out, 1 << 20);
  hipMalloc(&dclk, 2 * 1024 * 8);
  const uint64_t units = bytes / 4096;
  run<0>(buf, units, bytes - 1, out, dclk, hclk);
  run<1>(buf, units, (256u << 10) - 1, out, dclk, hclk);
  run<2>(buf, units, bytes - 1, out, dclk, hclk);
  for (int r = 0; r < 2; ++r) {
    run<0>(buf, units, bytes - 1, out, dclk, hclk);
    run<3>(buf, units, bytes - 1, out, dclk, hclk);
    run<4>(buf, units, bytes - 1, out, dclk, hclk);
    run<5>(buf, units, bytes - 1, out, dclk, hclk);
  }
  return 0;
}
