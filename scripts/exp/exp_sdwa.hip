// Experiment: rotr(d ^ a, 16) via two VOP2 SDWA xors vs v_xor + v_alignbit.
// Checks correctness (with/without s_nop padding) and times each form.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/exp/exp_sdwa.hip -o build/exp_sdwa
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int kMode>
__device__ __forceinline__ uint32_t xr16(uint32_t d, uint32_t a) {
  uint32_t t;
  if constexpr (kMode == 0) {
    t = __builtin_amdgcn_alignbit(d ^ a, d ^ a, 16);
  } else if constexpr (kMode == 1) {
    asm volatile(
        "v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n\t"
        "v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1"
        : "=&v"(t) : "v"(d), "v"(a));
  } else if constexpr (kMode == 2) {
    asm volatile(
        "s_nop 4\n\t"
        "v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n\t"
        "s_nop 4\n\t"
        "v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1"
        : "=&v"(t) : "v"(d), "v"(a));
  } else {
    // two independent halves into two registers, combined by v_or (no preserve)
    uint32_t hi, lo;
    asm volatile(
        "v_xor_b32_sdwa %0, %2, %3 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n\t"
        "v_xor_b32_sdwa %1, %2, %3 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1"
        : "=&v"(hi), "=&v"(lo) : "v"(d), "v"(a));
    t = hi | lo;
  }
  return t;
}

template <int kMode>
__global__ void k_check(const uint32_t* in, uint32_t* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t d = in[2 * i], a = in[2 * i + 1];
  // make d and a results of fresh VALU ops right before use (hazard exposure)
  d = d * 3u + 1u;
  a = a ^ (d >> 3);
  out[i] = xr16<kMode>(d, a);
}

template <int kMode>
__global__ void k_time(uint32_t* sink, uint32_t iters) {
  uint32_t d[8], a[8];
  for (int k = 0; k < 8; ++k) {
    d[k] = threadIdx.x * 0x9E3779B9u + k;
    a[k] = blockIdx.x * 0x85EBCA6Bu + 7 * k;
  }
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      d[k] = xr16<kMode>(d[k], a[k]);
      a[k] = a[k] + d[k];
    }
  }
  uint32_t x = 0;
  for (int k = 0; k < 8; ++k) x ^= d[k] ^ a[k];
  if (x == 0x1234567u) sink[blockIdx.x] = x;
}

template <int kMode>
void run(const uint32_t* din, uint32_t* dout, uint32_t* hout, const uint32_t* hin, int n,
         uint32_t* sink) {
  k_check<kMode><<<(n + 255) / 256, 256>>>(din, dout, n);
  hipMemcpy(hout, dout, n * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n; ++i) {
    uint32_t d = hin[2 * i] * 3u + 1u, a = hin[2 * i + 1] ^ (d >> 3);
    uint32_t x = d ^ a, ref = (x >> 16) | (x << 16);
    bad += hout[i] != ref;
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 256 * 32;
  k_time<kMode><<<blocks, 256>>>(sink, 16);
  hipEventRecord(e0);
  k_time<kMode><<<blocks, 256>>>(sink, 2048);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double per = double(blocks) * 256 * 2048 * 8;  // xr16+add pairs
  printf("mode %d: mismatches %d / %d   time %.3f ms   %.2f G (xr16+add)/s\n", kMode, bad, n, ms,
         per / ms / 1e6);
}

int main() {
  const int n = 1 << 20;
  uint32_t *hin = (uint32_t*)malloc(8 * n), *hout = (uint32_t*)malloc(4 * n);
  uint64_t s = 88172645463325252ull;
  for (int i = 0; i < 2 * n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    hin[i] = (uint32_t)s;
  }
  uint32_t *din, *dout, *sink;
  hipMalloc(&din, 8 * n);
  hipMalloc(&dout, 4 * n);
  hipMalloc(&sink, 1 << 20);
  hipMemcpy(din, hin, 8 * n, hipMemcpyHostToDevice);
  run<0>(din, dout, hout, hin, n, sink);
  run<1>(din, dout, hout, hin, n, sink);
  run<2>(din, dout, hout, hin, n, sink);
  run<3>(din, dout, hout, hin, n, sink);
  run<0>(din, dout, hout, hin, n, sink);
  return 0;
}
