// Experiment (not shipped): can BLAKE3's G issue faster on gfx950 with a
// different VOP2 / VOP3 mix?  Register-only compressions (no memory), 16 waves
// per CU, same harness as sdgpu_valu_probe_kind(5).  Variants of G:
//   V0  product: 2 x v_add3_u32 + 2 x v_add_u32 + 4 x v_xor_b32 + 4 x v_alignbit_b32
//       (12 VALU, 6 VOP3 : 6 VOP2)
//   V1  a = a + b + m as two v_add_u32 (14 VALU, 4 VOP3 : 10 VOP2)
//   V2  one of the two add3 split (13 VALU, 5 VOP3 : 8 VOP2)
//   V3  rotr 16 / rotr 8 as v_perm_b32 byte permutes instead of v_alignbit_b32
// Each line: compressions/s and VALU lane-ops/s (instructions x 64 lanes).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_g_mix.hip -o build/exp_g_mix
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

__device__ __forceinline__ uint32_t ror(uint32_t x, uint32_t n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}
__device__ __forceinline__ uint32_t add2(uint32_t a, uint32_t b) {
  uint32_t r;
  asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t perm(uint32_t x, uint32_t sel) {
  return __builtin_amdgcn_perm(x, x, sel);
}

template <int V>
__device__ __forceinline__ void G(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t x,
                                  uint32_t y) {
  if (V == 1 || V == 2) a = add2(add2(a, b), x);
  else a = a + b + x;
  if (V == 3) d = perm(d ^ a, 0x01000302u);  // rotr 16
  else d = ror(d ^ a, 16);
  c = c + d;
  b = ror(b ^ c, 12);
  if (V == 1) a = add2(add2(a, b), y);
  else a = a + b + y;
  if (V == 3) d = perm(d ^ a, 0x00030201u);  // rotr 8
  else d = ror(d ^ a, 8);
  c = c + d;
  b = ror(b ^ c, 7);
}

template <int V>
__device__ __forceinline__ void compress(uint32_t cv[8], const uint32_t m[16], uint32_t ctr) {
  uint32_t v[16] = {cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7],
                    0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au, ctr, 0u, 64u, 0u};
  const uint8_t S[7][16] = {{0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
                            {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8},
                            {3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1},
                            {10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6},
                            {12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4},
                            {9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7},
                            {11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13}};
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    G<V>(v[0], v[4], v[8], v[12], m[S[r][0]], m[S[r][1]]);
    G<V>(v[1], v[5], v[9], v[13], m[S[r][2]], m[S[r][3]]);
    G<V>(v[2], v[6], v[10], v[14], m[S[r][4]], m[S[r][5]]);
    G<V>(v[3], v[7], v[11], v[15], m[S[r][6]], m[S[r][7]]);
    G<V>(v[0], v[5], v[10], v[15], m[S[r][8]], m[S[r][9]]);
    G<V>(v[1], v[6], v[11], v[12], m[S[r][10]], m[S[r][11]]);
    G<V>(v[2], v[7], v[8], v[13], m[S[r][12]], m[S[r][13]]);
    G<V>(v[3], v[4], v[9], v[14], m[S[r][14]], m[S[r][15]]);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) cv[i] = v[i] ^ v[i + 8];
}

template <int V>
__global__ __launch_bounds__(256) void k_probe(uint32_t* sink, uint32_t iters) {
  uint32_t cv[8], m[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) cv[i] = 0x6A09E667u + i;
#pragma unroll
  for (int i = 0; i < 16; ++i) m[i] = threadIdx.x * 0x9E3779B9u + blockIdx.x * 7u + i;
  for (uint32_t it = 0; it < iters; ++it) {
    compress<V>(cv, m, it);
    m[it & 15] ^= cv[it & 7];
  }
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) x ^= cv[i];
  if (x == 0x12345u) sink[blockIdx.x] = x;
}

template <int V>
void run(const char* name, int instrs, uint32_t* sink) {
  const uint32_t iters = 2000, blocks = 256 * 16;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  k_probe<V><<<blocks, 256>>>(sink, 64);
  std::vector<float> t;
  for (int r = 0; r < 5; ++r) {
    (void)hipEventRecord(a, 0);
    k_probe<V><<<blocks, 256>>>(sink, iters);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  const double comp = double(iters) * blocks * 256 / (t[2] * 1e-3);
  printf("%-44s %6.2f G compressions/s  %5.1f T lane-ops/s (%d VALU)\n", name, comp / 1e9,
         comp * instrs / 1e12, instrs);
}

int main() {
  uint32_t* sink;
  (void)hipMalloc(&sink, 1 << 20);
  for (int rep = 0; rep < 2; ++rep) {
    run<0>("V0 product (add3; 6 VOP3 : 6 VOP2 per G)", 680, sink);
    run<1>("V1 both add3 -> 2 x v_add (4 : 10)", 792, sink);
    run<2>("V2 first add3 -> 2 x v_add (5 : 8)", 736, sink);
    run<3>("V3 rotr16/rotr8 as v_perm_b32", 680, sink);
  }
  return 0;
}
