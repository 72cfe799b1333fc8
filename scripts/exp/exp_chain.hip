// Experiment (single-file latency): what one wave's chain of
// dependent BLAKE3 compressions costs, in shader cycles and in wall time.
// The latency service hashes a 4 KiB cas message in ~34 us = 19 dependent
// compressions (16 blocks of one chunk + 3 tree levels): ~1.8 us each, where
// 680 VALU instructions at 4 cycles (VOP3) / 2 cycles (VOP2) per wave64
// instruction would take ~2030 cycles = 0.85 us at 2.4 GHz.  This measures,
// for one wave running N chained compressions (4 lanes = 4 chunks, as a 4 KiB
// message; or 1 lane), the shader-clock cycles (s_memtime, clock64) and the
// constant 100 MHz wall clock (s_memrealtime) around the chain: their ratio is
// the clock the device runs the chain at.
//   idle      the chain alone on the device
//   loaded    the same while every other CU runs a VALU spin kernel
// and the same chain with each compression spread over a quad of lanes.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_chain.hip -o build/exp_chain
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../../spacedrive_amd/csrc/b3_device.hpp"

using namespace sdgpu;

namespace {

__global__ __launch_bounds__(64) void k_chain(uint32_t n, uint32_t lanes, uint64_t* out,
                                              uint32_t* sink) {
  uint32_t cv[8], m[16];
  b3_iv(cv);
  for (int w = 0; w < 16; ++w) m[w] = threadIdx.x * 16 + w;
  __syncthreads();
  const uint64_t c0 = clock64(), w0 = wall_clock64();
  if (threadIdx.x < lanes)
    for (uint32_t i = 0; i < n; ++i) {
      b3_compress(cv, m, i, 0, 64, 0);  // the CV chains the blocks
    }
  __syncthreads();
  const uint64_t c1 = clock64(), w1 = wall_clock64();
  if (threadIdx.x == 0) {
    out[0] = c1 - c0;
    out[1] = w1 - w0;
  }
  uint32_t x = 0;
  for (int w = 0; w < 8; ++w) x ^= cv[w];
  if (x == 0x12345678u) sink[threadIdx.x] = x;
}


// The same chain with each compression spread over a QUAD of lanes: lane i of
// the quad holds state column i (v[i], v[4+i], v[8+i], v[12+i]) and computes
// G_i of the column step, then -- after DPP quad rotations of rows b, c, d --
// G_i of the diagonal step; its 4 message words per round come from LDS at
// per-lane offsets (the schedule), loaded before the chain.  Output: lane i
// holds cv[i] and cv[4+i], exactly the next block's a and b.
__device__ __constant__ uint8_t kSched[7][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8},
    {3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1},
    {10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6},
    {12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4},
    {9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7},
    {11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13}};

template <int kCtrl>
__device__ __forceinline__ uint32_t qperm(uint32_t x) {
  return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(x), kCtrl, 0xF, 0xF, false));
}
constexpr int kRot1 = 0x39, kRot2 = 0x4E, kRot3 = 0x93;  // lane i reads lane i+1 / i+2 / i+3

__device__ __forceinline__ void g1(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t x,
                                   uint32_t y) {
  a = a + b + x;
  d = rotr32(d ^ a, 16);
  c = c + d;
  b = rotr32(b ^ c, 12);
  a = a + b + y;
  d = rotr32(d ^ a, 8);
  c = c + d;
  b = rotr32(b ^ c, 7);
}

__global__ __launch_bounds__(64) void k_chain_quad(uint32_t n, uint32_t quads, uint64_t* out,
                                                   uint32_t* sink) {
  __shared__ uint32_t msg[16][16];  // a 64-B block per quad
  const uint32_t t = threadIdx.x, q = t >> 2, i = t & 3;
  for (uint32_t k = t; k < 256; k += 64) (&msg[0][0])[k] = k * 0x9E3779B9u;
  __syncthreads();
  uint32_t mw[28];
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    mw[4 * r] = msg[q][kSched[r][2 * i]];
    mw[4 * r + 1] = msg[q][kSched[r][2 * i + 1]];
    mw[4 * r + 2] = msg[q][kSched[r][8 + 2 * i]];
    mw[4 * r + 3] = msg[q][kSched[r][9 + 2 * i]];
  }
  const uint32_t iv[8] = {IV0, IV1, IV2, IV3, IV4, IV5, IV6, IV7};
  uint32_t h0 = iv[i], h1 = iv[4 + i];  // cv[i], cv[4+i]
  __syncthreads();
  const uint64_t c0 = clock64(), w0 = wall_clock64();
  if (q < quads)
    for (uint32_t k = 0; k < n; ++k) {
      uint32_t a = h0, b = h1, c = iv[i];
      uint32_t d = i == 0 ? k : i == 1 ? 0u : i == 2 ? 64u : 0u;  // counter lo/hi, len, flags
#pragma unroll
      for (int r = 0; r < 7; ++r) {
        g1(a, b, c, d, mw[4 * r], mw[4 * r + 1]);  // column step
        b = qperm<kRot1>(b);
        c = qperm<kRot2>(c);
        d = qperm<kRot3>(d);
        g1(a, b, c, d, mw[4 * r + 2], mw[4 * r + 3]);  // diagonal step
        b = qperm<kRot3>(b);
        c = qperm<kRot2>(c);
        d = qperm<kRot1>(d);
      }
      h0 = a ^ c;
      h1 = b ^ d;
    }
  __syncthreads();
  const uint64_t c1 = clock64(), w1 = wall_clock64();
  if (t == 0) {
    out[0] = c1 - c0;
    out[1] = w1 - w0;
  }
  if ((h0 ^ h1) == 0x12345678u) sink[t] = h0;
}

// Check: the quad form's CV of one block equals b3_compress's.
__global__ void k_quad_check(uint32_t* res) {
  __shared__ uint32_t msg[16][16];
  const uint32_t t = threadIdx.x, q = t >> 2, i = t & 3;
  for (uint32_t k = t; k < 256; k += 64) (&msg[0][0])[k] = k * 0x9E3779B9u;
  __syncthreads();
  const uint32_t iv[8] = {IV0, IV1, IV2, IV3, IV4, IV5, IV6, IV7};
  uint32_t a = iv[i], b = iv[4 + i], c = iv[i];
  uint32_t d = i == 0 ? 5u : i == 1 ? 0u : i == 2 ? 64u : 3u;
  for (int r = 0; r < 7; ++r) {
    g1(a, b, c, d, msg[q][kSched[r][2 * i]], msg[q][kSched[r][2 * i + 1]]);
    b = qperm<kRot1>(b);
    c = qperm<kRot2>(c);
    d = qperm<kRot3>(d);
    g1(a, b, c, d, msg[q][kSched[r][8 + 2 * i]], msg[q][kSched[r][9 + 2 * i]]);
    b = qperm<kRot3>(b);
    c = qperm<kRot2>(c);
    d = qperm<kRot1>(d);
  }
  uint32_t ok = 1;
  if (t < 4) {
    uint32_t cv[8], m[16];
    b3_iv(cv);
    for (int w = 0; w < 16; ++w) m[w] = msg[0][w];
    b3_compress(cv, m, 5u, 0u, 64u, 3u);
    ok = (cv[i] == (a ^ c)) && (cv[4 + i] == (b ^ d));
  }
  res[t] = ok;
}

__global__ __launch_bounds__(256) void k_spin(uint64_t ticks, uint32_t* sink) {
  const uint64_t w0 = wall_clock64();
  uint32_t a = threadIdx.x, b = blockIdx.x;
  while (wall_clock64() - w0 < ticks) {
#pragma unroll
    for (int k = 0; k < 64; ++k) {
      a = __builtin_amdgcn_alignbit(a ^ b, a, 7) + b;
      b = b + (a ^ 0x9E3779B9u);
    }
  }
  if (a == b) sink[threadIdx.x] = a;
}

}  // namespace

int main() {
  uint64_t* out;
  uint32_t* sink;
  (void)hipMalloc(&out, 16);
  (void)hipMalloc(&sink, 4096);
  hipStream_t s1, s2;
  (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  int wall_khz = 0;
  (void)hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0);
  const double wall_hz = wall_khz > 0 ? wall_khz * 1e3 : 1e8;
  const uint32_t n = 2000;
  {
    uint32_t* res;
    (void)hipMalloc(&res, 256);
    k_quad_check<<<1, 64>>>(res);
    uint32_t r[64];
    (void)hipMemcpy(r, res, 256, hipMemcpyDeviceToHost);
    uint32_t bad = 0;
    for (int k = 0; k < 4; ++k) bad += r[k] != 1;
    printf("quad-form compression vs b3_compress: %s\n", bad ? "MISMATCH" : "equal");
  }
  for (int loaded = 0; loaded < 2; ++loaded) {
    for (int form = 0; form < 2; ++form)
      for (uint32_t lanes : {1u, 4u, 16u}) {
        if (loaded) k_spin<<<255 * 4, 256, 0, s2>>>(static_cast<uint64_t>(wall_hz * 0.05), sink);
        if (form == 0) k_chain<<<1, 64, 0, s1>>>(n, lanes, out, sink);
        else k_chain_quad<<<1, 64, 0, s1>>>(n, lanes, out, sink);
        (void)hipStreamSynchronize(s1);
        (void)hipStreamSynchronize(s2);
        uint64_t h[2];
        (void)hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
        const double us = h[1] / wall_hz * 1e6;
        printf("%-6s %-5s %2u chains: %8.1f cycles/compression %7.3f us/compression  clock %.2f GHz\n",
               loaded ? "loaded" : "idle", form ? "quad" : "lane", lanes, double(h[0]) / n, us / n,
               h[0] / (us * 1e3));
      }
  }
  printf("(%s)\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
