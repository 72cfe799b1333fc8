// Experiment (round 6, f3 single-file latency): the quad-lane compression as
// the latency kernels run it -- its 28 message words read from LDS at the
// start of every compression -- against the same with the NEXT block's words
// read before the current block's rounds (software pipelining), and with the
// DPP row rotations folded into the instructions that consume them (the
// diagonal step's first uses as VOP2 ops with a quad_perm on src0).
// One wave, chains of n compressions over 16 LDS blocks (a chunk's blocks);
// shader cycles (clock64) and the 100 MHz wall clock around the chain.
//   lds      product form (b3_batch.hip QuadLane::compress)
//   piped    next block's words loaded before this block's rounds
//   piped+f  piped, rotations folded into VOP2 consumers where they allow it
// Each variant's final CVs are checked against the lane form (b3_compress).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_chain2.hip -o exp_bin/exp_chain2
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../../spacedrive_amd/csrc/b3_device.hpp"

using namespace sdgpu;

namespace {

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
// bound_ctrl set (every quad_perm source lane exists, so the value is the
// same): the form the backend's DPP combiner may fold into a VOP2 user
template <int kCtrl>
__device__ __forceinline__ uint32_t qpermf(uint32_t x) {
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), kCtrl, 0xF, 0xF, true));
}
constexpr int kRot1 = 0x39, kRot2 = 0x4E, kRot3 = 0x93;

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

// g1 with its b, c, d inputs read through a quad rotation (kB, kC, kD), the
// first uses written as VOP2 ops (src0 = the rotated value) so the backend's
// DPP combiner can fold each v_mov_dpp into its user
template <int kB, int kC, int kD>
__device__ __forceinline__ void g1_rot(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d,
                                       uint32_t x, uint32_t y) {
  const uint32_t br = qpermf<kB>(b), cr = qpermf<kC>(c), dr = qpermf<kD>(d);
  a = br + a;
  a = a + x;
  d = rotr32(dr ^ a, 16);
  c = cr + d;
  b = rotr32(br ^ c, 12);
  a = a + b + y;
  d = rotr32(d ^ a, 8);
  c = c + d;
  b = rotr32(b ^ c, 7);
}

struct Q {
  uint32_t i, iv_a, iv_b, woff[28];
  __device__ void init() {
    i = threadIdx.x & 3u;
    const uint32_t iv[8] = {IV0, IV1, IV2, IV3, IV4, IV5, IV6, IV7};
    iv_a = iv[i];
    iv_b = iv[4 + i];
#pragma unroll
    for (int r = 0; r < 7; ++r) {
      woff[4 * r] = 4u * kSched[r][2 * i];
      woff[4 * r + 1] = 4u * kSched[r][2 * i + 1];
      woff[4 * r + 2] = 4u * kSched[r][8 + 2 * i];
      woff[4 * r + 3] = 4u * kSched[r][9 + 2 * i];
    }
  }
  __device__ __forceinline__ void load(const uint8_t* blk, uint32_t (&w)[28]) const {
#pragma unroll
    for (int k = 0; k < 28; ++k) w[k] = *reinterpret_cast<const uint32_t*>(blk + woff[k]);
  }
  template <bool kFold>
  __device__ __forceinline__ void rounds(uint32_t& h0, uint32_t& h1, const uint32_t (&w)[28],
                                         uint32_t d) const {
    uint32_t a = h0, b = h1, c = iv_a;
    if (!kFold) {
#pragma unroll
      for (int r = 0; r < 7; ++r) {
        g1(a, b, c, d, w[4 * r], w[4 * r + 1]);
        b = qperm<kRot1>(b);
        c = qperm<kRot2>(c);
        d = qperm<kRot3>(d);
        g1(a, b, c, d, w[4 * r + 2], w[4 * r + 3]);
        b = qperm<kRot3>(b);
        c = qperm<kRot2>(c);
        d = qperm<kRot1>(d);
      }
    } else {
      // rows kept where the step left them; each step reads them rotated
      g1(a, b, c, d, w[0], w[1]);
      g1_rot<kRot1, kRot2, kRot3>(a, b, c, d, w[2], w[3]);
#pragma unroll
      for (int r = 1; r < 7; ++r) {
        g1_rot<kRot3, kRot2, kRot1>(a, b, c, d, w[4 * r], w[4 * r + 1]);
        g1_rot<kRot1, kRot2, kRot3>(a, b, c, d, w[4 * r + 2], w[4 * r + 3]);
      }
      b = qperm<kRot3>(b);
      c = qperm<kRot2>(c);
      d = qperm<kRot1>(d);
    }
    h0 = a ^ c;
    h1 = b ^ d;
  }
};

__device__ __forceinline__ uint32_t dword(uint32_t i, uint32_t k) {
  return i == 0 ? k : i == 1 ? 0u : i == 2 ? 64u : (k % 16 == 0 ? 1u : 0u);
}

// mode 0: lds (load at each compression), 1: piped, 2: piped + folded,
// 3: piped with two buffers in turn, 4: registers only (words loaded once,
// the r3 exp_chain form: the floor)
template <int kMode>
__global__ __launch_bounds__(64) void k_chain(uint32_t n, uint64_t* out, uint32_t* cvs) {
  __shared__ __attribute__((aligned(16))) uint8_t msg[16 * 64];
  for (uint32_t k = threadIdx.x; k < 256; k += 64)
    reinterpret_cast<uint32_t*>(msg)[k] = k * 0x9E3779B9u + 7;
  Q L;
  L.init();
  __syncthreads();
  uint32_t h0 = L.iv_a, h1 = L.iv_b;
  const uint64_t c0 = clock64(), w0 = wall_clock64();
  if (threadIdx.x < 4) {
    uint32_t w[28];
    L.load(msg, w);
    for (uint32_t k = 0; k < n; ++k) {
      if (kMode == 4) {
        L.rounds<false>(h0, h1, w, dword(L.i, k));
      } else if (kMode == 0) {
        L.load(msg + 64 * (k % 16), w);
        L.rounds<false>(h0, h1, w, dword(L.i, k));
      } else if (kMode == 3) {
        // two word buffers in turn (no register copies): the chain unrolled by 2
        uint32_t wn[28];
        L.load(msg + 64 * ((k + 1) % 16), wn);
        L.rounds<false>(h0, h1, w, dword(L.i, k));
        if (++k == n) break;
        L.load(msg + 64 * ((k + 1) % 16), w);
        L.rounds<false>(h0, h1, wn, dword(L.i, k));
      } else {
        uint32_t wn[28];
        L.load(msg + 64 * ((k + 1) % 16), wn);  // the next block's words, in flight
        L.rounds<kMode == 2>(h0, h1, w, dword(L.i, k));
#pragma unroll
        for (int x = 0; x < 28; ++x) w[x] = wn[x];
      }
    }
  }
  __syncthreads();
  const uint64_t c1 = clock64(), w1 = wall_clock64();
  if (threadIdx.x == 0) {
    out[0] = c1 - c0;
    out[1] = w1 - w0;
  }
  if (threadIdx.x < 4) {
    cvs[threadIdx.x] = h0;
    cvs[4 + threadIdx.x] = h1;
  }
}

// reference: the lane form over the same blocks and words
__global__ void k_ref(uint32_t n, uint32_t* cvs) {
  __shared__ uint32_t msg[256];
  for (uint32_t k = threadIdx.x; k < 256; k += 64) msg[k] = k * 0x9E3779B9u + 7;
  __syncthreads();
  if (threadIdx.x != 0) return;
  uint32_t cv[8], m[16];
  b3_iv(cv);
  for (uint32_t k = 0; k < n; ++k) {
    for (int x = 0; x < 16; ++x) m[x] = msg[16 * (k % 16) + x];
    b3_compress(cv, m, k, 0u, 64u, k % 16 == 0 ? 1u : 0u);
  }
  for (int x = 0; x < 8; ++x) cvs[x] = cv[x];
}

}  // namespace

int main() {
  uint64_t* out;
  uint32_t *cvs, *ref;
  (void)hipMalloc(&out, 16);
  (void)hipMalloc(&cvs, 64);
  (void)hipMalloc(&ref, 64);
  int wall_khz = 0;
  (void)hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0);
  const double wall_hz = wall_khz > 0 ? wall_khz * 1e3 : 1e8;
  const char* names[5] = {"lds", "piped", "piped+f", "piped2", "regs"};
  int bad = 0;
  for (uint32_t n : {19u, 2000u}) {
    k_ref<<<1, 64>>>(n, ref);
    uint32_t r[8];
    (void)hipMemcpy(r, ref, 32, hipMemcpyDeviceToHost);
    for (int rep = 0; rep < 3; ++rep)
      for (int mode = 0; mode < 5; ++mode) {
        if (mode == 0) k_chain<0><<<1, 64>>>(n, out, cvs);
        if (mode == 1) k_chain<1><<<1, 64>>>(n, out, cvs);
        if (mode == 2) k_chain<2><<<1, 64>>>(n, out, cvs);
        if (mode == 3) k_chain<3><<<1, 64>>>(n, out, cvs);
        if (mode == 4) k_chain<4><<<1, 64>>>(n, out, cvs);
        (void)hipDeviceSynchronize();
        uint64_t h[2];
        uint32_t g[8];
        (void)hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
        (void)hipMemcpy(g, cvs, 32, hipMemcpyDeviceToHost);
        bool eq = mode == 4;  // regs: one block's words throughout, not the reference chain
        if (mode != 4)
          for (int x = 0; x < 8; ++x) eq = (x == 0 || eq) && g[x] == r[x];
        bad += !eq;
        const double us = h[1] / wall_hz * 1e6;
        printf("n %5u %-8s %8.1f cycles/compression %7.3f us/compression clock %.2f GHz  %s\n", n,
               names[mode], double(h[0]) / n, us / n, h[0] / (us * 1e3), eq ? "equal" : "MISMATCH");
      }
  }
  printf("(%s) %s\n", hipGetErrorString(hipGetLastError()), bad ? "MISMATCHES" : "all equal");
  return bad ? 2 : 0;
}
