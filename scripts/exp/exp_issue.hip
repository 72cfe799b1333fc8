// Experiment: VALU issue model of gfx950 for BLAKE3's instruction classes.
// Is a VOP2 (v_xor_b32 / v_add_u32) really 2 cycles per wave64 and VOP3
// (v_alignbit_b32 / v_add3_u32) 4 cycles, and when does the 2x survive in a
// mixed stream?  Each mode is a 16-instruction inline-asm block over 8
// independent registers, looped; throughput in T lane-instr/s at
// 8 and 1 waves/SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/exp/exp_issue.hip -o build/exp_issue
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define X(i) "v_xor_b32 %" #i ", %8, %" #i "\n\t"
#define A(i) "v_alignbit_b32 %" #i ", %" #i ", %" #i ", 16\n\t"
#define D(i) "v_add_u32 %" #i ", %8, %" #i "\n\t"
#define T(i) "v_add3_u32 %" #i ", %" #i ", %8, %9\n\t"
#define XA(i, j) "v_xor_b32 %" #i ", %" #j ", %" #i "\n\t"   // a_i ^= a_j (dependent on j)

template <int kMode>
__global__ __launch_bounds__(256) void k_issue(uint32_t* sink, uint32_t iters) {
  uint32_t a0, a1, a2, a3, a4, a5, a6, a7;
  const uint32_t b = blockIdx.x * 0x85EBCA6Bu, c = threadIdx.x * 0x9E3779B9u;
  a0 = c; a1 = c + 1; a2 = c + 2; a3 = c + 3; a4 = c + 4; a5 = c + 5; a6 = c + 6; a7 = c + 7;
  const uint64_t t0 = __builtin_readcyclecounter();
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#define OPS "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c)
    if constexpr (kMode == 0)  // 16 xor
      asm volatile(X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) : OPS);
    if constexpr (kMode == 1)  // 16 alignbit
      asm volatile(A(0) A(1) A(2) A(3) A(4) A(5) A(6) A(7) A(0) A(1) A(2) A(3) A(4) A(5) A(6) A(7) : OPS);
    if constexpr (kMode == 2)  // alternating xor / alignbit, independent
      asm volatile(X(0) A(1) X(2) A(3) X(4) A(5) X(6) A(7) X(1) A(0) X(3) A(2) X(5) A(4) X(7) A(6) : OPS);
    if constexpr (kMode == 3)  // pairs of xor then pairs of alignbit
      asm volatile(X(0) X(1) A(2) A(3) X(4) X(5) A(6) A(7) X(2) X(3) A(0) A(1) X(6) X(7) A(4) A(5) : OPS);
    if constexpr (kMode == 4)  // 4 xor then 4 alignbit
      asm volatile(X(0) X(1) X(2) X(3) A(4) A(5) A(6) A(7) X(4) X(5) X(6) X(7) A(0) A(1) A(2) A(3) : OPS);
    if constexpr (kMode == 5)  // xor then dependent alignbit on the same register
      asm volatile(X(0) A(0) X(1) A(1) X(2) A(2) X(3) A(3) X(4) A(4) X(5) A(5) X(6) A(6) X(7) A(7) : OPS);
    if constexpr (kMode == 6)  // 16 add_u32
      asm volatile(D(0) D(1) D(2) D(3) D(4) D(5) D(6) D(7) D(0) D(1) D(2) D(3) D(4) D(5) D(6) D(7) : OPS);
    if constexpr (kMode == 7)  // 16 add3
      asm volatile(T(0) T(1) T(2) T(3) T(4) T(5) T(6) T(7) T(0) T(1) T(2) T(3) T(4) T(5) T(6) T(7) : OPS);
    if constexpr (kMode == 8)  // 16 xor, each dependent on the previous (one chain)
      asm volatile(XA(1, 0) XA(2, 1) XA(3, 2) XA(4, 3) XA(5, 4) XA(6, 5) XA(7, 6) XA(0, 7)
                   XA(1, 0) XA(2, 1) XA(3, 2) XA(4, 3) XA(5, 4) XA(6, 5) XA(7, 6) XA(0, 7) : OPS);
    if constexpr (kMode == 9)  // 12 xor + 4 alignbit (3:1), independent
      asm volatile(X(0) X(1) X(2) A(3) X(4) X(5) X(6) A(7) X(1) X(0) X(3) A(2) X(5) X(4) X(7) A(6) : OPS);
    if constexpr (kMode == 10)  // xor, add alternating (both VOP2)
      asm volatile(X(0) D(1) X(2) D(3) X(4) D(5) X(6) D(7) X(1) D(0) X(3) D(2) X(5) D(4) X(7) D(6) : OPS);
    }
  }
  const uint64_t t1 = __builtin_readcyclecounter();
  if ((threadIdx.x & 63) == 0) atomicAdd(reinterpret_cast<unsigned long long*>(sink) + 1024, t1 - t0);
  const uint32_t x = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (x == 0x12345678u) sink[blockIdx.x] = x;
}

template <int kMode>
void run(const char* name, uint32_t* sink, int cus) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const uint32_t iters = 20000;  // x 64 instructions per wave
  for (int wps : {8, 4, 2, 1}) {
    const int blocks = cus * wps;  // 256 threads = 4 waves = 1 per SIMD
    k_issue<kMode><<<blocks, 256>>>(sink, 100);
    (void)hipMemset(sink + 2048, 0, 8);
    (void)hipEventRecord(e0);
    k_issue<kMode><<<blocks, 256>>>(sink, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long cyc = 0;
    (void)hipMemcpy(&cyc, sink + 2048, 8, hipMemcpyDeviceToHost);
    const double waves = double(blocks) * 4;
    const double instr_per_wave = double(iters) * 64;
    const double avg_wave_cycles = double(cyc) / waves;
    // all waves of a SIMD run concurrently: SIMD issue cycles per instruction
    const double cpi = avg_wave_cycles / (instr_per_wave * wps);
    const double tops = waves * 64 * instr_per_wave / (ms * 1e-3) / 1e12;
    printf("mode %2d %-34s W=%d: %6.2f T lane-instr/s  %.2f cyc/instr/SIMD  clk %.2f GHz\n",
           kMode, name, wps, tops, cpi, avg_wave_cycles / (ms * 1e-3) / 1e9);
  }
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* sink;
  (void)hipMalloc(&sink, 1 << 20);
  for (int w = 0; w < 30; ++w) k_issue<7><<<cus * 8, 256>>>(sink, 20000);  // clock ramp
  (void)hipDeviceSynchronize();
  run<0>("16 xor (VOP2) indep", sink, cus);
  run<1>("16 alignbit (VOP3) indep", sink, cus);
  run<2>("xor/alignbit alternating indep", sink, cus);
  run<3>("xor,xor,ab,ab pairs indep", sink, cus);
  run<4>("4 xor, 4 ab indep", sink, cus);
  run<5>("xor -> dependent ab", sink, cus);
  run<6>("16 add_u32 (VOP2) indep", sink, cus);
  run<7>("16 add3 (VOP3) indep", sink, cus);
  run<8>("16 xor dependent chain", sink, cus);
  run<9>("3 xor : 1 ab indep", sink, cus);
  run<10>("xor/add alternating (VOP2)", sink, cus);
  return 0;
}
