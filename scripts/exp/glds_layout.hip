// Where does global_load_lds_dword{,x3,x4} put lane L's bytes in LDS?
// One wave copies 64 * size bytes of a counting pattern into LDS (m0 = 256),
// the LDS image is dumped and compared with the contiguous layout
// base + lane * size.  hipcc --offload-arch=gfx950 -O2 glds_layout.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

template <int SZ>
__global__ void k(const uint32_t* __restrict__ src, uint32_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = 0xDEADBEEFu;
  __syncthreads();
  const uint8_t* g = reinterpret_cast<const uint8_t*>(src) + threadIdx.x * SZ;
  auto* d = (__attribute__((address_space(3))) void*)((__attribute__((address_space(3))) uint8_t*)lds + 256);
  if constexpr (SZ == 4) __builtin_amdgcn_global_load_lds(g, d, 4, 0, 0);
  else if constexpr (SZ == 12) __builtin_amdgcn_global_load_lds(g, d, 12, 0, 0);
  else __builtin_amdgcn_global_load_lds(g, d, 16, 0, 0);
  __syncthreads();
  for (int i = threadIdx.x; i < 1024; i += 64) out[i] = lds[i];
}

template <int SZ>
int run(uint32_t* d_src, uint32_t* d_out) {
  hipLaunchKernelGGL(k<SZ>, dim3(1), dim3(64), 4096, 0, d_src, d_out);
  std::vector<uint32_t> h(1024);
  if (hipMemcpy(h.data(), d_out, 4096, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  int bad = 0, first = -1;
  for (int i = 0; i < 1024; ++i) {
    const int b = i * 4 - 256;
    const uint32_t want = (b >= 0 && b < 64 * SZ) ? static_cast<uint32_t>(b / 4) : 0xDEADBEEFu;
    if (h[i] != want) { if (first < 0) first = i; ++bad; }
  }
  printf("size %2d: %s (%d words differ from base + lane*size)", SZ, bad ? "NOT contiguous" : "contiguous", bad);
  if (bad) {
    printf("; words 64..%d:", 64 + 3 * 16);
    for (int i = 64; i < 64 + 48; ++i) printf(" %x", h[i]);
  }
  printf("\n");
  return bad ? 1 : 0;
}

int main() {
  uint32_t *d_src, *d_out;
  (void)hipMalloc(&d_src, 4096);
  (void)hipMalloc(&d_out, 4096);
  std::vector<uint32_t> s(1024);
  for (int i = 0; i < 1024; ++i) s[i] = i;
  (void)hipMemcpy(d_src, s.data(), 4096, hipMemcpyHostToDevice);
  int r = run<4>(d_src, d_out);
  r |= run<12>(d_src, d_out);
  r |= run<16>(d_src, d_out);
  (void)hipDeviceSynchronize();
  return 0 * r;
}
