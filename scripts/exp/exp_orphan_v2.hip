// Experiment (round 6): the orphan remover with the
// file_path ids partitioned by id range, one workgroup per range setting the
// range's bits in an LDS bitmap, against the product's XCD-ranged byte map
// (consumers.hip: every XCD reads all file_path ids and marks its eighth of
// a byte per Object id).
//   v1  sdgpu::orphan_objects_launch (the product)
//   v2  hist of ids by range (R <= 4096 ranges of 2^rb ids) -> scan ->
//       scatter of the ids by range -> one workgroup per range: LDS bitmap,
//       written whole -> count / scan / write over the Object list with a
//       bit test instead of a byte load
// 10 M Objects (ids 0..10M-1 in order), 12.5 M file_paths referencing random
// ids, every 1000th NULL -- the bench's consumers leg.  Checks v2 == v1.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_orphan_v2.hip -o exp_bin/exp_orphan_v2
#include "../../spacedrive_amd/csrc/consumers.hip"

#include <stdio.h>

#include <vector>

namespace v2 {

constexpr int kT = 1024;
constexpr uint32_t kP = 256;  // hist / scatter blocks (one per CU)
constexpr uint32_t kMaxR = 4096;

struct Plan {
  uint32_t rb, R;
};
Plan plan(uint32_t max_id) {
  uint32_t rb = 10;
  while (rb < 19 && (max_id >> rb) + 1u > 256u) ++rb;
  return {rb, (max_id >> rb) + 1u};
}

__device__ __forceinline__ void tile(uint64_t n, uint64_t& t0, uint64_t& t1) {
  const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
  t0 = min<uint64_t>(n, per * blockIdx.x);
  t1 = min<uint64_t>(n, t0 + per);
}

__device__ __forceinline__ bool valid_id(int32_t o, uint32_t max_id) {
  return o >= 0 && static_cast<uint32_t>(o) <= max_id;
}

__global__ __launch_bounds__(kT) void k_hist(const int32_t* __restrict__ fp, uint64_t n,
                                             uint32_t max_id, uint32_t rb, uint32_t R,
                                             uint32_t* __restrict__ hist) {
  __shared__ uint32_t cnt[kMaxR];
  for (uint32_t r = threadIdx.x; r < R; r += kT) cnt[r] = 0;
  __syncthreads();
  uint64_t t0, t1;
  tile(n, t0, t1);
  for (uint64_t i0 = t0 + threadIdx.x; i0 < t1; i0 += 4 * kT) {
    int32_t o[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) o[u] = fp[min(i0 + u * kT, t1 - 1)];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i0 + u * kT < t1 && valid_id(o[u], max_id)) atomicAdd(&cnt[static_cast<uint32_t>(o[u]) >> rb], 1u);
  }
  __syncthreads();
  for (uint32_t r = threadIdx.x; r < R; r += kT) hist[static_cast<uint64_t>(r) * kP + blockIdx.x] = cnt[r];
}

__global__ __launch_bounds__(kT) void k_scatter(const int32_t* __restrict__ fp, uint64_t n,
                                                uint32_t max_id, uint32_t rb, uint32_t R,
                                                const uint32_t* __restrict__ offs,
                                                uint32_t* __restrict__ ids) {
  __shared__ uint32_t cur[kMaxR];
  for (uint32_t r = threadIdx.x; r < R; r += kT) cur[r] = offs[static_cast<uint64_t>(r) * kP + blockIdx.x];
  __syncthreads();
  uint64_t t0, t1;
  tile(n, t0, t1);
  for (uint64_t i0 = t0 + threadIdx.x; i0 < t1; i0 += 4 * kT) {
    int32_t o[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) o[u] = fp[min(i0 + u * kT, t1 - 1)];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i0 + u * kT < t1 && valid_id(o[u], max_id))
        ids[atomicAdd(&cur[static_cast<uint32_t>(o[u]) >> rb], 1u)] = static_cast<uint32_t>(o[u]);
  }
}

// one workgroup per range: its ids' bits set in LDS, the bitmap written whole
__global__ __launch_bounds__(kT) void k_markbits(const uint32_t* __restrict__ ids,
                                                 const uint32_t* __restrict__ offs, uint32_t rb,
                                                 uint32_t* __restrict__ bits) {
  extern __shared__ uint32_t bm[];
  const uint32_t r = blockIdx.x, words = 1u << (rb - 5), mask = (1u << rb) - 1u;
  for (uint32_t w = threadIdx.x; w < words; w += kT) bm[w] = 0;
  __syncthreads();
  const uint32_t s0 = offs[static_cast<uint64_t>(r) * kP], s1 = offs[static_cast<uint64_t>(r + 1) * kP];
  for (uint32_t i0 = s0 + threadIdx.x; i0 < s1; i0 += 4 * kT) {
    uint32_t o[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) o[u] = ids[min(i0 + u * kT, s1 - 1)];  // a repeat sets its bit again
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t l = o[u] & mask;
      atomicOr(&bm[l >> 5], 1u << (l & 31u));
    }
  }
  __syncthreads();
  for (uint32_t w = threadIdx.x; w < words; w += kT) bits[static_cast<uint64_t>(r) * words + w] = bm[w];
}

constexpr int kThreads = 256, kORows = 16, kOWaves = kThreads / 64;
constexpr uint64_t kOTile = static_cast<uint64_t>(kORows) * kThreads;

__device__ __forceinline__ bool orphan(int32_t o, const uint32_t* bits, uint32_t max_id) {
  if (o < 0) return false;
  if (static_cast<uint32_t>(o) > max_id) return true;
  return ((bits[static_cast<uint32_t>(o) >> 5] >> (o & 31)) & 1u) == 0u;
}

__global__ __launch_bounds__(kThreads) void k_count(const int32_t* __restrict__ obj, uint64_t n,
                                                    const uint32_t* __restrict__ bits,
                                                    uint32_t max_id, uint32_t* __restrict__ cnt) {
  __shared__ uint32_t sw[kOWaves];
  const uint64_t t = static_cast<uint64_t>(blockIdx.x) * kOTile;
  int32_t o[kORows];
#pragma unroll
  for (int k = 0; k < kORows; ++k) o[k] = obj[min(t + k * kThreads + threadIdx.x, n - 1)];
#pragma unroll
  for (int k = 0; k < kORows; ++k)
    if (t + k * kThreads + threadIdx.x >= n) o[k] = -1;
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < kORows; ++k) c += orphan(o[k], bits, max_id) ? 1u : 0u;
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d);
  if (__lane_id() == 0) sw[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int w = 0; w < kOWaves; ++w) s += sw[w];
    cnt[blockIdx.x] = s;
  }
}

__global__ __launch_bounds__(kThreads) void k_write(const int32_t* __restrict__ obj, uint64_t n,
                                                    const uint32_t* __restrict__ bits,
                                                    uint32_t max_id,
                                                    const uint32_t* __restrict__ offs,
                                                    int32_t* __restrict__ out) {
  __shared__ uint32_t off[kORows][kOWaves];
  const uint64_t t = static_cast<uint64_t>(blockIdx.x) * kOTile;
  const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  int32_t o[kORows];
  uint32_t pre[kORows], f = 0;
#pragma unroll
  for (int k = 0; k < kORows; ++k) o[k] = obj[min(t + k * kThreads + threadIdx.x, n - 1)];
#pragma unroll
  for (int k = 0; k < kORows; ++k)
    if (t + k * kThreads + threadIdx.x >= n) o[k] = -1;
#pragma unroll
  for (int k = 0; k < kORows; ++k) {
    const bool is = orphan(o[k], bits, max_id);
    f |= (is ? 1u : 0u) << k;
    const uint64_t b = __ballot(is);
    pre[k] = __popcll(b & lt);
    if (lane == 0) off[k][w] = __popcll(b);
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    uint32_t* fo = &off[0][0];
    const uint32_t a = fo[lane];
    uint32_t inc = a;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t x = __shfl_up(inc, d);
      if (lane >= static_cast<uint32_t>(d)) inc += x;
    }
    fo[lane] = offs[blockIdx.x] + inc - a;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kORows; ++k)
    if (f >> k & 1u) out[off[k][w] + pre[k]] = o[k];
}

struct Ws {
  uint32_t *hist, *htiles, *ids, *bits, *cnt, *ctiles;
};

void launch(const int32_t* obj, uint64_t n_obj, const int32_t* fp, uint64_t n_fp, uint32_t max_id,
            int32_t* out, uint32_t* d_count, const Ws& w, hipStream_t s) {
  const Plan p = plan(max_id);
  const uint64_t nh = static_cast<uint64_t>(p.R) * kP;
  k_hist<<<kP, kT, 0, s>>>(fp, n_fp, max_id, p.rb, p.R, w.hist);
  sdgpu::scan::exclusive(w.hist, nh, w.hist, w.htiles, nullptr, s);
  k_scatter<<<kP, kT, 0, s>>>(fp, n_fp, max_id, p.rb, p.R, w.hist, w.ids);
  k_markbits<<<p.R, kT, (1u << (p.rb - 5)) * 4, s>>>(w.ids, w.hist, p.rb, w.bits);
  const uint64_t blocks = (n_obj + kOTile - 1) / kOTile;
  k_count<<<static_cast<uint32_t>(blocks), kThreads, 0, s>>>(obj, n_obj, w.bits, max_id, w.cnt);
  sdgpu::scan::exclusive(w.cnt, blocks, w.cnt, w.ctiles, d_count, s);
  k_write<<<static_cast<uint32_t>(blocks), kThreads, 0, s>>>(obj, n_obj, w.bits, max_id, w.cnt, out);
}

}  // namespace v2

__global__ void k_gen(int32_t* obj, uint64_t n_obj, int32_t* fp, uint64_t n_fp) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n_fp; i += stride) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull + 5;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    fp[i] = i % 1000 == 0 ? -1 : static_cast<int32_t>(z % n_obj);
    if (i < n_obj) obj[i] = static_cast<int32_t>(i);
  }
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  const uint64_t n_obj = 10000000, n_fp = 12500000;
  const uint32_t max_id = static_cast<uint32_t>(n_obj - 1);
  int32_t *obj, *fp, *out1, *out2;
  uint32_t *c1, *c2;
  CK(hipMalloc(&obj, 4 * n_obj));
  CK(hipMalloc(&fp, 4 * n_fp));
  CK(hipMalloc(&out1, 4 * n_obj));
  CK(hipMalloc(&out2, 4 * n_obj));
  CK(hipMalloc(&c1, 4));
  CK(hipMalloc(&c2, 4));
  k_gen<<<2048, 256>>>(obj, n_obj, fp, n_fp);
  void* ws1;
  CK(hipMalloc(&ws1, sdgpu::orphan_workspace_bytes(n_obj, max_id)));
  const v2::Plan p = v2::plan(max_id);
  const uint64_t nh = static_cast<uint64_t>(p.R) * v2::kP;
  const uint64_t blocks = (n_obj + v2::kOTile - 1) / v2::kOTile;
  v2::Ws w{};
  CK(hipMalloc(&w.hist, 4 * (nh + 1)));
  CK(hipMalloc(&w.htiles, 4 * (sdgpu::scan::tiles_for(nh) + 1)));
  CK(hipMalloc(&w.ids, 4 * n_fp));
  CK(hipMalloc(&w.bits, 4 * (static_cast<uint64_t>(p.R) << (p.rb - 5))));
  CK(hipMalloc(&w.cnt, 4 * (blocks + 1)));
  CK(hipMalloc(&w.ctiles, 4 * (sdgpu::scan::tiles_for(blocks) + 1)));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipDeviceSynchronize());
  printf("plan: rb %u ranges %u\n", p.rb, p.R);
  for (int rep = 0; rep < 3; ++rep) {
    for (int variant = 1; variant <= 2; ++variant) {
      auto run = [&] {
        if (variant == 1)
          (void)sdgpu::orphan_objects_launch(obj, n_obj, fp, n_fp, max_id, out1, c1, ws1, s);
        else
          v2::launch(obj, n_obj, fp, n_fp, max_id, out2, c2, w, s);
      };
      for (int i = 0; i < 3; ++i) run();
      CK(hipEventRecord(e0, s));
      constexpr int kSteps = 20;
      for (int i = 0; i < kSteps; ++i) run();
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("v%d: %.4f ms per call\n", variant, ms / kSteps);
    }
  }
  {  // v2 per kernel (events between the launches of one call, 10 calls)
    const char* names[7] = {"hist", "scan1", "scatter", "markbits", "count", "scan2", "write"};
    hipEvent_t ev[8];
    for (auto& e : ev) CK(hipEventCreate(&e));
    double acc[7] = {0};
    for (int it = 0; it < 10; ++it) {
      CK(hipEventRecord(ev[0], s));
      v2::k_hist<<<v2::kP, v2::kT, 0, s>>>(fp, n_fp, max_id, p.rb, p.R, w.hist);
      CK(hipEventRecord(ev[1], s));
      sdgpu::scan::exclusive(w.hist, nh, w.hist, w.htiles, nullptr, s);
      CK(hipEventRecord(ev[2], s));
      v2::k_scatter<<<v2::kP, v2::kT, 0, s>>>(fp, n_fp, max_id, p.rb, p.R, w.hist, w.ids);
      CK(hipEventRecord(ev[3], s));
      v2::k_markbits<<<p.R, v2::kT, (1u << (p.rb - 5)) * 4, s>>>(w.ids, w.hist, p.rb, w.bits);
      CK(hipEventRecord(ev[4], s));
      v2::k_count<<<static_cast<uint32_t>(blocks), v2::kThreads, 0, s>>>(obj, n_obj, w.bits, max_id, w.cnt);
      CK(hipEventRecord(ev[5], s));
      sdgpu::scan::exclusive(w.cnt, blocks, w.cnt, w.ctiles, c2, s);
      CK(hipEventRecord(ev[6], s));
      v2::k_write<<<static_cast<uint32_t>(blocks), v2::kThreads, 0, s>>>(obj, n_obj, w.bits, max_id, w.cnt, out2);
      CK(hipEventRecord(ev[7], s));
      CK(hipEventSynchronize(ev[7]));
      for (int k = 0; k < 7; ++k) {
        float ms = 0;
        CK(hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
        acc[k] += ms / 10;
      }
    }
    for (int k = 0; k < 7; ++k) printf("  v2 %-9s %.4f ms\n", names[k], acc[k]);
  }
  uint32_t h1 = 0, h2 = 0;
  CK(hipMemcpy(&h1, c1, 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&h2, c2, 4, hipMemcpyDeviceToHost));
  std::vector<int32_t> a(h1), b(h2);
  CK(hipMemcpy(a.data(), out1, 4ull * h1, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), out2, 4ull * h2, hipMemcpyDeviceToHost));
  const bool same = h1 == h2 && a == b;
  printf("orphans v1 %u v2 %u: %s\n", h1, h2, same ? "identical" : "DIFFER");
  return same ? 0 : 2;
}
