// Experiment (round 6, VERDICT r5 item 7, second try): the orphan remover's
// file_path ids read ONCE instead of once per XCD range, and no scan launch.
//   v1  sdgpu::orphan_objects_launch (the product): k_mark reads all 12.5 M
//       file_path ids 8 times (block b marks only range b % 8, so its byte
//       stores stay in its XCD's L2), then count -> scan -> write
//   v3  k_route: every file_path id read once; an id of the block's own range
//       (b % 8) is marked at once, the others are staged in LDS per range and
//       appended to the block's segment for that range (a fixed-capacity
//       slot per (block, range), overflow marked directly); k_seg_mark: block
//       j (on XCD j % 8) reads range j % 8's segments and marks; then count
//       and a write kernel that sums the counts before its tile itself (no
//       scan launch; the last tile writes the total)
//   v1w the product's mark + count + the self-summing write (isolates the
//       scan's share)
// Same data as exp_orphan_v2 (the bench's consumers leg: 10 M Objects, 12.5 M
// file_paths referencing random ids, every 1000th NULL).  Checks every
// variant's orphan list against v1's.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_orphan_v3.hip -o exp_bin/exp_orphan_v3
#include "../../spacedrive_amd/csrc/consumers.hip"

#include <stdio.h>

#include <vector>

namespace v3 {

using sdgpu::kThreads;
constexpr uint32_t kRanges = 8;
constexpr int kPer = 8;                            // ids per thread per round
constexpr uint32_t kRound = kThreads * kPer;       // 2048 ids per round
constexpr uint32_t kRouteBlocks = 2048;            // multiple of 8

struct Ws {
  int32_t* seg;     // [block][range][cap]
  uint32_t* scnt;   // [block][range]
  uint32_t* cnt;    // [tiles + 1]
  uint32_t cap;
  uint64_t chunk;
};

__device__ __forceinline__ uint32_t range_of(int32_t o, uint32_t span) {
  return static_cast<uint32_t>(o) / span;
}

__global__ __launch_bounds__(kThreads) void k_route(const int32_t* __restrict__ fp, uint64_t n,
                                                    uint8_t* __restrict__ mark, uint32_t max_id,
                                                    uint32_t span, uint64_t chunk, uint32_t cap,
                                                    int32_t* __restrict__ seg,
                                                    uint32_t* __restrict__ scnt) {
  // the round's staged ids, range-major (a scan of the 8 range counts): 8 KB
  __shared__ int32_t stage[kRound];
  __shared__ uint32_t rc[kRanges], pre[kRanges + 1], used[kRanges];
  const uint32_t own = blockIdx.x % kRanges;
  const uint64_t t0 = min<uint64_t>(n, chunk * blockIdx.x), t1 = min<uint64_t>(n, t0 + chunk);
  const uint32_t lane = __lane_id();
  const uint64_t lt = (1ull << lane) - 1ull;
  int32_t* myseg = seg + static_cast<uint64_t>(blockIdx.x) * kRanges * cap;
  if (threadIdx.x < kRanges) used[threadIdx.x] = 0;
  for (uint64_t r0 = t0; r0 < t1; r0 += kRound) {
    if (threadIdx.x < kRanges) rc[threadIdx.x] = 0;
    __syncthreads();
    int32_t o[kPer];
    uint32_t at[kPer], rg[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) o[u] = fp[min(r0 + u * kThreads + threadIdx.x, t1 - 1)];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const bool in = r0 + u * kThreads + threadIdx.x < t1 && o[u] >= 0 &&
                      static_cast<uint32_t>(o[u]) <= max_id;
      const uint32_t r = in ? range_of(o[u], span) : kRanges;
      if (r == own) mark[o[u]] = 1;
      const bool st = in && r != own;
      // lanes of the same range: 3 bit ballots (ranges are 3 bits)
      const uint64_t act = __ballot(st);
      const uint64_t b0 = __ballot(r & 1u), b1 = __ballot(r & 2u), b2 = __ballot(r & 4u);
      const uint64_t m = act & (r & 1u ? b0 : ~b0) & (r & 2u ? b1 : ~b1) & (r & 4u ? b2 : ~b2);
      uint32_t base = 0;
      const uint32_t leader = m ? static_cast<uint32_t>(__ffsll(static_cast<long long>(m)) - 1) : 64u;
      if (st && lane == leader) base = atomicAdd(&rc[r], static_cast<uint32_t>(__popcll(m)));
      base = __shfl(base, leader < 64u ? leader : 0u);
      rg[u] = st ? r : kRanges;
      at[u] = base + __popcll(m & lt);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t acc = 0;
      for (uint32_t q = 0; q < kRanges; ++q) {
        pre[q] = acc;
        acc += rc[q];
      }
      pre[kRanges] = acc;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kPer; ++u)
      if (rg[u] < kRanges) stage[pre[rg[u]] + at[u]] = o[u];
    __syncthreads();
    const uint32_t tot = pre[kRanges];
    for (uint32_t k = threadIdx.x; k < tot; k += kThreads) {
      uint32_t q = 0;
#pragma unroll
      for (uint32_t x = 1; x < kRanges; ++x) q += k >= pre[x] ? 1u : 0u;
      const uint32_t j = k - pre[q], u0 = used[q];
      const int32_t v = stage[k];
      if (u0 + j < cap)
        myseg[static_cast<uint64_t>(q) * cap + u0 + j] = v;
      else
        mark[v] = 1;  // segment full (skewed ids): a remote byte store
    }
    __syncthreads();
    if (threadIdx.x < kRanges) used[threadIdx.x] = min(cap, used[threadIdx.x] + rc[threadIdx.x]);
  }
  __syncthreads();
  if (threadIdx.x < kRanges) scnt[blockIdx.x * kRanges + threadIdx.x] = threadIdx.x == own ? 0u : used[threadIdx.x];
}

// one wave per source segment: block j (on XCD j % 8) takes range j % 8 of
// source blocks 4 (j / 8) .. 4 (j / 8) + 3, all of a segment's loads issued
// together
constexpr int kSegLoads = 24;  // 64 x 24 = 1536 = the segment capacity
__global__ __launch_bounds__(kThreads) void k_seg_mark(const int32_t* __restrict__ seg,
                                                       const uint32_t* __restrict__ scnt,
                                                       uint32_t nsrc, uint32_t cap,
                                                       uint8_t* __restrict__ mark) {
  const uint32_t q = blockIdx.x % kRanges;
  const uint32_t b = (blockIdx.x / kRanges) * (kThreads / 64) + (threadIdx.x >> 6);
  if (b >= nsrc) return;
  const uint32_t lane = __lane_id();
  const uint32_t c = scnt[b * kRanges + q];
  const int32_t* s = seg + (static_cast<uint64_t>(b) * kRanges + q) * cap;
  for (uint32_t k0 = 0; k0 < c; k0 += 64 * kSegLoads) {
    int32_t v[kSegLoads];
#pragma unroll
    for (int u = 0; u < kSegLoads; ++u) v[u] = s[min(k0 + u * 64 + lane, c - 1)];
#pragma unroll
    for (int u = 0; u < kSegLoads; ++u)
      if (k0 + u * 64 + lane < c) mark[v[u]] = 1;
  }
}

// the product's k_orphan_write, but its tile's offset summed here from the
// tile counts before it (no scan launch); the last tile writes the total
__global__ __launch_bounds__(kThreads) void k_write_self(const int32_t* __restrict__ obj, uint64_t n,
                                                         const uint8_t* __restrict__ bits,
                                                         uint32_t max_id,
                                                         const uint32_t* __restrict__ cnt,
                                                         int32_t* __restrict__ out,
                                                         uint32_t* __restrict__ d_count) {
  using namespace sdgpu;
  constexpr int kOW = kThreads / 64;
  __shared__ uint32_t off[kORows][kOW];
  __shared__ uint32_t part[kOW];
  const uint64_t tile = static_cast<uint64_t>(blockIdx.x) * kOTile;
  const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  int32_t o[kORows];
  uint8_t m[kORows];
  uint32_t pre[kORows], f = 0;
  obj_tile(obj, n, tile, bits, max_id, o, m);
  uint32_t s = 0;
  for (uint32_t k = threadIdx.x; k < blockIdx.x; k += kThreads) s += cnt[k];
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) s += __shfl_xor(s, d);
  if (lane == 0) part[w] = s;
#pragma unroll
  for (int k = 0; k < kORows; ++k) {
    const bool is = orphan(o[k], m[k], max_id);
    f |= (is ? 1u : 0u) << k;
    const uint64_t b = __ballot(is);
    pre[k] = __popcll(b & lt);
    if (lane == 0) off[k][w] = __popcll(b);
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    uint32_t base = 0;
#pragma unroll
    for (int x = 0; x < kOW; ++x) base += part[x];
    uint32_t* fl = &off[0][0];
    const uint32_t a = fl[lane];
    uint32_t inc = a;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t x = __shfl_up(inc, d);
      if (lane >= static_cast<uint32_t>(d)) inc += x;
    }
    fl[lane] = base + inc - a;
    if (blockIdx.x == gridDim.x - 1 && lane == 63) d_count[0] = base + inc;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kORows; ++k)
    if (f >> k & 1u) out[off[k][w] + pre[k]] = o[k];
}

void tail(const int32_t* obj, uint64_t n_obj, const uint8_t* bits, uint32_t max_id, uint32_t* cnt,
          int32_t* out, uint32_t* d_count, hipStream_t s) {
  const uint64_t blocks = (n_obj + sdgpu::kOTile - 1) / sdgpu::kOTile;
  sdgpu::k_orphan_count<<<static_cast<uint32_t>(blocks), kThreads, 0, s>>>(obj, n_obj, bits, max_id, cnt);
  k_write_self<<<static_cast<uint32_t>(blocks), kThreads, 0, s>>>(obj, n_obj, bits, max_id, cnt, out,
                                                                  d_count);
}

void mark_v3(const int32_t* fp, uint64_t n_fp, uint32_t max_id, uint8_t* bits, const Ws& w,
             hipStream_t s) {
  const uint32_t span = static_cast<uint32_t>((static_cast<uint64_t>(max_id) + kRanges) / kRanges);
  k_route<<<kRouteBlocks, kThreads, 0, s>>>(fp, n_fp, bits, max_id, span, w.chunk, w.cap, w.seg,
                                            w.scnt);
  k_seg_mark<<<kRanges * (kRouteBlocks / 4), kThreads, 0, s>>>(w.seg, w.scnt, kRouteBlocks, w.cap, bits);
}

}  // namespace v3

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
  const uint64_t map = (static_cast<uint64_t>(max_id) + 1 + 255) / 256 * 256;
  const uint64_t blocks = (n_obj + sdgpu::kOTile - 1) / sdgpu::kOTile;
  int32_t *obj, *fp, *out[3];
  uint32_t* cnt_out[3];
  CK(hipMalloc(&obj, 4 * n_obj));
  CK(hipMalloc(&fp, 4 * n_fp));
  for (int v = 0; v < 3; ++v) {
    CK(hipMalloc(&out[v], 4 * n_obj));
    CK(hipMalloc(&cnt_out[v], 4));
  }
  k_gen<<<2048, 256>>>(obj, n_obj, fp, n_fp);
  void* ws1;
  CK(hipMalloc(&ws1, sdgpu::orphan_workspace_bytes(n_obj, max_id)));
  uint8_t* bits3;
  CK(hipMalloc(&bits3, map));
  v3::Ws w{};
  w.chunk = (n_fp + v3::kRouteBlocks - 1) / v3::kRouteBlocks;
  w.cap = static_cast<uint32_t>((w.chunk / 4 + 63) / 64 * 64);
  CK(hipMalloc(&w.seg, 4ull * v3::kRouteBlocks * v3::kRanges * w.cap));
  CK(hipMalloc(&w.scnt, 4ull * v3::kRouteBlocks * v3::kRanges));
  CK(hipMalloc(&w.cnt, 4 * (blocks + 1)));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipDeviceSynchronize());
  printf("route: %u blocks, chunk %llu ids, segment cap %u (%.1f MB)\n", v3::kRouteBlocks,
         static_cast<unsigned long long>(w.chunk), w.cap,
         4.0 * v3::kRouteBlocks * v3::kRanges * w.cap / 1e6);
  const char* vname[3] = {"v1 ", "v3 ", "v1w"};
  auto run = [&](int v) {
    if (v == 0) {
      (void)sdgpu::orphan_objects_launch(obj, n_obj, fp, n_fp, max_id, out[0], cnt_out[0], ws1, s);
    } else if (v == 1) {
      (void)hipMemsetAsync(bits3, 0, map, s);
      v3::mark_v3(fp, n_fp, max_id, bits3, w, s);
      v3::tail(obj, n_obj, bits3, max_id, w.cnt, out[1], cnt_out[1], s);
    } else {
      // the product's mark, then the self-summing tail
      (void)hipMemsetAsync(bits3, 0, map, s);
      const uint32_t span = static_cast<uint32_t>((static_cast<uint64_t>(max_id) + 8) / 8);
      const uint64_t per = (n_fp + 4 * v3::kThreads - 1) / (4 * v3::kThreads);
      const uint32_t groups = static_cast<uint32_t>(per < 256 ? per : 256);
      sdgpu::k_mark<<<groups * 8, v3::kThreads, 0, s>>>(fp, n_fp, bits3, max_id, span, 8);
      v3::tail(obj, n_obj, bits3, max_id, w.cnt, out[2], cnt_out[2], s);
    }
  };
  for (int rep = 0; rep < 3; ++rep) {
    for (int v = 0; v < 3; ++v) {
      for (int i = 0; i < 3; ++i) run(v);
      CK(hipEventRecord(e0, s));
      constexpr int kSteps = 20;
      for (int i = 0; i < kSteps; ++i) run(v);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("%s: %.4f ms per call\n", vname[v], ms / kSteps);
    }
  }
  {  // v3 per kernel (events between the launches of one call, 10 calls)
    const char* names[5] = {"memset", "route", "seg_mark", "count", "write_self"};
    hipEvent_t ev[6];
    for (auto& e : ev) CK(hipEventCreate(&e));
    double acc[5] = {0};
    const uint32_t span = static_cast<uint32_t>((static_cast<uint64_t>(max_id) + 8) / 8);
    for (int it = 0; it < 10; ++it) {
      CK(hipEventRecord(ev[0], s));
      (void)hipMemsetAsync(bits3, 0, map, s);
      CK(hipEventRecord(ev[1], s));
      v3::k_route<<<v3::kRouteBlocks, v3::kThreads, 0, s>>>(fp, n_fp, bits3, max_id, span, w.chunk,
                                                            w.cap, w.seg, w.scnt);
      CK(hipEventRecord(ev[2], s));
      v3::k_seg_mark<<<v3::kRanges * (v3::kRouteBlocks / 4), v3::kThreads, 0, s>>>(w.seg, w.scnt, v3::kRouteBlocks,
                                                               w.cap, bits3);
      CK(hipEventRecord(ev[3], s));
      sdgpu::k_orphan_count<<<static_cast<uint32_t>(blocks), v3::kThreads, 0, s>>>(obj, n_obj, bits3,
                                                                                   max_id, w.cnt);
      CK(hipEventRecord(ev[4], s));
      v3::k_write_self<<<static_cast<uint32_t>(blocks), v3::kThreads, 0, s>>>(
          obj, n_obj, bits3, max_id, w.cnt, out[1], cnt_out[1]);
      CK(hipEventRecord(ev[5], s));
      CK(hipEventSynchronize(ev[5]));
      for (int k = 0; k < 5; ++k) {
        float ms = 0;
        CK(hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
        acc[k] += ms / 10;
      }
    }
    for (int k = 0; k < 5; ++k) printf("  v3 %-10s %.4f ms\n", names[k], acc[k]);
  }
  CK(hipDeviceSynchronize());
  uint32_t h[3];
  std::vector<int32_t> lists[3];
  for (int v = 0; v < 3; ++v) {
    CK(hipMemcpy(&h[v], cnt_out[v], 4, hipMemcpyDeviceToHost));
    lists[v].resize(h[v]);
    CK(hipMemcpy(lists[v].data(), out[v], 4ull * h[v], hipMemcpyDeviceToHost));
  }
  bool ok = true;
  for (int v = 1; v < 3; ++v) {
    const bool same = h[v] == h[0] && lists[v] == lists[0];
    printf("orphans %s %u vs v1 %u: %s\n", vname[v], h[v], h[0], same ? "identical" : "DIFFER");
    ok = ok && same;
  }
  return ok ? 0 : 2;
}
