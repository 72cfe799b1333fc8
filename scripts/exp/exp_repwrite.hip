// Experiment (round 4): the grouping's rep writes.
// K5 (k_bucket_group12_pk) writes rep[row] = f for every row that links to an
// earlier chunk: 20 M scattered 4-B stores into a 400 MB array at 100 M rows
// (PMC 0.64 GB written for 80 MB of reps).  Variants of the group kernel's
// OUTPUT, over the product's own partition (config-4-shaped rows in rank
// order: 12-byte records, 2^15 buckets at 100 M rows, 2^12 at 12.5 M):
//   G0  product: scattered rep writes (rep initialised = rank beforehand)
//   GN  no output at all (the group-by alone)
//   GF  fused job output: per bucket, in record order, the creator ranks
//       (who[start, split)) then the linked rows (who[split, end)) with their
//       Object's creator rank (obj[split, end)); coalesced, no rep array
//   GH  rows below `split` written to rep directly (a region that fits the
//       256 MB Infinity Cache), the others appended to a per-bucket pair list
//       ({row, f}, coalesced) and scattered by a second kernel
//   GP  every linked row as a pair, then the scatter kernel
//   GW  the pairs counting-sorted by row window (128 windows, ~3 MB of rep
//       each) + per-bucket window boundaries; then AW: each window's pairs
//       applied by the workgroups of ONE XCD, so its rep lines merge in L2
// and the partition's coarse pass with / without its rep = rank stores.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_repwrite.hip -o build/exp_repwrite
#include "../../spacedrive_amd/csrc/dedup.hip"

#include <stdio.h>

#include <algorithm>
#include <functional>
#include <vector>

using namespace sdgpu;

namespace {

__global__ void k_rows(uint64_t* key, uint8_t* has, uint64_t n, uint64_t distinct) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint64_t j = (i * 0x9E3779B1ull) % n;
    key[i] = row_hash((j % distinct) * 0x2545F4914F6CDD1Dull + 7);
    has[i] = (row_hash(i ^ 0x55ull) % 1000) != 0;
  }
}

enum Mode { kG0 = 0, kGN = 1, kGF = 2, kGH = 3, kGW = 4 };
constexpr uint32_t kNW = 128;  // row windows of the GW / AW pair lists

// group_bucket_packed with the output as a policy (buckets <= kPkCap only)
template <int kMode>
__global__ __launch_bounds__(kGroupThreads, 8) void k_group_x(
    const uint3* __restrict__ rec, uint32_t rank_base, const uint32_t* __restrict__ offs,
    uint32_t bits, ChunkOf chunk_of, uint32_t* __restrict__ rep, uint32_t* __restrict__ who,
    uint32_t* __restrict__ obj, uint32_t* __restrict__ split_out, uint2* __restrict__ pairs,
    uint32_t* __restrict__ npairs, uint32_t split_row, uint32_t never,
    uint32_t* __restrict__ bnd = nullptr, uint32_t win_rows = 1) {
  __shared__ uint64_t tab[kPkSlots];
  __shared__ uint32_t lmin[kPkCap + 1];
  __shared__ uint32_t oc[4][16], ol[4][16];
  __shared__ uint32_t wc[kNW], wp[kNW + 1];
  constexpr int kP = (kPkCap + kGroupThreads) / kGroupThreads;  // 4
  const uint32_t b = blockIdx.x;
  const uint32_t start = offs[b], end = offs[b + 1];
  const uint32_t m = end - start;
  const Rec12Src src{rec, rank_base};
  uint4 q[kP];
#pragma unroll
  for (int j = 0; j < kP; ++j) q[j] = src(min(start + threadIdx.x + j * kGroupThreads, end - 1));
#pragma unroll
  for (int j = 0; j < kP; ++j)
    if (start + threadIdx.x + j * kGroupThreads >= end || m == 0) q[j] = make_uint4(0, 0, kPadRow, kPadRow);
  for (uint32_t s = threadIdx.x; s < kPkSlots; s += kGroupThreads) tab[s] = 0ull;
  for (uint32_t s = threadIdx.x; s <= kPkCap; s += kGroupThreads) lmin[s] = 0xFFFFFFFFu;
  if (kMode == kGW && threadIdx.x < kNW) wc[threadIdx.x] = 0;
  __syncthreads();
  uint32_t slot[kP], step[kP], owner[kP];
  uint64_t mine[kP];
  uint32_t pend = 0;
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const uint64_t h = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
    const uint32_t idx = threadIdx.x + j * kGroupThreads;
    mine[j] = (key_rest(h, bits) << 12) | (idx + 1);
    slot[j] = static_cast<uint32_t>((static_cast<uint64_t>(static_cast<uint32_t>(h)) * kPkSlots) >> 32);
    uint32_t st = 1u + 2u * static_cast<uint32_t>((h >> 40) & 1023u);
    st += (st % 3u == 0) ? 2u : 0u;
    st += (st % 5u == 0) ? 2u : 0u;
    st += (st % 3u == 0) ? 2u : 0u;
    step[j] = st;
    owner[j] = idx;
    if (q[j].w != kPadRow) pend |= 1u << j;
  }
  const uint32_t live = pend;
  while (pend) {
    uint64_t prev[kP];
#pragma unroll
    for (int j = 0; j < kP; ++j)
      prev[j] = (pend >> j & 1u)
                    ? atomicCAS(reinterpret_cast<unsigned long long*>(&tab[slot[j]]), 0ull,
                                static_cast<unsigned long long>(mine[j]))
                    : 0ull;
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      if (!(pend >> j & 1u)) continue;
      if (prev[j] == 0ull) {
        pend &= ~(1u << j);
      } else if ((prev[j] >> 12) == (mine[j] >> 12)) {
        owner[j] = static_cast<uint32_t>(prev[j] & 0xFFFu) - 1;
        pend &= ~(1u << j);
      } else {
        const uint32_t sn = slot[j] + step[j];
        slot[j] = sn >= kPkSlots ? sn - kPkSlots : sn;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < kP; ++j)
    if (live >> j & 1u) atomicMin(&lmin[owner[j]], q[j].z);
  __syncthreads();
  uint32_t f[kP];
  bool lk[kP];
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    f[j] = lmin[owner[j]];
    lk[j] = (live >> j & 1u) && chunk_of(q[j].z) != chunk_of(f[j]);
  }
  if constexpr (kMode == kG0) {
#pragma unroll
    for (int j = 0; j < kP; ++j)
      if (lk[j]) rep[q[j].w] = f[j];
  } else if constexpr (kMode == kGW) {
    // linked pairs counting-sorted by row window (LDS counters), the
    // bucket's window boundaries written beside: bnd[b][0..kNW]
    uint32_t rk[kP], wn[kP];
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      wn[j] = lk[j] ? q[j].w / win_rows : 0u;
      rk[j] = lk[j] ? atomicAdd(&wc[wn[j]], 1u) : 0u;
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      const uint32_t lane = threadIdx.x;
      const uint32_t a0 = wc[2 * lane], a1 = wc[2 * lane + 1], v = a0 + a1;
      uint32_t inc = v;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(inc, d);
        if (lane >= static_cast<uint32_t>(d)) inc += o;
      }
      wp[2 * lane] = inc - v;
      wp[2 * lane + 1] = inc - v + a0;
      if (lane == 63) wp[kNW] = inc;
    }
    __syncthreads();
    if (threadIdx.x <= kNW) bnd[static_cast<uint64_t>(b) * (kNW + 1) + threadIdx.x] = wp[threadIdx.x];
#pragma unroll
    for (int j = 0; j < kP; ++j)
      if (lk[j]) pairs[start + wp[wn[j]] + rk[j]] = make_uint2(q[j].w, f[j]);
  } else if constexpr (kMode == kGN) {
#pragma unroll
    for (int j = 0; j < kP; ++j)
      if (lk[j] && f[j] == never) rep[0] = q[j].w;
  } else {
    // in-bucket ranks in record order: (j, wave) ballots, one wave scans the
    // 64 counts (j-major = record order)
    const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
    const uint64_t lt = (1ull << lane) - 1ull;
    bool c_[kP], l_[kP];
    uint32_t pc[kP], pl[kP];
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      if constexpr (kMode == kGF) {
        c_[j] = (live >> j & 1u) && !lk[j];
        l_[j] = lk[j];
      } else {  // kGH: pairs for linked rows at or above split_row
        c_[j] = false;
        l_[j] = lk[j] && q[j].w >= split_row;
      }
      const uint64_t bc = __ballot(c_[j]), bl = __ballot(l_[j]);
      pc[j] = __popcll(bc & lt);
      pl[j] = __popcll(bl & lt);
      if (lane == 0) {
        oc[j][w] = __popcll(bc);
        ol[j][w] = __popcll(bl);
      }
    }
    if constexpr (kMode == kGH) {
#pragma unroll
      for (int j = 0; j < kP; ++j)
        if (lk[j] && q[j].w < split_row) rep[q[j].w] = f[j];
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      uint32_t* fc = &oc[0][0];
      uint32_t* fl = &ol[0][0];
      const uint32_t a = fc[lane], bb = fl[lane];
      uint32_t ic = a, il = bb;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t xc = __shfl_up(ic, d), xl = __shfl_up(il, d);
        if (lane >= static_cast<uint32_t>(d)) {
          ic += xc;
          il += xl;
        }
      }
      const uint32_t C = __shfl(ic, 63);
      fc[lane] = ic - a;
      fl[lane] = (kMode == kGF ? C : 0u) + il - bb;
      if (lane == 63) {
        if constexpr (kMode == kGF) split_out[b] = start + C;
        else npairs[b] = il;
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      if constexpr (kMode == kGF) {
        if (c_[j]) who[start + oc[j][w] + pc[j]] = q[j].z;
        if (l_[j]) {
          const uint32_t p = start + ol[j][w] + pl[j];
          who[p] = q[j].z;
          obj[p] = f[j];
        }
      } else {
        if (l_[j]) pairs[start + ol[j][w] + pl[j]] = make_uint2(q[j].w, f[j]);
      }
    }
  }
}

// rep[row] = f for the pairs of every bucket (one 256-thread block per bucket)
__global__ __launch_bounds__(256) void k_pair_scatter(const uint2* __restrict__ pairs,
                                                      const uint32_t* __restrict__ offs,
                                                      const uint32_t* __restrict__ npairs,
                                                      uint32_t* __restrict__ rep) {
  const uint32_t b = blockIdx.x, s = offs[b], c = npairs[b];
  for (uint32_t k = threadIdx.x; k < c; k += 256) {
    const uint2 p = pairs[s + k];
    rep[p.x] = p.y;
  }
}

// AW: the pairs of row window j from every bucket, scattered into rep while
// the window's 3 MB of rep stay in one XCD's L2.  Workgroup b runs on XCD
// b % 8 (round-robin dispatch); the XCD's workgroups take its windows one at
// a time (32 workgroups per window, each a range of buckets: one per thread).
__global__ __launch_bounds__(1024) void k_window_apply(const uint2* __restrict__ pairs,
                                                       const uint32_t* __restrict__ offs,
                                                       const uint32_t* __restrict__ bnd,
                                                       uint32_t nb, uint32_t* __restrict__ rep,
                                                       bool xcd) {
  const uint32_t b = blockIdx.x;
  uint32_t j, part;
  if (xcd) {
    const uint32_t x = b & 7u, t = b >> 3;
    j = x + 8u * (t >> 5);
    part = t & 31u;
  } else {
    j = b >> 5;
    part = b & 31u;
  }
  const uint32_t per = (nb + 31) / 32;
  for (uint32_t bk = part * per + threadIdx.x; bk < min(nb, (part + 1) * per); bk += 1024) {
    const uint64_t e = static_cast<uint64_t>(bk) * (kNW + 1) + j;
    const uint32_t base = offs[bk];
    const uint32_t s = base + bnd[e], t = base + bnd[e + 1];
    for (uint32_t p = s; p < t; ++p) {
      const uint2 pr = pairs[p];
      rep[pr.x] = pr.y;
    }
  }
}

template <typename F>
float time_ms(F f, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  f();
  std::vector<float> v;
  for (int r = 0; r < reps; ++r) {
    (void)hipEventRecord(a, 0);
    f();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    v.push_back(ms);
  }
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

}  // namespace

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 100000000ull;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const GroupLayout L = group_layout(n);
  const uint32_t nb = 1u << L.bits;
  uint64_t* key;
  uint8_t* has;
  uint32_t *rep0, *rep1, *init, *who, *obj, *split, *npairs;
  uint2* pairs;
  (void)hipMalloc(&key, 8 * n);
  (void)hipMalloc(&has, n);
  (void)hipMalloc(&rep0, 4 * n);
  (void)hipMalloc(&rep1, 4 * n);
  (void)hipMalloc(&init, 4 * n);
  (void)hipMalloc(&who, 4 * n);
  (void)hipMalloc(&obj, 4 * n);
  (void)hipMalloc(&pairs, 8 * n);
  (void)hipMalloc(&split, 4 * (nb + 1));
  (void)hipMalloc(&npairs, 4 * (nb + 1));
  uint32_t* bnd;
  (void)hipMalloc(&bnd, 4ull * nb * (kNW + 1));
  const uint32_t win_rows = static_cast<uint32_t>((n + kNW - 1) / kNW);
  k_rows<<<4096, 256>>>(key, has, n, n * 4 / 5);
  void* ws;
  (void)hipMalloc(&ws, L.total);
  uint8_t* w = static_cast<uint8_t*>(ws);
  const uint3* rec = reinterpret_cast<const uint3*>(w + L.rec);
  uint32_t* fbase = reinterpret_cast<uint32_t*>(w + L.fbase);
  const ChunkOf c = ChunkOf::make(100);
  GroupInput gi;
  gi.key = key;
  gi.valid = has;
  gi.n = n;
  // the product's partition + group (records and bucket starts stay in ws)
  (void)dedup_local_launch(gi, 100, rep0, true, ws, 0, nullptr);
  (void)hipDeviceSynchronize();
  std::vector<uint32_t> a(n), b(n), rk(n);
  (void)hipMemcpy(a.data(), rep0, 4 * n, hipMemcpyDeviceToHost);
  for (uint64_t i = 0; i < n; ++i) rk[i] = static_cast<uint32_t>(i);
  (void)hipMemcpy(init, rk.data(), 4 * n, hipMemcpyHostToDevice);
  std::vector<uint32_t> starts(nb + 1);
  (void)hipMemcpy(starts.data(), fbase, 4 * (nb + 1), hipMemcpyDeviceToHost);
  uint32_t mx = 0;
  for (uint32_t i = 0; i < nb; ++i) mx = std::max(mx, starts[i + 1] - starts[i]);
  uint64_t linked = 0;
  for (uint64_t i = 0; i < n; ++i) linked += a[i] != i;
  printf("n %llu buckets %u (bits %u, cbits %u) largest bucket %u, linked rows %llu\n",
         (unsigned long long)n, nb, L.bits, L.cbits, mx, (unsigned long long)linked);
  if (mx > kPkCap) {
    printf("a bucket exceeds the LDS table: experiment needs <= %u\n", kPkCap);
    return 2;
  }
  const uint32_t bits = L.bits;
  auto G = [&](int mode, uint32_t split_row) {
    switch (mode) {
      case kG0:
        k_group_x<kG0><<<nb, kGroupThreads>>>(rec, 0, fbase, bits, c, rep1, who, obj, split, pairs,
                                              npairs, split_row, 0xFFFFFFFEu);
        break;
      case kGN:
        k_group_x<kGN><<<nb, kGroupThreads>>>(rec, 0, fbase, bits, c, rep1, who, obj, split, pairs,
                                              npairs, split_row, 0xFFFFFFFEu);
        break;
      case kGF:
        k_group_x<kGF><<<nb, kGroupThreads>>>(rec, 0, fbase, bits, c, rep1, who, obj, split, pairs,
                                              npairs, split_row, 0xFFFFFFFEu);
        break;
      default:
        k_group_x<kGH><<<nb, kGroupThreads>>>(rec, 0, fbase, bits, c, rep1, who, obj, split, pairs,
                                              npairs, split_row, 0xFFFFFFFEu);
        k_pair_scatter<<<nb, 256>>>(pairs, fbase, npairs, rep1);
    }
  };
  struct V {
    const char* name;
    std::function<void()> f;
    bool check_rep;
  };
  const uint32_t n32 = static_cast<uint32_t>(n);
  std::vector<V> vs = {
      {"G0 product (scattered rep)", [&] { G(kG0, 0); }, true},
      {"GN no output", [&] { G(kGN, 0); }, false},
      {"GF fused who/obj lists", [&] { G(kGF, 0); }, false},
      {"GH split n/2 + pair scatter", [&] { G(kGH, n32 / 2); }, true},
      {"GH split n/3 + pair scatter", [&] { G(kGH, n32 / 3); }, true},
      {"GH split n/4 + pair scatter", [&] { G(kGH, n32 / 4); }, true},
      {"GP all pairs + pair scatter", [&] { G(kGH, 0); }, true},
      {"GW window pairs + L2 window apply",
       [&] {
         k_group_x<kGW><<<nb, kGroupThreads>>>(rec, 0, fbase, bits, c, rep1, who, obj, split, pairs,
                                               npairs, 0, 0xFFFFFFFEu, bnd, win_rows);
         k_window_apply<<<kNW * 32, 1024>>>(pairs, fbase, bnd, nb, rep1, true);
       },
       true},
      {"  GW group only",
       [&] {
         k_group_x<kGW><<<nb, kGroupThreads>>>(rec, 0, fbase, bits, c, rep1, who, obj, split, pairs,
                                               npairs, 0, 0xFFFFFFFEu, bnd, win_rows);
       },
       false},
      {"  AW apply alone (XCD windows)",
       [&] { k_window_apply<<<kNW * 32, 1024>>>(pairs, fbase, bnd, nb, rep1, true); }, false},
      {"  AW apply alone (no XCD mapping)",
       [&] { k_window_apply<<<kNW * 32, 1024>>>(pairs, fbase, bnd, nb, rep1, false); }, false},
      {"  pairs only (GP without scatter)",
       [&] {
         k_group_x<kGH><<<nb, kGroupThreads>>>(rec, 0, fbase, bits, c, rep1, who, obj, split, pairs,
                                               npairs, 0, 0xFFFFFFFEu);
       },
       false},
      {"  pair scatter alone (all pairs)",
       [&] { k_pair_scatter<<<nb, 256>>>(pairs, fbase, npairs, rep1); }, false},
  };
  for (auto& v : vs) {
    if (!v.check_rep) continue;
    (void)hipMemcpy(rep1, init, 4 * n, hipMemcpyDeviceToDevice);
    v.f();
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(b.data(), rep1, 4 * n, hipMemcpyDeviceToHost);
    uint64_t bad = 0;
    for (uint64_t i = 0; i < n; ++i) bad += a[i] != b[i];
    printf("%-36s mismatches vs product: %llu  (%s)\n", v.name, (unsigned long long)bad,
           hipGetErrorString(hipGetLastError()));
  }
  {  // GF: the lists are the product's write set
    G(kGF, 0);
    (void)hipDeviceSynchronize();
    std::vector<uint32_t> hw(n), ho(n), hs(nb);
    (void)hipMemcpy(hw.data(), who, 4 * n, hipMemcpyDeviceToHost);
    (void)hipMemcpy(ho.data(), obj, 4 * n, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hs.data(), split, 4 * nb, hipMemcpyDeviceToHost);
    uint64_t bad = 0, nc = 0, nl = 0;
    std::vector<uint8_t> seen(n, 0);
    for (uint32_t bk = 0; bk < nb; ++bk) {
      for (uint32_t p = starts[bk]; p < starts[bk + 1]; ++p) {
        const uint32_t r = hw[p];
        if (r >= n || seen[r]) {
          ++bad;
          continue;
        }
        seen[r] = 1;
        if (p < hs[bk]) {
          ++nc;
          bad += a[r] != r;
        } else {
          ++nl;
          bad += a[r] != ho[p];
        }
      }
    }
    printf("%-36s creators %llu linked %llu, mismatches vs product reps: %llu\n", "GF lists",
           (unsigned long long)nc, (unsigned long long)nl, (unsigned long long)bad);
  }
  // the coarse pass with and without its rep = rank stores (two-level only)
  uint32_t* run_s = reinterpret_cast<uint32_t*>(w + L.run_s);
  uint32_t* run_l = reinterpret_cast<uint32_t*>(w + L.run_l);
  uint32_t* segtot = reinterpret_cast<uint32_t*>(w + L.segtot);
  uint32_t* fine = reinterpret_cast<uint32_t*>(w + L.fine);
  uint32_t* ovf = reinterpret_cast<uint32_t*>(w + L.ovf);
  uint4* rec1 = reinterpret_cast<uint4*>(w + L.rec1);
  const RowsIn in{key, has, nullptr, 0};
  if (L.cbits) {
    vs.push_back({"P1 coarse pass with rep = rank",
                  [&] {
                    k_zero_runs<<<1, 64>>>(segtot, ovf);
                    k_part_private<RowsIn, true, true><<<kPartBlocks, kPartThreads>>>(
                        in, n, kShardBits, L.cbits, rec1, rep1, L.bits, fine, ovf, run_s, run_l,
                        L.max_rounds, segtot);
                  },
                  false});
    vs.push_back({"P1 coarse pass without rep",
                  [&] {
                    k_zero_runs<<<1, 64>>>(segtot, ovf);
                    k_part_private<RowsIn, false, true><<<kPartBlocks, kPartThreads>>>(
                        in, n, kShardBits, L.cbits, rec1, rep1, L.bits, fine, ovf, run_s, run_l,
                        L.max_rounds, segtot);
                  },
                  false});
  }
  vs.push_back({"whole product grouping",
                [&] { (void)dedup_local_launch(gi, 100, rep0, true, ws, 0, nullptr); }, false});
  for (int r = 0; r < 2; ++r)
    for (auto& v : vs) printf("%-36s %.4f ms\n", v.name, time_ms(v.f, reps));
  return 0;
}
