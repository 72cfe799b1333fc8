// Experiment (not shipped): K5 bucket_group as a persistent kernel that loads
// the NEXT bucket's records while it groups the current one.  Each of the
// 2-per-CU workgroups walks buckets b, b + G, ...; the records of two buckets
// alternate between two register sets (ping-pong, so no register copy waits
// for the loads) and the phase barriers wait for LDS only, so the prefetch
// stays in flight across the table init / CAS inserts / lookups.
//   G0   the product k_bucket_group (one workgroup per bucket)
//   GP4  persistent, <= 4 records per thread in registers (LDS path to 4096 rows)
//   GP5  persistent, <= 5 records per thread (the product's 4608-row LDS cap)
//   GW   one workgroup per bucket; the inserting row stores its rank plainly,
//        only duplicate rows take a ds_min (after a barrier)
//   GR2/GR4  read-ahead probing: read 2 / 4 slots per round, CAS only the
//        first empty-or-equal one (fewer probe rounds, more registers)
//   GD   double hashing instead of linear probing (shorter longest chains)
// On the product's own records: 12.5 M rows (one-level) and 100 M rows (two-level).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_group_persist.hip -o build/exp_group_persist
#include "../../spacedrive_amd/csrc/dedup.hip"

#include <stdio.h>

#include <vector>

using namespace sdgpu;

namespace {

// linear probing, as the product kernel used before round 2's double hashing
__device__ __forceinline__ uint32_t lin_next(uint32_t h) {
  return h + 1 == kLdsSlots ? 0u : h + 1;
}

__global__ void k_rows(uint64_t* key, uint32_t* rank, uint8_t* has, uint64_t n, uint64_t distinct) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint64_t j = (i * 0x9E3779B1ull) % n;
    key[i] = row_hash((j % distinct) * 0x2545F4914F6CDD1Dull + 7);
    rank[i] = static_cast<uint32_t>((i * 0x9E3779B1ull) % n);
    has[i] = (row_hash(i ^ 0x55ull) % 1000) != 0;
  }
}

template <int kP>
__device__ __forceinline__ void load_k(const uint4* __restrict__ rec, uint32_t start, uint32_t end,
                                       uint4 (&q)[kP]) {
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const uint32_t i = start + threadIdx.x + j * kGroupThreads;
    q[j] = i < end ? rec[i] : make_uint4(0, 0, 0, 0);
  }
}

// The product's LDS path with LDS-only barriers.
template <int kP>
__device__ __forceinline__ void group_lds(const uint4 (&q)[kP], uint32_t start, uint32_t end,
                                          ChunkOf chunk_of, uint32_t* __restrict__ rep,
                                          uint64_t* lkey, uint32_t* lmin, uint32_t& special_min) {
  for (uint32_t s = threadIdx.x; s < kLdsSlots; s += kGroupThreads) {
    lkey[s] = kEmpty;
    lmin[s] = 0xFFFFFFFFu;
  }
  if (threadIdx.x == 0) special_min = 0xFFFFFFFFu;
  lds_barrier();
  uint32_t h[kP];
  uint32_t live = 0, pend = 0;
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const uint64_t k = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
    h[j] = lds_slot(k);
    if (start + threadIdx.x + j * kGroupThreads < end) {
      live |= 1u << j;
      if (k == kEmpty)
        atomicMin(&special_min, q[j].z);
      else
        pend |= 1u << j;
    }
  }
  const uint32_t keyed = pend;
  while (pend) {
    uint64_t prev[kP];
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      const uint64_t k = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
      prev[j] = (pend >> j & 1u)
                    ? atomicCAS(reinterpret_cast<unsigned long long*>(&lkey[h[j]]),
                                static_cast<unsigned long long>(kEmpty),
                                static_cast<unsigned long long>(k))
                    : 0ull;
    }
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      if (!(pend >> j & 1u)) continue;
      const uint64_t k = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
      if (prev[j] == kEmpty || prev[j] == k) {
        atomicMin(&lmin[h[j]], q[j].z);
        pend &= ~(1u << j);
      } else {
        h[j] = lin_next(h[j]);
      }
    }
  }
  lds_barrier();
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    if (!(live >> j & 1u)) continue;
    const uint32_t r = q[j].z;
    const uint32_t f = (keyed >> j & 1u) ? lmin[h[j]] : special_min;
    if (chunk_of(r) != chunk_of(f)) rep[q[j].w] = f;
  }
}

template <int kP>
__global__ __launch_bounds__(kGroupThreads, 8) void k_group_persist(
    const uint4* __restrict__ rec, const uint32_t* __restrict__ offs, uint32_t P, uint32_t nb,
    ChunkOf chunk_of, uint64_t* __restrict__ gkey, uint32_t* __restrict__ gmin,
    uint32_t* __restrict__ rep) {
  constexpr uint32_t kCap = kP * kGroupThreads < kLdsCap ? kP * kGroupThreads : kLdsCap;
  __shared__ uint64_t lkey[kLdsSlots];
  __shared__ uint32_t lmin[kLdsSlots];
  __shared__ uint32_t special_min;
  uint32_t b = blockIdx.x;
  if (b >= nb) return;
  uint4 qa[kP], qb[kP];
  uint32_t sa = offs[static_cast<uint64_t>(b) * P], ea = offs[static_cast<uint64_t>(b + 1) * P];
  uint32_t sb = 0, eb = 0;
  if (ea - sa <= kCap) load_k<kP>(rec, sa, ea, qa);
  auto process = [&](const uint4 (&q)[kP], uint32_t s, uint32_t e) {
    if (e - s <= kCap) {
      group_lds<kP>(q, s, e, chunk_of, rep, lkey, lmin, special_min);
    } else {  // the product's global-table path (its own __syncthreads)
      uint4 none[kPer];
      group_bucket(Rec16Src{rec}, s, e, none, chunk_of, gkey, gmin, rep, lkey, lmin, special_min);
    }
    lds_barrier();  // the table is re-initialised for the next bucket
  };
  for (;;) {
    uint32_t bn = b + gridDim.x;
    if (bn < nb) {
      sb = offs[static_cast<uint64_t>(bn) * P];
      eb = offs[static_cast<uint64_t>(bn + 1) * P];
      if (eb - sb <= kCap) load_k<kP>(rec, sb, eb, qb);
    }
    process(qa, sa, ea);
    if (bn >= nb) break;
    b = bn;
    bn = b + gridDim.x;
    if (bn < nb) {
      sa = offs[static_cast<uint64_t>(bn) * P];
      ea = offs[static_cast<uint64_t>(bn + 1) * P];
      if (ea - sa <= kCap) load_k<kP>(rec, sa, ea, qa);
    }
    process(qb, sb, eb);
    if (bn >= nb) break;
    b = bn;
  }
}


// GW: the product kernel, but the row that INSERTS a key stores its rank with a
// plain LDS write; only rows that find their key already present (duplicates,
// ~20 % of config 4) take a ds_min, after a barrier -- ~80 % fewer LDS atomics
// on the min table.
__global__ __launch_bounds__(kGroupThreads, 8) void k_group_winner(
    const uint4* __restrict__ rec, const uint32_t* __restrict__ offs, uint32_t P, ChunkOf chunk_of,
    uint64_t* __restrict__ gkey, uint32_t* __restrict__ gmin, uint32_t* __restrict__ rep) {
  __shared__ uint64_t lkey[kLdsSlots];
  __shared__ uint32_t lmin[kLdsSlots];
  __shared__ uint32_t special_min;
  const uint32_t b = blockIdx.x;
  const uint32_t start = offs[static_cast<uint64_t>(b) * P];
  const uint32_t end = offs[static_cast<uint64_t>(b + 1) * P];
  uint4 q[kPer];
  load_bucket(Rec16Src{rec}, start, end, q);
  if (end - start > kLdsCap) {
    group_bucket(Rec16Src{rec}, start, end, q, chunk_of, gkey, gmin, rep, lkey, lmin, special_min);
    return;
  }
  if (end == start) return;
  for (uint32_t s = threadIdx.x; s < kLdsSlots; s += kGroupThreads) lkey[s] = kEmpty;
  if (threadIdx.x == 0) special_min = 0xFFFFFFFFu;
  __syncthreads();
  uint32_t h[kPer];
  uint32_t live = 0, pend = 0, dup = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const uint64_t k = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
    h[j] = lds_slot(k);
    if (start + threadIdx.x + j * kGroupThreads < end) {
      live |= 1u << j;
      if (k == kEmpty)
        atomicMin(&special_min, q[j].z);
      else
        pend |= 1u << j;
    }
  }
  const uint32_t keyed = pend;
  while (pend) {
    uint64_t prev[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const uint64_t k = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
      prev[j] = (pend >> j & 1u)
                    ? atomicCAS(reinterpret_cast<unsigned long long*>(&lkey[h[j]]),
                                static_cast<unsigned long long>(kEmpty),
                                static_cast<unsigned long long>(k))
                    : 0ull;
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      if (!(pend >> j & 1u)) continue;
      const uint64_t k = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
      if (prev[j] == kEmpty) {  // inserted the key: first rank of the slot
        lmin[h[j]] = q[j].z;
        pend &= ~(1u << j);
      } else if (prev[j] == k) {  // key already there: min after the barrier
        dup |= 1u << j;
        pend &= ~(1u << j);
      } else {
        h[j] = lin_next(h[j]);
      }
    }
  }
  __syncthreads();
  if (__ballot(dup != 0)) {
#pragma unroll
    for (int j = 0; j < kPer; ++j)
      if (dup >> j & 1u) atomicMin(&lmin[h[j]], q[j].z);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    if (!(live >> j & 1u)) continue;
    const uint32_t r = q[j].z;
    const uint32_t f = (keyed >> j & 1u) ? lmin[h[j]] : special_min;
    if (chunk_of(r) != chunk_of(f)) rep[q[j].w] = f;
  }
}


// GR: the product kernel with read-ahead probing: each round a pending record
// first READS kLook consecutive slots from its probe position (plain ds_read,
// independent, issued together), picks the first that is empty or holds its
// key, and only then issues the CAS there; a lost race continues from that
// slot.  Linear probing's invariant is unchanged (a CAS only fills an empty
// slot), but one round now covers kLook slots instead of one.
template <int kLook>
__global__ __launch_bounds__(kGroupThreads, 8) void k_group_lookahead(
    const uint4* __restrict__ rec, const uint32_t* __restrict__ offs, uint32_t P, ChunkOf chunk_of,
    uint64_t* __restrict__ gkey, uint32_t* __restrict__ gmin, uint32_t* __restrict__ rep) {
  __shared__ uint64_t lkey[kLdsSlots];
  __shared__ uint32_t lmin[kLdsSlots];
  __shared__ uint32_t special_min;
  const uint32_t b = blockIdx.x;
  const uint32_t start = offs[static_cast<uint64_t>(b) * P];
  const uint32_t end = offs[static_cast<uint64_t>(b + 1) * P];
  uint4 q[kPer];
  load_bucket(Rec16Src{rec}, start, end, q);
  if (end - start > kLdsCap) {
    group_bucket(Rec16Src{rec}, start, end, q, chunk_of, gkey, gmin, rep, lkey, lmin, special_min);
    return;
  }
  if (end == start) return;
  for (uint32_t s = threadIdx.x; s < kLdsSlots; s += kGroupThreads) {
    lkey[s] = kEmpty;
    lmin[s] = 0xFFFFFFFFu;
  }
  if (threadIdx.x == 0) special_min = 0xFFFFFFFFu;
  __syncthreads();
  uint32_t h[kPer];
  uint32_t live = 0, pend = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const uint64_t k = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
    h[j] = lds_slot(k);
    if (start + threadIdx.x + j * kGroupThreads < end) {
      live |= 1u << j;
      if (k == kEmpty)
        atomicMin(&special_min, q[j].z);
      else
        pend |= 1u << j;
    }
  }
  const uint32_t keyed = pend;
  while (pend) {
    // read-ahead: kLook slots per pending record
    uint64_t look[kPer][kLook];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      if (!(pend >> j & 1u)) continue;
      uint32_t s = h[j];
#pragma unroll
      for (int t = 0; t < kLook; ++t) {
        look[j][t] = lkey[s];
        s = lin_next(s);
      }
    }
    uint64_t prev[kPer];
    uint32_t skip = 0;  // records whose kLook slots all hold other keys
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      prev[j] = 0;
      if (!(pend >> j & 1u)) continue;
      const uint64_t k = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
      // first slot (of the kLook read) that is empty or holds k; else the last
      int t0 = kLook;
#pragma unroll
      for (int t = kLook - 1; t >= 0; --t)
        if (look[j][t] == kEmpty || look[j][t] == k) t0 = t;
      if (t0 == kLook) {  // all kLook slots hold other keys: skip past them
#pragma unroll
        for (int t = 0; t < kLook; ++t) h[j] = lin_next(h[j]);
        skip |= 1u << j;
        continue;
      }
#pragma unroll
      for (int t = 0; t < kLook; ++t)
        if (t < t0) h[j] = lin_next(h[j]);
      if (look[j][t0] == k) {
        prev[j] = k;  // already there: no CAS needed
      } else {
        prev[j] = atomicCAS(reinterpret_cast<unsigned long long*>(&lkey[h[j]]),
                            static_cast<unsigned long long>(kEmpty),
                            static_cast<unsigned long long>(k));
      }
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      if (!(pend >> j & 1u) || (skip >> j & 1u)) continue;
      const uint64_t k = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
      if (prev[j] == kEmpty || prev[j] == k) {
        atomicMin(&lmin[h[j]], q[j].z);
        pend &= ~(1u << j);
      } else {
        h[j] = lin_next(h[j]);
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    if (!(live >> j & 1u)) continue;
    const uint32_t r = q[j].z;
    const uint32_t f = (keyed >> j & 1u) ? lmin[h[j]] : special_min;
    if (chunk_of(r) != chunk_of(f)) rep[q[j].w] = f;
  }
}


// GD: the product kernel with double hashing in place of linear probing: a
// record's probe step is 1 + 6 * ((h >> 40) % 1024) (coprime with the 6144
// slots), so probe sequences of different keys no longer run in clusters and
// a wave's longest probe chain -- the number of CAS rounds it makes -- shrinks.
__global__ __launch_bounds__(kGroupThreads, 8) void k_group_double(
    const uint4* __restrict__ rec, const uint32_t* __restrict__ offs, uint32_t P, ChunkOf chunk_of,
    uint64_t* __restrict__ gkey, uint32_t* __restrict__ gmin, uint32_t* __restrict__ rep,
    uint32_t* __restrict__ rounds_max) {
  __shared__ uint64_t lkey[kLdsSlots];
  __shared__ uint32_t lmin[kLdsSlots];
  __shared__ uint32_t special_min;
  const uint32_t b = blockIdx.x;
  const uint32_t start = offs[static_cast<uint64_t>(b) * P];
  const uint32_t end = offs[static_cast<uint64_t>(b + 1) * P];
  uint4 q[kPer];
  load_bucket(Rec16Src{rec}, start, end, q);
  if (end - start > kLdsCap) {
    group_bucket(Rec16Src{rec}, start, end, q, chunk_of, gkey, gmin, rep, lkey, lmin, special_min);
    return;
  }
  if (end == start) return;
  for (uint32_t s = threadIdx.x; s < kLdsSlots; s += kGroupThreads) {
    lkey[s] = kEmpty;
    lmin[s] = 0xFFFFFFFFu;
  }
  if (threadIdx.x == 0) special_min = 0xFFFFFFFFu;
  __syncthreads();
  uint32_t h[kPer], step[kPer];
  uint32_t live = 0, pend = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const uint64_t k = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
    h[j] = lds_slot(k);
    step[j] = 1u + 6u * static_cast<uint32_t>((k >> 40) & 1023u);
    if (start + threadIdx.x + j * kGroupThreads < end) {
      live |= 1u << j;
      if (k == kEmpty)
        atomicMin(&special_min, q[j].z);
      else
        pend |= 1u << j;
    }
  }
  const uint32_t keyed = pend;
  uint32_t rounds = 0;
  while (pend) {
    ++rounds;
    uint64_t prev[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const uint64_t k = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
      prev[j] = (pend >> j & 1u)
                    ? atomicCAS(reinterpret_cast<unsigned long long*>(&lkey[h[j]]),
                                static_cast<unsigned long long>(kEmpty),
                                static_cast<unsigned long long>(k))
                    : 0ull;
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      if (!(pend >> j & 1u)) continue;
      const uint64_t k = (static_cast<uint64_t>(q[j].y) << 32) | q[j].x;
      if (prev[j] == kEmpty || prev[j] == k) {
        atomicMin(&lmin[h[j]], q[j].z);
        pend &= ~(1u << j);
      } else {
        const uint32_t s = h[j] + step[j];
        h[j] = s >= kLdsSlots ? s - kLdsSlots : s;
      }
    }
  }
  if (rounds_max) atomicMax(rounds_max, rounds);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    if (!(live >> j & 1u)) continue;
    const uint32_t r = q[j].z;
    const uint32_t f = (keyed >> j & 1u) ? lmin[h[j]] : special_min;
    if (chunk_of(r) != chunk_of(f)) rep[q[j].w] = f;
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

uint64_t mismatches(const uint32_t* a_d, const uint32_t* b_d, uint64_t n) {
  std::vector<uint32_t> a(n), b(n);
  (void)hipMemcpy(a.data(), a_d, 4 * n, hipMemcpyDeviceToHost);
  (void)hipMemcpy(b.data(), b_d, 4 * n, hipMemcpyDeviceToHost);
  uint64_t bad = 0;
  for (uint64_t i = 0; i < n; ++i) bad += a[i] != b[i];
  return bad;
}

void run(uint64_t n) {
  uint64_t* key;
  uint32_t *rank, *rep, *rep2;
  uint8_t* has;
  (void)hipMalloc(&key, 8 * n);
  (void)hipMalloc(&rank, 4 * n);
  (void)hipMalloc(&has, n);
  (void)hipMalloc(&rep, 4 * n);
  (void)hipMalloc(&rep2, 4 * n);
  k_rows<<<4096, 256>>>(key, rank, has, n, n * 4 / 5);
  const GroupLayout L = group_layout(n);
  void* ws;
  (void)hipMalloc(&ws, L.total);
  GroupInput in;
  in.key = key;
  in.rank = rank;
  in.valid = has;
  in.n = n;
  (void)dedup_local_launch(in, 100, rep, true, ws, 0, nullptr);
  (void)hipDeviceSynchronize();
  uint8_t* w = static_cast<uint8_t*>(ws);
  const uint4* rec = reinterpret_cast<const uint4*>(w + L.rec);
  // bucket starts: the fine-count paths (12-bit one-level, two-level) publish
  // them with stride 1; narrower one-level partitions use the digit-major scan
  const bool fine = L.cbits || L.bits == kStageBits;
  const uint32_t* offs = reinterpret_cast<const uint32_t*>(w + (fine ? L.fbase : L.hist));
  const uint32_t P = fine ? 1u : kPartBlocks, nb = 1u << L.bits;
  uint64_t* gkey = reinterpret_cast<uint64_t*>(w + L.gkey);
  uint32_t* gmin = reinterpret_cast<uint32_t*>(w + L.gmin);
  const ChunkOf c = ChunkOf::make(100);
  const uint32_t G = 2 * 256;
  printf("n %llu buckets %u\n", (unsigned long long)n, nb);
  auto g0 = [&] { k_bucket_group<<<nb, kGroupThreads>>>(rec, offs, P, c, gkey, gmin, rep2); };
  auto gp4 = [&] { k_group_persist<4><<<std::min(G, nb), kGroupThreads>>>(rec, offs, P, nb, c, gkey, gmin, rep2); };
  auto gp5 = [&] { k_group_persist<5><<<std::min(G, nb), kGroupThreads>>>(rec, offs, P, nb, c, gkey, gmin, rep2); };
  auto gw = [&] { k_group_winner<<<nb, kGroupThreads>>>(rec, offs, P, c, gkey, gmin, rep2); };
  auto gr2 = [&] { k_group_lookahead<2><<<nb, kGroupThreads>>>(rec, offs, P, c, gkey, gmin, rep2); };
  auto gr4 = [&] { k_group_lookahead<4><<<nb, kGroupThreads>>>(rec, offs, P, c, gkey, gmin, rep2); };
  auto gd = [&] { k_group_double<<<nb, kGroupThreads>>>(rec, offs, P, c, gkey, gmin, rep2, nullptr); };
  for (int v = 0; v < 7; ++v) {
    (void)hipMemcpy(rep2, rank, 4 * n, hipMemcpyDeviceToDevice);  // rows keep their rank
    // (keyless rows: rank; the product's init_rep wrote rank for every row)
    if (v == 0) g0();
    else if (v == 1) gp4();
    else if (v == 2) gp5();
    else if (v == 3) gw();
    else if (v == 4) gr2();
    else if (v == 5) gr4();
    else gd();
    (void)hipDeviceSynchronize();
    printf("%s mismatches vs product grouping: %llu\n", v == 0 ? "G0 " : v == 1 ? "GP4" : v == 2 ? "GP5" : v == 3 ? "GW " : v == 4 ? "GR2" : v == 5 ? "GR4" : "GD ",
           (unsigned long long)mismatches(rep, rep2, n));
  }
  for (int r = 0; r < 2; ++r) {
    printf("G0  product group        %.4f ms\n", time_ms(g0, 9));
    printf("GP4 persistent 4/thread  %.4f ms\n", time_ms(gp4, 9));
    printf("GP5 persistent 5/thread  %.4f ms\n", time_ms(gp5, 9));
    printf("GW  winner-store         %.4f ms\n", time_ms(gw, 9));
    printf("GR2 read-ahead 2 slots   %.4f ms\n", time_ms(gr2, 9));
    printf("GR4 read-ahead 4 slots   %.4f ms\n", time_ms(gr4, 9));
    printf("GD  double hashing       %.4f ms\n", time_ms(gd, 9));
  }
  {  // longest probe chain (CAS rounds of a thread) with double hashing
    uint32_t* rm;
    (void)hipMalloc(&rm, 4);
    (void)hipMemset(rm, 0, 4);
    k_group_double<<<nb, kGroupThreads>>>(rec, offs, P, c, gkey, gmin, rep2, rm);
    uint32_t h_rm = 0;
    (void)hipMemcpy(&h_rm, rm, 4, hipMemcpyDeviceToHost);
    printf("GD  max CAS rounds of a thread: %u\n", h_rm);
    (void)hipFree(rm);
  }
  (void)hipFree(ws);
  (void)hipFree(key);
  (void)hipFree(rank);
  (void)hipFree(has);
  (void)hipFree(rep);
  (void)hipFree(rep2);
}

}  // namespace

int main() {
  run(12500000ull);
  run(100000000ull);
  return 0;
}
