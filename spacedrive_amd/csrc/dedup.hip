// K4-K6: cas_id -> Object grouping as a radix partition + per-bucket group-by.
//
// Replaces the Object link/create decisions of identifier_job_step
// (/root/reference/core/src/object/file_identifier/mod.rs:136-333): the
// HashSet of chunk cas_ids (:136-141), the per-row `find` of an Object owning
// the same cas_id (:196-206) and the one-new-Object-per-remaining-row rule
// (:233-297), evaluated for ALL rows of a batch at once instead of 100 per job
// step.  The library-wide find_many over file_path.cas_id (:168-175), i.e.
// Objects that already exist before the batch, is the Object index of
// index.hip, consulted before this grouping (sdgpu_group_rows_indexed_device).
//
// Rows are (key, rank): key = the cas_id's 8 digest bytes as a little-endian
// u64, rank = position of the file_path in ascending-id order.  The grouping
// rule (canonical form):
//   f      = lowest rank carrying key k
//   rep(r) = r  if r / chunk_rows == f / chunk_rows   (new Object in f's chunk)
//            f  otherwise                               (linked to f's Object)
//
// Digits come from h = mix64(key) (splitmix64 finalizer), not from the raw key
// bits: the shard of the multi-GPU exchange is h's top 8 bits, a bucket is the
// `bits` hash bits below them, and the LDS slot uses h's low 32 bits.  Buckets
// are therefore balanced for any key distribution and any world size (raw key
// bits left half the buckets empty at 3 ranks), and the three are independent.
// mix64 is a bijection of u64, so the bucket records carry h itself in place of
// the key: the group-by compares hashes (equal iff the keys are) and never
// recomputes one.
//
// Pipeline (all asynchronous, no host synchronisation):
//   K6 partition: digit = `bits` hash bits below the top `skip` bits.
//      hist:    each of P blocks histograms its contiguous tile in LDS and
//               writes its counts (no global atomics): block-major rows for
//               the 12-bit bucket partition, digit-major elsewhere;
//      offsets: k_fine_scan (block-major: every block's start inside every
//               bucket, one launch; bucket starts scanned in the scatter's
//               prologue) or scan::exclusive (digit-major);
//      scatter: each block re-reads its tile and scatters its rows through LDS
//               cursors (16-B bucket records, or the exchange's send layout).
//      Used by shard (multi-GPU exchange) and by bucket; past 2^12 buckets the
//      bucket partition takes two passes, the coarse one counting every row's
//      final bucket for the second (group_layout).
//   K5 group:   one workgroup per bucket builds a linear-probing hash table of
//               (key -> min rank) in LDS (ds_cmpst_b64 / ds_min_u32), then maps
//               every row to its rep.  Buckets too large for LDS use a private
//               region of a global table instead (same code path, agent-scope
//               atomics), so any key distribution (e.g. one file duplicated a
//               million times) is handled.
#include <errno.h>

#include "internal.hpp"
#include "rows_device.hpp"
#include "scan_device.hpp"

#include <algorithm>
#include <type_traits>
#include <cstdlib>

namespace sdgpu {

namespace {

constexpr int kPartThreads = 1024;
constexpr uint32_t kPartBlocks = 256;  // one per CU
constexpr uint32_t kMaxPartBlocks = 1024;  // bucket partition: sizes the workspace
constexpr int kGroupThreads = 1024;
// 6144 slots x 12 B = 72 KiB of LDS, so two buckets share a CU (8 waves/SIMD)
// and one bucket's loads overlap the other's LDS atomics.  The slot count is
// not a power of two: slots are indexed by the high half of hash * tsize.
constexpr uint32_t kLdsSlots = 6144;
constexpr uint32_t kLdsCap = 4608;     // rows per bucket handled in LDS (load <= 75%)
constexpr uint64_t kBucketRows = 3072; // target mean rows per bucket (bucket_bits_for)
constexpr uint32_t kMaxBucketBits = 15;  // 2^15 buckets: 100 M rows stay in LDS
constexpr uint32_t kShardBits = 8;       // multi-GPU shards: h >> 56
constexpr uint64_t kEmpty = ~0ull;
constexpr uint32_t kPadRow = 0xFFFFFFFFu;  // a record's row field: padding, not a row

// `bits` hash bits below the top `skip` bits of h.
__device__ __forceinline__ uint32_t digit_of(uint64_t h, uint32_t skip, uint32_t bits) {
  return bits == 0 ? 0u : static_cast<uint32_t>((h << skip) >> (64u - bits));
}

// XCD-aware block numbering: workgroups are dispatched round-robin over the 8
// XCDs, so physical block i runs on XCD i % 8.  Logical block (i % 8) * P/8 +
// i / 8 gives each XCD a contiguous run of logical blocks; the 16 per-block
// counters of one digit that share a 64-B line of the digit-major histogram
// (and the offsets the scatter reads back) then come from one XCD's L2.
__device__ __forceinline__ uint32_t part_block() {
  const uint32_t P = gridDim.x;
  return (P & 7u) ? blockIdx.x : (blockIdx.x & 7u) * (P >> 3) + (blockIdx.x >> 3);
}

__device__ __forceinline__ void tile_of(uint64_t n, uint32_t P, uint64_t& t0, uint64_t& t1) {
  const uint64_t per = (n + P - 1) / P;
  t0 = min<uint64_t>(n, per * part_block());
  t1 = min<uint64_t>(n, t0 + per);
}

// Rows per thread per step of the partition kernels: the loads of a step are
// issued back to back, so one tile costs a few memory latencies, not one per row.
constexpr int kUnroll = 8;

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS
// operations, not for its global loads and stores (__syncthreads' release
// fence waits for all of them: vmcnt(0) before every round barrier).  The
// "memory" clobber keeps the compiler from moving memory accesses across it.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Partition digit of a row hash: the destination rank of the multi-GPU
// exchange when world != 0 (shard s = top `bits` hash bits belongs to rank
// s * world >> bits), else `bits` hash bits below the top `skip` bits.
__device__ __forceinline__ uint32_t part_digit(uint64_t h, uint32_t skip, uint32_t bits,
                                               uint32_t world) {
  return world ? static_cast<uint32_t>(((h >> (64 - bits)) * world) >> bits)
               : digit_of(h, skip, bits);
}

// Wave-aggregated LDS counter add for few, heavily shared bins (the exchange's
// W destination ranks): one atomic per distinct digit in the wave instead of
// one per row.  Every active lane of the wave must call it (v = row counts;
// digits d < 2^nbits); returns the row's slot (base of its bin + its rank
// among the wave's lanes with the same digit).  The lanes sharing a digit
// come from nbits ballots, one per digit bit, and the groups' atomics issue
// together (round 5: a loop over the distinct digits took up to W dependent
// atomic round trips per row step).
__device__ __forceinline__ uint32_t wave_add(uint32_t* cnt, uint32_t d, bool v, uint32_t nbits) {
  const uint32_t lane = __lane_id();
  uint64_t peers = __ballot(v);
  for (uint32_t k = 0; k < nbits; ++k) {  // wave-uniform
    const bool bit = (d >> k) & 1u;
    const uint64_t mk = __ballot(bit);
    peers &= bit ? mk : ~mk;
  }
  const uint32_t rank = static_cast<uint32_t>(__popcll(peers & ((1ull << lane) - 1ull)));
  uint32_t base = 0;
  if (v && rank == 0) base = atomicAdd(&cnt[d], static_cast<uint32_t>(__popcll(peers)));
  const int leader = __ffsll(static_cast<unsigned long long>(peers)) - 1;
  base = __shfl(base, v ? leader : static_cast<int>(lane));
  return v ? base + rank : 0u;
}
// digit bits of bins 0 .. world - 1
__device__ __forceinline__ uint32_t world_bits(uint32_t world) {
  return world > 1 ? 32u - static_cast<uint32_t>(__clz(world - 1)) : 0u;
}

// The valid keyless rows of a fused grouping call (ListOut without an Object
// index; mod.rs:238-239: each is its own Object), collected by the FIRST
// partition pass that already reads every row's has_key.  Each WAVE appends the
// ranks of its keyless rows with valid[i] != 0 (valid null: all) to its own
// segment st[(block * 16 + wave) * cap, ...), counting them in a register (a
// ballot per test, no LDS atomic and no barrier), and stores the count in
// cnt[block * 16 + wave]; k_list_finish moves them behind the keyed entries.
// This replaced a separate pass over has_key / valid (three launches, 0.062 ms
// at 100 M rows, 0.017 ms at 12.5 M).
constexpr uint32_t kSinkWaves = kPartThreads / 64;
struct XSink {
  const uint8_t* valid = nullptr;
  uint32_t* st = nullptr;  // null: no sink
  uint32_t* cnt = nullptr;
  uint32_t cap = 0;        // rows per wave segment (>= the rows a wave reads)
};

// Called by every lane of a wave that is still in the partition's row loop
// (the lanes that left it never return to it, so the active lanes' `wn`
// agree, and lane 0 -- the last to leave -- holds the wave's count);
// `keyless`: row i is in range with has_key == 0.  kImplicit: in.rank is
// null (rank = rank_base + row; no load).  Segment offsets fit 32 bits (n <
// 2^31, 16 x 256 segments of a 16th of a tile + 520 rows).
template <bool kImplicit = false>
__device__ __forceinline__ void sink_keyless(const XSink& x, const RowsIn& in, bool keyless,
                                             uint64_t i, uint32_t& wn) {
  const bool e = keyless && (!x.valid || x.valid[i] != 0);
  const uint64_t b = __ballot(e);
  if (!b) return;
  if (e) {
    const uint32_t seg = part_block() * kSinkWaves + (threadIdx.x >> 6);
    const uint32_t r = in.rank_base + static_cast<uint32_t>(i);
    x.st[seg * x.cap + wn + __popcll(b & ((1ull << __lane_id()) - 1ull))] =
        kImplicit ? r : (in.rank ? in.rank[i] : r);
  }
  wn += static_cast<uint32_t>(__popcll(b));
}
__device__ __forceinline__ void sink_count(const XSink& x, uint32_t wn) {
  if (__lane_id() == 0) x.cnt[part_block() * kSinkWaves + (threadIdx.x >> 6)] = wn;
}

template <typename In, bool kX = false>
__global__ __launch_bounds__(kPartThreads) void k_part_hist(In in, uint64_t n, uint32_t skip,
                                                            uint32_t bits, uint32_t world,
                                                            uint32_t* __restrict__ hist,
                                                            uint32_t* __restrict__ zero = nullptr,
                                                            bool blk_major = false,
                                                            XSink xs = XSink{}) {
  extern __shared__ __attribute__((aligned(16))) uint32_t cnt[];
  uint32_t wn = 0;  // the wave's keyless rows (XSink)
  const uint32_t nbins = world ? world : 1u << bits;
  if (zero && blockIdx.x == 0 && threadIdx.x == 0) *zero = 0;  // a flag of the next kernels
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads) cnt[b] = 0;
  __syncthreads();
  auto sink_done = [&]() {
    if constexpr (kX) sink_count(xs, wn);
  };
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  if constexpr (std::is_same<In, RowsIn>::value) {
    // Row order does not matter to a histogram: the keys of row pairs as one
    // 16-B load per lane (8-B loads run at ~0.6x the 16-B rate), has_key as
    // one 2-B load; the odd rows at the tile's ends one by one.
    if (!world && (reinterpret_cast<uintptr_t>(in.key) & 15u) == 0 &&
        (reinterpret_cast<uintptr_t>(in.valid) & 1u) == 0) {
      auto count = [&](uint64_t k, bool v) {
        if (v) atomicAdd(&cnt[part_digit(row_hash(k), skip, bits, 0)], 1u);
      };
      const uint64_t p0 = (t0 + 1) / 2, p1 = t1 / 2;  // whole pairs: rows [2 p0, 2 p1)
      const bool e0 = (t0 & 1u) && t0 < t1, e1 = (t1 & 1u) && t1 - 1 >= 2 * p0;
      if (threadIdx.x == 0 && e0) count(in.key[t0], !in.valid || in.valid[t0]);
      if (threadIdx.x == 1 && e1) count(in.key[t1 - 1], !in.valid || in.valid[t1 - 1]);
      if constexpr (kX) {
        if (threadIdx.x < 64) {  // the whole wave 0 (its ballots)
          sink_keyless(xs, in, threadIdx.x == 0 && e0 && !in.valid[t0], t0, wn);
          sink_keyless(xs, in, threadIdx.x == 1 && e1 && !in.valid[t1 - 1], t1 - 1, wn);
        }
      }
      const uint4* __restrict__ k4 = reinterpret_cast<const uint4*>(in.key);
      const uint16_t* __restrict__ v2 = reinterpret_cast<const uint16_t*>(in.valid);
      constexpr int kP = kUnroll / 2;
      for (uint64_t q0 = p0 + threadIdx.x; q0 < p1; q0 += kP * kPartThreads) {
        uint4 kk[kP];
        uint32_t vv[kP];
#pragma unroll
        for (int u = 0; u < kP; ++u) {
          const uint64_t q = q0 + static_cast<uint64_t>(u) * kPartThreads;
          kk[u] = k4[q < p1 ? q : q0];
          vv[u] = v2 ? v2[q < p1 ? q : q0] : 0x0101u;
        }
#pragma unroll
        for (int u = 0; u < kP; ++u) {
          const uint64_t q = q0 + static_cast<uint64_t>(u) * kPartThreads;
          if (q >= p1) continue;
          count((static_cast<uint64_t>(kk[u].y) << 32) | kk[u].x, (vv[u] & 0xFFu) != 0);
          count((static_cast<uint64_t>(kk[u].w) << 32) | kk[u].z, (vv[u] >> 8) != 0);
        }
        if constexpr (kX) {  // keyless rows are rare: bit 2 u + h = row 2 q_u + h
          uint32_t km = 0;
#pragma unroll
          for (int u = 0; u < kP; ++u)
            if (q0 + static_cast<uint64_t>(u) * kPartThreads < p1)
              km |= (static_cast<uint32_t>((vv[u] & 0xFFu) == 0) |
                     (static_cast<uint32_t>((vv[u] & 0xFF00u) == 0) << 1)) << (2 * u);
          // one pass per bit position some lane has (usually none, else one)
          for (uint64_t b = __ballot(km != 0); b; b = __ballot(km != 0)) {
            const uint32_t p = __ffs(__shfl(km, __ffsll(static_cast<unsigned long long>(b)) - 1)) - 1;
            const uint64_t q = q0 + static_cast<uint64_t>(p >> 1) * kPartThreads;
            sink_keyless(xs, in, (km >> p) & 1u, 2 * q + (p & 1u), wn);
            km &= ~(1u << p);
          }
        }
      }
      __syncthreads();
      for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads)
        hist[blk_major ? static_cast<uint64_t>(part_block()) * nbins + b
                       : static_cast<uint64_t>(b) * gridDim.x + part_block()] = cnt[b];
      sink_done();
      return;
    }
  }
  for (uint64_t i0 = t0 + threadIdx.x; i0 < t1; i0 += kUnroll * kPartThreads) {
    RowBatch<kUnroll> q;
    in.template load_many<kUnroll>(i0, kPartThreads, t1, i0, q);
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const bool v = in.valid_of(q, u);
      const uint64_t k = in.key_of(q, u);
      if constexpr (kX) sink_keyless(xs, in, q.in[u] && !v, q.row[u], wn);
      if (world) {
        (void)wave_add(cnt, v ? part_digit(in_hash<In>(k), skip, bits, world) : 0u, v, world_bits(world));
      } else if (v) {
        atomicAdd(&cnt[part_digit(in_hash<In>(k), skip, bits, world)], 1u);
      }
    }
  }
  __syncthreads();
  // digit-major [digit][block] for scan::exclusive, or block-major (one
  // coalesced row per block) for k_fine_scan
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads)
    hist[blk_major ? static_cast<uint64_t>(part_block()) * nbins + b
                   : static_cast<uint64_t>(b) * gridDim.x + part_block()] = cnt[b];
  sink_done();
}

// Shard partition of the multi-GPU exchange: keyed rows packed by digit (the
// destination rank, or a shard) at the scanned offsets.
//   kRec12: one packed 12-byte send record {key lo, key hi, rank} per row
//           (what travels over xGMI) and, per SOURCE row i, out_pos[i] = its
//           send position (~0 for keyless rows): a coalesced write, and the
//           reps come back through a gather (k_gather_rep);
//   else:   separate key / rank arrays and out_pos[p] = source row of packed
//           row p (the single-step ABI for hosts with their own collectives).
// kRec12 with out_pos null: the write-set form, which needs no send
// positions (no rep comes back).
template <typename In, bool kRec12>
__global__ __launch_bounds__(kPartThreads) void k_part_scatter(
    In in, uint64_t n, uint32_t skip, uint32_t bits, uint32_t world,
    const uint32_t* __restrict__ offs, uint64_t* __restrict__ out_key,
    uint32_t* __restrict__ out_rank, uint3* __restrict__ out_rec, uint32_t* __restrict__ out_pos) {
  extern __shared__ __attribute__((aligned(16))) uint32_t cur[];
  const uint32_t nbins = world ? world : 1u << bits;
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads)
    cur[b] = offs[static_cast<uint64_t>(b) * gridDim.x + part_block()];
  __syncthreads();
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  constexpr int U = kUnroll / 2;
  for (uint64_t i0 = t0 + threadIdx.x; i0 < t1; i0 += U * kPartThreads) {
    RowBatch<U> q;
    in.template load_many<U>(i0, kPartThreads, t1, i0, q);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = i0 + static_cast<uint64_t>(u) * kPartThreads;
      const bool v = in.valid_of(q, u);
      const uint64_t k = in.key_of(q, u);
      const uint32_t d = v ? part_digit(in_hash<In>(k), skip, bits, world) : 0u;
      const uint32_t p = world ? wave_add(cur, d, v, world_bits(world)) : (v ? atomicAdd(&cur[d], 1u) : 0u);
      if (!v) {
        if (kRec12 && q.in[u] && out_pos) out_pos[i] = 0xFFFFFFFFu;
        continue;
      }
      const uint32_t r = in.rank_of(q, u);
      if (kRec12) {
        out_rec[p] = make_uint3(static_cast<uint32_t>(k), static_cast<uint32_t>(k >> 32), r);
        if (out_pos) out_pos[i] = p;
      } else {
        out_key[p] = k;
        out_rank[p] = r;
        out_pos[p] = static_cast<uint32_t>(i);
      }
    }
  }
}

// Padded exchange partition (round 5; shard.cpp padded exchange): ONE pass
// over the caller's rows, no histogram or scan.  Each round of kPadR rows a
// block counting-sorts its keyed rows by owner in LDS, reserves each owner's
// run inside that owner's fixed-capacity message with ONE global atomic per
// owner (cursor[d], zeroed before the launch), and copies the runs out
// coalesced.  Message d = slots d * (cap + 1) .. of the send buffer (slot 0
// its header, k_pad_fill); the message to this rank itself (d == me) is
// written straight into the receive buffer (self_out, same slots): no copy.
// The order of the rows inside a message follows the reservations, not row
// order -- the grouping reads ranks, not positions.  Slots past cap are not
// written (cursor[d] > cap: k_pad_fill raises the overflow bit).  out_pos
// (rep form; null for the write set): the send slot of row i, ~0 for keyless
// or unsent rows.  xs (the write set): the valid keyless rows are collected
// into the XSink segments on the way (as the fused call's first pass does),
// for the owner's k_list_finish -- no extra-entry pass.  Round r + 1's rows
// are loaded before round r's atomics.
constexpr int kPadU = 4;
constexpr uint32_t kPadR = kPadU * kPartThreads;
constexpr uint32_t kXShardBitsDev = 8;  // shard = top 8 hash bits (shard.cpp kXShardBits)
__global__ __launch_bounds__(kPartThreads) void k_part_padded(
    RowsIn in, uint64_t n, uint32_t world, uint32_t me, uint32_t cap, uint3* __restrict__ out,
    uint3* __restrict__ self_out, uint32_t* __restrict__ out_pos,
    uint32_t* __restrict__ cursor, XSink xs) {
  __shared__ uint3 buf[kPadR];
  __shared__ uint32_t cnt[kMaxWorld], lb[kMaxWorld + 1], gb[kMaxWorld];
  const uint64_t c1 = cap + 1ull;
  uint32_t wn = 0;  // the wave's keyless rows (XSink)
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  auto round = [&](const RowBatch<kPadU>& q, uint64_t i0) {
    if (threadIdx.x < world) cnt[threadIdx.x] = 0;
    lds_barrier();
    uint32_t dg[kPadU], lr[kPadU];
#pragma unroll
    for (int u = 0; u < kPadU; ++u) {
      const bool v = in.valid_of(q, u);
      const uint32_t d = v ? part_digit(row_hash(in.key_of(q, u)), 0, kXShardBitsDev, world) : 0u;
      lr[u] = wave_add(cnt, d, v, world_bits(world));
      dg[u] = v ? d : ~0u;
      if (xs.st)  // uniform; a ballot, and a store only for the rare valid keyless row
        sink_keyless(xs, in, q.in[u] && !v, i0 + threadIdx.x + static_cast<uint64_t>(u) * kPartThreads,
                     wn);
    }
    lds_barrier();
    if (threadIdx.x < 64) {  // one wave: the round's run starts and the reservations
      const uint32_t lane = threadIdx.x;
      const uint32_t c = lane < world ? cnt[lane] : 0u;
      uint32_t inc = c;
#pragma unroll
      for (int s = 1; s < 64; s <<= 1) {
        const uint32_t o = __shfl_up(inc, s);
        if (lane >= static_cast<uint32_t>(s)) inc += o;
      }
      if (lane < world) lb[lane] = inc - c;
      if (lane == world - 1) lb[world] = inc;
      if (lane < world && c) gb[lane] = atomicAdd(&cursor[lane], c);
    }
    lds_barrier();
#pragma unroll
    for (int u = 0; u < kPadU; ++u) {
      const uint64_t i = i0 + threadIdx.x + static_cast<uint64_t>(u) * kPartThreads;
      if (dg[u] == ~0u) {
        if (out_pos && q.in[u]) out_pos[i] = 0xFFFFFFFFu;
        continue;
      }
      const uint32_t d = dg[u];
      const uint64_t k = in.key_of(q, u);
      buf[lb[d] + lr[u]] = make_uint3(static_cast<uint32_t>(k), static_cast<uint32_t>(k >> 32),
                                      in.rank_of(q, u));
      if (out_pos) {
        const uint32_t pos = gb[d] + lr[u];
        out_pos[i] = pos < cap ? static_cast<uint32_t>(d * c1 + 1 + pos) : 0xFFFFFFFFu;
      }
    }
    lds_barrier();
    const uint32_t total = lb[world];
    for (uint32_t k = threadIdx.x; k < total; k += kPartThreads) {
      uint32_t lo = 0, hi = world - 1;  // the owner of slot k: last d with lb[d] <= k
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (lb[mid] <= k) lo = mid;
        else hi = mid - 1;
      }
      const uint32_t pos = gb[lo] + (k - lb[lo]);
      if (pos < cap) (lo == me ? self_out : out)[lo * c1 + 1 + pos] = buf[k];
    }
    lds_barrier();  // buf, cnt and lb are rewritten by the next round
  };
  if (t0 < t1) {
    RowBatch<kPadU> qa, qb;
    in.template load_many<kPadU>(t0 + threadIdx.x, kPartThreads, t1, t0, qa);
    for (uint64_t i0 = t0;; i0 += 2 * kPadR) {  // uniform trip count
      in.template load_many<kPadU>(i0 + kPadR + threadIdx.x, kPartThreads, t1, t0, qb);
      round(qa, i0);
      if (i0 + kPadR >= t1) break;
      in.template load_many<kPadU>(i0 + 2 * kPadR + threadIdx.x, kPartThreads, t1, t0, qa);
      round(qb, i0 + kPadR);
      if (i0 + 2 * kPadR >= t1) break;
    }
  }
  if (xs.st) sink_count(xs, wn);
}

// Bucket partition writing ONE 16-byte record {hash lo, hash hi, rank, row}
// per keyed row (a single scattered store instead of three).  kInitRep: every
// row's rep is first set to its own rank here (one coalesced store); rows
// without a key are not partitioned, and K5 rewrites only the rows that link
// to an earlier chunk.  (The indexed grouping initialises rep in its probe.)
template <typename In, bool kInitRep>
__global__ __launch_bounds__(kPartThreads) void k_part_scatter_rec(
    In in, uint64_t n, uint32_t skip, uint32_t bits, const uint32_t* __restrict__ offs,
    uint4* __restrict__ rec, uint32_t* __restrict__ rep) {
  extern __shared__ __attribute__((aligned(16))) uint32_t cur[];
  const uint32_t nbins = 1u << bits;
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads)
    cur[b] = offs[static_cast<uint64_t>(b) * gridDim.x + part_block()];
  __syncthreads();
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  constexpr int U = kUnroll;
  for (uint64_t i0 = t0 + threadIdx.x; i0 < t1; i0 += U * kPartThreads) {
    RowBatch<U> q;
    in.template load_many<U>(i0, kPartThreads, t1, i0, q);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = i0 + static_cast<uint64_t>(u) * kPartThreads;
      const uint32_t r = in.rank_of(q, u);
      // every row starts as its own Object (coalesced store): rows without a
      // key stay so (mod.rs:238-239); K5 overwrites only the rows that link
      if (kInitRep && q.in[u]) rep[i] = r;
      if (!in.valid_of(q, u)) continue;
      const uint64_t h = in_hash<In>(in.key_of(q, u));
      const uint32_t p = atomicAdd(&cur[digit_of(h, skip, bits)], 1u);
      rec[p] = make_uint4(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32), r,
                          in.row_of(q, u));
    }
  }
}

// Partition into few digits (<= 64: the coarse pass of the two-level
// partition) in sorted runs: each round the block's kPartThreads x 4 rows are
// counting-sorted by digit in LDS (64 KiB) and leave as one contiguous run per
// digit (~4096 / nbins records, consecutive lanes on consecutive addresses)
// instead of one scattered 16-B store per row.  The next round's rows are
// loaded during the current one (ping-pong batches, LDS-only barriers).
// The block also counts its rows per FINAL bucket (the fbits hash bits below
// `skip`: coarse digit + second-pass digit) in 16-bit LDS counters and writes
// them to fine[block][bucket] -- the second pass's histogram, which therefore
// needs no pass over the records of its own.  A counter that would pass 65535
// (one key filling more than 64 Ki rows of a block's tile) sets *ovf, and
// k_fine_recount rebuilds the counts from the records instead.
// kRec12: 12-byte records {hash lo, hash hi, row} (rank = rank_base + row).
constexpr uint32_t kRunMaxBins = 64;
template <typename In, bool kInitRep, bool kRec12 = false>
__global__ __launch_bounds__(kPartThreads) void k_part_scatter_runs(
    In in, uint64_t n, uint32_t skip, uint32_t bits, const uint32_t* __restrict__ offs,
    uint4* __restrict__ rec, uint32_t* __restrict__ rep, uint32_t fbits,
    uint32_t* __restrict__ fine, uint32_t* __restrict__ ovf) {
  constexpr int U = 4;
  constexpr uint32_t R = U * kPartThreads;
  using RecT = typename std::conditional<kRec12, uint3, uint4>::type;
  __shared__ RecT buf[R];
  RecT* __restrict__ out = reinterpret_cast<RecT*>(rec);
  __shared__ uint32_t cnt[kRunMaxBins], base[kRunMaxBins + 1], cur[kRunMaxBins];
  __shared__ uint32_t fc[1u << (kMaxBucketBits - 1)];  // 2 x 16-bit counters per word
  const uint32_t nbins = 1u << bits, nfine = 1u << fbits;
  if (threadIdx.x < nbins)
    cur[threadIdx.x] = offs[static_cast<uint64_t>(threadIdx.x) * gridDim.x + part_block()];
  for (uint32_t b = threadIdx.x; b < nfine / 2; b += kPartThreads) fc[b] = 0;
  bool over = false;
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  auto round = [&](const RowBatch<U>& q, uint64_t i0) {
    if (threadIdx.x < nbins) cnt[threadIdx.x] = 0;
    lds_barrier();
    uint32_t dg[U], lr[U];
    RecT rq[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = i0 + threadIdx.x + static_cast<uint64_t>(u) * kPartThreads;
      dg[u] = ~0u;
      if (!q.in[u]) continue;
      const uint32_t r = in.rank_of(q, u);
      if (kInitRep) rep[i] = r;
      if (!in.valid_of(q, u)) continue;
      const uint64_t h = in_hash<In>(in.key_of(q, u));
      dg[u] = digit_of(h, skip, bits);
      lr[u] = atomicAdd(&cnt[dg[u]], 1u);
      const uint32_t fb = digit_of(h, skip, fbits), sh = (fb & 1u) << 4;
      over |= ((atomicAdd(&fc[fb >> 1], 1u << sh) >> sh) & 0xFFFFu) == 0xFFFFu;
      if constexpr (kRec12)
        rq[u] = make_uint3(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32), in.row_of(q, u));
      else
        rq[u] = make_uint4(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32), r,
                           in.row_of(q, u));
    }
    lds_barrier();
    if (threadIdx.x < 64) {  // the (<= 64) run starts: one wave's shuffle scan
      static_assert(kRunMaxBins <= 64, "one wave scans the run starts");
      const uint32_t lane = threadIdx.x;
      const uint32_t v = lane < nbins ? cnt[lane] : 0u;
      uint32_t inc = v;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(inc, d);
        if (lane >= static_cast<uint32_t>(d)) inc += o;
      }
      if (lane < nbins) base[lane] = inc - v;
      if (lane == nbins - 1) base[nbins] = inc;
    }
    lds_barrier();
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (dg[u] != ~0u) buf[base[dg[u]] + lr[u]] = rq[u];
    lds_barrier();
    const uint32_t total = base[nbins];
    for (uint32_t k = threadIdx.x; k < total; k += kPartThreads) {
      const RecT v = buf[k];
      const uint32_t b = digit_of((static_cast<uint64_t>(v.y) << 32) | v.x, skip, bits);
      out[cur[b] + (k - base[b])] = v;
    }
    lds_barrier();
    if (threadIdx.x < nbins) cur[threadIdx.x] += cnt[threadIdx.x];
  };
  constexpr uint64_t kStep = R;
  if (t0 < t1) {
    RowBatch<U> qa, qb;
    in.template load_many<U>(t0 + threadIdx.x, kPartThreads, t1, t0, qa);
    for (uint64_t i0 = t0;; i0 += 2 * kStep) {  // uniform trip count
      in.template load_many<U>(i0 + kStep + threadIdx.x, kPartThreads, t1, t0, qb);
      round(qa, i0);
      if (i0 + kStep >= t1) break;
      in.template load_many<U>(i0 + 2 * kStep + threadIdx.x, kPartThreads, t1, t0, qa);
      round(qb, i0 + kStep);
      if (i0 + 2 * kStep >= t1) break;
    }
  }
  if (over) *ovf = 1u;
  __syncthreads();
  uint32_t* f = fine + static_cast<uint64_t>(part_block()) * nfine;
  for (uint32_t b = threadIdx.x; b < nfine; b += kPartThreads)
    f[b] = (fc[b >> 1] >> ((b & 1u) << 4)) & 0xFFFFu;
}

// The coarse pass WITHOUT a histogram pass before it (round 3): each block
// writes its keyed rows into its own tile's range of the record array,
// [t0, t0 + keyed rows), round after round, each round counting-sorted by
// coarse digit in LDS and stored as ONE contiguous chunk; a run table records
// where every (block, round, digit) run starts and how long it is, and the
// block adds its per-digit totals to segtot (the segment sizes).  The second
// pass (k_part2_runs) reads a segment's records as those runs, so no global
// offsets -- and no k_part_hist pass over all rows -- are needed.  Fine
// counts per final bucket as in k_part_scatter_runs.
// Rows per thread per round of k_part_private: 12-byte records take 8192-row
// rounds (96 KiB of sort buffer beside 8-bit fine counters): half the runs of
// 4096-row rounds, each twice as long, for the second pass to read.  16-byte
// records keep 4096-row rounds and 16-bit counters (64 KiB + 64 KiB).
template <bool kRec12>
constexpr int priv_rows() { return kRec12 ? 8 : 4; }
template <bool kRec12>
constexpr uint32_t priv_round() { return static_cast<uint32_t>(priv_rows<kRec12>()) * kPartThreads; }

template <typename In, bool kInitRep, bool kRec12 = false, bool kX = false>
__global__ __launch_bounds__(kPartThreads) void k_part_private(
    In in, uint64_t n, uint32_t skip, uint32_t bits, uint4* __restrict__ rec,
    uint32_t* __restrict__ rep, uint32_t fbits, uint32_t* __restrict__ fine,
    uint32_t* __restrict__ ovf, uint32_t* __restrict__ run_start, uint32_t* __restrict__ run_len,
    uint32_t max_rounds, uint32_t* __restrict__ segtot, XSink xs = XSink{}) {
  constexpr int U = priv_rows<kRec12>();
  constexpr uint32_t R = priv_round<kRec12>();
  using RecT = typename std::conditional<kRec12, uint3, uint4>::type;
  __shared__ RecT buf[R];
  RecT* __restrict__ out = reinterpret_cast<RecT*>(rec);
  __shared__ uint32_t cnt[2][kRunMaxBins];  // digit counts, by round parity
  // fine counters, kFc bits each, 32 / kFc per word, added to without a
  // return value.  A counter that wraps (a key filling 256 / 65536 rows of
  // one tile's final bucket) loses 2^kFc and gives its neighbour at most 1,
  // so the block's counters then sum to less than its rows: that sets the
  // overflow flag, and k_fine_recount_runs rebuilds every count from the
  // records.
  constexpr uint32_t kFc = kRec12 ? 8u : 16u, kFcPer = 32u / kFc, kFcMax = (1u << kFc) - 1u;
  constexpr uint32_t kFcShift = kRec12 ? 2u : 1u;
  static_assert((1u << kFcShift) == kFcPer, "counters per word");
  __shared__ uint32_t fc[(1u << kMaxBucketBits) / kFcPer];
  const uint32_t nbins = 1u << bits, nfine = 1u << fbits;
  const uint32_t blk = part_block();
  uint32_t wn = 0;  // the wave's keyless rows (XSink)
  for (uint32_t b = threadIdx.x; b < nfine / kFcPer; b += kPartThreads) fc[b] = 0;
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  uint32_t acc = 0, r = 0, dsum = 0;  // records written, rounds done; wave 0: its digit's total
  // XSink: the keyless rows of kKmRounds rounds as bits of km (bit U k + u:
  // round rbase + k, the thread's row u), sunk together -- the rounds' own
  // loops carry one OR on their rare keyless branch, nothing else (a ballot
  // test per round measured +0.02 ms at 100 M rows)
  constexpr uint32_t kKmRounds = 32u / U;
  static_assert((kKmRounds & (kKmRounds - 1)) == 0, "rounds per sink flush: a power of two");
  uint32_t km = 0;
  auto flush = [&](uint32_t rbase) {
    if constexpr (kX) {
      for (uint64_t b = __ballot(km != 0); b; b = __ballot(km != 0)) {
        const uint32_t p = __ffs(__shfl(km, __ffsll(static_cast<unsigned long long>(b)) - 1)) - 1;
        const uint64_t i = t0 + static_cast<uint64_t>(rbase + p / U) * R + threadIdx.x +
                           static_cast<uint64_t>(p % U) * kPartThreads;
        sink_keyless<kRec12>(xs, in, (km >> p) & 1u, i, wn);
        km &= ~(1u << p);
      }
    }
    (void)rbase;
  };
  // Digit counters by round parity: every wave reads round r's after the
  // first barrier, so wave 0 zeroes the OTHER array (read in round r - 1)
  // for round r + 1 -- no barrier of its own.  Three barriers per round:
  // counted, sorted into the buffer, stored.
  if (threadIdx.x < 2 * kRunMaxBins) (&cnt[0][0])[threadIdx.x] = 0;
  __syncthreads();
  auto round = [&](const RowBatch<U>& q, uint64_t i0) {
    const uint32_t p = r & 1u;
    uint32_t dg[U], lr[U];
    RecT rq[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = i0 + threadIdx.x + static_cast<uint64_t>(u) * kPartThreads;
      dg[u] = ~0u;
      if (!q.in[u]) continue;
      const uint32_t rk = in.rank_of(q, u);
      if (kInitRep) rep[i] = rk;
      if (!in.valid_of(q, u)) {
        if constexpr (kX) km |= 1u << (U * (r & (kKmRounds - 1)) + u);  // sunk every kKmRounds
        continue;
      }
      const uint64_t h = in_hash<In>(in.key_of(q, u));
      dg[u] = digit_of(h, skip, bits);
      lr[u] = atomicAdd(&cnt[p][dg[u]], 1u);
      const uint32_t fb = digit_of(h, skip, fbits), sh = (fb & (kFcPer - 1u)) * kFc;
      atomicAdd(&fc[fb >> kFcShift], 1u << sh);
      if constexpr (kRec12)
        rq[u] = make_uint3(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32), in.row_of(q, u));
      else
        rq[u] = make_uint4(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32), rk,
                           in.row_of(q, u));
    }
    lds_barrier();
    // every wave scans the (<= 64) digit counts itself, lane d holding digit
    // d's run start, so the buffer scatter reads its bases by a lane shuffle
    // instead of from LDS written behind a second barrier
    static_assert(kRunMaxBins <= 64, "one wave scans the run starts");
    const uint32_t lane = __lane_id();
    const uint32_t v = lane < nbins ? cnt[p][lane] : 0u;
    uint32_t inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = __shfl_up(inc, d);
      if (lane >= static_cast<uint32_t>(d)) inc += o;
    }
    const uint32_t excl = inc - v;
    const uint32_t total = __shfl(inc, 63);
    if (threadIdx.x < 64) {  // the run table row; the other parity's counters zeroed
      if (lane < nbins) cnt[p ^ 1u][lane] = 0;
      const uint64_t e = (static_cast<uint64_t>(blk) * max_rounds + r) * kRunMaxBins + lane;
      run_start[e] = static_cast<uint32_t>(t0) + acc + excl;
      run_len[e] = v;
      dsum += v;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t bb = __shfl(excl, static_cast<int>(dg[u] & 63u));
      if (dg[u] != ~0u) buf[bb + lr[u]] = rq[u];
    }
    lds_barrier();
    for (uint32_t k = threadIdx.x; k < total; k += kPartThreads) out[t0 + acc + k] = buf[k];
    acc += total;
    ++r;
    if constexpr (kX)
      if ((r & (kKmRounds - 1)) == 0) flush(r - kKmRounds);
    lds_barrier();
  };
  constexpr uint64_t kStep = R;
  if (t0 < t1) {
    RowBatch<U> qa, qb;
    in.template load_many<U>(t0 + threadIdx.x, kPartThreads, t1, t0, qa);
    for (uint64_t i0 = t0;; i0 += 2 * kStep) {  // uniform trip count
      in.template load_many<U>(i0 + kStep + threadIdx.x, kPartThreads, t1, t0, qb);
      round(qa, i0);
      if (i0 + kStep >= t1) break;
      in.template load_many<U>(i0 + 2 * kStep + threadIdx.x, kPartThreads, t1, t0, qa);
      round(qb, i0 + kStep);
      if (i0 + 2 * kStep >= t1) break;
    }
  }
  if constexpr (kX) flush(r & ~(kKmRounds - 1));
  if (threadIdx.x < 64) {  // rounds this tile did not have: empty runs
    for (uint32_t rr = r; rr < max_rounds; ++rr)
      run_len[(static_cast<uint64_t>(blk) * max_rounds + rr) * kRunMaxBins + threadIdx.x] = 0u;
    if (threadIdx.x < nbins && dsum) atomicAdd(&segtot[threadIdx.x], dsum);
  }
  __syncthreads();
  if constexpr (kX) sink_count(xs, wn);
  uint32_t* f = fine + static_cast<uint64_t>(blk) * nfine;
  uint32_t fsum = 0;
  for (uint32_t b = threadIdx.x; b < nfine; b += kPartThreads) {
    const uint32_t v = (fc[b >> kFcShift] >> ((b & (kFcPer - 1u)) * kFc)) & kFcMax;
    f[b] = v;
    fsum += v;
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) fsum += __shfl_xor(fsum, d);
  __shared__ uint32_t wsum[kPartThreads / 64];
  if (__lane_id() == 0) wsum[threadIdx.x >> 6] = fsum;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t tsum = 0;
    for (uint32_t w = 0; w < kPartThreads / 64; ++w) tsum += wsum[w];
    if (tsum != acc) *ovf = 1u;  // a counter wrapped (see fc)
  }
}

// Only after a 16-bit counter overflow in k_part_scatter_runs (*ovf): for
// every (coarse block j, segment c) -- a grid-stride loop, so the usual call
// costs one small launch -- recount the records j wrote to segment c
// ([seg[c * P + j], seg[c * P + j + 1])) on the kB2 second-pass digit bits.
template <uint32_t kB2, typename RecT = uint4>
__global__ __launch_bounds__(kPartThreads) void k_fine_recount(const RecT* __restrict__ rec,
                                                                uint32_t skip,
                                                                const uint32_t* __restrict__ seg,
                                                                uint32_t P, uint32_t nseg,
                                                                uint32_t fbits,
                                                                uint32_t* __restrict__ fine,
                                                                const uint32_t* __restrict__ ovf) {
  if (*ovf == 0) return;
  constexpr uint32_t nb = 1u << kB2;
  __shared__ uint32_t cnt[nb];
  for (uint32_t jc = blockIdx.x; jc < P * nseg; jc += gridDim.x) {
    const uint32_t j = jc % P, c = jc / P;
    for (uint32_t b = threadIdx.x; b < nb; b += kPartThreads) cnt[b] = 0;
    __syncthreads();
    const uint32_t s0 = seg[static_cast<uint64_t>(c) * P + j];
    const uint32_t s1 = seg[static_cast<uint64_t>(c) * P + j + 1];
    for (uint32_t i = s0 + threadIdx.x; i < s1; i += kPartThreads) {
      const RecT v = rec[i];
      atomicAdd(&cnt[digit_of((static_cast<uint64_t>(v.y) << 32) | v.x, skip, kB2)], 1u);
    }
    __syncthreads();
    uint32_t* f = fine + static_cast<uint64_t>(j) * (1u << fbits) + (static_cast<uint64_t>(c) << kB2);
    for (uint32_t b = threadIdx.x; b < nb; b += kPartThreads) f[b] = cnt[b];
    __syncthreads();
  }
}

// k_fine_recount for the run layout of k_part_private: the records coarse
// block j wrote to segment c are its runs (j, r, c), r < max_rounds.
template <uint32_t kB2, typename RecT = uint4>
__global__ __launch_bounds__(kPartThreads) void k_fine_recount_runs(
    const RecT* __restrict__ rec, uint32_t skip, const uint32_t* __restrict__ run_start,
    const uint32_t* __restrict__ run_len, uint32_t max_rounds, uint32_t P, uint32_t nseg,
    uint32_t fbits, uint32_t* __restrict__ fine, const uint32_t* __restrict__ ovf) {
  if (*ovf == 0) return;
  constexpr uint32_t nb = 1u << kB2;
  __shared__ uint32_t cnt[nb];
  for (uint32_t jc = blockIdx.x; jc < P * nseg; jc += gridDim.x) {
    const uint32_t j = jc % P, c = jc / P;
    for (uint32_t b = threadIdx.x; b < nb; b += kPartThreads) cnt[b] = 0;
    __syncthreads();
    for (uint32_t r = 0; r < max_rounds; ++r) {
      const uint64_t e = (static_cast<uint64_t>(j) * max_rounds + r) * kRunMaxBins + c;
      const uint32_t s0 = run_start[e], len = run_len[e];
      for (uint32_t i = threadIdx.x; i < len; i += kPartThreads) {
        const RecT v = rec[s0 + i];
        atomicAdd(&cnt[digit_of((static_cast<uint64_t>(v.y) << 32) | v.x, skip, kB2)], 1u);
      }
    }
    __syncthreads();
    uint32_t* f = fine + static_cast<uint64_t>(j) * (1u << fbits) + (static_cast<uint64_t>(c) << kB2);
    for (uint32_t b = threadIdx.x; b < nb; b += kPartThreads) f[b] = cnt[b];
    __syncthreads();
  }
}

// Per final bucket b: E[j][b] = rows of b that coarse blocks [0, kR j) wrote
// (the start of second-pass block j inside bucket b; block j takes coarse
// blocks [kR j, kR (j + 1))) and tot[b] = the bucket's size.  A block covers 64
// buckets x kP2 blocks: thread (bi, jg) sums the fine counts of its kP2 / 16
// second-pass blocks (each wave reads 256 contiguous bytes per load), then the
// 16 partial sums of a bucket are scanned in LDS.  Resets *ovf for the next call.
template <uint32_t kP2, uint32_t kR>
__global__ __launch_bounds__(1024) void k_fine_scan(const uint32_t* __restrict__ fine,
                                                    uint32_t nfine, uint32_t* __restrict__ E,
                                                    uint32_t* __restrict__ tot,
                                                    uint32_t* __restrict__ ovf) {
  static_assert(kP2 % 16 == 0, "second-pass blocks per thread");
  constexpr uint32_t kJ = kP2 / 16;
  __shared__ uint32_t part[16][64];
  const uint32_t bi = threadIdx.x & 63u, jg = threadIdx.x >> 6;
  const uint32_t b = blockIdx.x * 64 + bi;
  if (blockIdx.x == 0 && threadIdx.x == 0) *ovf = 0;
  uint32_t sj[kJ], local = 0;
#pragma unroll
  for (uint32_t k = 0; k < kJ; ++k) {
    const uint64_t j = jg * kJ + k;
    uint32_t v = 0;
#pragma unroll
    for (uint32_t r = 0; r < kR; ++r)
      v += b < nfine ? fine[(j * kR + r) * nfine + b] : 0u;
    sj[k] = v;
    local += v;
  }
  part[jg][bi] = local;
  __syncthreads();
  uint32_t pre = 0, all = 0;
#pragma unroll
  for (uint32_t g = 0; g < 16; ++g) {
    const uint32_t v = part[g][bi];
    pre += g < jg ? v : 0u;
    all += v;
  }
  if (b >= nfine) return;
#pragma unroll
  for (uint32_t k = 0; k < kJ; ++k) {
    E[static_cast<uint64_t>(jg * kJ + k) * nfine + b] = pre;
    pre += sj[k];
  }
  if (jg == 0) tot[b] = all;
}

// Bucket partition with LDS staging (12-bit digits, 2 slots in the product): a
// keyed row is parked in its bucket's kSlots-record LDS slot and leaves with
// the slot's other rows as one kSlots x 16-B run, so the scattered writes are
// kSlots times fewer and wider.  Rows arriving at a full slot are written
// directly.  Rows are taken kRows per thread per round; each round ends with a
// flush of the full slots; partly filled slots go out at the end.
// Two-level use (n > 4096 x kBucketRows): blockIdx.y = segment c of a first,
// coarse pass ([seg[c * P1], seg[(c + 1) * P1]) of its records), the digit is
// the kBits hash bits below the segment's, and the offsets are laid out
// [c][digit][block] -- so the group kernel sees 2^(cbits + kBits) buckets.
constexpr uint32_t kStageBits = 12;
// Second pass of the two-level partition: 9 digit bits, 16-record runs, 4 rows
// per thread per round, 128 blocks per coarse segment (each takes what 2
// coarse blocks wrote to its segment).  Wider runs write fewer partial lines:
// on the staged scatter alone 12/2 0.163 ms, 10/8 0.123 ms
// (profiles/r2/exp_scatter_slots_r2t.log); at 100 M rows the 6 + 9-bit split
// with 16-record runs beat 5 + 10 with 8 (profiles/r2/exp_twolevel_r2E.log).
// Blocks per segment at 100 M rows (scripts/exp_twolevel_s2.hip,
// profiles/r3/exp_twolevel_s2/): 64 -> 128 2.25 -> 2.21 ms, 256 2.40 ms;
// 8-record runs (two blocks per CU) 2.37 ms; 2 or 8 rows per thread slower.
constexpr uint32_t kStage2Bits = 9;
constexpr uint32_t kStage2Slots = 16;
constexpr int kStage2Rows = 4;
constexpr uint32_t kStage2Blocks = 128;
// kRec12: 12-byte records {hash lo, hash hi, row} for rows whose rank is
// rank_base + row (RowsIn without a rank array): a quarter less to write here
// and to read in the group kernel (k_bucket_group12).
template <typename In, bool kInitRep, uint32_t kBits = kStageBits, uint32_t kSlots = 2, int kRows = 2,
          bool kRec12 = false>
__global__ __launch_bounds__(kPartThreads) void k_part_scatter_rec_staged(
    In in, uint64_t n, uint32_t skip, const uint32_t* __restrict__ offs, uint4* __restrict__ rec,
    uint32_t* __restrict__ rep, const uint32_t* __restrict__ seg, uint32_t P1,
    const uint32_t* __restrict__ ftot = nullptr, uint32_t* __restrict__ fbase = nullptr,
    uint32_t R = 1) {
  constexpr uint32_t nbins = 1u << kBits;
  using RecT = typename std::conditional<kRec12, uint3, uint4>::type;
  __shared__ RecT stage[nbins][kSlots];
  RecT* __restrict__ out = reinterpret_cast<RecT*>(rec);
  __shared__ uint32_t fill[nbins];
  __shared__ uint32_t cur[nbins];
  // Fewer buckets than threads (the two-level second pass): the row that
  // fills a bucket's kSlots slots lists the bucket, and the flush writes each
  // listed bucket's run with kSlots ADJACENT lanes, so a store instruction
  // covers 64 / kSlots whole runs.  (Two lanes per bucket, each writing every
  // other record, touched 32 runs per instruction: the store pattern, not the
  // bytes, set the pass's time -- scripts/exp_stores.hip, runs of 2 vs 16:
  // 0.133 vs 0.033 ms for 201 MB.)  full_n by round parity: the count of
  // round r + 1 is cleared during round r's flush, when nothing reads it.
  constexpr bool kCoop = nbins < kPartThreads;
  static_assert(!kCoop || (64 % kSlots == 0 && kPartThreads % kSlots == 0),
                "a bucket's run is written by lanes of one wave");
  // (absent from the 12-bit 16-byte variant, whose stage, fill and cur fill
  // the 160 KiB exactly: referenced only under kCoop)
  __shared__ uint16_t full[kCoop ? nbins : 1];
  __shared__ uint32_t full_n[kCoop ? 2 : 1];
  const uint32_t c = blockIdx.y;
  uint64_t t0 = 0, t1 = 0;
  if (ftot) {
    // offsets from block-major counts (k_fine_scan): offs = E[j][bucket], the
    // rows of each bucket that blocks before j hold; ftot = bucket sizes.
    // Two-level second pass (seg): block j takes what coarse blocks
    // [R j, R (j + 1)) wrote to segment c, whose first record is seg[c P1].
    // One level (no seg): block j takes tile j of the rows.  Bucket starts:
    // segment start + exclusive scan of the segment's bucket sizes, scanned
    // here (kPerT per thread); block 0 of each segment publishes them (fbase,
    // + the total) for the group kernel.
    constexpr uint32_t kPerT = nbins > kPartThreads ? nbins / kPartThreads : 1u;
    static_assert(nbins <= kPartThreads || nbins % kPartThreads == 0, "buckets per thread");
    uint32_t* wsum = fill;  // scratch for the 16 wave sums (LDS is full)
    const uint32_t j = part_block(), t = threadIdx.x, lane = __lane_id();
    const uint64_t nfine = static_cast<uint64_t>(gridDim.y) << kBits, b0 = static_cast<uint64_t>(c) << kBits;
    // every prologue load issued up front (clamped, selected at use): the
    // bucket sizes, this block's starts inside them and the segment bounds
    uint32_t v[kPerT], ov[kPerT], sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < kPerT; ++k) {
      const uint32_t b = min(t * kPerT + k, nbins - 1);
      v[k] = ftot[b0 + b];
      ov[k] = offs[j * nfine + b0 + b];
    }
    uint32_t seg_c = 0, seg_t0 = 0, seg_t1 = 0, seg_end = 0;
    if (seg) {
      seg_c = seg[static_cast<uint64_t>(c) * P1];
      seg_t0 = seg[static_cast<uint64_t>(c) * P1 + min(P1, R * j)];
      seg_t1 = seg[static_cast<uint64_t>(c) * P1 + min(P1, R * (j + 1))];
      seg_end = seg[static_cast<uint64_t>(gridDim.y) * P1];
    }
#pragma unroll
    for (uint32_t k = 0; k < kPerT; ++k) {
      if (t * kPerT + k >= nbins) v[k] = 0u;
      sum += v[k];
    }
    uint32_t inc = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = __shfl_up(inc, d);
      if (lane >= static_cast<uint32_t>(d)) inc += o;
    }
    if (lane == 63) wsum[t >> 6] = inc;
    __syncthreads();
    uint32_t base = seg_c + inc - sum, total = 0;
    for (uint32_t w = 0; w < kPartThreads / 64; ++w) {
      if (w < (t >> 6)) base += wsum[w];
      total += wsum[w];
    }
    __syncthreads();  // wsum (= fill) is cleared below
#pragma unroll
    for (uint32_t k = 0; k < kPerT; ++k) {
      const uint32_t b = t * kPerT + k;
      if (b < nbins) {
        cur[b] = base + ov[k];
        fill[b] = 0;
        if (j == 0) fbase[b0 + b] = base;
      }
      base += v[k];
    }
    if (j == 0 && c == gridDim.y - 1 && t == 0)
      fbase[nfine] = seg ? seg_end : total;
    if (seg) {
      t0 = seg_t0;
      t1 = seg_t1;
    } else {
      tile_of(n, gridDim.x, t0, t1);
    }
  } else {
    const uint64_t obase = static_cast<uint64_t>(c) * nbins * gridDim.x;
    for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads) {
      cur[b] = offs[obase + static_cast<uint64_t>(b) * gridDim.x + part_block()];
      fill[b] = 0;
    }
  }
  if constexpr (kCoop)
    if (threadIdx.x == 0) full_n[0] = full_n[1] = 0;
  __syncthreads();
  if (ftot) {
    // tile set above
  } else if (seg) {
    const uint64_t s0 = seg[static_cast<uint64_t>(c) * P1], s1 = seg[static_cast<uint64_t>(c + 1) * P1];
    tile_of(s1 - s0, gridDim.x, t0, t1);
    t0 += s0;
    t1 += s0;
  } else {
    tile_of(n, gridDim.x, t0, t1);
  }
  constexpr int U = kRows;
  constexpr uint64_t kStep = static_cast<uint64_t>(U) * kPartThreads;
  // one round: stage (or write) the batch's rows, then flush the full slots.
  // The round barriers wait for LDS only (lds_barrier), so the next round's
  // loads and this round's record stores stay in flight across them.
  auto round = [&](const RowBatch<U>& q, uint64_t i0, uint32_t par) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = i0 + threadIdx.x + static_cast<uint64_t>(u) * kPartThreads;
      if (!q.in[u]) continue;
      const uint32_t r = in.rank_of(q, u);
      if (kInitRep) rep[i] = r;
      if (!in.valid_of(q, u)) continue;
      const uint64_t h = in_hash<In>(in.key_of(q, u));
      const uint32_t b = digit_of(h, skip, kBits);
      RecT rq;
      if constexpr (kRec12)
        rq = make_uint3(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32), in.row_of(q, u));
      else
        rq = make_uint4(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32), r, in.row_of(q, u));
      const uint32_t sl = atomicAdd(&fill[b], 1u);
      if (sl < kSlots) {
        stage[b][sl] = rq;
        if constexpr (kCoop)
          if (sl == kSlots - 1)
            full[atomicAdd(&full_n[par & (kCoop ? 1u : 0u)], 1u)] = static_cast<uint16_t>(b);
      } else {
        out[atomicAdd(&cur[b], 1u)] = rq;
      }
    }
    lds_barrier();
    // unrolled, not a loop: the compiler drains every load in flight before a
    // store-only loop that reads registers loaded outside it (vmcnt(0))
    if constexpr (nbins >= kPartThreads) {
      static_assert(nbins % kPartThreads == 0, "flush slots per thread");
#pragma unroll
      for (uint32_t j = 0; j < nbins / kPartThreads; ++j) {
        const uint32_t b = threadIdx.x + j * kPartThreads;
        if (fill[b] >= kSlots) {
          const uint32_t p = cur[b];
          cur[b] = p + kSlots;
#pragma unroll
          for (uint32_t k = 0; k < kSlots; ++k) out[p + k] = stage[b][k];
          fill[b] = 0;
        }
      }
    } else {
      // lane group x / kSlots writes listed bucket e's record x % kSlots; the
      // group's lanes read cur[b] in the same instruction, before its first
      // lane advances it
      const uint32_t nf = full_n[par & (kCoop ? 1u : 0u)];
      if (threadIdx.x == 0) full_n[(par ^ 1u) & (kCoop ? 1u : 0u)] = 0;
      for (uint32_t x = threadIdx.x; x < nf * kSlots; x += kPartThreads) {
        const uint32_t e = x / kSlots, k = x % kSlots;
        const uint32_t b = full[e];
        const uint32_t p = cur[b];
        out[p + k] = stage[b][k];
        if (k == 0) {
          cur[b] = p + kSlots;
          fill[b] = 0;
        }
      }
    }
    lds_barrier();
  };
  // Software pipeline: round r + 1's rows are loaded while round r is staged
  // and flushed.  Two batches in ping-pong (a register copy between rounds
  // would wait for the loads just issued), and the prefetches unconditional
  // (past the tile they re-read row t0) so that the compiler's wait counts need
  // not cover a path without them.
  if (t0 < t1) {
    RowBatch<U> qa, qb;
    in.template load_many<U>(t0 + threadIdx.x, kPartThreads, t1, t0, qa);
    for (uint64_t i0 = t0;; i0 += 2 * kStep) {  // uniform trip count
      in.template load_many<U>(i0 + kStep + threadIdx.x, kPartThreads, t1, t0, qb);
      round(qa, i0, 0u);
      if (i0 + kStep >= t1) break;
      in.template load_many<U>(i0 + 2 * kStep + threadIdx.x, kPartThreads, t1, t0, qa);
      round(qb, i0 + kStep, 1u);
      if (i0 + 2 * kStep >= t1) break;
    }
  }
  // the slots' remainders, kSlots adjacent lanes per bucket (as k_part2_runs)
  for (uint32_t x = threadIdx.x; x < nbins * kSlots; x += kPartThreads) {
    const uint32_t b = x / kSlots, k = x % kSlots;
    if (k < fill[b]) out[cur[b] + k] = stage[b][k];
  }
}

// Second pass of the two-level partition over k_part_private's runs: block
// (j, c) takes the runs coarse blocks [R j, R (j + 1)) wrote for segment c --
// up to kMaxRuns (block, round) runs, listed with their exclusive prefix in LDS
// -- and stages their records exactly as k_part_scatter_rec_staged's second
// pass does (kS2-record slots, listed full buckets flushed by adjacent lanes).
// Record k of the block's virtual range is found by a 9-step binary search
// of the run prefix.  Segment starts from segtot (sizes summed by the first
// pass); bucket starts from the fine scan's sizes as before.  kF: a bucket is
// listed for the round-end flush once it holds kF records (kF = kS2: full
// buckets only).  Flushing from 8 or 12 staged records cuts the arrivals that
// meet a full slot array (single-record stores, ~20 % of records at kF = 16)
// but measured slower at 100 M rows (2.02 ms at 16, 2.06 at 12, 2.10 at 8,
// profiles/r3/exp_twolevel_s2/run_r3I.log): a block's stores into one bucket
// fill one contiguous range, so the L2 merges the single stores anyway.
constexpr uint32_t kMaxRuns = 512;  // R x max_rounds (host: two_level_launch)
template <bool kRec12, uint32_t kB2, uint32_t kS2, int kRows, uint32_t kF = kS2>
__global__ __launch_bounds__(kPartThreads) void k_part2_runs(
    const uint4* __restrict__ rec1, uint32_t skip, const uint32_t* __restrict__ offs,
    uint4* __restrict__ rec, const uint32_t* __restrict__ run_start,
    const uint32_t* __restrict__ run_len, uint32_t max_rounds, uint32_t P1, uint32_t R,
    const uint32_t* __restrict__ segtot, const uint32_t* __restrict__ ftot,
    uint32_t* __restrict__ fbase) {
  constexpr uint32_t nbins = 1u << kB2;
  using RecT = typename std::conditional<kRec12, uint3, uint4>::type;
  static_assert(nbins < kPartThreads && 64 % kS2 == 0 && kPartThreads % kS2 == 0,
                "listed buckets flushed by adjacent lanes of one wave");
  static_assert(kF >= 1 && kF <= kS2, "flush threshold within the slots");
  static_assert(kMaxRuns < kPartThreads, "one run per thread in the prologue");
  __shared__ RecT stage[nbins][kS2];
  __shared__ uint32_t fill[nbins], cur[nbins];
  __shared__ uint16_t full[nbins];
  __shared__ uint32_t full_n[2];
  __shared__ uint32_t rpre[kMaxRuns + 1], rst[kMaxRuns];
  __shared__ uint32_t wsum[kPartThreads / 64], wsumb[kPartThreads / 64];
  __shared__ uint32_t s_segbase, s_all;
  const RecT* __restrict__ in = reinterpret_cast<const RecT*>(rec1);
  RecT* __restrict__ out = reinterpret_cast<RecT*>(rec);
  const uint32_t c = blockIdx.y, j = part_block(), t = threadIdx.x, lane = __lane_id();
  const uint32_t nseg = gridDim.y;
  const uint64_t nfine = static_cast<uint64_t>(nseg) << kB2, b0 = static_cast<uint64_t>(c) << kB2;
  const uint32_t nr = R * max_rounds;
  // Every prologue load is issued here, up front and unconditionally (clamped
  // indices, values selected at use): their addresses are independent, so the
  // block waits out ONE memory latency instead of four in a row (a block's
  // prologue overlaps nothing else: one block per CU).
  const uint32_t seg_v = segtot[min(t, nseg - 1)];
  const uint32_t tr = min(t, nr - 1), cb = R * j + tr / max_rounds, rr = tr % max_rounds;
  const uint64_t e = (static_cast<uint64_t>(min(cb, P1 - 1)) * max_rounds + rr) * kRunMaxBins + c;
  const uint32_t len_v = run_len[e], st_v = run_start[e];
  const uint32_t tb = min(t, nbins - 1);
  const uint32_t ft_v = ftot[b0 + tb];
  const uint32_t off_v = offs[static_cast<uint64_t>(j) * nfine + b0 + tb];
  if (t < 64) {  // this segment's start and the total, from the (<= 64) segment sizes
    const uint32_t v = t < nseg ? seg_v : 0u;
    uint32_t inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = __shfl_up(inc, d);
      if (lane >= static_cast<uint32_t>(d)) inc += o;
    }
    if (t == c) s_segbase = inc - v;
    if (t == 63) s_all = inc;
  }
  {  // the block's runs (prefix of their lengths) and its bucket starts
     // (segment start + the segment's bucket sizes scanned): both block
     // scans share their barriers (two, not four: a block lives ~2 rounds)
    static_assert(nbins <= kPartThreads, "one bucket per thread");
    const bool has = t < nr && cb < P1;
    const uint32_t len = has ? len_v : 0u, st = has ? st_v : 0u;
    const uint32_t v = t < nbins ? ft_v : 0u;
    uint32_t inc = len, incb = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = __shfl_up(inc, d), ob = __shfl_up(incb, d);
      if (lane >= static_cast<uint32_t>(d)) {
        inc += o;
        incb += ob;
      }
    }
    if (lane == 63) {
      wsum[t >> 6] = inc;
      wsumb[t >> 6] = incb;
    }
    __syncthreads();  // wsum, wsumb; s_segbase / s_segend / s_all (wave 0 above)
    uint32_t before = 0, base = s_segbase + incb - v;
    for (uint32_t w = 0; w < (t >> 6); ++w) {
      before += wsum[w];
      base += wsumb[w];
    }
    if (t <= kMaxRuns) rpre[t] = before + inc - len;  // rpre[kMaxRuns] = the block's total
    if (t < kMaxRuns) rst[t] = st;
    if (t < nbins) {
      cur[t] = base + off_v;
      fill[t] = 0;
      if (j == 0) fbase[b0 + t] = base;
    }
    if (j == 0 && c == nseg - 1 && t == 0) fbase[nfine] = s_all;
    if (t == 0) full_n[0] = full_n[1] = 0;
  }
  __syncthreads();
  const uint32_t T = rpre[kMaxRuns];
  constexpr uint32_t kStep = static_cast<uint32_t>(kRows) * kPartThreads;
  // record k of the block's runs (k < T): the run whose prefix is the last <= k
  auto src_of = [&](uint32_t k) {
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t s = kMaxRuns / 2; s >= 1; s >>= 1)
      if (rpre[pos + s] <= k) pos += s;
    return rst[pos] + (k - rpre[pos]);
  };
  struct Batch {
    RecT v[kRows];
  };
  auto load = [&](uint32_t k0, Batch& q) {
    uint32_t s[kRows];
#pragma unroll
    for (int u = 0; u < kRows; ++u) s[u] = src_of(min(k0 + t + u * kPartThreads, T - 1));
#pragma unroll
    for (int u = 0; u < kRows; ++u) q.v[u] = in[s[u]];
  };
  auto round = [&](const Batch& q, uint32_t k0, uint32_t par) {
#pragma unroll
    for (int u = 0; u < kRows; ++u) {
      if (k0 + t + u * kPartThreads >= T) continue;
      const RecT rq = q.v[u];
      const uint32_t b = digit_of((static_cast<uint64_t>(rq.y) << 32) | rq.x, skip, kB2);
      const uint32_t sl = atomicAdd(&fill[b], 1u);
      if (sl < kS2) {
        stage[b][sl] = rq;
        if (sl == kF - 1) full[atomicAdd(&full_n[par], 1u)] = static_cast<uint16_t>(b);
      } else {
        out[atomicAdd(&cur[b], 1u)] = rq;
      }
    }
    lds_barrier();
    const uint32_t nf = full_n[par];
    if (t == 0) full_n[par ^ 1u] = 0;
    for (uint32_t x = t; x < nf * kS2; x += kPartThreads) {
      const uint32_t e = x / kS2, k = x % kS2;
      const uint32_t b = full[e];
      const uint32_t p = cur[b], len = min(fill[b], kS2);
      if (k < len) out[p + k] = stage[b][k];
      if (k == 0) {
        cur[b] = p + len;
        fill[b] = 0;
      }
    }
    lds_barrier();
  };
  if (T > 0) {  // the next round's records are loaded during the current one
    Batch qa, qb;
    load(0, qa);
    for (uint32_t k0 = 0;; k0 += 2 * kStep) {  // uniform trip count
      load(k0 + kStep, qb);
      round(qa, k0, 0u);
      if (k0 + kStep >= T) break;
      load(k0 + 2 * kStep, qa);
      round(qb, k0 + kStep, 1u);
      if (k0 + 2 * kStep >= T) break;
    }
  }
  // what is left in the slots (< kS2 per bucket, ~40 % of a block's records
  // at 100 M rows): kS2 adjacent lanes per bucket, so a store instruction
  // writes a few short runs instead of one record in each of 64 buckets
  for (uint32_t x = t; x < nbins * kS2; x += kPartThreads) {
    const uint32_t b = x / kS2, k = x % kS2;
    if (k < fill[b]) out[cur[b] + k] = stage[b][k];
  }
}

// The 12-bit staged scatter of rows in rank order (RowsIn without a rank
// array: 12-byte records, rank = rank_base + row), WARP-SPECIALISED.  Waves
// 0-7 only load and stage: their rows are prefetched two rounds ahead and they
// never store, so the compiler's waits before a round cover their loads only
// (in k_part_scatter_rec_staged the conditional record stores sit between a
// round's prefetch and its use, and the waits there drain them too).  Waves
// 8-15 only store: the full slot pairs, the rows that met a full slot (an LDS
// overflow list, kept in arrival order per bucket by an LDS cursor) and, with
// kInitRep, rep = rank of the round's rows (computed, nothing loaded).  Two
// barriers per round: staged (A), flushed (B) -- the bucket cursors advance
// atomically and the overflow count alternates by round parity, so the
// barrier between the pair flush and the overflow rows (round 3-4's M) is
// gone.
// scripts/exp_scatter_align.hip: 12.5 M rows 0.136 -> 0.123 ms
// (profiles/r3/exp_scatter_align/run.log).
constexpr uint32_t kWsProd = 512;   // producer threads (waves 0-7)
constexpr int kWsRows = 4;          // rows per producer thread per round
// In: the caller's rows (RowsIn, rank = rank_base + row) or received exchange
// records (RecRankIn: the rank in the record's third word).
template <typename In, bool kInitRep>
__global__ __launch_bounds__(kPartThreads) void k_part_scatter_ws(
    In in, uint64_t n, uint32_t skip, const uint32_t* __restrict__ offs,
    const uint32_t* __restrict__ ftot, uint3* __restrict__ out, uint32_t* __restrict__ rep,
    uint32_t* __restrict__ fbase) {
  constexpr uint32_t nbins = 1u << kStageBits;
  constexpr uint32_t kRound = kWsProd * kWsRows;  // 2048 rows
  static_assert(2 * kWsProd == kPartThreads, "half producers, half consumers");
  __shared__ uint3 stage[nbins][2];
  __shared__ uint32_t fill[nbins], cur[nbins];
  __shared__ uint3 ovf[kRound];
  __shared__ uint32_t ovf_n[2];  // by round parity (no barrier to reset it)
  // bucket starts: the segment's sizes scanned here, block 0 publishes them
  constexpr uint32_t kPerT = nbins / kPartThreads;
  const uint32_t t = threadIdx.x, lane = __lane_id();
  const uint32_t j = part_block();
  // the block's starts inside its buckets loaded with the bucket sizes (one
  // memory latency for both, not one after the other around the scan)
  uint32_t v[kPerT], ov[kPerT], sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPerT; ++k) {
    v[k] = ftot[t * kPerT + k];
    ov[k] = offs[static_cast<uint64_t>(j) * nbins + t * kPerT + k];
  }
#pragma unroll
  for (uint32_t k = 0; k < kPerT; ++k) sum += v[k];
  uint32_t inc = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d);
    if (lane >= static_cast<uint32_t>(d)) inc += o;
  }
  if (lane == 63) fill[t >> 6] = inc;
  __syncthreads();
  uint32_t base = inc - sum, total = 0;
  for (uint32_t w = 0; w < kPartThreads / 64; ++w) {
    if (w < (t >> 6)) base += fill[w];
    total += fill[w];
  }
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < kPerT; ++k) {
    const uint32_t b = t * kPerT + k;
    cur[b] = base + ov[k];
    fill[b] = 0;
    if (j == 0) fbase[b] = base;
    base += v[k];
  }
  if (j == 0 && t == 0) fbase[nbins] = total;
  if (t < 2) ovf_n[t] = 0;
  __syncthreads();
  uint64_t t0, t1;
  tile_of(n, gridDim.x, t0, t1);
  const uint32_t rounds = t1 > t0 ? static_cast<uint32_t>((t1 - t0 + kRound - 1) / kRound) : 0u;
  if (t < kWsProd) {
    RowBatch<kWsRows> qa, qb;
    in.template load_many<kWsRows>(t0 + t, kWsProd, t1, t0, qa);
    in.template load_many<kWsRows>(t0 + kRound + t, kWsProd, t1, t0, qb);
    auto stage_round = [&](const RowBatch<kWsRows>& q, uint32_t par) {
#pragma unroll
      for (int u = 0; u < kWsRows; ++u) {
        if (!in.valid_of(q, u)) continue;
        const uint64_t h = in_hash<In>(in.key_of(q, u));
        const uint32_t b = digit_of(h, skip, kStageBits);
        const uint3 rq = make_uint3(static_cast<uint32_t>(h), static_cast<uint32_t>(h >> 32),
                                    in.row_of(q, u));
        const uint32_t sl = atomicAdd(&fill[b], 1u);
        if (sl < 2)
          stage[b][sl] = rq;
        else
          ovf[atomicAdd(&ovf_n[par], 1u)] = rq;
      }
    };
    // per round exactly the consumers' two barriers (A, B); the loads of
    // round r + 2 go out between A and B, while the consumers store
    for (uint32_t r = 0; r < rounds; r += 2) {
      stage_round(qa, 0u);
      lds_barrier();  // A
      in.template load_many<kWsRows>(t0 + (r + 2) * static_cast<uint64_t>(kRound) + t, kWsProd, t1,
                                     t0, qa);
      lds_barrier();  // B
      if (r + 1 >= rounds) break;
      stage_round(qb, 1u);
      lds_barrier();  // A
      in.template load_many<kWsRows>(t0 + (r + 3) * static_cast<uint64_t>(kRound) + t, kWsProd, t1,
                                     t0, qb);
      lds_barrier();  // B
    }
  } else {
    const uint32_t c = t - kWsProd;
    for (uint32_t r = 0; r < rounds; ++r) {
      lds_barrier();  // A
      if constexpr (kInitRep) {
        // every row starts as its own Object: rows without a key stay so
        // (mod.rs:238-239); K5 overwrites only the rows that link
        const uint64_t r0 = t0 + static_cast<uint64_t>(r) * kRound;
#pragma unroll
        for (uint32_t u = 0; u < kRound / kWsProd; ++u) {
          const uint64_t i = r0 + c + u * kWsProd;
          if (i < t1) rep[i] = in.rank_base + static_cast<uint32_t>(i);
        }
      }
#pragma unroll
      for (uint32_t k = 0; k < nbins / kWsProd; ++k) {
        const uint32_t b = c + k * kWsProd;
        if (fill[b] >= 2) {
          // an atomic cursor: the overflow rows below advance it too, with
          // no barrier between (a pair and an overflow row of one bucket may
          // take either order; every position is taken once)
          const uint32_t p = atomicAdd(&cur[b], 2u);
          out[p] = stage[b][0];
          out[p + 1] = stage[b][1];
          fill[b] = 0;
        }
      }
      const uint32_t par = r & 1u, no = ovf_n[par];
      if (c == 0) ovf_n[par ^ 1u] = 0;  // last round's, read by every consumer before its B
      for (uint32_t o = c; o < no; o += kWsProd) {
        const uint3 rq = ovf[o];
        out[atomicAdd(&cur[digit_of((static_cast<uint64_t>(rq.y) << 32) | rq.x, skip, kStageBits)],
                      1u)] = rq;
      }
      lds_barrier();  // B
    }
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += kPartThreads)
    for (uint32_t k = 0; k < fill[b]; ++k) out[cur[b] + k] = stage[b][k];
}

// First probe slot of a record in the LDS table (kLdsSlots, any size): the
// low 32 bits of its hash, scaled.  The digit bits (the top ones) are constant
// inside a bucket, the low ones are not.
__device__ __forceinline__ uint32_t lds_slot(uint64_t h) {
  return static_cast<uint32_t>((static_cast<uint64_t>(static_cast<uint32_t>(h)) * kLdsSlots) >> 32);
}

// Double hashing: a key's probe step is 1 + 6 * (10 low hash bits, below the
// slot's), coprime with the 6144 (= 2^11 * 3) slots, so every probe sequence
// visits every slot and sequences of different keys do not run together in
// clusters.  A wave probes until its longest chain is placed; with linear
// probing those chains were clustered: 12.5 M rows 0.099 -> 0.081 ms
// (scripts/exp_group_persist.hip, profiles/r2/exp_group_persist_r2AG.log).
// (Round 5: the 10 bits are the LOW bits of h lo -- bits 40-49 overlapped the
// bucket's own digit bits, so inside a bucket the step took only 2^(10 -
// overlap) values; the slot comes from the top bits of h lo.)
__device__ __forceinline__ uint32_t lds_step(uint64_t h) {
  return 1u + 6u * (static_cast<uint32_t>(h) & 1023u);
}

__device__ __forceinline__ uint32_t next_slot(uint32_t h, uint32_t step) {
  const uint32_t s = h + step;  // h, step < kLdsSlots
  return s >= kLdsSlots ? s - kLdsSlots : s;
}

// Global-table slot (tsize a power of two, up to 2^34 for a 2^32-row bucket).
__device__ __forceinline__ uint64_t global_slot(uint64_t h, uint64_t tsize) {
  return h & (tsize - 1);
}

constexpr int kPer = (kLdsCap + kGroupThreads - 1) / kGroupThreads;

// Where K5 puts a bucket's result.  Per record: live (a keyed row of the
// bucket), r (its rank), w (its row), f (the lowest rank of its key).
//   RepOut:  rep[w] = f for the rows that link to an earlier chunk (the
//            partition initialised rep = rank): one scattered 4-B store each.
//   ListOut: the Object write set itself (round 4; sdgpu_group_link_device),
//            in the bucket's own record range [start, end) -- one entry per
//            keyed row, so the positions need no global coordination:
//            creators from the front, who = rank; linked rows from the back,
//            who = rank | SDGPU_LINKED, obj = f.  Coalesced;
//            no rep array.  lcnt[bucket] = its linked rows; the last bucket
//            stores the keyed total in lcnt[buckets]; k_list_finish then sets
//            counts[0..2] (no same-address atomics: 32 k workgroups adding
//            to one word serialised at ~4 ns each, +0.29 ms at 100 M rows in
//            r4e's fused_job leg).
struct RepOut {
  static constexpr int kScratch = 1;
  uint32_t* rep;
  template <int kSteps>
  __device__ __forceinline__ void emit(const bool (&live)[kSteps], const bool (&lk)[kSteps],
                                       const uint32_t (&r)[kSteps], const uint32_t (&w)[kSteps],
                                       const uint32_t (&f)[kSteps], uint32_t, uint32_t, uint32_t&,
                                       uint32_t&, uint32_t*, bool) const {
#pragma unroll
    for (int j = 0; j < kSteps; ++j)
      if (lk[j]) rep[w[j]] = f[j];  // others keep rank
    (void)live;
    (void)r;
  }
};
// Block 0 sets counts[] from the buckets' linked counts lcnt[] and K = the
// keyed entries, lcnt[nb] (the last bucket's end): counts[1] = L, [0] = K - L
// + E, [2] = K + E -- loads issued 8 at a time (a plain loop over the 32 k
// counts of 100 M rows took ~10 us).  With a keyless sink (XSink, E rows)
// block 1 + j moves the 16 wave segments of first-pass block j (valid keyless
// rows, who = rank: own Objects) to who[K + (rows of the segments before)
// ...], one wave per segment.  (Every block reducing a slice and adding it
// with atomics took 9 us: 512 same-address atomics, r4zd.)
__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t* sw) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d);
  if (__lane_id() == 0) sw[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t t = 0;
  for (uint32_t w = 0; w < blockDim.x / 64; ++w) t += sw[w];
  __syncthreads();  // sw reusable
  return t;
}
// cap / nospc: the caller's list capacity (ListOut); sink rows past it are
// not written and the total past it raises *nospc.
__global__ __launch_bounds__(1024) void k_list_finish(const uint32_t* __restrict__ lcnt,
                                                      uint32_t nb, uint32_t* __restrict__ counts,
                                                      uint32_t* __restrict__ who, XSink xs,
                                                      uint32_t cap, uint32_t* __restrict__ nospc) {
  __shared__ uint32_t sw[16], sseg[kSinkWaves];
  constexpr uint32_t kPerT = kPartBlocks * kSinkWaves / 1024;
  static_assert(kPartBlocks * kSinkWaves % 1024 == 0, "segments per thread");
  const uint32_t lane = __lane_id(), wv = threadIdx.x >> 6;
  const uint32_t seg0 = blockIdx.x ? (blockIdx.x - 1) * kSinkWaves : 0u;
  uint32_t e = 0, bf = 0;  // sink rows: all, in the segments before this block's
  if (xs.st) {             // the segment counts loaded together (one latency)
    uint32_t cv[kPerT];
#pragma unroll
    for (uint32_t k = 0; k < kPerT; ++k) cv[k] = xs.cnt[threadIdx.x + k * 1024];
#pragma unroll
    for (uint32_t k = 0; k < kPerT; ++k) {
      const uint32_t g = threadIdx.x + k * 1024;
      e += cv[k];
      if (g < seg0) bf += cv[k];
      if (blockIdx.x && g - seg0 < kSinkWaves) sseg[g - seg0] = cv[k];
    }
  }
  if (blockIdx.x == 0) {
    const uint32_t K = lcnt[nb];
    uint32_t l = 0;
    constexpr uint32_t kB = 8;
    for (uint32_t i0 = 0; i0 < nb; i0 += kB * 1024) {
      uint32_t v[kB];
#pragma unroll
      for (uint32_t k = 0; k < kB; ++k) {
        const uint32_t i = i0 + threadIdx.x + k * 1024;
        v[k] = i < nb ? lcnt[i] : 0u;
      }
#pragma unroll
      for (uint32_t k = 0; k < kB; ++k) l += v[k];
    }
    const uint32_t L = block_sum(l, sw), E = block_sum(e, sw);
    if (threadIdx.x == 0) {
      counts[1] = L;
      counts[0] = K - L + E;
      counts[2] = K + E;
      if (nospc && static_cast<uint64_t>(K) + E > cap) *nospc = 1u;
    }
    return;
  }
  const uint32_t before = block_sum(bf, sw);
  uint32_t o = lcnt[nb] + before;  // wave wv copies segment wv of first-pass block j
  for (uint32_t w = 0; w < wv; ++w) o += sseg[w];
  const uint32_t c = sseg[wv];
  const uint32_t* src = xs.st + static_cast<uint64_t>(seg0 + wv) * xs.cap;
  for (uint32_t k = lane; k < c; k += 64)
    if (o + k < cap) who[o + k] = src[k];
}
hipError_t out_finish(const RepOut&, uint32_t, hipStream_t) { return hipSuccess; }
// ListOut: each wave reserves the slots of ALL its entries with ONE LDS
// atomic per list on the bucket's creator / linked counters (scr[0..1],
// zeroed with the table) and places step j's entries after those of steps
// < j (round 5: one atomic round trip per wave instead of one per step and
// list -- the group kernel is VALU-issue bound).  No barrier
// in emit, one at the end for the linked total.  The entries' order inside a
// bucket depends on wave timing (not part of the contract).  Workgroup-wide
// ranks in record order (two barriers + a one-wave scan per emit) measured
// slower: 100 M rows 1.870 -> 1.850 ms, 12.5 M rows 0.246 -> 0.244 ms
// (profiles/r4/listranks_ab/).
constexpr uint32_t kLinkedBit = 0x80000000u;
struct ListOut {
  static constexpr int kScratch = 2;
  uint32_t* who;
  uint32_t* obj;
  uint32_t* counts;
  uint32_t* lcnt;  // [bucket]: linked rows; [buckets]: the keyed total
  XSink x;         // the valid keyless rows, when the partition collects them
  // entries who / obj hold (the sharded write set's caller capacity): a
  // bucket ending past it writes nothing and sets *nospc (the call then
  // fails with -ENOSPC); ~0: unbounded (n entries at most)
  uint32_t cap = 0xFFFFFFFFu;
  uint32_t* nospc = nullptr;
  template <int kSteps>
  __device__ __forceinline__ void emit(const bool (&live)[kSteps], const bool (&lk)[kSteps],
                                       const uint32_t (&r)[kSteps], const uint32_t (&w)[kSteps],
                                       const uint32_t (&f)[kSteps], uint32_t start, uint32_t end,
                                       uint32_t&, uint32_t&, uint32_t* scr, bool) const {
    if (end > cap) {  // uniform per bucket
      if (threadIdx.x == 0) *nospc = 1u;
      return;
    }
    uint64_t bc[kSteps], bl[kSteps];
    uint32_t nc = 0, nl = 0;
#pragma unroll
    for (int j = 0; j < kSteps; ++j) {
      bc[j] = __ballot(live[j] && !lk[j]);
      bl[j] = __ballot(lk[j]);
      nc += static_cast<uint32_t>(__popcll(bc[j]));
      nl += static_cast<uint32_t>(__popcll(bl[j]));
    }
    uint32_t cb = 0, lb = 0;
    if (__lane_id() == 0) {
      if (nc) cb = atomicAdd(&scr[0], nc);
      if (nl) lb = atomicAdd(&scr[1], nl);
    }
    cb = __builtin_amdgcn_readfirstlane(cb);  // lane 0 is active here
    lb = __builtin_amdgcn_readfirstlane(lb);
#pragma unroll
    for (int j = 0; j < kSteps; ++j) {
      const uint32_t bc_lo = static_cast<uint32_t>(bc[j]), bc_hi = static_cast<uint32_t>(bc[j] >> 32);
      const uint32_t bl_lo = static_cast<uint32_t>(bl[j]), bl_hi = static_cast<uint32_t>(bl[j] >> 32);
      if (live[j] && !lk[j])
        who[start + cb + __builtin_amdgcn_mbcnt_hi(bc_hi, __builtin_amdgcn_mbcnt_lo(bc_lo, 0u))] = r[j];
      if (lk[j]) {
        const uint32_t p =
            end - 1 - (lb + __builtin_amdgcn_mbcnt_hi(bl_hi, __builtin_amdgcn_mbcnt_lo(bl_lo, 0u)));
        who[p] = r[j] | kLinkedBit;
        obj[p] = f[j];
      }
      cb += static_cast<uint32_t>(__popcll(bc[j]));
      lb += static_cast<uint32_t>(__popcll(bl[j]));
    }
    (void)w;
  }
};
__device__ __forceinline__ void out_init(const RepOut&, uint32_t*) {}
__device__ __forceinline__ void out_init(const ListOut&, uint32_t* scr) {
  if (threadIdx.x < 2) scr[threadIdx.x] = 0;  // before the bucket's first barrier
}
__device__ __forceinline__ void out_done(const ListOut& o, uint32_t, uint32_t, uint32_t end,
                                         const uint32_t* scr) {
  __syncthreads();  // every wave's atomics on the counters are done
  if (threadIdx.x == 0) {
    o.lcnt[blockIdx.x] = scr[1];
    if (blockIdx.x == gridDim.x - 1) o.lcnt[gridDim.x] = end;
  }
}
__device__ __forceinline__ void out_done(const RepOut&, uint32_t, uint32_t, uint32_t,
                                         const uint32_t*) {}
hipError_t out_finish(const ListOut& o, uint32_t nb, hipStream_t s) {
  k_list_finish<<<o.x.st ? 1 + kPartBlocks : 1u, 1024, 0, s>>>(o.lcnt, nb, o.counts, o.who, o.x,
                                                                 o.cap, o.nospc);
  return hipGetLastError();
}

// Bucket records as {hash lo, hash hi, rank, row}: 16-byte records as stored,
// or 12-byte ones {hash lo, hash hi, row} with rank = rank_base + row.
struct Rec16Src {
  const uint4* __restrict__ p;
  __device__ __forceinline__ uint4 operator()(uint32_t i) const { return p[i]; }
};
struct Rec12Src {
  const uint3* __restrict__ p;
  uint32_t rank_base;
  __device__ __forceinline__ uint4 operator()(uint32_t i) const {
    const uint3 v = p[i];
    return make_uint4(v.x, v.y, rank_base + v.z, v.z);
  }
};

// LDS-sized bucket: every thread loads its (at most kPer) records at once and
// keeps them in registers for both phases.
template <typename Src>
__device__ __forceinline__ void load_bucket(Src rec, uint32_t start, uint32_t end,
                                            uint4 (&q_reg)[kPer]) {
  if (end - start > kLdsCap || end == start) return;
  // unconditional loads, selected after (see group_bucket_packed)
#pragma unroll
  for (int j = 0; j < kPer; ++j) q_reg[j] = rec(min(start + threadIdx.x + j * kGroupThreads, end - 1));
#pragma unroll
  for (int j = 0; j < kPer; ++j)
    if (start + threadIdx.x + j * kGroupThreads >= end) q_reg[j] = make_uint4(0, 0, 0, 0);
}

// Group-by of one bucket too large for LDS: a private region of the global
// table (4 slots per row, agent-scope atomics).  The results leave in chunks of
// kGroupThreads records (uniform trip count: the list output ranks each chunk
// across the workgroup).
template <typename Src, typename Out>
__device__ __forceinline__ void group_bucket_global(Src rec, uint32_t start, uint32_t end,
                                                    ChunkOf chunk_of, uint64_t* __restrict__ gkey,
                                                    uint32_t* __restrict__ gmin, const Out& out,
                                                    uint32_t& special_min, uint32_t* scr) {
  const uint32_t m = end - start;
  uint64_t tsize = 1;
  while (tsize * 2 <= 4ull * m) tsize *= 2;  // 2m < tsize <= 4m (64-bit: no wrap)
  uint64_t* tk = gkey + 4ull * start;
  uint32_t* tm = gmin + 4ull * start;
  for (uint64_t s = threadIdx.x; s < tsize; s += kGroupThreads) {
    tk[s] = kEmpty;
    tm[s] = 0xFFFFFFFFu;
  }
  if (threadIdx.x == 0) special_min = 0xFFFFFFFFu;
  out_init(out, scr);
  __syncthreads();
  for (uint32_t i = start + threadIdx.x; i < end; i += kGroupThreads) {
    const uint4 q = rec(i);
    const uint64_t k = (static_cast<uint64_t>(q.y) << 32) | q.x;
    const uint32_t r = q.z;
    if (k == kEmpty) {
      atomicMin(&special_min, r);
      continue;
    }
    uint64_t h = global_slot(k, tsize);
    for (;;) {
      const uint64_t prev = atomicCAS(reinterpret_cast<unsigned long long*>(&tk[h]),
                                      static_cast<unsigned long long>(kEmpty),
                                      static_cast<unsigned long long>(k));
      if (prev == kEmpty || prev == k) {
        atomicMin(&tm[h], r);
        break;
      }
      h = (h + 1) & (tsize - 1);
    }
  }
  __syncthreads();
  uint32_t c_run = 0, l_run = 0;
  for (uint32_t i0 = start; i0 < end; i0 += kGroupThreads) {
    const uint32_t i = i0 + threadIdx.x;
    bool live[1] = {false}, lk[1] = {false};
    uint32_t r[1] = {0}, w[1] = {0}, f[1] = {0};
    if (i < end) {
      const uint4 q = rec(i);
      const uint64_t k = (static_cast<uint64_t>(q.y) << 32) | q.x;
      uint32_t fv;
      if (k == kEmpty) {
        fv = special_min;
      } else {
        uint64_t h = global_slot(k, tsize);
        for (;;) {
          const uint64_t kk =
              __hip_atomic_load(&tk[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (kk == k) break;
          h = (h + 1) & (tsize - 1);
        }
        fv = __hip_atomic_load(&tm[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      live[0] = true;
      r[0] = q.z;
      w[0] = q.w;
      f[0] = fv;
      lk[0] = chunk_of(q.z) != chunk_of(fv);
    }
    out.template emit<1>(live, lk, r, w, f, start, end, c_run, l_run, scr, true);
  }
  out_done(out, c_run, l_run, end, scr);
}

// Group-by of one bucket, rows [start, end) of rec (q_reg preloaded by
// load_bucket when the bucket fits the LDS table).
template <typename Src, typename Out>
__device__ __forceinline__ void group_bucket(Src rec, uint32_t start,
                                             uint32_t end, const uint4 (&q_reg)[kPer],
                                             ChunkOf chunk_of, uint64_t* __restrict__ gkey,
                                             uint32_t* __restrict__ gmin, const Out& out,
                                             uint64_t* lkey, uint32_t* lmin, uint32_t& special_min,
                                             uint32_t* scr) {
  const uint32_t m = end - start;
  if (m == 0) {
    out_init(out, scr);  // an empty bucket: counters zeroed for done
    out_done(out, 0u, 0u, end, scr);
    return;
  }
  if (m > kLdsCap) {
    group_bucket_global(rec, start, end, chunk_of, gkey, gmin, out, special_min, scr);
    return;
  }
  // (the LDS code names lkey / lmin directly: through generic pointers shared
  // with the global table the compiler emits FLAT atomics, ~30 % slower)
  for (uint32_t s = threadIdx.x; s < kLdsSlots; s += kGroupThreads) {
    lkey[s] = kEmpty;
    lmin[s] = 0xFFFFFFFFu;
  }
  if (threadIdx.x == 0) special_min = 0xFFFFFFFFu;
  out_init(out, scr);
  __syncthreads();
  // A thread's records probe in lock step: every pass issues the LDS
  // round trips of all its pending records back to back and only then
  // inspects the results, so their latencies overlap (the probe loops are
  // latency-bound, not LDS-bandwidth-bound).
  uint32_t h[kPer], step[kPer];
  uint32_t live = 0, pend = 0;  // bit j: record j exists / is still probing
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const uint64_t k = (static_cast<uint64_t>(q_reg[j].y) << 32) | q_reg[j].x;
    h[j] = lds_slot(k);
    step[j] = lds_step(k);
    if (start + threadIdx.x + j * kGroupThreads < end) {
      live |= 1u << j;
      if (k == kEmpty)
        atomicMin(&special_min, q_reg[j].z);
      else
        pend |= 1u << j;
    }
  }
  const uint32_t keyed = pend;
  while (pend) {
    uint64_t prev[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const uint64_t k = (static_cast<uint64_t>(q_reg[j].y) << 32) | q_reg[j].x;
      prev[j] = (pend >> j & 1u)
                    ? atomicCAS(reinterpret_cast<unsigned long long*>(&lkey[h[j]]),
                                static_cast<unsigned long long>(kEmpty),
                                static_cast<unsigned long long>(k))
                    : 0ull;
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      if (!(pend >> j & 1u)) continue;
      const uint64_t k = (static_cast<uint64_t>(q_reg[j].y) << 32) | q_reg[j].x;
      if (prev[j] == kEmpty || prev[j] == k) {
        atomicMin(&lmin[h[j]], q_reg[j].z);
        pend &= ~(1u << j);
      } else {
        h[j] = next_slot(h[j], step[j]);
      }
    }
  }
  __syncthreads();
  // every keyed record's final probe slot h[j] holds its key: read the
  // group minimum there (no second probe sequence needed)
  bool lv[kPer], lk[kPer];
  uint32_t r[kPer], w[kPer], f[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    lv[j] = live >> j & 1u;
    r[j] = q_reg[j].z;
    w[j] = q_reg[j].w;
    f[j] = lv[j] ? ((keyed >> j & 1u) ? lmin[h[j]] : special_min) : 0u;
    lk[j] = lv[j] && chunk_of(r[j]) != chunk_of(f[j]);
  }
  uint32_t c_run = 0, l_run = 0;
  out.template emit<kPer>(lv, lk, r, w, f, start, end, c_run, l_run, scr, false);
  out_done(out, c_run, l_run, end, scr);
}

// K5 with a PACKED 8-byte LDS table, for buckets of 12-15 digit bits (the
// one-level 12-bit path and the two-level path).  Inside a bucket the digit
// bits of h are implied, so a key is known by its other 64 - bits (<= 52)
// bits; with the record's index in the bucket + 1 (12 bits, 0 = empty) a
// slot is ONE 64-bit word.  The CAS that places or finds a key also names the
// record that owns it, the group minimum lives per owner (lmin[4096]), and
// 7680 slots fit where 6144 twelve-byte ones did: load ~0.4 instead of ~0.5,
// shorter probe chains.  scripts/exp/exp_group_packed.hip: 12.5 M rows 0.078
// -> 0.072 ms (profiles/r3/exp_group_packed/run.log).
// Round 5: the kernel is VALU-issue bound (SQ counters,
// VALU busy 73 % of the SIMD cycles at 12.5 M rows, 82 % at
// 100 M), so the VALU per record was cut twice.  First: the word assembled
// from 32-bit halves, and a double-hashing step from the LOW bits of h lo
// (the old one overlapped the digit bits: nearly linear probing).  Second:
// 2^13 slots (a step wraps as a 16-bit add of byte offsets; the odd step
// from the 13 low bits of h lo, the slot from its 13 top bits); the probe
// loop without branches per record (see below); the owner read from the
// record's final slot after the loop.  Probe-loop VALU per record and round
// ~16 -> 7.  64 KiB of table + a 4096-word area = exactly half the CU's LDS
// (two workgroups per CU, as before); the area holds lmin[kPkCap],
// special_min and the output's scratch, so kPkCap = 4093.  (Linear probing,
// step 1, lengthened the probe chains: 12.5 M rows 0.079 -> 0.085 ms,
// profiles/r5/pk_ab/.)
// Buckets above kPkCap records take the global table; pads (row ~0) are skipped.
constexpr uint32_t kPkSlots = 8192;  // 2^13
constexpr uint32_t kPkWords = 4096;  // lmin[kPkCap] | special_min | scr[2]
constexpr uint32_t kPkCap = kPkWords - 3;

// The packed group-by of one bucket whose records are in registers (q[j] =
// {h lo, h hi, rank, row}, row kPadRow past the end), m = end - start <=
// kPkCap, bits in 12..15 (the word's key field; group_launch picks this
// kernel only for those).
template <int kP, typename Out>
__device__ __forceinline__ void group_packed_regs(const uint4 (&q)[kP], uint32_t start, uint32_t end,
                                                  uint32_t bits, ChunkOf chunk_of, const Out& out,
                                                  uint64_t* tab, uint32_t* lmin, uint32_t* scr) {
  for (uint32_t s = threadIdx.x; s < kPkSlots; s += kGroupThreads) tab[s] = 0ull;
  for (uint32_t s = threadIdx.x; s < kPkCap; s += kGroupThreads) lmin[s] = 0xFFFFFFFFu;
  out_init(out, scr);
  __syncthreads();
  // word hi: the 24 - bits hi-word bits below the digit, the 8 shard bits
  // above it, then index + 1 in bits 20..31 (bits in 12..15: <= 20 key bits)
  const uint32_t kb = 24u - bits, lowm = (1u << kb) - 1u;
  uint32_t sa[kP], sst[kP], own1[kP], khi[kP];
  uint64_t word[kP];  // the record's word; 0 for a pad
  bool live[kP];
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    const uint32_t idx1 = threadIdx.x + j * kGroupThreads + 1u;
    khi[j] = (q[j].y & lowm) | ((q[j].y >> 24) << kb);
    live[j] = q[j].w != kPadRow;
    word[j] = live[j] ? (static_cast<uint64_t>(khi[j] | (idx1 << 20)) << 32) | q[j].x : 0ull;
    // byte offsets: the slot from the top 13 bits of h lo, the (odd) step
    // from its low 13 bits -- both independent of the digit bits (h hi)
    // (a pad: a slot of its own lane -- pads share the last record's h, and
    // 64 lanes CASing one word serialise)
    sa[j] = live[j] ? (q[j].x >> 16) & 0xFFF8u : threadIdx.x << 3;
    sst[j] = ((q[j].x << 3) | 8u) & 0xFFF8u;
  }
  // The records of a thread probe in lock step, without branches: every
  // round CASes all four words and the round's results decide.  A record
  // that has found its key CASes the same slot again, which holds that key
  // (its own word or its owner's) and so leaves it unchanged and finds it
  // again; a pad's word is 0, and CAS(0 -> 0) changes nothing.  Branches
  // per record (the lanes' pending masks) made the compiler wait out each
  // CAS before issuing the next.
  for (;;) {
    uint64_t prev[kP];
#pragma unroll
    for (int j = 0; j < kP; ++j)
      prev[j] = atomicCAS(reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(tab) + sa[j]),
                          0ull, static_cast<unsigned long long>(word[j]));
    bool all = true;
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      const uint32_t plo = static_cast<uint32_t>(prev[j]), phi = static_cast<uint32_t>(prev[j] >> 32);
      const bool hit = !live[j] || prev[j] == 0ull || (plo == q[j].x && (phi & 0xFFFFFu) == khi[j]);
      sa[j] = static_cast<uint16_t>(sa[j] + (hit ? 0u : sst[j]));  // 2^13 slots x 8 B
      all = all && hit;
    }
    if (all) break;
  }
  // each record's slot now holds its key's word: the owner's index + 1 (a
  // pad's slot may be empty: index 0 then, so that its unused lmin read
  // stays inside lmin)
#pragma unroll
  for (int j = 0; j < kP; ++j)
    own1[j] = max(1u, *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(tab) + sa[j] + 4) >> 20);
#pragma unroll
  for (int j = 0; j < kP; ++j)
    if (live[j]) atomicMin(&lmin[own1[j] - 1u], q[j].z);
  __syncthreads();
  bool lk[kP];
  uint32_t r[kP], w[kP], f[kP];
#pragma unroll
  for (int j = 0; j < kP; ++j) {
    r[j] = q[j].z;
    w[j] = q[j].w;
    f[j] = lmin[own1[j] - 1u];
    lk[j] = live[j] && r[j] != f[j] && chunk_of(r[j]) != chunk_of(f[j]);
  }
  uint32_t c_run = 0, l_run = 0;
  out.template emit<kP>(live, lk, r, w, f, start, end, c_run, l_run, scr, false);
}

// Records of a bucket into registers, kP per thread: every load issued
// unconditionally (past the end: the bucket's last record) and the pad
// selected after -- a guarded `i < end ? rec(i) : pad` made the compiler
// branch around each load and wait out its latency before the next one
// (four serial memory latencies per workgroup).  Only the row marks a pad:
// nothing reads a pad's other fields.
template <int kP, typename Src, typename Out>
__device__ __forceinline__ void group_packed_load(Src rec, uint32_t start, uint32_t end,
                                                  uint32_t bits, ChunkOf chunk_of, const Out& out,
                                                  uint64_t* tab, uint32_t* lmin, uint32_t* scr) {
  uint4 q[kP];
#pragma unroll
  for (int j = 0; j < kP; ++j) q[j] = rec(min(start + threadIdx.x + j * kGroupThreads, end - 1));
#pragma unroll
  for (int j = 0; j < kP; ++j)
    if (start + threadIdx.x + j * kGroupThreads >= end) q[j].w = kPadRow;
  group_packed_regs(q, start, end, bits, chunk_of, out, tab, lmin, scr);
}

template <typename Src, typename Out>
__device__ __forceinline__ void group_bucket_packed(Src rec, uint32_t start, uint32_t end,
                                                    uint32_t bits, ChunkOf chunk_of,
                                                    uint64_t* __restrict__ gkey,
                                                    uint32_t* __restrict__ gmin, const Out& out,
                                                    uint64_t* tab, uint32_t* lmin,
                                                    uint32_t& special_min, uint32_t* scr) {
  const uint32_t m = end - start;
  if (m == 0) {
    out_init(out, scr);  // an empty bucket: counters zeroed for done
    out_done(out, 0u, 0u, end, scr);
    return;
  }
  if (m > kPkCap) {
    group_bucket_global(rec, start, end, chunk_of, gkey, gmin, out, special_min, scr);
    return;
  }
  // three records per thread when they suffice (uniform per bucket; ~3 k
  // records is the mean bucket): a fourth of pads would still probe
  static_assert(kPkCap <= 4 * kGroupThreads, "four records per thread hold a bucket");
  if (m <= 3 * kGroupThreads)
    group_packed_load<3>(rec, start, end, bits, chunk_of, out, tab, lmin, scr);
  else
    group_packed_load<4>(rec, start, end, bits, chunk_of, out, tab, lmin, scr);
  out_done(out, 0u, 0u, end, scr);
}


// One workgroup per bucket.  Rows of bucket b: [offs[b*P], offs[(b+1)*P]).
template <typename Out>
__global__ __launch_bounds__(kGroupThreads, 8) void k_bucket_group(
    const uint4* __restrict__ rec, const uint32_t* __restrict__ offs, uint32_t P,
    ChunkOf chunk_of, uint64_t* __restrict__ gkey, uint32_t* __restrict__ gmin, Out out) {
  __shared__ uint64_t lkey[kLdsSlots];
  __shared__ uint32_t lmin[kLdsSlots];
  __shared__ uint32_t special_min;  // min rank of key == kEmpty (sentinel clash)
  __shared__ uint32_t scr[Out::kScratch];
  const uint32_t b = blockIdx.x;
  const uint32_t start = offs[static_cast<uint64_t>(b) * P];
  const uint32_t end = offs[static_cast<uint64_t>(b + 1) * P];  // offs[nb*P] = total
  uint4 q_reg[kPer];
  load_bucket(Rec16Src{rec}, start, end, q_reg);
  group_bucket(Rec16Src{rec}, start, end, q_reg, chunk_of, gkey, gmin, out, lkey, lmin,
               special_min, scr);
}

// k_bucket_group over 12-byte records (rank = rank_base + row).
template <typename Out>
__global__ __launch_bounds__(kGroupThreads, 8) void k_bucket_group12(
    const uint3* __restrict__ rec, uint32_t rank_base, const uint32_t* __restrict__ offs,
    ChunkOf chunk_of, uint64_t* __restrict__ gkey, uint32_t* __restrict__ gmin, Out out) {
  __shared__ uint64_t lkey[kLdsSlots];
  __shared__ uint32_t lmin[kLdsSlots];
  __shared__ uint32_t special_min;
  __shared__ uint32_t scr[Out::kScratch];
  const uint32_t b = blockIdx.x;
  const uint32_t start = offs[b], end = offs[b + 1];
  const Rec12Src src{rec, rank_base};
  uint4 q_reg[kPer];
  load_bucket(src, start, end, q_reg);
  group_bucket(src, start, end, q_reg, chunk_of, gkey, gmin, out, lkey, lmin, special_min, scr);
}

// Packed-table K5 (>= 12 digit bits): rows of bucket b in [offs[b*P], offs[(b+1)*P]).
template <typename Out>
__global__ __launch_bounds__(kGroupThreads, 8) void k_bucket_group_pk(
    const uint4* __restrict__ rec, const uint32_t* __restrict__ offs, uint32_t P, uint32_t bits,
    ChunkOf chunk_of, uint64_t* __restrict__ gkey, uint32_t* __restrict__ gmin, Out out) {
  __shared__ uint64_t tab[kPkSlots];
  __shared__ uint32_t lw[kPkWords];  // lmin | special_min | scr (80 KiB in all)
  static_assert(Out::kScratch <= 2, "scratch fits the word area");
  uint32_t* lmin = lw;
  uint32_t& special_min = lw[kPkCap];
  uint32_t* scr = lw + kPkCap + 1;
  const uint32_t b = blockIdx.x;
  group_bucket_packed(Rec16Src{rec}, offs[static_cast<uint64_t>(b) * P],
                      offs[static_cast<uint64_t>(b + 1) * P], bits, chunk_of, gkey, gmin, out, tab,
                      lmin, special_min, scr);
}

template <typename Out>
__global__ __launch_bounds__(kGroupThreads, 8) void k_bucket_group12_pk(
    const uint3* __restrict__ rec, uint32_t rank_base, const uint32_t* __restrict__ offs,
    uint32_t bits, ChunkOf chunk_of, uint64_t* __restrict__ gkey, uint32_t* __restrict__ gmin,
    Out out) {
  __shared__ uint64_t tab[kPkSlots];
  __shared__ uint32_t lw[kPkWords];  // lmin | special_min | scr (80 KiB in all)
  static_assert(Out::kScratch <= 2, "scratch fits the word area");
  uint32_t* lmin = lw;
  uint32_t& special_min = lw[kPkCap];
  uint32_t* scr = lw + kPkCap + 1;
  const uint32_t b = blockIdx.x;
  group_bucket_packed(Rec12Src{rec, rank_base}, offs[b], offs[b + 1], bits, chunk_of, gkey, gmin,
                      out, tab, lmin, special_min, scr);
}

// the segment sizes k_part_private adds to, and the fine-count overflow flag
__global__ void k_zero_runs(uint32_t* __restrict__ segtot, uint32_t* __restrict__ ovf) {
  if (threadIdx.x < kRunMaxBins) segtot[threadIdx.x] = 0;
  if (threadIdx.x == 0) *ovf = 0;
}

__global__ __launch_bounds__(256) void k_fill_init(uint32_t* __restrict__ dst, uint64_t n,
                                                   const uint32_t* __restrict__ init) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += stride)
    dst[i] = init ? init[i] : static_cast<uint32_t>(i);
}

__global__ __launch_bounds__(256) void k_scatter(const uint32_t* __restrict__ src,
                                                 const uint32_t* __restrict__ pos, uint64_t n,
                                                 uint32_t* __restrict__ dst) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += stride)
    dst[pos[i]] = src[i];
}

__global__ void k_copy_counts(const uint32_t* __restrict__ offs, uint32_t nbins,
                              uint64_t* __restrict__ counts) {
  const uint32_t b = threadIdx.x;
  if (b < nbins)
    counts[b] = offs[static_cast<uint64_t>(b + 1) * kPartBlocks] -
                offs[static_cast<uint64_t>(b) * kPartBlocks];
}

// Rows per destination rank of the exchange, from the scanned offsets of the
// destination-digit partition.
// msgs (may be NULL): the count messages of the exchange, {rows for d, n,
// code} per destination d (every rank learns every rank's n with the counts;
// code = the call's form and return leg, which every rank must share --
// checked by the receivers).
__global__ void k_dest_counts(const uint32_t* __restrict__ offs, uint32_t world,
                              int64_t* __restrict__ counts, int64_t* __restrict__ msgs,
                              int64_t n, int64_t code) {
  const uint32_t d = threadIdx.x;
  if (d < world) {
    const int64_t c = static_cast<int64_t>(offs[static_cast<uint64_t>(d + 1) * kPartBlocks]) -
                      offs[static_cast<uint64_t>(d) * kPartBlocks];
    counts[d] = c;
    if (msgs) {
      msgs[3 * d] = c;
      msgs[3 * d + 1] = n;
      msgs[3 * d + 2] = code;
    }
  }
}

// rep[i] of the sender's rows from the reps returned in send order: row i was
// sent at position pos[i] (~0: no key, it keeps its own rank).  Every sent
// position holds a rep: the full return writes all of them, the compact one
// starts from each record's own rank (k_back_init).  (Round 4 marked "no
// pair came back" with back == ~0, which is also the legal rep
// SDGPU_REP_EXISTING | 0x7FFFFFFF: ADVICE r4.)
// Positions in [self_lo, self_hi) read self[p]: the padded exchange's
// message to this rank itself, whose reps the owner side wrote locally.
__global__ __launch_bounds__(256) void k_gather_rep(const uint32_t* __restrict__ back,
                                                    const uint32_t* __restrict__ pos,
                                                    const uint32_t* __restrict__ rank, uint64_t n,
                                                    uint32_t* __restrict__ rep,
                                                    const uint32_t* __restrict__ self,
                                                    uint32_t self_lo, uint32_t self_hi) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += stride) {
    const uint32_t p = pos[i];
    const bool mine = p - self_lo < self_hi - self_lo;  // never for p == ~0 (< 2^32 slots)
    const uint32_t b = (mine ? self : back)[p == 0xFFFFFFFFu ? 0u : p];
    rep[i] = p == 0xFFFFFFFFu ? rank[i] : b;
  }
}

// Compact return leg, source side: back[p] = the rank in send record p (a
// row whose rep is its own rank gets no pair back).
__global__ __launch_bounds__(256) void k_back_init(const uint3* __restrict__ srec, uint64_t n,
                                                   uint32_t* __restrict__ back) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += stride)
    back[i] = srec[i].z;
}

// Fixed-capacity exchange messages (shard.cpp, padded exchange): the message
// to rank d is C1 = cap + 1 12-byte slots at d * C1 of the send buffer --
// slot 0 the header {rows for d | this source's overflow bit << 31, this
// source's n, kPadRank}, slots 1..cap the records (k_part_scatter with
// k_part_padded), the rest padding {0, 0, kPadRank}; the message to this
// rank itself lives in the receive buffer (self_out).  The owner's grouping drops
// every kPadRank record (RecIn::valid_of).  The overflow bit (some count of
// this source > cap: rows were not sent) goes to EVERY owner, so all ranks
// learn the same "some message overflowed" from their headers.  Block (0, 0)
// also writes summary[3] = rows this source sent, clears summary[4] (the
// list kernels' -ENOSPC flag) and zero3[0..2] (the write set's counts).
// counts (cnt: the reservation cursors) < 2^31 (n < 2^31 on this path).
__global__ __launch_bounds__(256) void k_pad_fill(const uint32_t* __restrict__ cnt, uint32_t world,
                                                  uint32_t me, uint32_t cap, uint32_t n,
                                                  uint3* __restrict__ out,
                                                  uint3* __restrict__ self_out,
                                                  uint32_t* __restrict__ summary,
                                                  uint32_t* __restrict__ zero3,
                                                  uint32_t* __restrict__ next_cursor) {
  const uint32_t d = blockIdx.y;
  bool ovf = false;
  uint32_t sent = 0;
  for (uint32_t p = 0; p < world; ++p) {
    const uint32_t c = cnt[p];
    ovf |= c > cap;
    sent += min(c, cap);
  }
  uint3* rec = d == me ? self_out : out;
  const uint64_t base = static_cast<uint64_t>(d) * (cap + 1ull);
  const uint32_t c = cnt[d];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    rec[base] = make_uint3(c | (ovf ? 0x80000000u : 0u), n, kPadRank);
    if (d == 0) {
      summary[3] = sent;
      summary[4] = 0u;
      if (world == 1) {  // nothing to receive: the owner's summary is this one
        summary[0] = ovf ? 1u : 0u;
        summary[1] = n;
        summary[2] = sent;
      }
      if (zero3) zero3[0] = zero3[1] = zero3[2] = 0u;
    }
  }
  // the next call's reservation cursors (the previous call used them; this
  // call's stay untouched while its blocks read them)
  if (blockIdx.x == 0 && threadIdx.x == 0) next_cursor[d] = 0u;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256;
  for (uint64_t j = min(c, cap) + static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; j < cap;
       j += stride)
    rec[base + 1 + j] = make_uint3(0u, 0u, kPadRank);
}

// Owner side, after the records arrived: summary[0] = some source overflowed
// (the same on every rank), [1] = the largest source n, [2] = rows received.
__global__ void k_recv_summary(const uint3* __restrict__ rrec, uint32_t world, uint32_t cap,
                               uint32_t* __restrict__ summary) {
  const uint32_t p = threadIdx.x;
  uint32_t ovf = 0, nmax = 0, rows = 0;
  if (p < world) {
    const uint3 h = rrec[static_cast<uint64_t>(p) * (cap + 1ull)];
    ovf = h.x >> 31;
    nmax = h.y;
    rows = min(h.x & 0x7FFFFFFFu, cap);
  }
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) {
    ovf |= __shfl_xor(ovf, s);
    nmax = max(nmax, __shfl_xor(nmax, s));
    rows += __shfl_xor(rows, s);
  }
  if (p == 0) {
    summary[0] = ovf;
    summary[1] = nmax;
    summary[2] = rows;
  }
}

// Compact return leg of the exchange (round 4): an owner sends back only the
// received rows whose rep is not their own rank, as {index of the row inside
// its (source -> owner) message, rep} -- 8 B per linked row instead of 4 B
// per row.  Tiles of kRetTile received rows never straddle a source's
// segment (the host lays them out per segment, RetTiles), so the pairs come
// out grouped by source in row order: tile counts, one scan, ranked writes.
constexpr int kRetThreads = 256;
constexpr int kRetRows = 16;
constexpr uint32_t kRetTile = kRetThreads * kRetRows;

__device__ __forceinline__ uint32_t ret_segment(const RetTiles& st, uint32_t blk) {
  uint32_t p = 0;
  while (p + 1 < st.world && st.tstart[p + 1] <= blk) ++p;
  return p;
}

__global__ __launch_bounds__(kRetThreads) void k_ret_count(RetTiles st, const uint3* __restrict__ rrec,
                                                           const uint32_t* __restrict__ rrep,
                                                           uint32_t* __restrict__ cnt) {
  __shared__ uint32_t sc[kRetThreads / 64];
  const uint32_t blk = blockIdx.x;
  uint32_t c = 0;
  if (blk < st.tstart[st.world]) {
    const uint32_t p = ret_segment(st, blk);
    const uint32_t k0 = st.roff[p] + (blk - st.tstart[p]) * kRetTile, k1 = st.roff[p + 1];
#pragma unroll
    for (int u = 0; u < kRetRows; ++u) {
      const uint32_t k = k0 + u * kRetThreads + threadIdx.x;
      if (k < k1) c += rrep[k] != rrec[k].z;
    }
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d);
  if (__lane_id() == 0) sc[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blk] = sc[0] + sc[1] + sc[2] + sc[3];
}

// cnt: exclusive scan of the tile counts (cnt[tiles] = total).  retcnt[p] =
// pairs for source p (int64, the count exchange's unit).
__global__ __launch_bounds__(kRetThreads) void k_ret_write(RetTiles st, const uint3* __restrict__ rrec,
                                                           const uint32_t* __restrict__ rrep,
                                                           const uint32_t* __restrict__ cnt,
                                                           uint2* __restrict__ ret,
                                                           int64_t* __restrict__ retcnt) {
  __shared__ uint32_t oc[kRetRows][kRetThreads / 64];
  const uint32_t blk = blockIdx.x, lane = __lane_id(), w = threadIdx.x >> 6;
  if (blk == 0 && threadIdx.x < st.world)
    retcnt[threadIdx.x] = static_cast<int64_t>(cnt[st.tstart[threadIdx.x + 1]]) -
                          static_cast<int64_t>(cnt[st.tstart[threadIdx.x]]);
  if (blk >= st.tstart[st.world]) return;  // the one block of an empty receive
  const uint32_t p = ret_segment(st, blk);
  const uint32_t k0 = st.roff[p] + (blk - st.tstart[p]) * kRetTile, k1 = st.roff[p + 1];
  const uint64_t lt = (1ull << lane) - 1ull;
  bool f[kRetRows];
  uint32_t v[kRetRows], pr[kRetRows];
#pragma unroll
  for (int u = 0; u < kRetRows; ++u) {
    const uint32_t k = k0 + u * kRetThreads + threadIdx.x;
    const uint32_t kk = k < k1 ? k : k1 - 1;
    v[u] = rrep[kk];
    f[u] = k < k1 && v[u] != rrec[kk].z;
    const uint64_t b = __ballot(f[u]);
    pr[u] = __popcll(b & lt);
    if (lane == 0) oc[u][w] = __popcll(b);
  }
  __syncthreads();
  static_assert(kRetRows * (kRetThreads / 64) == 64, "one wave scans the (row step, wave) counts");
  if (threadIdx.x < 64) {
    uint32_t* e = &oc[0][0];
    const uint32_t a = e[lane];
    uint32_t inc = a;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = __shfl_up(inc, d);
      if (lane >= static_cast<uint32_t>(d)) inc += o;
    }
    e[lane] = cnt[blk] - cnt[st.tstart[p]] + inc - a;  // index inside the segment's pairs
  }
  __syncthreads();
  const uint32_t seg0 = cnt[st.tstart[p]];
#pragma unroll
  for (int u = 0; u < kRetRows; ++u)
    if (f[u]) {
      const uint32_t k = k0 + u * kRetThreads + threadIdx.x;
      ret[seg0 + oc[u][w] + pr[u]] = make_uint2(k - st.roff[p], v[u]);
    }
}

// Source side: back[soff[d] + idx] = rep for every pair received from owner d
// (pairs of d at [poff[d], poff[d + 1]) of rback); back was set to ~0.
__global__ __launch_bounds__(256) void k_ret_apply(RetApply ap, const uint2* __restrict__ rback,
                                                   uint32_t* __restrict__ back) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256;
  const uint64_t total = ap.poff[ap.world];
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; i < total; i += stride) {
    uint32_t d = 0;
    while (d + 1 < ap.world && ap.poff[d + 1] <= i) ++d;
    const uint2 q = rback[i];
    back[ap.soff[d] + q.x] = q.y;
  }
}

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Blocks of the bucket partition: one per CU.  Each block keeps one open
// output line per bucket, so the blocks resident on one XCD hold blocks/8 x
// buckets x 128 B of partially written lines in its 4 MB L2.
uint32_t bucket_part_blocks() { return kPartBlocks; }

// ~kBucketRows rows per bucket (LDS table load <= 75 % with slack), up to 2^15
// buckets: 100 M rows on one GPU still group in LDS.
uint32_t bucket_bits_for(uint64_t n) {
  uint32_t bits = 1;
  while (bits < kMaxBucketBits && (n >> bits) > kBucketRows) ++bits;
  return bits;
}

// Above 2^12 buckets (n > ~12.6 M rows) the partition runs in two passes: a
// coarse one on the top cbits = bits - 9 digit bits (<= 64 output streams per
// block) into rec1, which also counts every row's final bucket (fine counts),
// then a 9-bit LDS-staged pass per coarse segment into rec (16-record runs, 64
// blocks per segment).  A single 2^15-way scatter keeps 32 k partially written
// lines open per block and ran 3.7 ms for 100 M rows
// (profiles/r2/bench_r2b.json); the two passes move 2 x 32 B per row instead.
struct GroupLayout {
  uint32_t bits, cbits;
  size_t hist, tiles, rec, hist1, rec1, gkey, gmin;
  size_t fine, fE, ftot, fbase, ovf;  // two-level only: the coarse pass's fine counts
  // two-level without a histogram pass (k_part_private / k_part2_runs): the
  // run table [block][round][digit] (starts, lengths) and the segment sizes
  uint32_t max_rounds;
  size_t run_s, run_l, segtot;
  size_t lcnt;
  size_t xst, xcnt;  // ListOut's keyless sink (XSink)
  size_t total;
};


// Rows per XSink wave segment: at least the rows one wave of a first-pass
// block reads -- a 16th of the block's tile plus one step of rows
// (k_part_private: 256 per round; k_part_hist: 512 per step, +2 edge rows).
uint32_t sink_cap(uint64_t n) {
  const uint64_t tile = (n + kPartBlocks - 1) / kPartBlocks;
  return static_cast<uint32_t>((tile + kSinkWaves - 1) / kSinkWaves + 520);
}

// bits_rows (0: n): the rows the buckets are sized for -- the keyed rows of a
// padded exchange receive, whose n counts the padding slots too (buckets
// over the LDS capacity stay correct through the global table, so the hint
// only chooses the layout).  with_sink: room for ListOut's keyless sink
// (~4 B per row; only the fused call without an index uses it).
GroupLayout group_layout(uint64_t n, uint64_t bits_rows = 0, bool with_sink = false) {
  constexpr uint32_t b2 = kStage2Bits;
  GroupLayout L;
  L.bits = bucket_bits_for(bits_rows && bits_rows < n ? bits_rows : n);
  L.cbits = L.bits > kStageBits ? L.bits - b2 : 0;
  const uint64_t nh = (static_cast<uint64_t>(1) << L.bits) * kMaxPartBlocks;
  const uint64_t nh1 = (static_cast<uint64_t>(1) << L.cbits) * kMaxPartBlocks;
  size_t o = 0;
  L.hist = o; o = align_up(o + 4 * (nh + 1), 256);
  L.tiles = o; o = align_up(o + 4 * (scan::tiles_for(nh) + 1), 256);
  L.rec = o; o = align_up(o + 16 * n, 256);
  L.hist1 = o; o = align_up(o + 4 * (nh1 + 1), 256);
  L.rec1 = o; o = align_up(o + (L.cbits ? 16 * n : 0), 256);
  L.gkey = o; o = align_up(o + 8 * 4 * n, 256);
  L.gmin = o; o = align_up(o + 4 * 4 * n, 256);
  const uint64_t nf = static_cast<uint64_t>(1) << L.bits;  // block-major counts (12-bit and two-level)
  L.fine = o; o = align_up(o + 4 * nf * kPartBlocks, 256);
  L.fE = o; o = align_up(o + 4 * nf * kPartBlocks, 256);
  L.ftot = o; o = align_up(o + 4 * nf, 256);
  L.fbase = o; o = align_up(o + 4 * (nf + 1), 256);
  L.ovf = o; o = align_up(o + 4, 256);
  // rounds in the largest coarse tile (kPartBlocks tiles), sized for the
  // shorter 4096-row rounds (k_part_private: priv_round)
  const uint64_t tile = (n + kPartBlocks - 1) / kPartBlocks;
  L.max_rounds = L.cbits ? static_cast<uint32_t>((tile + priv_round<false>() - 1) / priv_round<false>()) : 0u;
  const uint64_t nrun = static_cast<uint64_t>(kPartBlocks) * L.max_rounds * kRunMaxBins;
  L.run_s = o; o = align_up(o + 4 * nrun, 256);
  L.run_l = o; o = align_up(o + 4 * nrun, 256);
  L.segtot = o; o = align_up(o + 4 * kRunMaxBins, 256);
  L.lcnt = o; o = align_up(o + 4 * (nf + 1), 256);  // ListOut: linked rows per bucket, keyed total
  L.xst = o;
  if (with_sink) o = align_up(o + 4 * static_cast<uint64_t>(kPartBlocks) * kSinkWaves * sink_cap(n), 256);
  L.xcnt = o;
  if (with_sink) o = align_up(o + 4 * kPartBlocks * kSinkWaves, 256);
  L.total = o;
  return L;
}

// Dynamic LDS above the default 64 KiB (cursors of up to 2^15 digits).
template <typename K>
void allow_lds(K kernel, size_t bytes) {
  if (bytes > (size_t(64) << 10))
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(bytes));
}


// K5 over 12-byte records, one workgroup per bucket (nb buckets).  Round 5 measured a persistent,
// LDS-staged variant (one workgroup per CU copying the next bucket's records
// to LDS with global_load_lds while grouping the current one): 2.2x slower
// (it halves the resident workgroups of a VALU-bound kernel; DESIGN.md 4.3,
// commit 1346212).
template <typename Out>
void group12_launch(const uint3* rec, uint32_t rank_base, const uint32_t* offs, uint32_t nb,
                    uint32_t bits, ChunkOf chunk_of, uint64_t* gkey, uint32_t* gmin, const Out& out,
                    hipStream_t s) {
  k_bucket_group12_pk<Out><<<nb, kGroupThreads, 0, s>>>(rec, rank_base, offs, bits, chunk_of, gkey,
                                                        gmin, out);
}

XSink sink_of(const RepOut&) { return XSink{}; }
XSink sink_of(const ListOut& o) { return o.x; }

// A first-pass histogram, with the keyless sink when the output has one
// (RowsIn only: the rows the caller passed).
template <typename In>
void hist_launch(const XSink& xs, size_t lds, hipStream_t s, In in, uint64_t n, uint32_t skip,
                 uint32_t bits, uint32_t* hist, uint32_t* zero = nullptr, bool blk_major = false) {
  const uint32_t P = bucket_part_blocks();
  if constexpr (std::is_same<In, RowsIn>::value) {
    if (xs.st) {
      allow_lds(k_part_hist<In, true>, lds);
      k_part_hist<In, true><<<P, kPartThreads, lds, s>>>(in, n, skip, bits, 0, hist, zero,
                                                         blk_major, xs);
      return;
    }
  }
  allow_lds(k_part_hist<In>, lds);
  k_part_hist<In><<<P, kPartThreads, lds, s>>>(in, n, skip, bits, 0, hist, zero, blk_major);
}

// Two-level partition (n > 4096 x kBucketRows) + group: see group_layout.
// kB2 digit bits per segment in the second pass, kS2-record staging runs, kR2
// rows per thread per round, kP2 blocks per segment.  The second pass's offsets
// come from the coarse pass's fine counts (k_fine_scan; bucket starts scanned
// in the second pass's prologue): no histogram pass over the coarse records.
// kRec12: rows without a rank array (rank = rank_base + row), 12-byte records
// in both passes.
template <typename In, uint32_t kB2, uint32_t kS2, int kR2, uint32_t kP2, bool kRec12 = false,
          uint32_t kF2 = kS2, typename Out>
hipError_t two_level_launch(In in, uint64_t n, const GroupLayout& L, uint32_t chunk_rows,
                            uint32_t* rep, bool init_rep, Out out, void* ws, hipStream_t s,
                            KTimer* timer, uint32_t rank_base = 0) {
  using RecT = typename std::conditional<kRec12, uint3, uint4>::type;
  uint8_t* w = static_cast<uint8_t*>(ws);
  uint32_t* tiles = reinterpret_cast<uint32_t*>(w + L.tiles);
  uint4* rec = reinterpret_cast<uint4*>(w + L.rec);
  uint64_t* gkey = reinterpret_cast<uint64_t*>(w + L.gkey);
  uint32_t* gmin = reinterpret_cast<uint32_t*>(w + L.gmin);
  uint32_t* fine = reinterpret_cast<uint32_t*>(w + L.fine);
  uint32_t* fE = reinterpret_cast<uint32_t*>(w + L.fE);
  uint32_t* ftot = reinterpret_cast<uint32_t*>(w + L.ftot);
  uint32_t* fbase = reinterpret_cast<uint32_t*>(w + L.fbase);
  uint32_t* ovf = reinterpret_cast<uint32_t*>(w + L.ovf);
  const uint32_t bits = L.bits, nfine = 1u << bits;
  const uint32_t P = bucket_part_blocks();
  const uint32_t skip2 = kShardBits + L.cbits;
  static_assert(kMaxBucketBits - kB2 <= 6, "coarse digits fit k_part_scatter_runs");
  static_assert(kP2 <= kPartBlocks && kPartBlocks % kP2 == 0, "second-pass blocks per segment");
  static_assert((1u << kB2) <= kPartThreads, "second-pass bucket starts: one bucket per thread");
  // rounds of the coarse pass in the largest tile (the layout sized the run
  // table for 4096-row rounds, the most this variant can have)
  const uint64_t tile = (n + P - 1) / P;
  const uint32_t mr = static_cast<uint32_t>((tile + priv_round<kRec12>() - 1) / priv_round<kRec12>());
  if (kPartBlocks / kP2 * mr <= kMaxRuns) {
    // no histogram pass: the coarse pass writes each block's records into its
    // own tile range as runs, the second pass reads segments as run lists
    uint32_t* run_s = reinterpret_cast<uint32_t*>(w + L.run_s);
    uint32_t* run_l = reinterpret_cast<uint32_t*>(w + L.run_l);
    uint32_t* segtot = reinterpret_cast<uint32_t*>(w + L.segtot);
    uint4* rec1 = reinterpret_cast<uint4*>(w + L.rec1);
    const uint32_t nseg = 1u << L.cbits;
    k_zero_runs<<<1, 64, 0, s>>>(segtot, ovf);
    {
      KScope k(timer, "bucket_scatter1", s);
      bool sunk = false;
      if constexpr (std::is_same<In, RowsIn>::value) {
        const XSink xs = sink_of(out);
        if (xs.st) {
          k_part_private<In, false, kRec12, true><<<P, kPartThreads, 0, s>>>(
              in, n, kShardBits, L.cbits, rec1, rep, bits, fine, ovf, run_s, run_l, mr,
              segtot, xs);
          sunk = true;
        }
      }
      if (sunk) {
      } else if (init_rep) {
        k_part_private<In, true, kRec12><<<P, kPartThreads, 0, s>>>(
            in, n, kShardBits, L.cbits, rec1, rep, bits, fine, ovf, run_s, run_l, mr, segtot);
      } else {
        k_part_private<In, false, kRec12><<<P, kPartThreads, 0, s>>>(
            in, n, kShardBits, L.cbits, rec1, rep, bits, fine, ovf, run_s, run_l, mr, segtot);
      }
    }
    {
      KScope k(timer, "bucket_fine_scan", s);
      k_fine_recount_runs<kB2, RecT><<<kPartBlocks, kPartThreads, 0, s>>>(
          reinterpret_cast<const RecT*>(rec1), skip2, run_s, run_l, mr, P, nseg, bits, fine,
          ovf);
      k_fine_scan<kP2, kPartBlocks / kP2><<<(nfine + 63) / 64, 1024, 0, s>>>(fine, nfine, fE, ftot, ovf);
    }
    // second pass over all segments, then the group-by over all buckets.
    // (Round 5 tried the two interleaved per group of segments, so the group
    // kernel would read records still in the Infinity Cache: slower at every
    // G, 1.807 -> 1.831-1.990 ms at 100 M rows, and removed in round 6 --
    // DESIGN.md 4.3, "segment groups".)
    {
      KScope k(timer, "bucket_scatter", s);
      k_part2_runs<kRec12, kB2, kS2, kR2, kF2><<<dim3(kP2, nseg), kPartThreads, 0, s>>>(
          rec1, skip2, fE, rec, run_s, run_l, mr, P, kPartBlocks / kP2, segtot, ftot, fbase);
    }
    KScope k(timer, "bucket_group", s);
    if constexpr (kRec12)
      group12_launch(reinterpret_cast<const uint3*>(rec), rank_base, fbase, nfine, bits,
                     ChunkOf::make(chunk_rows), gkey, gmin, out, s);
    else
      k_bucket_group_pk<Out><<<nfine, kGroupThreads, 0, s>>>(rec, fbase, 1, bits,
                                                             ChunkOf::make(chunk_rows), gkey, gmin, out);
    return out_finish(out, nfine, s);
  }
  // pass 1: coarse partition on the top cbits digit bits (rep initialised
  // here), counting every row's final bucket on the way
  uint32_t* hist1 = reinterpret_cast<uint32_t*>(w + L.hist1);
  uint4* rec1 = reinterpret_cast<uint4*>(w + L.rec1);
  const uint32_t nseg = 1u << L.cbits;
  const size_t lds1 = sizeof(uint32_t) << L.cbits;
  {
    KScope k(timer, "bucket_hist", s);
    hist_launch(sink_of(out), lds1, s, in, n, kShardBits, L.cbits, hist1, ovf);
  }
  scan::exclusive(hist1, static_cast<uint64_t>(nseg) * P, hist1, tiles, nullptr, s);
  {
    KScope k(timer, "bucket_scatter1", s);
    if (init_rep)
      k_part_scatter_runs<In, true, kRec12><<<P, kPartThreads, 0, s>>>(
          in, n, kShardBits, L.cbits, hist1, rec1, rep, bits, fine, ovf);
    else
      k_part_scatter_runs<In, false, kRec12><<<P, kPartThreads, 0, s>>>(
          in, n, kShardBits, L.cbits, hist1, rec1, rep, bits, fine, ovf);
  }
  // pass 2: kB2 bits below, per coarse segment, staged in kS2-record runs
  using In2 = typename std::conditional<kRec12, Rec12In, Rec16In>::type;
  In2 in2;
  if constexpr (kRec12)
    in2 = Rec12In{reinterpret_cast<const uint3*>(rec1), rank_base};
  else
    in2 = Rec16In{rec1};
  constexpr uint32_t P2 = kP2;
  {
    KScope k(timer, "bucket_fine_scan", s);
    k_fine_recount<kB2, RecT><<<kPartBlocks, kPartThreads, 0, s>>>(
        reinterpret_cast<const RecT*>(rec1), skip2, hist1, P, nseg, bits, fine, ovf);
    k_fine_scan<P2, kPartBlocks / kP2><<<(nfine + 63) / 64, 1024, 0, s>>>(fine, nfine, fE, ftot,
                                                                          ovf);
  }
  {
    KScope k(timer, "bucket_scatter", s);
    k_part_scatter_rec_staged<In2, false, kB2, kS2, kR2, kRec12>
        <<<dim3(P2, nseg), kPartThreads, 0, s>>>(in2, 0, skip2, fE, rec, nullptr, hist1, P, ftot,
                                                 fbase, kPartBlocks / kP2);
  }
  KScope k(timer, "bucket_group", s);
  if constexpr (kRec12)
    group12_launch(reinterpret_cast<const uint3*>(rec), rank_base, fbase, nfine, bits,
                   ChunkOf::make(chunk_rows), gkey, gmin, out, s);
  else
    k_bucket_group_pk<Out><<<nfine, kGroupThreads, 0, s>>>(rec, fbase, 1, bits,
                                                           ChunkOf::make(chunk_rows), gkey, gmin, out);
  return out_finish(out, nfine, s);
}

// Rows whose bucket records can be 12 bytes {hash, z} with rank = rank_base
// + z: the caller's rows without a rank array (z = row), and received
// exchange records for an output that needs no row (RecRankIn: z = rank).
template <typename In>
bool rank_in_z(const In& in) {
  if constexpr (std::is_same<In, RowsIn>::value) return !in.rank;
  else return std::is_same<In, RecRankIn>::value;
}
template <typename In>
uint32_t z_rank_base(const In& in) {
  if constexpr (std::is_same<In, RowsIn>::value) return in.rank_base;
  else return 0u;
}

template <typename In, typename Out>
hipError_t group_launch(In in, uint64_t n, uint32_t chunk_rows, uint32_t* rep, bool init_rep,
                        Out out, void* ws, hipStream_t s, KTimer* timer, uint64_t bits_rows = 0) {
  const GroupLayout L = group_layout(n, bits_rows, sink_of(out).st != nullptr);
  uint8_t* w = static_cast<uint8_t*>(ws);
  uint32_t* hist = reinterpret_cast<uint32_t*>(w + L.hist);
  uint32_t* tiles = reinterpret_cast<uint32_t*>(w + L.tiles);
  uint4* rec = reinterpret_cast<uint4*>(w + L.rec);
  uint64_t* gkey = reinterpret_cast<uint64_t*>(w + L.gkey);
  uint32_t* gmin = reinterpret_cast<uint32_t*>(w + L.gmin);
  const uint32_t bits = L.bits;
  const uint32_t P = bucket_part_blocks();
  const uint64_t nh = (static_cast<uint64_t>(1) << bits) * P;
  const size_t lds = sizeof(uint32_t) << bits;
  if (L.cbits) {
    if constexpr (std::is_same<In, RowsIn>::value || std::is_same<In, RecRankIn>::value) {
      if (rank_in_z(in))  // 12-byte records
        return two_level_launch<In, kStage2Bits, kStage2Slots, kStage2Rows, kStage2Blocks, true,
                                kStage2Slots>(in, n, L, chunk_rows, rep, init_rep, out, ws, s,
                                              timer, z_rank_base(in));
    }
    return two_level_launch<In, kStage2Bits, kStage2Slots, kStage2Rows, kStage2Blocks, false,
                            kStage2Slots>(in, n, L, chunk_rows, rep, init_rep, out, ws, s, timer);
  }
  if (bits == kStageBits) {
    // 12-bit digits: block-major counts, k_fine_scan for every block's start
    // inside every bucket (one launch instead of the 3-launch scan), bucket
    // starts scanned in the staged scatter's prologue
    uint32_t* fine = reinterpret_cast<uint32_t*>(w + L.fine);
    uint32_t* fE = reinterpret_cast<uint32_t*>(w + L.fE);
    uint32_t* ftot = reinterpret_cast<uint32_t*>(w + L.ftot);
    uint32_t* fbase = reinterpret_cast<uint32_t*>(w + L.fbase);
    uint32_t* ovf = reinterpret_cast<uint32_t*>(w + L.ovf);
    const uint32_t nb = 1u << kStageBits;
    static_assert(kPartBlocks % 16 == 0, "k_fine_scan: blocks per thread");
    {
      KScope k(timer, "bucket_hist", s);
      hist_launch(sink_of(out), lds, s, in, n, kShardBits, bits, fine, nullptr, true);
      k_fine_scan<kPartBlocks, 1><<<nb / 64, 1024, 0, s>>>(fine, nb, fE, ftot, ovf);
    }
    if constexpr (std::is_same<In, RowsIn>::value || std::is_same<In, RecRankIn>::value) {
      if (rank_in_z(in)) {  // rank = rank_base + z: 12-byte records
        {
          KScope k(timer, "bucket_scatter", s);
          uint3* rec12 = reinterpret_cast<uint3*>(rec);
          if (init_rep) {
            if constexpr (std::is_same<In, RowsIn>::value)
              k_part_scatter_ws<In, true><<<P, kPartThreads, 0, s>>>(in, n, kShardBits, fE, ftot,
                                                                     rec12, rep, fbase);
          } else {
            k_part_scatter_ws<In, false><<<P, kPartThreads, 0, s>>>(in, n, kShardBits, fE, ftot,
                                                                    rec12, rep, fbase);
          }
        }
        KScope k(timer, "bucket_group", s);
        group12_launch(reinterpret_cast<const uint3*>(rec), z_rank_base(in), fbase, nb, kStageBits,
                       ChunkOf::make(chunk_rows), gkey, gmin, out, s);
        return out_finish(out, nb, s);
      }
    }
    {
      KScope k(timer, "bucket_scatter", s);
      if (init_rep)
        k_part_scatter_rec_staged<In, true><<<P, kPartThreads, 0, s>>>(
            in, n, kShardBits, fE, rec, rep, nullptr, 0, ftot, fbase);
      else
        k_part_scatter_rec_staged<In, false><<<P, kPartThreads, 0, s>>>(
            in, n, kShardBits, fE, rec, rep, nullptr, 0, ftot, fbase);
    }
    KScope k(timer, "bucket_group", s);
    k_bucket_group_pk<Out><<<nb, kGroupThreads, 0, s>>>(rec, fbase, 1, kStageBits,
                                                        ChunkOf::make(chunk_rows), gkey, gmin, out);
    return out_finish(out, nb, s);
  }
  {
    KScope k(timer, "bucket_hist", s);
    hist_launch(sink_of(out), lds, s, in, n, kShardBits, bits, hist);
  }
  scan::exclusive(hist, nh, hist, tiles, nullptr, s);
  {
    KScope k(timer, "bucket_scatter", s);
    if (init_rep) {
      allow_lds(k_part_scatter_rec<In, true>, lds);
      k_part_scatter_rec<In, true><<<P, kPartThreads, lds, s>>>(in, n, kShardBits, bits, hist, rec,
                                                                rep);
    } else {
      allow_lds(k_part_scatter_rec<In, false>, lds);
      k_part_scatter_rec<In, false><<<P, kPartThreads, lds, s>>>(in, n, kShardBits, bits, hist,
                                                                 rec, rep);
    }
  }
  KScope k(timer, "bucket_group", s);
  k_bucket_group<Out><<<1u << bits, kGroupThreads, 0, s>>>(rec, hist, P, ChunkOf::make(chunk_rows),
                                                           gkey, gmin, out);
  return out_finish(out, 1u << bits, s);
}

size_t shard_hist_bytes(uint32_t shard_bits) {
  const uint64_t nh = (static_cast<uint64_t>(1) << shard_bits) * kPartBlocks;
  return align_up(4 * (nh + 1), 256);
}

// Shard histogram + scan (+ scatter when outputs are given) of the caller's
// rows; digit = destination rank when world != 0, else the top shard_bits.
hipError_t shard_partition(const RowsIn& in, uint64_t n, uint32_t shard_bits, uint32_t world,
                           uint32_t* hist, uint32_t* tiles, uint64_t* okey, uint32_t* orank,
                           uint3* orec, uint32_t* opos, hipStream_t s, KTimer* timer) {
  const uint32_t nbins = world ? world : 1u << shard_bits;
  const uint64_t nh = static_cast<uint64_t>(nbins) * kPartBlocks;
  const size_t lds = sizeof(uint32_t) * nbins;
  {
    KScope k(timer, "shard_hist", s);
    k_part_hist<RowsIn><<<kPartBlocks, kPartThreads, lds, s>>>(in, n, 0, shard_bits, world, hist);
  }
  scan::exclusive(hist, nh, hist, tiles, nullptr, s);
  if (opos || orec) {
    KScope k(timer, "shard_scatter", s);
    if (orec)
      k_part_scatter<RowsIn, true><<<kPartBlocks, kPartThreads, lds, s>>>(
          in, n, 0, shard_bits, world, hist, nullptr, nullptr, orec, opos);
    else
      k_part_scatter<RowsIn, false><<<kPartBlocks, kPartThreads, lds, s>>>(
          in, n, 0, shard_bits, world, hist, okey, orank, nullptr, opos);
  }
  return hipGetLastError();
}

}  // namespace

size_t dedup_workspace_bytes(uint64_t n, bool with_sink) {
  return group_layout(n, 0, with_sink).total;
}

hipError_t dedup_local_launch(const GroupInput& in, uint32_t chunk_rows, uint32_t* rep,
                              bool init_rep, void* ws, hipStream_t s, KTimer* timer) {
  if (in.n == 0) return hipSuccess;
  if (in.rec12)
    return group_launch(RecIn{reinterpret_cast<const uint3*>(in.rec12), in.valid}, in.n,
                        chunk_rows, rep, init_rep, RepOut{rep}, ws, s, timer, in.bits_rows);
  return group_launch(RowsIn{in.key, in.valid, in.rank, in.rank_base}, in.n, chunk_rows, rep,
                      init_rep, RepOut{rep}, ws, s, timer, in.bits_rows);
}

hipError_t dedup_list_launch(const GroupInput& in, uint32_t chunk_rows, uint32_t* who,
                             uint32_t* obj, uint32_t* counts, void* ws, hipStream_t s,
                             KTimer* timer, bool sink_keyless, const uint8_t* keyless_valid,
                             uint32_t cap, uint32_t* nospc, const KeylessSink* moved) {
  if (in.n == 0) return hipSuccess;
  uint8_t* w = static_cast<uint8_t*>(ws);
  const bool sink = sink_keyless && !in.rec12 && in.valid;
  const GroupLayout L = group_layout(in.n, in.bits_rows, sink);
  ListOut out{who, obj, counts, reinterpret_cast<uint32_t*>(w + L.lcnt), XSink{}};
  if (nospc) {
    out.cap = cap;
    out.nospc = nospc;
  }
  if (sink) {
    out.x.valid = keyless_valid;
    out.x.st = reinterpret_cast<uint32_t*>(w + L.xst);
    out.x.cnt = reinterpret_cast<uint32_t*>(w + L.xcnt);
    out.x.cap = sink_cap(in.n);
  } else if (moved) {  // segments filled by the exchange's partition (k_part_padded)
    out.x.valid = moved->valid;
    out.x.st = moved->st;
    out.x.cnt = moved->cnt;
    out.x.cap = moved->cap;
  }
  if (in.rec12)  // the list needs no row index: 12-byte bucket records carrying the rank
    return group_launch(RecRankIn{{reinterpret_cast<const uint3*>(in.rec12), in.valid}}, in.n,
                        chunk_rows, nullptr, false, out, ws, s, timer, in.bits_rows);
  return group_launch(RowsIn{in.key, in.valid, in.rank, in.rank_base}, in.n, chunk_rows, nullptr,
                      false, out, ws, s, timer, in.bits_rows);
}

size_t shard_workspace_bytes(uint32_t shard_bits) {
  const uint64_t nh = (static_cast<uint64_t>(1) << shard_bits) * kPartBlocks;
  return shard_hist_bytes(shard_bits) + align_up(4 * (scan::tiles_for(nh) + 1), 256) +
         align_up(8 * (static_cast<uint64_t>(1) << shard_bits), 256);
}

hipError_t shard_count_launch(const uint64_t* key, const uint8_t* has_key, uint64_t n,
                              uint32_t shard_bits, uint64_t* d_counts, void* ws, hipStream_t s) {
  uint8_t* w = static_cast<uint8_t*>(ws);
  uint32_t* hist = reinterpret_cast<uint32_t*>(w);
  uint32_t* tiles = reinterpret_cast<uint32_t*>(w + shard_hist_bytes(shard_bits));
  hipError_t e = shard_partition(RowsIn{key, has_key, nullptr, 0}, n, shard_bits, 0, hist, tiles,
                                 nullptr, nullptr, nullptr, nullptr, s, nullptr);
  if (e != hipSuccess) return e;
  k_copy_counts<<<1, 256, 0, s>>>(hist, 1u << shard_bits, d_counts);
  return hipGetLastError();
}

hipError_t shard_partition_launch(const uint64_t* key, const uint8_t* has_key,
                                  const uint32_t* rank, uint64_t n, uint32_t shard_bits,
                                  uint64_t* out_key, uint32_t* out_rank, uint32_t* out_pos,
                                  void* ws, hipStream_t s, KTimer* timer) {
  uint8_t* w = static_cast<uint8_t*>(ws);
  uint32_t* hist = reinterpret_cast<uint32_t*>(w);
  uint32_t* tiles = reinterpret_cast<uint32_t*>(w + shard_hist_bytes(shard_bits));
  return shard_partition(RowsIn{key, has_key, rank, 0}, n, shard_bits, 0, hist, tiles, out_key,
                         out_rank, nullptr, out_pos, s, timer);
}

hipError_t shard_exchange_launch(const uint64_t* key, const uint8_t* has_key,
                                 const uint32_t* rank, uint64_t n, uint32_t shard_bits,
                                 uint32_t world, uint64_t* out_key, uint32_t* out_rank,
                                 uint32_t* out_rec12, uint32_t* out_pos, int64_t* d_dest_counts,
                                 void* ws, hipStream_t s, KTimer* timer, int64_t* d_count_msgs,
                                 int64_t msg_code) {
  uint8_t* w = static_cast<uint8_t*>(ws);
  uint32_t* hist = reinterpret_cast<uint32_t*>(w);
  uint32_t* tiles = reinterpret_cast<uint32_t*>(w + shard_hist_bytes(shard_bits));
  hipError_t e = shard_partition(RowsIn{key, has_key, rank, 0}, n, shard_bits, world, hist, tiles,
                                 out_key, out_rank, reinterpret_cast<uint3*>(out_rec12), out_pos,
                                 s, timer);
  if (e != hipSuccess) return e;
  k_dest_counts<<<1, 64, 0, s>>>(hist, world, d_dest_counts, d_count_msgs,
                                 static_cast<int64_t>(n), msg_code);
  return hipGetLastError();
}

uint32_t ret_tiles(const RetTiles& st) { return st.tstart[st.world]; }

size_t ret_workspace_bytes(uint32_t tiles) {
  return align_up(4ull * (tiles + 2), 256) + align_up(4ull * (scan::tiles_for(tiles + 1) + 1), 256);
}

hipError_t ret_compact_launch(const RetTiles& st, const uint32_t* rrec, const uint32_t* rrep,
                              uint2* ret, int64_t* retcnt, void* ws, hipStream_t s, KTimer* timer) {
  const uint32_t nt = st.tstart[st.world];
  uint8_t* b = static_cast<uint8_t*>(ws);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(b);
  uint32_t* tiles = reinterpret_cast<uint32_t*>(b + align_up(4ull * (nt + 2), 256));
  KScope k(timer, "ret_compact", s);
  const uint32_t g = nt ? nt : 1;  // one block writes the (zero) counts of an empty receive
  const uint3* rr = reinterpret_cast<const uint3*>(rrec);
  if (nt) {
    k_ret_count<<<nt, kRetThreads, 0, s>>>(st, rr, rrep, cnt);
    scan::exclusive(cnt, nt, cnt, tiles, nullptr, s);
  } else {
    const hipError_t e = hipMemsetAsync(cnt, 0, 4, s);
    if (e != hipSuccess) return e;
  }
  k_ret_write<<<g, kRetThreads, 0, s>>>(st, rr, rrep, cnt, ret, retcnt);
  return hipGetLastError();
}

hipError_t ret_apply_launch(const RetApply& ap, const uint2* rback, uint32_t* back,
                            uint64_t n_back, const uint32_t* srec12, hipStream_t s) {
  if (n_back) {
    const uint64_t g = std::min<uint64_t>((n_back + 255) / 256, 16384);
    k_back_init<<<static_cast<uint32_t>(g), 256, 0, s>>>(reinterpret_cast<const uint3*>(srec12),
                                                         n_back, back);
  }
  const uint64_t total = ap.poff[ap.world];
  if (total) {
    const uint64_t g = std::min<uint64_t>((total + 255) / 256, 16384);
    k_ret_apply<<<static_cast<uint32_t>(g), 256, 0, s>>>(ap, rback, back);
  }
  return hipGetLastError();
}

hipError_t gather_rep_launch(const uint32_t* back, const uint32_t* pos, const uint32_t* rank,
                             uint64_t n, uint32_t* rep, hipStream_t s, const uint32_t* self,
                             uint64_t self_lo, uint64_t self_hi) {
  if (n) {
    const uint64_t g = std::min<uint64_t>((n + 255) / 256, 16384);
    k_gather_rep<<<static_cast<uint32_t>(g), 256, 0, s>>>(
        back, pos, rank, n, rep, self ? self : back, static_cast<uint32_t>(self_lo),
        static_cast<uint32_t>(self ? self_hi : self_lo));
  }
  return hipGetLastError();
}

hipError_t padded_partition_launch(const uint64_t* key, const uint8_t* has_key,
                                   const uint32_t* rank, uint64_t n, uint32_t world, uint32_t me,
                                   uint32_t cap, uint32_t* out_rec12, uint32_t* self_rec12,
                                   uint32_t* out_pos, uint32_t* cursor, const KeylessSink* sink,
                                   hipStream_t s, KTimer* timer) {
  XSink xs{};
  if (sink) {
    xs.valid = sink->valid;
    xs.st = sink->st;
    xs.cnt = sink->cnt;
    xs.cap = sink->cap;
  }
  if (n) {
    KScope k(timer, "shard_padded", s);
    k_part_padded<<<kPartBlocks, kPartThreads, 0, s>>>(
        RowsIn{key, has_key, rank, 0}, n, world, me, cap, reinterpret_cast<uint3*>(out_rec12),
        reinterpret_cast<uint3*>(self_rec12), out_pos, cursor, xs);
  } else if (sink) {  // no rows: the segments are empty
    const hipError_t e =
        hipMemsetAsync(sink->cnt, 0, 4ull * keyless_sink_segments(), s);
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}

uint32_t keyless_sink_segments() { return kPartBlocks * kSinkWaves; }
uint32_t keyless_sink_cap(uint64_t n) { return sink_cap(n); }

hipError_t pad_fill_launch(const uint32_t* cursor, uint32_t world, uint32_t me, uint32_t cap,
                           uint64_t n, uint32_t* rec12, uint32_t* self_rec12, uint32_t* summary,
                           uint32_t* zero3, uint32_t* next_cursor, hipStream_t s) {
  const uint32_t bx = std::min<uint32_t>(64u, (cap + 1023u) / 1024u + 1u);
  k_pad_fill<<<dim3(bx, world), 256, 0, s>>>(cursor, world, me, cap, static_cast<uint32_t>(n),
                                             reinterpret_cast<uint3*>(rec12),
                                             reinterpret_cast<uint3*>(self_rec12), summary, zero3,
                                             next_cursor);
  return hipGetLastError();
}

hipError_t recv_summary_launch(const uint32_t* rrec12, uint32_t world, uint32_t cap,
                               uint32_t* summary, hipStream_t s) {
  k_recv_summary<<<1, 64, 0, s>>>(reinterpret_cast<const uint3*>(rrec12), world, cap, summary);
  return hipGetLastError();
}

hipError_t scatter_rep_launch(const uint32_t* src, const uint32_t* pos, uint64_t n, uint32_t* dst,
                              uint64_t n_dst, const uint32_t* init, bool do_init, hipStream_t s) {
  if (do_init && n_dst) {
    const uint64_t g = std::min<uint64_t>((n_dst + 255) / 256, 16384);
    k_fill_init<<<static_cast<uint32_t>(g), 256, 0, s>>>(dst, n_dst, init);
  }
  if (n) {
    const uint64_t g = std::min<uint64_t>((n + 255) / 256, 16384);
    k_scatter<<<static_cast<uint32_t>(g), 256, 0, s>>>(src, pos, n, dst);
  }
  return hipGetLastError();
}

}  // namespace sdgpu
