// Device-side row access shared by the grouping (dedup.hip) and the Object
// index (index.hip): the key hash and the two row layouts the kernels read.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sdgpu {

// splitmix64 finalizer: the partition digits, LDS slots and index slots of a
// key.  cas keys are already uniform; the mix makes the layout independent of
// the caller's key distribution (tests use small integers).
__device__ __forceinline__ uint64_t row_hash(uint64_t z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// floor(r / d) for a runtime divisor d, without the ~40-instruction integer
// division: m = floor((2^64 - 1) / d) + 1 = ceil(2^64 / d) and
// floor(r / d) = (m * r) >> 64 for every 32-bit r (Lemire, Kaser, Kurz 2019);
// m = 0 encodes d = 1.
struct ChunkOf {
  uint64_t m;
  static ChunkOf make(uint32_t d) { return ChunkOf{d <= 1 ? 0ull : ~0ull / d + 1}; }
  __device__ __forceinline__ uint32_t operator()(uint32_t r) const {
    if (m == 0) return r;
    const uint64_t lo = static_cast<uint64_t>(static_cast<uint32_t>(m)) * r;
    const uint64_t hi = (m >> 32) * r;
    return static_cast<uint32_t>((hi + (lo >> 32)) >> 32);
  }
};

// Row sources: (key, rank, keyed?) of row i.  kHashed: the source already
// carries row_hash(key) in place of the key (the bucket records: row_hash is a
// bijection, so equal hashes are equal keys and the grouping reads the hash).
//   RowsIn: the caller's rows -- key[i], valid[i] (null: all keyed), rank[i]
//           (null: rank_base + i);
//   RecIn:  packed 12-byte exchange records {key lo, key hi, rank} as received
//           from the other GPUs, valid[i] optional (the Object-index probe's mask).
//   Rec16In: 16-byte bucket records {hash lo, hash hi, rank, row} of a first
//           partition pass (the row is carried, not the position).
// get / get_row read one row (get_row also returns the row whose rep the
// record answers for).  The partition kernels read U rows per thread with
// load_many into a RowBatch: every load is issued, and nothing derived from a
// loaded value is computed, before the batch is used (key_of / rank_of /
// valid_of resolve a row at its use) -- guarded one-row reads, or a validity
// test right after the byte load, made the compiler wait out each row's
// memory latency in turn.  Rows at or past `end` read row `safe` (in = false).
template <int U>
struct RowBatch {
  uint64_t k[U];
  uint32_t a[U];    // rank as loaded (RowsIn with rank / records)
  uint32_t b[U];    // valid byte as loaded (RowsIn / RecIn), or the record's row
  uint32_t row[U];  // the row index read
  bool in[U];
};

template <int U>
__device__ __forceinline__ void batch_index(uint64_t i0, uint64_t stride, uint64_t end,
                                            uint64_t safe, RowBatch<U>& q) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t i = i0 + static_cast<uint64_t>(u) * stride;
    q.in[u] = i < end;
    q.row[u] = static_cast<uint32_t>(q.in[u] ? i : safe);
  }
}

struct RowsIn {
  static constexpr bool kHashed = false;
  const uint64_t* key;
  const uint8_t* valid;
  const uint32_t* rank;
  uint32_t rank_base;
  __device__ __forceinline__ void get(uint64_t i, uint64_t& k, uint32_t& r, bool& v) const {
    k = key[i];
    r = rank ? rank[i] : rank_base + static_cast<uint32_t>(i);
    v = !valid || valid[i] != 0;
  }
  __device__ __forceinline__ void get_row(uint64_t i, uint64_t& k, uint32_t& r, uint32_t& row,
                                          bool& v) const {
    get(i, k, r, v);
    row = static_cast<uint32_t>(i);
  }
  // null rank / valid: the load reads the row's own key word instead (the
  // line its key load brings in) and the value is replaced at use, so the
  // batch has no branch.  (Indexing the key array as a u32 / u8 array by row
  // read a DIFFERENT line, the first half / eighth of the key array: +4 B of
  // HBM per row, 1.30 GB fetched per 100 M-row coarse pass for 0.9 GB of
  // rows, profiles/r3/prof_r3J/pmc_dedup_full.txt.)
  template <int U>
  __device__ __forceinline__ void load_many(uint64_t i0, uint64_t stride, uint64_t end,
                                            uint64_t safe, RowBatch<U>& q) const {
    batch_index(i0, stride, end, safe, q);
    const uint32_t* ka = reinterpret_cast<const uint32_t*>(key);
#pragma unroll
    for (int u = 0; u < U; ++u) q.k[u] = key[q.row[u]];
#pragma unroll
    for (int u = 0; u < U; ++u)
      q.a[u] = *(rank ? rank + q.row[u] : ka + 2ull * q.row[u]);
#pragma unroll
    for (int u = 0; u < U; ++u)
      q.b[u] = *(valid ? valid + q.row[u] : reinterpret_cast<const uint8_t*>(ka + 2ull * q.row[u]));
  }
  template <int U>
  __device__ __forceinline__ uint64_t key_of(const RowBatch<U>& q, int u) const { return q.k[u]; }
  template <int U>
  __device__ __forceinline__ uint32_t rank_of(const RowBatch<U>& q, int u) const {
    return rank ? q.a[u] : rank_base + q.row[u];
  }
  template <int U>
  __device__ __forceinline__ bool valid_of(const RowBatch<U>& q, int u) const {
    return q.in[u] && (!valid || (q.b[u] & 0xFFu) != 0);
  }
  template <int U>
  __device__ __forceinline__ uint32_t row_of(const RowBatch<U>& q, int u) const {
    return q.row[u];
  }
};
// A record whose rank is kPadRank is not a row: the padding and the header
// slot of a fixed-capacity exchange message (shard.cpp).  Row ranks are below
// 2^31 on every path that builds records, so no row carries it.
constexpr uint32_t kPadRank = 0xFFFFFFFFu;

struct RecIn {
  static constexpr bool kHashed = false;
  const uint3* rec;
  const uint8_t* valid;
  __device__ __forceinline__ void get(uint64_t i, uint64_t& k, uint32_t& r, bool& v) const {
    const uint3 q = rec[i];
    k = (static_cast<uint64_t>(q.y) << 32) | q.x;
    r = q.z;
    v = q.z != kPadRank && (!valid || valid[i] != 0);
  }
  __device__ __forceinline__ void get_row(uint64_t i, uint64_t& k, uint32_t& r, uint32_t& row,
                                          bool& v) const {
    get(i, k, r, v);
    row = static_cast<uint32_t>(i);
  }
  template <int U>
  __device__ __forceinline__ void load_many(uint64_t i0, uint64_t stride, uint64_t end,
                                            uint64_t safe, RowBatch<U>& q) const {
    batch_index(i0, stride, end, safe, q);
    uint3 t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) t[u] = rec[q.row[u]];
#pragma unroll
    for (int u = 0; u < U; ++u)  // null valid: the record's own line (see RowsIn)
      q.b[u] = *(valid ? valid + q.row[u] : reinterpret_cast<const uint8_t*>(rec + q.row[u]));
#pragma unroll
    for (int u = 0; u < U; ++u) {
      q.k[u] = (static_cast<uint64_t>(t[u].y) << 32) | t[u].x;
      q.a[u] = t[u].z;
    }
  }
  template <int U>
  __device__ __forceinline__ uint64_t key_of(const RowBatch<U>& q, int u) const { return q.k[u]; }
  template <int U>
  __device__ __forceinline__ uint32_t rank_of(const RowBatch<U>& q, int u) const { return q.a[u]; }
  template <int U>
  __device__ __forceinline__ bool valid_of(const RowBatch<U>& q, int u) const {
    return q.in[u] && q.a[u] != kPadRank && (!valid || (q.b[u] & 0xFFu) != 0);
  }
  template <int U>
  __device__ __forceinline__ uint32_t row_of(const RowBatch<U>& q, int u) const {
    return q.row[u];
  }
};
// RecRankIn: exchange records grouped for an output that needs no row index
// (the Object write set, ListOut): the 12-byte bucket records carry the RANK
// in their third word (rank_base 0), so the owner's partition moves 12 bytes
// per row instead of 16 (the Rec12 paths of dedup.hip).
struct RecRankIn : RecIn {
  template <int U>
  __device__ __forceinline__ uint32_t row_of(const RowBatch<U>& q, int u) const {
    return q.a[u];
  }
};
struct Rec16In {
  static constexpr bool kHashed = true;
  const uint4* rec;
  __device__ __forceinline__ void get(uint64_t i, uint64_t& k, uint32_t& r, bool& v) const {
    const uint4 q = rec[i];
    k = (static_cast<uint64_t>(q.y) << 32) | q.x;
    r = q.z;
    v = true;
  }
  __device__ __forceinline__ void get_row(uint64_t i, uint64_t& k, uint32_t& r, uint32_t& row,
                                          bool& v) const {
    const uint4 q = rec[i];
    k = (static_cast<uint64_t>(q.y) << 32) | q.x;
    r = q.z;
    row = q.w;
    v = true;
  }
  template <int U>
  __device__ __forceinline__ void load_many(uint64_t i0, uint64_t stride, uint64_t end,
                                            uint64_t safe, RowBatch<U>& q) const {
    batch_index(i0, stride, end, safe, q);
    uint4 t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) t[u] = rec[q.row[u]];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      q.k[u] = (static_cast<uint64_t>(t[u].y) << 32) | t[u].x;
      q.a[u] = t[u].z;
      q.b[u] = t[u].w;
    }
  }
  template <int U>
  __device__ __forceinline__ uint64_t key_of(const RowBatch<U>& q, int u) const { return q.k[u]; }
  template <int U>
  __device__ __forceinline__ uint32_t rank_of(const RowBatch<U>& q, int u) const { return q.a[u]; }
  template <int U>
  __device__ __forceinline__ bool valid_of(const RowBatch<U>& q, int u) const { return q.in[u]; }
  template <int U>
  __device__ __forceinline__ uint32_t row_of(const RowBatch<U>& q, int u) const { return q.b[u]; }
};

// Rec12In: 12-byte bucket records {hash lo, hash hi, row} of a first pass over
// rows without a rank array (rank = rank_base + row).
struct Rec12In {
  static constexpr bool kHashed = true;
  const uint3* rec;
  uint32_t rank_base;
  template <int U>
  __device__ __forceinline__ void load_many(uint64_t i0, uint64_t stride, uint64_t end,
                                            uint64_t safe, RowBatch<U>& q) const {
    batch_index(i0, stride, end, safe, q);
    uint3 t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) t[u] = rec[q.row[u]];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      q.k[u] = (static_cast<uint64_t>(t[u].y) << 32) | t[u].x;
      q.b[u] = t[u].z;
    }
  }
  template <int U>
  __device__ __forceinline__ uint64_t key_of(const RowBatch<U>& q, int u) const { return q.k[u]; }
  template <int U>
  __device__ __forceinline__ uint32_t rank_of(const RowBatch<U>& q, int u) const {
    return rank_base + q.b[u];
  }
  template <int U>
  __device__ __forceinline__ bool valid_of(const RowBatch<U>& q, int u) const { return q.in[u]; }
  template <int U>
  __device__ __forceinline__ uint32_t row_of(const RowBatch<U>& q, int u) const { return q.b[u]; }
};

template <typename In>
__device__ __forceinline__ uint64_t in_hash(uint64_t k) {
  if constexpr (In::kHashed) return k;
  else return row_hash(k);
}

}  // namespace sdgpu
