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

// Row sources: (key, rank, keyed?) of row i.
//   RowsIn: the caller's rows -- key[i], valid[i] (null: all keyed), rank[i]
//           (null: rank_base + i);
//   RecIn:  packed 12-byte exchange records {key lo, key hi, rank} as received
//           from the other GPUs, valid[i] optional (the Object-index probe's mask).
//   Rec16In: 16-byte bucket records {key lo, key hi, rank, row} of a first
//           partition pass (the row is carried, not the position).
// get_row also returns the row whose rep the record answers for.
struct RowsIn {
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
};
struct RecIn {
  const uint3* rec;
  const uint8_t* valid;
  __device__ __forceinline__ void get(uint64_t i, uint64_t& k, uint32_t& r, bool& v) const {
    const uint3 q = rec[i];
    k = (static_cast<uint64_t>(q.y) << 32) | q.x;
    r = q.z;
    v = !valid || valid[i] != 0;
  }
  __device__ __forceinline__ void get_row(uint64_t i, uint64_t& k, uint32_t& r, uint32_t& row,
                                          bool& v) const {
    get(i, k, r, v);
    row = static_cast<uint32_t>(i);
  }
};
struct Rec16In {
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
};

}  // namespace sdgpu
