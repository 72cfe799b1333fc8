// Object index: the library-wide "which Object already owns this cas_id"
// lookup of identifier_job_step, on the device.
//
// Reference: file_identifier/mod.rs:168-185 fetches every Object that has a
// file_path whose cas_id is in the step's set (library-wide, across locations
// and earlier runs), and :189-225 links each row whose cas_id matches one of
// them to that Object; only the remaining rows (:233-241) create new Objects.
// A batch grouped in isolation would miss those links, so the grouping of a
// batch first probes this index and then, after the batch, records the keys
// whose Objects it created.  Batches processed in id order then give exactly
// the grouping of the whole run (test_gpu_index.py).
//
// Table: open addressing in HBM, 16-byte slots {key lo, key hi, value, 0},
// linear probing from row_hash(key) & (cap - 1) (four slots per 64-B line, so a
// probe is one line read at load <= 1/2).  Empty slot: key == ~0; the key ~0
// itself lives in a separate special slot.  Inserts: 64-bit agent-scope CAS
// on the key, then atomicMin on the value's slot encoding, so one key keeps
// the first Object in this order: any pre-existing Object (lowest handle)
// before any Object created during the run (lowest rank) -- the reference's
// find_many (mod.rs:168-185) returns Objects already in the database, so an
// Object registered with add_objects wins whatever the call order.  Slot
// encoding: enc = value ^ EXISTING (existing handles map below 2^31, ranks
// above; the empty value 0xFFFFFFFF stays above both).
//
// Values: a row rank r (< 2^31) -- the Object created by row r of this or an
// earlier batch of the same run -- or SDGPU_REP_EXISTING | handle for an
// Object that existed before the run (registered by the caller).  The probe of
// a keyed row r that finds value v writes
//   rep[r] = v                       if v is an existing Object,
//            r  if chunk(r) == chunk(v), else v   (the grouping rule of a6),
// and removes the row from the batch's own grouping; other rows keep rep = r
// and valid = 1.  After the grouping, the rows that created an Object
// (rep == rank) are inserted with their rank.
#include "internal.hpp"
#include "rows_device.hpp"

namespace sdgpu {

namespace {

constexpr uint64_t kEmptyKey = ~0ull;
constexpr int kThreads = 256;

__device__ __forceinline__ uint64_t slot_key(const uint4& q) {
  return (static_cast<uint64_t>(q.y) << 32) | q.x;
}

__device__ __forceinline__ uint32_t enc_value(uint32_t v) { return v ^ kRepExisting; }

// Insert (k, v): keeps the minimum enc_value over inserts (existing Objects
// first).  Returns 1 when k took a new slot (the caller adds those up per wave:
// one atomic per wave on t.count instead of one per key -- same-address
// device atomics serialise at a few ns each).
__device__ __forceinline__ uint32_t index_insert(const IndexRef& t, uint64_t k, uint32_t v) {
  const uint32_t e = enc_value(v);
  if (k == kEmptyKey) {
    atomicMax(&t.special[0], 1u);
    atomicMin(&t.special[1], e);
    return 0;
  }
  uint64_t h = row_hash(k) & (t.cap - 1);
  for (;;) {
    unsigned long long* kp = reinterpret_cast<unsigned long long*>(&t.slots[h]);
    const unsigned long long prev =
        atomicCAS(kp, static_cast<unsigned long long>(kEmptyKey), static_cast<unsigned long long>(k));
    if (prev == kEmptyKey || prev == k) {
      atomicMin(&t.slots[h].z, e);
      return prev == kEmptyKey ? 1u : 0u;
    }
    h = (h + 1) & (t.cap - 1);
  }
}

// after a grid-stride loop (every lane of the wave arrives): the wave's new keys
__device__ __forceinline__ void count_added(const IndexRef& t, uint32_t added) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) added += __shfl_xor(added, d);
  if (__lane_id() == 0 && added) atomicAdd(t.count, static_cast<unsigned long long>(added));
}

// Value of k, or false.
__device__ __forceinline__ bool index_find(const IndexRef& t, uint64_t k, uint32_t& v) {
  if (k == kEmptyKey) {
    v = enc_value(t.special[1]);
    return t.special[0] != 0;
  }
  uint64_t h = row_hash(k) & (t.cap - 1);
  for (;;) {
    const uint4 q = t.slots[h];
    const uint64_t sk = slot_key(q);
    if (sk == k) {
      v = enc_value(q.z);
      return true;
    }
    if (sk == kEmptyKey) return false;
    h = (h + 1) & (t.cap - 1);
  }
}

__global__ __launch_bounds__(kThreads) void k_index_clear(IndexRef t) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x; i < t.cap;
       i += stride)
    t.slots[i] = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *t.count = 0;
    t.special[0] = 0;
    t.special[1] = 0xFFFFFFFFu;
  }
}

// Re-insert every entry of `from` into the (cleared, larger) `to`.
__global__ __launch_bounds__(kThreads) void k_index_rehash(IndexRef from, IndexRef to) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
  uint32_t added = 0;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x; i < from.cap;
       i += stride) {
    const uint4 q = from.slots[i];
    if (slot_key(q) != kEmptyKey) added += index_insert(to, slot_key(q), enc_value(q.z));
  }
  count_added(to, added);
  if (blockIdx.x == 0 && threadIdx.x == 0 && from.special[0]) {
    to.special[0] = 1;
    to.special[1] = from.special[1];
  }
}

// Pre-existing Objects: key[i] -> EXISTING | handle[i], for the keys whose
// shard (top 8 hash bits) belongs to `rank` of `world` (world 1: every key).
__global__ __launch_bounds__(kThreads) void k_index_objects(IndexRef t, const uint64_t* __restrict__ key,
                                                            const uint32_t* __restrict__ handle,
                                                            uint64_t n, uint32_t world,
                                                            uint32_t rank) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
  uint32_t added = 0;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x; i < n;
       i += stride) {
    const uint64_t k = key[i];
    if (world > 1 && ((row_hash(k) >> 56) * world) >> 8 != rank) continue;
    added += index_insert(t, k, kRepExisting | (handle[i] & ~kRepExisting));
  }
  count_added(t, added);
}

template <typename In>
__global__ __launch_bounds__(kThreads) void k_index_probe(IndexRef t, In in, uint64_t n,
                                                          uint32_t chunk_rows,
                                                          uint32_t* __restrict__ rep,
                                                          uint8_t* __restrict__ valid_out) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x; i < n;
       i += stride) {
    uint64_t k;
    uint32_t r;
    bool v;
    in.get(i, k, r, v);
    uint32_t out = r, f;
    bool group = v;
    if (v && index_find(t, k, f)) {
      group = false;
      if (f & kRepExisting) out = f;                         // existing Object (mod.rs:189-225)
      else if (r / chunk_rows != f / chunk_rows) out = f;    // Object of an earlier chunk
    }
    rep[i] = out;
    valid_out[i] = group ? 1 : 0;
  }
}

// After the grouping: rows that created an Object (grouped, rep == rank).
// skip (may be null): *skip != 0 -- the rows of a padded exchange that
// overflowed, whose grouping is re-run through the counted exchange -- inserts
// nothing (the index must not learn creators of an incomplete grouping).
template <typename In>
__global__ __launch_bounds__(kThreads) void k_index_creators(IndexRef t, In in, uint64_t n,
                                                             const uint32_t* __restrict__ rep,
                                                             const uint8_t* __restrict__ grouped,
                                                             const uint32_t* __restrict__ skip) {
  if (skip && *skip) return;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
  uint32_t added = 0;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x; i < n;
       i += stride) {
    if (!grouped[i]) continue;
    uint64_t k;
    uint32_t r;
    bool v;
    in.get(i, k, r, v);
    if (rep[i] == r) added += index_insert(t, k, r);
  }
  count_added(t, added);
}

uint32_t grid_for(uint64_t n) {
  const uint64_t g = (n + kThreads - 1) / kThreads;
  return static_cast<uint32_t>(g == 0 ? 1 : (g < 8192 ? g : 8192));
}

}  // namespace

hipError_t index_clear_launch(const IndexRef& t, hipStream_t s) {
  k_index_clear<<<grid_for(t.cap), kThreads, 0, s>>>(t);
  return hipGetLastError();
}

hipError_t index_rehash_launch(const IndexRef& from, const IndexRef& to, hipStream_t s) {
  k_index_clear<<<grid_for(to.cap), kThreads, 0, s>>>(to);
  k_index_rehash<<<grid_for(from.cap), kThreads, 0, s>>>(from, to);
  return hipGetLastError();
}

hipError_t index_objects_launch(const IndexRef& t, const uint64_t* key, const uint32_t* handle,
                                uint64_t n, uint32_t world, uint32_t rank, hipStream_t s) {
  if (n) k_index_objects<<<grid_for(n), kThreads, 0, s>>>(t, key, handle, n, world, rank);
  return hipGetLastError();
}

hipError_t index_probe_launch(const IndexRef& t, const GroupInput& in, uint32_t chunk_rows,
                              uint32_t* rep, uint8_t* valid_out, hipStream_t s, KTimer* timer) {
  if (in.n == 0) return hipSuccess;
  KScope k(timer, "index_probe", s);
  if (in.rec12)
    k_index_probe<<<grid_for(in.n), kThreads, 0, s>>>(
        t, RecIn{reinterpret_cast<const uint3*>(in.rec12), in.valid}, in.n, chunk_rows, rep,
        valid_out);
  else
    k_index_probe<<<grid_for(in.n), kThreads, 0, s>>>(
        t, RowsIn{in.key, in.valid, in.rank, in.rank_base}, in.n, chunk_rows, rep, valid_out);
  return hipGetLastError();
}

hipError_t index_creators_launch(const IndexRef& t, const GroupInput& in, const uint32_t* rep,
                                 const uint8_t* grouped, hipStream_t s, KTimer* timer,
                                 const uint32_t* skip) {
  if (in.n == 0) return hipSuccess;
  KScope k(timer, "index_insert", s);
  if (in.rec12)
    k_index_creators<<<grid_for(in.n), kThreads, 0, s>>>(
        t, RecIn{reinterpret_cast<const uint3*>(in.rec12), nullptr}, in.n, rep, grouped, skip);
  else
    k_index_creators<<<grid_for(in.n), kThreads, 0, s>>>(
        t, RowsIn{in.key, nullptr, in.rank, in.rank_base}, in.n, rep, grouped, skip);
  return hipGetLastError();
}

}  // namespace sdgpu
