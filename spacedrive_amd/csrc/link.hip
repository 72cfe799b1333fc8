// K7: Object link batch -- the write set of identifier_job_step as dense arrays.
//
// Replaces the per-100-row database decisions of
// /root/reference/core/src/object/file_identifier/mod.rs:189-333: every row
// whose cas_id matched an existing Object is connected to it (`file_path`
// update + `object::connect`, mod.rs:189-225) and every other row gets a new
// Object (`object::create_many` + connect, mod.rs:243-333).  Given the grouping
// rep[] (rank of the row whose Object a row joins; rep == own rank = creates),
// one pass compacts the whole batch into
//   create[0..C)            ranks of the rows that create an Object, ascending
//   link_row/link_obj[0..L) (row rank, creator rank) of the rows that connect
// so the host issues one create_many + one batched connect per large batch
// instead of 4-5 queries per 100 rows.  Rows with valid == 0 (metadata or
// hash failed, mod.rs:113,127) are in neither list: they stay orphans.
// HBM-bound: reads 4-9 B/row, writes 4 B per created row and 8 B per linked row.
#include "internal.hpp"
#include "scan_device.hpp"

namespace sdgpu {

namespace {

constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void k_link_flags(const uint32_t* __restrict__ rep,
                                                         const uint32_t* __restrict__ rank,
                                                         const uint8_t* __restrict__ valid,
                                                         uint32_t first_rank, uint64_t n,
                                                         uint32_t* __restrict__ fc,
                                                         uint32_t* __restrict__ fl) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = rank ? rank[i] : first_rank + static_cast<uint32_t>(i);
  const bool v = valid ? valid[i] != 0 : true;
  const bool self = rep[i] == r;
  fc[i] = (v && self) ? 1u : 0u;
  fl[i] = (v && !self) ? 1u : 0u;
}

__global__ __launch_bounds__(kThreads) void k_link_scatter(const uint32_t* __restrict__ rep,
                                                           const uint32_t* __restrict__ rank,
                                                           const uint8_t* __restrict__ valid,
                                                           uint32_t first_rank, uint64_t n,
                                                           const uint32_t* __restrict__ pc,
                                                           const uint32_t* __restrict__ pl,
                                                           uint32_t* __restrict__ create,
                                                           uint32_t* __restrict__ link_row,
                                                           uint32_t* __restrict__ link_obj) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (i >= n) return;
  if (valid && valid[i] == 0) return;
  const uint32_t r = rank ? rank[i] : first_rank + static_cast<uint32_t>(i);
  const uint32_t p = rep[i];
  if (p == r) {
    create[pc[i]] = r;
  } else {
    const uint32_t k = pl[i];
    link_row[k] = r;
    link_obj[k] = p;
  }
}

}  // namespace

size_t link_workspace_bytes(uint64_t n) {
  const size_t a = ((n + 1) * 4 + 255) / 256 * 256;
  const size_t t = ((scan::tiles_for(n) + 1) * 4 + 255) / 256 * 256;
  return 2 * a + 2 * t;
}

hipError_t link_batch_launch(const uint32_t* rep, const uint32_t* rank, const uint8_t* valid,
                             uint32_t first_rank, uint64_t n, uint32_t* create, uint32_t* link_row,
                             uint32_t* link_obj, uint32_t* d_counts, void* ws, hipStream_t s,
                             KTimer* timer) {
  if (n == 0) return hipMemsetAsync(d_counts, 0, 2 * sizeof(uint32_t), s);
  const size_t a = ((n + 1) * 4 + 255) / 256 * 256;
  const size_t t = ((scan::tiles_for(n) + 1) * 4 + 255) / 256 * 256;
  uint8_t* b = static_cast<uint8_t*>(ws);
  uint32_t* fc = reinterpret_cast<uint32_t*>(b);
  uint32_t* fl = reinterpret_cast<uint32_t*>(b + a);
  uint32_t* tc = reinterpret_cast<uint32_t*>(b + 2 * a);
  uint32_t* tl = reinterpret_cast<uint32_t*>(b + 2 * a + t);
  const uint32_t blocks = static_cast<uint32_t>((n + kThreads - 1) / kThreads);
  KScope k(timer, "link_batch", s);
  k_link_flags<<<blocks, kThreads, 0, s>>>(rep, rank, valid, first_rank, n, fc, fl);
  scan::exclusive(fc, n, fc, tc, d_counts, s);
  scan::exclusive(fl, n, fl, tl, d_counts + 1, s);
  k_link_scatter<<<blocks, kThreads, 0, s>>>(rep, rank, valid, first_rank, n, fc, fl, create,
                                             link_row, link_obj);
  return hipGetLastError();
}

}  // namespace sdgpu
