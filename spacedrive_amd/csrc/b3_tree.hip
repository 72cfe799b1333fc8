// K2/K3: tree-parallel BLAKE3 of large segments -- the file_checksum path.
//
// Replaces the serial 1 MiB-read / Hasher::update loop of file_checksum
// (/root/reference/core/src/object/validation/hash.rs:10-24), run one file per
// step by the object validator (/root/reference/core/src/object/validation/
// validator_job.rs:126-169).
//
// A segment is `len` bytes at chunk counter `chunk_offset`; it is either a whole
// file (root=1: emits the 32-byte digest) or an aligned power-of-two slice of a
// streamed file (root=0: emits the slice's subtree chaining value).
//
// Level 0 (K2): ONE LANE PER GROUP OF 16 CONSECUTIVE CHUNKS (a complete 16 KiB
//   subtree unless it is the segment's ragged tail).  The lane hashes its chunks
//   in order and merges them with a 4-deep CV stack kept in LDS (lane-minor
//   layout: conflict-free), so the 15 parents of the group cost one lane 15
//   compressions and no lane ever idles in a log-depth tree.
// Level l >= 1 (K3): one lane per group of 16 CVs of the previous level, same
//   stack fold.  The level whose input fits one group is the segment's last; its
//   final parent carries ROOT.  Aligned groups of 2^k nodes are subtrees of
//   BLAKE3's left-complete tree, so the result equals the serial hash.
#include "b3_device.hpp"
#include "internal.hpp"
#include "tree_plan.hpp"

#include <algorithm>
#include <cstring>
#include <vector>

namespace sdgpu {

namespace {

constexpr int kThreads = 256;
constexpr uint32_t kStackDepth = 4;  // log2(kGroup)
using treeplan::kGroup;
using treeplan::kMaxLevels;
using treeplan::LevelSeg;
using treeplan::HostPlan;
using treeplan::Layout;
using treeplan::ceil_div;
using treeplan::layout_for;
using treeplan::plan_tree;

__device__ __forceinline__ void stk_push(uint32_t (*stk)[8][kThreads], uint32_t& sp,
                                         const uint32_t cv[8]) {
#pragma unroll
  for (int w = 0; w < 8; ++w) stk[sp][w][threadIdx.x] = cv[w];
  ++sp;
}

__device__ __forceinline__ void stk_pop(uint32_t (*stk)[8][kThreads], uint32_t& sp,
                                        uint32_t cv[8]) {
  --sp;
#pragma unroll
  for (int w = 0; w < 8; ++w) cv[w] = stk[sp][w][threadIdx.x];
}

__device__ __forceinline__ uint32_t find_seg(const uint64_t* __restrict__ group_base,
                                             uint32_t nseg, uint64_t t) {
  uint32_t lo = 0, hi = nseg;  // invariant: group_base[lo] <= t < group_base[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (group_base[mid] <= t) lo = mid; else hi = mid;
  }
  return lo;
}

template <bool kLeaves>
__global__ __launch_bounds__(kThreads) void k_tree_level(const LevelSeg* __restrict__ segs,
                                                         const uint64_t* __restrict__ group_base,
                                                         uint32_t nseg,
                                                         const uint32_t* __restrict__ in_cvs,
                                                         uint32_t* __restrict__ out_cvs,
                                                         uint32_t* __restrict__ seg_out) {
  __shared__ uint32_t stk[kStackDepth][8][kThreads];
  const uint64_t total = group_base[nseg];
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
  for (uint64_t t = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x; t < total;
       t += stride) {
    const uint32_t s = find_seg(group_base, nseg, t);
    const LevelSeg d = segs[s];
    const uint64_t g = t - group_base[s];
    const uint64_t first = g * kGroup;
    const uint32_t cnt = static_cast<uint32_t>(min<uint64_t>(kGroup, d.in_count - first));
    const bool fin = d.final_level != 0;
    uint32_t cv[8], l[8];
    uint32_t sp = 0;
    for (uint32_t i = 0; i < cnt; ++i) {
      const uint64_t node = first + i;
      if (kLeaves) {
        const uint64_t off = node * B3_CHUNK_LEN;
        const uint32_t clen = static_cast<uint32_t>(min<uint64_t>(B3_CHUNK_LEN, d.len - off));
        // a single-chunk root segment puts ROOT on the chunk's last block
        const uint32_t rf = (fin && d.root && d.in_count == 1) ? B3_ROOT : 0u;
        const uint8_t* cp = reinterpret_cast<const uint8_t*>(d.src) + off;
        if (clen == B3_CHUNK_LEN && rf == 0)
          b3_chunk_full(cp, d.chunk_offset + node, cv);
        else
          b3_chunk(cp, clen, d.chunk_offset + node, rf, cv);
      } else {
        const uint4* p = reinterpret_cast<const uint4*>(in_cvs + (d.src + node) * 8);
        const uint4 a = p[0], b = p[1];
        cv[0] = a.x; cv[1] = a.y; cv[2] = a.z; cv[3] = a.w;
        cv[4] = b.x; cv[5] = b.y; cv[6] = b.z; cv[7] = b.w;
      }
      if (i + 1 == cnt) break;  // the last node is never merged eagerly
      for (uint32_t tot = i + 1; (tot & 1u) == 0; tot >>= 1) {
        stk_pop(stk, sp, l);
        b3_parent(cv, l, cv, 0u);
      }
      stk_push(stk, sp, cv);
    }
    while (sp > 0) {
      stk_pop(stk, sp, l);
      b3_parent(cv, l, cv, (sp == 0 && fin && d.root) ? B3_ROOT : 0u);
    }
    uint4* o = reinterpret_cast<uint4*>(fin ? seg_out + static_cast<uint64_t>(s) * 8
                                            : out_cvs + (d.out_base + g) * 8);
    o[0] = make_uint4(cv[0], cv[1], cv[2], cv[3]);
    o[1] = make_uint4(cv[4], cv[5], cv[6], cv[7]);
  }
}

}  // namespace

size_t tree_workspace_bytes(const TreeSeg* segs, uint32_t nseg, bool cv_input) {
  const HostPlan hp = plan_tree(segs, nseg, cv_input, nullptr, nullptr);
  return layout_for(hp, nseg).total;
}

size_t tree_plan_bytes(uint32_t nseg) {
  HostPlan hp;
  return layout_for(hp, nseg).plan_bytes;
}

hipError_t tree_hash_launch(const TreeSeg* segs, uint32_t nseg, bool cv_input, uint8_t* out,
                            void* d_ws, void* h_ws, hipStream_t s, KTimer* timer) {
  if (nseg == 0) return hipSuccess;
  HostPlan hp = plan_tree(segs, nseg, cv_input, nullptr, nullptr);
  const Layout L = layout_for(hp, nseg);
  uint8_t* hb = static_cast<uint8_t*>(h_ws);
  uint8_t* db = static_cast<uint8_t*>(d_ws);
  std::memset(hb, 0, L.plan_bytes);
  plan_tree(segs, nseg, cv_input, reinterpret_cast<LevelSeg*>(hb + L.desc_off),
            reinterpret_cast<uint64_t*>(hb + L.gbase_off));
  hipError_t e = hipMemcpyAsync(db, hb, L.plan_bytes, hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return e;
  uint32_t* cva = reinterpret_cast<uint32_t*>(db + L.cva_off);
  uint32_t* cvb = reinterpret_cast<uint32_t*>(db + L.cvb_off);
  uint32_t* so = reinterpret_cast<uint32_t*>(out);
  for (int lv = 0; lv < hp.levels; ++lv) {
    const LevelSeg* dd = reinterpret_cast<const LevelSeg*>(db + L.desc_off) +
                         static_cast<size_t>(lv) * nseg;
    const uint64_t* gb = reinterpret_cast<const uint64_t*>(db + L.gbase_off) +
                         static_cast<size_t>(lv) * (nseg + 1);
    // level l reads level l-1's output; with CV input, level 0 reads the caller's CVs
    const uint32_t* in = (lv == 0) ? reinterpret_cast<const uint32_t*>(segs[0].data)
                                   : ((lv % 2 == 0) ? cvb : cva);
    uint32_t* o = (lv % 2 == 0) ? cva : cvb;
    const uint64_t want = ceil_div(hp.total_groups[lv], kThreads);
    const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>(std::max<uint64_t>(want, 1), 65536));
    if (lv == 0 && !cv_input) {
      KScope k(timer, "tree_leaves", s);
      k_tree_level<true><<<grid, kThreads, 0, s>>>(dd, gb, nseg, in, o, so);
    } else {
      KScope k(timer, "tree_parents", s);
      k_tree_level<false><<<grid, kThreads, 0, s>>>(dd, gb, nseg, in, o, so);
    }
  }
  return hipGetLastError();
}

}  // namespace sdgpu
