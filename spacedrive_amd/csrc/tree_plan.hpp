// Host-side planning of the tree kernels (K2/K3, b3_tree.hip): per level and
// segment, the groups of <= 16 nodes one lane folds, the CV buffer sizes and
// the plan's byte layout.  Host-only C++ (no HIP), so the sanitizer driver
// tests/c/host_sanitize.cpp exercises it on the CPU.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

namespace sdgpu {

// ---- tree BLAKE3 of large segments (file_checksum, K2/K3) -------------------
struct TreeSeg {
  const uint8_t* data;    // device pointer, 16-B aligned (bytes, or CVs when cv_input)
  uint64_t len;           // bytes (or number of CVs when cv_input)
  uint64_t chunk_offset;  // chunk counter of the first chunk
  uint32_t root;          // 1: emit the ROOT digest, 0: emit the subtree CV
  uint32_t pad;
};

namespace treeplan {

constexpr uint64_t kChunk = 1024;
constexpr uint32_t kGroup = 16;  // nodes per lane per level
constexpr int kMaxLevels = 16;   // 16^16 chunks >> any file

struct LevelSeg {
  uint64_t src;           // level 0: data pointer; else first input CV index
  uint64_t len;           // level 0: byte length of the segment
  uint64_t in_count;      // input nodes at this level (chunks at level 0)
  uint64_t out_base;      // first output CV index (non-final levels)
  uint64_t chunk_offset;  // level 0: chunk counter of the first chunk
  uint32_t root;          // ROOT on the segment's final compression
  uint32_t final_level;   // this level emits the segment's result
};

struct HostPlan {
  int levels = 0;
  uint64_t total_groups[kMaxLevels] = {};
  uint64_t cv_a = 0, cv_b = 0;  // ping-pong CV buffer sizes (in CVs)
};

inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

// Walks the levels; optionally fills descriptors [level][nseg] and group bases
// [level][nseg + 1].
inline HostPlan plan_tree(const TreeSeg* segs, uint32_t nseg, bool cv_input, LevelSeg* desc,
                   uint64_t* gbase) {
  HostPlan hp;
  std::vector<uint64_t> count(nseg), src(nseg);
  for (uint32_t s = 0; s < nseg; ++s) {
    if (cv_input) {
      count[s] = std::max<uint64_t>(segs[s].len, 1);
      src[s] = 0;  // index into the CV input (set per segment below)
    } else {
      count[s] = segs[s].len <= kChunk ? 1 : ceil_div(segs[s].len, kChunk);
      src[s] = reinterpret_cast<uint64_t>(segs[s].data);
    }
  }
  // CV input: the segments' CV arrays are concatenated into one device array
  // by the caller; seg s starts at the running sum of the preceding lengths.
  if (cv_input) {
    uint64_t run = 0;
    for (uint32_t s = 0; s < nseg; ++s) {
      src[s] = run;
      run += count[s];
    }
  }
  std::vector<bool> done(nseg, false);
  for (int lv = 0; lv < kMaxLevels; ++lv) {
    uint64_t groups = 0, outs = 0;
    bool any = false;
    for (uint32_t s = 0; s < nseg; ++s) {
      LevelSeg d{};
      uint64_t ng = 0;
      if (!done[s]) {
        any = true;
        ng = ceil_div(count[s], kGroup);
        d.src = src[s];
        d.len = (lv == 0 && !cv_input) ? segs[s].len : 0;
        d.in_count = count[s];
        d.chunk_offset = (lv == 0 && !cv_input) ? segs[s].chunk_offset : 0;
        d.root = segs[s].root;
        d.final_level = count[s] <= kGroup ? 1u : 0u;
        d.out_base = outs;
        if (!d.final_level) {
          src[s] = outs;
          outs += ng;
          count[s] = ng;
        } else {
          done[s] = true;
        }
      }
      if (desc) desc[static_cast<size_t>(lv) * nseg + s] = d;
      if (gbase) gbase[static_cast<size_t>(lv) * (nseg + 1) + s] = groups;
      groups += ng;
    }
    if (!any) break;
    if (gbase) gbase[static_cast<size_t>(lv) * (nseg + 1) + nseg] = groups;
    hp.total_groups[lv] = groups;
    if (lv % 2 == 0) hp.cv_a = std::max(hp.cv_a, outs); else hp.cv_b = std::max(hp.cv_b, outs);
    hp.levels = lv + 1;
  }
  return hp;
}

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct Layout {
  size_t desc_off, gbase_off, plan_bytes, cva_off, cvb_off, total;
};

inline Layout layout_for(const HostPlan& hp, uint32_t nseg) {
  Layout L;
  L.desc_off = 0;
  L.gbase_off = align_up(sizeof(LevelSeg) * kMaxLevels * nseg, 256);
  L.plan_bytes = align_up(L.gbase_off + sizeof(uint64_t) * kMaxLevels * (nseg + 1), 256);
  L.cva_off = L.plan_bytes;
  L.cvb_off = align_up(L.cva_off + hp.cv_a * 32, 256);
  L.total = align_up(L.cvb_off + hp.cv_b * 32, 256);
  return L;
}

}  // namespace treeplan
}  // namespace sdgpu
